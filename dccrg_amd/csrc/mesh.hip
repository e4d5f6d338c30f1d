// The rank's leaf knowledge (dccrgx_mesh.hpp) and the local structures built
// from it: slots, inner / outer classification, send / receive lists
// (update_remote_neighbor_info dccrg.hpp:8992-9095,
// recalculate_neighbor_update_send_receive_lists 8590-8752), the neighbor
// CSRs (initialize_neighbors 8240-8289), face tables and advection tiles.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <set>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

// the ids owned by `rank`: each lane a run of kAppendRun entries, one counter
// atomic per wave (launch: select_owner_grid)
__global__ void select_owner_kernel(const uint64_t* ids, const int32_t* own, size_t n, int rank, uint64_t* out,
                                    unsigned long long* counter) {
	const size_t i0 = (blockIdx.x * size_t(blockDim.x) + threadIdx.x) * kAppendRun;
	unsigned c = 0;
	for (int k = 0; k < kAppendRun; k++)
		if (i0 + k < n && own[i0 + k] == rank) c++;
	unsigned long long at = wave_reserve(counter, c);
	for (int k = 0; k < kAppendRun && c; k++)
		if (i0 + k < n && own[i0 + k] == rank) {
			out[at++] = ids[i0 + k];
			c--;
		}
}

// the entries NOT owned by `rank`, with their owners (same launch)
__global__ void select_other_kernel(const uint64_t* ids, const int32_t* own, size_t n, int rank, uint64_t* out,
                                    int32_t* out_own, unsigned long long* counter) {
	const size_t i0 = (blockIdx.x * size_t(blockDim.x) + threadIdx.x) * kAppendRun;
	unsigned c = 0;
	for (int k = 0; k < kAppendRun; k++)
		if (i0 + k < n && own[i0 + k] != rank) c++;
	unsigned long long at = wave_reserve(counter, c);
	for (int k = 0; k < kAppendRun && c; k++)
		if (i0 + k < n && own[i0 + k] != rank) {
			out[at] = ids[i0 + k];
			out_own[at++] = own[i0 + k];
			c--;
		}
}

unsigned select_owner_grid(size_t n) { return unsigned((n + size_t(256) * kAppendRun - 1) / (size_t(256) * kAppendRun)); }

__global__ void fill_owner_kernel(int32_t* own, size_t n, int32_t v) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) own[i] = v;
}

}  // namespace

std::vector<int> HaloPlan::peers() const {
	std::vector<int> p;
	for (auto& kv : send_ids) p.push_back(kv.first);
	for (auto& kv : recv_ids) p.push_back(kv.first);
	std::sort(p.begin(), p.end());
	p.erase(std::unique(p.begin(), p.end()), p.end());
	return p;
}

static int ghost_radius(const Grid& g) { return std::max(1, int(g.hood_len)); }

// table entries per known leaf, x4: 8 = at least two entries per leaf (load
// factor 0.25..0.5)
#ifndef DCCRGX_HASH_ROOM4
#define DCCRGX_HASH_ROOM4 8
#endif

void mesh_build_hash(Mesh& M, const uint64_t* ids, const int32_t* owners, size_t n, hipStream_t s, size_t slot_upto) {
	uint32_t bits = 4;
	while ((uint64_t(4) << bits) < uint64_t(DCCRGX_HASH_ROOM4) * uint64_t(n)) bits++;
	M.tab.alloc(size_t(1) << bits);
	HIP_CHECK(hipMemsetAsync(M.tab.p, 0, M.tab.n * sizeof(HashEntry), s));
	M.mask = (uint64_t(1) << bits) - 1;
	M.shift = 64u - bits;
	k_hash_insert(M.tab.p, M.mask, M.shift, ids, owners, -2, n, s, slot_upto);
}

// The range map (dccrgx_mesh.hpp) when the known ids' per-level ranges hold
// at most 32 ids per known leaf (+16 M) - one process, or slab partitions -
// else the hash table.  DCCRGX_RANGE_MAP=0 forces the table.  The grid's
// cleared spare map (the previous mesh's, Grid::rmap_spare) is taken when its
// ranges cover these, so a mesh that changes every step (adaptive runs on
// slabs) writes only its own entries; a map made afresh gets a quarter of
// each level's range as room on either side (within the level, and the
// 32-per-leaf bound) so that the next meshes' ranges fit in it too.
// DCCRGX_RANGE_SPARE=0 always makes the map afresh, without room.
void mesh_build_range(Grid& g, Mesh& M, const uint64_t* ids, const int32_t* owners, size_t n, hipStream_t s,
                      size_t slot_upto) {
	static const char* env = std::getenv("DCCRGX_RANGE_MAP");
	static const char* senv = std::getenv("DCCRGX_RANGE_SPARE");
	const bool allowed = !(env && env[0] == '0');
	const bool spare_ok = !(senv && senv[0] == '0');
	const MapCtx& m = g.m;
	uint64_t lo[kRangeLevels], hi[kRangeLevels];
	M.rmap.release();
	M.rlev = 0;
	bool ranged;
	{
		DX_PHASE("rb.1a0_level_ranges", s);
		ranged = allowed && n && k_level_ranges(m, ids, n, lo, hi, s);
	}
	if (ranged) {
		const uint64_t limit = 32 * uint64_t(n) + (uint64_t(1) << 24);
		// the spare covers every level's range: take it as it is
		bool covered = spare_ok && g.rmap_spare.p && g.rmap_spare_rlev > 0;
		for (int L = 0; covered && L < kRangeLevels; L++) {
			if (hi[L] == 0) continue;
			bool in = false;
			for (int q = 0; q < g.rmap_spare_rlev; q++)
				in = in || (g.rmap_spare_rl[q].lo <= lo[L] && hi[L] < g.rmap_spare_rl[q].hi);
			covered = in;
		}
		if (covered && g.rmap_spare.n <= 2 * limit) {
			M.rmap.swap(g.rmap_spare);
			M.rlev = g.rmap_spare_rlev;
			for (int L = 0; L < M.rlev; L++) M.rl[L] = g.rmap_spare_rl[L];
			g.rmap_spare_rlev = 0;
			M.tab.release();
			M.mask = 0;
			k_range_insert(M.rmap.p, M.dev(m.last), ids, owners, n, slot_upto, s);
			return;
		}
		g.rmap_spare.release();
		g.rmap_spare_rlev = 0;
		for (int room = spare_ok ? 1 : 0; room >= 0; room--) {
			uint64_t total = 0;
			std::vector<RangeLevel> rl;
			for (int L = 0; L < kRangeLevels; L++) {
				if (hi[L] == 0) continue;  // no id of this level
				uint64_t a = lo[L], b = hi[L] + 1;
				if (room && L <= m.R) {
					const uint64_t w = (b - a) / 4;
					a = std::max<uint64_t>(m.first[L], a > w ? a - w : 0);
					b = std::min<uint64_t>(m.first[L + 1], b + w);
				}
				rl.push_back(RangeLevel{a, b, total});
				total += b - a;
			}
			if (total <= limit && total < (uint64_t(1) << 31)) {
				M.rlev = int(rl.size());
				for (int L = 0; L < M.rlev; L++) M.rl[L] = rl[size_t(L)];
				M.rmap.alloc(size_t(total));
				HIP_CHECK(hipMemsetAsync(M.rmap.p, 0xff, size_t(total) * sizeof(int2), s));
				M.tab.release();
				M.mask = 0;
				k_range_insert(M.rmap.p, M.dev(m.last), ids, owners, n, slot_upto, s);
				return;
			}
		}
	}
	mesh_build_hash(M, ids, owners, n, s, slot_upto);
}

// the retiring mesh's own range map, its entries cleared, as the grid's spare
static void mesh_retire_range(Grid& g, Mesh& old, hipStream_t s) {
	static const char* senv = std::getenv("DCCRGX_RANGE_SPARE");
	if ((senv && senv[0] == '0') || !old.rmap.p || old.rmap_shared || old.implicit || !old.rlev) return;
	if (old.n_known) k_range_clear(old.rmap.p, old.dev(g.m.last), old.kid.p, old.n_known, s);
	g.rmap_spare.swap(old.rmap);
	old.rmap.release();
	for (int L = 0; L < old.rlev; L++) g.rmap_spare_rl[L] = old.rl[L];
	g.rmap_spare_rlev = old.rlev;
}

// rebuild's direct mode (one process, the own leaves in slot order): the
// grid's persistent map over every level's whole id range when that is at
// most 32 entries per known leaf (+16 M); the previous mesh's entries are
// cleared one by one (its known list), not the whole map
static bool mesh_build_range_full(Grid& g, Mesh& M, const Mesh& old, size_t slot_upto, hipStream_t s) {
	static const char* env = std::getenv("DCCRGX_RANGE_MAP");
	if (env && env[0] == '0') return false;
	const MapCtx& m = g.m;
	if (m.R >= kRangeLevels || !M.n_known) return false;
	const uint64_t total = m.last;  // ids 1..last, entry id - 1
	if (total > 32 * uint64_t(M.n_known) + (uint64_t(1) << 24) || total >= (uint64_t(1) << 31)) return false;
	if (!g.rmap_full.p || g.rmap_full.n != size_t(total)) {
		g.rmap_full.alloc(size_t(total));
		g.rmap_full_clean = false;
	}
	Mesh probe;
	probe.rmap_shared = g.rmap_full.p;
	probe.rlev = m.R + 1;
	for (int L = 0; L <= m.R; L++) probe.rl[L] = RangeLevel{m.first[L], m.first[L + 1], m.first[L] - 1};
	const DevMesh pd = probe.dev(m.last);
	if (old.rmap_shared == g.rmap_full.p && old.kid.p && old.n_known) {
		k_range_clear(g.rmap_full.p, pd, old.kid.p, old.n_known, s);  // the entries the previous mesh wrote
	} else if (!g.rmap_full_clean) {
		HIP_CHECK(hipMemsetAsync(g.rmap_full.p, 0xff, g.rmap_full.n * sizeof(int2), s));
	}
	g.rmap_full_clean = false;
	M.tab.release();
	M.rmap.release();
	M.mask = 0;
	M.rmap_shared = g.rmap_full.p;
	M.rlev = m.R + 1;
	for (int L = 0; L <= m.R; L++) M.rl[L] = probe.rl[L];
	k_range_insert(g.rmap_full.p, pd, M.kid.p, M.kown.p, M.n_known, slot_upto, s);
	return true;
}

void mesh_init_implicit(Grid& g) {
	if (g.mesh.rmap_shared) g.rmap_full_clean = false;
	g.mesh = Mesh{};
	g.mesh.implicit = true;
	g.mesh.bp.init(g.m.first[1] - 1, uint64_t(g.size));
}

// keep the own leaves and the ghost leaves (level-0 parent within the ghost
// radius of an own leaf's level-0 parent) of a global list
void mesh_from_global(Grid& g, Mesh& out, const std::vector<uint64_t>& ids, const std::vector<int32_t>& owners) {
	const MapCtx& m = g.m;
	std::vector<uint64_t> lp;
	for (size_t i = 0; i < ids.size(); i++)
		if (owners[i] == g.rank) lp.push_back(map_level0_parent(m, ids[i]));
	std::sort(lp.begin(), lp.end());
	lp.erase(std::unique(lp.begin(), lp.end()), lp.end());
	const int r = ghost_radius(g);
	const int side = 2 * r + 1;
	MapCtx m0;
	{
		const int per[3] = {m.periodic[0], m.periodic[1], m.periodic[2]};
		map_init(m0, m.len, 0, per);
	}
	std::vector<uint64_t> need;
	for (uint64_t p : lp) {
		uint64_t x, y, z;
		map_indices(m0, p, x, y, z);
		for (int k = 0; k < side * side * side; k++) {
			const int dx = k % side - r, dy = (k / side) % side - r, dz = k / (side * side) - r;
			uint64_t w[3];
			if (!map_wrap(m0, 0, int64_t(x) + dx, w[0]) || !map_wrap(m0, 1, int64_t(y) + dy, w[1]) ||
			    !map_wrap(m0, 2, int64_t(z) + dz, w[2]))
				continue;
			need.push_back(map_from_indices(m0, w[0], w[1], w[2], 0));
		}
	}
	std::sort(need.begin(), need.end());
	need.erase(std::unique(need.begin(), need.end()), need.end());
	std::vector<uint64_t> kid;
	std::vector<int32_t> kown;
	for (size_t i = 0; i < ids.size(); i++) {
		if (owners[i] == g.rank || std::binary_search(need.begin(), need.end(), map_level0_parent(m, ids[i]))) {
			kid.push_back(ids[i]);
			kown.push_back(owners[i]);
		}
	}
	out = Mesh{};
	out.implicit = false;
	out.bp.init(m.first[1] - 1, uint64_t(g.size));
	upload(out.kid, kid, g.s_comp);
	upload(out.kown, kown, g.s_comp);
	out.n_known = kid.size();
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
}

// explicit own + ghost list of the current mesh
void mesh_materialize(Grid& g, Mesh& out) {
	hipStream_t s = g.s_comp;
	out = Mesh{};
	out.implicit = false;
	out.bp = g.mesh.bp;
	if (!g.mesh.implicit) {
		out.kid.alloc(g.mesh.n_known + 1);
		out.kown.alloc(g.mesh.n_known + 1);
		out.n_known = g.mesh.n_known;
		out.n_prefix = g.mesh.n_prefix;
		out.prefix_run1 = g.mesh.prefix_run1;
		if (out.n_known) {
			HIP_CHECK(hipMemcpyAsync(out.kid.p, g.mesh.kid.p, out.n_known * 8, hipMemcpyDeviceToDevice, s));
			HIP_CHECK(hipMemcpyAsync(out.kown.p, g.mesh.kown.p, out.n_known * 4, hipMemcpyDeviceToDevice, s));
		}
		HIP_CHECK(hipStreamSynchronize(s));
		return;
	}
	// implicit: the block of own level-0 cells + the ring of level-0 cells
	// around it (owners by the block partition)
	uint64_t f, c;
	g.mesh.bp.range(uint64_t(g.rank), f, c);
	DBuf<uint64_t> local;
	local.alloc(c + 1);
	k_iota_u64(local.p, f, c, s);
	const std::vector<uint64_t> ring = k_ghost_level0(g.m, g.dm(), g.rank, local.p, c, ghost_radius(g), s);
	std::vector<int32_t> rown(ring.size());
	for (size_t i = 0; i < ring.size(); i++) rown[i] = g.mesh.bp.owner(ring[i]);
	out.n_known = c + ring.size();
	out.kid.alloc(out.n_known + 1);
	out.kown.alloc(out.n_known + 1);
	if (c) {
		HIP_CHECK(hipMemcpyAsync(out.kid.p, local.p, c * 8, hipMemcpyDeviceToDevice, s));
		fill_owner_kernel<<<grid_for(c, 256), 256, 0, s>>>(out.kown.p, c, g.rank);
		HIP_CHECK(hipGetLastError());
	}
	if (!ring.empty()) {
		h2d(out.kid.p + c, ring.data(), ring.size() * 8, s);
		h2d(out.kown.p + c, rown.data(), ring.size() * 4, s);
	}
	HIP_CHECK(hipStreamSynchronize(s));
}

// Own leaves `local` (device, n) after a repartition; the ghost leaves are
// asked from whoever owns them: every rank sends every other rank the
// level-0 cells of its ghost region, and gets back the leaves it owns under
// them (finish_balance_load 3942-4147 all-gathers every added cell instead).
void mesh_from_local(Grid& g, Mesh& out, DBuf<uint64_t>& local, size_t n) {
	hipStream_t s = g.s_comp;
	DevMesh probe{};
	probe.implicit = 0;
	probe.last = g.m.last;
	const std::vector<uint64_t> need = k_ghost_level0(g.m, probe, g.rank, local.p, n, ghost_radius(g), s);
	const auto reqs = comm_allgather_u64(g, need);
	std::vector<std::vector<uint64_t>> replies(size_t(g.size));
	for (int p = 0; p < g.size; p++)
		if (p != g.rank) replies[size_t(p)] = k_cells_under(g.m, local.p, n, reqs[size_t(p)], s);
	const auto ghosts = comm_alltoall_u64(g, replies);
	std::vector<uint64_t> gid;
	std::vector<int32_t> gown;
	for (int p = 0; p < g.size; p++) {
		if (p == g.rank) continue;
		gid.insert(gid.end(), ghosts[size_t(p)].begin(), ghosts[size_t(p)].end());
		gown.insert(gown.end(), ghosts[size_t(p)].size(), p);
	}
	out = Mesh{};
	out.implicit = false;
	out.bp.init(g.m.first[1] - 1, uint64_t(g.size));
	out.n_known = n + gid.size();
	out.kid.alloc(out.n_known + 1);
	out.kown.alloc(out.n_known + 1);
	if (n) {
		HIP_CHECK(hipMemcpyAsync(out.kid.p, local.p, n * 8, hipMemcpyDeviceToDevice, s));
		fill_owner_kernel<<<grid_for(n, 256), 256, 0, s>>>(out.kown.p, n, g.rank);
		HIP_CHECK(hipGetLastError());
	}
	if (!gid.empty()) {
		h2d(out.kid.p + n, gid.data(), gid.size() * 8, s);
		h2d(out.kown.p + n, gown.data(), gid.size() * 4, s);
	}
	HIP_CHECK(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------------------
// (Re)build every local structure from `nm`.  Field payloads of cells that
// stay on this rank are carried over (old slot -> new slot); freshly created
// children inherit their parent's payload.
void rebuild(Grid& g, Mesh& nm) {
	hipStream_t s = g.s_comp;
	const MapCtx& m = g.m;
	const int nh = int(g.hood.size() / 3);
	DX_LAPS(s);

	DBuf<uint64_t> old_slot_ids;
	old_slot_ids.swap(g.slot_ids);
	Mesh old = std::move(g.mesh);
	const size_t old_n_local = g.n_local;
	g.mesh = std::move(nm);
	Mesh& M = g.mesh;
	M.tab.release();
	M.rmap.release();
	M.rmap_shared = nullptr;

	// slot order: Morton order of the min corner on refined grids (step 2)
	int order = g.slot_order;
	if (order < 0) order = g.R > 0 ? 1 : 0;
	bool fits = true;
	for (int d = 0; d < 3; d++) fits = fits && m.glen[d] <= (uint64_t(1) << 21);
	g.morton_slots = order == 1 && fits;

	// 1. own leaves, ascending (in any order when the Morton sort of step 2
	// decides the slot order)
	DBuf<uint64_t> d_local;
	bool prefix_sorted = false;  // d_local already in Morton order
	bool direct = false;         // ... and slot i = d_local[i] (table slots set on insert)
	bool solo = false;           // ... on one process: the slots are kid itself (no copies)
	if (M.implicit) {
		uint64_t f, c;
		M.bp.range(uint64_t(g.rank), f, c);
		d_local.alloc(c + 1);
		k_iota_u64(d_local.p, f, c, s);
		g.n_local = c;
	} else {
		// one process, own leaves already in Morton order: the prefix is the
		// slot order, so the table gets its slots as it is built
		direct = g.size == 1 && M.n_prefix && g.morton_slots && M.prefix_run1 == M.n_prefix && M.n_known == M.n_prefix;
		if (!(direct && mesh_build_range_full(g, M, old, M.n_prefix, s))) {
			// a mesh of its own; the shared map (if the previous mesh used it)
			// keeps that mesh's entries
			if (old.rmap_shared) g.rmap_full_clean = false;
			mesh_build_range(g, M, M.kid.p, M.kown.p, M.n_known, s, direct ? M.n_prefix : 0);
		}
		DX_LAP("rb.1a_hash");
		solo = direct && g.size == 1;
		if (solo) {
			// every known leaf is an own leaf, kid in slot order: read in place
			g.n_local = M.n_prefix;
			prefix_sorted = true;
		} else if (M.n_prefix && g.morton_slots) {
			// the own leaves are kid's prefix, in (at most two runs of) Morton order
			g.n_local = M.n_prefix;
			d_local.alloc(g.n_local + 1);
			HIP_CHECK(hipMemcpyAsync(d_local.p, M.kid.p, g.n_local * 8, hipMemcpyDeviceToDevice, s));
			prefix_sorted = M.prefix_run1 == M.n_prefix;
			if (!prefix_sorted && M.prefix_run1 > 0) {
				// two runs: merged once here, the stable inner / outer split
				// below then keeps both parts in Morton order (no sorts)
				k_morton_merge2(m, d_local.p, g.n_local, M.prefix_run1, s);
				prefix_sorted = true;
			}
		} else {
			d_local.alloc(M.n_known + 1);
			DBuf<unsigned long long> ctr;
			ctr.alloc(1);
			HIP_CHECK(hipMemsetAsync(ctr.p, 0, 8, s));
			if (M.n_known) {
				select_owner_kernel<<<select_owner_grid(M.n_known), 256, 0, s>>>(M.kid.p, M.kown.p, M.n_known, g.rank,
				                                                              d_local.p, ctr.p);
				HIP_CHECK(hipGetLastError());
			}
			unsigned long long hn = 0;
			d2h_small(&hn, ctr.p, 8, s);
			g.n_local = size_t(hn);
			if (!g.morton_slots) sort_u64(d_local.p, g.n_local, s);
		}
	}
	const size_t nl = g.n_local;
	DevMesh dm = g.dm();  // implicit: no table yet (owners by formula)
	DX_LAP("rb.1_local");

	// 2. inner / outer classification (update_remote_neighbor_info 8992-9095)
	DBuf<uint64_t> local_slots;
	if (solo) {
		g.n_outer = 0;
		g.n_inner = nl;
	} else {
		DBuf<uint32_t> flag, scan;
		flag.alloc(nl + 1);
		scan.alloc(nl + 1);
		HIP_CHECK(hipMemsetAsync(flag.p, 0, (nl + 1) * sizeof(uint32_t), s));
		if (g.size > 1) {
			// only leaves near a ghost leaf can have a remote neighbor
			// (DCCRGX_NEAR_FILTER=0: examine every leaf, for A/Bs)
			static const char* nf = std::getenv("DCCRGX_NEAR_FILTER");
			DBuf<uint8_t> near;
			uint64_t near_lo = 0;
			const bool use = !M.implicit && !(nf && nf[0] == '0') &&
			                 k_level0_near(m, M.kid.p, M.kown.p, M.n_known, g.rank, ghost_radius(g), near, near_lo, s);
			DX_LAP("rb.2a0_near");
			k_remote_flags(m, g.d_hood.p, g.d_hood_to.p, nh, dm, g.rank, d_local.p, nl, flag.p, s,
			               use ? near.p : nullptr, near_lo, use ? near.n : 0);
		}
		DX_LAP("rb.2a_remote_flags");
		g.n_outer = scan_exclusive_u32(flag.p, scan.p, nl, s);
		g.n_inner = nl - g.n_outer;
		local_slots.alloc(nl + 1);
		k_assign_slots2(flag.p, scan.p, nl, g.n_inner, d_local.p, local_slots.p, s);
		d_local.release();
	}
	const uint64_t* lsp = solo ? M.kid.p : local_slots.p;  // the own leaves in slot order
	DX_LAP("rb.2b_scan_assign");
	if (g.morton_slots && !prefix_sorted) {
		// (a Morton-ordered d_local stays so in both runs: the split is stable)
		k_morton_sort(m, local_slots.p, g.n_inner, s);
		k_morton_sort(m, local_slots.p + g.n_inner, g.n_outer, s);
	}
#if DCCRGX_PHASE_TIMING
	if (std::getenv("DCCRGX_MESH_NOTES"))
		std::fprintf(stderr, "[mesh r%d] local %zu inner %zu outer %zu known %zu prefix %zu run1 %zu sorted %d range-map levels %d\n",
		             g.rank, nl, g.n_inner, g.n_outer, M.n_known, M.n_prefix, M.prefix_run1, int(prefix_sorted), M.rlev);
#endif

	DX_LAP("rb.2_classify_sort");
	// 3. neighbor lists of outer cells -> send / receive lists (8590-8752)
	HaloPlan& H = g.halo;
	H.send_ids.clear();
	H.recv_ids.clear();
	g.extra_remote.clear();
	HaloLists HL;  // the lists' device copies (k_halo_lists), for steps 4 and 5
	bool hl = false;
	if (g.n_outer > 0) {
		const size_t no = g.n_outer;
		DBuf<uint32_t> c_of, c_to, p_of, p_to;
		c_of.alloc(no + 1);
		c_to.alloc(no + 1);
		p_of.alloc(no + 1);
		p_to.alloc(no + 1);
		k_count_rows(m, g.d_hood.p, g.d_hood_to.p, nh, dm, lsp, g.n_inner, no, c_of.p, c_to.p, s);
		size_t t_of = 0, t_to = 0;
		scan_exclusive_u32_pair(c_of.p, p_of.p, c_to.p, p_to.p, no, s, t_of, t_to);
		DBuf<uint64_t> of_id, to_id;
		DBuf<int32_t> of_off;
		of_id.alloc(t_of + 1);
		of_off.alloc(3 * t_of + 3);
		to_id.alloc(t_to + 1);
		k_fill_neighbors_of(m, g.d_hood.p, nh, dm, lsp, g.n_inner, no, p_of.p, of_id.p, of_off.p, s);
		k_fill_neighbors_to(m, g.d_hood_to.p, nh, dm, lsp, g.n_inner, no, p_to.p, to_id.p, s);
		DX_LAP("rb.3a_outer_rows");
		std::vector<uint64_t> extra;
		// the receive / send lists and the neighbors_to-only ids in one device
		// pass and two reads (DCCRGX_HALO_LISTS=split: the three separate
		// passes below)
		const char* hls = std::getenv("DCCRGX_HALO_LISTS");
		hl = !(hls && std::strcmp(hls, "split") == 0) &&
		     k_halo_lists(of_id.p, t_of, to_id.p, p_to.p, t_to, lsp, g.n_inner, no, dm, g.rank, g.size, HL, s);
		if (hl) {
			H.recv_ids = std::move(HL.recv);
			H.send_ids = std::move(HL.send);
			extra = HL.extra;
		}
		DBuf<uint64_t> of_keys;
		size_t n_of_keys = 0;
		if (!hl) k_remote_by_owner(of_id.p, t_of, dm, g.rank, g.size, H.recv_ids, s, &of_keys, &n_of_keys);
		DX_LAP("rb.3b_recv_lists");
		if (!hl) k_send_by_owner(to_id.p, p_to.p, t_to, lsp, g.n_inner, no, dm, g.rank, g.size, H.send_ids, s);
		DX_LAP("rb.3c_send_lists");
		// remote neighbors_to that are no neighbors_of: found on the device
		// (none for a symmetric neighborhood), the pairs path on the host
		if (!hl && !k_remote_extra(to_id.p, t_to, dm, g.rank, g.size, of_keys.p, n_of_keys, extra, s)) {
			std::map<int, std::vector<uint64_t>> rem_to;
			k_remote_by_owner(to_id.p, t_to, dm, g.rank, g.size, rem_to, s);
			for (auto& kv : rem_to) {
				const auto it = H.recv_ids.find(kv.first);
				for (uint64_t id : kv.second)
					if (it == H.recv_ids.end() || !std::binary_search(it->second.begin(), it->second.end(), id))
						extra.push_back(id);
			}
			std::sort(extra.begin(), extra.end());
		}
		DX_LAP("rb.3d_extra");
#if DCCRGX_PHASE_TIMING
		if (std::getenv("DCCRGX_MESH_NOTES")) {
			size_t nr = 0, ns = 0;
			for (auto& kv : H.recv_ids) nr += kv.second.size();
			for (auto& kv : H.send_ids) ns += kv.second.size();
			std::fprintf(stderr, "[mesh r%d] of entries %zu to entries %zu recv %zu send %zu extra %zu\n", g.rank, t_of,
			             t_to, nr, ns, extra.size());
		}
#endif
		g.extra_remote = extra;
	}
	g.peers = H.peers();
	DX_LAP("rb.3_lists");

	// 4. slots: local | halo (per peer, ascending) | remote neighbors_to-only
	std::vector<uint64_t> halo;
	H.recv_off.clear();
	for (auto& kv : H.recv_ids) {
		H.recv_off[kv.first] = halo.size();
		halo.insert(halo.end(), kv.second.begin(), kv.second.end());
	}
	H.n_recv = halo.size();
	g.n_recv = H.n_recv;
	halo.insert(halo.end(), g.extra_remote.begin(), g.extra_remote.end());
	g.n_slots = nl + halo.size();
	g.slot_ids.alloc(g.n_slots + 1);
	if (nl) HIP_CHECK(hipMemcpyAsync(g.slot_ids.p, lsp, nl * 8, hipMemcpyDeviceToDevice, s));
	if (hl && HL.n_recv == H.n_recv) {
		// the receive ids already on the device in this order; the few
		// neighbors_to-only ones uploaded
		if (H.n_recv)
			HIP_CHECK(hipMemcpyAsync(g.slot_ids.p + nl, HL.recv_ids.p, H.n_recv * 8, hipMemcpyDeviceToDevice, s));
		if (!g.extra_remote.empty())
			h2d(g.slot_ids.p + nl + H.n_recv, g.extra_remote.data(), g.extra_remote.size() * 8, s);
	} else if (!halo.empty()) {
		h2d(g.slot_ids.p + nl, halo.data(), halo.size() * 8, s);
	}
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	if (M.implicit) mesh_build_hash(M, g.slot_ids.p, nullptr, g.n_slots, s);
	dm = g.dm();
	DX_REQUIRE(!direct || (g.n_slots == nl && g.n_inner == nl), "internal error: direct slots with halo or outer cells");
	if (!direct) k_hash_set_slots(dm, g.slot_ids.p, g.n_slots, err.p, s);
	H.recv_slots.alloc(H.n_recv + 1);
	k_iota_i32(H.recv_slots.p, H.n_recv, int32_t(nl), s);

	DX_LAP("rb.4_slots_hash");
	// 5. send slots (ascending id per peer = wire order)
	std::vector<uint64_t> sids;
	H.send_off.clear();
	for (auto& kv : H.send_ids) {
		H.send_off[kv.first] = sids.size();
		sids.insert(sids.end(), kv.second.begin(), kv.second.end());
	}
	H.n_send = sids.size();
	{
		DBuf<uint64_t> d;
		const uint64_t* dsid = nullptr;
		if (hl && HL.n_send == sids.size()) {
			dsid = HL.send_ids.p;  // the send cells already on the device in this order
		} else {
			upload(d, sids, s);
			dsid = d.p;
		}
		H.send_slots.alloc(sids.size() + 1);
		k_lookup_slots(dsid, sids.size(), dm, H.send_slots.p, err.p, s);
		// (direct slots without send cells: nothing above can set the flag)
		if (!(direct && sids.empty())) {
			int32_t herr = 0;
			d2h_small(&herr, err.p, 4, s);
			DX_REQUIRE(herr == 0, "internal error: slot of a local, halo or send cell missing from the mesh table");
		}
	}

	DX_LAP("rb.5_send_slots");
	// 6. carry field payloads over: one source slot per new slot (one pair of
	// hash lookups for all fields), then one gather per field
	const DevMesh odm = old.dev(m.last);
	DBuf<int32_t> src;
	if (old_slot_ids.p && std::any_of(g.fields.begin(), g.fields.end(), [](const Field& f) { return !f.var; })) {
		if (direct && M.carry.n >= g.n_slots) {
			src.swap(M.carry);  // from k_apply_refines: new prefix index = new slot
		} else {
			src.alloc(g.n_slots + 1);
			k_carry_src(g.slot_ids.p, g.n_slots, nl, m, odm, old_n_local, src.p, s);
		}
	}
	M.carry.release();
	for (auto& f : g.fields) {
		f.local_zero = false;
		field_written(f);
		f.external = false;  // the array moves: a pointer handed out before is void
		if (f.var) {  // children and new copies start empty (the reference default-constructs them)
			var_remap(f, old_slot_ids.p, old_slot_ids.p ? old_n_local : 0, dm, g.n_slots, s);
			continue;
		}
		DBuf<uint8_t> nd;
		nd.alloc(g.n_slots * f.elem);
		if (f.no_carry && nd.n) {
			if (g.n_slots > nl) HIP_CHECK(hipMemsetAsync(nd.p + nl * f.elem, 0, (g.n_slots - nl) * f.elem, s));
		} else if (f.data.p && old_slot_ids.p) {
			k_gather_rows(f.data.p, src.p, g.n_slots, f.elem, nd.p, s);  // zeros where no source
		} else if (nd.n) {
			HIP_CHECK(hipMemsetAsync(nd.p, 0, nd.n, s));
		}
		f.no_carry = false;
		f.data.swap(nd);
		f.scratch.release();
	}
	// (stream-ordered: the old arrays go back to the pool, reused only after a
	// device sync)
	DX_LAP("rb.6_carry_fields");
	// the known list as [own leaves in slot order | the others] for the next
	// refinement (Mesh::n_prefix)
	M.n_prefix = M.prefix_run1 = 0;
	if (solo) {
		// kid is already [slot order], every owner this rank
		M.n_prefix = M.prefix_run1 = nl;
	} else if (!M.implicit && g.morton_slots && nl) {
		DBuf<uint64_t> kid;
		DBuf<int32_t> kown;
		kid.alloc(M.n_known + 1);
		kown.alloc(M.n_known + 1);
		HIP_CHECK(hipMemcpyAsync(kid.p, g.slot_ids.p, nl * 8, hipMemcpyDeviceToDevice, s));
		k_fill_i32(kown.p, nl, g.rank, s);
		size_t ng = 0;
		if (M.n_known > nl) {
			DBuf<unsigned long long> ctr;
			ctr.alloc(1);
			HIP_CHECK(hipMemsetAsync(ctr.p, 0, 8, s));
			select_other_kernel<<<select_owner_grid(M.n_known), 256, 0, s>>>(M.kid.p, M.kown.p, M.n_known, g.rank, kid.p + nl,
			                                                          kown.p + nl, ctr.p);
			HIP_CHECK(hipGetLastError());
			unsigned long long hn = 0;
			d2h_small(&hn, ctr.p, 8, s);
			ng = size_t(hn);
		}
		DX_REQUIRE(nl + ng == M.n_known, "internal error: known leaves are not own + others");
		M.kid.swap(kid);
		M.kown.swap(kown);
		M.n_prefix = nl;
		M.prefix_run1 = g.n_inner;
		HIP_CHECK(hipStreamSynchronize(s));
	}
	DX_LAP("rb.7_known_order");
	mesh_retire_range(g, old, s);  // after the carry step, the last reader of the old map
	DX_LAP("rb.8_retire_map");
	g.csr_valid = false;
	g.face_valid = false;
	g.tiles_valid = false;
	g.adv_commits_on_mesh = 0;
	g.slot_ids_h_valid = false;
	g.index_h_valid = false;
	g.po.valid = false;
	g.gol_plan_valid = false;
	g.gola.valid = false;
	for (auto& kv : g.uhoods) kv.second.valid = false;
}

// full neighbors_of / neighbors_to / iterator CSR for all local rows
void ensure_csr(Grid& g) {
	if (g.csr_valid) return;
	hipStream_t s = g.s_comp;
	const int nh = int(g.hood.size() / 3);
	const size_t nl = g.n_local;
	const DevMesh dm = g.dm();
	DBuf<uint32_t> c_of, c_to;
	c_of.alloc(nl + 1);
	c_to.alloc(nl + 1);
	g.nof_ptr.alloc(nl + 1);
	g.nto_ptr.alloc(nl + 1);
	g.it_ptr.alloc(nl + 1);
	k_count_rows(g.m, g.d_hood.p, g.d_hood_to.p, nh, dm, g.slot_ids.p, 0, nl, c_of.p, c_to.p, s);
	size_t t_of = 0, t_to = 0;
	scan_exclusive_u32_pair(c_of.p, g.nof_ptr.p, c_to.p, g.nto_ptr.p, nl, s, t_of, t_to);
	g.nof_id.alloc(t_of + 1);
	g.nof_off.alloc(3 * t_of + 3);
	g.nof_slot.alloc(t_of + 1);
	g.nto_id.alloc(t_to + 1);
	k_fill_neighbors_of(g.m, g.d_hood.p, nh, dm, g.slot_ids.p, 0, nl, g.nof_ptr.p, g.nof_id.p, g.nof_off.p, s);
	k_fill_neighbors_to(g.m, g.d_hood_to.p, nh, dm, g.slot_ids.p, 0, nl, g.nto_ptr.p, g.nto_id.p, s);
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	k_lookup_slots(g.nof_id.p, t_of, dm, g.nof_slot.p, err.p, s);
	DBuf<uint8_t> cls;
	cls.alloc(t_of + 1);
	k_iterator_lists(g.nof_ptr.p, g.nof_id.p, g.nof_off.p, g.nof_slot.p, g.nto_ptr.p, g.nto_id.p, nl, cls.p, c_of.p,
	                 nullptr, nullptr, nullptr, 0, s);
	const size_t t_it = scan_exclusive_u32(c_of.p, g.it_ptr.p, nl, s);
	g.it_slot.alloc(t_it + 1);
	g.it_off.alloc(3 * t_it + 3);
	k_iterator_lists(g.nof_ptr.p, g.nof_id.p, g.nof_off.p, g.nof_slot.p, g.nto_ptr.p, g.nto_id.p, nl, cls.p, nullptr,
	                 g.it_ptr.p, g.it_slot.p, g.it_off.p, 1, s);
	int32_t herr = 0;
	d2h_small(&herr, err.p, 4, s);
	DX_REQUIRE(herr == 0, "neighbor list references a cell unknown to this rank (unbalanced mesh?)");
	g.csr_valid = true;
}

void ensure_face(Grid& g) {
	if (g.face_valid) return;
	hipStream_t s = g.s_comp;
	DX_PHASE("face.build", s);
	const size_t nl = g.n_local;
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	g.face_ell.alloc(6 * nl + 6);
	g.n_fine_faces = k_face_table(g.m, g.dm(), g.slot_ids.p, nl, g.n_inner, g.morton_slots, g.face_ell.p,
	                              g.face_fine, err.p, s);
	g.slot_lvl.alloc(g.n_slots + 1);
	k_slot_levels(g.m, g.slot_ids.p, g.n_slots, g.slot_lvl.p, s);
	int32_t herr = 0;
	d2h_small(&herr, err.p, 4, s);
	DX_REQUIRE(herr == 0, "face neighbor without a local slot or remote copy");
	g.face_valid = true;
	g.face_csr_valid = false;
	g.face_gen++;
}

void ensure_face_csr(Grid& g) {
	ensure_face(g);
	if (g.face_csr_valid) return;
	k_face_csr(g.face_ell.p, g.face_fine.p, g.n_local, g.face_ptr, g.face_ent, g.s_comp);
	// consumers read the rows with blocking copies on the null stream
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
	g.face_csr_valid = true;
}

void ensure_tiles(Grid& g) {
	ensure_face_csr(g);
	if (g.tiles_valid) return;
	DX_LAPS(g.s_comp);
	const int T = g.tile;
	const TileBuild tb = k_build_tiles(g.face_ptr.p, g.face_ent.p, g.slot_ids.p, g.m, g.morton_slots, g.n_inner,
	                                   g.n_local, T, g.tstart, g.tell, g.ext_ptr, g.ext, g.ext_pk, g.fine_base, g.tfine,
	                                   g.s_comp);
	g.n_tiles_inner = tb.n_tiles_inner;
	g.n_tiles_outer = tb.n_tiles_outer;
	g.max_ext = tb.max_ext;
	g.total_ext = tb.total_ext;
	DX_LAP("tiles.1_build");
	k_classify_tiles(g.m, g.tstart.p, g.n_tiles_inner, g.n_tiles_outer, g.slot_ids.p, g.face_ell.p, g.tlists, g.tnb,
	                 g.tregmeta, g.tcount, g.s_comp);
	DX_LAP("tiles.2_classify");
	// records of the irregular tiles for the pipelined tile kernel
	const size_t nt = g.n_tiles_inner + g.n_tiles_outer, ni = g.tcount[2] + g.tcount[3];
	const auto ts = download(g.tstart.p, nt + 1, g.s_comp);
	const auto li = download(g.tlists.p + g.tcount[0] + g.tcount[1], ni, g.s_comp);
	std::vector<uint32_t> rec(8 * ni, 0u);
	bool fits = true;
	for (size_t i = 0; i < ni; i++) {
		const uint32_t t = li[i];
		uint32_t* r = &rec[8 * i];
		r[0] = ts[t];
		r[1] = ts[t + 1] - ts[t];
		r[2] = tb.ext_off[t];
		r[3] = tb.ext_n[t];
		r[4] = tb.fine_off[t];
		r[5] = tb.fine_n[t];
		if (r[3] > 1024u || r[5] > 512u || r[1] > 512u) fits = false;
	}
	if (std::getenv("DCCRGX_TILE_REASONS") && ni) {  // diagnostics: the irregular tiles' ext lists
		std::map<uint32_t, size_t> hist;
		uint32_t emax = 0;
		size_t etot = 0, ax_n[4] = {0, 0, 0, 0};
		const auto pk = download(g.ext_pk.p, g.total_ext, g.s_comp);
		for (size_t i = 0; i < ni; i++) {
			const uint32_t e = rec[8 * i + 3];
			hist[e / 128u * 128u]++;
			emax = std::max(emax, e);
			etot += e;
			for (uint32_t k = 0; k < e; k++) ax_n[__builtin_popcount(pk[rec[8 * i + 2] + k] >> 29)]++;
		}
		std::fprintf(stderr, "[tiles] irregular: %zu tiles, ext total %zu, max %u (all tiles: max %zu)\n", ni, etot, emax,
		             g.max_ext);
		for (auto& kv : hist) std::fprintf(stderr, "[tiles] ext %u..%u: %zu tiles\n", kv.first, kv.first + 127, kv.second);
		std::fprintf(stderr, "[tiles] ext axes per entry: 0:%zu 1:%zu 2:%zu 3:%zu\n", ax_n[0], ax_n[1], ax_n[2], ax_n[3]);
	}
	g.tmeta.release();
	if (fits && ni) upload(g.tmeta, rec, g.s_comp);
	// the same records merged with the regular tiles' in tile order (only for
	// the fused-sweep experiment, sweep_kernels.hip)
	g.tfused.release();
	g.tfused_n[0] = g.tfused_n[1] = 0;
#if DCCRGX_FUSED_SWEEP
	if (fits && nt) {
		const size_t nr = g.tcount[0] + g.tcount[1];
		const auto lr = download(g.tlists.p, nr, g.s_comp);
		std::vector<RegTileMeta> rm(nr);
		if (nr) d2h_small(rm.data(), g.tregmeta.p, nr * sizeof(RegTileMeta), g.s_comp);
		std::vector<int64_t> where(nt, -1);  // tile -> regular list index (>= 0) or -(irregular index) - 2
		for (size_t i = 0; i < nr; i++) where[lr[i]] = int64_t(i);
		for (size_t i = 0; i < ni; i++) where[li[i]] = -int64_t(i) - 2;
		std::vector<uint32_t> fu(8 * nt, 0u);
		for (size_t t = 0; t < nt; t++) {
			uint32_t* r = &fu[8 * t];
			if (where[t] >= 0) {
				const RegTileMeta& m = rm[size_t(where[t])];
				r[0] = m.ts;
				for (int d = 0; d < 6; d++) r[1 + d] = uint32_t(m.nst[d]);
				r[7] = 1u;
			} else {
				const uint32_t* q = &rec[8 * size_t(-where[t] - 2)];
				for (int k = 0; k < 8; k++) r[k] = q[k];
			}
		}
		upload(g.tfused, fu, g.s_comp);
		g.tfused_n[0] = g.n_tiles_inner;
		g.tfused_n[1] = g.n_tiles_outer;
	}
#endif
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
	DX_LAP("tiles.3_meta");
	g.tiles_valid = true;
	g.tiles_gen++;
}

const std::vector<uint64_t>& slot_ids_host(Grid& g) {
	if (!g.slot_ids_h_valid) {
		g.slot_ids_h = download(g.slot_ids.p, g.n_slots, g.s_comp);
		g.slot_ids_h_valid = true;
	}
	return g.slot_ids_h;
}

void lookup_batch(Grid& g, const uint64_t* ids, size_t n, int32_t* owner, int32_t* slot) {
	if (!n) return;
	hipStream_t s = g.s_comp;
	DBuf<uint64_t> d;
	d.alloc(n);
	h2d(d.p, ids, n * 8, s);
	DBuf<int32_t> o, sl;
	o.alloc(n);
	sl.alloc(n);
	k_lookup(g.dm(), d.p, n, o.p, sl.p, s);
	// both reads end in a stream sync (d2h_small): the callers read `owner` /
	// `slot` on return
	if (owner) d2h_small(owner, o.p, n * 4, s);
	if (slot) d2h_small(slot, sl.p, n * 4, s);
}

// slot of a slotted id from the host index, -1 if it has no slot
int64_t host_slot_of(Grid& g, uint64_t id);
static int64_t host_slot(Grid& g, uint64_t id) { return host_slot_of(g, id); }
int64_t host_slot_of(Grid& g, uint64_t id) {
	if (!g.index_h_valid) {
		k_sorted_slot_index(g.slot_ids.p, g.n_slots, g.index_ids_h, g.index_slots_h, g.s_comp);
		g.index_h_valid = true;
	}
	auto it = std::lower_bound(g.index_ids_h.begin(), g.index_ids_h.end(), id);
	if (it == g.index_ids_h.end() || *it != id) return -1;
	return g.index_slots_h[size_t(it - g.index_ids_h.begin())];
}

bool is_local_cell(Grid& g, uint64_t id) {
	if (!g.initialized || id == error_cell || id > g.m.last) return false;
	if (g.mesh.implicit) return id <= g.mesh.bp.n0 && g.mesh.bp.owner(id) == g.rank;
	const int64_t s = host_slot(g, id);
	return s >= 0 && size_t(s) < g.n_local;
}

int32_t lookup_owner(Grid& g, uint64_t id) {
	if (!g.initialized || id == error_cell || id > g.m.last) return -1;
	if (g.mesh.implicit) return id <= g.mesh.bp.n0 ? g.mesh.bp.owner(id) : -1;
	const int64_t s = host_slot(g, id);
	if (s >= 0 && size_t(s) < g.n_local) return g.rank;
	int32_t o = -1;  // a ghost leaf (or none): the device table knows
	lookup_batch(g, &id, 1, &o, nullptr);
	return o;
}

int64_t lookup_slot(Grid& g, uint64_t id) {
	if (!g.initialized || id == error_cell || id > g.m.last) return -1;
	return host_slot(g, id);
}

void known_leaves(Grid& g, std::vector<uint64_t>& ids, std::vector<int32_t>& owners) {
	const Mesh* src = &g.mesh;
	Mesh tmp;
	if (g.mesh.implicit) {
		mesh_materialize(g, tmp);
		src = &tmp;
	}
	std::vector<uint64_t> k = download(src->kid.p, src->n_known, g.s_comp);
	std::vector<int32_t> o = download(src->kown.p, src->n_known, g.s_comp);
	std::vector<size_t> idx(k.size());
	std::iota(idx.begin(), idx.end(), size_t(0));
	std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return k[a] < k[b]; });
	ids.resize(k.size());
	owners.resize(k.size());
	for (size_t i = 0; i < idx.size(); i++) {
		ids[i] = k[idx[i]];
		owners[i] = o[idx[i]];
	}
}

}  // namespace dccrgx
