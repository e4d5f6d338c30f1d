// dccrgx: host side of the MI355X-native dccrg hot path + the C ABI
// (include/dccrgx.h).  Owns the global leaf set (the reference's
// cell_process, dccrg.hpp:7197), drives the device neighbor build, the halo
// exchange over RCCL and the built-in sweeps.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>
#include <set>
#include <unordered_set>

#include <fcntl.h>
#include <unistd.h>

#include <cstring>

#include "dccrgx_internal.hpp"

namespace dccrgx {

static thread_local std::string g_last_error;

template <class F>
static int guard(F&& f) {
	try {
		return f();
	} catch (const Error& e) {
		g_last_error = e.what();
		return e.code;
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return DCCRGX_EINVAL;
	}
}

static inline unsigned grid_for(size_t n, unsigned per_block, unsigned cap = 256u * 32u) {
	size_t g = (n + per_block - 1) / per_block;
	if (g > cap) g = cap;
	if (g == 0) g = 1;
	return unsigned(g);
}

// ---------------------------------------------------------------------------
// small kernels local to the host driver
__global__ void block_owner_kernel(int32_t* owner_by_id, uint64_t total, uint64_t P) {
	// create_level_0_cells (dccrg.hpp:7967-8013): contiguous id blocks, the
	// first `fewer` processes get one cell less
	uint64_t cpp = total < P ? 1 : (total % P ? total / P + 1 : total / P);
	const uint64_t fewer = cpp * P - total;
	const uint64_t K = fewer * (cpp - 1);
	for (uint64_t k = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; k < total; k += uint64_t(gridDim.x) * blockDim.x) {
		uint64_t p;
		if (k < K) p = k / (cpp - 1);
		else p = fewer + (k - K) / cpp;
		owner_by_id[k + 1] = int32_t(p);
	}
}

__global__ void iota_u64_kernel(uint64_t* out, uint64_t first, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = first + i;
}

__global__ void unpack_kernel(const uint8_t* in, size_t elem, const int32_t* slots, size_t n, uint8_t* field) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n * elem; i += size_t(gridDim.x) * blockDim.x) {
		const size_t k = i / elem, b = i - k * elem;
		field[size_t(slots[k]) * elem + b] = in[i];
	}
}

// ---------------------------------------------------------------------------
// block partition on the host (same formula as block_owner_kernel)
static void block_range(uint64_t total, uint64_t P, uint64_t p, uint64_t& first, uint64_t& count) {
	const uint64_t cpp = total < P ? 1 : (total % P ? total / P + 1 : total / P);
	const uint64_t fewer = cpp * P - total;
	if (p < fewer) {
		first = 1 + p * (cpp - 1);
		count = cpp - 1;
	} else {
		first = 1 + fewer * (cpp - 1) + (p - fewer) * cpp;
		count = cpp;
	}
}

struct HostExists {
	const Grid* g;
	bool operator()(uint64_t id) const {
		if (id == error_cell || id > g->m.last) return false;
		if (g->leaves.empty()) return id < g->m.first[1];  // implicit uniform level-0 grid
		return std::binary_search(g->leaves.begin(), g->leaves.end(), id);
	}
};

static bool implicit_mesh(const Grid& g) { return g.leaves.empty(); }

static void materialize(Grid& g) {
	if (!implicit_mesh(g)) return;
	const uint64_t total = g.m.first[1] - 1;
	g.leaves.resize(total);
	g.owners.resize(total);
	for (int p = 0; p < g.size; p++) {
		uint64_t f, c;
		block_range(total, uint64_t(g.size), uint64_t(p), f, c);
		for (uint64_t i = 0; i < c; i++) {
			g.leaves[f - 1 + i] = f + i;
			g.owners[f - 1 + i] = p;
		}
	}
}

static int host_owner(const Grid& g, uint64_t id) {
	if (id == error_cell || id > g.m.last) return -1;
	if (implicit_mesh(g)) {
		if (id >= g.m.first[1]) return -1;
		const uint64_t total = g.m.first[1] - 1;
		for (int p = 0; p < g.size; p++) {
			uint64_t f, c;
			block_range(total, uint64_t(g.size), uint64_t(p), f, c);
			if (id >= f && id < f + c) return p;
		}
		return -1;
	}
	auto it = std::lower_bound(g.leaves.begin(), g.leaves.end(), id);
	if (it == g.leaves.end() || *it != id) return -1;
	return g.owners[size_t(it - g.leaves.begin())];
}

static void decode_keys(const std::vector<uint64_t>& keys, uint64_t stride, std::map<int, std::vector<uint64_t>>& out) {
	out.clear();
	for (uint64_t k : keys) out[int(k / stride)].push_back(k % stride);
}

// ---------------------------------------------------------------------------
// (Re)build every local structure from the global leaf set.  Field payloads
// of cells that stay on this rank are carried over (old slot -> new slot);
// freshly created children inherit their parent's payload.
static void rebuild(Grid& g) {
	hipStream_t s = g.s_comp;
	const MapCtx& m = g.m;
	const int nh = int(g.hood.size() / 3);

	DBuf<uint64_t> old_slot_ids;
	old_slot_ids.swap(g.slot_ids);
	DBuf<int32_t> old_slot_by_id;
	old_slot_by_id.swap(g.slot_by_id);
	const size_t old_n_local = g.n_local;

	// 1. global owner table (replaces the cell_process hash map)
	g.owner_by_id.alloc(m.last + 1);
	k_fill_i32(g.owner_by_id.p, m.last + 1, -1, s);
	DBuf<uint64_t> d_local;
	if (implicit_mesh(g)) {
		const uint64_t total = m.first[1] - 1;
		block_owner_kernel<<<grid_for(total, 256), 256, 0, s>>>(g.owner_by_id.p, total, uint64_t(g.size));
		HIP_CHECK(hipGetLastError());
		uint64_t f, c;
		block_range(total, uint64_t(g.size), uint64_t(g.rank), f, c);
		d_local.alloc(c);
		if (c) {
			iota_u64_kernel<<<grid_for(c, 256), 256, 0, s>>>(d_local.p, f, c);
			HIP_CHECK(hipGetLastError());
		}
		g.n_local = c;
	} else {
		DBuf<uint64_t> dl;
		DBuf<int32_t> dow;
		upload(dl, g.leaves, s);
		upload(dow, g.owners, s);
		k_scatter_owner(g.owner_by_id.p, dl.p, dow.p, g.leaves.size(), s);
		std::vector<uint64_t> local;
		for (size_t i = 0; i < g.leaves.size(); i++)
			if (g.owners[i] == g.rank) local.push_back(g.leaves[i]);
		upload(d_local, local, s);
		g.n_local = local.size();
		HIP_CHECK(hipStreamSynchronize(s));
	}
	const size_t nl = g.n_local;

	// 2. inner / outer classification (update_remote_neighbor_info 8992-9095)
	DBuf<uint32_t> flag, scan;
	flag.alloc(nl + 1);
	scan.alloc(nl + 1);
	HIP_CHECK(hipMemsetAsync(flag.p, 0, (nl + 1) * sizeof(uint32_t), s));
	if (g.size > 1) k_remote_flags(m, g.d_hood.p, g.d_hood_to.p, nh, g.owner_by_id.p, g.rank, d_local.p, nl, flag.p, s);
	g.n_outer = scan_exclusive_u32(flag.p, scan.p, nl, s);
	g.n_inner = nl - g.n_outer;
	DBuf<uint64_t> local_slots;
	local_slots.alloc(nl);
	k_assign_slots2(flag.p, scan.p, nl, g.n_inner, d_local.p, local_slots.p, s);
	d_local.release();
	int order = g.slot_order;
	if (const char* e = getenv("DCCRGX_SLOT_ORDER")) order = atoi(e);
	if (order < 0) order = g.R > 0 ? 1 : 0;
	bool fits = true;
	for (int d = 0; d < 3; d++) fits = fits && m.glen[d] <= (uint64_t(1) << 21);
	g.morton_slots = order == 1 && fits;
	if (g.morton_slots) {
		k_morton_sort(m, local_slots.p, g.n_inner, s);
		k_morton_sort(m, local_slots.p + g.n_inner, g.n_outer, s);
	}

	// 3. neighbor lists of outer cells -> send / receive lists (8590-8752)
	g.send_ids.clear();
	g.recv_ids.clear();
	g.extra_remote.clear();
	const uint64_t stride = m.last + 1;
	if (g.n_outer > 0) {
		const size_t no = g.n_outer;
		DBuf<uint32_t> c_of, c_to, p_of, p_to;
		c_of.alloc(no + 1);
		c_to.alloc(no + 1);
		p_of.alloc(no + 1);
		p_to.alloc(no + 1);
		k_count_rows(m, g.d_hood.p, g.d_hood_to.p, nh, g.owner_by_id.p, local_slots.p, g.n_inner, no, c_of.p, c_to.p,
		             s);
		const size_t t_of = scan_exclusive_u32(c_of.p, p_of.p, no, s);
		const size_t t_to = scan_exclusive_u32(c_to.p, p_to.p, no, s);
		DBuf<uint64_t> of_id, to_id, keys;
		DBuf<int32_t> of_off;
		of_id.alloc(t_of);
		of_off.alloc(3 * t_of);
		to_id.alloc(t_to);
		keys.alloc(std::max(t_of, t_to) + 1);
		k_fill_neighbors_of(m, g.d_hood.p, nh, g.owner_by_id.p, local_slots.p, g.n_inner, no, p_of.p, of_id.p,
		                    of_off.p, s);
		k_fill_neighbors_to(m, g.d_hood_to.p, nh, g.owner_by_id.p, local_slots.p, g.n_inner, no, p_to.p, to_id.p, s);
		size_t nk = k_extract_remote(of_id.p, t_of, g.owner_by_id.p, g.rank, stride, keys.p, s);
		nk = sort_unique_u64(keys.p, nk, s);
		decode_keys(download(keys.p, nk, s), stride, g.recv_ids);
		nk = k_extract_send(to_id.p, p_to.p, local_slots.p, g.n_inner, no, g.owner_by_id.p, g.rank, stride, keys.p, s);
		nk = sort_unique_u64(keys.p, nk, s);
		decode_keys(download(keys.p, nk, s), stride, g.send_ids);
		nk = k_extract_remote(to_id.p, t_to, g.owner_by_id.p, g.rank, stride, keys.p, s);
		nk = sort_unique_u64(keys.p, nk, s);
		std::map<int, std::vector<uint64_t>> rem_to;
		decode_keys(download(keys.p, nk, s), stride, rem_to);
		std::set<uint64_t> extra;
		for (auto& kv : rem_to) {
			const auto& rv = g.recv_ids[kv.first];
			for (uint64_t id : kv.second)
				if (!std::binary_search(rv.begin(), rv.end(), id)) extra.insert(id);
		}
		for (auto it = g.recv_ids.begin(); it != g.recv_ids.end();) {
			if (it->second.empty()) it = g.recv_ids.erase(it);
			else ++it;
		}
		g.extra_remote.assign(extra.begin(), extra.end());
	}
	std::set<int> peerset;
	for (auto& kv : g.send_ids) peerset.insert(kv.first);
	for (auto& kv : g.recv_ids) peerset.insert(kv.first);
	g.peers.assign(peerset.begin(), peerset.end());

	// 4. slots: local | halo (per peer, ascending) | remote neighbors_to-only
	std::vector<uint64_t> halo;
	g.recv_slot0.clear();
	for (auto& kv : g.recv_ids) {
		g.recv_slot0[kv.first] = nl + halo.size();
		halo.insert(halo.end(), kv.second.begin(), kv.second.end());
	}
	g.n_recv = halo.size();
	halo.insert(halo.end(), g.extra_remote.begin(), g.extra_remote.end());
	g.n_slots = nl + halo.size();
	g.slot_ids.alloc(g.n_slots);
	if (nl) HIP_CHECK(hipMemcpyAsync(g.slot_ids.p, local_slots.p, nl * 8, hipMemcpyDeviceToDevice, s));
	if (!halo.empty())
		HIP_CHECK(hipMemcpyAsync(g.slot_ids.p + nl, halo.data(), halo.size() * 8, hipMemcpyHostToDevice, s));
	g.slot_by_id.alloc(m.last + 1);
	k_fill_i32(g.slot_by_id.p, m.last + 1, -1, s);
	k_scatter_slots(g.slot_by_id.p, g.slot_ids.p, g.n_slots, s);

	// 5. send slots (ascending id per peer = wire order)
	std::vector<uint64_t> sids;
	g.send_off.clear();
	for (auto& kv : g.send_ids) {
		g.send_off[kv.first] = sids.size();
		sids.insert(sids.end(), kv.second.begin(), kv.second.end());
	}
	g.n_send_total = sids.size();
	{
		DBuf<uint64_t> d;
		upload(d, sids, s);
		g.send_slots.alloc(sids.size());
		DBuf<int32_t> err;
		err.alloc(1);
		HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
		k_lookup_slots(d.p, sids.size(), g.slot_by_id.p, g.send_slots.p, err.p, s);
		int32_t herr = 0;
		HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		DX_REQUIRE(herr == 0, "internal error: send cell without a slot");
	}

	// 6. carry field payloads over
	for (auto& f : g.fields) {
		DBuf<uint8_t> nd;
		nd.alloc(g.n_slots * f.elem);
		if (nd.n) HIP_CHECK(hipMemsetAsync(nd.p, 0, nd.n, s));
		if (f.data.p && old_slot_ids.p) {
			k_remap_field2(f.data.p, old_slot_ids.p, old_n_local, g.slot_by_id.p, m.last, nd.p, f.elem, s);
			k_parent_fill(nd.p, g.slot_ids.p, nl, g.slot_by_id.p, m, f.data.p, old_slot_by_id.p, f.elem, s);
		}
		f.data.swap(nd);
		f.scratch.release();
	}
	HIP_CHECK(hipStreamSynchronize(s));
	g.csr_valid = false;
	g.face_valid = false;
	g.tiles_valid = false;
	g.slot_ids_h_valid = false;
	g.po.valid = false;
	for (auto& kv : g.uhoods) kv.second.valid = false;
}

// full neighbors_of / neighbors_to / iterator CSR for all local rows
static void ensure_csr(Grid& g) {
	if (g.csr_valid) return;
	hipStream_t s = g.s_comp;
	const int nh = int(g.hood.size() / 3);
	const size_t nl = g.n_local;
	DBuf<uint32_t> c_of, c_to;
	c_of.alloc(nl + 1);
	c_to.alloc(nl + 1);
	g.nof_ptr.alloc(nl + 1);
	g.nto_ptr.alloc(nl + 1);
	g.it_ptr.alloc(nl + 1);
	k_count_rows(g.m, g.d_hood.p, g.d_hood_to.p, nh, g.owner_by_id.p, g.slot_ids.p, 0, nl, c_of.p, c_to.p, s);
	const size_t t_of = scan_exclusive_u32(c_of.p, g.nof_ptr.p, nl, s);
	const size_t t_to = scan_exclusive_u32(c_to.p, g.nto_ptr.p, nl, s);
	g.nof_id.alloc(t_of);
	g.nof_off.alloc(3 * t_of);
	g.nof_slot.alloc(t_of);
	g.nto_id.alloc(t_to);
	k_fill_neighbors_of(g.m, g.d_hood.p, nh, g.owner_by_id.p, g.slot_ids.p, 0, nl, g.nof_ptr.p, g.nof_id.p,
	                    g.nof_off.p, s);
	k_fill_neighbors_to(g.m, g.d_hood_to.p, nh, g.owner_by_id.p, g.slot_ids.p, 0, nl, g.nto_ptr.p, g.nto_id.p, s);
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	k_lookup_slots(g.nof_id.p, t_of, g.slot_by_id.p, g.nof_slot.p, err.p, s);
	k_iterator_lists(g.nof_ptr.p, g.nof_id.p, g.nof_off.p, g.nof_slot.p, nl, c_of.p, nullptr, nullptr, 0, s);
	const size_t t_it = scan_exclusive_u32(c_of.p, g.it_ptr.p, nl, s);
	g.it_slot.alloc(t_it);
	k_iterator_lists(g.nof_ptr.p, g.nof_id.p, g.nof_off.p, g.nof_slot.p, nl, nullptr, g.it_ptr.p, g.it_slot.p, 1, s);
	int32_t herr = 0;
	HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	DX_REQUIRE(herr == 0, "neighbor list references a cell unknown to this rank (unbalanced mesh?)");
	g.csr_valid = true;
}

static void ensure_face(Grid& g) {
	if (g.face_valid) return;
	hipStream_t s = g.s_comp;
	const size_t nl = g.n_local;
	DBuf<uint32_t> cnt;
	cnt.alloc(nl + 1);
	g.face_ptr.alloc(nl + 1);
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	k_face_lists(g.m, g.owner_by_id.p, g.slot_by_id.p, g.slot_ids.p, nl, cnt.p, nullptr, nullptr, err.p, 0, s);
	const size_t t = scan_exclusive_u32(cnt.p, g.face_ptr.p, nl, s);
	g.face_ent.alloc(t);
	k_face_lists(g.m, g.owner_by_id.p, g.slot_by_id.p, g.slot_ids.p, nl, nullptr, g.face_ptr.p, g.face_ent.p, err.p, 1,
	             s);
	int32_t herr = 0;
	HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	DX_REQUIRE(herr == 0, "face neighbor without a local slot or remote copy");
	g.face_ell.alloc(6 * nl);
	g.face_fine.alloc(t / 4 + 4);
	g.n_fine_faces = k_face_ell(g.face_ptr.p, g.face_ent.p, nl, g.face_ell.p, g.face_fine.p, s);
	g.face_valid = true;
}

static int tile_size_setting() {
	static const int t = [] {
		const char* e = getenv("DCCRGX_TILE");
		return e ? atoi(e) : 512;
	}();
	return t;
}

static void ensure_tiles(Grid& g) {
	ensure_face(g);
	const int T = tile_size_setting();
	if (g.tiles_valid && g.tile == T) return;
	const TileBuild tb = k_build_tiles(g.face_ptr.p, g.face_ent.p, g.slot_ids.p, g.m, g.morton_slots, g.n_inner,
	                                   g.n_local, T, g.tstart, g.tell, g.ext_ptr, g.ext, g.ext_pk, g.fine_base, g.tfine, g.s_comp);
	g.tile = T;
	g.n_tiles_inner = tb.n_tiles_inner;
	g.n_tiles_outer = tb.n_tiles_outer;
	g.max_ext = tb.max_ext;
	g.total_ext = tb.total_ext;
	k_classify_tiles(g.m, g.tstart.p, g.n_tiles_inner, g.n_tiles_outer, g.slot_ids.p, g.face_ell.p, g.tlists, g.tnb,
	                 g.tregmeta, g.tcount, g.s_comp);
	{
		// records of the irregular tiles for the pipelined tile kernel
		const size_t nt = g.n_tiles_inner + g.n_tiles_outer, ni = g.tcount[2] + g.tcount[3];
		const auto ts = download(g.tstart.p, nt + 1, g.s_comp);
		const auto ep = download(g.ext_ptr.p, nt + 1, g.s_comp);
		const auto fb = download(g.fine_base.p, nt + 1, g.s_comp);
		const auto li = download(g.tlists.p + g.tcount[0] + g.tcount[1], ni, g.s_comp);
		std::vector<uint32_t> rec(8 * ni, 0u);
		bool fits = true;
		for (size_t i = 0; i < ni; i++) {
			const uint32_t t = li[i];
			// finer faces of tile t: up to the next tile's first one (fine_base is
			// the exclusive scan at each tile's first slot)
			const uint32_t fend = t + 1 < nt ? fb[t + 1] : uint32_t(g.n_fine_faces);
			uint32_t* r = &rec[8 * i];
			r[0] = ts[t];
			r[1] = ts[t + 1] - ts[t];
			r[2] = ep[t];
			r[3] = ep[t + 1] - ep[t];
			r[4] = fb[t];
			r[5] = fend - fb[t];
			if (r[3] > 1024u || r[5] > 512u || r[1] > 512u) fits = false;
		}
		g.tmeta.release();
		if (fits && ni) upload(g.tmeta, rec, g.s_comp);
		// records of every tile, slot order, for the fused sweep
		const size_t nr = g.tcount[0] + g.tcount[1];
		const auto lr = download(g.tlists.p, nr, g.s_comp);
		const auto nb = download(g.tnb.p, 6 * nt, g.s_comp);
		std::vector<uint8_t> is_reg(nt, 0);
		for (uint32_t t : lr) is_reg[t] = 1;
		std::vector<uint32_t> fr(16 * nt, 0u);
		bool ffits = true;
		for (size_t t = 0; t < nt; t++) {
			uint32_t* r = &fr[16 * t];
			const uint32_t fend = t + 1 < nt ? fb[t + 1] : uint32_t(g.n_fine_faces);
			r[0] = ts[t];
			r[1] = ts[t + 1] - ts[t];
			r[2] = ep[t];
			r[3] = ep[t + 1] - ep[t];
			r[4] = fb[t];
			r[5] = fend - fb[t];
			for (int d = 0; d < 6; d++) r[6 + d] = is_reg[t] ? uint32_t(nb[6 * t + size_t(d)]) : 0xffffffffu;
			r[12] = is_reg[t];
			if (!is_reg[t] && (r[3] > 1024u || r[5] > 512u || r[1] > 512u)) ffits = false;
		}
		g.tfmeta.release();
		if (ffits && nt && g.tile == 512) upload(g.tfmeta, fr, g.s_comp);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
	}
	g.tiles_valid = true;
}

static const std::vector<uint64_t>& slot_ids_host(Grid& g) {
	if (!g.slot_ids_h_valid) {
		g.slot_ids_h = download(g.slot_ids.p, g.n_slots, g.s_comp);
		g.slot_ids_h_valid = true;
	}
	return g.slot_ids_h;
}

static int64_t slot_of(Grid& g, uint64_t id) {
	if (id == error_cell || id > g.m.last || !g.initialized) return -1;
	int32_t s = -1;
	HIP_CHECK(hipMemcpy(&s, g.slot_by_id.p + id, 4, hipMemcpyDeviceToHost));
	return s;
}

static Field& field(Grid& g, int fid) {
	DX_REQUIRE(fid >= 0 && size_t(fid) < g.fields.size(), "invalid field id");
	return g.fields[size_t(fid)];
}

static void ensure_scratch(Grid& g, Field& f) {
	if (f.scratch.n != f.data.n) f.scratch.alloc(f.data.n);
}

// commit a double-buffered sweep: swap, and carry the current remote copies
// over so they hold the last received values (as the reference's copies do)
static void commit(Grid& g, Field& f) {
	DX_REQUIRE(f.scratch.n == f.data.n && f.data.p, "nothing to commit");
	const size_t halo = (g.n_slots - g.n_local) * f.elem;
	if (halo)
		HIP_CHECK(hipMemcpyAsync(f.scratch.p + g.n_local * f.elem, f.data.p + g.n_local * f.elem, halo,
		                         hipMemcpyDeviceToDevice, g.s_comp));
	f.data.swap(f.scratch);
}

static void region_range(const Grid& g, int region, size_t& s0, size_t& s1) {
	switch (region) {
	case DCCRGX_REGION_ALL: s0 = 0; s1 = g.n_local; break;
	case DCCRGX_REGION_INNER: s0 = 0; s1 = g.n_inner; break;
	case DCCRGX_REGION_OUTER: s0 = g.n_inner; s1 = g.n_local; break;
	default: throw Error(DCCRGX_EINVAL, "invalid region");
	}
}

void k_time_begin(Grid& g) {
	if (!g.timing) return;
	hipEvent_t a, b;
	HIP_CHECK(hipEventCreate(&a));
	HIP_CHECK(hipEventCreate(&b));
	HIP_CHECK(hipEventRecord(a, g.s_comp));
	g.pending_events.push_back({a, b});
}

void k_time_end(Grid& g) {
	if (!g.timing) return;
	HIP_CHECK(hipEventRecord(g.pending_events.back().second, g.s_comp));
}

static void drain_timing(Grid& g) {
	for (auto& ab : g.pending_events) {
		HIP_CHECK(hipEventSynchronize(ab.second));
		float ms = 0;
		HIP_CHECK(hipEventElapsedTime(&ms, ab.first, ab.second));
		g.timed_ms += ms;
		g.timed_count++;
		(void)hipEventDestroy(ab.first);
		(void)hipEventDestroy(ab.second);
	}
	g.pending_events.clear();
}

// --------------------------------------------------------------------------- halo
static void halo_start(Grid& g) {
	if (g.size == 1 || g.peers.empty()) return;
	DX_REQUIRE(g.comm, "halo exchange needs a communicator (grid created without an RCCL id)");
	DX_REQUIRE(!g.halo_in_flight, "remote neighbor update already in flight");
	std::vector<Field*> tf;
	size_t bytes_per_cell = 0;
	for (auto& f : g.fields)
		if (f.transfer) {
			tf.push_back(&f);
			bytes_per_cell += f.elem;
		}
	if (tf.empty()) return;
	if (g.sendbuf.n < g.n_send_total * bytes_per_cell) g.sendbuf.alloc(g.n_send_total * bytes_per_cell);
	HIP_CHECK(hipEventRecord(g.ev_comp, g.s_comp));
	HIP_CHECK(hipStreamWaitEvent(g.s_comm, g.ev_comp, 0));
	size_t off = 0;
	std::vector<size_t> foff;
	for (Field* f : tf) {
		foff.push_back(off);
		k_pack(f->data.p, f->elem, g.send_slots.p, g.n_send_total, g.sendbuf.p + off, g.s_comm);
		off += g.n_send_total * f->elem;
	}
	NCCL_CHECK(ncclGroupStart());
	for (int p : g.peers) {
		auto si = g.send_ids.find(p);
		auto ri = g.recv_ids.find(p);
		for (size_t k = 0; k < tf.size(); k++) {
			Field* f = tf[k];
			if (si != g.send_ids.end() && !si->second.empty())
				NCCL_CHECK(ncclSend(g.sendbuf.p + foff[k] + g.send_off[p] * f->elem, si->second.size() * f->elem,
				                    ncclUint8, p, g.comm, g.s_comm));
			if (ri != g.recv_ids.end() && !ri->second.empty())
				NCCL_CHECK(ncclRecv(f->data.p + g.recv_slot0[p] * f->elem, ri->second.size() * f->elem, ncclUint8, p,
				                    g.comm, g.s_comm));
		}
	}
	NCCL_CHECK(ncclGroupEnd());
	HIP_CHECK(hipEventRecord(g.ev_halo, g.s_comm));
	g.halo_in_flight = true;
}

static void halo_wait(Grid& g) {
	if (!g.halo_in_flight) return;
	HIP_CHECK(hipStreamWaitEvent(g.s_comp, g.ev_halo, 0));
	g.halo_in_flight = false;
}

// --------------------------------------------------------------------------- user neighborhoods
// neighbors of / to every local cell for hood id (find_neighbors_of /
// find_neighbors_to with user_hood_of / user_hood_to, 8974-8980), then the
// send / receive lists of the id: receive from p = the cells of p in the
// neighbors_of of local cells, send to p = the local cells in whose
// neighbors_to a cell of p appears, both ascending (the wire order)
static UserHood& ensure_uhood(Grid& g, int id) {
	auto it = g.uhoods.find(id);
	DX_REQUIRE(it != g.uhoods.end(), "no such neighborhood id");
	UserHood& h = it->second;
	if (h.valid) return h;
	hipStream_t s = g.s_comp;
	const int nh = int(h.of.size() / 3);
	const size_t nl = g.n_local;
	DBuf<uint32_t> c_of, c_to;
	c_of.alloc(nl + 1);
	c_to.alloc(nl + 1);
	h.nof_ptr.alloc(nl + 1);
	h.nto_ptr.alloc(nl + 1);
	k_count_rows(g.m, h.d_of.p, h.d_to.p, nh, g.owner_by_id.p, g.slot_ids.p, 0, nl, c_of.p, c_to.p, s);
	const size_t t_of = scan_exclusive_u32(c_of.p, h.nof_ptr.p, nl, s);
	const size_t t_to = scan_exclusive_u32(c_to.p, h.nto_ptr.p, nl, s);
	h.nof_id.alloc(t_of + 1);
	h.nof_off.alloc(3 * t_of + 3);
	h.nto_id.alloc(t_to + 1);
	k_fill_neighbors_of(g.m, h.d_of.p, nh, g.owner_by_id.p, g.slot_ids.p, 0, nl, h.nof_ptr.p, h.nof_id.p, h.nof_off.p,
	                    s);
	k_fill_neighbors_to(g.m, h.d_to.p, nh, g.owner_by_id.p, g.slot_ids.p, 0, nl, h.nto_ptr.p, h.nto_id.p, s);
	h.send_ids.clear();
	h.recv_ids.clear();
	if (g.size > 1) {
		const auto pof = download(h.nof_ptr.p, nl + 1, s);
		const auto pto = download(h.nto_ptr.p, nl + 1, s);
		const auto iof = download(h.nof_id.p, t_of, s);
		const auto ito = download(h.nto_id.p, t_to, s);
		const auto& sid = slot_ids_host(g);
		std::map<int, std::vector<uint64_t>> snd, rcv;
		for (size_t r = 0; r < nl; r++) {
			for (uint32_t j = pof[r]; j < pof[r + 1]; j++) {
				const int o = host_owner(g, iof[j]);
				if (o >= 0 && o != g.rank) rcv[o].push_back(iof[j]);
			}
			for (uint32_t j = pto[r]; j < pto[r + 1]; j++) {
				const int o = host_owner(g, ito[j]);
				if (o >= 0 && o != g.rank) snd[o].push_back(sid[r]);
			}
		}
		auto uniq = [](std::map<int, std::vector<uint64_t>>& mp) {
			for (auto& kv : mp) {
				std::sort(kv.second.begin(), kv.second.end());
				kv.second.erase(std::unique(kv.second.begin(), kv.second.end()), kv.second.end());
			}
		};
		uniq(snd);
		uniq(rcv);
		h.send_ids = snd;
		h.recv_ids = rcv;
	}
	std::vector<uint64_t> sall, rall;
	h.send_off.clear();
	h.recv_off.clear();
	for (auto& kv : h.send_ids) {
		h.send_off[kv.first] = sall.size();
		sall.insert(sall.end(), kv.second.begin(), kv.second.end());
	}
	for (auto& kv : h.recv_ids) {
		h.recv_off[kv.first] = rall.size();
		rall.insert(rall.end(), kv.second.begin(), kv.second.end());
	}
	h.n_send = sall.size();
	h.n_recv = rall.size();
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	h.send_slots.alloc(h.n_send + 1);
	h.recv_slots.alloc(h.n_recv + 1);
	if (h.n_send) {
		DBuf<uint64_t> d;
		upload(d, sall, s);
		k_lookup_slots(d.p, h.n_send, g.slot_by_id.p, h.send_slots.p, err.p, s);
		HIP_CHECK(hipStreamSynchronize(s));
	}
	if (h.n_recv) {
		DBuf<uint64_t> d;
		upload(d, rall, s);
		k_lookup_slots(d.p, h.n_recv, g.slot_by_id.p, h.recv_slots.p, err.p, s);
		HIP_CHECK(hipStreamSynchronize(s));
	}
	int herr = 0;
	HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	DX_REQUIRE(herr == 0, "user neighborhood references a cell without a local slot or remote copy");
	h.valid = true;
	return h;
}

// update_copies_of_remote_neighbors(id) (966-1000 with a user id): every
// transferred field's payload of the id's send lists, packed in wire order,
// grouped RCCL send / recv per peer, unpacked into the halo slots of the
// id's receive lists; the compute stream waits for it
static void uhood_halo(Grid& g, int id) {
	UserHood& h = ensure_uhood(g, id);
	if (g.size == 1 || (h.send_ids.empty() && h.recv_ids.empty())) return;
	DX_REQUIRE(g.comm, "halo exchange needs a communicator (grid created without an RCCL id)");
	DX_REQUIRE(!g.halo_in_flight, "remote neighbor update already in flight");
	std::vector<Field*> tf;
	size_t bpc = 0;
	for (auto& f : g.fields)
		if (f.transfer) {
			tf.push_back(&f);
			bpc += f.elem;
		}
	if (tf.empty()) return;
	if (h.sendbuf.n < h.n_send * bpc + 1) h.sendbuf.alloc(h.n_send * bpc + 1);
	if (h.recvbuf.n < h.n_recv * bpc + 1) h.recvbuf.alloc(h.n_recv * bpc + 1);
	HIP_CHECK(hipEventRecord(g.ev_comp, g.s_comp));
	HIP_CHECK(hipStreamWaitEvent(g.s_comm, g.ev_comp, 0));
	std::vector<size_t> so, ro;
	size_t a = 0, b = 0;
	for (Field* f : tf) {
		so.push_back(a);
		ro.push_back(b);
		k_pack(f->data.p, f->elem, h.send_slots.p, h.n_send, h.sendbuf.p + a, g.s_comm);
		a += h.n_send * f->elem;
		b += h.n_recv * f->elem;
	}
	NCCL_CHECK(ncclGroupStart());
	for (size_t k = 0; k < tf.size(); k++) {
		const size_t e = tf[k]->elem;
		for (auto& kv : h.send_ids)
			NCCL_CHECK(ncclSend(h.sendbuf.p + so[k] + h.send_off[kv.first] * e, kv.second.size() * e, ncclUint8,
			                    kv.first, g.comm, g.s_comm));
		for (auto& kv : h.recv_ids)
			NCCL_CHECK(ncclRecv(h.recvbuf.p + ro[k] + h.recv_off[kv.first] * e, kv.second.size() * e, ncclUint8,
			                    kv.first, g.comm, g.s_comm));
	}
	NCCL_CHECK(ncclGroupEnd());
	for (size_t k = 0; k < tf.size(); k++) {
		unpack_kernel<<<grid_for(h.n_recv * tf[k]->elem, 256), 256, 0, g.s_comm>>>(
		    h.recvbuf.p + ro[k], tf[k]->elem, h.recv_slots.p, h.n_recv, tf[k]->data.p);
		HIP_CHECK(hipGetLastError());
	}
	HIP_CHECK(hipEventRecord(g.ev_halo, g.s_comm));
	HIP_CHECK(hipStreamWaitEvent(g.s_comp, g.ev_halo, 0));
}

// --------------------------------------------------------------------------- collectives
static void allgather_u64(Grid& g, const std::vector<uint64_t>& mine, std::vector<std::vector<uint64_t>>& all) {
	all.assign(size_t(g.size), {});
	DX_REQUIRE(g.size == 1 || g.comm, "collective needs a communicator (grid created without an RCCL id)");
	if (g.size == 1) {
		all[0] = mine;
		return;
	}
	hipStream_t s = g.s_comm;
	DBuf<uint64_t> cnt, cnts;
	cnt.alloc(1);
	cnts.alloc(size_t(g.size));
	uint64_t n = mine.size();
	HIP_CHECK(hipMemcpyAsync(cnt.p, &n, 8, hipMemcpyHostToDevice, s));
	NCCL_CHECK(ncclAllGather(cnt.p, cnts.p, 1, ncclUint64, g.comm, s));
	std::vector<uint64_t> hc = download(cnts.p, size_t(g.size), s);
	const uint64_t mx = std::max<uint64_t>(1, *std::max_element(hc.begin(), hc.end()));
	DBuf<uint64_t> buf, out;
	buf.alloc(mx);
	out.alloc(mx * uint64_t(g.size));
	if (n) HIP_CHECK(hipMemcpyAsync(buf.p, mine.data(), n * 8, hipMemcpyHostToDevice, s));
	NCCL_CHECK(ncclAllGather(buf.p, out.p, mx, ncclUint64, g.comm, s));
	std::vector<uint64_t> h = download(out.p, mx * uint64_t(g.size), s);
	for (int p = 0; p < g.size; p++) all[size_t(p)].assign(h.begin() + p * mx, h.begin() + p * mx + hc[size_t(p)]);
}

static void allreduce_f64(Grid& g, double* v, int count, int op) {
	if (g.size == 1) return;
	DX_REQUIRE(g.comm, "collective needs a communicator (grid created without an RCCL id)");
	DBuf<double> d;
	d.alloc(size_t(count));
	HIP_CHECK(hipMemcpyAsync(d.p, v, size_t(count) * 8, hipMemcpyHostToDevice, g.s_comm));
	const ncclRedOp_t rop = op == 0 ? ncclSum : (op == 1 ? ncclMin : ncclMax);
	NCCL_CHECK(ncclAllReduce(d.p, d.p, size_t(count), ncclFloat64, rop, g.comm, g.s_comm));
	HIP_CHECK(hipMemcpyAsync(v, d.p, size_t(count) * 8, hipMemcpyDeviceToHost, g.s_comm));
	HIP_CHECK(hipStreamSynchronize(g.s_comm));
}

// --------------------------------------------------------------------------- refinement
// induce_refines (dccrg.hpp:9591-9720): close the request set under "a
// neighbors_of / neighbors_to entry coarser than a refined cell is refined
// too", then execute_refines (10104-10554): children inherit the owner.
static std::vector<uint64_t> stop_refining_impl(Grid& g) {
	std::vector<std::vector<uint64_t>> all;
	allgather_u64(g, g.refine_requests, all);
	g.refine_requests.clear();
	materialize(g);
	std::unordered_set<uint64_t> S;
	std::vector<uint64_t> fresh;
	const HostExists ex{&g};
	for (auto& v : all)
		for (uint64_t c : v)
			if (ex(c) && map_level(g.m, c) < g.R && S.insert(c).second) fresh.push_back(c);
	const int nh = int(g.hood.size() / 3);
	while (!fresh.empty()) {
		std::vector<uint64_t> next;
		for (uint64_t r : fresh) {
			uint64_t c[3];
			const int lvl = map_indices(g.m, r, c[0], c[1], c[2]);
			auto consider = [&](uint64_t n) {
				if (n == error_cell || !ex(n)) return;
				if (map_level(g.m, n) < lvl && S.insert(n).second) next.push_back(n);
			};
			for (int k = 0; k < nh; k++) {
				ItemOut o;
				nof_item(g.m, c, lvl, &g.hood[3 * k], ex, o);
				for (int i = 0; i < o.n; i++) consider(o.id[i]);
			}
			for (int k = 0; k < 10 * nh; k++) consider(nto_candidate(g.m, c, lvl, g.hood_to.data(), nh, k, ex));
		}
		fresh.swap(next);
	}
	if (S.empty()) return {};
	std::vector<uint64_t> nl;
	std::vector<int32_t> no;
	std::vector<std::pair<uint64_t, int32_t>> created;
	for (size_t i = 0; i < g.leaves.size(); i++) {
		if (S.count(g.leaves[i])) {
			uint64_t ch[8];
			map_all_children(g.m, g.leaves[i], ch);
			for (auto c : ch) created.push_back({c, g.owners[i]});
		} else {
			nl.push_back(g.leaves[i]);
			no.push_back(g.owners[i]);
		}
	}
	std::vector<std::pair<uint64_t, int32_t>> merged;
	merged.reserve(nl.size() + created.size());
	for (size_t i = 0; i < nl.size(); i++) merged.push_back({nl[i], no[i]});
	merged.insert(merged.end(), created.begin(), created.end());
	std::sort(merged.begin(), merged.end());
	g.leaves.resize(merged.size());
	g.owners.resize(merged.size());
	for (size_t i = 0; i < merged.size(); i++) {
		g.leaves[i] = merged[i].first;
		g.owners[i] = merged[i].second;
	}
	rebuild(g);
	std::vector<uint64_t> mine;
	for (auto& c : created)
		if (c.second == g.rank) mine.push_back(c.first);
	std::sort(mine.begin(), mine.end());
	return mine;
}

// --------------------------------------------------------------------------- load balance
// balance_load with pins (dccrg.hpp:1024-1044, make_new_partition 8426-8518,
// migration continue_balance_load 3899-3934): pinned cells move, the rest
// keep their owner; payloads of moved cells travel over RCCL.
// Move every leaf to new_owner[i] (g.leaves order): migration plan in
// ascending id per (source, destination) as make_new_partition sorts its
// receive lists (8482-8493), payloads of every field packed in that order and
// moved with grouped RCCL send/recv (continue_balance_load 3899-3934), then
// the rebuild and the unpack into the new slots.  A detached view (size > 1,
// no communicator) rebuilds its structures only; the payload of a cell it
// receives is left to its caller (the multi-rank tests move it).
static void migrate_to(Grid& g, const std::vector<int32_t>& new_owner) {
	DX_REQUIRE(new_owner.size() == g.leaves.size(), "one new owner per leaf");
	for (int32_t o : new_owner) DX_REQUIRE(o >= 0 && o < g.size, "new owner out of range");
	const bool transport = g.size > 1 && g.comm;
	// migration plan: ascending id per (source, destination)
	std::map<int, std::vector<uint64_t>> out, in;
	for (size_t i = 0; i < g.leaves.size(); i++) {
		if (g.owners[i] == new_owner[i]) continue;
		if (g.owners[i] == g.rank) out[new_owner[i]].push_back(g.leaves[i]);
		if (new_owner[i] == g.rank) in[g.owners[i]].push_back(g.leaves[i]);
	}
	hipStream_t s = g.s_comp;
	std::vector<DBuf<uint8_t>> sbufs(g.fields.size()), rbufs(g.fields.size());
	std::vector<uint64_t> out_ids, in_ids;
	std::map<int, size_t> out_off, in_off;
	for (auto& kv : out) {
		out_off[kv.first] = out_ids.size();
		out_ids.insert(out_ids.end(), kv.second.begin(), kv.second.end());
	}
	for (auto& kv : in) {
		in_off[kv.first] = in_ids.size();
		in_ids.insert(in_ids.end(), kv.second.begin(), kv.second.end());
	}
	if (transport) {
		DBuf<uint64_t> dids;
		upload(dids, out_ids, s);
		DBuf<int32_t> oslots, err;
		oslots.alloc(out_ids.size());
		err.alloc(1);
		HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
		k_lookup_slots(dids.p, out_ids.size(), g.slot_by_id.p, oslots.p, err.p, s);
		for (size_t k = 0; k < g.fields.size(); k++) {
			Field& f = g.fields[k];
			sbufs[k].alloc(out_ids.size() * f.elem);
			rbufs[k].alloc(in_ids.size() * f.elem);
			k_pack(f.data.p, f.elem, oslots.p, out_ids.size(), sbufs[k].p, s);
		}
		HIP_CHECK(hipStreamSynchronize(s));
		if (!g.fields.empty()) {
			NCCL_CHECK(ncclGroupStart());
			for (size_t k = 0; k < g.fields.size(); k++) {
				const size_t e = g.fields[k].elem;
				for (auto& kv : out)
					NCCL_CHECK(ncclSend(sbufs[k].p + out_off[kv.first] * e, kv.second.size() * e, ncclUint8, kv.first,
					                    g.comm, s));
				for (auto& kv : in)
					NCCL_CHECK(ncclRecv(rbufs[k].p + in_off[kv.first] * e, kv.second.size() * e, ncclUint8, kv.first,
					                    g.comm, s));
			}
			NCCL_CHECK(ncclGroupEnd());
		}
		HIP_CHECK(hipStreamSynchronize(s));
	}
	g.owners = new_owner;
	rebuild(g);
	if (transport && !in_ids.empty()) {
		DBuf<uint64_t> dids;
		upload(dids, in_ids, s);
		DBuf<int32_t> islots, err;
		islots.alloc(in_ids.size());
		err.alloc(1);
		HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
		k_lookup_slots(dids.p, in_ids.size(), g.slot_by_id.p, islots.p, err.p, s);
		for (size_t k = 0; k < g.fields.size(); k++) {
			Field& f = g.fields[k];
			unpack_kernel<<<grid_for(in_ids.size() * f.elem, 256), 256, 0, s>>>(rbufs[k].p, f.elem, islots.p,
			                                                                    in_ids.size(), f.data.p);
			HIP_CHECK(hipGetLastError());
		}
		HIP_CHECK(hipStreamSynchronize(s));
	}
}

// balance_load with pins (dccrg.hpp:1024-1044; update_pin_requests
// all-gathers them, make_new_partition 8426-8518 moves every pinned cell to
// its process): pins stay in force until unpin (5909), as the reference's
// pin_requests do; the rest keep their owner (no third-party partitioner).
static void balance_load_impl(Grid& g) {
	std::vector<uint64_t> mine;
	for (auto& kv : g.pins) {
		mine.push_back(kv.first);
		mine.push_back(uint64_t(kv.second));
	}
	std::vector<std::vector<uint64_t>> all;
	allgather_u64(g, mine, all);
	materialize(g);
	std::vector<int32_t> new_owner = g.owners;
	for (auto& v : all)
		for (size_t i = 0; i + 1 < v.size(); i += 2) {
			auto it = std::lower_bound(g.leaves.begin(), g.leaves.end(), v[i]);
			if (it == g.leaves.end() || *it != v[i]) continue;
			if (int64_t(v[i + 1]) < 0 || int64_t(v[i + 1]) >= g.size) continue;
			new_owner[size_t(it - g.leaves.begin())] = int32_t(v[i + 1]);
		}
	migrate_to(g, new_owner);
}

// --------------------------------------------------------------------------- Poisson
// Poisson_Solve (tests/poisson/poisson_solve.hpp:156-1056) over device fields.

// halo update of exactly the given fields (the reference's
// Poisson_Cell::transfer_switch, 92-140)
static void halo_only(Grid& g, const std::vector<int>& fids) {
	if (g.size == 1 || g.peers.empty()) return;
	std::vector<char> saved(g.fields.size());
	for (size_t i = 0; i < g.fields.size(); i++) {
		saved[i] = g.fields[i].transfer;
		g.fields[i].transfer = false;
	}
	for (int f : fids) field(g, f).transfer = true;
	try {
		halo_start(g);
	} catch (...) {
		for (size_t i = 0; i < g.fields.size(); i++) g.fields[i].transfer = saved[i];
		throw;
	}
	for (size_t i = 0; i < g.fields.size(); i++) g.fields[i].transfer = saved[i];
	halo_wait(g);
}

__global__ void po_classify_kernel(int32_t* cls, const int32_t* slot_by_id, const uint64_t* ids, size_t n,
                                   uint64_t last, size_t n_local, int32_t value) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		if (id == 0 || id > last) continue;
		const int32_t sl = slot_by_id[id];
		if (sl >= 0 && size_t(sl) < n_local) cls[sl] = value;  // only local cells (is_local, 839-878)
	}
}

static int po_field(Grid& g, const char* name, size_t elem) {
	Field f;
	f.name = name;
	f.elem = elem;
	f.transfer = false;
	g.fields.push_back(std::move(f));
	Field& nf = g.fields.back();
	nf.data.alloc(g.n_slots * elem);
	if (nf.data.n) HIP_CHECK(hipMemset(nf.data.p, 0, nf.data.n));
	return int(g.fields.size() - 1);
}

static void po_ensure_fields(Grid& g) {
	PoissonState& P = g.po;
	if (P.type >= 0) return;
	P.type = po_field(g, "poisson.type", 4);
	P.p0 = po_field(g, "poisson.p0", 8);
	P.p1 = po_field(g, "poisson.p1", 8);
	P.r0 = po_field(g, "poisson.r0", 8);
	P.r1 = po_field(g, "poisson.r1", 8);
	P.ap0 = po_field(g, "poisson.A_dot_p0", 8);
	P.best = po_field(g, "poisson.best_solution", 8);
	P.sf = po_field(g, "poisson.scaling_factor", 8);
	static const char* fn[6] = {"poisson.f_x_neg", "poisson.f_x_pos", "poisson.f_y_neg",
	                            "poisson.f_y_pos", "poisson.f_z_neg", "poisson.f_z_pos"};
	for (int k = 0; k < 6; k++) P.f[k] = po_field(g, fn[k], 8);
}

static PoArrays po_arrays(Grid& g) {
	PoissonState& P = g.po;
	auto d = [&](int f) { return (double*)field(g, f).data.p; };
	PoArrays a{};
	a.ell = P.ell.p;
	a.fine = P.fine.p;
	a.type = (const int32_t*)field(g, P.type).data.p;
	a.rhs = d(P.rhs);
	a.sol = d(P.sol);
	a.best = d(P.best);
	a.p0 = d(P.p0);
	a.p1 = d(P.p1);
	a.r0 = d(P.r0);
	a.r1 = d(P.r1);
	a.ap0 = d(P.ap0);
	a.sf = d(P.sf);
	for (int k = 0; k < 6; k++) a.f[k] = d(P.f[k]);
	return a;
}

// cache_system_info 827-971
static void po_cache(Grid& g, int rhs, int sol, const uint64_t* solve, size_t ns, const uint64_t* skip, size_t nk) {
	DX_REQUIRE(field(g, rhs).elem == 8 && field(g, sol).elem == 8, "rhs and solution must be fp64 fields");
	po_ensure_fields(g);
	PoissonState& P = g.po;
	P.rhs = rhs;
	P.sol = sol;
	ensure_face(g);
	hipStream_t s = g.s_comp;
	const size_t nl = g.n_local;
	int32_t* type = (int32_t*)field(g, P.type).data.p;
	// classify: local cells boundary, then skip, then solve (836-878)
	k_fill_i32(type, nl, 1, s);
	for (int pass = 0; pass < 2; pass++) {
		const uint64_t* ids = pass == 0 ? skip : solve;
		const size_t n = pass == 0 ? nk : ns;
		if (!n) continue;
		DBuf<uint64_t> d;
		d.alloc(n);
		HIP_CHECK(hipMemcpyAsync(d.p, ids, n * 8, hipMemcpyHostToDevice, s));
		po_classify_kernel<<<grid_for(n, 256), 256, 0, s>>>(type, g.slot_by_id.p, d.p, n, g.m.last, nl,
		                                                    pass == 0 ? 2 : 0);
		HIP_CHECK(hipGetLastError());
		HIP_CHECK(hipStreamSynchronize(s));
	}
	halo_only(g, {P.type});  // TYPE (880-881)
	DBuf<int32_t> cls;
	cls.alloc(g.n_slots);
	if (g.n_slots) HIP_CHECK(hipMemcpyAsync(cls.p, type, g.n_slots * 4, hipMemcpyDeviceToDevice, s));
	P.ell.alloc(6 * nl);
	P.fine.alloc(g.face_fine.n);
	const PoArrays a = po_arrays(g);
	k_po_cache(g.m, g.l0, g.slot_ids.p, cls.p, g.face_ell.p, g.face_fine.p, nl, P.ell.p, P.fine.p, type, a, s);
	HIP_CHECK(hipStreamSynchronize(s));
	std::vector<int> geo{P.sf};  // GEOMETRY (969-970)
	for (int k = 0; k < 6; k++) geo.push_back(P.f[k]);
	halo_only(g, geo);
	HIP_CHECK(hipStreamSynchronize(s));
	P.valid = true;
}

// sums of the last phase -> (all ranks) -> scalar control flow
static void po_reduce(Grid& g, int k, unsigned nb, const PoParams& prm, int stage) {
	PoissonState& P = g.po;
	const bool one = g.size == 1;
	k_po_reduce(k, P.part.p, nb, P.red.p, P.st.p, prm, stage, one, g.s_comp);
	if (!one) {
		DX_REQUIRE(g.comm, "Poisson solve on several ranks needs a communicator");
		NCCL_CHECK(ncclAllReduce(P.red.p, P.red.p, size_t(k), ncclFloat64, ncclSum, g.comm, g.s_comp));
		k_po_scalar(P.red.p, P.st.p, prm, stage, g.s_comp);
	}
}

static PoScalars po_read_scalars(Grid& g) {
	PoScalars h{};
	HIP_CHECK(hipMemcpyAsync(&h, g.po.st.p, sizeof(h), hipMemcpyDeviceToHost, g.s_comp));
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
	return h;
}

// solve 251-522 / solve_failsafe 531-634 after po_cache; the host only
// enqueues kernels and polls the device's `done` flag every few iterations
static PoScalars po_solve(Grid& g, const PoParams& prm, bool failsafe) {
	PoissonState& P = g.po;
	DX_REQUIRE(P.valid, "Poisson system not cached for the current mesh");
	hipStream_t s = g.s_comp;
	const size_t n = g.n_local;
	const unsigned nb = k_po_blocks(n);
	if (P.part.n < 2 * size_t(nb)) P.part.alloc(2 * size_t(nb));
	P.red.alloc(2);
	P.st.alloc(1);
	const PoArrays a = po_arrays(g);
	const int poll = 8;
	if (!failsafe) {
		halo_only(g, {P.sol});  // INIT (983-984)
		k_po_phase(PO_PHASE_INIT, a, n, prm, P.st.p, P.part.p, s);
		po_reduce(g, 1, nb, prm, PO_STAGE_INIT);
		for (unsigned it = 0; it < prm.max_it; it++) {
			halo_only(g, {P.p0, P.p1});  // SOLVING (283-284)
			k_time_begin(g);
			k_po_phase(PO_PHASE_A, a, n, prm, P.st.p, P.part.p, s);
			k_time_end(g);
			po_reduce(g, 2, nb, prm, PO_STAGE_A);
			k_time_begin(g);
			k_po_phase(PO_PHASE_B, a, n, prm, P.st.p, P.part.p, s);
			k_time_end(g);
			po_reduce(g, 1, nb, prm, PO_STAGE_B);
			k_time_begin(g);
			k_po_phase(PO_PHASE_C, a, n, prm, P.st.p, P.part.p, s);
			k_time_end(g);
			if ((it + 1) % poll == 0 && po_read_scalars(g).done) break;
		}
		k_po_phase(PO_PHASE_FINISH, a, n, prm, P.st.p, P.part.p, s);
	} else {
		k_po_reduce(1, P.part.p, 0, P.red.p, P.st.p, prm, PO_STAGE_JACOBI_INIT, true, s);
		for (unsigned it = 0; it < prm.max_it; it++) {
			halo_only(g, {P.sol});  // INIT (545, 551)
			k_time_begin(g);
			k_po_phase(PO_PHASE_JACOBI, a, n, prm, P.st.p, P.part.p, s);
			k_time_end(g);
			po_reduce(g, 1, nb, prm, PO_STAGE_JACOBI);
			k_po_phase(PO_PHASE_JACOBI_COPY, a, n, prm, P.st.p, P.part.p, s);
			if ((it + 1) % poll == 0 && po_read_scalars(g).done) break;
		}
	}
	return po_read_scalars(g);
}

}  // namespace dccrgx

// ============================================================================
// C ABI
// ============================================================================
using namespace dccrgx;

struct dccrgx_grid {
	Grid g;
};

#define GRID_OR_FAIL(gp) \
	if (!(gp)) throw Error(DCCRGX_EINVAL, "null grid"); \
	Grid& g = (gp)->g

static int copy_out_u64(const std::vector<uint64_t>& v, uint64_t* out, size_t cap, size_t* n) {
	if (n) *n = v.size();
	if (v.size() > cap || (!out && !v.empty())) return DCCRGX_ERANGE;
	if (!v.empty()) std::memcpy(out, v.data(), v.size() * 8);
	return DCCRGX_OK;
}

extern "C" {

const char* dccrgx_last_error(void) { return g_last_error.c_str(); }
int dccrgx_abi_version(void) { return 1; }

int dccrgx_get_unique_id(void* out) {
	return guard([&] {
		ncclUniqueId id;
		NCCL_CHECK(ncclGetUniqueId(&id));
		std::memcpy(out, &id, sizeof(id));
		return 0;
	});
}

int dccrgx_create(int rank, int size, int device, const void* nccl_id, dccrgx_grid** out) {
	return guard([&] {
		DX_REQUIRE(out && size >= 1 && rank >= 0 && rank < size, "invalid rank/size");
		HIP_CHECK(hipSetDevice(device));
		auto* h = new dccrgx_grid();
		Grid& g = h->g;
		g.rank = rank;
		g.size = size;
		g.device = device;
		HIP_CHECK(hipStreamCreateWithFlags(&g.s_comp, hipStreamNonBlocking));
		HIP_CHECK(hipStreamCreateWithFlags(&g.s_comm, hipStreamNonBlocking));
		HIP_CHECK(hipEventCreateWithFlags(&g.ev_comp, hipEventDisableTiming));
		HIP_CHECK(hipEventCreateWithFlags(&g.ev_halo, hipEventDisableTiming));
		if (size > 1 && nccl_id) {  // without an id: a detached view of one rank (no halo transport)
			ncclUniqueId id;
			std::memcpy(&id, nccl_id, sizeof(id));
			NCCL_CHECK(ncclCommInitRank(&g.comm, size, id, rank));
		}
		*out = h;
		return 0;
	});
}

int dccrgx_destroy(dccrgx_grid* gp) {
	return guard([&] {
		if (!gp) return 0;
		Grid& g = gp->g;
		(void)hipDeviceSynchronize();
		drain_timing(g);
		if (g.comm) ncclCommDestroy(g.comm);
		if (g.ev_comp) (void)hipEventDestroy(g.ev_comp);
		if (g.ev_halo) (void)hipEventDestroy(g.ev_halo);
		if (g.ev_fork) (void)hipEventDestroy(g.ev_fork);
		if (g.ev_join) (void)hipEventDestroy(g.ev_join);
		if (g.s_adv2) (void)hipStreamDestroy(g.s_adv2);
		if (g.s_comp) (void)hipStreamDestroy(g.s_comp);
		if (g.s_comm) (void)hipStreamDestroy(g.s_comm);
		delete gp;
		return 0;
	});
}

int dccrgx_set_initial_length(dccrgx_grid* gp, const uint64_t length[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_initial_length after initialize");
		for (int d = 0; d < 3; d++) DX_REQUIRE(length[d] > 0, "grid length must be > 0");
		for (int d = 0; d < 3; d++) g.len[d] = length[d];
		return 0;
	});
}

int dccrgx_set_maximum_refinement_level(dccrgx_grid* gp, int level) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_maximum_refinement_level after initialize");
		// dccrg_mapping.hpp:316-329: the largest level whose ids fit in 64 bits
		const double gl = double(g.len[0]) * double(g.len[1]) * double(g.len[2]);
		int lvl = 0;
		double cur = 0;
		while (cur <= double(~uint64_t(0))) {
			cur += gl * std::pow(8.0, double(lvl));
			lvl++;
		}
		const int maxpos = lvl - 2;
		if (level < 0) level = maxpos;
		DX_REQUIRE(level <= maxpos && level < kMaxLevels, "refinement level too large for the grid");
		g.R = level;
		return 0;
	});
}

int dccrgx_get_maximum_refinement_level(dccrgx_grid* gp, int* level) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		*level = g.R;
		return 0;
	});
}

int dccrgx_set_periodic(dccrgx_grid* gp, int x, int y, int z) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_periodic after initialize");
		g.per[0] = x != 0;
		g.per[1] = y != 0;
		g.per[2] = z != 0;
		return 0;
	});
}

int dccrgx_set_neighborhood_length(dccrgx_grid* gp, unsigned length) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_neighborhood_length after initialize");
		DX_REQUIRE(length <= 8, "neighborhood length > 8 not supported");
		g.hood_len = length;
		return 0;
	});
}

static void init_impl(Grid& g) {
	DX_REQUIRE(!g.initialized, "already initialized");
	map_init(g.m, g.len, g.R, g.per);
	std::vector<int32_t> h(3 * 2000);
	const int nh = default_hood(g.hood_len, h.data());
	g.hood.assign(h.begin(), h.begin() + 3 * nh);
	g.hood_to.resize(g.hood.size());
	for (size_t i = 0; i < g.hood.size(); i++) g.hood_to[i] = -g.hood[i];
	upload(g.d_hood, g.hood, g.s_comp);
	upload(g.d_hood_to, g.hood_to, g.s_comp);
	g.leaves.clear();
	g.owners.clear();
	rebuild(g);
	g.initialized = true;
}

int dccrgx_initialize(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		init_impl(g);
		return 0;
	});
}

int dccrgx_set_geometry(dccrgx_grid* gp, const double start[3], const double l0[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (int d = 0; d < 3; d++) DX_REQUIRE(l0[d] > 0, "cell length must be > 0");
		for (int d = 0; d < 3; d++) {
			g.start[d] = start[d];
			g.l0[d] = l0[d];
		}
		return 0;
	});
}

int dccrgx_geometry_batch(dccrgx_grid* gp, const uint64_t* ids, size_t n, double* center, double* length) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(ids || !n, "null ids");
		const double nan = std::numeric_limits<double>::quiet_NaN();
		for (size_t i = 0; i < n; i++) {
			uint64_t ind[3];
			const int lvl = map_indices(g.m, ids[i], ind[0], ind[1], ind[2]);
			for (int d = 0; d < 3; d++) {
				double L = nan, c = nan;
				if (lvl >= 0) {  // dccrg_cartesian_geometry.hpp:299-303, 334-359
					L = g.l0[d] * (1.0 / double(uint64_t(1) << lvl));
					c = g.start[d] + double(ind[d]) * g.l0[d] / double(uint64_t(1) << g.R) + L / 2;
				}
				if (length) length[3 * i + d] = L;
				if (center) center[3 * i + d] = c;
			}
		}
		return 0;
	});
}

uint64_t dccrgx_get_cell_from_indices(dccrgx_grid* gp, const uint64_t ind[3], int level) {
	if (!gp) return error_cell;
	MapCtx m;
	map_init(m, gp->g.len, gp->g.R, gp->g.per);
	return map_from_indices(m, ind[0], ind[1], ind[2], level);
}

int dccrgx_get_indices(dccrgx_grid* gp, uint64_t cell, uint64_t ind[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		MapCtx m;
		map_init(m, g.len, g.R, g.per);
		const int l = map_indices(m, cell, ind[0], ind[1], ind[2]);
		return l < 0 ? DCCRGX_ENOTFOUND : 0;
	});
}

int dccrgx_get_refinement_level(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return -1;
	MapCtx m;
	map_init(m, gp->g.len, gp->g.R, gp->g.per);
	return map_level(m, cell);
}

uint64_t dccrgx_get_last_cell(dccrgx_grid* gp) {
	if (!gp) return 0;
	MapCtx m;
	map_init(m, gp->g.len, gp->g.R, gp->g.per);
	return m.last;
}

int dccrgx_get_counts(dccrgx_grid* gp, size_t* ni, size_t* no, size_t* nr, size_t* ns) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (ni) *ni = g.n_inner;
		if (no) *no = g.n_outer;
		if (nr) *nr = g.n_recv;
		if (ns) *ns = g.n_slots;
		return 0;
	});
}

int dccrgx_get_cells(dccrgx_grid* gp, int which, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		const auto& ids = slot_ids_host(g);
		std::vector<uint64_t> v;
		switch (which) {
		case DCCRGX_CELLS_LOCAL: v.assign(ids.begin(), ids.begin() + g.n_local); break;
		case DCCRGX_CELLS_INNER: v.assign(ids.begin(), ids.begin() + g.n_inner); break;
		case DCCRGX_CELLS_OUTER: v.assign(ids.begin() + g.n_inner, ids.begin() + g.n_local); break;
		case DCCRGX_CELLS_REMOTE: v.assign(ids.begin() + g.n_local, ids.end()); break;
		case DCCRGX_CELLS_ALL: v = ids; break;
		default: throw Error(DCCRGX_EINVAL, "invalid selection");
		}
		std::sort(v.begin(), v.end());
		return copy_out_u64(v, out, cap, n);
	});
}

int dccrgx_get_slot_ids(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		return copy_out_u64(slot_ids_host(g), out, cap, n);
	});
}

int dccrgx_get_neighbors_of(dccrgx_grid* gp, uint64_t cell, uint64_t* ids, int32_t* offs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const int64_t s = slot_of(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		ensure_csr(g);
		uint32_t be[2];
		HIP_CHECK(hipMemcpy(be, g.nof_ptr.p + s, 8, hipMemcpyDeviceToHost));
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		if (k) {
			HIP_CHECK(hipMemcpy(ids, g.nof_id.p + be[0], k * 8, hipMemcpyDeviceToHost));
			if (offs) HIP_CHECK(hipMemcpy(offs, g.nof_off.p + 3 * size_t(be[0]), k * 12, hipMemcpyDeviceToHost));
		}
		return 0;
	});
}

int dccrgx_get_neighbors_to(dccrgx_grid* gp, uint64_t cell, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const int64_t s = slot_of(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		ensure_csr(g);
		uint32_t be[2];
		HIP_CHECK(hipMemcpy(be, g.nto_ptr.p + s, 8, hipMemcpyDeviceToHost));
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		if (k) HIP_CHECK(hipMemcpy(ids, g.nto_id.p + be[0], k * 8, hipMemcpyDeviceToHost));
		return 0;
	});
}

int dccrgx_get_face_neighbors_of(dccrgx_grid* gp, uint64_t cell, uint64_t* ids, int32_t* dirs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const int64_t s = slot_of(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		ensure_face(g);
		uint32_t be[2];
		HIP_CHECK(hipMemcpy(be, g.face_ptr.p + s, 8, hipMemcpyDeviceToHost));
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		std::vector<int32_t> ent(k);
		if (k) HIP_CHECK(hipMemcpy(ent.data(), g.face_ent.p + be[0], k * 4, hipMemcpyDeviceToHost));
		const auto& sid = slot_ids_host(g);
		static const int dmap[6] = {-1, +1, -2, +2, -3, +3};
		for (size_t i = 0; i < k; i++) {
			ids[i] = sid[size_t(ent[i] >> 3)];
			if (dirs) dirs[i] = dmap[ent[i] & 7];
		}
		return 0;
	});
}

/* bulk download of a local CSR in slot order:
   kind 0 neighbors_of (aux = offsets x3), 1 neighbors_to, 2 face (aux = dir),
   3 iterator neighbors_of (ids only) */
int dccrgx_download_csr(dccrgx_grid* gp, int kind, uint32_t* ptr, uint64_t* ids, int32_t* aux, size_t cap,
                        size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const size_t nl = g.n_local;
		const uint32_t* dptr = nullptr;
		if (kind == 2) {
			ensure_face(g);
			dptr = g.face_ptr.p;
		} else {
			ensure_csr(g);
			dptr = kind == 0 ? g.nof_ptr.p : kind == 1 ? g.nto_ptr.p : g.it_ptr.p;
		}
		std::vector<uint32_t> hp = download(dptr, nl + 1, g.s_comp);
		const size_t tot = hp[nl];
		if (n) *n = tot;
		if (tot > cap) return DCCRGX_ERANGE;
		std::memcpy(ptr, hp.data(), (nl + 1) * 4);
		if (!tot) return 0;
		const auto& sid = slot_ids_host(g);
		if (kind == 0) {
			HIP_CHECK(hipMemcpy(ids, g.nof_id.p, tot * 8, hipMemcpyDeviceToHost));
			if (aux) HIP_CHECK(hipMemcpy(aux, g.nof_off.p, tot * 12, hipMemcpyDeviceToHost));
		} else if (kind == 1) {
			HIP_CHECK(hipMemcpy(ids, g.nto_id.p, tot * 8, hipMemcpyDeviceToHost));
		} else if (kind == 2) {
			std::vector<int32_t> ent = download(g.face_ent.p, tot, g.s_comp);
			static const int dmap[6] = {-1, +1, -2, +2, -3, +3};
			for (size_t i = 0; i < tot; i++) {
				ids[i] = sid[size_t(ent[i] >> 3)];
				if (aux) aux[i] = dmap[ent[i] & 7];
			}
		} else {
			std::vector<int32_t> sl = download(g.it_slot.p, tot, g.s_comp);
			for (size_t i = 0; i < tot; i++) ids[i] = sid[size_t(sl[i])];
		}
		return 0;
	});
}

int dccrgx_is_local(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return 0;
	return host_owner(gp->g, cell) == gp->g.rank ? 1 : 0;
}

int dccrgx_get_process(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return -1;
	return host_owner(gp->g, cell);
}

int64_t dccrgx_get_slot(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return -1;
	try {
		return slot_of(gp->g, cell);
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return -1;
	}
}

int dccrgx_get_peers(dccrgx_grid* gp, int32_t* peers, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (n) *n = g.peers.size();
		if (g.peers.size() > cap) return DCCRGX_ERANGE;
		for (size_t i = 0; i < g.peers.size(); i++) peers[i] = g.peers[i];
		return 0;
	});
}

int dccrgx_get_cells_to_send(dccrgx_grid* gp, int peer, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		auto it = g.send_ids.find(peer);
		static const std::vector<uint64_t> empty;
		return copy_out_u64(it == g.send_ids.end() ? empty : it->second, ids, cap, n);
	});
}

int dccrgx_get_cells_to_receive(dccrgx_grid* gp, int peer, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		auto it = g.recv_ids.find(peer);
		static const std::vector<uint64_t> empty;
		return copy_out_u64(it == g.recv_ids.end() ? empty : it->second, ids, cap, n);
	});
}

int dccrgx_get_cell_process(dccrgx_grid* gp, uint64_t* ids, int32_t* owners, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		// an implicit (initial uniform) mesh stays implicit: the structured
		// sweeps key on it
		const bool imp = implicit_mesh(g);
		const uint64_t total = imp ? g.m.first[1] - 1 : g.leaves.size();
		*n = size_t(total);
		if (!ids) return 0;
		if (cap < total) return int(DCCRGX_ERANGE);
		if (!imp) {
			std::copy(g.leaves.begin(), g.leaves.end(), ids);
			if (owners) std::copy(g.owners.begin(), g.owners.end(), owners);
			return 0;
		}
		for (int p = 0; p < g.size; p++) {
			uint64_t f, c;
			block_range(total, uint64_t(g.size), uint64_t(p), f, c);
			for (uint64_t i = 0; i < c; i++) {
				ids[f - 1 + i] = f + i;
				if (owners) owners[f - 1 + i] = p;
			}
		}
		return 0;
	});
}

int dccrgx_get_number_of_update_cells(dccrgx_grid* gp, uint64_t* ns, uint64_t* nr) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (ns) *ns = g.n_send_total;
		if (nr) *nr = g.n_recv;
		return 0;
	});
}

int dccrgx_refine_completely(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		if (host_owner(g, cell) != g.rank) return DCCRGX_ENOTFOUND;  // 2449-2459: only local cells
		if (map_level(g.m, cell) >= g.R) return 0;                   // 2474-2477: no-op at max level
		g.refine_requests.push_back(cell);
		return 0;
	});
}

int dccrgx_stop_refining(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		g.last_new_cells = stop_refining_impl(g);
		if (!out) {
			if (n) *n = g.last_new_cells.size();
			return 0;
		}
		return copy_out_u64(g.last_new_cells, out, cap, n);
	});
}

int dccrgx_get_new_cells(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		return copy_out_u64(g.last_new_cells, out, cap, n);
	});
}

int dccrgx_set_cells(dccrgx_grid* gp, const uint64_t* ids, const int32_t* owners, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		std::vector<uint64_t> L(ids, ids + n);
		std::vector<int32_t> O(owners, owners + n);
		for (size_t i = 0; i < n; i++) {
			DX_REQUIRE(L[i] != error_cell && L[i] <= g.m.last, "invalid cell id");
			DX_REQUIRE(i == 0 || L[i] > L[i - 1], "cell ids must be strictly ascending");
			DX_REQUIRE(O[i] >= 0 && O[i] < g.size, "invalid owner");
		}
		g.leaves.swap(L);
		g.owners.swap(O);
		rebuild(g);
		return 0;
	});
}

int dccrgx_pin(dccrgx_grid* gp, uint64_t cell, int process) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(process >= 0 && process < g.size, "invalid process");
		if (host_owner(g, cell) != g.rank) return DCCRGX_ENOTFOUND;
		g.pins[cell] = process;
		return 0;
	});
}

int dccrgx_unpin(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		g.pins.erase(cell);
		return 0;
	});
}

int dccrgx_add_neighborhood(dccrgx_grid* gp, int id, const int32_t* offsets, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		// add_neighborhood 6383-6520: the reference returns false for these
		DX_REQUIRE(id != DCCRGX_DEFAULT_HOOD, "neighborhood id is the default id");
		DX_REQUIRE(!g.uhoods.count(id), "neighborhood id already exists");
		for (size_t i = 0; i < n; i++) {
			const int32_t* o = offsets + 3 * i;
			if (g.hood_len > 0) {
				for (int d = 0; d < 3; d++)
					DX_REQUIRE(unsigned(std::abs(o[d])) <= g.hood_len, "offset outside the default neighborhood");
				DX_REQUIRE(o[0] || o[1] || o[2], "offset (0, 0, 0)");
			} else {
				int zeros = 0;
				for (int d = 0; d < 3; d++) {
					zeros += o[d] == 0;
					DX_REQUIRE(std::abs(o[d]) <= 1, "offset outside the face neighborhood");
				}
				DX_REQUIRE(zeros == 2, "face neighborhood offsets must be unit face offsets");
			}
		}
		UserHood& h = g.uhoods[id];
		h.of.assign(offsets, offsets + 3 * n);
		h.to.resize(h.of.size());
		for (size_t i = 0; i < h.of.size(); i++) h.to[i] = -h.of[i];
		upload(h.d_of, h.of, g.s_comp);
		upload(h.d_to, h.to, g.s_comp);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		ensure_uhood(g, id);
		return 0;
	});
}

int dccrgx_remove_neighborhood(dccrgx_grid* gp, int id) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		g.uhoods.erase(id);
		return 0;
	});
}

int dccrgx_get_user_neighbors(dccrgx_grid* gp, int id, uint64_t cell, int kind, uint64_t* ids, int32_t* offs,
                              size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (!g.uhoods.count(id)) return DCCRGX_ENOTFOUND;
		const int64_t s = slot_of(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		UserHood& h = ensure_uhood(g, id);
		const DBuf<uint32_t>& ptr = kind == 0 ? h.nof_ptr : h.nto_ptr;
		uint32_t be[2];
		HIP_CHECK(hipMemcpy(be, ptr.p + s, 8, hipMemcpyDeviceToHost));
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		if (k) {
			HIP_CHECK(hipMemcpy(ids, (kind == 0 ? h.nof_id.p : h.nto_id.p) + be[0], k * 8, hipMemcpyDeviceToHost));
			if (offs && kind == 0)
				HIP_CHECK(hipMemcpy(offs, h.nof_off.p + 3 * size_t(be[0]), k * 12, hipMemcpyDeviceToHost));
		}
		return 0;
	});
}

int dccrgx_get_user_update_list(dccrgx_grid* gp, int id, int peer, int receive, uint64_t* ids, size_t cap,
                                size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (!g.uhoods.count(id)) return DCCRGX_ENOTFOUND;
		UserHood& h = ensure_uhood(g, id);
		const auto& mp = receive ? h.recv_ids : h.send_ids;
		auto it = mp.find(peer);
		static const std::vector<uint64_t> empty;
		return copy_out_u64(it == mp.end() ? empty : it->second, ids, cap, n);
	});
}

int dccrgx_update_copies_of_remote_neighbors_hood(dccrgx_grid* gp, int id) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (id == DCCRGX_DEFAULT_HOOD) {
			halo_start(g);
			halo_wait(g);
		} else {
			uhood_halo(g, id);
		}
		return 0;
	});
}

int dccrgx_balance_load_to(dccrgx_grid* gp, const uint64_t* ids, const int32_t* new_owner, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		materialize(g);
		DX_REQUIRE(n == g.leaves.size(), "balance_load_to needs one owner per leaf of the grid");
		for (size_t i = 0; i < n; i++) DX_REQUIRE(ids[i] == g.leaves[i], "leaf ids must be the grid's, ascending");
		migrate_to(g, std::vector<int32_t>(new_owner, new_owner + n));
		return 0;
	});
}

int dccrgx_balance_load(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		balance_load_impl(g);
		return 0;
	});
}

// --------------------------------------------------------------------------- grid files
// save_grid_data / load_grid_data (dccrg.hpp:1089-1740, 1742-2425), file
// layout 1104-1120: `offset` bytes left alone, the caller's header, uint64
// 0x1234567890abcdef, the grid block (Mapping::write dccrg_mapping.hpp:576 =
// 3 x uint64 length + int max_ref_lvl; the neighborhood length as unsigned;
// Grid_Topology::write dccrg_topology.hpp:144 = 3 x uint8 periodic;
// Cartesian_Geometry::write dccrg_cartesian_geometry.hpp:618 = int id 1 +
// 3 x double start + 3 x double level-0 length), uint64 total cells, per
// cell (uint64 id, uint64 absolute byte offset of its data) rank by rank,
// then the cell data in the same order.  A cell's data = the payload of
// every transferred field, in field order (the reference writes what
// get_mpi_datatype describes at save time).  Cells of a rank in ascending id
// (the reference: get_cells() order).  Every rank writes its own records with
// pwrite at offsets it derives from the global leaf/owner knowledge, so no
// collective is needed.
static constexpr uint64_t kEndianCheck = 0x1234567890abcdefULL;
static constexpr int kCartesianGeometryId = 1;

static std::vector<uint8_t> grid_block(const Grid& g) {
	std::vector<uint8_t> b;
	auto put = [&b](const void* p, size_t n) {
		const uint8_t* q = static_cast<const uint8_t*>(p);
		b.insert(b.end(), q, q + n);
	};
	put(g.len, 24);
	const int32_t R = g.R;
	put(&R, 4);
	const uint32_t hood = g.hood_len;
	put(&hood, 4);
	const uint8_t per[3] = {uint8_t(g.per[0] != 0), uint8_t(g.per[1] != 0), uint8_t(g.per[2] != 0)};
	put(per, 3);
	const int32_t gid = kCartesianGeometryId;
	put(&gid, 4);
	put(g.start, 24);
	put(g.l0, 24);
	return b;
}

static void pwrite_all(int fd, const void* p, size_t n, uint64_t off) {
	const uint8_t* q = static_cast<const uint8_t*>(p);
	while (n) {
		const ssize_t w = ::pwrite(fd, q, n, off_t(off));
		DX_REQUIRE(w > 0, "grid file write failed");
		q += w;
		n -= size_t(w);
		off += uint64_t(w);
	}
}

static void pread_all(int fd, void* p, size_t n, uint64_t off) {
	uint8_t* q = static_cast<uint8_t*>(p);
	while (n) {
		const ssize_t r = ::pread(fd, q, n, off_t(off));
		DX_REQUIRE(r > 0, "grid file truncated");
		q += r;
		n -= size_t(r);
		off += uint64_t(r);
	}
}

// cells per rank (global leaf knowledge, like cell_process)
static std::vector<uint64_t> rank_counts(Grid& g) {
	std::vector<uint64_t> c(size_t(g.size), 0);
	if (implicit_mesh(g)) {
		const uint64_t total = g.m.first[1] - 1;
		for (int p = 0; p < g.size; p++) {
			uint64_t f, n;
			block_range(total, uint64_t(g.size), uint64_t(p), f, n);
			c[size_t(p)] = n;
		}
	} else {
		for (int32_t o : g.owners) c[size_t(o)]++;
	}
	return c;
}

int dccrgx_save_grid_data(dccrgx_grid* gp, const char* path, uint64_t offset, const void* header,
                          size_t header_bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		std::vector<Field*> tf;
		size_t bpc = 0;
		for (auto& f : g.fields)
			if (f.transfer) {
				tf.push_back(&f);
				bpc += f.elem;
			}
		const int fd = ::open(path, O_CREAT | O_WRONLY, 0644);
		DX_REQUIRE(fd >= 0, std::string("cannot open grid file ") + path);
		struct Closer {
			int fd;
			~Closer() { ::close(fd); }
		} closer{fd};
		uint64_t off = offset;
		if (g.rank == 0 && header_bytes) pwrite_all(fd, header, header_bytes, off);
		off += header_bytes;
		if (g.rank == 0) pwrite_all(fd, &kEndianCheck, 8, off);
		off += 8;
		const std::vector<uint8_t> block = grid_block(g);
		if (g.rank == 0) pwrite_all(fd, block.data(), block.size(), off);
		off += block.size();
		const std::vector<uint64_t> cnt = rank_counts(g);
		uint64_t total = 0, before = 0;
		for (int p = 0; p < g.size; p++) {
			if (p < g.rank) before += cnt[size_t(p)];
			total += cnt[size_t(p)];
		}
		if (g.rank == 0) pwrite_all(fd, &total, 8, off);
		off += 8;
		const uint64_t list0 = off, data0 = off + 16 * total;
		// local cells ascending, with their slots
		const size_t nl = g.n_local;
		const auto& sid = slot_ids_host(g);
		std::vector<uint32_t> order(nl);
		for (size_t i = 0; i < nl; i++) order[i] = uint32_t(i);
		std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return sid[a] < sid[b]; });
		std::vector<uint64_t> list(2 * nl);
		for (size_t i = 0; i < nl; i++) {
			list[2 * i] = sid[order[i]];
			list[2 * i + 1] = data0 + bpc * (before + i);
		}
		if (nl) pwrite_all(fd, list.data(), 16 * nl, list0 + 16 * before);
		if (nl && bpc) {
			std::vector<uint8_t> data(nl * bpc);
			size_t fo = 0;
			for (Field* f : tf) {
				const std::vector<uint8_t> h = download(f->data.p, nl * f->elem, g.s_comp);
				for (size_t i = 0; i < nl; i++)
					std::memcpy(&data[i * bpc + fo], &h[size_t(order[i]) * f->elem], f->elem);
				fo += f->elem;
			}
			pwrite_all(fd, data.data(), data.size(), data0 + bpc * before);
		}
		return 0;
	});
}

int dccrgx_load_grid_data(dccrgx_grid* gp, const char* path, uint64_t offset, size_t header_bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "load_grid_data initializes the grid: call it instead of initialize");
		const int fd = ::open(path, O_RDONLY);
		DX_REQUIRE(fd >= 0, std::string("cannot open grid file ") + path);
		struct Closer {
			int fd;
			~Closer() { ::close(fd); }
		} closer{fd};
		uint64_t off = offset + header_bytes, endian = 0;
		pread_all(fd, &endian, 8, off);
		DX_REQUIRE(endian == kEndianCheck, "grid file endianness check failed");
		off += 8;
		uint8_t blk[87];
		pread_all(fd, blk, sizeof(blk), off);
		off += sizeof(blk);
		uint64_t len[3];
		int32_t R, gid;
		uint32_t hood;
		double start[3], l0[3];
		std::memcpy(len, blk, 24);
		std::memcpy(&R, blk + 24, 4);
		std::memcpy(&hood, blk + 28, 4);
		std::memcpy(&gid, blk + 35, 4);
		std::memcpy(start, blk + 39, 24);
		std::memcpy(l0, blk + 63, 24);
		DX_REQUIRE(gid == kCartesianGeometryId, "grid file geometry is not Cartesian_Geometry");
		for (int d = 0; d < 3; d++) {
			g.len[d] = len[d];
			g.per[d] = blk[32 + d] != 0;
			g.start[d] = start[d];
			g.l0[d] = l0[d];
		}
		g.R = R;
		g.hood_len = hood;
		init_impl(g);
		uint64_t total = 0;
		pread_all(fd, &total, 8, off);
		off += 8;
		std::vector<uint64_t> list(2 * total);
		if (total) pread_all(fd, list.data(), 16 * total, off);
		std::vector<std::pair<uint64_t, uint64_t>> cells(total);
		for (size_t i = 0; i < total; i++) cells[i] = {list[2 * i], list[2 * i + 1]};
		std::sort(cells.begin(), cells.end());
		// owners as load_cells (3647) produces them: the level-0 block
		// partition (create_level_0_cells), refined cells inherit it
		const uint64_t n0 = g.m.first[1] - 1;
		std::vector<uint64_t> ids(total);
		std::vector<int32_t> own(total);
		for (size_t i = 0; i < total; i++) {
			ids[i] = cells[i].first;
			const uint64_t l0p = map_level0_parent(g.m, ids[i]);
			DX_REQUIRE(l0p != error_cell, "grid file lists an invalid cell");
			for (int p = 0; p < g.size; p++) {
				uint64_t f, c;
				block_range(n0, uint64_t(g.size), uint64_t(p), f, c);
				if (l0p >= f && l0p < f + c) own[i] = p;
			}
		}
		g.leaves = ids;
		g.owners = own;
		rebuild(g);
		// payloads of the local cells
		std::vector<Field*> tf;
		size_t bpc = 0;
		for (auto& f : g.fields)
			if (f.transfer) {
				tf.push_back(&f);
				bpc += f.elem;
			}
		const size_t nl = g.n_local;
		if (!nl || !bpc) return 0;
		const auto& sid = slot_ids_host(g);
		std::vector<uint64_t> where(nl);
		uint64_t lo = ~uint64_t(0), hi = 0;
		for (size_t i = 0; i < nl; i++) {
			auto it = std::lower_bound(cells.begin(), cells.end(), std::make_pair(sid[i], uint64_t(0)));
			DX_REQUIRE(it != cells.end() && it->first == sid[i], "local cell missing from grid file");
			where[i] = it->second;
			lo = std::min(lo, where[i]);
			hi = std::max(hi, where[i] + bpc);
		}
		std::vector<uint8_t> raw(hi - lo);
		pread_all(fd, raw.data(), raw.size(), lo);
		size_t fo = 0;
		for (Field* f : tf) {
			std::vector<uint8_t> h(nl * f->elem);
			for (size_t i = 0; i < nl; i++) std::memcpy(&h[i * f->elem], &raw[where[i] - lo + fo], f->elem);
			HIP_CHECK(hipMemcpy(f->data.p, h.data(), h.size(), hipMemcpyHostToDevice));
			fo += f->elem;
		}
		return 0;
	});
}

int dccrgx_add_field(dccrgx_grid* gp, const char* name, size_t elem, int transfer, int* fid) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(elem > 0, "element size must be > 0");
		Field f;
		f.name = name ? name : "";
		f.elem = elem;
		f.transfer = transfer != 0;
		g.fields.push_back(std::move(f));
		Field& nf = g.fields.back();
		if (g.initialized) {
			nf.data.alloc(g.n_slots * elem);
			if (nf.data.n) HIP_CHECK(hipMemset(nf.data.p, 0, nf.data.n));
		}
		*fid = int(g.fields.size() - 1);
		return 0;
	});
}

int dccrgx_set_field_transfer(dccrgx_grid* gp, int fid, int transfer) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		field(g, fid).transfer = transfer != 0;
		return 0;
	});
}

int dccrgx_field_device_ptr(dccrgx_grid* gp, int fid, void** ptr) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		*ptr = field(g, fid).data.p;
		return 0;
	});
}

int dccrgx_field_upload(dccrgx_grid* gp, int fid, size_t slot0, size_t n, const void* host) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = field(g, fid);
		DX_REQUIRE(slot0 + n <= g.n_slots, "slot range out of bounds");
		if (n) HIP_CHECK(hipMemcpy(f.data.p + slot0 * f.elem, host, n * f.elem, hipMemcpyHostToDevice));
		return 0;
	});
}

int dccrgx_field_download(dccrgx_grid* gp, int fid, size_t slot0, size_t n, void* host) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = field(g, fid);
		DX_REQUIRE(slot0 + n <= g.n_slots, "slot range out of bounds");
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		if (n) HIP_CHECK(hipMemcpy(host, f.data.p + slot0 * f.elem, n * f.elem, hipMemcpyDeviceToHost));
		return 0;
	});
}

int dccrgx_update_copies_of_remote_neighbors(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_start(g);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_start_remote_neighbor_copy_updates(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_start(g);
		return 0;
	});
}

int dccrgx_wait_remote_neighbor_copy_update_receives(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_wait_remote_neighbor_copy_update_sends(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_wait_remote_neighbor_copy_updates(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_gol_step(dccrgx_grid* gp, int sf, int region) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = field(g, sf);
		DX_REQUIRE(f.elem == 4, "game of life state must be a 4-byte field");
		ensure_scratch(g, f);
		size_t s0, s1;
		region_range(g, region, s0, s1);
		if (s1 <= s0) return 0;
		const bool structured = g.R == 0 && g.hood_len == 1 && g.n_outer == 0 && g.n_slots == g.n_local && s0 == 0 &&
		                        s1 == g.n_local && implicit_mesh(g) && g.size == 1;
		k_time_begin(g);
		if (structured) {
			k_gol_structured((const uint32_t*)f.data.p, (uint32_t*)f.scratch.p, g.len, g.per, g.s_comp);
		} else {
			ensure_csr(g);
			k_gol_csr((const uint32_t*)f.data.p, (uint32_t*)f.scratch.p, g.it_ptr.p, g.it_slot.p, s0, s1, g.s_comp);
		}
		k_time_end(g);
		return 0;
	});
}

int dccrgx_gol_commit(dccrgx_grid* gp, int sf) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		commit(g, field(g, sf));
		return 0;
	});
}

// get_live_neighbors of tests/game_of_life/solve.hpp:37-170, split at its
// halo: phase 0 = the collect loop (46-110), phase 1 = spread + rule
// (113-167); see gol_amr.hip
int dccrgx_gol_amr(dccrgx_grid* gp, int phase, int sf, int lf, int region) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(phase == 0 || phase == 1, "phase must be 0 (collect) or 1 (spread)");
		Field& st = field(g, sf);
		Field& ls = field(g, lf);
		DX_REQUIRE(st.elem == 4, "game of life state must be a 4-byte field");
		DX_REQUIRE(ls.elem == 64, "live level-0 neighbor list must be a 64-byte field (8 x uint64)");
		size_t s0, s1;
		region_range(g, region, s0, s1);
		if (s1 <= s0) return 0;
		ensure_csr(g);
		DBuf<int> err;
		err.alloc(1);
		HIP_CHECK(hipMemsetAsync(err.p, 0, sizeof(int), g.s_comp));
		k_time_begin(g);
		if (g.gol_l0p.n < g.n_slots) g.gol_l0p.alloc(g.n_slots);
		k_gol_amr(phase, g.m, g.slot_ids.p, g.n_slots, g.gol_l0p.p, (uint32_t*)st.data.p, (uint64_t*)ls.data.p,
		          g.nof_ptr.p, g.nof_slot.p, s0, s1, err.p, g.s_comp);
		k_time_end(g);
		int h = 0;
		HIP_CHECK(hipMemcpyAsync(&h, err.p, sizeof(int), hipMemcpyDeviceToHost, g.s_comp));
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		DX_REQUIRE(!(h & 1), "No more room in live neighbor list (more than 8 live level-0 neighbors)");
		DX_REQUIRE(!(h & 2), "a dead neighbor's level-0 parent was recorded alive (siblings disagree)");
		return 0;
	});
}

static void adv_fields(Grid& g, const int fids[7], const double* f[7]) {
	for (int k = 0; k < 7; k++) {
		Field& F = field(g, fids[k]);
		DX_REQUIRE(F.elem == 8, "advection fields must be fp64");
		f[k] = (const double*)F.data.p;
	}
}

int dccrgx_advection_step(dccrgx_grid* gp, const int fids[7], double dt, int region) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		ensure_face(g);
		const double* f[7];
		adv_fields(g, fids, f);
		Field& rho = field(g, fids[0]);
		ensure_scratch(g, rho);
		size_t s0, s1;
		region_range(g, region, s0, s1);
		if (s1 <= s0) return 0;
		k_time_begin(g);
		if (adv_variant() == 11) {
			ensure_tiles(g);
			// tiles never straddle the inner / outer runs
			if (s0 < g.n_inner) k_advection_tiles(f, (double*)rho.scratch.p, g, 0, dt, g.s_comp);
			if (s1 > g.n_inner) k_advection_tiles(f, (double*)rho.scratch.p, g, 1, dt, g.s_comp);
		} else {
			k_advection(f, (double*)rho.scratch.p, g.face_ptr.p, g.face_ent.p, g.face_ell.p, g.face_fine.p, s0, s1, dt,
			            g.s_comp);
		}
		k_time_end(g);
		return 0;
	});
}

int dccrgx_advection_layout(dccrgx_grid* gp, uint64_t out[10]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(out, "null output");
		ensure_tiles(g);
		const uint64_t nt = g.n_tiles_inner + g.n_tiles_outer;
		uint32_t entries = 0;
		HIP_CHECK(hipMemcpy(&entries, g.face_ptr.p + g.n_local, 4, hipMemcpyDeviceToHost));
		const uint64_t n = g.n_local;
		out[0] = uint64_t(g.tile);
		out[1] = nt;
		out[2] = g.total_ext;
		out[3] = g.max_ext;
		out[4] = g.n_fine_faces;
		out[5] = entries;
		// 64 B per cell (7 fp64 fields read, density written) +
		// the face CSR (4 B per entry + 4 B row pointer)
		out[6] = 64 * n + 4 * (n + 1) + 4 * uint64_t(entries);
		out[7] = 64 * n;
		out[8] = g.tcount[0] + g.tcount[1];
		out[9] = 512 * (g.tcount[0] + g.tcount[1]);
		return 0;
	});
}

int dccrgx_advection_commit(dccrgx_grid* gp, int df) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		commit(g, field(g, df));
		return 0;
	});
}

// tests/advection/initialize.hpp:36-82 + Cartesian_Geometry get_center /
// get_length (dccrg_cartesian_geometry.hpp:282-362), evaluated on the host
// with the reference's expression order so the initial state is bitwise the
// reference's.
int dccrgx_advection_initialize(dccrgx_grid* gp, const int fids[7]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		// local cells and remote copies alike: the analytic initial state of a
		// remote copy is what initialize() + update_copies_of_remote_neighbors()
		// with transfer_all_data = true would deliver (initialize.hpp:80)
		const auto& ids = slot_ids_host(g);
		const size_t n = g.n_slots;
		std::vector<double> a[7];
		for (auto& v : a) v.resize(n);
		for (size_t i = 0; i < n; i++) {
			uint64_t ind[3];
			const int lvl = map_indices(g.m, ids[i], ind[0], ind[1], ind[2]);
			const double sf = 1.0 / double(uint64_t(1) << lvl);
			double L[3], c[3];
			for (int d = 0; d < 3; d++) L[d] = g.l0[d] * sf;
			for (int d = 0; d < 3; d++)
				c[d] = g.start[d] + double(ind[d]) * g.l0[d] / double(uint64_t(1) << g.R) + L[d] / 2;
			const double radius = 0.15;
			const double hr = std::min(std::sqrt(std::pow(c[0] - 0.25, 2.0) + std::pow(c[1] - 0.5, 2.0)), radius) / radius;
			a[0][i] = 0.25 * (1 + std::cos(M_PI * hr));
			a[1][i] = -c[1] + 0.5;
			a[2][i] = +c[0] - 0.5;
			a[3][i] = 0;
			a[4][i] = L[0];
			a[5][i] = L[1];
			a[6][i] = L[2];
		}
		for (int k = 0; k < 7; k++) {
			Field& F = field(g, fids[k]);
			DX_REQUIRE(F.elem == 8, "advection fields must be fp64");
			if (n) HIP_CHECK(hipMemcpy(F.data.p, a[k].data(), n * 8, hipMemcpyHostToDevice));
		}
		return 0;
	});
}

int dccrgx_advection_max_time_step(dccrgx_grid* gp, const int fids[7], double* out) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const double* f[7];
		adv_fields(g, fids, f);
		const size_t nb = 512;
		DBuf<double> part;
		part.alloc(nb);
		k_adv_dt(f, g.n_local, part.p, nb, g.s_comp);
		auto h = download(part.p, nb, g.s_comp);
		*out = *std::min_element(h.begin(), h.end());
		return 0;
	});
}

int dccrgx_advection_refine_candidates(dccrgx_grid* gp, int df, double diff_increase, double diff_threshold,
                                       uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		ensure_face(g);
		Field& F = field(g, df);
		DBuf<uint64_t> d;
		d.alloc(g.n_local + 1);
		const size_t k = k_adv_candidates(g.m, (const double*)F.data.p, g.face_ptr.p, g.face_ent.p, g.slot_ids.p,
		                                  g.n_local, diff_increase, diff_threshold, d.p, g.s_comp);
		auto v = download(d.p, k, g.s_comp);
		std::sort(v.begin(), v.end());
		return copy_out_u64(v, out, cap, n);
	});
}

int dccrgx_allreduce_f64(dccrgx_grid* gp, double* v, int count, int op) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		allreduce_f64(g, v, count, op);
		return 0;
	});
}

int dccrgx_barrier(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		double z = 0;
		allreduce_f64(g, &z, 1, 0);
		return 0;
	});
}

int dccrgx_synchronize(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		HIP_CHECK(hipStreamSynchronize(g.s_comm));
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		return 0;
	});
}

void* dccrgx_compute_stream(dccrgx_grid* gp) { return gp ? (void*)gp->g.s_comp : nullptr; }

int dccrgx_kernel_timing(dccrgx_grid* gp, int enable, double* total_ms, int64_t* count) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		drain_timing(g);
		if (total_ms) *total_ms = g.timed_ms;
		if (count) *count = g.timed_count;
		if (enable == 1) {
			g.timing = true;
			g.timed_ms = 0;
			g.timed_count = 0;
		} else if (enable == 0) {
			g.timing = false;
		}
		return 0;
	});
}

// ---- Poisson (tests/poisson/poisson_solve.hpp) ----------------------------
int dccrgx_poisson_cache(dccrgx_grid* gp, int rhs_field, int solution_field, const uint64_t* solve_cells,
                         size_t n_solve, const uint64_t* skip_cells, size_t n_skip) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "grid not initialized");
		DX_REQUIRE((solve_cells || !n_solve) && (skip_cells || !n_skip), "null cell list");
		po_cache(g, rhs_field, solution_field, solve_cells, n_solve, skip_cells, n_skip);
		return 0;
	});
}

int dccrgx_poisson_solve(dccrgx_grid* gp, unsigned max_iterations, unsigned min_iterations, double stop_residual,
                         double p_of_norm, double stop_after_residual_increase, int failsafe, unsigned* iterations,
                         double* residual) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(p_of_norm > 0, "p_of_norm must be > 0");
		// solve() is a do-while (279-506): at least one iteration
		const unsigned max_it = failsafe ? max_iterations : std::max(1u, max_iterations);
		const PoParams prm{max_it, min_iterations, stop_residual, p_of_norm, stop_after_residual_increase};
		const PoScalars st = po_solve(g, prm, failsafe != 0);
		if (iterations) *iterations = st.iteration;
		if (residual) *residual = failsafe ? st.norm : st.residual_min;
		return 0;
	});
}

int dccrgx_poisson_field(dccrgx_grid* gp, const char* name, int* fid) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(name && fid, "null argument");
		DX_REQUIRE(g.po.type >= 0, "Poisson system not cached yet");
		const std::string want = std::string("poisson.") + name;
		for (size_t i = 0; i < g.fields.size(); i++)
			if (g.fields[i].name == want) {
				*fid = int(i);
				return 0;
			}
		throw Error(DCCRGX_ENOTFOUND, "no Poisson field " + std::string(name));
	});
}

}  // extern "C"
