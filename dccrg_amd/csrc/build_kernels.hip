// Device construction of the neighbor structures (replaces the reference's
// per-cell std::map walks: update_neighbors_ dccrg.hpp:9313-9458,
// initialize_neighbors 8240-8289, find_neighbors_of 4339-4680,
// find_neighbors_to 4708-4861, update_remote_neighbor_info 8992-9270,
// recalculate_neighbor_update_send_receive_lists 8590-8752,
// get_face_neighbors_of 2806-2933, update_cell_pointers 11314-11628) and of
// the rank's leaf knowledge (dccrgx_mesh.hpp: hash table, ghost region,
// refinement closure induce_refines 9591-9720, execute_refines 10104-10554).
//
// Layout: one wavefront (64 lanes) per cell; lanes own stencil items (or
// neighbors_to candidates); per-cell output positions come from a wave
// prefix scan (shuffle) / ballot + popcount compaction, so every row is
// written in the reference's order without atomics.  Existence / owner /
// slot of a leaf is one 16-byte probe sequence in the rank's hash table (or
// the block-partition formula on the initial level-0 grid).
#include <cstring>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_merge.hpp>

#include <algorithm>
#include <cstdlib>
#include <functional>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

constexpr int WAVE = 64;
constexpr int kMaxNtoLds = 8192;  // u64 entries of the neighbors_to dedupe (64 KB of LDS)

__device__ __forceinline__ int lane_id() { return threadIdx.x & (WAVE - 1); }

__device__ __forceinline__ uint64_t lanemask_lt() {
	const int l = lane_id();
	return l == 0 ? 0ull : (~0ull >> (64 - l));
}

__device__ __forceinline__ int wave_incl_scan(int v) {
	const int l = lane_id();
	for (int d = 1; d < WAVE; d <<= 1) {
		const int t = __shfl_up(v, d, WAVE);
		if (l >= d) v += t;
	}
	return v;
}

__device__ __forceinline__ int wave_sum(int v) {
	for (int d = WAVE / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, WAVE);
	return v;
}

__device__ void cell_coords(const MapCtx& m, uint64_t id, uint64_t c[3], int& lvl) {
	lvl = map_indices(m, id, c[0], c[1], c[2]);
}

// --------------------------------------------------------------------------
__global__ void fill_i32_kernel(int32_t* p, size_t n, int32_t v) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		p[i] = v;
}

__global__ void iota_u64_kernel(uint64_t* out, uint64_t first, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = first + i;
}

// insert (id, owner, slot = -1); keys are unique
__global__ void hash_insert_kernel(HashEntry* tab, uint64_t mask, uint32_t shift, const uint64_t* ids,
                                   const int32_t* owners, int32_t owner_const, size_t n, size_t slot_upto) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		uint64_t h = hash_home(id, shift);
		for (;;) {
			unsigned long long* kp = reinterpret_cast<unsigned long long*>(&tab[h].key);
			const unsigned long long prev = atomicCAS(kp, 0ull, (unsigned long long)id);
			if (prev == 0ull || prev == id) {
				tab[h].owner = owners ? owners[i] : owner_const;
				tab[h].slot = i < slot_upto ? int32_t(i) : -1;
				break;
			}
			h = (h + 1) & mask;
		}
	}
}

// per refinement level the smallest and largest id of a list (one atomic
// per block and bound, the block's bounds reduced in LDS first)
__global__ __launch_bounds__(256) void level_ranges_kernel(MapCtx m, const uint64_t* __restrict__ ids, size_t n,
                                                           unsigned long long* lo, unsigned long long* hi) {
	__shared__ unsigned long long slo[kRangeLevels], shi[kRangeLevels];
	if (threadIdx.x < kRangeLevels) {
		slo[threadIdx.x] = ~0ull;
		shi[threadIdx.x] = 0ull;
	}
	__syncthreads();
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		const int L = map_level(m, id);
		if (L < 0 || L >= kRangeLevels) continue;
		atomicMin(&slo[L], (unsigned long long)id);
		atomicMax(&shi[L], (unsigned long long)id);
	}
	__syncthreads();
	if (threadIdx.x < kRangeLevels && shi[threadIdx.x]) {
		atomicMin(lo + threadIdx.x, slo[threadIdx.x]);
		atomicMax(hi + threadIdx.x, shi[threadIdx.x]);
	}
}

// every id of the list written by one thread: no atomics
__global__ void range_insert_kernel(int2* __restrict__ rmap, DevMesh M, const uint64_t* __restrict__ ids,
                                    const int32_t* __restrict__ owners, size_t n, size_t slot_upto) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int64_t k = dm_range_index(M, ids[i]);
		if (k >= 0) rmap[k] = make_int2(owners ? owners[i] : -2, i < slot_upto ? int32_t(i) : -1);
	}
}

__global__ void range_clear_kernel(int2* __restrict__ rmap, DevMesh M, const uint64_t* __restrict__ ids, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int64_t k = dm_range_index(M, ids[i]);
		if (k >= 0) rmap[k] = make_int2(-1, -1);
	}
}

__global__ void hash_set_slots_kernel(DevMesh M, const uint64_t* slot_ids, size_t n, int32_t* err) {
	if (M.rmap) {
		int2* rmap = const_cast<int2*>(M.rmap);
		for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
			const int64_t k = dm_range_index(M, slot_ids[i]);
			if (k < 0 || rmap[k].x < 0) atomicExch(err, 1);
			else rmap[k].y = int32_t(i);
		}
		return;
	}
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = slot_ids[i];
		uint64_t h = hash_home(id, M.shift);
		HashEntry* tab = const_cast<HashEntry*>(M.tab);
		for (;;) {
			const uint64_t k = tab[h].key;
			if (k == id) {
				tab[h].slot = int32_t(i);
				break;
			}
			if (k == 0) {
				atomicExch(err, 1);
				break;
			}
			h = (h + 1) & M.mask;
		}
	}
}

__global__ void lookup_kernel(DevMesh M, const uint64_t* ids, size_t n, int32_t* owner, int32_t* slot) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		if (owner) owner[i] = dm_owner(M, id);
		if (slot) slot[i] = dm_slot(M, id);
	}
}

// --------------------------------------------------------------------------
// Pass 1: does a local cell have any remote neighbors_of / neighbors_to?
// (update_remote_neighbor_info 8992-9095).  One wave per cell.
__global__ void remote_flags_kernel(MapCtx m, const int32_t* hood, const int32_t* hood_to, int nh, DevMesh M, int rank,
                                    const uint64_t* cells, size_t n, uint32_t* flag) {
	const DevExists ex{M};
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t w = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; w < n; w += waves) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, cells[w], c, lvl);
		bool remote = false;
		for (int k = lane_id(); k < nh; k += WAVE) {
			uint64_t w[3];
			const int kind = nof_item_case(m, c, lvl, hood + 3 * k, ex, w);
			for (int i = 0; i < item_count(kind); i++) {
				const int32_t ow = dm_owner(M, item_id(m, lvl, hood + 3 * k, kind, w, i, nullptr));
				if (ow >= 0 && ow != rank) remote = true;
			}
		}
		for (int k = lane_id(); k < 10 * nh; k += WAVE) {
			const uint64_t f = nto_candidate(m, c, lvl, hood_to, nh, k, ex);
			if (f != error_cell && dm_owner(M, f) != rank) remote = true;
		}
		const bool any = __any(remote);
		if (lane_id() == 0) flag[w] = any ? 1u : 0u;
	}
}

// The same classification with one thread per cell, for small hoods (the
// face hood: 6 neighbors_of items + 60 neighbors_to candidates per cell): a
// wave then holds 64 cells whose lookups are independent, where the wave per
// cell above issues its cell's 66 lookups as two dependent rounds and leaves
// 62 lanes idle in the second.  The walk stops at the first remote neighbor.
__global__ __launch_bounds__(256) void remote_flags_thread_kernel(MapCtx m, const int32_t* __restrict__ hood,
                                                                  const int32_t* __restrict__ hood_to, int nh,
                                                                  DevMesh M, int rank, const uint64_t* __restrict__ cells,
                                                                  size_t n, uint32_t* __restrict__ flag,
                                                                  const uint8_t* __restrict__ near, uint64_t near_lo,
                                                                  uint64_t near_n) {
	const DevExists ex{M};
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (near) {
			const uint64_t q = map_level0_parent(m, cells[i]) - near_lo;
			if (q < near_n && !near[q]) {
				flag[i] = 0u;
				continue;
			}
		}
		uint64_t c[3];
		int lvl;
		cell_coords(m, cells[i], c, lvl);
		bool remote = false;
		for (int k = 0; k < nh && !remote; k++) {
			uint64_t w[3];
			const int kind = nof_item_case(m, c, lvl, hood + 3 * k, ex, w);
			for (int j = 0; j < item_count(kind); j++) {
				const int32_t ow = dm_owner(M, item_id(m, lvl, hood + 3 * k, kind, w, j, nullptr));
				if (ow >= 0 && ow != rank) remote = true;
			}
		}
		for (int k = 0; k < 10 * nh && !remote; k++) {
			const uint64_t f = nto_candidate(m, c, lvl, hood_to, nh, k, ex);
			if (f != error_cell && dm_owner(M, f) != rank) remote = true;
		}
		flag[i] = remote ? 1u : 0u;
	}
}

__global__ void assign_slots_kernel(const uint32_t* flag, const uint32_t* scan_outer, size_t n, size_t n_inner,
                                    const uint64_t* cells, uint64_t* slot_ids) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const size_t so = scan_outer[i];
		const size_t s = flag[i] ? n_inner + so : i - so;
		slot_ids[s] = cells[i];
	}
}

// --------------------------------------------------------------------------
// neighbors_to of one cell, sorted & deduplicated in LDS by the wave.
// Returns the unique count; when `out` is non-null, writes them ascending.
__device__ int nto_row(const MapCtx& m, const int32_t* hood_to, int nh, const DevExists& ex, const uint64_t c[3],
                       int lvl, uint64_t* lds, int cap, uint64_t* out) {
	int cnt = 0;
	const int seg_lo[3] = {0, nh, 9 * nh};
	const int seg_hi[3] = {nh, 9 * nh, 10 * nh};
	const bool seg_on[3] = {lvl > 0, lvl < m.R, true};
	for (int sgi = 0; sgi < 3; sgi++) {
		if (!seg_on[sgi]) continue;
		for (int k0 = seg_lo[sgi]; k0 < seg_hi[sgi]; k0 += WAVE) {
			const int k = k0 + lane_id();
			uint64_t f = error_cell;
			if (k < seg_hi[sgi]) f = nto_candidate(m, c, lvl, hood_to, nh, k, ex);
			const bool valid = f != error_cell;
			const uint64_t mask = __ballot(valid);
			const int pos = cnt + __popcll(mask & lanemask_lt());
			if (valid && pos < cap) lds[pos] = f;
			cnt += __popcll(mask);
		}
	}
	if (cnt > cap) cnt = cap;  // cap >= 10*nh (max_hood_items): never reached
	int P = 1;
	while (P < cnt) P <<= 1;
	for (int i = cnt + lane_id(); i < P; i += WAVE) lds[i] = ~0ull;
	__syncthreads();
	for (int k = 2; k <= P; k <<= 1) {
		for (int j = k >> 1; j > 0; j >>= 1) {
			for (int i = lane_id(); i < P; i += WAVE) {
				const int ixj = i ^ j;
				if (ixj > i) {
					const uint64_t a = lds[i], b = lds[ixj];
					const bool up = (i & k) == 0;
					if ((a > b) == up) {
						lds[i] = b;
						lds[ixj] = a;
					}
				}
			}
			__syncthreads();
		}
	}
	int base = 0;
	for (int i0 = 0; i0 < cnt; i0 += WAVE) {
		const int i = i0 + lane_id();
		const bool u = i < cnt && (i == 0 || lds[i] != lds[i - 1]);
		const uint64_t mask = __ballot(u);
		if (out && u) out[base + __popcll(mask & lanemask_lt())] = lds[i];
		base += __popcll(mask);
	}
	__syncthreads();
	return base;
}

// per-row counts in slot order (one wave = one block per row)
__global__ void count_rows_kernel(MapCtx m, const int32_t* hood, const int32_t* hood_to, int nh, DevMesh M,
                                  const uint64_t* slot_ids, size_t row0, size_t nrows, uint32_t* nof_cnt,
                                  uint32_t* nto_cnt, int cap) {
	extern __shared__ uint64_t lds[];
	const DevExists ex{M};
	for (size_t r = blockIdx.x; r < nrows; r += gridDim.x) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[row0 + r], c, lvl);
		int n = 0;
		for (int k = lane_id(); k < nh; k += WAVE) {
			uint64_t w[3];
			n += item_count(nof_item_case(m, c, lvl, hood + 3 * k, ex, w));
		}
		n = wave_sum(n);
		const int t = nto_row(m, hood_to, nh, ex, c, lvl, lds, cap, nullptr);
		if (lane_id() == 0) {
			nof_cnt[r] = uint32_t(n);
			nto_cnt[r] = uint32_t(t);
		}
	}
}

// neighbors_of rows in stencil order (4339-4680 semantics, see dccrgx_neighbors.hpp)
__global__ void fill_nof_kernel(MapCtx m, const int32_t* hood, int nh, DevMesh M, const uint64_t* slot_ids, size_t row0,
                                size_t nrows, const uint32_t* ptr, uint64_t* ids, int32_t* offs) {
	const DevExists ex{M};
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t r = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; r < nrows; r += waves) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[row0 + r], c, lvl);
		size_t base = ptr[r];
		for (int k0 = 0; k0 < nh; k0 += WAVE) {
			const int k = k0 + lane_id();
			uint64_t w[3] = {0, 0, 0};
			const int kind = k < nh ? nof_item_case(m, c, lvl, hood + 3 * k, ex, w) : 0;
			const int no = item_count(kind);
			const int incl = wave_incl_scan(no);
			const size_t pos = base + size_t(incl - no);
			for (int i = 0; i < no; i++) {
				int32_t off[3];
				ids[pos + i] = item_id(m, lvl, hood + 3 * k, kind, w, i, off);
				offs[3 * (pos + i) + 0] = off[0];
				offs[3 * (pos + i) + 1] = off[1];
				offs[3 * (pos + i) + 2] = off[2];
			}
			base += size_t(__shfl(incl, WAVE - 1, WAVE));
		}
	}
}

__global__ void fill_nto_kernel(MapCtx m, const int32_t* hood_to, int nh, DevMesh M, const uint64_t* slot_ids,
                                size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids, int cap) {
	extern __shared__ uint64_t lds[];
	const DevExists ex{M};
	for (size_t r = blockIdx.x; r < nrows; r += gridDim.x) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[row0 + r], c, lvl);
		nto_row(m, hood_to, nh, ex, c, lvl, lds, cap, ids + ptr[r]);
	}
}

// --------------------------------------------------------------------------
// owned-elsewhere entries as keys owner * stride + id, or (owners != nullptr,
// ids too deep for such keys) as the id in keys[] and the owner in owners[]
__global__ void extract_remote_kernel(const uint64_t* ids, size_t n, DevMesh M, int rank, uint64_t stride,
                                      uint64_t* keys, uint32_t* owners, unsigned long long* counter) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		if (id == error_cell) continue;
		const int32_t o = dm_owner(M, id);
		if (o < 0 || o == rank) continue;
		const unsigned long long at = atomicAdd(counter, 1ull);
		if (owners) {
			keys[at] = id;
			owners[at] = uint32_t(o);
		} else {
			keys[at] = uint64_t(o) * stride + id;
		}
	}
}

__global__ void extract_send_kernel(const uint64_t* nto_id, const uint32_t* nto_ptr, const uint64_t* slot_ids,
                                    size_t row0, size_t nrows, DevMesh M, int rank, uint64_t stride, uint64_t* keys,
                                    uint32_t* owners, unsigned long long* counter) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		const uint64_t self = slot_ids[row0 + r];
		for (uint32_t e = nto_ptr[r]; e < nto_ptr[r + 1]; e++) {
			const int32_t o = dm_owner(M, nto_id[e]);
			if (o < 0 || o == rank) continue;
			const unsigned long long at = atomicAdd(counter, 1ull);
			if (owners) {
				keys[at] = self;
				owners[at] = uint32_t(o);
			} else {
				keys[at] = uint64_t(o) * stride + self;
			}
		}
	}
}

// the remote ids of a neighbors_to list whose (owner, id) key is not among
// the sorted neighbors_of keys: cells that only this rank's cells' neighbors_to
// reach (the reference's remote neighbors_to-only copies)
__global__ void extract_extra_kernel(const uint64_t* ids, size_t n, DevMesh M, int rank, uint64_t stride,
                                     const uint64_t* of_keys, size_t n_of, uint64_t* out, unsigned long long* counter,
                                     const unsigned long long* n_of_dev = nullptr) {
	if (n_of_dev) n_of = size_t(*n_of_dev);
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		if (id == error_cell) continue;
		const int32_t o = dm_owner(M, id);
		if (o < 0 || o == rank) continue;
		const uint64_t key = uint64_t(o) * stride + id;
		size_t lo = 0, hi = n_of;
		while (lo < hi) {
			const size_t mid = (lo + hi) >> 1;
			if (of_keys[mid] < key)
				lo = mid + 1;
			else
				hi = mid;
		}
		if (lo < n_of && of_keys[lo] == key) continue;
		out[atomicAdd(counter, 1ull)] = id;
	}
}

// 1 where a (owner, id) pair differs from the one before it
__global__ void pair_heads_kernel(const uint64_t* ids, const uint32_t* owners, size_t n, uint8_t* head) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		head[i] = (i == 0 || ids[i] != ids[i - 1] || owners[i] != owners[i - 1]) ? 1 : 0;
}

__global__ void lookup_slots_kernel(const uint64_t* ids, size_t n, DevMesh M, int32_t* out, int32_t* err) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int32_t s = dm_slot(M, ids[i]);
		out[i] = s;
		if (s < 0) atomicExch(err, 1);
	}
}

// (id, offset) order of std::set<pair<uint64_t, array<int, 3>>>
__device__ __forceinline__ bool key_less(uint64_t ia, const int32_t* oa, uint64_t ib, const int32_t* ob) {
	if (ia != ib) return ia < ib;
	if (oa[0] != ob[0]) return oa[0] < ob[0];
	if (oa[1] != ob[1]) return oa[1] < ob[1];
	return oa[2] < ob[2];
}

// iterator neighbor range cell.neighbors_of (update_cell_pointers
// 11451-11500): the distinct (id, offset) pairs of the row, the ones whose id
// is not in the row's neighbors_to first ("only_of"), then the ones whose id
// is ("both"), each class in (id, offset) order.  One wave per row, one lane
// per entry; the loops over the row's other entries are wave-uniform, so
// every lane reads the same entry (one broadcast load).
// Pass 0 classifies every entry (0 repeat of an earlier pair, 1 only_of,
// 2 both) and counts the distinct pairs; pass 1 places each entry at its
// rank within its class.
__device__ __forceinline__ bool same_pair(const uint64_t* id, const int32_t* off, uint32_t i, uint32_t j) {
	return id[i] == id[j] && off[3 * i] == off[3 * j] && off[3 * i + 1] == off[3 * j + 1] &&
	       off[3 * i + 2] == off[3 * j + 2];
}

__global__ void iterator_class_kernel(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                                      const uint32_t* nto_ptr, const uint64_t* nto_id, size_t nrows, uint8_t* cls,
                                      uint32_t* it_cnt) {
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t r = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; r < nrows; r += waves) {
		const uint32_t b = nof_ptr[r], e = nof_ptr[r + 1];
		const uint32_t tb = nto_ptr[r], te = nto_ptr[r + 1];
		uint32_t n_all = 0;
		for (uint32_t j0 = b; j0 < e; j0 += WAVE) {
			const uint32_t j = j0 + lane_id();
			uint8_t c = 0;
			if (j < e) {
				bool dup = false;
				for (uint32_t i = b; i < j && !dup; i++) dup = same_pair(nof_id, nof_off, i, j);
				if (!dup) {
					const uint64_t id = nof_id[j];
					uint32_t lo = tb, hi = te;
					while (lo < hi) {
						const uint32_t mid = (lo + hi) >> 1;
						if (nto_id[mid] < id) lo = mid + 1;
						else hi = mid;
					}
					c = (lo < te && nto_id[lo] == id) ? 2 : 1;
				}
				cls[j] = c;
			}
			n_all += uint32_t(__popcll(__ballot(c != 0)));
		}
		if (lane_id() == 0) it_cnt[r] = n_all;
	}
}

__global__ void iterator_fill_kernel(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                                     const int32_t* nof_slot, const uint8_t* cls, size_t nrows, const uint32_t* it_ptr,
                                     int32_t* it_slot, int32_t* it_off) {
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t r = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; r < nrows; r += waves) {
		const uint32_t b = nof_ptr[r], e = nof_ptr[r + 1];
		uint32_t n_only = 0;
		for (uint32_t j0 = b; j0 < e; j0 += WAVE) {
			const uint32_t j = j0 + lane_id();
			n_only += uint32_t(__popcll(__ballot(j < e && cls[j] == 1)));
		}
		for (uint32_t j0 = b; j0 < e; j0 += WAVE) {
			const uint32_t j = j0 + lane_id();
			const uint8_t cj = j < e ? cls[j] : 0;
			uint32_t rank = 0;
			for (uint32_t i = b; i < e; i++)
				if (cj != 0 && cls[i] == cj && key_less(nof_id[i], nof_off + 3 * i, nof_id[j], nof_off + 3 * j)) rank++;
			if (cj == 0) continue;
			const uint32_t pos = it_ptr[r] + (cj == 2 ? n_only : 0u) + rank;
			it_slot[pos] = nof_slot[j];
			if (it_off) {
				it_off[3 * pos] = nof_off[3 * j];
				it_off[3 * pos + 1] = nof_off[3 * j + 1];
				it_off[3 * pos + 2] = nof_off[3 * j + 2];
			}
		}
	}
}

// The fixed-width face table (get_face_neighbors_of semantics), one thread
// per local slot: ell[6 r + d] = the slot of the single (same-size or
// coarser) face neighbor in direction d, -1 none, or -2 - f for the finer
// face f whose 4 slots are fine[4 f ..] in the reference's order.  Finer faces
// are numbered in (row, direction) order: face_table_kernel writes the
// directions with one neighbor and appends the finer ones' keys
// (row << 3 | d); after a sort of the keys face_fine_kernel probes those again.
// A single neighbor without a slot sets *err.
struct SlotExists {
	DevMesh M;
	mutable int32_t slot = -1;
	// DevExists's answer, and the slot of the cell it found
	__device__ __forceinline__ bool operator()(uint64_t id) const {
		slot = -1;
		if (id == 0 || id > M.last) return false;
		if (M.implicit) {
			if (id > M.bp.n0) return false;
			slot = dm_slot(M, id);
			return true;
		}
		int32_t o, sl;
		if (!dm_lookup(M, id, o, sl)) return false;
		slot = sl;
		return o >= 0;
	}
};

__device__ __forceinline__ uint64_t spread3(uint64_t v) {
	v &= 0x1FFFFFull;
	v = (v | (v << 32)) & 0x1F00000000FFFFull;
	v = (v | (v << 16)) & 0x1F0000FF0000FFull;
	v = (v | (v << 8)) & 0x100F00F00F00F00Full;
	v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
	v = (v | (v << 2)) & 0x1249249249249249ull;
	return v;
}

__device__ __forceinline__ uint64_t morton3(const uint64_t c[3]) {
	return spread3(c[0]) | (spread3(c[1]) << 1) | (spread3(c[2]) << 2);
}

// morton: the rows [0, nrows) are Morton-ordered runs [0, run1) and [run1,
// nrows) (k_morton_sort of rebuild step 2).  Then a same-size face neighbor
// is predicted at the row its Morton distance away - exact whenever every
// leaf between the two has that size - and taken when the row holds its id:
// a same-size leaf is the one face neighbor in that direction (no finer or
// coarser probe needed).  o6[dir] = -1 (no face neighbor), the predicted row,
// or kFaceMiss (the probes of face_dir decide).
constexpr int32_t kFaceMiss = -3;
__device__ __forceinline__ void face_predict(const MapCtx& m, const uint64_t* __restrict__ slot_ids, size_t r,
                                             size_t run1, size_t nrows, uint64_t id, const uint64_t c[3], int lvl,
                                             int32_t o6[6]) {
	int32_t h[6];
	uint64_t want[6], got[6];
	bool probe[6];
	const int sh = 3 * (m.R - lvl);
	const uint64_t len = uint64_t(1) << (m.R - lvl);
	const uint64_t key = morton3(c) >> sh;
	const int64_t lo = r < run1 ? 0 : int64_t(run1), hi = r < run1 ? int64_t(run1) : int64_t(nrows);
	// the neighbor's id and Morton key from this cell's: one step along d is
	// +-stride[d] in the id and a dilated +-1 in the key (no re-interleave,
	// no index -> id products); a periodic wrap takes the general form
	const uint64_t lx = m.len[0] << lvl, ly = m.len[1] << lvl;
	const uint64_t stride[3] = {1, lx, lx * ly};
#pragma unroll
	for (int dir = 0; dir < 6; dir++) {
		const int d = dir >> 1;
		uint64_t p[3];
		h[dir] = -1;
		want[dir] = ~uint64_t(0);
		probe[dir] = face_probe(m, c, lvl, dir, p);
		if (!probe[dir]) continue;
		p[d] &= ~(len - 1);  // the other two are c's, aligned
		const uint64_t M = uint64_t(0x1249249249249249ull) << d, u = uint64_t(1) << d;
		uint64_t nkey;
		if ((dir & 1) ? p[d] == c[d] + len : p[d] + len == c[d])
			nkey = (dir & 1) ? ((((key | ~M) + u) & M) | (key & ~M)) : ((((key & M) - u) & M) | (key & ~M));
		else
			nkey = morton3(p) >> sh;
		const int64_t q = int64_t(r) + (int64_t(nkey) - int64_t(key));
		if (q >= lo && q < hi) {
			h[dir] = int32_t(q);
			want[dir] = id + ((p[d] >> (m.R - lvl)) - (c[d] >> (m.R - lvl))) * stride[d];
		}
	}
	// the six row loads in flight together
#pragma unroll
	for (int dir = 0; dir < 6; dir++) got[dir] = h[dir] >= 0 ? slot_ids[h[dir]] : 0;
#pragma unroll
	for (int dir = 0; dir < 6; dir++)
		o6[dir] = !probe[dir] ? -1 : (h[dir] >= 0 && got[dir] == want[dir] ? h[dir] : kFaceMiss);
}

// One thread per row: the predictions, then face_dir's probes for the
// directions they leave open.  The loop runs whole waves (wave_reserve needs
// every lane).
// chunk_keys (non-null): a wave's 64 rows are one chunk (r / 64); its finer
// faces' keys go to chunk_keys[384 c ...] in (row, direction) order and
// their number to chunk_cnt[c], so a scan of the counts numbers every finer
// face in (row, direction) order - no sort of the keys
constexpr uint32_t kChunkKeys = 6 * 64;
__global__ void face_table_kernel(MapCtx m, DevMesh M, const uint64_t* slot_ids, size_t nrows, size_t run1,
                                  bool morton, int32_t* ell, unsigned long long* n_fine, uint32_t* fine_keys,
                                  size_t key_cap, int32_t* err, uint32_t* chunk_keys, uint32_t* chunk_cnt) {
	const SlotExists ex{M};
	const size_t stride = size_t(gridDim.x) * blockDim.x;
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r - lane_id() < nrows; r += stride) {
		const bool live = r < nrows;
		int32_t o6[6];
		uint32_t kf = 0;  // finer faces
		if (live) {
			uint64_t c[3];
			int lvl;
			const uint64_t id = slot_ids[r];
			cell_coords(m, id, c, lvl);
			if (morton) face_predict(m, slot_ids, r, run1, nrows, id, c, lvl, o6);
#pragma unroll
			for (int dir = 0; dir < 6; dir++) {
				if (morton && o6[dir] != kFaceMiss) continue;
				uint64_t out[4];
				const int nf = face_dir(m, c, lvl, dir, ex, out);
				// a single neighbor was the last cell found (face_dir returns on it)
				if (nf == 1 && ex.slot < 0) atomicExch(err, 1);
				o6[dir] = nf == 0 ? -1 : (nf == 4 ? -2 : (ex.slot >= 0 ? ex.slot : -1));
				kf += nf == 4 ? 1u : 0u;
			}
			typedef int i2v __attribute__((ext_vector_type(2)));
			i2v* ev = reinterpret_cast<i2v*>(ell + 6 * r);
#pragma unroll
			for (int j = 0; j < 3; j++) ev[j] = i2v{o6[2 * j], o6[2 * j + 1]};
		}
		if (chunk_keys) {
			const int incl = wave_incl_scan(int(kf));
			const size_t c = (r - lane_id()) >> 6;
			if (lane_id() == WAVE - 1) chunk_cnt[c] = uint32_t(incl);
			uint32_t at = uint32_t(incl) - kf;
			if (live)
				for (int dir = 0; dir < 6; dir++)
					if (o6[dir] == -2) chunk_keys[kChunkKeys * c + at++] = (uint32_t(r) << 3) | uint32_t(dir);
			continue;
		}
		if (__ballot(kf != 0) == 0) continue;
		unsigned long long at = wave_reserve(n_fine, kf);
		if (live)
			for (int dir = 0; dir < 6; dir++)
				if (o6[dir] == -2) {
					if (at < key_cap) fine_keys[at] = (uint32_t(r) << 3) | uint32_t(dir);  // else counted only
					at++;
				}
	}
}

// the finer faces in key order: f = the key's position
__global__ void face_fine_kernel(MapCtx m, DevMesh M, const uint64_t* slot_ids, const uint32_t* fine_keys, size_t n,
                                 int32_t* ell, int32_t* fine, int32_t* err, const uint32_t* chunk_keys,
                                 const uint32_t* chunk_off, uint32_t n_chunks) {
	const DevExists ex{M};
	for (size_t f = blockIdx.x * size_t(blockDim.x) + threadIdx.x; f < n; f += size_t(gridDim.x) * blockDim.x) {
		uint32_t key;
		if (chunk_keys) {
			// the chunk holding finer face f: the last offset <= f
			uint32_t lo = 0, hi = n_chunks;
			while (hi - lo > 1) {
				const uint32_t mid = (lo + hi) >> 1;
				if (chunk_off[mid] <= uint32_t(f)) lo = mid;
				else hi = mid;
			}
			key = chunk_keys[size_t(kChunkKeys) * lo + (uint32_t(f) - chunk_off[lo])];
		} else {
			key = fine_keys[f];
		}
		const size_t r = size_t(key >> 3);
		const int dir = int(key & 7);
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[r], c, lvl);
		uint64_t out[4];
		const int nf = face_dir(m, c, lvl, dir, ex, out);
		if (nf != 4) atomicExch(err, 1);
		int32_t sl[4];
#pragma unroll
		for (int i = 0; i < 4; i++) {
			sl[i] = i < nf ? dm_slot(M, out[i]) : -1;
			if (sl[i] < 0) atomicExch(err, 1);
		}
		reinterpret_cast<int4*>(fine)[f] = int4{sl[0], sl[1], sl[2], sl[3]};
		ell[6 * r + dir] = -2 - int32_t(f);
	}
}

// the CSR form of the table (rows of slot * 8 + direction entries, a row's
// directions ascending, a finer face's four slots in table order): counts,
// then entries from the scan
__global__ void face_csr_count_kernel(const int32_t* ell, size_t nrows, uint32_t* cnt) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		uint32_t k = 0;
		for (int d = 0; d < 6; d++) {
			const int32_t e = ell[6 * r + d];
			k += e >= 0 ? 1u : (e <= -2 ? 4u : 0u);
		}
		cnt[r] = k;
	}
}

__global__ void face_csr_fill_kernel(const int32_t* ell, const int32_t* fine, size_t nrows, const uint32_t* ptr,
                                     int32_t* ent) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		uint32_t k = ptr[r];
		for (int d = 0; d < 6; d++) {
			const int32_t e = ell[6 * r + d];
			if (e >= 0) {
				ent[k++] = e * 8 + d;
			} else if (e <= -2) {
				const size_t f = size_t(-2 - e);
				for (int i = 0; i < 4; i++) ent[k++] = fine[4 * f + i] * 8 + d;
			}
		}
	}
}

// where each slot of a rebuilt mesh takes its payload from (rebuild step 6;
// the gathers below write zeros where there is no source):
// the old local slot of the same cell, else (a new local cell absent from the
// old mesh: a refined cell's child) the old slot of its parent, else nothing
__global__ void carry_src_kernel(const uint64_t* __restrict__ slot_ids, size_t n_slots, size_t nl, MapCtx m,
                                 DevMesh oldM, size_t old_n_local, int32_t* __restrict__ src) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n_slots; s += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = slot_ids[s];
		const int32_t o = dm_slot(oldM, id);
		int32_t r = -1;
		if (o >= 0) {
			if (size_t(o) < old_n_local) r = o;
		} else if (s < nl) {
			const uint64_t p = map_parent(m, id);
			if (p != error_cell && p != id) r = dm_slot(oldM, p);
		}
		src[s] = r;
	}
}

template <class T>
__global__ void gather_rows_kernel(const T* __restrict__ old, const int32_t* __restrict__ src, size_t n,
                                   T* __restrict__ out) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x)
		out[s] = src[s] >= 0 ? old[src[s]] : T{};
}

__global__ void gather_bytes_kernel(const uint8_t* __restrict__ old, const int32_t* __restrict__ src, size_t n,
                                    size_t elem, uint8_t* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n * elem; i += size_t(gridDim.x) * blockDim.x) {
		const size_t s = i / elem;
		out[i] = src[s] >= 0 ? old[size_t(src[s]) * elem + (i - s * elem)] : uint8_t(0);
	}
}

__global__ void morton_keys_kernel(MapCtx m, const uint64_t* ids, size_t n, uint64_t* keys) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		map_indices(m, ids[i], x, y, z);
		keys[i] = spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
	}
}

// ---- ghost region ---------------------------------------------------------------
// (level-0 parent, volume in finest-level cells) of every local cell
__global__ void l0_volume_kernel(MapCtx m, const uint64_t* ids, size_t n, uint64_t* l0, uint64_t* vol) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int lvl = map_level(m, ids[i]);
		l0[i] = map_level0_parent(m, ids[i]);
		vol[i] = uint64_t(1) << (3 * (m.R - lvl));
	}
}

__device__ __forceinline__ bool sorted_has(const uint64_t* a, size_t n, uint64_t v) {
	size_t lo = 0, hi = n;
	while (lo < hi) {
		const size_t mid = (lo + hi) >> 1;
		if (a[mid] < v) lo = mid + 1;
		else hi = mid;
	}
	return lo < n && a[lo] == v;
}

// keys-only hash set (wholly local level-0 cells): same probing as the mesh table
__global__ void keyset_insert_kernel(uint64_t* tab, uint64_t mask, uint32_t shift, const uint64_t* keys,
                                     const uint64_t* vals, uint64_t want, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (vals && vals[i] != want) continue;
		const uint64_t id = keys[i];
		uint64_t h = hash_home(id, shift);
		for (;;) {
			const unsigned long long prev =
			    atomicCAS(reinterpret_cast<unsigned long long*>(tab + h), 0ull, (unsigned long long)id);
			if (prev == 0ull || prev == id) break;
			h = (h + 1) & mask;
		}
	}
}

struct KeySet {
	const uint64_t* tab;
	uint64_t mask;
	uint32_t shift;
	__device__ __forceinline__ bool has(uint64_t id) const {
		if (!tab) return false;
		uint64_t h = hash_home(id, shift);
		for (;;) {
			const uint64_t k = tab[h];
			if (k == id) return true;
			if (k == 0) return false;
			h = (h + 1) & mask;
		}
	}
};

// per distinct level-0 parent p of local cells: every level-0 cell q within
// Chebyshev distance `radius` (periodic wrap) that is not wholly local
// (full[] sorted; implicit grids: the block partition decides) is emitted
__global__ void ghost_l0_kernel(MapCtx m, DevMesh M, int rank, const uint64_t* par, size_t n, KeySet full,
                                int radius, uint64_t* out, unsigned long long* counter, unsigned long long cap) {
	MapCtx m0 = m;  // level-0 index space
	const int side = 2 * radius + 1;
	const int cube = side * side * side;
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		map_indices(m, par[i], x, y, z);
		const int64_t len0 = int64_t(1) << m.R;
		const int64_t b[3] = {int64_t(x), int64_t(y), int64_t(z)};
		for (int k = 0; k < cube; k++) {
			const int dx = k % side - radius, dy = (k / side) % side - radius, dz = k / (side * side) - radius;
			uint64_t w[3];
			if (!map_wrap(m0, 0, b[0] + dx * len0, w[0]) || !map_wrap(m0, 1, b[1] + dy * len0, w[1]) ||
			    !map_wrap(m0, 2, b[2] + dz * len0, w[2]))
				continue;
			const uint64_t q = map_from_indices(m, w[0], w[1], w[2], 0);
			bool local_full;
			if (M.implicit) local_full = M.bp.owner(q) == rank;
			else local_full = full.has(q);
			if (local_full) continue;
			const unsigned long long pos = atomicAdd(counter, 1ull);
			if (pos < cap) out[pos] = q;
		}
	}
}

__global__ void cells_under_kernel(MapCtx m, const uint64_t* ids, size_t n, const uint64_t* l0, size_t nl0,
                                   uint64_t* out, unsigned long long* counter) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (sorted_has(l0, nl0, map_level0_parent(m, ids[i]))) out[atomicAdd(counter, 1ull)] = ids[i];
	}
}

// ---- refinement -------------------------------------------------------------------
// induce_refines (9591-9720): for a requested local cell r, every existing
// neighbors_of / neighbors_to entry coarser than r must be refined as well
// neighbors_of / neighbors_to of the local cells of req that are coarser
// (induce_refines 9591-9720) or, with finer != 0, finer (the dont_refine
// spread of override_refines 9991-10038) than the cell
__global__ void induced_kernel(MapCtx m, const int32_t* hood, const int32_t* hood_to, int nh, DevMesh M, int rank,
                               const uint64_t* req, size_t n, uint64_t* out, unsigned long long* counter,
                               unsigned long long cap, int finer) {
	const DevExists ex{M};
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t w = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; w < n; w += waves) {
		const uint64_t r = req[w];
		if (dm_owner(M, r) != rank) continue;  // wave-uniform
		uint64_t c[3];
		int lvl;
		cell_coords(m, r, c, lvl);
		auto emit = [&](uint64_t q) {
			if (q == error_cell || !ex(q)) return;
			const int ql = map_level(m, q);
			if (finer ? ql <= lvl : ql >= lvl) return;
			const unsigned long long pos = atomicAdd(counter, 1ull);
			if (pos < cap) out[pos] = q;
		};
		// nof_item's leaves from the item's case (no ItemOut in private memory)
		for (int k = lane_id(); k < nh; k += WAVE) {
			uint64_t w[3];
			const int kind = nof_item_case(m, c, lvl, hood + 3 * k, ex, w);
			for (int i = 0; i < item_count(kind); i++) emit(item_id(m, lvl, hood + 3 * k, kind, w, i, nullptr));
		}
		for (int k = lane_id(); k < 10 * nh; k += WAVE) emit(nto_candidate(m, c, lvl, hood_to, nh, k, ex));
	}
}

// override_unrefines (9796-9898): the family under parent p (children of
// level L) may merge only if no leaf in p's neighborhood is finer than L and
// none of level L is being refined.  The reference walks the face-neighbor
// graph from the unrefined cell while is_neighbor(p, .) holds; the leaves it
// reaches are the ones inside p's neighborhood boxes, checked here box by
// box: a box covered by one leaf of p's level or coarser passes, otherwise
// each of its eight level-L cells must be a leaf that is not being refined.
__global__ void unrefine_check_kernel(MapCtx m, const int32_t* hood, int nh, DevMesh M, const uint64_t* parents,
                                      size_t n, const uint64_t* S, size_t nS, uint32_t* ok) {
	// one thread per (parent, neighborhood box); ok starts 1, a failing box
	// clears it
	const DevExists ex{M};
	for (size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x; t < n * size_t(nh); t += size_t(gridDim.x) * blockDim.x) {
		const size_t i = t / size_t(nh);
		const int k = int(t - i * size_t(nh));
		uint64_t c[3];
		int pl;
		cell_coords(m, parents[i], c, pl);
		const int64_t len = int64_t(1) << (m.R - pl);
		uint64_t w[3];
		bool inside = true;
		for (int d = 0; d < 3; d++) inside = inside && map_wrap(m, d, int64_t(c[d]) + int64_t(hood[3 * k + d]) * len, w[d]);
		if (!inside) continue;
		bool covered = false;
		for (int l = pl; l >= 0 && !covered; l--) covered = ex(map_from_indices(m, w[0], w[1], w[2], l));
		if (covered) continue;
		const uint64_t hl = uint64_t(len / 2);
		bool good = true;
		for (int q = 0; q < 8 && good; q++) {
			const uint64_t id = map_from_indices(m, w[0] + (q & 1) * hl, w[1] + ((q >> 1) & 1) * hl,
			                                     w[2] + ((q >> 2) & 1) * hl, pl + 1);
			if (!ex(id) || sorted_has(S, nS, id)) good = false;
		}
		if (!good) ok[i] = 0;
	}
}

// override_unrefines' candidates (9796-9898): the parents of the requested
// cells (level-0 cells have none: ~0, dropped by the sort)
__global__ void request_parents_kernel(MapCtx m, const uint64_t* req, size_t n, uint64_t* par) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t c = req[i];
		par[i] = map_level(m, c) > 0 ? map_parent(m, c) : ~uint64_t(0);
	}
}

// a family is blocked when one of its children is being refined or is
// marked dont_unrefine
__global__ void family_blocked_kernel(MapCtx m, const uint64_t* cand, size_t n, const uint64_t* S, size_t nS,
                                      const uint64_t* DU, size_t nDU, uint32_t* ok) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t ch[8];
		map_all_children(m, cand[i], ch);
		bool blocked = false;
		for (int k = 0; k < 8; k++) blocked = blocked || sorted_has(S, nS, ch[k]) || sorted_has(DU, nDU, ch[k]);
		if (blocked) ok[i] = 0;
	}
}

// execute_refines (10104-10554): children replace refined leaves and inherit
// the owner (10228-10237); the children of an unrefined parent are replaced
// by the parent, owned by the owner of its first child (10298)
__global__ void refine_count_kernel(MapCtx m, const uint64_t* kid, size_t n, const uint64_t* S, size_t nS,
                                    const uint64_t* F, size_t nF, uint32_t* cnt) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t c = kid[i];
		uint32_t k = 1u;
		if (sorted_has(S, nS, c)) {
			k = 8u;
		} else if (nF) {
			const uint64_t p = map_parent(m, c);
			if (p != c && sorted_has(F, nF, p)) k = map_child(m, p) == c ? 1u : 0u;
		}
		cnt[i] = k;
	}
}

__global__ void refine_fill_kernel(MapCtx m, const uint64_t* kid, const int32_t* kown, size_t n, const uint32_t* pos,
                                   const uint32_t* cnt, const uint64_t* F, size_t nF, uint64_t* oid, int32_t* oown) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const size_t p = pos[i];
		if (cnt[i] == 0u) continue;
		if (cnt[i] == 1u) {
			uint64_t c = kid[i];
			if (nF) {
				const uint64_t par = map_parent(m, c);
				if (par != c && sorted_has(F, nF, par)) c = par;
			}
			oid[p] = c;
			oown[p] = kown[i];
		} else {
			uint64_t ch[8];
			map_all_children(m, kid[i], ch);
			for (int k = 0; k < 8; k++) {
				oid[p + k] = ch[k];
				oown[p + k] = kown[i];
			}
		}
	}
}

// The own-leaf prefix of the known list (Mesh::n_prefix: kid index = slot)
// classified by lookups of the refined cells and the merged families'
// children instead of a search per entry: cls 1 refined, 2 a family's first
// child (becomes the parent), 3 another child (drops out), 0 unchanged.
__global__ void mark_refined_kernel(DevMesh M, const uint64_t* S, size_t nS, size_t n_prefix, uint8_t* cls) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < nS; i += size_t(gridDim.x) * blockDim.x) {
		const int32_t sl = dm_slot(M, S[i]);
		if (sl >= 0 && size_t(sl) < n_prefix) cls[sl] = 1;
	}
}

__global__ void mark_families_kernel(MapCtx m, DevMesh M, const uint64_t* F, size_t nF, size_t n_prefix, uint8_t* cls) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < 8 * nF; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t ch[8];
		map_all_children(m, F[i >> 3], ch);
		const int k = int(i & 7);
		const int32_t sl = dm_slot(M, ch[k]);
		if (sl >= 0 && size_t(sl) < n_prefix) cls[sl] = k == 0 ? 2 : 3;
	}
}

__global__ void prefix_count_kernel(const uint8_t* cls, size_t n, uint32_t* cnt) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint8_t c = cls[i];
		cnt[i] = c == 1 ? 8u : (c == 3 ? 0u : 1u);
	}
}

// src (optional): per output entry the input index its payload comes from
// (-1: a merged parent, which starts zeroed)
__global__ void prefix_fill_kernel(MapCtx m, const uint64_t* kid, const int32_t* kown, const uint8_t* cls, size_t n,
                                   const uint32_t* pos, uint64_t* oid, int32_t* oown, int32_t* src) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint8_t c = cls[i];
		const size_t p = pos[i];
		if (c == 3) continue;
		if (c == 1) {
			uint64_t ch[8];
			map_all_children(m, kid[i], ch);
			for (int k = 0; k < 8; k++) {
				oid[p + k] = ch[k];
				oown[p + k] = kown[i];
				if (src) src[p + k] = int32_t(i);
			}
		} else {
			oid[p] = c == 2 ? map_parent(m, kid[i]) : kid[i];
			oown[p] = kown[i];
			if (src) src[p] = c == 2 ? -1 : int32_t(i);
		}
	}
}

// the children of the refined cells owned by `rank` (stop_refining's
// created cells); one thread per refined cell, full waves (wave_reserve)
__global__ void created_children_kernel(MapCtx m, DevMesh M, int rank, const uint64_t* S, size_t nS, uint64_t* out,
                                        unsigned long long* ctr) {
	const size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	const bool mine = i < nS && dm_owner(M, S[i]) == rank;
	const unsigned long long at = wave_reserve(ctr, mine ? 8u : 0u);
	if (!mine) return;
	uint64_t ch[8];
	map_all_children(m, S[i], ch);
	for (int k = 0; k < 8; k++) out[at + k] = ch[k];
}

// the children of merged families that stay on `rank` (owned here, as is the
// family's first child, which becomes the parent's owner), with their slots
__global__ void kept_children_kernel(MapCtx m, DevMesh M, int rank, const uint64_t* F, size_t nF, uint64_t* out,
                                     int32_t* out_slot, unsigned long long* ctr) {
	const size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	bool keep = false;
	uint64_t c = 0;
	int32_t sl = -1;
	if (t < 8 * nF) {
		uint64_t ch[8];
		map_all_children(m, F[t >> 3], ch);
		c = ch[t & 7];
		keep = dm_owner(M, c) == rank && dm_owner(M, ch[0]) == rank;
		if (keep) sl = dm_slot(M, c);
	}
	const unsigned long long at = wave_reserve(ctr, keep ? 1u : 0u);
	if (!keep) return;
	out[at] = c;
	out_slot[at] = sl;
}

// Every child of every merged family local (one process): the children in
// ascending id without a sort.  F ascending, so its families come in level
// groups, and within a group the children of one octant k ascend with their
// parents (the id's (z, y, x) digits are the parent's doubled plus the
// octant's bits), so a child's position is the number of smaller children of
// each octant in its group, found by binary search of that octant's stream.
struct LevelGroups {
	uint32_t lo[kRangeLevels + 1];  // group g: families [lo[g], lo[g + 1])
	int n;
};
__global__ void family_children_kernel(MapCtx m, const uint64_t* __restrict__ F, size_t nF, uint64_t* __restrict__ ch) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < nF; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t c[8];
		map_all_children(m, F[i], c);
#pragma unroll
		for (int k = 0; k < 8; k++) ch[8 * i + k] = c[k];
	}
}
__global__ void kept_ordered_kernel(DevMesh M, const uint64_t* __restrict__ ch, size_t nF, LevelGroups G,
                                    uint64_t* __restrict__ out, int32_t* __restrict__ out_slot) {
	for (size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x; t < 8 * nF; t += size_t(gridDim.x) * blockDim.x) {
		const uint32_t i = uint32_t(t >> 3);
		const int k = int(t & 7);
		uint32_t g0 = 0, g1 = uint32_t(nF);
		for (int g = 0; g < G.n; g++)
			if (i >= G.lo[g] && i < G.lo[g + 1]) {
				g0 = G.lo[g];
				g1 = G.lo[g + 1];
			}
		const uint64_t c = ch[t];
		size_t pos = 8 * size_t(g0) + (i - g0);  // its own octant's smaller ones
		for (int q = 0; q < 8; q++) {
			if (q == k) continue;
			uint32_t lo = g0, hi = g1;
			while (lo < hi) {
				const uint32_t mid = (lo + hi) >> 1;
				if (ch[8 * size_t(mid) + q] < c) lo = mid + 1;
				else hi = mid;
			}
			pos += lo - g0;
		}
		out[pos] = c;
		out_slot[pos] = dm_slot(M, c);
	}
}

// bits 0-4: the level; bits 5-7: the cell's octant in its parent (bit k set
// when its index along axis k is odd at its level; 0 at level 0), which is
// the corner test of adapter.hpp:84-102 without the cell's indices
__global__ void slot_levels_kernel(MapCtx m, const uint64_t* slot_ids, size_t n, uint8_t* lvl) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		const int l = map_indices(m, slot_ids[i], x, y, z);
		const int sh = m.R - l;
		const unsigned oct = l ? unsigned(((x >> sh) & 1) | (((y >> sh) & 1) << 1) | (((z >> sh) & 1) << 2)) : 0u;
		lvl[i] = uint8_t(unsigned(l) | (oct << 5));
	}
}

}  // namespace

// ============================================================================
int max_hood_items() { return kMaxNtoLds / 10; }

static int nto_cap(int nh) {
	int P = 1;
	while (P < 10 * nh) P <<= 1;
	return P;
}

void k_fill_i32(int32_t* p, size_t n, int32_t v, hipStream_t s) {
	if (!n) return;
	fill_i32_kernel<<<grid_for(n, 256), 256, 0, s>>>(p, n, v);
	HIP_CHECK(hipGetLastError());
}

void k_iota_u64(uint64_t* out, uint64_t first, size_t n, hipStream_t s) {
	if (!n) return;
	iota_u64_kernel<<<grid_for(n, 256), 256, 0, s>>>(out, first, n);
	HIP_CHECK(hipGetLastError());
}

void k_hash_insert(HashEntry* tab, uint64_t mask, uint32_t shift, const uint64_t* ids, const int32_t* owners,
                   int32_t owner_const, size_t n, hipStream_t s, size_t slot_upto) {
	if (!n) return;
	hash_insert_kernel<<<grid_for(n, 256), 256, 0, s>>>(tab, mask, shift, ids, owners, owner_const, n, slot_upto);
	HIP_CHECK(hipGetLastError());
}

bool k_level_ranges(const MapCtx& m, const uint64_t* ids, size_t n, uint64_t* lo, uint64_t* hi, hipStream_t s) {
	if (m.R >= kRangeLevels) return false;
	DBuf<unsigned long long> d;
	d.alloc(2 * kRangeLevels);
	std::vector<unsigned long long> h(2 * kRangeLevels);
	for (int L = 0; L < kRangeLevels; L++) {
		h[size_t(L)] = ~0ull;
		h[size_t(kRangeLevels + L)] = 0ull;
	}
	h2d(d.p, h.data(), h.size() * 8, s);
	if (n) {
		level_ranges_kernel<<<std::min<unsigned>(grid_for(n, 256), 2048), 256, 0, s>>>(m, ids, n, d.p,
		                                                                              d.p + kRangeLevels);
		HIP_CHECK(hipGetLastError());
	}
	d2h_small(h.data(), d.p, h.size() * 8, s);
	for (int L = 0; L < kRangeLevels; L++) {
		lo[L] = h[size_t(L)];
		hi[L] = h[size_t(kRangeLevels + L)];
	}
	return true;
}

void k_range_insert(int2* rmap, const DevMesh& M, const uint64_t* ids, const int32_t* owners, size_t n, size_t slot_upto,
                    hipStream_t s) {
	if (!n) return;
	range_insert_kernel<<<grid_for(n, 256), 256, 0, s>>>(rmap, M, ids, owners, n, slot_upto);
	HIP_CHECK(hipGetLastError());
}

void k_range_clear(int2* rmap, const DevMesh& M, const uint64_t* ids, size_t n, hipStream_t s) {
	if (!n) return;
	range_clear_kernel<<<grid_for(n, 256), 256, 0, s>>>(rmap, M, ids, n);
	HIP_CHECK(hipGetLastError());
}

void k_hash_set_slots(const DevMesh& M, const uint64_t* slot_ids, size_t n, int32_t* err, hipStream_t s) {
	if (!n) return;
	hash_set_slots_kernel<<<grid_for(n, 256), 256, 0, s>>>(M, slot_ids, n, err);
	HIP_CHECK(hipGetLastError());
}

void k_lookup(const DevMesh& M, const uint64_t* ids, size_t n, int32_t* owner, int32_t* slot, hipStream_t s) {
	if (!n) return;
	lookup_kernel<<<grid_for(n, 256), 256, 0, s>>>(M, ids, n, owner, slot);
	HIP_CHECK(hipGetLastError());
}

void k_remote_flags(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const DevMesh& M, int rank,
                    const uint64_t* cells, size_t n, uint32_t* flag, hipStream_t s, const uint8_t* near,
                    uint64_t near_lo, size_t near_n) {
	if (!n) return;
	static const char* env = std::getenv("DCCRGX_FLAGS_WAVE");  // A/B: the wave-per-cell form
	if ((nh <= 6 || near) && !(env && env[0] == '1'))
		remote_flags_thread_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, hood, hood_to, nh, M, rank, cells, n, flag, near,
		                                                            near_lo, near_n);
	else
		remote_flags_kernel<<<grid_for(n, 4), 256, 0, s>>>(m, hood, hood_to, nh, M, rank, cells, n, flag);
	HIP_CHECK(hipGetLastError());
}

namespace {
// min / max level-0 parent of the ids: wave then block reduction, one
// atomic pair per block (per wave, 134 K pairs on one address cost 0.75 ms)
__global__ __launch_bounds__(256) void level0_span_kernel(MapCtx m, const uint64_t* __restrict__ ids, size_t n,
                                                          unsigned long long* mm) {
	__shared__ unsigned long long slo[256 / WAVE], shi[256 / WAVE];
	unsigned long long lo = ~0ull, hi = 0;
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const unsigned long long p = map_level0_parent(m, ids[i]);
		lo = p < lo ? p : lo;
		hi = p > hi ? p : hi;
	}
	for (int o = WAVE / 2; o > 0; o >>= 1) {
		const unsigned long long a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
		lo = a < lo ? a : lo;
		hi = b > hi ? b : hi;
	}
	if (lane_id() == 0) {
		slo[threadIdx.x / WAVE] = lo;
		shi[threadIdx.x / WAVE] = hi;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < 256 / WAVE; w++) {
			lo = slo[w] < lo ? slo[w] : lo;
			hi = shi[w] > hi ? shi[w] : hi;
		}
		if (lo <= hi) {
			atomicMin(mm, lo);
			atomicMax(mm + 1, hi);
		}
	}
}

// mark the level-0 cells within r of every ghost leaf's level-0 parent
__global__ void level0_near_kernel(MapCtx m, MapCtx m0, const uint64_t* __restrict__ kid,
                                   const int32_t* __restrict__ kown, size_t n, int rank, int r, uint64_t lo,
                                   uint64_t span, uint8_t* __restrict__ near) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (kown[i] == rank) continue;
		uint64_t x, y, z;
		map_indices(m0, map_level0_parent(m, kid[i]), x, y, z);
		for (int dz = -r; dz <= r; dz++) {
			uint64_t wz;
			if (!map_wrap(m0, 2, int64_t(z) + dz, wz)) continue;
			for (int dy = -r; dy <= r; dy++) {
				uint64_t wy;
				if (!map_wrap(m0, 1, int64_t(y) + dy, wy)) continue;
				for (int dx = -r; dx <= r; dx++) {
					uint64_t wx;
					if (!map_wrap(m0, 0, int64_t(x) + dx, wx)) continue;
					const uint64_t q = map_from_indices(m0, wx, wy, wz, 0) - lo;
					if (q < span) near[q] = 1;
				}
			}
		}
	}
}
}  // namespace

bool k_level0_near(const MapCtx& m, const uint64_t* kid, const int32_t* kown, size_t n_known, int rank, int radius,
                   DBuf<uint8_t>& near, uint64_t& near_lo, hipStream_t s) {
	if (!n_known) return false;
	DBuf<unsigned long long> mm;
	mm.alloc(2);
	const unsigned long long init[2] = {~0ull, 0ull};
	h2d(mm.p, init, sizeof(init), s);
	level0_span_kernel<<<grid_for(n_known, 256, 1024), 256, 0, s>>>(m, kid, n_known, mm.p);
	HIP_CHECK(hipGetLastError());
	unsigned long long h[2] = {0, 0};
	d2h_small(h, mm.p, sizeof(h), s);
	if (h[0] > h[1]) return false;
	const uint64_t span = h[1] - h[0] + 1;
	if (span > 8 * uint64_t(n_known) + (uint64_t(1) << 24)) return false;
	near.alloc(size_t(span));
	HIP_CHECK(hipMemsetAsync(near.p, 0, size_t(span), s));
	MapCtx m0;
	const uint64_t len[3] = {m.len[0], m.len[1], m.len[2]};
	const int per[3] = {m.periodic[0], m.periodic[1], m.periodic[2]};
	map_init(m0, len, 0, per);
	level0_near_kernel<<<grid_for(n_known, 256), 256, 0, s>>>(m, m0, kid, kown, n_known, rank, radius, h[0], span,
	                                                          near.p);
	HIP_CHECK(hipGetLastError());
	near_lo = h[0];
	return true;
}

void k_assign_slots2(const uint32_t* flag, const uint32_t* scan_outer, size_t n, size_t n_inner, const uint64_t* cells,
                     uint64_t* slot_ids, hipStream_t s) {
	if (!n) return;
	assign_slots_kernel<<<grid_for(n, 256), 256, 0, s>>>(flag, scan_outer, n, n_inner, cells, slot_ids);
	HIP_CHECK(hipGetLastError());
}

void k_count_rows(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const DevMesh& M,
                  const uint64_t* slot_ids, size_t row0, size_t nrows, uint32_t* nof_cnt, uint32_t* nto_cnt,
                  hipStream_t s) {
	if (!nrows) return;
	const int cap = nto_cap(nh);
	DX_REQUIRE(cap <= kMaxNtoLds, "neighborhood too large for the neighbors_to build");
	count_rows_kernel<<<grid_for(nrows, 1, 256u * 64u), WAVE, size_t(cap) * 8, s>>>(m, hood, hood_to, nh, M, slot_ids,
	                                                                                  row0, nrows, nof_cnt, nto_cnt, cap);
	HIP_CHECK(hipGetLastError());
}

void k_fill_neighbors_of(const MapCtx& m, const int32_t* hood, int nh, const DevMesh& M, const uint64_t* slot_ids,
                         size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids, int32_t* offs, hipStream_t s) {
	if (!nrows) return;
	fill_nof_kernel<<<grid_for(nrows, 4), 256, 0, s>>>(m, hood, nh, M, slot_ids, row0, nrows, ptr, ids, offs);
	HIP_CHECK(hipGetLastError());
}

void k_fill_neighbors_to(const MapCtx& m, const int32_t* hood_to, int nh, const DevMesh& M, const uint64_t* slot_ids,
                         size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids, hipStream_t s) {
	if (!nrows) return;
	const int cap = nto_cap(nh);
	DX_REQUIRE(cap <= kMaxNtoLds, "neighborhood too large for the neighbors_to build");
	fill_nto_kernel<<<grid_for(nrows, 1, 256u * 64u), WAVE, size_t(cap) * 8, s>>>(m, hood_to, nh, M, slot_ids, row0,
	                                                                                nrows, ptr, ids, cap);
	HIP_CHECK(hipGetLastError());
}

static size_t read_counter(const DBuf<unsigned long long>& ctr, hipStream_t s) {
	unsigned long long h = 0;
	d2h_small(&h, ctr.p, sizeof(h), s);
	return size_t(h);
}

static void zero_counter(DBuf<unsigned long long>& ctr, hipStream_t s) {
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, sizeof(unsigned long long), s));
}

// the n extracted entries grouped by owner, each group's ids ascending and
// unique: one 64-bit key sort, or for pairs a sort by id then a stable sort
// by owner and a select of the pair heads
static size_t group_by_owner(uint64_t* keys, uint32_t* owners, size_t n, uint64_t stride, int size,
                             std::map<int, std::vector<uint64_t>>& out, hipStream_t s) {
	out.clear();
	if (!n) return 0;
	if (!owners) {
		// keys = owner * stride + id < size * stride: only those bits sorted
		int bits = 1;
		const uint64_t top = uint64_t(size) * stride;
		while (bits < 64 && (top >> bits)) bits++;
		n = sort_unique_u64(keys, n, s, bits);
		for (uint64_t k : download(keys, n, s)) out[int(k / stride)].push_back(k % stride);
		return n;
	}
	DBuf<uint64_t> k2;
	DBuf<uint32_t> o2;
	k2.alloc(n);
	o2.alloc(n);
	int obits = 1;
	while (obits < 32 && (uint64_t(size) >> obits)) obits++;
	size_t b1 = 0, b2 = 0, b3 = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, keys, k2.p, owners, o2.p, n, 0, 64, s));
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b2, o2.p, owners, k2.p, keys, n, 0, obits, s));
	DBuf<uint8_t> head;
	head.alloc(n);
	DBuf<unsigned long long> nsel;
	nsel.alloc(1);
	size_t b4 = 0;
	HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, b3, keys, head.p, k2.p, nsel.p, n, s));
	HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, b4, owners, head.p, o2.p, nsel.p, n, s));
	DBuf<uint8_t> temp;
	temp.alloc(std::max(std::max(b1, b2), std::max(b3, b4)));
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, b1, keys, k2.p, owners, o2.p, n, 0, 64, s));
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, b2, o2.p, owners, k2.p, keys, n, 0, obits, s));
	pair_heads_kernel<<<grid_for(n, 256), 256, 0, s>>>(keys, owners, n, head.p);
	HIP_CHECK(hipGetLastError());
	HIP_CHECK(hipcub::DeviceSelect::Flagged(temp.p, b3, keys, head.p, k2.p, nsel.p, n, s));
	HIP_CHECK(hipcub::DeviceSelect::Flagged(temp.p, b4, owners, head.p, o2.p, nsel.p, n, s));
	const size_t u = read_counter(nsel, s);
	const std::vector<uint64_t> ids = download(k2.p, u, s);
	const std::vector<uint32_t> own = download(o2.p, u, s);
	for (size_t i = 0; i < u; i++) out[int(own[i])].push_back(ids[i]);
	return u;
}

void k_remote_by_owner(const uint64_t* ids, size_t n, const DevMesh& M, int rank, int size,
                       std::map<int, std::vector<uint64_t>>& out, hipStream_t s, DBuf<uint64_t>* keep, size_t* keep_n) {
	out.clear();
	if (keep_n) *keep_n = 0;
	if (!n) return;
	const uint64_t stride = M.last + 1;
	const bool pairs = uint64_t(size) > ~uint64_t(0) / stride;
	DBuf<uint64_t> keys;
	DBuf<uint32_t> owners;
	keys.alloc(n);
	if (pairs) owners.alloc(n);
	DBuf<unsigned long long> ctr;
	zero_counter(ctr, s);
	extract_remote_kernel<<<grid_for(n, 256), 256, 0, s>>>(ids, n, M, rank, stride, keys.p, owners.p, ctr.p);
	HIP_CHECK(hipGetLastError());
	const size_t u = group_by_owner(keys.p, owners.p, read_counter(ctr, s), stride, size, out, s);
	if (keep && !pairs) {
		keep->swap(keys);  // sorted unique (owner * stride + id) keys
		*keep_n = u;
	}
}

bool k_remote_extra(const uint64_t* ids, size_t n, const DevMesh& M, int rank, int size, const uint64_t* of_keys,
                    size_t n_of, std::vector<uint64_t>& out, hipStream_t s) {
	out.clear();
	const uint64_t stride = M.last + 1;
	if (uint64_t(size) > ~uint64_t(0) / stride) return false;  // keys would overflow: the caller's pair path
	if (!n) return true;
	DBuf<uint64_t> ex;
	ex.alloc(n);
	DBuf<unsigned long long> ctr;
	zero_counter(ctr, s);
	extract_extra_kernel<<<grid_for(n, 256), 256, 0, s>>>(ids, n, M, rank, stride, of_keys, n_of, ex.p, ctr.p);
	HIP_CHECK(hipGetLastError());
	const size_t k = read_counter(ctr, s);
	if (k) {
		out = download(ex.p, k, s);
		std::sort(out.begin(), out.end());
		out.erase(std::unique(out.begin(), out.end()), out.end());
	}
	return true;
}

void k_send_by_owner(const uint64_t* nto_id, const uint32_t* nto_ptr, size_t n_entries, const uint64_t* slot_ids,
                     size_t row0, size_t nrows, const DevMesh& M, int rank, int size,
                     std::map<int, std::vector<uint64_t>>& out, hipStream_t s) {
	out.clear();
	if (!nrows || !n_entries) return;
	const uint64_t stride = M.last + 1;
	const bool pairs = uint64_t(size) > ~uint64_t(0) / stride;
	DBuf<uint64_t> keys;
	DBuf<uint32_t> owners;
	keys.alloc(n_entries);
	if (pairs) owners.alloc(n_entries);
	DBuf<unsigned long long> ctr;
	zero_counter(ctr, s);
	extract_send_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(nto_id, nto_ptr, slot_ids, row0, nrows, M, rank, stride,
	                                                         keys.p, owners.p, ctr.p);
	HIP_CHECK(hipGetLastError());
	group_by_owner(keys.p, owners.p, read_counter(ctr, s), stride, size, out, s);
}

namespace {
__global__ void fill_u64_kernel(uint64_t* __restrict__ p, size_t n, uint64_t v) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = v;
}
// a sorted unique list padded with one sentinel group: drop it from the count
__global__ void drop_sentinel_kernel(const uint64_t* __restrict__ u, unsigned long long* __restrict__ cnt, uint64_t v) {
	if (threadIdx.x == 0 && *cnt > 0 && u[*cnt - 1] == v) *cnt -= 1;
}
__global__ void strip_owner_kernel(const uint64_t* __restrict__ keys, const unsigned long long* __restrict__ cnt,
                                   uint64_t stride, uint64_t* __restrict__ ids) {
	const size_t n = size_t(*cnt);
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		ids[i] = keys[i] % stride;
}
}  // namespace

// keys padded with sentinels to their capacity, sorted and made unique on
// the device, the count left on the device (no host read)
static void sort_unique_padded(DBuf<uint64_t>& keys, size_t cap, int bits, uint64_t sentinel, DBuf<uint64_t>& uniq,
                               unsigned long long* d_count, hipStream_t s) {
	DBuf<uint64_t> tmp;
	tmp.alloc(cap + 1);
	uniq.alloc(cap + 1);
	size_t b1 = 0, b2 = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, keys.p, tmp.p, cap, 0, bits, s));
	HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, b2, tmp.p, uniq.p, d_count, cap, s));
	DBuf<uint8_t> temp;
	temp.alloc(std::max(b1, b2) + 1);
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, b1, keys.p, tmp.p, cap, 0, bits, s));
	HIP_CHECK(hipcub::DeviceSelect::Unique(temp.p, b2, tmp.p, uniq.p, d_count, cap, s));
	drop_sentinel_kernel<<<1, 64, 0, s>>>(uniq.p, d_count, sentinel);
	HIP_CHECK(hipGetLastError());
}

bool k_halo_lists(const uint64_t* of_id, size_t t_of, const uint64_t* to_id, const uint32_t* p_to, size_t t_to,
                  const uint64_t* slot_ids, size_t row0, size_t nrows, const DevMesh& M, int rank, int size,
                  HaloLists& out, hipStream_t s) {
	out.recv.clear();
	out.send.clear();
	out.extra.clear();
	out.n_recv = out.n_send = 0;
	const uint64_t stride = M.last + 1;
	if (uint64_t(size) > ~uint64_t(0) / stride) return false;  // keys would overflow: the pair path
	int bits = 1;
	const uint64_t top = uint64_t(size) * stride;
	while (bits < 64 && (top >> bits)) bits++;
	const uint64_t sentinel = bits >= 64 ? ~uint64_t(0) : (uint64_t(1) << bits) - 1;  // > every key
	DBuf<unsigned long long> cnt;  // 0 of keys, 1 to keys, 2 extra ids, 3 extract counter of, 4 of to
	cnt.alloc(5);
	HIP_CHECK(hipMemsetAsync(cnt.p, 0, 5 * sizeof(unsigned long long), s));
	DBuf<uint64_t> kof, kto;
	const size_t cof = std::max<size_t>(t_of, 1), cto = std::max<size_t>(t_to, 1);
	kof.alloc(cof + 1);
	kto.alloc(cto + 1);
	fill_u64_kernel<<<grid_for(cof, 256), 256, 0, s>>>(kof.p, cof, sentinel);
	fill_u64_kernel<<<grid_for(cto, 256), 256, 0, s>>>(kto.p, cto, sentinel);
	if (t_of)
		extract_remote_kernel<<<grid_for(t_of, 256), 256, 0, s>>>(of_id, t_of, M, rank, stride, kof.p, nullptr, cnt.p + 3);
	if (nrows && t_to)
		extract_send_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(to_id, p_to, slot_ids, row0, nrows, M, rank, stride, kto.p,
		                                                         nullptr, cnt.p + 4);
	HIP_CHECK(hipGetLastError());
	// the extracted counts first: sorting the capacity (several times the
	// remote entries) costs more than this read
	unsigned long long ext[2] = {0, 0};
	d2h_small(ext, cnt.p + 3, sizeof(ext), s);
	if (ext[0]) sort_unique_padded(kof, size_t(ext[0]), bits, sentinel, out.recv_keys, cnt.p + 0, s);
	else out.recv_keys.alloc(1);
	if (ext[1]) sort_unique_padded(kto, size_t(ext[1]), bits, sentinel, out.send_keys, cnt.p + 1, s);
	else out.send_keys.alloc(1);
	// remote neighbors_to that are no neighbors_of (none for a symmetric hood)
	DBuf<uint64_t> ex;
	ex.alloc(cto + 1);
	if (t_to)
		extract_extra_kernel<<<grid_for(t_to, 256), 256, 0, s>>>(to_id, t_to, M, rank, stride, out.recv_keys.p, 0, ex.p,
		                                                         cnt.p + 2, cnt.p + 0);
	HIP_CHECK(hipGetLastError());
	unsigned long long h[3] = {0, 0, 0};
	d2h_small(h, cnt.p, sizeof(h), s);
	out.n_recv = size_t(h[0]);
	out.n_send = size_t(h[1]);
	// the three lists in one read
	const size_t b0 = 8 * size_t(h[0]), b1 = 8 * size_t(h[1]), b2 = 8 * size_t(h[2]);
	std::vector<uint64_t> all((b0 + b1 + b2) / 8);
	if (!all.empty()) {
		DBuf<uint8_t> stage;
		stage.alloc(b0 + b1 + b2);
		if (b0) HIP_CHECK(hipMemcpyAsync(stage.p, out.recv_keys.p, b0, hipMemcpyDeviceToDevice, s));
		if (b1) HIP_CHECK(hipMemcpyAsync(stage.p + b0, out.send_keys.p, b1, hipMemcpyDeviceToDevice, s));
		if (b2) HIP_CHECK(hipMemcpyAsync(stage.p + b0 + b1, ex.p, b2, hipMemcpyDeviceToDevice, s));
		d2h_small(all.data(), stage.p, b0 + b1 + b2, s);
	}
	for (size_t i = 0; i < size_t(h[0]); i++) out.recv[int(all[i] / stride)].push_back(all[i] % stride);
	for (size_t i = 0; i < size_t(h[1]); i++) out.send[int(all[h[0] + i] / stride)].push_back(all[h[0] + i] % stride);
	out.extra.assign(all.begin() + ptrdiff_t(h[0] + h[1]), all.end());
	std::sort(out.extra.begin(), out.extra.end());
	out.extra.erase(std::unique(out.extra.begin(), out.extra.end()), out.extra.end());
	// the lists' ids on the device in wire order (peer, then id): halo slot
	// ids and send cells without an upload
	out.recv_ids.alloc(size_t(h[0]) + 1);
	out.send_ids.alloc(size_t(h[1]) + 1);
	if (h[0]) strip_owner_kernel<<<grid_for(size_t(h[0]), 256), 256, 0, s>>>(out.recv_keys.p, cnt.p + 0, stride, out.recv_ids.p);
	if (h[1]) strip_owner_kernel<<<grid_for(size_t(h[1]), 256), 256, 0, s>>>(out.send_keys.p, cnt.p + 1, stride, out.send_ids.p);
	HIP_CHECK(hipGetLastError());
	return true;
}

namespace {
__global__ void iota_i32_from_kernel(int32_t* out, size_t n, int32_t first) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = first + int32_t(i);
}
}  // namespace

void k_iota_i32(int32_t* out, size_t n, int32_t first, hipStream_t s) {
	if (!n) return;
	iota_i32_from_kernel<<<grid_for(n, 256), 256, 0, s>>>(out, n, first);
	HIP_CHECK(hipGetLastError());
}

__global__ void iota_i32_kernel(int32_t* out, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = int32_t(i);
}

void k_sorted_slot_index(const uint64_t* slot_ids, size_t n, std::vector<uint64_t>& ids, std::vector<int32_t>& slots,
                         hipStream_t s) {
	ids.clear();
	slots.clear();
	if (!n) return;
	DBuf<uint64_t> k2;
	DBuf<int32_t> v1, v2;
	k2.alloc(n);
	v1.alloc(n);
	v2.alloc(n);
	iota_i32_kernel<<<grid_for(n, 256), 256, 0, s>>>(v1.p, n);
	HIP_CHECK(hipGetLastError());
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, slot_ids, k2.p, v1.p, v2.p, n, 0, 64, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes);
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, bytes, slot_ids, k2.p, v1.p, v2.p, n, 0, 64, s));
	ids = download(k2.p, n, s);
	slots = download(v2.p, n, s);
}

// a host list sorted (and deduplicated): by the device radix sort above a few
// thousand ids (std::sort of 200 K ids takes 5-15 ms on the host), else here
void host_sort_u64(std::vector<uint64_t>& v, bool unique, hipStream_t s) {
	// already in order (lists that arrive sorted: one rank's own, merged runs)
	if (unique ? std::adjacent_find(v.begin(), v.end(), std::greater_equal<uint64_t>()) == v.end()
	           : std::is_sorted(v.begin(), v.end()))
		return;
	if (v.size() < 8192) {
		std::sort(v.begin(), v.end());
		if (unique) v.erase(std::unique(v.begin(), v.end()), v.end());
		return;
	}
	DBuf<uint64_t> d;
	upload(d, v, s);
	const size_t n = unique ? sort_unique_u64(d.p, v.size(), s) : (sort_u64(d.p, v.size(), s), v.size());
	v = download(d.p, n, s);
}

void sort_u64(uint64_t* keys, size_t n, hipStream_t s, int end_bit) {
	if (n < 2) return;
	DBuf<uint64_t> tmp;
	tmp.alloc(n);
	size_t b1 = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, keys, tmp.p, n, 0, end_bit, s));
	DBuf<uint8_t> temp;
	temp.alloc(b1);
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, b1, keys, tmp.p, n, 0, end_bit, s));
	// stream-ordered: every caller reads the keys on `s` (device consumers)
	// or through a download that drains it.  (Round 5 restored a sync here
	// after a Poisson transport failure; the cause was null-stream memsets
	// racing the compute stream, DESIGN.md section 6, not this function.)
	HIP_CHECK(hipMemcpyAsync(keys, tmp.p, n * 8, hipMemcpyDeviceToDevice, s));
}

size_t sort_unique_u64(uint64_t* keys, size_t n, hipStream_t s, int end_bit) {
	if (n == 0) return 0;
	DBuf<uint64_t> tmp;
	tmp.alloc(n);
	DBuf<unsigned long long> nsel;
	nsel.alloc(1);
	size_t b1 = 0, b2 = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, keys, tmp.p, n, 0, end_bit, s));
	HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, b2, tmp.p, keys, nsel.p, n, s));
	DBuf<uint8_t> temp;
	temp.alloc(std::max(b1, b2));
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, b1, keys, tmp.p, n, 0, end_bit, s));
	HIP_CHECK(hipcub::DeviceSelect::Unique(temp.p, b2, tmp.p, keys, nsel.p, n, s));
	return read_counter(nsel, s);
}

namespace {
struct PickU32 {
	size_t at[4];
	int k;
};
__global__ void pick_u32_kernel(const uint32_t* __restrict__ v, PickU32 p, uint32_t* __restrict__ out) {
	if (int(threadIdx.x) < p.k) out[threadIdx.x] = v[p.at[threadIdx.x]];
}
}  // namespace

uint32_t scan_exclusive_u32_at(const uint32_t* in, uint32_t* out, size_t n, hipStream_t s, const size_t* at, int k,
                               uint32_t* vals) {
	DX_REQUIRE(k >= 0 && k <= 3, "internal error: too many scan positions");
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n + 1, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes);
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp.p, bytes, in, out, n + 1, s));
	// the total and the k positions in one read
	PickU32 p{{n, 0, 0, 0}, k + 1};
	for (int j = 0; j < k; j++) p.at[j + 1] = at[j];
	DBuf<uint32_t> picked;
	picked.alloc(4);
	pick_u32_kernel<<<1, 64, 0, s>>>(out, p, picked.p);
	HIP_CHECK(hipGetLastError());
	uint32_t h[4] = {0, 0, 0, 0};
	d2h_small(h, picked.p, sizeof(uint32_t) * size_t(k + 1), s);
	for (int j = 0; j < k; j++) vals[j] = h[j + 1];
	return h[0];
}

void scan_exclusive_u32_pair(const uint32_t* in1, uint32_t* out1, const uint32_t* in2, uint32_t* out2, size_t n,
                             hipStream_t s, size_t& t1, size_t& t2) {
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in1, out1, n + 1, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes + 1);
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp.p, bytes, in1, out1, n + 1, s));
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp.p, bytes, in2, out2, n + 1, s));
	DBuf<uint32_t> tot;
	tot.alloc(2);
	HIP_CHECK(hipMemcpyAsync(tot.p, out1 + n, 4, hipMemcpyDeviceToDevice, s));
	HIP_CHECK(hipMemcpyAsync(tot.p + 1, out2 + n, 4, hipMemcpyDeviceToDevice, s));
	uint32_t h[2] = {0, 0};
	d2h_small(h, tot.p, sizeof(h), s);
	t1 = h[0];
	t2 = h[1];
}

uint32_t scan_exclusive_u32(const uint32_t* in, uint32_t* out, size_t n, hipStream_t s) {
	// scans n + 1 entries: out[n] = sum(in[0..n))
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n + 1, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes);
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp.p, bytes, in, out, n + 1, s));
	uint32_t h = 0;
	d2h_small(&h, out + n, sizeof(h), s);
	return h;
}

void k_lookup_slots(const uint64_t* ids, size_t n, const DevMesh& M, int32_t* out, int32_t* err_flag, hipStream_t s) {
	if (!n) return;
	lookup_slots_kernel<<<grid_for(n, 256), 256, 0, s>>>(ids, n, M, out, err_flag);
	HIP_CHECK(hipGetLastError());
}

void k_iterator_lists(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                      const int32_t* nof_slot, const uint32_t* nto_ptr, const uint64_t* nto_id, size_t nrows,
                      uint8_t* cls, uint32_t* it_cnt, const uint32_t* it_ptr, int32_t* it_slot, int32_t* it_off,
                      int pass, hipStream_t s) {
	if (!nrows) return;
	if (pass == 0)
		iterator_class_kernel<<<grid_for(nrows, 4), 256, 0, s>>>(nof_ptr, nof_id, nof_off, nto_ptr, nto_id, nrows, cls,
		                                                         it_cnt);
	else
		iterator_fill_kernel<<<grid_for(nrows, 4), 256, 0, s>>>(nof_ptr, nof_id, nof_off, nof_slot, cls, nrows, it_ptr,
		                                                        it_slot, it_off);
	HIP_CHECK(hipGetLastError());
}

size_t k_face_table(const MapCtx& m, const DevMesh& M, const uint64_t* slot_ids, size_t nrows, size_t run1,
                    bool morton, int32_t* ell, DBuf<int32_t>& fine, int32_t* err, hipStream_t s) {
	DX_REQUIRE(nrows < (size_t(1) << 29), "too many local cells for the face keys");
	if (nrows && !(std::getenv("DCCRGX_FACE_KEYS") && std::strcmp(std::getenv("DCCRGX_FACE_KEYS"), "sort") == 0)) {
		// finer faces numbered by a scan of per-chunk counts (face_table_kernel)
		const size_t nch = (nrows + 63) / 64;
		DX_REQUIRE(nch * kChunkKeys < (size_t(1) << 32), "too many rows for the chunked face keys");
		DBuf<uint32_t> ckeys, ccnt, coff;
		ckeys.alloc(nch * kChunkKeys);
		ccnt.alloc(nch + 1);
		coff.alloc(nch + 1);
		face_table_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(m, M, slot_ids, nrows, run1, morton && !M.implicit, ell,
		                                                       nullptr, nullptr, 0, err, ckeys.p, ccnt.p);
		HIP_CHECK(hipGetLastError());
		const size_t nf = scan_exclusive_u32(ccnt.p, coff.p, nch, s);
		fine.alloc(4 * nf + 4);
		if (!nf) return 0;
		face_fine_kernel<<<grid_for(nf, 256), 256, 0, s>>>(m, M, slot_ids, nullptr, nf, ell, fine.p, err, ckeys.p, coff.p,
		                                                   uint32_t(nch));
		HIP_CHECK(hipGetLastError());
		return nf;
	}
	DBuf<unsigned long long> n_fine;
	n_fine.alloc(1);
	HIP_CHECK(hipMemsetAsync(n_fine.p, 0, 8, s));
	// finer faces: at most 6 per row, in practice a few percent of the rows;
	// keys row << 3 | direction, room for a quarter of the rows first (the
	// pass runs again with room for all of them if that was too little: it
	// rewrites every row of the table)
	DBuf<uint32_t> keys;
	const char* kc = std::getenv("DCCRGX_FACE_KEY_CAP");  // tests: a small first room forces the second pass
	size_t cap = kc && *kc ? size_t(std::strtoull(kc, nullptr, 10)) : nrows / 4 + 1024;
	size_t nf = 0;
	for (;;) {
		keys.alloc(cap);
		if (nrows)
			face_table_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(m, M, slot_ids, nrows, run1, morton && !M.implicit,
			                                                       ell, n_fine.p, keys.p, cap, err, nullptr, nullptr);
		HIP_CHECK(hipGetLastError());
		nf = size_t(read_counter(n_fine, s));
		if (nf <= cap) break;
		cap = nf;
		HIP_CHECK(hipMemsetAsync(n_fine.p, 0, 8, s));
	}
	fine.alloc(4 * nf + 4);
	if (!nf) return 0;
	int bits = 4;
	while (bits < 32 && (uint64_t(nrows) << 3) >> bits) bits++;
	if (nf > 1) {
		DBuf<uint32_t> sorted;
		sorted.alloc(nf);
		size_t b1 = 0;
		HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, keys.p, sorted.p, nf, 0, bits, s));
		DBuf<uint8_t> temp;
		temp.alloc(b1);
		HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, b1, keys.p, sorted.p, nf, 0, bits, s));
		keys.swap(sorted);
	}
	face_fine_kernel<<<grid_for(nf, 256), 256, 0, s>>>(m, M, slot_ids, keys.p, nf, ell, fine.p, err, nullptr, nullptr, 0);
	HIP_CHECK(hipGetLastError());
	return nf;
}

void k_face_csr(const int32_t* ell, const int32_t* fine, size_t nrows, DBuf<uint32_t>& ptr, DBuf<int32_t>& ent,
                hipStream_t s) {
	DBuf<uint32_t> cnt;
	cnt.alloc(nrows + 1);
	ptr.alloc(nrows + 1);
	if (nrows) face_csr_count_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(ell, nrows, cnt.p);
	HIP_CHECK(hipGetLastError());
	const size_t t = scan_exclusive_u32(cnt.p, ptr.p, nrows, s);
	ent.alloc(t + 1);
	if (nrows) face_csr_fill_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(ell, fine, nrows, ptr.p, ent.p);
	HIP_CHECK(hipGetLastError());
}

void k_carry_src(const uint64_t* slot_ids, size_t n_slots, size_t nl, const MapCtx& m, const DevMesh& oldM,
                 size_t old_n_local, int32_t* src, hipStream_t s) {
	if (!n_slots) return;
	carry_src_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(slot_ids, n_slots, nl, m, oldM, old_n_local, src);
	HIP_CHECK(hipGetLastError());
}

void k_gather_rows(const uint8_t* old_data, const int32_t* src, size_t n, size_t elem, uint8_t* out, hipStream_t s) {
	if (!n || !elem) return;
	if (elem == 4)
		gather_rows_kernel<uint32_t><<<grid_for(n, 256), 256, 0, s>>>((const uint32_t*)old_data, src, n, (uint32_t*)out);
	else if (elem == 8)
		gather_rows_kernel<uint64_t><<<grid_for(n, 256), 256, 0, s>>>((const uint64_t*)old_data, src, n, (uint64_t*)out);
	else if (elem == 16)
		gather_rows_kernel<uint4><<<grid_for(n, 256), 256, 0, s>>>((const uint4*)old_data, src, n, (uint4*)out);
	else
		gather_bytes_kernel<<<grid_for(n * elem, 256), 256, 0, s>>>(old_data, src, n, elem, out);
	HIP_CHECK(hipGetLastError());
}



// Reorder a run of cell ids along the Morton (z-order) curve of their min
// corners at finest-level resolution (leaves have distinct min corners).
void k_morton_sort(const MapCtx& m, uint64_t* ids, size_t n, hipStream_t s) {
	if (n < 2) return;
	DBuf<uint64_t> keys, keys2, ids2;
	keys.alloc(n);
	keys2.alloc(n);
	ids2.alloc(n);
	morton_keys_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, ids, n, keys.p);
	HIP_CHECK(hipGetLastError());
	// the keys' bits: 3 per level of the finest index (9 levels on a 512-wide
	// finest grid: 27 bits, 4 radix passes instead of 8)
	int b = 1;
	while (b < 21 && (uint64_t(1) << b) < std::max(m.glen[0], std::max(m.glen[1], m.glen[2]))) b++;
	const int end_bit = std::min(63, 3 * b);
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, keys.p, keys2.p, ids, ids2.p, n, 0, end_bit, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes);
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, bytes, keys.p, keys2.p, ids, ids2.p, n, 0, end_bit, s));
	HIP_CHECK(hipMemcpyAsync(ids, ids2.p, n * 8, hipMemcpyDeviceToDevice, s));
	HIP_CHECK(hipStreamSynchronize(s));
}

// ids[0, run1) and ids[run1, n) each in Morton order -> ids in Morton order:
// one merge pass (rocprim::merge over the Morton keys) instead of a sort
void k_morton_merge2(const MapCtx& m, uint64_t* ids, size_t n, size_t run1, hipStream_t s) {
	if (run1 == 0 || run1 >= n) return;
	DBuf<uint64_t> keys, keys2, ids2;
	keys.alloc(n);
	keys2.alloc(n);
	ids2.alloc(n);
	morton_keys_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, ids, n, keys.p);
	HIP_CHECK(hipGetLastError());
	size_t bytes = 0;
	HIP_CHECK(rocprim::merge(nullptr, bytes, keys.p, keys.p + run1, keys2.p, ids, ids + run1, ids2.p, run1, n - run1,
	                         rocprim::less<uint64_t>(), s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes + 1);
	HIP_CHECK(rocprim::merge(temp.p, bytes, keys.p, keys.p + run1, keys2.p, ids, ids + run1, ids2.p, run1, n - run1,
	                         rocprim::less<uint64_t>(), s));
	HIP_CHECK(hipMemcpyAsync(ids, ids2.p, n * 8, hipMemcpyDeviceToDevice, s));
	HIP_CHECK(hipStreamSynchronize(s));
}

// ---- ghost region ---------------------------------------------------------------
std::vector<uint64_t> k_ghost_level0(const MapCtx& m, const DevMesh& M, int rank, const uint64_t* local, size_t n,
                                     int radius, hipStream_t s) {
	if (!n) return {};
	// distinct level-0 parents of the local cells; the wholly local ones
	// (leaf volume 8^R) in a keys-only hash set.  Implicit grids: every local
	// cell is a level-0 cell and the block partition tells what is local.
	DBuf<uint64_t> uk, uv, set;
	const uint64_t* par = local;
	size_t np = n;
	KeySet ks{nullptr, 0, 63};
	if (!M.implicit) {
		DBuf<uint64_t> l0, vol, l0s, vols;
		l0.alloc(n);
		vol.alloc(n);
		l0s.alloc(n);
		vols.alloc(n);
		uk.alloc(n);
		uv.alloc(n);
		l0_volume_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, local, n, l0.p, vol.p);
		HIP_CHECK(hipGetLastError());
		DBuf<unsigned long long> nu;
		nu.alloc(1);
		size_t b1 = 0, b2 = 0;
		HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, l0.p, l0s.p, vol.p, vols.p, n, 0, 64, s));
		HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(nullptr, b2, l0s.p, uk.p, vols.p, uv.p, nu.p, hipcub::Sum(), n, s));
		DBuf<uint8_t> temp;
		temp.alloc(std::max(b1, b2));
		HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, b1, l0.p, l0s.p, vol.p, vols.p, n, 0, 64, s));
		HIP_CHECK(hipcub::DeviceReduce::ReduceByKey(temp.p, b2, l0s.p, uk.p, vols.p, uv.p, nu.p, hipcub::Sum(), n, s));
		np = read_counter(nu, s);
		par = uk.p;
		uint32_t bits = 4;
		while ((uint64_t(1) << bits) < 2 * np) bits++;
		set.alloc(size_t(1) << bits);
		HIP_CHECK(hipMemsetAsync(set.p, 0, set.n * 8, s));
		ks = KeySet{set.p, set.n - 1, 64u - bits};
		keyset_insert_kernel<<<grid_for(np, 256), 256, 0, s>>>(set.p, ks.mask, ks.shift, uk.p, uv.p,
		                                                       uint64_t(1) << (3 * m.R), np);
		HIP_CHECK(hipGetLastError());
	}
	unsigned long long cap = 1ull << 22;
	for (;;) {
		DBuf<uint64_t> out;
		out.alloc(size_t(cap));
		DBuf<unsigned long long> ctr;
		zero_counter(ctr, s);
		ghost_l0_kernel<<<grid_for(np, 256), 256, 0, s>>>(m, M, rank, par, np, ks, radius, out.p, ctr.p, cap);
		HIP_CHECK(hipGetLastError());
		const size_t k = read_counter(ctr, s);
		if (k > cap) {
			cap = k;
			continue;
		}
		const size_t u = sort_unique_u64(out.p, k, s, map_id_bits(m));
		return download(out.p, u, s);
	}
}

std::vector<uint64_t> k_cells_under(const MapCtx& m, const uint64_t* local, size_t n, const std::vector<uint64_t>& l0,
                                    hipStream_t s) {
	if (!n || l0.empty()) return {};
	DBuf<uint64_t> dl0, out;
	upload(dl0, l0, s);
	out.alloc(n);
	DBuf<unsigned long long> ctr;
	zero_counter(ctr, s);
	cells_under_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, local, n, dl0.p, l0.size(), out.p, ctr.p);
	HIP_CHECK(hipGetLastError());
	const size_t k = read_counter(ctr, s);
	sort_u64(out.p, k, s, map_id_bits(m));
	return download(out.p, k, s);
}

std::vector<uint64_t> k_induced_refines(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh,
                                        const DevMesh& M, int rank, const std::vector<uint64_t>& req, hipStream_t s,
                                        bool finer, const uint64_t* dreq_given) {
	if (req.empty()) return {};
	DBuf<uint64_t> dreq_own;
	if (!dreq_given) upload(dreq_own, req, s);
	struct {
		const uint64_t* p;
	} dreq{dreq_given ? dreq_given : dreq_own.p};
	unsigned long long cap = req.size() * 16 + 1024;
	for (;;) {
		DBuf<uint64_t> out;
		out.alloc(size_t(cap));
		DBuf<unsigned long long> ctr;
		zero_counter(ctr, s);
		induced_kernel<<<grid_for(req.size(), 4), 256, 0, s>>>(m, hood, hood_to, nh, M, rank, dreq.p, req.size(), out.p,
		                                                       ctr.p, cap, finer ? 1 : 0);
		HIP_CHECK(hipGetLastError());
		const size_t k = read_counter(ctr, s);
		if (k > cap) {
			cap = k;
			continue;
		}
		const size_t u = sort_unique_u64(out.p, k, s, map_id_bits(m));
		return download(out.p, u, s);
	}
}

std::vector<uint64_t> k_unrefine_families(const MapCtx& m, const int32_t* hood, int nh, const DevMesh& M,
                                          const std::vector<uint64_t>& req, const std::vector<uint64_t>& S,
                                          const std::vector<uint64_t>& DU, hipStream_t s, const uint64_t* dS_given,
                                          const uint64_t* dreq_heads) {
	// dreq_heads: req on the device, ascending octant-0 children of level > 0,
	// so their parents come out ascending and distinct (no sort, no marker)
	if (req.empty()) return {};
	DBuf<uint64_t> dr_own, par, dS, dDU;
	if (!dreq_heads) upload(dr_own, req, s);
	const uint64_t* drp = dreq_heads ? dreq_heads : dr_own.p;
	if (!dS_given) upload(dS, S, s);
	const uint64_t* dSp = dS_given ? dS_given : dS.p;
	upload(dDU, DU, s);
	par.alloc(req.size() + 1);
	request_parents_kernel<<<grid_for(req.size(), 256), 256, 0, s>>>(m, drp, req.size(), par.p);
	HIP_CHECK(hipGetLastError());
	size_t n = dreq_heads ? req.size() : sort_unique_u64(par.p, req.size(), s);
	if (!dreq_heads) {
		// the level-0 requests' marker sorts last
		uint64_t last = 0;
		if (n) d2h_small(&last, par.p + n - 1, 8, s);
		if (n && last == ~uint64_t(0)) n--;
	}
	if (!n) return {};
	DBuf<uint32_t> ok;
	ok.alloc(n);
	k_fill_i32(reinterpret_cast<int32_t*>(ok.p), n, 1, s);
	family_blocked_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, par.p, n, dSp, S.size(), dDU.p, DU.size(), ok.p);
	if (nh > 0)
		unrefine_check_kernel<<<grid_for(n * size_t(nh), 256), 256, 0, s>>>(m, hood, nh, M, par.p, n, dSp, S.size(),
		                                                                    ok.p);
	HIP_CHECK(hipGetLastError());
	// candidates and verdicts in one read
	DBuf<uint8_t> stage;
	stage.alloc(12 * n);
	HIP_CHECK(hipMemcpyAsync(stage.p, par.p, 8 * n, hipMemcpyDeviceToDevice, s));
	HIP_CHECK(hipMemcpyAsync(stage.p + 8 * n, ok.p, 4 * n, hipMemcpyDeviceToDevice, s));
	const std::vector<uint8_t> hb = download(stage.p, 12 * n, s);
	std::vector<uint64_t> out;
	for (size_t i = 0; i < n; i++) {
		uint32_t v;
		std::memcpy(&v, hb.data() + 8 * n + 4 * i, 4);
		if (v) {
			uint64_t c;
			std::memcpy(&c, hb.data() + 8 * i, 8);
			out.push_back(c);
		}
	}
	return out;
}

void k_apply_refines(const MapCtx& m, const uint64_t* kid, const int32_t* kown, size_t n, const std::vector<uint64_t>& S,
                     const std::vector<uint64_t>& F, DBuf<uint64_t>& out_id, DBuf<int32_t>& out_own, size_t& n_out,
                     hipStream_t s, const size_t* at, size_t* pos_at, int n_at, size_t n_prefix, const DevMesh* dm,
                     DBuf<int32_t>* src, const uint64_t* dS_given, const uint64_t* dF_given) {
	DBuf<uint64_t> dS_own, dF_own;
	if (!dS_given) upload(dS_own, S, s);
	if (!dF_given) upload(dF_own, F, s);
	struct {
		const uint64_t* p;
	} dS{dS_given ? dS_given : dS_own.p}, dF{dF_given ? dF_given : dF_own.p};
	DBuf<uint32_t> cnt, pos;
	cnt.alloc(n + 1);
	pos.alloc(n + 1);
	HIP_CHECK(hipMemsetAsync(cnt.p, 0, (n + 1) * 4, s));
	// [0, np): the own-leaf prefix classified by lookups; the rest searched
	const size_t np = dm ? std::min(n_prefix, n) : 0;
	DBuf<uint8_t> cls;
	if (np) {
		cls.alloc(np);
		HIP_CHECK(hipMemsetAsync(cls.p, 0, np, s));
		if (!S.empty()) mark_refined_kernel<<<grid_for(S.size(), 256), 256, 0, s>>>(*dm, dS.p, S.size(), np, cls.p);
		if (!F.empty())
			mark_families_kernel<<<grid_for(8 * F.size(), 256), 256, 0, s>>>(m, *dm, dF.p, F.size(), np, cls.p);
		prefix_count_kernel<<<grid_for(np, 256), 256, 0, s>>>(cls.p, np, cnt.p);
		HIP_CHECK(hipGetLastError());
	}
	if (n > np) {
		refine_count_kernel<<<grid_for(n - np, 256), 256, 0, s>>>(m, kid + np, n - np, dS.p, S.size(), dF.p, F.size(),
		                                                          cnt.p + np);
		HIP_CHECK(hipGetLastError());
	}
	// the total and where input positions at[k] land (the expanded list's run
	// boundaries), one read
	DX_REQUIRE(n_at >= 0 && n_at <= 3, "internal error: too many run boundaries");
	uint32_t landed[3] = {0, 0, 0};
	n_out = scan_exclusive_u32_at(cnt.p, pos.p, n, s, at, n_at, landed);
	for (int k = 0; k < n_at; k++) pos_at[k] = landed[k];
	out_id.alloc(n_out + 1);
	out_own.alloc(n_out + 1);
	if (src) {
		src->alloc(n_out + 1);
		// prefix_fill_kernel writes every output of the prefix; only the rest
		// (refine_fill_kernel writes no sources) starts at -1
		if (np < n) HIP_CHECK(hipMemsetAsync(src->p, 0xff, (n_out + 1) * 4, s));
		else HIP_CHECK(hipMemsetAsync(src->p + n_out, 0xff, 4, s));
	}
	if (np) {
		prefix_fill_kernel<<<grid_for(np, 256), 256, 0, s>>>(m, kid, kown, cls.p, np, pos.p, out_id.p, out_own.p,
		                                                     src ? src->p : nullptr);
		HIP_CHECK(hipGetLastError());
	}
	if (n > np) {
		refine_fill_kernel<<<grid_for(n - np, 256), 256, 0, s>>>(m, kid + np, kown + np, n - np, pos.p + np, cnt.p + np,
		                                                         dF.p, F.size(), out_id.p, out_own.p);
		HIP_CHECK(hipGetLastError());
	}
	// stream-ordered for rebuild (its readers run on s); the temporaries go
	// back to the pool, which holds them until a device sync
}

size_t k_created_children(const MapCtx& m, const DevMesh& M, int rank, const std::vector<uint64_t>& S,
                          DBuf<uint64_t>& out, hipStream_t s, const uint64_t* dS_given, bool sorted) {
	if (S.empty()) return 0;
	DBuf<uint64_t> dS_own;
	if (!dS_given) upload(dS_own, S, s);
	struct {
		const uint64_t* p;
	} dS{dS_given ? dS_given : dS_own.p};
	out.alloc(8 * S.size() + 1);
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, 8, s));
	created_children_kernel<<<unsigned((S.size() + 255) / 256), 256, 0, s>>>(m, M, rank, dS.p, S.size(), out.p, ctr.p);
	HIP_CHECK(hipGetLastError());
	const size_t n = read_counter(ctr, s);
	if (sorted) sort_u64(out.p, n, s, map_id_bits(m));
	return n;
}

size_t k_kept_children(const MapCtx& m, const DevMesh& M, int rank, const std::vector<uint64_t>& F,
                       DBuf<uint64_t>& ids, DBuf<int32_t>& slots, hipStream_t s, const uint64_t* dF_given,
                       bool all_local) {
	ids.release();
	slots.release();
	if (F.empty()) return 0;
	DBuf<uint64_t> dF_own, k1, k2;
	DBuf<int32_t> v1;
	if (!dF_given) upload(dF_own, F, s);
	struct {
		const uint64_t* p;
	} dF{dF_given ? dF_given : dF_own.p};
	const size_t cap = 8 * F.size();
	if (all_local && F.size() < (size_t(1) << 31)) {
		LevelGroups G{};
		G.n = 0;
		int last = -1;
		for (size_t i = 0; i < F.size(); i++) {
			const int L = map_level(m, F[i]);
			if (L != last) {
				DX_REQUIRE(G.n < kRangeLevels && L > last, "internal error: merged families not ascending");
				G.lo[G.n++] = uint32_t(i);
				last = L;
			}
		}
		G.lo[G.n] = uint32_t(F.size());
		ids.alloc(cap + 1);
		slots.alloc(cap + 1);
		k1.alloc(cap + 1);
		family_children_kernel<<<grid_for(F.size(), 256), 256, 0, s>>>(m, dF.p, F.size(), k1.p);
		kept_ordered_kernel<<<grid_for(cap, 256), 256, 0, s>>>(M, k1.p, F.size(), G, ids.p, slots.p);
		HIP_CHECK(hipGetLastError());
		return cap;
	}
	k1.alloc(cap + 1);
	k2.alloc(cap + 1);
	v1.alloc(cap + 1);
	slots.alloc(cap + 1);
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, 8, s));
	kept_children_kernel<<<unsigned((cap + 255) / 256), 256, 0, s>>>(m, M, rank, dF.p, F.size(), k1.p, v1.p, ctr.p);
	HIP_CHECK(hipGetLastError());
	const size_t n = read_counter(ctr, s);
	if (n) {
		size_t bytes = 0;
		HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k1.p, k2.p, v1.p, slots.p, n, 0, map_id_bits(m), s));
		DBuf<uint8_t> temp;
		temp.alloc(bytes + 1);
		HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, bytes, k1.p, k2.p, v1.p, slots.p, n, 0, map_id_bits(m), s));
		ids.swap(k2);
	}
	return n;
}

void k_slot_levels(const MapCtx& m, const uint64_t* slot_ids, size_t n, uint8_t* lvl, hipStream_t s) {
	if (!n) return;
	slot_levels_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, slot_ids, n, lvl);
	HIP_CHECK(hipGetLastError());
}

}  // namespace dccrgx
