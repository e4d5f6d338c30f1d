// Device construction of the neighbor structures (replaces the reference's
// per-cell std::map walks: update_neighbors_ dccrg.hpp:9313-9458,
// initialize_neighbors 8240-8289, find_neighbors_of 4339-4680,
// find_neighbors_to 4708-4861, update_remote_neighbor_info 8992-9270,
// recalculate_neighbor_update_send_receive_lists 8590-8752,
// get_face_neighbors_of 2806-2933).
//
// Layout: one wavefront (64 lanes) per cell; lanes own stencil items (or
// neighbors_to candidates); per-cell output positions come from a wave
// prefix scan (shuffle) / ballot + popcount compaction, so every row is
// written in the reference's order without atomics.  Existence of a leaf is
// one load from a dense id-indexed owner table (HBM is 288 GB; the table is
// 4 B per possible id).
#include <hipcub/hipcub.hpp>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

constexpr int WAVE = 64;

struct DevExists {
	const int32_t* owner;
	uint64_t last;
	__device__ bool operator()(uint64_t id) const { return id != 0 && id <= last && owner[id] >= 0; }
};

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

inline unsigned grid_for(size_t n, unsigned per_block, unsigned cap = 256u * 32u) {
	size_t g = (n + per_block - 1) / per_block;
	if (g > cap) g = cap;
	if (g == 0) g = 1;
	return unsigned(g);
}

__device__ void cell_coords(const MapCtx& m, uint64_t id, uint64_t c[3], int& lvl) {
	lvl = map_indices(m, id, c[0], c[1], c[2]);
}

// --------------------------------------------------------------------------
__global__ void fill_i32_kernel(int32_t* p, size_t n, int32_t v) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		p[i] = v;
}

__global__ void scatter_owner_kernel(int32_t* owner_by_id, const uint64_t* ids, const int32_t* owners, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		owner_by_id[ids[i]] = owners[i];
}

__global__ void scatter_slots_kernel(int32_t* slot_by_id, const uint64_t* slot_ids, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		slot_by_id[slot_ids[i]] = int32_t(i);
}

// --------------------------------------------------------------------------
// Pass 1: does a local cell have any remote neighbors_of / neighbors_to?
// (update_remote_neighbor_info 8992-9095).  One wave per cell.
__global__ void remote_flags_kernel(MapCtx m, const int32_t* hood, const int32_t* hood_to, int nh,
                                    const int32_t* owner_by_id, int rank, const uint64_t* cells, size_t n,
                                    uint32_t* flag) {
	const DevExists ex{owner_by_id, m.last};
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t w = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; w < n; w += waves) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, cells[w], c, lvl);
		bool remote = false;
		for (int k = lane_id(); k < nh; k += WAVE) {
			ItemOut o;
			nof_item(m, c, lvl, hood + 3 * k, ex, o);
			for (int i = 0; i < o.n; i++) {
				if (o.id[i] == error_cell) continue;
				const int32_t ow = (o.id[i] <= m.last) ? owner_by_id[o.id[i]] : -1;
				if (ow >= 0 && ow != rank) remote = true;
			}
		}
		for (int k = lane_id(); k < 10 * nh; k += WAVE) {
			const uint64_t f = nto_candidate(m, c, lvl, hood_to, nh, k, ex);
			if (f != error_cell && owner_by_id[f] != rank) remote = true;
		}
		const bool any = __any(remote);
		if (lane_id() == 0) flag[w] = any ? 1u : 0u;
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
	if (cnt > cap) cnt = cap;  // cap = 10*nh rounded up: never reached
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
__global__ void count_rows_kernel(MapCtx m, const int32_t* hood, const int32_t* hood_to, int nh,
                                  const int32_t* owner_by_id, const uint64_t* slot_ids, size_t row0, size_t nrows,
                                  uint32_t* nof_cnt, uint32_t* nto_cnt, int cap) {
	extern __shared__ uint64_t lds[];
	const DevExists ex{owner_by_id, m.last};
	for (size_t r = blockIdx.x; r < nrows; r += gridDim.x) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[row0 + r], c, lvl);
		int n = 0;
		for (int k = lane_id(); k < nh; k += WAVE) {
			ItemOut o;
			nof_item(m, c, lvl, hood + 3 * k, ex, o);
			n += o.n;
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
__global__ void fill_nof_kernel(MapCtx m, const int32_t* hood, int nh, const int32_t* owner_by_id,
                                const uint64_t* slot_ids, size_t row0, size_t nrows, const uint32_t* ptr,
                                uint64_t* ids, int32_t* offs) {
	const DevExists ex{owner_by_id, m.last};
	const size_t waves = size_t(gridDim.x) * (blockDim.x / WAVE);
	for (size_t r = blockIdx.x * size_t(blockDim.x / WAVE) + threadIdx.x / WAVE; r < nrows; r += waves) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[row0 + r], c, lvl);
		size_t base = ptr[r];
		for (int k0 = 0; k0 < nh; k0 += WAVE) {
			const int k = k0 + lane_id();
			ItemOut o;
			o.n = 0;
			if (k < nh) nof_item(m, c, lvl, hood + 3 * k, ex, o);
			const int incl = wave_incl_scan(o.n);
			const size_t pos = base + size_t(incl - o.n);
			for (int i = 0; i < o.n; i++) {
				ids[pos + i] = o.id[i];
				offs[3 * (pos + i) + 0] = o.off[i][0];
				offs[3 * (pos + i) + 1] = o.off[i][1];
				offs[3 * (pos + i) + 2] = o.off[i][2];
			}
			base += size_t(__shfl(incl, WAVE - 1, WAVE));
		}
	}
}

__global__ void fill_nto_kernel(MapCtx m, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                                const uint64_t* slot_ids, size_t row0, size_t nrows, const uint32_t* ptr,
                                uint64_t* ids, int cap) {
	extern __shared__ uint64_t lds[];
	const DevExists ex{owner_by_id, m.last};
	for (size_t r = blockIdx.x; r < nrows; r += gridDim.x) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[row0 + r], c, lvl);
		nto_row(m, hood_to, nh, ex, c, lvl, lds, cap, ids + ptr[r]);
	}
}

// --------------------------------------------------------------------------
__global__ void extract_remote_kernel(const uint64_t* ids, size_t n, const int32_t* owner_by_id, int rank,
                                      uint64_t stride, uint64_t* keys, unsigned long long* counter) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = ids[i];
		if (id == error_cell) continue;
		const int32_t o = owner_by_id[id];
		if (o >= 0 && o != rank) keys[atomicAdd(counter, 1ull)] = uint64_t(o) * stride + id;
	}
}

__global__ void extract_send_kernel(const uint64_t* nto_id, const uint32_t* nto_ptr, const uint64_t* slot_ids,
                                    size_t row0, size_t nrows, const int32_t* owner_by_id, int rank, uint64_t stride,
                                    uint64_t* keys, unsigned long long* counter) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		const uint64_t self = slot_ids[row0 + r];
		for (uint32_t e = nto_ptr[r]; e < nto_ptr[r + 1]; e++) {
			const int32_t o = owner_by_id[nto_id[e]];
			if (o >= 0 && o != rank) keys[atomicAdd(counter, 1ull)] = uint64_t(o) * stride + self;
		}
	}
}

__global__ void lookup_slots_kernel(const uint64_t* ids, size_t n, const int32_t* slot_by_id, int32_t* out,
                                    int32_t* err) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int32_t s = slot_by_id[ids[i]];
		out[i] = s;
		if (s < 0) atomicExch(err, 1);
	}
}

// iterator neighbor list (update_cell_pointers 11451-11500): the row's
// (id, offset) pairs without duplicates.  One thread per row.
__global__ void iterator_lists_kernel(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                                      const int32_t* nof_slot, size_t nrows, uint32_t* it_cnt, const uint32_t* it_ptr,
                                      int32_t* it_slot, int pass) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		const uint32_t b = nof_ptr[r], e = nof_ptr[r + 1];
		uint32_t k = 0;
		for (uint32_t j = b; j < e; j++) {
			bool dup = false;
			for (uint32_t i = b; i < j && !dup; i++) {
				dup = nof_id[i] == nof_id[j] && nof_off[3 * i] == nof_off[3 * j] &&
				      nof_off[3 * i + 1] == nof_off[3 * j + 1] && nof_off[3 * i + 2] == nof_off[3 * j + 2];
			}
			if (dup) continue;
			if (pass == 1) it_slot[it_ptr[r] + k] = nof_slot[j];
			k++;
		}
		if (pass == 0) it_cnt[r] = k;
	}
}

// face lists (get_face_neighbors_of semantics), one thread per local slot
__global__ void face_lists_kernel(MapCtx m, const int32_t* owner_by_id, const int32_t* slot_by_id,
                                  const uint64_t* slot_ids, size_t nrows, uint32_t* cnt, const uint32_t* ptr,
                                  int32_t* ent, int32_t* err, int pass) {
	const DevExists ex{owner_by_id, m.last};
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		uint64_t c[3];
		int lvl;
		cell_coords(m, slot_ids[r], c, lvl);
		uint32_t k = 0;
		for (int dir = 0; dir < 6; dir++) {
			uint64_t out[4];
			const int nf = face_dir(m, c, lvl, dir, ex, out);
			for (int i = 0; i < nf; i++) {
				if (pass == 1) {
					const int32_t s = slot_by_id[out[i]];
					if (s < 0) atomicExch(err, 1);
					ent[ptr[r] + k] = s * 8 + dir;
				}
				k++;
			}
		}
		if (pass == 0) cnt[r] = k;
	}
}

__global__ void remap_field_kernel(const uint8_t* old_data, const uint64_t* old_ids, size_t n_old,
                                   const int32_t* new_slot_by_id, uint64_t last, uint8_t* new_data, size_t elem) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n_old; i += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = old_ids[i];
		if (id == 0 || id > last) continue;
		const int32_t s = new_slot_by_id[id];
		if (s < 0) continue;
		for (size_t b = 0; b < elem; b++) new_data[size_t(s) * elem + b] = old_data[i * elem + b];
	}
}

__global__ void parent_fill_kernel(uint8_t* data, const uint64_t* slot_ids, size_t n, MapCtx m,
                                   const uint8_t* old_data, const int32_t* old_slot_by_id, size_t elem) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = slot_ids[s];
		if (old_slot_by_id[id] >= 0) continue;
		const uint64_t p = map_parent(m, id);
		if (p == error_cell || p == id) continue;
		const int32_t ps = old_slot_by_id[p];
		if (ps < 0) continue;
		for (size_t b = 0; b < elem; b++) data[s * elem + b] = old_data[size_t(ps) * elem + b];
	}
}

__device__ __forceinline__ uint64_t spread3(uint64_t v) {
	v &= 0x1FFFFFull;
	v = (v | (v << 32)) & 0x1F00000000FFFFull;
	v = (v | (v << 16)) & 0x1F0000FF0000FFull;
	v = (v | (v << 8)) & 0x100F00F00F00F00Full;
	v = (v | (v << 4)) & 0x10C30C30C30C30C3ull;
	v = (v | (v << 2)) & 0x1249249249249249ull;
	return v;
}

__global__ void morton_keys_kernel(MapCtx m, const uint64_t* ids, size_t n, uint64_t* keys) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		map_indices(m, ids[i], x, y, z);
		keys[i] = spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
	}
}

// fixed-width face table: per local slot and direction one int32 = the
// neighbor's slot (same size or coarser), -1 (no neighbor), or -2 - k for a
// finer face whose 4 slots are fine[4k..4k+3] (reference order)
__global__ void face_ell_kernel(const uint32_t* ptr, const int32_t* ent, size_t nrows, int32_t* ell, int32_t* fine,
                                unsigned int* nfine) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < nrows; r += size_t(gridDim.x) * blockDim.x) {
		int32_t row[6] = {-1, -1, -1, -1, -1, -1};
		uint32_t e = ptr[r];
		const uint32_t e1 = ptr[r + 1];
		while (e < e1) {
			const int d = ent[e] & 7;
			uint32_t k = e + 1;
			while (k < e1 && (ent[k] & 7) == d) k++;
			if (k - e == 1) {
				row[d] = ent[e] >> 3;
			} else {
				const unsigned int f = atomicAdd(nfine, 1u);
				for (int i = 0; i < 4; i++) fine[4 * size_t(f) + i] = ent[e + i] >> 3;
				row[d] = -2 - int32_t(f);
			}
			e = k;
		}
		for (int d = 0; d < 6; d++) ell[6 * r + d] = row[d];
	}
}

int nto_cap(int nh) {
	int P = 1;
	while (P < 10 * nh) P <<= 1;
	return P;
}

}  // namespace

// ============================================================================
void k_fill_i32(int32_t* p, size_t n, int32_t v, hipStream_t s) {
	if (!n) return;
	fill_i32_kernel<<<grid_for(n, 256), 256, 0, s>>>(p, n, v);
	HIP_CHECK(hipGetLastError());
}

void k_scatter_owner(int32_t* owner_by_id, const uint64_t* ids, const int32_t* owners, size_t n, hipStream_t s) {
	if (!n) return;
	scatter_owner_kernel<<<grid_for(n, 256), 256, 0, s>>>(owner_by_id, ids, owners, n);
	HIP_CHECK(hipGetLastError());
}

void k_scatter_slots(int32_t* slot_by_id, const uint64_t* slot_ids, size_t n, hipStream_t s) {
	if (!n) return;
	scatter_slots_kernel<<<grid_for(n, 256), 256, 0, s>>>(slot_by_id, slot_ids, n);
	HIP_CHECK(hipGetLastError());
}

void k_remote_flags(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                    int rank, const uint64_t* cells, size_t n, uint32_t* flag, hipStream_t s) {
	if (!n) return;
	remote_flags_kernel<<<grid_for(n, 4), 256, 0, s>>>(m, hood, hood_to, nh, owner_by_id, rank, cells, n, flag);
	HIP_CHECK(hipGetLastError());
}

void k_assign_slots2(const uint32_t* flag, const uint32_t* scan_outer, size_t n, size_t n_inner, const uint64_t* cells,
                     uint64_t* slot_ids, hipStream_t s) {
	if (!n) return;
	assign_slots_kernel<<<grid_for(n, 256), 256, 0, s>>>(flag, scan_outer, n, n_inner, cells, slot_ids);
	HIP_CHECK(hipGetLastError());
}

void k_count_rows(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                  const uint64_t* slot_ids, size_t row0, size_t nrows, uint32_t* nof_cnt, uint32_t* nto_cnt,
                  hipStream_t s) {
	if (!nrows) return;
	const int cap = nto_cap(nh);
	count_rows_kernel<<<grid_for(nrows, 1, 256u * 64u), WAVE, size_t(cap) * 8, s>>>(
	    m, hood, hood_to, nh, owner_by_id, slot_ids, row0, nrows, nof_cnt, nto_cnt, cap);
	HIP_CHECK(hipGetLastError());
}

void k_fill_neighbors_of(const MapCtx& m, const int32_t* hood, int nh, const int32_t* owner_by_id,
                         const uint64_t* slot_ids, size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids,
                         int32_t* offs, hipStream_t s) {
	if (!nrows) return;
	fill_nof_kernel<<<grid_for(nrows, 4), 256, 0, s>>>(m, hood, nh, owner_by_id, slot_ids, row0, nrows, ptr, ids,
	                                                    offs);
	HIP_CHECK(hipGetLastError());
}

void k_fill_neighbors_to(const MapCtx& m, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                         const uint64_t* slot_ids, size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids,
                         hipStream_t s) {
	if (!nrows) return;
	const int cap = nto_cap(nh);
	fill_nto_kernel<<<grid_for(nrows, 1, 256u * 64u), WAVE, size_t(cap) * 8, s>>>(m, hood_to, nh, owner_by_id,
	                                                                                slot_ids, row0, nrows, ptr, ids, cap);
	HIP_CHECK(hipGetLastError());
}

size_t k_extract_remote(const uint64_t* ids, size_t n, const int32_t* owner_by_id, int rank, uint64_t stride,
                        uint64_t* keys_out, hipStream_t s) {
	if (!n) return 0;
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, sizeof(unsigned long long), s));
	extract_remote_kernel<<<grid_for(n, 256), 256, 0, s>>>(ids, n, owner_by_id, rank, stride, keys_out, ctr.p);
	HIP_CHECK(hipGetLastError());
	unsigned long long h = 0;
	HIP_CHECK(hipMemcpyAsync(&h, ctr.p, sizeof(h), hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return size_t(h);
}

size_t k_extract_send(const uint64_t* nto_id, const uint32_t* nto_ptr, const uint64_t* slot_ids, size_t row0,
                      size_t nrows, const int32_t* owner_by_id, int rank, uint64_t stride, uint64_t* keys_out,
                      hipStream_t s) {
	if (!nrows) return 0;
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, sizeof(unsigned long long), s));
	extract_send_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(nto_id, nto_ptr, slot_ids, row0, nrows, owner_by_id, rank,
	                                                         stride, keys_out, ctr.p);
	HIP_CHECK(hipGetLastError());
	unsigned long long h = 0;
	HIP_CHECK(hipMemcpyAsync(&h, ctr.p, sizeof(h), hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return size_t(h);
}

size_t sort_unique_u64(uint64_t* keys, size_t n, hipStream_t s) {
	if (n == 0) return 0;
	DBuf<uint64_t> tmp;
	tmp.alloc(n);
	DBuf<unsigned int> nsel;
	nsel.alloc(1);
	size_t b1 = 0, b2 = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, b1, keys, tmp.p, int(n), 0, 64, s));
	HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, b2, tmp.p, keys, nsel.p, int(n), s));
	DBuf<uint8_t> temp;
	temp.alloc(std::max(b1, b2));
	HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, b1, keys, tmp.p, int(n), 0, 64, s));
	HIP_CHECK(hipcub::DeviceSelect::Unique(temp.p, b2, tmp.p, keys, nsel.p, int(n), s));
	unsigned int h = 0;
	HIP_CHECK(hipMemcpyAsync(&h, nsel.p, sizeof(h), hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return size_t(h);
}

uint32_t scan_exclusive_u32(const uint32_t* in, uint32_t* out, size_t n, hipStream_t s) {
	// scans n + 1 entries: out[n] = sum(in[0..n))
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, int(n + 1), s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes);
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp.p, bytes, in, out, int(n + 1), s));
	uint32_t h = 0;
	HIP_CHECK(hipMemcpyAsync(&h, out + n, sizeof(h), hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return h;
}

void k_lookup_slots(const uint64_t* ids, size_t n, const int32_t* slot_by_id, int32_t* out, int32_t* err_flag,
                    hipStream_t s) {
	if (!n) return;
	lookup_slots_kernel<<<grid_for(n, 256), 256, 0, s>>>(ids, n, slot_by_id, out, err_flag);
	HIP_CHECK(hipGetLastError());
}

void k_iterator_lists(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                      const int32_t* nof_slot, size_t nrows, uint32_t* it_cnt, const uint32_t* it_ptr,
                      int32_t* it_slot, int pass, hipStream_t s) {
	if (!nrows) return;
	iterator_lists_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(nof_ptr, nof_id, nof_off, nof_slot, nrows, it_cnt,
	                                                           it_ptr, it_slot, pass);
	HIP_CHECK(hipGetLastError());
}

void k_face_lists(const MapCtx& m, const int32_t* owner_by_id, const int32_t* slot_by_id, const uint64_t* slot_ids,
                  size_t nrows, uint32_t* cnt, const uint32_t* ptr, int32_t* ent, int32_t* err_flag, int pass,
                  hipStream_t s) {
	if (!nrows) return;
	face_lists_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(m, owner_by_id, slot_by_id, slot_ids, nrows, cnt, ptr, ent,
	                                                       err_flag, pass);
	HIP_CHECK(hipGetLastError());
}

void k_remap_field2(const uint8_t* old_data, const uint64_t* old_ids, size_t n_old, const int32_t* new_slot_by_id,
                    uint64_t last, uint8_t* new_data, size_t elem, hipStream_t s) {
	if (!n_old) return;
	remap_field_kernel<<<grid_for(n_old, 256), 256, 0, s>>>(old_data, old_ids, n_old, new_slot_by_id, last, new_data,
	                                                        elem);
	HIP_CHECK(hipGetLastError());
}

void k_parent_fill(uint8_t* data, const uint64_t* slot_ids, size_t n, const int32_t* slot_by_id, const MapCtx& m,
                   const uint8_t* old_data, const int32_t* old_slot_by_id, size_t elem, hipStream_t s) {
	(void)slot_by_id;
	if (!n) return;
	parent_fill_kernel<<<grid_for(n, 256), 256, 0, s>>>(data, slot_ids, n, m, old_data, old_slot_by_id, elem);
	HIP_CHECK(hipGetLastError());
}

size_t k_face_ell(const uint32_t* ptr, const int32_t* ent, size_t nrows, int32_t* ell, int32_t* fine, hipStream_t s) {
	if (!nrows) return 0;
	DBuf<unsigned int> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, 4, s));
	face_ell_kernel<<<grid_for(nrows, 256), 256, 0, s>>>(ptr, ent, nrows, ell, fine, ctr.p);
	HIP_CHECK(hipGetLastError());
	unsigned int h = 0;
	HIP_CHECK(hipMemcpyAsync(&h, ctr.p, 4, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return h;
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
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, keys.p, keys2.p, ids, ids2.p, int(n), 0, 63, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes);
	HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp.p, bytes, keys.p, keys2.p, ids, ids2.p, int(n), 0, 63, s));
	HIP_CHECK(hipMemcpyAsync(ids, ids2.p, n * 8, hipMemcpyDeviceToDevice, s));
	HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace dccrgx
