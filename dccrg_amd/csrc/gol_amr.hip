// Game of life on a refined grid that emulates the unrefined game
// (tests/game_of_life/solve.hpp:37-170, get_live_neighbors; driven by
// tests/game_of_life/unrefined2d.cpp:183-240).  Every leaf carries its state
// and a list of the distinct level-0 parents of its live neighbors
// (the reference's Cell_Data::data = array<uint64_t, 9>: data[0] the state,
// data[1..8] the list, error_cell = 0 terminated, tests/game_of_life/cell.hpp).
//
//   collect  (solve.hpp:46-110): per leaf, walk neighbors_of in stencil
//            order, skip neighbors of the same level-0 parent, append the
//            level-0 parent of every live neighbor once;
//   halo     (solve.hpp:111) - the caller's update_copies_of_remote_neighbors;
//   spread   (solve.hpp:113-150) + rule (152-167): merge the lists of the
//            same-parent neighbors (the siblings) into the own list, count
//            the distinct entries, apply B3/S23.
//
// The reference spreads in place while it loops over cells, so a sibling's
// list may already hold merged entries when it is read.  With at most one
// refinement level (the reference's stated precondition, solve.hpp:35) every
// sibling of a leaf is in its 26-neighborhood, so both the in-place and the
// read-only merge yield the union of all siblings' collected lists: the
// spread kernel reads the collected lists and writes only the state.
//
// Errors are the reference's aborts, raised as status codes: a live
// neighbor list over 8 entries (solve.hpp:98-101, 139-146) and a dead
// neighbor whose level-0 parent was recorded alive through a sibling
// (solve.hpp:81-90, the siblings disagree).  One thread per leaf; the
// neighbor rows are the device neighbors_of CSR (slots); the level-0 parent
// of every slot is decoded once per call.  Integer work, latency bound
// (a dependent gather per neighbor entry).
#include <cstdlib>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

constexpr int kList = 8;  // data[1..8]

__device__ __forceinline__ bool list_insert(uint64_t (&l)[kList], int& n, uint64_t v) {
#pragma unroll
	for (int i = 0; i < kList; i++)
		if (i < n && l[i] == v) return true;
	if (n == kList) return false;
#pragma unroll
	for (int i = 0; i < kList; i++)
		if (i == n) l[i] = v;
	n++;
	return true;
}

__global__ void level0_parent_kernel(MapCtx m, const uint64_t* __restrict__ slot_ids, size_t n,
                                     uint64_t* __restrict__ l0p) {
	const size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	if (s < n) l0p[s] = map_level0_parent(m, slot_ids[s]);
}

// l0p: level-0 parent per slot (local and remote copies), computed once per
// call so the neighbor walks do no id decoding
// The neighbor walks gather K rows ahead (slots, then their level-0 parents
// and states) before consuming them in row order, so K independent gathers
// are in flight per thread instead of one dependent chain.
template <int K>
__global__ void gol_amr_collect_kernel(const uint64_t* __restrict__ l0p, const uint32_t* __restrict__ state,
                                       uint64_t* __restrict__ lst, const uint32_t* __restrict__ ptr,
                                       const int32_t* __restrict__ nslot, size_t s0, size_t s1,
                                       int* __restrict__ err) {
	const size_t s = s0 + blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	if (s >= s1) return;
	const uint64_t parent = l0p[s];
	uint64_t l[kList];
#pragma unroll
	for (int i = 0; i < kList; i++) l[i] = error_cell;
	int n = 0;
	for (uint32_t j = ptr[s], e = ptr[s + 1]; j < e; j += K) {
		int32_t nsk[K];
		uint64_t qk[K];
		uint32_t stk[K];
#pragma unroll
		for (int k = 0; k < K; k++) nsk[k] = j + k < e ? nslot[j + k] : -1;
#pragma unroll
		for (int k = 0; k < K; k++) {
			qk[k] = nsk[k] >= 0 ? l0p[nsk[k]] : parent;
			stk[k] = nsk[k] >= 0 ? state[nsk[k]] : 0u;
		}
#pragma unroll
		for (int k = 0; k < K; k++) {
			const uint64_t q = qk[k];
			if (q == parent) continue;  // also the padding past the row
			if (stk[k] == 0) {
				bool seen = false;
#pragma unroll
				for (int i = 0; i < kList; i++) seen |= (i < n && l[i] == q);
				if (seen) atomicOr(err, 2);
				continue;
			}
			if (!list_insert(l, n, q)) atomicOr(err, 1);
		}
	}
	uint64_t* o = lst + s * kList;
#pragma unroll
	for (int i = 0; i < kList; i++) o[i] = l[i];
}

template <int K>
__global__ void gol_amr_spread_kernel(const uint64_t* __restrict__ slot_ids, const uint64_t* __restrict__ l0p,
                                      uint32_t* __restrict__ state, const uint64_t* __restrict__ lst,
                                      const uint32_t* __restrict__ ptr, const int32_t* __restrict__ nslot,
                                      size_t s0, size_t s1, int* __restrict__ err) {
	const size_t s = s0 + blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	if (s >= s1) return;
	const uint64_t parent = l0p[s];
	uint64_t l[kList];
	int n = 0;
#pragma unroll
	for (int i = 0; i < kList; i++) {
		l[i] = lst[s * kList + i];
		n += l[i] != error_cell;
	}
	// a level-0 leaf is its own level-0 parent: no neighbor shares it
	if (parent != slot_ids[s]) {
		for (uint32_t j = ptr[s], e = ptr[s + 1]; j < e; j += K) {
			int32_t nsk[K];
			bool sib[K];
#pragma unroll
			for (int k = 0; k < K; k++) nsk[k] = j + k < e ? nslot[j + k] : -1;
#pragma unroll
			for (int k = 0; k < K; k++) sib[k] = nsk[k] >= 0 && l0p[nsk[k]] == parent;
#pragma unroll
			for (int k = 0; k < K; k++) {
				if (!sib[k]) continue;
				const uint64_t* nl = lst + size_t(nsk[k]) * kList;
				for (int i = 0; i < kList; i++) {
					const uint64_t v = nl[i];
					if (v == error_cell) break;
					if (!list_insert(l, n, v)) atomicOr(err, 1);
				}
			}
		}
	}
	if (n == 3) state[s] = 1;
	else if (n != 2) state[s] = 0;
}

inline unsigned blocks_for(size_t n, unsigned b) { return unsigned((n + b - 1) / b); }

}  // namespace

void k_gol_amr(int phase, const MapCtx& m, const uint64_t* slot_ids, size_t n_slots, uint64_t* l0p, uint32_t* state,
               uint64_t* lst, const uint32_t* ptr, const int32_t* nslot, size_t s0, size_t s1, int* err,
               hipStream_t s) {
	if (s1 <= s0) return;
	level0_parent_kernel<<<blocks_for(n_slots, 256), 256, 0, s>>>(m, slot_ids, n_slots, l0p);
	// eight neighbor rows gathered ahead (measured on the bench's 11.5 M
	// leaves: 3.02 / 2.25 / 2.20 ms per step with one / four / eight)
	const unsigned nb = blocks_for(s1 - s0, 256);
	if (phase == 0) gol_amr_collect_kernel<8><<<nb, 256, 0, s>>>(l0p, state, lst, ptr, nslot, s0, s1, err);
	else gol_amr_spread_kernel<8><<<nb, 256, 0, s>>>(slot_ids, l0p, state, lst, ptr, nslot, s0, s1, err);
	HIP_CHECK(hipGetLastError());
}

}  // namespace dccrgx
