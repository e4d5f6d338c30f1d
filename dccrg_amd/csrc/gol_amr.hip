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
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

constexpr int kList = 8;  // data[1..8]
constexpr uint32_t kLevel0 = 0x80000000u;  // mesh table: the slot is a level-0 leaf

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

// per mesh: the level-0 parent of every slot (local and remote copies), with
// kLevel0 set on level-0 leaves; and the sort keys (level-0 parent, slot) of
// the slots of refined level-0 cells, whose runs are the sibling groups
__global__ void l0_table_kernel(MapCtx m, const uint64_t* __restrict__ slot_ids, size_t n, uint32_t* __restrict__ l0,
                                uint64_t* __restrict__ keys, unsigned long long* __restrict__ n_level0) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const uint64_t id = slot_ids[s];
		const uint64_t p = map_level0_parent(m, id);
		const bool lvl0 = p == id;
		l0[s] = uint32_t(p) | (lvl0 ? kLevel0 : 0u);
		keys[s] = lvl0 ? ~0ull : ((p << 32) | s);
		if (lvl0) atomicAdd(n_level0, 1ull);
	}
}

__global__ void group_heads_kernel(const uint64_t* __restrict__ keys, size_t n, uint32_t* __restrict__ head) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		head[i] = keys[i] != ~0ull && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32)) ? 1u : 0u;
}

__global__ void group_fill_kernel(const uint64_t* __restrict__ keys, size_t n, const uint32_t* __restrict__ head,
                                  const uint32_t* __restrict__ pos, uint32_t* __restrict__ gptr,
                                  uint32_t* __restrict__ gslot, uint32_t* __restrict__ lvl0, unsigned long long* n_lvl0,
                                  const uint32_t* __restrict__ l0, size_t n_local) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (keys[i] != ~0ull) {
			gslot[i] = uint32_t(keys[i]);
			if (head[i]) gptr[pos[i]] = uint32_t(i);
		}
		if (i < n_local && (l0[i] & kLevel0)) lvl0[atomicAdd(n_lvl0, 1ull)] = uint32_t(i);
	}
}

// per call: (level-0 parent << 1) | alive of every slot, one 4-byte gather
// per neighbor entry in the collect walk
__global__ void pack_kernel(const uint32_t* __restrict__ l0, const uint32_t* __restrict__ state, size_t n,
                            uint32_t* __restrict__ pack) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x)
		pack[s] = ((l0[s] & ~kLevel0) << 1) | (state[s] ? 1u : 0u);
}

// collect (solve.hpp:46-110): the neighbor rows are walked K entries ahead,
// so K independent gathers are in flight per thread
template <int K>
__global__ void gol_amr_collect_kernel(const uint32_t* __restrict__ pack, uint64_t* __restrict__ lst,
                                       const uint32_t* __restrict__ ptr, const int32_t* __restrict__ nslot, size_t s0,
                                       size_t s1, int* __restrict__ err) {
	const size_t s = s0 + blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	if (s >= s1) return;
	const uint32_t parent = pack[s] >> 1;
	uint64_t l[kList];
#pragma unroll
	for (int i = 0; i < kList; i++) l[i] = error_cell;
	int n = 0;
	for (uint32_t j = ptr[s], e = ptr[s + 1]; j < e; j += K) {
		uint32_t pk[K];
#pragma unroll
		for (int k = 0; k < K; k++) {
			const int32_t ns = j + k < e ? nslot[j + k] : -1;
			pk[k] = ns >= 0 ? pack[ns] : (parent << 1);
		}
#pragma unroll
		for (int k = 0; k < K; k++) {
			const uint32_t q = pk[k] >> 1;
			if (q == parent) continue;  // also the padding past the row
			if (!(pk[k] & 1u)) {
				bool seen = false;
#pragma unroll
				for (int i = 0; i < kList; i++) seen |= (i < n && l[i] == uint64_t(q));
				if (seen) atomicOr(err, 2);
				continue;
			}
			if (!list_insert(l, n, uint64_t(q))) atomicOr(err, 1);
		}
	}
	uint64_t* o = lst + s * kList;
#pragma unroll
	for (int i = 0; i < kList; i++) o[i] = l[i];
}

__device__ __forceinline__ void gol_rule(uint32_t* state, size_t s, int n) {
	if (n == 3) state[s] = 1;
	else if (n != 2) state[s] = 0;
}

// spread + rule (solve.hpp:113-167) of a level-0 leaf: no neighbor shares its
// level-0 parent, its own list decides
__global__ void gol_amr_spread0_kernel(const uint32_t* __restrict__ lvl0, size_t n0, uint32_t* __restrict__ state,
                                       const uint64_t* __restrict__ lst, size_t s0, size_t s1) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n0; i += size_t(gridDim.x) * blockDim.x) {
		const size_t s = lvl0[i];
		if (s < s0 || s >= s1) continue;
		int n = 0;
#pragma unroll
		for (int k = 0; k < kList; k++) n += lst[s * kList + k] != error_cell;
		gol_rule(state, s, n);
	}
}

// spread + rule of the leaves of one refined level-0 cell: every member
// merges the lists of its same-parent neighbors, which with one refinement
// level are all its siblings (local or remote copies), so each member's
// merged list is the group's union; computed once, the rule applied to the
// group's members in [s0, s1)
__global__ void gol_amr_spread_groups_kernel(const uint32_t* __restrict__ gptr, size_t ng,
                                             const uint32_t* __restrict__ gslot, uint32_t* __restrict__ state,
                                             const uint64_t* __restrict__ lst, size_t s0, size_t s1,
                                             int* __restrict__ err) {
	for (size_t gi = blockIdx.x * size_t(blockDim.x) + threadIdx.x; gi < ng; gi += size_t(gridDim.x) * blockDim.x) {
		const uint32_t b = gptr[gi], e = gptr[gi + 1];
		bool any = false;
		for (uint32_t j = b; j < e; j++) any |= gslot[j] >= s0 && gslot[j] < s1;
		if (!any) continue;
		uint64_t l[kList];
		int n = 0;
		for (uint32_t j = b; j < e; j++) {
			const uint64_t* nl = lst + size_t(gslot[j]) * kList;
			for (int i = 0; i < kList; i++) {
				const uint64_t v = nl[i];
				if (v == error_cell) break;
				if (!list_insert(l, n, v)) atomicOr(err, 1);
			}
		}
		for (uint32_t j = b; j < e; j++)
			if (gslot[j] >= s0 && gslot[j] < s1) gol_rule(state, gslot[j], n);
	}
}

}  // namespace

void k_gol_amr_tables(const MapCtx& m, const uint64_t* slot_ids, size_t n_slots, size_t n_local, GolAmrTables& T,
                      hipStream_t s) {
	DX_REQUIRE(m.first[1] - 1 <= 0x7fffffffull && n_slots <= 0xffffffffull,
	           "refined game of life: level-0 ids must fit 31 bits");
	T.l0.alloc(n_slots + 1);
	T.pack.alloc(n_slots + 1);
	DBuf<uint64_t> keys, sorted;
	keys.alloc(n_slots + 1);
	sorted.alloc(n_slots + 1);
	DBuf<unsigned long long> cnt;
	cnt.alloc(2);
	HIP_CHECK(hipMemsetAsync(cnt.p, 0, 16, s));
	if (n_slots) {
		l0_table_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(m, slot_ids, n_slots, T.l0.p, keys.p, cnt.p);
		HIP_CHECK(hipGetLastError());
		size_t bytes = 0;
		HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, keys.p, sorted.p, n_slots, 0, 64, s));
		DBuf<uint8_t> temp;
		temp.alloc(bytes + 1);
		HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp.p, bytes, keys.p, sorted.p, n_slots, 0, 64, s));
	}
	DBuf<uint32_t> head, pos;
	head.alloc(n_slots + 1);
	pos.alloc(n_slots + 1);
	HIP_CHECK(hipMemsetAsync(head.p, 0, (n_slots + 1) * 4, s));
	if (n_slots) {
		group_heads_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(sorted.p, n_slots, head.p);
		HIP_CHECK(hipGetLastError());
	}
	const size_t ng = scan_exclusive_u32(head.p, pos.p, n_slots, s);
	T.gptr.alloc(ng + 1);
	T.gslot.alloc(n_slots + 1);
	T.lvl0.alloc(n_local + 1);
	if (n_slots) {
		group_fill_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(sorted.p, n_slots, head.p, pos.p, T.gptr.p, T.gslot.p,
		                                                        T.lvl0.p, cnt.p + 1, T.l0.p, n_local);
		HIP_CHECK(hipGetLastError());
	}
	unsigned long long h[2] = {0, 0};
	HIP_CHECK(hipMemcpyAsync(h, cnt.p, 16, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	// the level-0 slots' keys sort last: the groups end where they begin
	const uint32_t grouped = uint32_t(n_slots - size_t(h[0]));
	HIP_CHECK(hipMemcpyAsync(T.gptr.p + ng, &grouped, 4, hipMemcpyHostToDevice, s));
	HIP_CHECK(hipStreamSynchronize(s));
	T.ng = ng;
	T.n_lvl0 = size_t(h[1]);
	T.valid = true;
}

void k_gol_amr(int phase, GolAmrTables& T, size_t n_slots, uint32_t* state, uint64_t* lst, const uint32_t* ptr,
               const int32_t* nslot, size_t s0, size_t s1, int* err, hipStream_t s) {
	if (s1 <= s0) return;
	if (phase == 0) {
		pack_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(T.l0.p, state, n_slots, T.pack.p);
		HIP_CHECK(hipGetLastError());
		// eight neighbor rows gathered ahead (round 1: 3.02 / 2.25 / 2.20 ms
		// per step with one / four / eight)
		gol_amr_collect_kernel<8><<<unsigned((s1 - s0 + 255) / 256), 256, 0, s>>>(T.pack.p, lst, ptr, nslot, s0, s1,
		                                                                         err);
	} else {
		if (T.n_lvl0)
			gol_amr_spread0_kernel<<<grid_for(T.n_lvl0, 256), 256, 0, s>>>(T.lvl0.p, T.n_lvl0, state, lst, s0, s1);
		if (T.ng)
			gol_amr_spread_groups_kernel<<<grid_for(T.ng, 256), 256, 0, s>>>(T.gptr.p, T.ng, T.gslot.p, state, lst, s0,
			                                                                 s1, err);
	}
	HIP_CHECK(hipGetLastError());
}

}  // namespace dccrgx
