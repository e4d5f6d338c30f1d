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

#include <algorithm>
#include <cstdlib>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

constexpr int kList = 8;  // data[1..8]
constexpr uint32_t kLevel0 = 0x80000000u;  // mesh table: the slot is a level-0 leaf

// the list in registers as 32-bit level-0 ids (< 2^31, checked when the
// tables are built): half the compares of the reference's uint64_t entries
__device__ __forceinline__ bool list_insert(uint32_t (&l)[kList], int& n, uint32_t v) {
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
__global__ void gol_amr_pack_kernel(const uint32_t* __restrict__ l0, const uint32_t* __restrict__ state, size_t n,
                            uint32_t* __restrict__ pack) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x)
		pack[s] = ((l0[s] & ~kLevel0) << 1) | (state[s] ? 1u : 0u);
}

// collect (solve.hpp:46-110), one block per 256 consecutive rows: the
// block's neighbor entries (one contiguous run of the CSR) are read coalesced
// and their packed (level-0 parent, alive) values gathered eight per thread
// in flight into LDS; then every thread walks its own row from LDS (entries
// past the LDS window, in blocks with very long rows, are gathered directly).
// Entries without a slot hold kNoSlot and are skipped like same-parent ones.
constexpr uint32_t kNoSlot = 0xffffffffu;

// XCD-contiguous block order: hardware block b runs on XCD b % 8, so XCD x
// gets the x-th eighth of the logical blocks and the rows neighboring its
// rows (whose packed values it gathers) are fetched into its own L2 once,
// not into all eight (gridDim.x is a multiple of 8)
__device__ __forceinline__ uint32_t xcd_block() {
	return (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
}
__host__ __device__ constexpr unsigned xcd_grid(size_t blocks) { return unsigned((blocks + 7) / 8 * 8); }
constexpr int kCollectRows = 256;
constexpr uint32_t kCollectLds = 8192;  // packed entries staged per block (32 KB)

__device__ __forceinline__ uint32_t gather_pack(const uint32_t* __restrict__ pack, int32_t ns) {
	return ns >= 0 ? pack[ns] : kNoSlot;
}

__global__ __launch_bounds__(kCollectRows) void gol_amr_collect_kernel(const uint32_t* __restrict__ pack,
                                                                      uint64_t* __restrict__ lst,
                                                                      const uint32_t* __restrict__ ptr,
                                                                      const int32_t* __restrict__ nslot, size_t s0,
                                                                      size_t s1, int* __restrict__ err) {
	__shared__ uint32_t sp[kCollectLds];
	const uint32_t tid = threadIdx.x;
	const size_t r0 = s0 + size_t(xcd_block()) * kCollectRows;
	if (r0 >= s1) return;  // block-uniform (the grid is rounded up to whole XCD shares)
	const size_t r1 = r0 + kCollectRows < s1 ? r0 + kCollectRows : s1;
	const uint32_t E0 = ptr[r0], E1 = ptr[r1];
	const uint32_t nE = E1 - E0 < kCollectLds ? E1 - E0 : kCollectLds;
	// stage: 8 coalesced index loads, then their 8 gathers, per thread and round
	for (uint32_t b = 0; b < nE; b += 8 * kCollectRows) {
		int32_t ns[8];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const uint32_t j = b + uint32_t(k) * kCollectRows + tid;
			ns[k] = j < nE ? nslot[E0 + j] : -1;
		}
		uint32_t v[8];
#pragma unroll
		for (int k = 0; k < 8; k++) v[k] = gather_pack(pack, ns[k]);
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const uint32_t j = b + uint32_t(k) * kCollectRows + tid;
			if (j < nE) sp[j] = v[k];
		}
	}
	__syncthreads();
	const size_t s = r0 + tid;
	if (s >= r1) return;
	const uint32_t parent = pack[s] >> 1;
	uint32_t l[kList];
#pragma unroll
	for (int i = 0; i < kList; i++) l[i] = 0;
	int n = 0;
	for (uint32_t j = ptr[s], e = ptr[s + 1]; j < e; j++) {
		const uint32_t pk = j - E0 < nE ? sp[j - E0] : gather_pack(pack, nslot[j]);
		if (pk == kNoSlot) continue;
		const uint32_t q = pk >> 1;
		if (q == parent) continue;
		if (!(pk & 1u)) {
			bool seen = false;
#pragma unroll
			for (int i = 0; i < kList; i++) seen |= (i < n && l[i] == q);
			if (seen) atomicOr(err, 2);
			continue;
		}
		if (!list_insert(l, n, q)) atomicOr(err, 1);
	}
	uint64_t* o = lst + s * kList;
#pragma unroll
	for (int i = 0; i < kList; i++) o[i] = l[i];  // error_cell (0) padded
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
	const size_t gi = size_t(xcd_block()) * blockDim.x + threadIdx.x;
	if (gi >= ng) return;
	const uint32_t b = gptr[gi], e = gptr[gi + 1];
	bool any = false;
	for (uint32_t j = b; j < e; j++) any |= gslot[j] >= s0 && gslot[j] < s1;
	if (!any) return;
	uint32_t l[kList];
	int n = 0;
	for (uint32_t j = b; j < e; j++) {
		// a sibling's whole list in four 16-byte loads, then merged
		const ulonglong2* q = reinterpret_cast<const ulonglong2*>(lst + size_t(gslot[j]) * kList);
		uint64_t v[kList];
#pragma unroll
		for (int i = 0; i < kList / 2; i++) {
			const ulonglong2 t = q[i];
			v[2 * i] = t.x;
			v[2 * i + 1] = t.y;
		}
		bool end = false;
#pragma unroll
		for (int i = 0; i < kList; i++) {
			end |= v[i] == error_cell;
			if (!end && !list_insert(l, n, uint32_t(v[i]))) atomicOr(err, 1);
		}
	}
	for (uint32_t j = b; j < e; j++)
		if (gslot[j] >= s0 && gslot[j] < s1) gol_rule(state, gslot[j], n);
}

// ---- mask path -------------------------------------------------------------
struct L0Geom {
	uint32_t lx, ly, lz, bx, by;
};

__device__ __forceinline__ void l0_unpack(uint32_t c, const L0Geom& G, int& x, int& y, int& z) {
	x = int(c & ((1u << G.bx) - 1u));
	y = int((c >> G.bx) & ((1u << G.by) - 1u));
	z = int(c >> (G.bx + G.by));
}

// offset of level-0 coordinate q from p along an axis of length L, in
// [-1, 1] for a neighbor's parent (a periodic wrap undone); 2 if not
__device__ __forceinline__ int l0_rel(int q, int p, int L) {
	int d = q - p;
	if (d > 1) d -= L;
	else if (d < -1) d += L;
	return d >= -1 && d <= 1 ? d : 2;
}

__global__ void mask_l0c_kernel(MapCtx m, const uint64_t* __restrict__ slot_ids, size_t n, L0Geom G,
                                uint32_t* __restrict__ l0c) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const uint64_t i = map_level0_parent(m, slot_ids[s]) - 1;
		const uint64_t x = i % G.lx, y = (i / G.lx) % G.ly, z = i / (uint64_t(G.lx) * G.ly);
		l0c[s] = uint32_t(x) | (uint32_t(y) << G.bx) | (uint32_t(z) << (G.bx + G.by));
	}
}

// per neighbor entry: slot | code << 27 (code = 9 (dz+1) + 3 (dy+1) + dx+1 of
// the neighbor's level-0 parent from the row's), kEntNone without a slot
constexpr uint32_t kEntNone = 0xffffffffu;
#ifndef DCCRGX_COLLECT_WORDS
#define DCCRGX_COLLECT_WORDS 4
#endif
__global__ void mask_ent_kernel(const uint32_t* __restrict__ ptr, const int32_t* __restrict__ nslot, size_t rows,
                                const uint32_t* __restrict__ l0c, L0Geom G, uint32_t* __restrict__ ent,
                                int* __restrict__ bad) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < rows; r += size_t(gridDim.x) * blockDim.x) {
		int px, py, pz;
		l0_unpack(l0c[r], G, px, py, pz);
		for (uint32_t j = ptr[r], e = ptr[r + 1]; j < e; j++) {
			const int32_t ns = nslot[j];
			if (ns < 0) {
				ent[j] = kEntNone;
				continue;
			}
			int qx, qy, qz;
			l0_unpack(l0c[ns], G, qx, qy, qz);
			const int dx = l0_rel(qx, px, int(G.lx)), dy = l0_rel(qy, py, int(G.ly)), dz = l0_rel(qz, pz, int(G.lz));
			if (dx == 2 || dy == 2 || dz == 2) {
				*bad = 1;
				ent[j] = kEntNone;
				continue;
			}
			ent[j] = uint32_t(ns) | (uint32_t(9 * (dz + 1) + 3 * (dy + 1) + dx + 1) << 27);
		}
	}
}

// collect (solve.hpp:46-110) on the mask path, one block per 256 consecutive
// rows.  Phase 1, over the block's neighbor entries (one contiguous run of
// the CSR): one byte per entry, code | alive << 5 (31: no slot), built from
// the entry's (slot, code) word and a gather of the neighbor's state, four
// entries per 16-byte index load and eight gathers in flight per thread,
// written straight into LDS.  Phase 2, one thread per row: the row walk
// tests and sets bits instead of comparing ids and appends a parent to the
// reference's list (data[1..8], first-seen order) only when its bit is new.
// Entries past the LDS window (blocks with very long rows) are built where
// they are walked.
__device__ __forceinline__ uint32_t mask_entry_byte(uint32_t q, const uint32_t* __restrict__ state) {
	if (q == kEntNone) return 31u;
	return (q >> 27) | (state[q & 0x7ffffffu] ? 32u : 0u);
}

__global__ __launch_bounds__(kCollectRows) void gol_amr_collect_mask_kernel(
    const uint32_t* __restrict__ state, const uint32_t* __restrict__ ent, const uint32_t* __restrict__ ptr,
    const uint32_t* __restrict__ l0c, L0Geom G, uint64_t* __restrict__ lst, uint32_t* __restrict__ mask_out, size_t s0,
    size_t s1, size_t w0, int* __restrict__ err, const int* __restrict__ gate) {
	// entry bytes staged per block; after the walks the same 16 KB hold the
	// block's lists (256 rows x 64 B) for a coalesced store
	// (the lists at a row stride of 80 B: five 16-B slots, conflict-free
	// 16-B stores across a 16-lane group)
	constexpr uint32_t kRowSlots = kList / 2 + 1;
	constexpr uint32_t cap = kCollectRows * kRowSlots * 16;
	static_assert(cap >= 8192, "LDS too small for the entry bytes");
	__shared__ uint32_t sp32[cap / 4];
	const uint32_t tid = threadIdx.x;
	// gated (the exact collect behind the geometric one): nothing to do
	// unless that one met a disagreeing family or an unknown reached cell
	// (err[0] bits 4 | 8); a gated launch has a capped grid whose blocks walk
	// the chunks, an ungated one a block per chunk
	if (gate && (*gate & (4 | 8)) == 0) return;  // block-uniform
	const size_t nchunk = (s1 - s0 + kCollectRows - 1) / kCollectRows;
	for (size_t ch = gate ? blockIdx.x : xcd_block(); ch < nchunk; ch += gate ? gridDim.x : nchunk) {
		const size_t r0 = s0 + ch * kCollectRows;
		const size_t r1 = r0 + kCollectRows < s1 ? r0 + kCollectRows : s1;
		const uint32_t E0 = ptr[r0] & ~3u, E1 = ptr[r1];
		const uint32_t nB = E1 - E0 < cap ? E1 - E0 : cap;
		const uint32_t nw = (nB + 3) / 4;
		const uint4* ent4 = reinterpret_cast<const uint4*>(ent) + (E0 >> 2);
		// the row's own words, needed after the barrier, fly with phase 1
		const size_t s = r0 + tid;
		const bool act = s < r1;
		const uint32_t rb = act ? ptr[s] : 0u, re = act ? ptr[s + 1] : 0u, pc = act ? l0c[s] : 0u;
		// phase 1: kWords index words (4 kWords state gathers) in flight per thread
		constexpr int kWords = DCCRGX_COLLECT_WORDS;
		for (uint32_t w = tid; w < nw; w += kWords * kCollectRows) {
			uint32_t q[4 * kWords];
	#pragma unroll
			for (int c = 0; c < kWords; c++) {
				const uint32_t wc = w + uint32_t(c) * kCollectRows;
				const uint4 e4 = wc < nw ? ent4[wc] : make_uint4(kEntNone, kEntNone, kEntNone, kEntNone);
				q[4 * c] = e4.x;
				q[4 * c + 1] = e4.y;
				q[4 * c + 2] = e4.z;
				q[4 * c + 3] = e4.w;
			}
			uint32_t st[4 * kWords];
	#pragma unroll
			for (int k = 0; k < 4 * kWords; k++) st[k] = q[k] == kEntNone ? 0u : state[q[k] & 0x7ffffffu];
	#pragma unroll
			for (int c = 0; c < kWords; c++) {
				uint32_t out = 0;
	#pragma unroll
				for (int k = 4 * c; k < 4 * c + 4; k++) {
					const uint32_t v = q[k] == kEntNone ? 31u : ((q[k] >> 27) | (st[k] ? 32u : 0u));
					out |= v << (8 * (k & 3));
				}
				const uint32_t wc = w + uint32_t(c) * kCollectRows;
				if (wc < nw) sp32[wc] = out;
			}
		}
		__syncthreads();
		// the walk, branch-free: `mask` the bits of the live parents seen so far,
		// `codes` the list (5 bits per entry, first-seen order), `ebits` the
		// reference's aborts (1: a ninth live parent, 2: a dead neighbor whose
		// parent was already recorded alive); entries without a slot (31) and of
		// the own parent (13) change nothing
		uint32_t mask = 0, n = 0, ebits = 0;
		uint64_t codes = 0;
		auto visit = [&](uint32_t v) {
			const uint32_t c = v & 31u;
			const uint32_t bit = (c != 31u && c != 13u) ? (1u << c) : 0u;
			const uint32_t alive = (v >> 5) & 1u;
			const uint32_t seen = (mask & bit) != 0u ? 1u : 0u;
			const uint32_t fresh = alive & (bit != 0u ? 1u : 0u) & (seen ^ 1u);
			ebits |= ((alive ^ 1u) & seen) << 1;
			ebits |= fresh & (n >= uint32_t(kList) ? 1u : 0u);
			const uint32_t app = fresh & (n < uint32_t(kList) ? 1u : 0u);
			codes |= uint64_t(app ? c : 0u) << (5u * n);
			n += app;
			mask |= alive ? bit : 0u;
		};
		// the row's entry bytes a 4-byte word at a time (E0 is word aligned);
		// bytes of the word outside the row count as "no slot"
		for (uint32_t j = rb & ~3u; j < re; j += 4) {
			uint32_t word;
			if (j - E0 < nB) {
				word = sp32[(j - E0) >> 2];
			} else {
				word = 0;
	#pragma unroll
				for (uint32_t b = 0; b < 4; b++)
					word |= (j + b < re ? mask_entry_byte(ent[j + b], state) : 31u) << (8 * b);
			}
	#pragma unroll
			for (uint32_t b = 0; b < 4; b++) {
				const bool in = j + b >= rb && j + b < re;
				visit(in ? (word >> (8 * b)) & 0xffu : 31u);
			}
		}
		if (ebits) atomicOr(err, int(ebits));
		uint32_t l[kList];
	#pragma unroll
		for (int i = 0; i < kList; i++) l[i] = uint32_t(codes >> (5 * i)) & 31u;
		// level-0 ids of the listed positions: the row's three wrapped x, y, z
		// coordinates once, then per entry 1 + x + y lx + z lx ly
		int px, py, pz;
		l0_unpack(pc, G, px, py, pz);
		auto wrap = [](int v, int L) { return v < 0 ? v + L : (v >= L ? v - L : v); };
		const uint64_t lxy = uint64_t(G.lx) * G.ly;
		const uint64_t X[3] = {uint64_t(wrap(px - 1, int(G.lx))) + 1, uint64_t(px) + 1, uint64_t(wrap(px + 1, int(G.lx))) + 1};
		const uint64_t Y[3] = {uint64_t(wrap(py - 1, int(G.ly))) * G.lx, uint64_t(py) * G.lx,
		                       uint64_t(wrap(py + 1, int(G.ly))) * G.lx};
		const uint64_t Z[3] = {uint64_t(wrap(pz - 1, int(G.lz))) * lxy, uint64_t(pz) * lxy, uint64_t(wrap(pz + 1, int(G.lz))) * lxy};
		uint64_t out[kList];
	#pragma unroll
		for (int i = 0; i < kList; i++) {
			const uint32_t c = l[i], cz = (c * 57u) >> 9, cy = ((c * 11u) >> 5) - 3u * cz, cx = c - 3u * ((c * 11u) >> 5);
			out[i] = uint32_t(i) < n ? X[cx] + Y[cy] + Z[cz] : error_cell;
		}
		// the lists of rows [w0, s1) through LDS: each row's 64 B at its place,
		// then the block's rows stored as one contiguous run, 16 B per lane and
		// instruction, non-temporal (paired A/B: 0.713 -> 0.693 ms per step).
		// Rows below w0 keep their lists in the mask only (the turn's inner
		// cells: no other process reads them, block-uniform skip)
		if (r1 > w0) {
			const size_t rs = r0 > w0 ? r0 : w0;
			__syncthreads();  // every walk done: the staged entry bytes are free
			ulonglong2* so = reinterpret_cast<ulonglong2*>(sp32);
			if (act)
	#pragma unroll
				for (int i = 0; i < kList / 2; i++) so[tid * kRowSlots + i] = make_ulonglong2(out[2 * i], out[2 * i + 1]);
			__syncthreads();
			ulonglong2* dst = reinterpret_cast<ulonglong2*>(lst + rs * kList);
			const uint32_t skip = uint32_t(rs - r0);
			const uint32_t n16 = uint32_t(r1 - rs) * (kList / 2);
			for (uint32_t k = tid; k < n16; k += kCollectRows) {
				typedef unsigned long long u2v __attribute__((ext_vector_type(2)));
				const ulonglong2 v = so[(skip + k / (kList / 2)) * kRowSlots + k % (kList / 2)];
				const u2v w = {v.x, v.y};
				__builtin_nontemporal_store(w, reinterpret_cast<u2v*>(dst + k));
			}
		}
		if (act) mask_out[s] = mask;
		__syncthreads();  // a next chunk reuses the LDS
	}
}

__global__ void gol_amr_spread0_mask_kernel(const uint32_t* __restrict__ lvl0, size_t n0, uint32_t* __restrict__ state,
                                            const uint32_t* __restrict__ mask, size_t s0, size_t s1,
                                            const int* __restrict__ gate) {
	if (gate && (*gate & (4 | 8)) == 0) return;  // block-uniform: the level-0 game did the turn
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n0; i += size_t(gridDim.x) * blockDim.x) {
		const size_t s = lvl0[i];
		if (s < s0 || s >= s1) continue;
		gol_rule(state, s, __popc(mask[s]));
	}
}

// spread + rule of one refined level-0 cell's leaves: the union of the
// siblings' parents is the OR of their masks (a sibling held as a remote
// copy contributes its received list, turned into bits).  Eight lanes per
// group, one member each (a group of more members loops in steps of eight):
// the members' slots and masks are loaded side by side, OR-ed by shuffles.
__device__ __forceinline__ uint32_t remote_mask(const uint64_t* __restrict__ lst, const uint32_t* __restrict__ l0c,
                                                const L0Geom& G, uint32_t gs, int* __restrict__ err) {
	int px, py, pz;
	l0_unpack(l0c[gs], G, px, py, pz);
	uint32_t u = 0;
	for (int i = 0; i < kList; i++) {
		const uint64_t id = lst[size_t(gs) * kList + i];
		if (id == error_cell) break;
		const uint64_t k = id - 1;
		const int qx = int(k % G.lx), qy = int((k / G.lx) % G.ly), qz = int(k / (uint64_t(G.lx) * G.ly));
		const int dx = l0_rel(qx, px, int(G.lx)), dy = l0_rel(qy, py, int(G.ly)), dz = l0_rel(qz, pz, int(G.lz));
		if (dx == 2 || dy == 2 || dz == 2) {
			atomicOr(err, 4);
			continue;
		}
		u |= 1u << (9 * (dz + 1) + 3 * (dy + 1) + dx + 1);
	}
	return u;
}

__global__ void gol_amr_spread_groups_mask_kernel(const uint32_t* __restrict__ gptr, size_t ng,
                                                  const uint32_t* __restrict__ gslot, uint32_t* __restrict__ state,
                                                  const uint32_t* __restrict__ mask, const uint64_t* __restrict__ lst,
                                                  const uint32_t* __restrict__ l0c, L0Geom G, size_t n_local,
                                                  size_t s0, size_t s1, int* __restrict__ err,
                                                  const int* __restrict__ gate) {
	if (gate && (*gate & (4 | 8)) == 0) return;  // block-uniform: the level-0 game did the turn
	// an ungated launch has a thread per group member; a gated one (mostly
	// exiting at once) a capped grid walking the groups
	const size_t stride = size_t(gridDim.x) * blockDim.x;  // a multiple of 64: lanes keep their place
	for (size_t t = size_t(gate ? blockIdx.x : xcd_block()) * blockDim.x + threadIdx.x;; t += stride) {
		const size_t gi = t >> 3;
		if ((t - (t & 63u)) >> 3 >= ng) break;  // the wave's first group is past the end (wave-uniform)
		const uint32_t m = uint32_t(t & 7u);
		const bool live_group = gi < ng;  // lanes of one group share a wave (8 | 64): no early exit
		const uint32_t b = live_group ? gptr[gi] : 0u, e = live_group ? gptr[gi + 1] : 0u;
		uint32_t u = 0, any = 0;
		for (uint32_t j = b + m; j < e; j += 8) {
			const uint32_t gs = gslot[j];
			any |= (gs >= s0 && gs < s1) ? 1u : 0u;
			u |= gs < n_local ? mask[gs] : remote_mask(lst, l0c, G, gs, err);
		}
#pragma unroll
		for (int o = 1; o < 8; o <<= 1) {
			u |= __shfl_xor(u, o, 8);
			any |= __shfl_xor(any, o, 8);
		}
		if (any) {
			const int n = __popc(u);
			if (n > kList && m == 0) atomicOr(err, 1);
			for (uint32_t j = b + m; j < e; j += 8)
				if (gslot[j] >= s0 && gslot[j] < s1) gol_rule(state, gslot[j], n);
		}
		if (!gate) break;  // ungated: one group member per thread
	}
}

// ---- geometric collect ------------------------------------------------------
// With at most one refinement level, the level-0 cells a leaf's stencil
// reaches are fixed by geometry: a level-0 leaf's item h reaches the level-0
// cell at offset h; a level-1 leaf (child octant c) reaches, per axis,
// floor((c + h) / 2) (-1, 0 or +1).  Every neighbor leaf the reference's
// walk (find_neighbors_of, dccrg.hpp:4339-4680) lists for that item lies in
// that level-0 cell, and every level-0 cell reached holds at least one of
// them.  When the known leaves of every level-0 cell agree on their state
// (siblings always do in the emulated game; the reference aborts otherwise,
// solve.hpp:81-90), the live level-0 parents of a row are the reached cells
// whose leaves are alive: the collect needs one byte per level-0 cell instead
// of the row's neighbor entries.  Disagreeing families, or a reached cell
// without a known leaf, set an error bit and the caller runs the exact
// per-entry collect instead.
// The table is laid out in blocks of 2^lb[0] x 2^lb[1] x 2^lb[2] cells (128
// B: 16 x 8 x 1 on a one-layer grid, else 8 x 4 x 4), so the few cells a
// stencil reaches share lines; an axis' part of a cell's index is
// (k >> lb) * bstride + (k & (2^lb - 1)) * istride, the three parts summed
// (lb = 0 everywhere is the plain raster order)
struct GeoBox {
	uint32_t x0, y0, z0, nx, ny, nz;
	int px, py, pz;
	uint32_t lb[3], bstride[3], istride[3];
	__device__ __forceinline__ uint32_t part(int a, uint32_t k) const {
		return (k >> lb[a]) * bstride[a] + (k & ((1u << lb[a]) - 1u)) * istride[a];
	}
	__device__ __forceinline__ bool index(const L0Geom& G, int x, int y, int z, uint32_t& out) const {
		if (x < 0 || x >= int(G.lx)) {
			if (!px) return false;
			x = x < 0 ? x + int(G.lx) : x - int(G.lx);
		}
		if (y < 0 || y >= int(G.ly)) {
			if (!py) return false;
			y = y < 0 ? y + int(G.ly) : y - int(G.ly);
		}
		if (z < 0 || z >= int(G.lz)) {
			if (!pz) return false;
			z = z < 0 ? z + int(G.lz) : z - int(G.lz);
		}
		const uint32_t ix = uint32_t(x) - x0, iy = uint32_t(y) - y0, iz = uint32_t(z) - z0;
		out = ix < nx && iy < ny && iz < nz ? part(0, ix) + part(1, iy) + part(2, iz) : 0xffffffffu;
		return true;
	}
};

// level-0 leaves: their own state (one writer per cell)
__global__ void geo_l0_leaves_kernel(const uint32_t* __restrict__ l0, const uint32_t* __restrict__ l0c,
                                     const uint32_t* __restrict__ state, size_t n, L0Geom G, GeoBox B,
                                     uint8_t* __restrict__ tab) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		if (!(l0[s] & kLevel0)) continue;
		int x, y, z;
		l0_unpack(l0c[s], G, x, y, z);
		uint32_t k;
		if (B.index(G, x, y, z, k) && k != 0xffffffffu) tab[k] = state[s] ? 1u : 2u;
	}
}

// refined level-0 cells: the OR of their known leaves' states (a group is
// one level-0 parent's leaves), eight lanes per group side by side, OR-ed by
// shuffles; both bits set = the leaves disagree
__global__ void geo_l0_groups_kernel(const uint32_t* __restrict__ gptr, size_t ng, const uint32_t* __restrict__ gslot,
                                     const uint32_t* __restrict__ l0c, const uint32_t* __restrict__ state, size_t n_state,
                                     L0Geom G, GeoBox B, uint8_t* __restrict__ tab, int* __restrict__ err) {
	const size_t t = size_t(xcd_block()) * blockDim.x + threadIdx.x;
	const size_t gi = t >> 3;
	const uint32_t m = uint32_t(t & 7u);
	const bool live = gi < ng;  // the eight lanes of a group share a wave: no early exit
	const uint32_t b = live ? gptr[gi] : 0u, e = live ? gptr[gi + 1] : 0u;
	uint32_t v = 0, any = 0;
	for (uint32_t j = b + m; j < e; j += 8) {
		const uint32_t gs = gslot[j];
		if (gs >= n_state) continue;  // a remote cell whose state is never received
		v |= state[gs] ? 1u : 2u;
		any = gs + 1;
	}
#pragma unroll
	for (int o = 1; o < 8; o <<= 1) {
		v |= __shfl_xor(v, o, 8);
		any = max(any, uint32_t(__shfl_xor(int(any), o, 8)));
	}
	if (!live || !any || m != 0) return;
	if (v == 3u) atomicOr(err, 4);
	int x, y, z;
	l0_unpack(l0c[any - 1], G, x, y, z);
	uint32_t k;
	if (B.index(G, x, y, z, k) && k != 0xffffffffu) tab[k] = uint8_t(v);
}

// one axis of a row's reach: for offsets -1, 0, +1 whether the row's stencil
// reaches that level-0 layer (a level-1 leaf only its own and the one on its
// octant's side; nothing beyond a non-periodic boundary), whether that layer
// lies in the table's box, and its offset into the table
__device__ __forceinline__ void geo_axis(int p, uint32_t L, uint32_t b0, uint32_t bn, int per, bool lvl0, int side,
                                         const GeoBox& B, int axis, bool (&reach)[3], bool (&in)[3],
                                         uint32_t (&off)[3]) {
#pragma unroll
	for (int i = 0; i < 3; i++) {
		const int d = i - 1;
		int q = p + d;
		bool r = lvl0 || d == 0 || d == side;
		if (q < 0 || q >= int(L)) {
			r = r && per;
			q = q < 0 ? q + int(L) : q - int(L);
		}
		const uint32_t k = uint32_t(q) - b0;
		reach[i] = r;
		in[i] = k < bn;
		off[i] = B.part(axis, k);
	}
}

// CUBE: neighborhood length 1 (the 26 offsets around the cell: a level-0
// leaf reaches the 26 level-0 cells around it, a level-1 leaf the 7 of its
// octant's 2 x 2 x 2 corner); else length 0 (the 6 faces: a level-0 leaf its
// 6 face neighbors' level-0 cells, a level-1 leaf the 3 on its octant's sides)
template <bool CUBE>
__global__ __launch_bounds__(256) void geo_collect_kernel(const uint32_t* __restrict__ l0c,
                                                          const uint8_t* __restrict__ corner,
                                                          const uint8_t* __restrict__ tab, L0Geom G, GeoBox B,
                                                          size_t n, uint32_t* __restrict__ mask_out,
                                                          uint64_t* __restrict__ lst, size_t w0, int* __restrict__ err) {
	const size_t s = size_t(xcd_block()) * blockDim.x + threadIdx.x;
	if (s >= n) return;
	int px, py, pz;
	l0_unpack(l0c[s], G, px, py, pz);
	const uint32_t c = corner[s];
	const bool lvl0 = c & 0x80u;
	bool rx[3], ry[3], rz[3], ix[3], iy[3], iz[3];
	uint32_t ox[3], oy[3], oz[3];
	geo_axis(px, G.lx, B.x0, B.nx, B.px, lvl0, (c & 1u) ? 1 : -1, B, 0, rx, ix, ox);
	geo_axis(py, G.ly, B.y0, B.ny, B.py, lvl0, (c & 2u) ? 1 : -1, B, 1, ry, iy, oy);
	geo_axis(pz, G.lz, B.z0, B.nz, B.pz, lvl0, (c & 4u) ? 1 : -1, B, 2, rz, iz, oz);
	// every reached cell's byte in flight at once, then the bits; the own
	// level-0 parent (solve.hpp:72-74) is never read
	constexpr int K = CUBE ? 27 : 7;
	uint32_t v[K];
	bool r[K];
#pragma unroll
	for (int t = 0; t < K; t++) {
		int a, b, d;
		if (CUBE) {
			a = t % 3;
			b = (t / 3) % 3;
			d = t / 9;
		} else {  // the centre, then -x, +x, -y, +y, -z, +z
			a = t == 1 ? 0 : (t == 2 ? 2 : 1);
			b = t == 3 ? 0 : (t == 4 ? 2 : 1);
			d = t == 5 ? 0 : (t == 6 ? 2 : 1);
		}
		const bool centre = a == 1 && b == 1 && d == 1;
		r[t] = !centre && rx[a] && ry[b] && rz[d];
		const bool inb = ix[a] && iy[b] && iz[d];
		v[t] = r[t] ? (inb ? uint32_t(tab[ox[a] + oy[b] + oz[d]]) : 0u) : 0u;
	}
	uint32_t mask = 0, e = 0;
#pragma unroll
	for (int t = 0; t < K; t++) {
		int a, b, d;
		if (CUBE) {
			a = t % 3;
			b = (t / 3) % 3;
			d = t / 9;
		} else {
			a = t == 1 ? 0 : (t == 2 ? 2 : 1);
			b = t == 3 ? 0 : (t == 4 ? 2 : 1);
			d = t == 5 ? 0 : (t == 6 ? 2 : 1);
		}
		e |= (r[t] && v[t] == 0u) ? 8u : 0u;  // a reached cell without a known leaf
		mask |= (r[t] && v[t] == 1u) ? (1u << (9 * d + 3 * b + a)) : 0u;
	}
	const uint32_t cnt = __popc(mask);
	if (cnt > uint32_t(kList)) e |= 1u;
	if (e) atomicOr(err, int(e));
	mask_out[s] = mask;
	if (s < w0) return;
	// the row's list for the processes that receive it: the live parents in
	// position order (a set to the receiver's spread), error_cell padded
	auto wrap = [](int v, int L) { return v < 0 ? v + L : (v >= L ? v - L : v); };
	const uint64_t lxy = uint64_t(G.lx) * G.ly;
	uint64_t out[kList];
	uint32_t m = mask;
#pragma unroll
	for (int i = 0; i < kList; i++) {
		out[i] = error_cell;
		if (!m) continue;
		const int b = __ffs(m) - 1;
		m &= m - 1u;
		const int bz = b / 9, by = (b / 3) % 3, bx = b % 3;
		out[i] = 1 + uint64_t(wrap(px + bx - 1, int(G.lx))) + uint64_t(wrap(py + by - 1, int(G.ly))) * G.lx +
		         uint64_t(wrap(pz + bz - 1, int(G.lz))) * lxy;
	}
	ulonglong2* o = reinterpret_cast<ulonglong2*>(lst + s * kList);
#pragma unroll
	for (int i = 0; i < kList / 2; i++) o[i] = make_ulonglong2(out[2 * i], out[2 * i + 1]);
}

// ---- the level-0 game -------------------------------------------------------
// On one process with at most one refinement level every leaf is local and a
// refined level-0 cell's whole family is: the union of the children's reaches
// (each its octant's corner) is the parent's own 3 x 3 x 3 (or 6-face) reach,
// so the spread's count for every leaf of a level-0 cell is the number of
// live level-0 cells around that cell.  One row per level-0 cell instead of
// one per leaf: a level-0 leaf, or a family - the eight children of a refined
// level-0 cell are eight consecutive slots in Morton order, octant 0 first.
// Both passes run over the slots (coalesced reads of the octant byte, the
// packed level-0 coordinates and the states); the first slot of a family
// speaks for it.  The table pass writes each level-0 cell's byte (the
// family's OR, a disagreement flagged as the geometric collect does), the
// game pass counts the row's live neighbors in the table once and applies
// the rule (solve.hpp:150-167) to its leaves.  Same table, same error bits;
// no masks, no lists (none leave the process).
__global__ __launch_bounds__(256) void lg_table_kernel(const uint32_t* __restrict__ rows, size_t nrows,
                                                       const uint8_t* __restrict__ corner,
                                                       const uint32_t* __restrict__ l0c,
                                                       const uint32_t* __restrict__ state, L0Geom G, GeoBox B,
                                                       uint8_t* __restrict__ tab, int* __restrict__ err) {
	const size_t r = size_t(xcd_block()) * blockDim.x + threadIdx.x;
	if (r >= nrows) return;
	const uint32_t s = rows[r];
	const uint32_t c = corner[s];
	uint32_t v;
	if (c & 0x80u) {
		v = state[s] ? 1u : 2u;
	} else {
		v = 0;
#pragma unroll
		for (int k = 0; k < 8; k++) v |= state[s + k] ? 1u : 2u;
		if (v == 3u) atomicOr(err, 4);
	}
	int x, y, z;
	l0_unpack(l0c[s], G, x, y, z);
	uint32_t k;
	if (B.index(G, x, y, z, k) && k != 0xffffffffu) tab[k] = uint8_t(v);
}

// live level-0 cells among the reach items t = t0, t0 + DT, ... (< 27, or 7
// for the faces) around the level-0 cell (px, py, pz): the three axes'
// offsets into the table first (geo_axis, a level-0 reach), then every item's
// byte in flight at once; bit 3 of `e` for a reached cell without a known
// leaf
// FLAT: a one-cell-thick, non-periodic z axis (a 2-D game such as
// unrefined2d.cpp): only the own plane is reached, so the items off it are
// dropped at compile time (the same count: they were unreached)
template <bool CUBE, int T0MAX, int DT, bool FLAT = false>
__device__ __forceinline__ uint32_t lg_count(const uint8_t* __restrict__ tab, const L0Geom& G, const GeoBox& B, int px,
                                             int py, int pz, int t0, uint32_t& e) {
	constexpr int K = CUBE ? 27 : 7;
	constexpr int N = (K + DT - 1) / DT;  // items per caller
	bool rx[3], ry[3], rz[3], ix[3], iy[3], iz[3];
	uint32_t ox[3], oy[3], oz[3];
	geo_axis(px, G.lx, B.x0, B.nx, B.px, true, 0, B, 0, rx, ix, ox);
	geo_axis(py, G.ly, B.y0, B.ny, B.py, true, 0, B, 1, ry, iy, oy);
	if (FLAT) {
#pragma unroll
		for (int i = 0; i < 3; i++) {
			rz[i] = i == 1;
			iz[i] = i == 1;
			oz[i] = i == 1 ? B.part(2, uint32_t(pz) - B.z0) : 0u;
		}
	} else {
		geo_axis(pz, G.lz, B.z0, B.nz, B.pz, true, 0, B, 2, rz, iz, oz);
	}
	uint32_t v[N];
	bool r[N];
#pragma unroll
	for (int j = 0; j < N; j++) {
		const int t = (T0MAX == 0 ? 0 : t0) + j * DT;
		int a = 1, b = 1, d = 1;
		if (CUBE) {
			a = t % 3;
			b = (t / 3) % 3;
			d = t / 9;
		} else {  // the centre, then -x, +x, -y, +y, -z, +z
			a = t == 1 ? 0 : (t == 2 ? 2 : 1);
			b = t == 3 ? 0 : (t == 4 ? 2 : 1);
			d = t == 5 ? 0 : (t == 6 ? 2 : 1);
		}
		const bool centre = a == 1 && b == 1 && d == 1;  // the own level-0 cell (solve.hpp:72-74)
		if (FLAT && d != 1) {  // off the own plane: never reached
			r[j] = false;
			v[j] = 0;
			continue;
		}
		// a, b, d in 0..2 (clamped for the lanes past the last item)
		a = min(max(a, 0), 2);
		b = min(max(b, 0), 2);
		d = min(max(d, 0), 2);
		r[j] = t < K && !centre && rx[a] && ry[b] && rz[d];
		const bool inb = ix[a] && iy[b] && iz[d];
		v[j] = r[j] ? (inb ? uint32_t(tab[ox[a] + oy[b] + oz[d]]) : 0u) : 0u;
	}
	uint32_t cnt = 0;
#pragma unroll
	for (int j = 0; j < N; j++) {
		e |= (r[j] && v[j] == 0u) ? 8u : 0u;
		cnt += (r[j] && v[j] == 1u) ? 1u : 0u;
	}
	return cnt;
}

// whether every family is eight consecutive slots, octant 0 first (the
// level-0 game's layout): bad = 1 otherwise
__global__ void lg_layout_check_kernel(const uint8_t* __restrict__ corner, const uint32_t* __restrict__ l0c, size_t n,
                                       int* __restrict__ bad) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const uint32_t c = corner[s];
		if (c & 0x80u) continue;
		if (c != 0u) {
			if (s < c || corner[s - c] != 0u || l0c[s - c] != l0c[s]) atomicExch(bad, 1);
			continue;
		}
		for (uint32_t k = 1; k < 8; k++)
			if (s + k >= n || corner[s + k] != k || l0c[s + k] != l0c[s]) {
				atomicExch(bad, 1);
				break;
			}
	}
}

// the level-0 game's rows: the slots of level-0 leaves and of families'
// first children, ascending (flags, then the scan's positions)
__global__ void lg_row_flags_kernel(const uint8_t* __restrict__ corner, size_t n, uint32_t* __restrict__ flag) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const uint32_t c = corner[s];
		flag[s] = ((c & 0x80u) || c == 0u) ? 1u : 0u;
	}
}

__global__ void lg_row_fill_kernel(const uint32_t* __restrict__ flag, const uint32_t* __restrict__ pos, size_t n,
                                   uint32_t* __restrict__ rows) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x)
		if (flag[s]) rows[pos[s]] = uint32_t(s);
}

// gated on err[0]: a disagreeing family (bit 2, from the table pass) leaves
// every state to the exact collect + spread that run instead
template <bool CUBE, bool FLAT>
__global__ __launch_bounds__(256) void lg_game_kernel(const uint32_t* __restrict__ rows, size_t nrows,
                                                      const uint8_t* __restrict__ corner,
                                                      const uint32_t* __restrict__ l0c, uint32_t* __restrict__ state,
                                                      const uint8_t* __restrict__ tab, L0Geom G, GeoBox B,
                                                      int* __restrict__ err) {
	if (__builtin_nontemporal_load(err) & 4) return;  // uniform
	const size_t r = size_t(xcd_block()) * blockDim.x + threadIdx.x;
	if (r >= nrows) return;
	const uint32_t s = rows[r];
	const uint32_t c = corner[s];
	int x, y, z;
	l0_unpack(l0c[s], G, x, y, z);
	uint32_t e = 0;
	const uint32_t cnt = lg_count<CUBE, 0, 1, FLAT>(tab, G, B, x, y, z, 0, e);
	if (cnt > uint32_t(kList)) e |= 1u;
	if (e) atomicOr(err, int(e));
	const int nm = (c & 0x80u) ? 1 : 8;
	for (int k = 0; k < nm; k++) gol_rule(state, size_t(s) + size_t(k), int(cnt));
}

// per local slot: the child octant of a level-1 leaf, bit 7 for a level-0 leaf
__global__ void geo_corner_kernel(MapCtx m, const uint64_t* __restrict__ ids, size_t n, uint8_t* __restrict__ corner) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		const int l = map_indices(m, ids[s], x, y, z);
		corner[s] = l <= 0 ? 0x80u : uint8_t((x & 1u) | ((y & 1u) << 1) | ((z & 1u) << 2));
	}
}

// bounding box of the known level-0 coordinates (min / max per axis)
__global__ void geo_bbox_kernel(const uint32_t* __restrict__ l0c, size_t n, L0Geom G, int* __restrict__ mm) {
	int lo[3] = {1 << 30, 1 << 30, 1 << 30}, hi[3] = {-1, -1, -1};
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		int v[3];
		l0_unpack(l0c[s], G, v[0], v[1], v[2]);
		for (int d = 0; d < 3; d++) {
			lo[d] = min(lo[d], v[d]);
			hi[d] = max(hi[d], v[d]);
		}
	}
	for (int d = 0; d < 3; d++) {
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			lo[d] = min(lo[d], __shfl_xor(lo[d], o, 64));
			hi[d] = max(hi[d], __shfl_xor(hi[d], o, 64));
		}
	}
	// one atomic per block and bound (same-address atomics serialise)
	__shared__ int sl[3][4], shh[3][4];
	const unsigned w = threadIdx.x >> 6;
	if ((threadIdx.x & 63u) == 0)
		for (int d = 0; d < 3; d++) {
			sl[d][w] = lo[d];
			shh[d][w] = hi[d];
		}
	__syncthreads();
	if (threadIdx.x < 3) {
		const int d = int(threadIdx.x);
		int a = sl[d][0], b = shh[d][0];
		for (unsigned k = 1; k < (blockDim.x >> 6); k++) {
			a = min(a, sl[d][k]);
			b = max(b, shh[d][k]);
		}
		atomicMin(mm + d, a);
		atomicMax(mm + 3 + d, b);
	}
}

}  // namespace

static uint32_t bits_for(uint64_t len) {
	uint32_t b = 0;
	while ((uint64_t(1) << b) < len) b++;
	return b;
}

void k_gol_amr_tables(const MapCtx& m, const uint64_t* slot_ids, size_t n_slots, size_t n_local, unsigned hood_len,
                      const uint32_t* ptr, const int32_t* nslot, GolAmrTables& T, hipStream_t s) {
	DX_REQUIRE(m.first[1] - 1 < 0x7fffffffull && n_slots <= 0xffffffffull,
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
	d2h_small(h, cnt.p, 16, s);
	// the level-0 slots' keys sort last: the groups end where they begin
	const uint32_t grouped = uint32_t(n_slots - size_t(h[0]));
	h2d(T.gptr.p + ng, &grouped, 4, s);
	HIP_CHECK(hipStreamSynchronize(s));
	T.ng = ng;
	T.n_lvl0 = size_t(h[1]);

	// mask path: neighborhood length <= 1, slots < 2^27, packed level-0 coordinates in 31 bits
	const uint32_t bx = bits_for(m.len[0]), by = bits_for(m.len[1]), bz = bits_for(m.len[2]);
	T.mask_path = false;
	T.l0c.release();
	T.ent.release();
	T.mask.release();
	if (hood_len <= 1 && n_slots < (size_t(1) << 27) && bx + by + bz <= 31) {
		const L0Geom G{uint32_t(m.len[0]), uint32_t(m.len[1]), uint32_t(m.len[2]), bx, by};
		T.bx = bx;
		T.by = by;
		T.lx = G.lx;
		T.ly = G.ly;
		T.lz = G.lz;
		T.l0c.alloc(n_slots + 1);
		T.mask.alloc(n_slots + 1);
		uint32_t total = 0;
		if (n_local) d2h_small(&total, ptr + n_local, 4, s);
		T.ent.alloc(size_t(total) + 4);  // whole 16-byte words for the values pass
		T.n_ent = total;
		HIP_CHECK(hipMemsetAsync(T.ent.p, 0xff, T.ent.n * 4, s));  // padding = no slot
		DBuf<int> bad;
		bad.alloc(1);
		HIP_CHECK(hipMemsetAsync(bad.p, 0, 4, s));
		if (n_slots) {
			mask_l0c_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(m, slot_ids, n_slots, G, T.l0c.p);
			HIP_CHECK(hipGetLastError());
		}
		if (n_local) {
			mask_ent_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(ptr, nslot, n_local, T.l0c.p, G, T.ent.p, bad.p);
			HIP_CHECK(hipGetLastError());
		}
		int hb = 0;
		d2h_small(&hb, bad.p, 4, s);
		T.mask_path = hb == 0;
	}
	// geometric collect: maximum refinement level <= 1 on the mask path, the
	// level-0 cells of the known region's bounding box in one table
	T.geo = false;
	T.lg_layout = false;
	T.corner.release();
	T.l0tab.release();
	if (T.mask_path && m.R <= 1 && n_slots) {
		const L0Geom G{T.lx, T.ly, T.lz, T.bx, T.by};
		DBuf<int> mm;
		mm.alloc(6);
		const int init[6] = {1 << 30, 1 << 30, 1 << 30, -1, -1, -1};
		h2d(mm.p, init, sizeof(init), s);
		geo_bbox_kernel<<<std::min<unsigned>(grid_for(n_slots, 256), 1024), 256, 0, s>>>(T.l0c.p, n_slots, G, mm.p);
		HIP_CHECK(hipGetLastError());
		int h[6];
		d2h_small(h, mm.p, sizeof(h), s);
		const uint32_t L[3] = {T.lx, T.ly, T.lz};
		for (int d = 0; d < 3; d++) {
			T.per[d] = m.periodic[d];
			// a periodic axis whose known coordinates touch both ends wraps:
			// the whole axis
			const bool whole = m.periodic[d] && h[d] == 0 && h[3 + d] == int(L[d]) - 1;
			T.box0[d] = whole ? 0u : uint32_t(h[d]);
			T.boxn[d] = whole ? L[d] : uint32_t(h[3 + d] - h[d] + 1);
		}
		// 128-cell blocks (GeoBox), the box rounded up to whole blocks
#if DCCRGX_GEO_RASTER
		const uint32_t lb[3] = {0, 0, 0};
#else
		const uint32_t lb[3] = {T.boxn[2] == 1 ? 4u : 3u, T.boxn[2] == 1 ? 3u : 2u, T.boxn[2] == 1 ? 0u : 2u};
#endif
		uint64_t nb[3], vol = uint64_t(1) << (lb[0] + lb[1] + lb[2]);
		for (int d = 0; d < 3; d++) {
			nb[d] = (uint64_t(T.boxn[d]) + (uint64_t(1) << lb[d]) - 1) >> lb[d];
			vol *= nb[d];
		}
		const uint64_t bv = uint64_t(1) << (lb[0] + lb[1] + lb[2]);
		for (int d = 0; d < 3; d++) T.geo_lb[d] = lb[d];
		T.geo_bstride[0] = uint32_t(bv);
		T.geo_bstride[1] = uint32_t(std::min<uint64_t>(nb[0] * bv, 0xffffffffu));
		T.geo_bstride[2] = uint32_t(std::min<uint64_t>(nb[0] * nb[1] * bv, 0xffffffffu));
		T.geo_istride[0] = 1u;
		T.geo_istride[1] = 1u << lb[0];
		T.geo_istride[2] = 1u << (lb[0] + lb[1]);
		if (vol < (uint64_t(1) << 31)) {
			T.l0tab.alloc(size_t(vol));
			HIP_CHECK(hipMemsetAsync(T.l0tab.p, 0, size_t(vol), s));
			T.corner.alloc(n_local + 1);
			if (n_local) {
				geo_corner_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(m, slot_ids, n_local, T.corner.p);
				HIP_CHECK(hipGetLastError());
			}
			// the level-0 game's layout (families as eight consecutive slots)
			T.lg_layout = false;
			if (n_local) {
				DBuf<int> bad;
				bad.alloc(1);
				HIP_CHECK(hipMemsetAsync(bad.p, 0, 4, s));
				lg_layout_check_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(T.corner.p, T.l0c.p, n_local, bad.p);
				HIP_CHECK(hipGetLastError());
				int hb = 1;
				d2h_small(&hb, bad.p, 4, s);
				T.lg_layout = hb == 0;
			}
			if (T.lg_layout) {
				DBuf<uint32_t> flag, pos;
				flag.alloc(n_local + 1);
				pos.alloc(n_local + 1);
				lg_row_flags_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(T.corner.p, n_local, flag.p);
				HIP_CHECK(hipGetLastError());
				T.n_lg_rows = scan_exclusive_u32(flag.p, pos.p, n_local, s);
				T.lg_rows.alloc(T.n_lg_rows + 1);
				lg_row_fill_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(flag.p, pos.p, n_local, T.lg_rows.p);
				HIP_CHECK(hipGetLastError());
			}
			HIP_CHECK(hipStreamSynchronize(s));
			T.geo = true;
		}
	}
	T.valid = true;
}

void k_gol_amr_geo(GolAmrTables& T, const int32_t* hood, int nh, const uint32_t* state, size_t n_local, size_t n_state,
                   uint64_t* lst, size_t list_from, int* err, hipStream_t s) {
	DX_REQUIRE(T.geo && (nh == 26 || nh == 6), "geometric collect not available");
	const L0Geom G{T.lx, T.ly, T.lz, T.bx, T.by};
	const GeoBox B{T.box0[0],
	               T.box0[1],
	               T.box0[2],
	               T.boxn[0],
	               T.boxn[1],
	               T.boxn[2],
	               T.per[0],
	               T.per[1],
	               T.per[2],
	               {T.geo_lb[0], T.geo_lb[1], T.geo_lb[2]},
	               {T.geo_bstride[0], T.geo_bstride[1], T.geo_bstride[2]},
	               {T.geo_istride[0], T.geo_istride[1], T.geo_istride[2]}};
	if (n_state) {
		geo_l0_leaves_kernel<<<grid_for(n_state, 256), 256, 0, s>>>(T.l0.p, T.l0c.p, state, n_state, G, B, T.l0tab.p);
		HIP_CHECK(hipGetLastError());
	}
	if (T.ng) {
		geo_l0_groups_kernel<<<xcd_grid((8 * T.ng + 255) / 256), 256, 0, s>>>(T.gptr.p, T.ng, T.gslot.p, T.l0c.p, state,
		                                                                      n_state, G, B, T.l0tab.p, err);
		HIP_CHECK(hipGetLastError());
	}
	if (n_local) {
		const unsigned nb = xcd_grid((n_local + 255) / 256);
		if (nh == 26)
			geo_collect_kernel<true><<<nb, 256, 0, s>>>(T.l0c.p, T.corner.p, T.l0tab.p, G, B, n_local, T.mask.p, lst,
			                                            list_from, err);
		else
			geo_collect_kernel<false><<<nb, 256, 0, s>>>(T.l0c.p, T.corner.p, T.l0tab.p, G, B, n_local, T.mask.p, lst,
			                                             list_from, err);
		HIP_CHECK(hipGetLastError());
	}
}

// the level-0 game (one process): table + game, two launches over the slots
void k_gol_amr_level0_game(GolAmrTables& T, const int32_t* hood, int nh, uint32_t* state, size_t n_local, int* err,
                           hipStream_t s) {
	DX_REQUIRE(T.geo && T.lg_layout && (nh == 26 || nh == 6), "level-0 game not available");
	if (!n_local) return;
	const L0Geom G{T.lx, T.ly, T.lz, T.bx, T.by};
	const GeoBox B{T.box0[0],
	               T.box0[1],
	               T.box0[2],
	               T.boxn[0],
	               T.boxn[1],
	               T.boxn[2],
	               T.per[0],
	               T.per[1],
	               T.per[2],
	               {T.geo_lb[0], T.geo_lb[1], T.geo_lb[2]},
	               {T.geo_bstride[0], T.geo_bstride[1], T.geo_bstride[2]},
	               {T.geo_istride[0], T.geo_istride[1], T.geo_istride[2]}};
	const size_t nr = T.n_lg_rows;
	if (!nr) return;
	const unsigned nb = xcd_grid((nr + 255) / 256);
	lg_table_kernel<<<nb, 256, 0, s>>>(T.lg_rows.p, nr, T.corner.p, T.l0c.p, state, G, B, T.l0tab.p, err);
	HIP_CHECK(hipGetLastError());
	// a one-cell-thick non-periodic z axis: the 2-D form of the count
	// (DCCRGX_LG_FLAT=0: the general one)
	static const bool no_flat = std::getenv("DCCRGX_LG_FLAT") && std::atoi(std::getenv("DCCRGX_LG_FLAT")) == 0;
	const bool flat = !no_flat && T.lz == 1 && !T.per[2];
	if (nh == 26 && flat)
		lg_game_kernel<true, true><<<nb, 256, 0, s>>>(T.lg_rows.p, nr, T.corner.p, T.l0c.p, state, T.l0tab.p, G, B, err);
	else if (nh == 26)
		lg_game_kernel<true, false><<<nb, 256, 0, s>>>(T.lg_rows.p, nr, T.corner.p, T.l0c.p, state, T.l0tab.p, G, B, err);
	else if (flat)
		lg_game_kernel<false, true><<<nb, 256, 0, s>>>(T.lg_rows.p, nr, T.corner.p, T.l0c.p, state, T.l0tab.p, G, B, err);
	else
		lg_game_kernel<false, false><<<nb, 256, 0, s>>>(T.lg_rows.p, nr, T.corner.p, T.l0c.p, state, T.l0tab.p, G, B,
		                                                err);
	HIP_CHECK(hipGetLastError());
}

void k_gol_amr(int phase, GolAmrTables& T, size_t n_slots, size_t n_local, uint32_t* state, uint64_t* lst, const uint32_t* ptr,
               const int32_t* nslot, size_t s0, size_t s1, int* err, hipStream_t s, size_t list_from, const int* gate) {
	if (s1 <= s0) return;
	DX_REQUIRE(!gate || T.mask_path, "internal error: gated refined-game launch off the mask path");
	if (T.mask_path) {
		const L0Geom G{T.lx, T.ly, T.lz, T.bx, T.by};
		if (phase == 0) {
			const size_t nchunk = (s1 - s0 + kCollectRows - 1) / kCollectRows;
			gol_amr_collect_mask_kernel<<<gate ? unsigned(std::min<size_t>(nchunk, 256)) : xcd_grid(nchunk), kCollectRows, 0,
			                              s>>>(
			    state, T.ent.p, ptr, T.l0c.p, G, lst, T.mask.p, s0, s1, list_from < s0 ? s0 : list_from, err, gate);
		} else {
			if (T.n_lvl0)
				gol_amr_spread0_mask_kernel<<<gate ? std::min(grid_for(T.n_lvl0, 256), 256u) : grid_for(T.n_lvl0, 256),
				                              256, 0, s>>>(T.lvl0.p, T.n_lvl0, state, T.mask.p, s0, s1, gate);
			if (T.ng)
				gol_amr_spread_groups_mask_kernel<<<gate ? std::min(xcd_grid((8 * T.ng + 255) / 256), 256u)
				                                         : xcd_grid((8 * T.ng + 255) / 256),
				                                    256, 0, s>>>(
				    T.gptr.p, T.ng, T.gslot.p, state, T.mask.p, lst, T.l0c.p, G, n_local, s0, s1, err, gate);
		}
		HIP_CHECK(hipGetLastError());
		return;
	}
	if (phase == 0) {
		gol_amr_pack_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(T.l0.p, state, n_slots, T.pack.p);
		HIP_CHECK(hipGetLastError());
		gol_amr_collect_kernel<<<xcd_grid((s1 - s0 + kCollectRows - 1) / kCollectRows), kCollectRows, 0, s>>>(
		    T.pack.p, lst, ptr, nslot, s0, s1, err);
	} else {
		if (T.n_lvl0)
			gol_amr_spread0_kernel<<<grid_for(T.n_lvl0, 256), 256, 0, s>>>(T.lvl0.p, T.n_lvl0, state, lst, s0, s1);
		if (T.ng)
			gol_amr_spread_groups_kernel<<<xcd_grid((T.ng + 255) / 256), 256, 0, s>>>(T.gptr.p, T.ng, T.gslot.p, state, lst, s0,
			                                                                 s1, err);
	}
	HIP_CHECK(hipGetLastError());
}

}  // namespace dccrgx
