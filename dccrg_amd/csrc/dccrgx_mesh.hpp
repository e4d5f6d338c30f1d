// What one rank knows about the leaf cells of the grid.
//
// The reference keeps `cell_process` (dccrg.hpp:7197), an id -> rank map of
// EVERY leaf of the grid, on every rank, and builds neighbor lists for every
// leaf everywhere (initialize_neighbors 8240-8289) - O(N_global) time and
// memory per rank.  Here a rank knows only
//   - its own leaves, and
//   - the "ghost" leaves under every level-0 cell within max(hood length, 1)
//     level-0 cells of the level-0 parent of one of its own leaves.
// Every neighbors_of / neighbors_to / face-neighbor probe made for a local
// cell (and every probe of the refinement closure) lands inside that region
// (DESIGN.md §4), so the local structures are exactly the reference's.
//
// Two representations:
//   implicit - the initial level-0 grid with the level-0 block partition
//              (create_level_0_cells 7967-8102): existence and owner are a
//              formula; the hash holds only the cells that have a slot;
//   explicit - every known leaf is a key of the hash table.
// The hash is open addressing with linear probing over 16-byte entries
// (one dwordx4 load per probe), Fibonacci hashing of the 64-bit id, load
// factor <= 1/2.  Key 0 (= error_cell) marks an empty entry.
#pragma once

#include "dccrgx_mapping.hpp"

namespace dccrgx {

struct alignas(16) HashEntry {
	uint64_t key;
	int32_t owner;  // rank owning the leaf (explicit meshes)
	int32_t slot;   // local slot or -1
};

constexpr uint64_t kHashMul = 0x9E3779B97F4A7C15ull;

// level-0 block partition (create_level_0_cells, dccrg.hpp:7981-8013):
// cells_per_process = ceil(N0 / P), the first P * cpp - N0 ranks get one
// cell less
struct BlockPart {
	uint64_t n0 = 0, P = 1, cpp = 0, fewer = 0, K = 0;
	DX_HD void init(uint64_t total, uint64_t procs) {
		n0 = total;
		P = procs;
		cpp = total < procs ? 1 : (total % procs ? total / procs + 1 : total / procs);
		fewer = cpp * procs - total;
		K = fewer * (cpp - 1);
	}
	// owner of level-0 id (1-based, <= n0)
	DX_HD int32_t owner(uint64_t id) const {
		const uint64_t k = id - 1;
		return int32_t(k < K ? k / (cpp - 1) : fewer + (k - K) / cpp);
	}
	DX_HD void range(uint64_t p, uint64_t& first, uint64_t& count) const {
		if (p < fewer) {
			first = 1 + p * (cpp - 1);
			count = cpp - 1;
		} else {
			first = 1 + fewer * (cpp - 1) + (p - fewer) * cpp;
			count = cpp;
		}
	}
};

// Range map: an explicit mesh whose known ids span few ids per refinement
// level (one process, or z-slab partitions: the known leaves of level L lie
// in [rlo[L], rhi[L]) and that range is not much larger than the known set)
// keeps one 8-byte entry {owner, slot} per id of those ranges instead of the
// hash table: no probing, no atomics to build (every id is written by one
// thread), one load per lookup.  Absent = {-1, -1}.
constexpr int kRangeLevels = 8;

// one level's id range [lo, hi) and its first entry in the map
struct RangeLevel {
	uint64_t lo, hi, off;
};

struct DevMesh {
	const HashEntry* tab;  // nullptr: no table
	uint64_t mask;
	uint32_t shift;
	int implicit;
	BlockPart bp;
	uint64_t last;
	const int2* rmap;       // non-null: the range map replaces the table
	// the rlev ranges, by value: a kernel reads them at lane-uniform indices
	// from its arguments (scalar loads, no dependent global load per probe)
	RangeLevel rl[kRangeLevels];
	int rlev;
};

DX_HD uint64_t hash_home(uint64_t id, uint32_t shift) { return (id * kHashMul) >> shift; }

#if defined(__HIPCC__)
// index of `id` in the range map, -1 outside its ranges
__device__ __forceinline__ int64_t dm_range_index(const DevMesh& M, uint64_t id) {
#pragma unroll
	for (int L = 0; L < kRangeLevels; L++) {
		if (L >= M.rlev) break;
		const RangeLevel q = M.rl[L];
		if (id >= q.lo && id < q.hi) return int64_t(q.off + (id - q.lo));
	}
	return -1;
}

// one probe sequence; returns true and the entry's owner / slot if present
__device__ __forceinline__ bool dm_lookup(const DevMesh& M, uint64_t id, int32_t& owner, int32_t& slot) {
	if (M.rmap) {
		const int64_t k = dm_range_index(M, id);
		if (k < 0) return false;
		const int2 e = M.rmap[k];
		if (e.x < 0) return false;
		owner = e.x;
		slot = e.y;
		return true;
	}
	if (!M.tab) return false;
	uint64_t h = hash_home(id, M.shift);
	for (;;) {
		const uint4 v = *reinterpret_cast<const uint4*>(M.tab + h);
		const uint64_t k = uint64_t(v.x) | (uint64_t(v.y) << 32);
		if (k == id) {
			owner = int32_t(v.z);
			slot = int32_t(v.w);
			return true;
		}
		if (k == 0) return false;
		h = (h + 1) & M.mask;
	}
}

// rank owning leaf `id`, -1 if `id` is not a known leaf
__device__ __forceinline__ int32_t dm_owner(const DevMesh& M, uint64_t id) {
	if (id == 0 || id > M.last) return -1;
	if (M.implicit) return id <= M.bp.n0 ? M.bp.owner(id) : -1;
	int32_t o, s;
	return dm_lookup(M, id, o, s) ? o : -1;
}

// local / halo slot of `id`, -1 if none
__device__ __forceinline__ int32_t dm_slot(const DevMesh& M, uint64_t id) {
	if (id == 0 || id > M.last) return -1;
	int32_t o, s;
	return dm_lookup(M, id, o, s) ? s : -1;
}

struct DevExists {
	DevMesh M;
	__device__ __forceinline__ bool operator()(uint64_t id) const { return dm_owner(M, id) >= 0; }
};
#endif

}  // namespace dccrgx
