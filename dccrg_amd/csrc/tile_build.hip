// Face tiles for the advection sweep (built once per mesh, from the face CSR
// of get_face_neighbors_of, dccrg.hpp:2806-2933).
//
// The inner and the outer run of local slots are cut into tiles of at most
// T consecutive slots (Morton order on refined grids; cuts on aligned box
// corners where possible, so a tile is a compact box of space).  A tile's sweep stages its own cells and the distinct
// cells just outside it ("ext") in LDS; every face of every cell then reads
// its neighbor from LDS through a 16-bit tile-local index.  Construction:
//   1. one key (tile << 32 | slot) per out-of-tile face entry,
//   2. radix sort + unique  -> per-tile ascending ext lists,
//   3. per-tile ext ranges by binary search,
//   4. finer faces (4 cells behind one face) numbered by a scan,
//   5. per cell: six tile-local indices (binary search in the tile's ext).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <map>
#include <cstdio>
#include <cstdlib>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

struct TileGeom {
	const uint32_t* tstart;  // ntiles + 1 tile boundaries (slots)
	uint32_t ntiles, n_local;
	// tile of row r: global tile index, first and one-past-last slot
	__device__ void of(uint32_t r, uint32_t& gt, uint32_t& ts, uint32_t& te) const {
		uint32_t lo = 0, hi = ntiles;  // last tile with tstart <= r
		while (hi - lo > 1) {
			const uint32_t mid = (lo + hi) / 2;
			if (tstart[mid] <= r) lo = mid;
			else hi = mid;
		}
		gt = lo;
		ts = tstart[lo];
		te = tstart[lo + 1];
	}
};

// alignment of each slot's min corner on the Morton curve: the number of
// trailing zero 3-bit groups of its finest-level key (a tile that starts at
// a slot with alignment k starts on the corner of a 2^k-box)
__global__ void align_kernel(MapCtx m, const uint64_t* __restrict__ ids, uint32_t n, uint8_t* __restrict__ al) {
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		uint64_t x, y, z;
		map_indices(m, ids[i], x, y, z);
		const uint64_t k = x | y | z;  // a key has 3k trailing zeros iff all three indices have k
		al[i] = uint8_t(k ? __builtin_ctzll(k) : 63);
	}
}

struct OutOfTile {
	__host__ __device__ bool operator()(const uint64_t& k) const { return k != ~0ull; }
};

__global__ void ext_keys_kernel(TileGeom tg, const uint32_t* __restrict__ ptr, const int32_t* __restrict__ ent,
                                uint64_t* __restrict__ keys) {
	for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < tg.n_local; r += gridDim.x * blockDim.x) {
		uint32_t gt, ts, te;
		tg.of(r, gt, ts, te);
		for (uint32_t e = ptr[r]; e < ptr[r + 1]; e++) {
			const uint32_t n = uint32_t(ent[e] >> 3);
			keys[e] = (n >= ts && n < te) ? ~0ull : ((uint64_t(gt) << 32) | n);
		}
	}
}

__device__ size_t lower_bound_u64(const uint64_t* a, size_t n, uint64_t v) {
	size_t lo = 0, hi = n;
	while (lo < hi) {
		const size_t mid = (lo + hi) / 2;
		if (a[mid] < v) lo = mid + 1;
		else hi = mid;
	}
	return lo;
}

__global__ void ext_ranges_kernel(const uint64_t* __restrict__ keys, size_t m, uint32_t ntiles,
                                  uint32_t* __restrict__ ext_ptr, uint32_t* __restrict__ ext) {
	const size_t i0 = blockIdx.x * size_t(blockDim.x) + threadIdx.x, step = size_t(gridDim.x) * blockDim.x;
	for (size_t i = i0; i <= ntiles; i += step) ext_ptr[i] = uint32_t(lower_bound_u64(keys, m, uint64_t(i) << 32));
	for (size_t k = i0; k < m; k += step) ext[k] = uint32_t(keys[k]);
}

// number of finer faces (a direction with 4 face neighbors) of each row
__global__ void fine_count_kernel(uint32_t n, const uint32_t* __restrict__ ptr, const int32_t* __restrict__ ent,
                                  uint32_t* __restrict__ cnt) {
	for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
		uint32_t c = 0;
		uint32_t e = ptr[r];
		const uint32_t e1 = ptr[r + 1];
		while (e < e1) {
			const int d = ent[e] & 7;
			uint32_t k = e + 1;
			while (k < e1 && (ent[k] & 7) == d) k++;
			c += (k - e) > 1;
			e = k;
		}
		cnt[r] = c;
	}
}

__global__ void fine_base_kernel(TileGeom tg, const uint32_t* __restrict__ fine_idx, uint32_t* __restrict__ fine_base) {
	for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < tg.ntiles; t += gridDim.x * blockDim.x)
		fine_base[t] = fine_idx[tg.tstart[t]];
}

__device__ uint32_t local_index(uint32_t n, uint32_t ts, uint32_t te, uint32_t T, const uint32_t* ext, uint32_t e0,
                                uint32_t e1, int* err) {
	// T = the tile capacity: ext entries follow the largest possible tile
	if (n >= ts && n < te) return n - ts;
	uint32_t lo = e0, hi = e1;
	while (lo < hi) {
		const uint32_t mid = (lo + hi) / 2;
		if (ext[mid] < n) lo = mid + 1;
		else hi = mid;
	}
	if (lo >= e1 || ext[lo] != n) {
		atomicExch(err, 1);
		return 0;
	}
	return T + (lo - e0);
}

__global__ void tile_ell_kernel(TileGeom tg, uint32_t T, const uint32_t* __restrict__ ptr, const int32_t* __restrict__ ent,
                                const uint32_t* __restrict__ ext_ptr, const uint32_t* __restrict__ ext,
                                const uint32_t* __restrict__ fine_idx, const uint32_t* __restrict__ fine_base,
                                uint32_t* __restrict__ tell, uint32_t* __restrict__ tfine, uint32_t* __restrict__ ext_ax,
                                int* err) {
	for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < tg.n_local; r += gridDim.x * blockDim.x) {
		uint32_t gt, ts, te;
		tg.of(r, gt, ts, te);
		const uint32_t e0 = ext_ptr[gt], e1 = ext_ptr[gt + 1];
		uint32_t code[6] = {0xffffu, 0xffffu, 0xffffu, 0xffffu, 0xffffu, 0xffffu};
		uint32_t fk = fine_idx[r];
		uint32_t e = ptr[r];
		const uint32_t eend = ptr[r + 1];
		while (e < eend) {
			const int d = ent[e] & 7;
			uint32_t k = e + 1;
			while (k < eend && (ent[k] & 7) == d) k++;
			// axes through which each ext cell is reached (its velocity
			// component along them is the only one a face reads)
			const uint32_t axbit = 1u << (d >> 1);
			if (k - e == 1) {
				code[d] = local_index(uint32_t(ent[e] >> 3), ts, te, T, ext, e0, e1, err);
				if (code[d] >= T) atomicOr(&ext_ax[e0 + code[d] - T], axbit);
			} else {
				uint32_t li[4];
				for (int i = 0; i < 4; i++) {
					li[i] = local_index(uint32_t(ent[e + i] >> 3), ts, te, T, ext, e0, e1, err);
					if (li[i] >= T) atomicOr(&ext_ax[e0 + li[i] - T], axbit);
				}
				tfine[2 * size_t(fk)] = li[0] | (li[1] << 16);
				tfine[2 * size_t(fk) + 1] = li[2] | (li[3] << 16);
				code[d] = 0x8000u | (fk - fine_base[gt]);
				fk++;
			}
			e = k;
		}
		// three planes of n_local + 1 words (x, y, z pairs of codes), so the
		// sweep reads each plane with one coalesced load per cell
		const size_t pl = size_t(tg.n_local) + 1;
		tell[size_t(r)] = code[0] | (code[1] << 16);
		tell[pl + size_t(r)] = code[2] | (code[3] << 16);
		tell[2 * pl + size_t(r)] = code[4] | (code[5] << 16);
	}
}


// ---------------------------------------------------------------------------
// Per-tile build (tiles of at most kXT slots), steps 1-5 without a global
// sort: one 512-thread block per tile gathers its out-of-tile face entries in
// LDS, sorts them (bitonic) and drops repeats - the tile's ascending ext list
// - and writes its cells' tile-local rows.  A tile's ext list and finer faces
// go to fixed places that need no scan: the ext list at the tile's first face
// entry (it has at most as many cells as the tile has face entries), the
// finer faces at a quarter of that (each has four entries).  A tile with more
// than kXCap out-of-tile entries sets err bit 2 (then the global build).
constexpr uint32_t kXT = 512;
constexpr uint32_t kXCap = 8192;

// exclusive scan over a 512-thread block; sh: 8 words of LDS
__device__ __forceinline__ uint32_t block_scan512(uint32_t v, uint32_t* sh, uint32_t& total) {
	const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
	uint32_t incl = v;
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t x = __shfl_up(incl, o);
		if (lane >= uint32_t(o)) incl += x;
	}
	if (lane == 63) sh[w] = incl;
	__syncthreads();
	uint32_t base = 0;
	total = 0;
	for (uint32_t k = 0; k < 8; k++) {
		const uint32_t x = sh[k];
		base += k < w ? x : 0u;
		total += x;
	}
	__syncthreads();
	return base + incl - v;
}

__global__ __launch_bounds__(512) void tile_ext_kernel(const uint32_t* __restrict__ tstart, uint32_t T,
                                                        const uint32_t* __restrict__ ptr, const int32_t* __restrict__ ent,
                                                        uint32_t* __restrict__ ext_n, uint32_t* __restrict__ fine_n,
                                                        uint32_t* __restrict__ scr_off,
                                                        uint32_t* __restrict__ ext_pk, uint32_t* __restrict__ tell,
                                                        size_t pl, uint32_t* __restrict__ tfine, int* __restrict__ err) {
	__shared__ uint32_t key[kXCap];
	__shared__ uint32_t sh[8];
	__shared__ uint32_t n_raw;
	const uint32_t t = blockIdx.x, tid = threadIdx.x;
	const uint32_t ts = tstart[t], te = tstart[t + 1];
	if (tid == 0) n_raw = 0;
	__syncthreads();
	const uint32_t r = ts + tid;
	const bool row = r < te;  // tiles hold at most kXT = blockDim.x slots
	const uint32_t e0 = row ? ptr[r] : 0u, e1 = row ? ptr[r + 1] : 0u;
	for (uint32_t e = e0; e < e1; e++) {
		const uint32_t n = uint32_t(ent[e] >> 3);
		if (n >= ts && n < te) continue;
		const uint32_t i = atomicAdd(&n_raw, 1u);
		if (i < kXCap) key[i] = n;
	}
	__syncthreads();
	const uint32_t N = n_raw;
	if (N > kXCap) {  // block-uniform
		if (tid == 0) atomicOr(err, 2);
		return;
	}
	uint32_t P = 64;
	while (P < N) P <<= 1;
	for (uint32_t i = N + tid; i < P; i += 512) key[i] = 0xffffffffu;
	// bitonic sort of key[0, P)
	for (uint32_t k = 2; k <= P; k <<= 1)
		for (uint32_t j = k >> 1; j > 0; j >>= 1) {
			__syncthreads();
			for (uint32_t i = tid; i < P; i += 512) {
				const uint32_t q = i ^ j;
				if (q > i) {
					const uint32_t x = key[i], y = key[q];
					const bool up = (i & k) == 0;
					if ((x > y) == up) {
						key[i] = y;
						key[q] = x;
					}
				}
			}
		}
	__syncthreads();
	// distinct values, compacted in place: each thread a contiguous chunk
	const uint32_t chunk = (P + 511) / 512;  // <= kXCap / 512 = 16
	uint32_t v[16];
	uint32_t nu = 0;
#pragma unroll
	for (uint32_t j = 0; j < 16; j++) {
		const uint32_t i = tid * chunk + j;
		v[j] = 0xffffffffu;
		if (j < chunk && i < N && (i == 0 || key[i] != key[i - 1])) v[j] = key[i];
		nu += v[j] != 0xffffffffu;
	}
	uint32_t U;
	const uint32_t ub = block_scan512(nu, sh, U);  // (its barriers also end the reads above)
	uint32_t o = ub;
#pragma unroll
	for (uint32_t j = 0; j < 16; j++)
		if (v[j] != 0xffffffffu) key[o++] = v[j];
	// finer faces of this thread's row, numbered in row order
	uint32_t nf = 0;
	for (uint32_t e = e0; e < e1;) {
		const int d = ent[e] & 7;
		uint32_t k = e + 1;
		while (k < e1 && (ent[k] & 7) == d) k++;
		nf += (k - e) > 1;
		e = k;
	}
	uint32_t F;
	const uint32_t fb = block_scan512(nf, sh, F);
	const uint32_t eoff = ptr[ts], foff = eoff / 4;
	if (tid == 0) {
		ext_n[t] = U;
		fine_n[t] = F;
		scr_off[t] = eoff;
	}
	// tile-local rows (tile_ell_kernel's codes); the axis bits are ORed into
	// the ext entries' top bits (slots < 2^29)
	auto local = [&](uint32_t n) -> uint32_t {
		if (n >= ts && n < te) return n - ts;
		uint32_t lo = 0, hi = U;
		while (lo < hi) {
			const uint32_t mid = (lo + hi) >> 1;
			if ((key[mid] & 0x1fffffffu) < n) lo = mid + 1;
			else hi = mid;
		}
		if (lo >= U || (key[lo] & 0x1fffffffu) != n) {
			atomicOr(err, 1);
			return 0;
		}
		return T + lo;
	};
	if (row) {
		uint32_t fk = fb;
		uint32_t code[6] = {0xffffu, 0xffffu, 0xffffu, 0xffffu, 0xffffu, 0xffffu};
		for (uint32_t e = e0; e < e1;) {
			const int d = ent[e] & 7;
			uint32_t k = e + 1;
			while (k < e1 && (ent[k] & 7) == d) k++;
			const uint32_t axbit = 1u << (29 + (d >> 1));
			if (k - e == 1) {
				code[d] = local(uint32_t(ent[e] >> 3));
				if (code[d] >= T) atomicOr(&key[code[d] - T], axbit);
			} else {
				uint32_t li[4];
				for (int i = 0; i < 4; i++) {
					li[i] = local(uint32_t(ent[e + i] >> 3));
					if (li[i] >= T) atomicOr(&key[li[i] - T], axbit);
				}
				tfine[2 * size_t(foff + fk)] = li[0] | (li[1] << 16);
				tfine[2 * size_t(foff + fk) + 1] = li[2] | (li[3] << 16);
				code[d] = 0x8000u | fk;
				fk++;
			}
			e = k;
		}
		tell[size_t(r)] = code[0] | (code[1] << 16);
		tell[pl + size_t(r)] = code[2] | (code[3] << 16);
		tell[2 * pl + size_t(r)] = code[4] | (code[5] << 16);
	}
	__syncthreads();
	for (uint32_t i = tid; i < U; i += 512) ext_pk[eoff + i] = key[i];
}

// the per-tile lists from their scratch places to dense arrays (off: per tile
// the dense ext offset, then per tile the dense finer-face offset)
__global__ void tile_compact_kernel(const uint32_t* __restrict__ ext_n, const uint32_t* __restrict__ fine_n,
                                    const uint32_t* __restrict__ scr_off, const uint32_t* __restrict__ off,
                                    uint32_t ntiles, const uint32_t* __restrict__ scr_ext,
                                    const uint32_t* __restrict__ scr_fine, uint32_t* __restrict__ ext_pk,
                                    uint32_t* __restrict__ tfine) {
	const uint32_t t = blockIdx.x;
	const uint32_t so = scr_off[t], eo = off[t], fo = off[ntiles + t], ne = ext_n[t], nf = 2 * fine_n[t];
	for (uint32_t i = threadIdx.x; i < ne; i += blockDim.x) ext_pk[eo + i] = scr_ext[so + i];
	for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) tfine[2 * size_t(fo) + i] = scr_fine[2 * size_t(so / 4) + i];
}

// ---------------------------------------------------------------------------
// Regular tiles: a tile of exactly 512 slots that is an aligned 8x8x8 box of
// cells of one level whose face neighbors on each of its six sides are,
// all of them, either absent (non-periodic boundary) or the same-level
// cells of one neighbor box stored Morton-consecutively from a single slot.
// Such a tile's sweep needs no per-cell face rows: neighbors are found by
// Morton arithmetic from the tile's start slot and the six neighbor-box
// starts.  One 512-thread block per tile; thread t = local Morton index t.
__device__ __forceinline__ uint32_t morton9(uint32_t x, uint32_t y, uint32_t z) {
	uint32_t m = 0;
	for (int b = 0; b < 3; b++) m |= (((x >> b) & 1u) << (3 * b)) | (((y >> b) & 1u) << (3 * b + 1)) | (((z >> b) & 1u) << (3 * b + 2));
	return m;
}

__global__ __launch_bounds__(512) void classify_tiles_kernel(MapCtx m, const uint32_t* __restrict__ tstart,
                                                              const uint64_t* __restrict__ slot_ids,
                                                              const int32_t* __restrict__ face_ell,
                                                              uint32_t* __restrict__ treg, int32_t* __restrict__ tnb) {
	__shared__ int ok;
	__shared__ int32_t nst[6];
	__shared__ int has_nb[6], no_nb[6];
	__shared__ uint64_t corner[4];
	const uint32_t gt = blockIdx.x, tid = threadIdx.x;
	const uint32_t ts = tstart[gt], te = tstart[gt + 1];
	if (tid == 0) {
		ok = (te - ts == 512u);
		for (int d = 0; d < 6; d++) {
			nst[d] = -1;
			has_nb[d] = 0;
			no_nb[d] = 0;
		}
	}
	__syncthreads();
	if (!ok) {
		if (tid == 0) treg[gt] = 0x10u;  // reason: not 512 slots
		return;
	}
	const uint32_t s = ts + tid;
	uint64_t x, y, z;
	const int lvl = map_indices(m, slot_ids[s], x, y, z);
	if (tid == 0) {
		corner[0] = x;
		corner[1] = y;
		corner[2] = z;
		corner[3] = uint64_t(lvl);
	}
	__syncthreads();
	const uint64_t len = uint64_t(1) << (m.R - lvl);
	bool good = lvl >= 0 && uint64_t(lvl) == corner[3];
	uint32_t l[3] = {0, 0, 0};
	if (good) {
		const uint64_t c[3] = {x, y, z};
		for (int d = 0; d < 3; d++) {
			if (corner[d] % (8 * len) != 0 || c[d] < corner[d]) good = false;
			const uint64_t r = (c[d] - corner[d]) / len;
			if (r > 7 || (c[d] - corner[d]) % len) good = false;
			l[d] = uint32_t(r & 7u);
		}
		if (good && morton9(l[0], l[1], l[2]) != tid) good = false;
	}
	const bool box_good = good;
	if (good) {
		for (int d = 0; d < 6; d++) {
			const int a = d >> 1;
			const bool plus = d & 1;
			const int32_t e = face_ell[6 * size_t(s) + d];
			const bool boundary = plus ? l[a] == 7 : l[a] == 0;
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] = boundary ? (plus ? 0u : 7u) : (plus ? q[a] + 1 : q[a] - 1);
			const uint32_t mq = morton9(q[0], q[1], q[2]);
			if (!boundary) {
				if (e != int32_t(ts + mq)) good = false;
				continue;
			}
			if (e == -1) {
				atomicOr(&no_nb[d], 1);
				continue;
			}
			if (e < -1) {
				good = false;
				continue;
			}
			if (map_level(m, slot_ids[e]) != lvl || uint32_t(e) < mq) {
				good = false;
				continue;
			}
			const int32_t st = e - int32_t(mq);
			atomicOr(&has_nb[d], 1);
			atomicMax(&nst[d], st);  // all must agree: checked below
		}
	}
	__shared__ int box_ok;
	if (tid == 0) box_ok = 1;
	__syncthreads();
	if (!box_good) atomicAnd(&box_ok, 0);
	if (!good) atomicAnd(&ok, 0);
	__syncthreads();
	// second pass: every boundary neighbor consistent with the agreed start
	if (ok) {
		for (int d = 0; d < 6; d++) {
			const int a = d >> 1;
			const bool plus = d & 1;
			const bool boundary = plus ? l[a] == 7 : l[a] == 0;
			if (!boundary) continue;
			if (has_nb[d] && no_nb[d]) good = false;
			const int32_t e = face_ell[6 * size_t(s) + d];
			if (e == -1) continue;
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] = plus ? 0u : 7u;
			if (e != nst[d] + int32_t(morton9(q[0], q[1], q[2]))) good = false;
		}
		if (!good) atomicAnd(&ok, 0);
	}
	__syncthreads();
	if (tid == 0) {
		treg[gt] = ok ? 1u : (box_ok ? 0x30u : 0x20u);  // reasons: 0x20 not a uniform box, 0x30 irregular side
		for (int d = 0; d < 6; d++) tnb[6 * size_t(gt) + d] = (ok && has_nb[d]) ? nst[d] : -1;
	}
}

}  // namespace

// Tile boundaries of one run [r0, r1): greedy, each tile ends at the
// best-aligned slot among the last three quarters of its allowed length
// (the latest one on ties), so that on
// Morton-ordered slots tiles coincide with aligned boxes wherever the mesh
// allows (fewer distinct out-of-tile neighbors than arbitrary cuts).
// (a lower bound of T/8 or 3T/4 gives fewer general tiles but more of them
// irregular and a slower sweep, r01l)
static uint32_t tile_lo(uint32_t T) { return std::max<uint32_t>(1u, T / 4u); }

static void cut_run(const std::vector<uint8_t>& al, uint32_t r0, uint32_t r1, uint32_t T, std::vector<uint32_t>& out) {
	uint32_t a = r0;
	const uint32_t lo = tile_lo(T);
	while (a < r1) {
		out.push_back(a);
		if (r1 - a <= T) break;
		uint32_t best = a + T;
		int best_al = -1;
		for (uint32_t b = a + T; b >= a + lo && b > a; b--) {
			const int v = al.empty() ? 0 : int(al[b]);
			if (v > best_al) {
				best_al = v;
				best = b;
			}
		}
		a = best;
	}
}

// The greedy cut of cut_run on the device.  next[a] = the start of the tile
// after one starting at slot a of its run [r0, r1): r1 when the rest fits one
// tile, else the best-aligned slot in [a + lo, a + T], the latest on ties -
// for every slot at once (one block per 256 slots, their windows staged in
// LDS).  The tile starts are then the chain 0, next[0], next[next[0]], ...
// (through the inner run's end into the outer run), listed by pointer
// jumping: next^64 by six doublings, the anchors next^(64 i)(0) walked by one
// thread, each anchor's 64 successors by one thread each.
constexpr uint32_t kCutBlock = 256;
constexpr uint32_t kCutMaxT = 4096;

__global__ __launch_bounds__(kCutBlock) void cut_next_kernel(const uint8_t* __restrict__ al, uint32_t r0, uint32_t r1,
                                                              uint32_t T, uint32_t lo, uint32_t* __restrict__ next) {
	// window maxima by doubling (a sparse table level by level): key of LDS
	// position p = alignment << 16 | p, so the max is the best alignment at
	// its latest position, and the window [lo, T] of every slot is the max of
	// two overlapping power-of-two spans
	__shared__ uint32_t kb[2][kCutBlock + kCutMaxT + 1];
	const uint32_t a0 = r0 + blockIdx.x * kCutBlock;
	if (a0 >= r1) return;  // block-uniform
	const uint32_t span = kCutBlock + T + 1;
	for (uint32_t i = threadIdx.x; i < span; i += kCutBlock) kb[0][i] = ((a0 + i < r1 ? uint32_t(al[a0 + i]) : 0u) << 16) | i;
	const uint32_t len = T - lo + 1;  // window length
	int lv = 0;
	while ((2u << lv) <= len) lv++;  // 2^lv <= len < 2^(lv+1)
	int cur = 0;
	for (int k = 0; k < lv; k++) {
		__syncthreads();
		const uint32_t h = 1u << k;
		for (uint32_t i = threadIdx.x; i < span; i += kCutBlock) {
			const uint32_t x = kb[cur][i];
			kb[cur ^ 1][i] = i + h < span ? max(x, kb[cur][i + h]) : x;
		}
		cur ^= 1;
	}
	__syncthreads();
	const uint32_t a = a0 + threadIdx.x;
	if (a >= r1) return;
	if (r1 - a <= T) {
		next[a] = r1;
		return;
	}
	const uint32_t best = max(kb[cur][threadIdx.x + lo], kb[cur][threadIdx.x + T + 1 - (1u << lv)]);
	next[a] = a0 + (best & 0xffffu);
}

__global__ void jump_double_kernel(const uint32_t* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = in[in[i]];
}

// one thread: the anchors 0, J64[0], ... up to the terminal n
__global__ void chain_anchors_kernel(const uint32_t* __restrict__ j64, uint32_t n, uint32_t* __restrict__ anchors,
                                     uint32_t cap, uint32_t* __restrict__ count) {
	if (blockIdx.x != 0 || threadIdx.x != 0) return;
	uint32_t a = 0, k = 0;
	while (k < cap) {
		anchors[k++] = a;
		if (a >= n) break;
		a = j64[a];
	}
	*count = k;
}

// anchor i expands into starts[64 i .. 64 i + 63]; n marks the end
__global__ void chain_expand_kernel(const uint32_t* __restrict__ next, const uint32_t* __restrict__ anchors,
                                    const uint32_t* __restrict__ count, uint32_t n, uint32_t* __restrict__ starts) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= *count) return;
	uint32_t a = anchors[i];
	for (uint32_t j = 0; j < 64; j++) {
		starts[size_t(i) * 64 + j] = a;
		if (a >= n) break;
		a = next[a];
	}
}

__global__ void pack_ext_kernel(const uint32_t* __restrict__ ext, const uint32_t* __restrict__ ax, size_t m,
                                uint32_t* __restrict__ out) {
	for (size_t k = blockIdx.x * size_t(blockDim.x) + threadIdx.x; k < m; k += size_t(gridDim.x) * blockDim.x)
		out[k] = ext[k] | (ax[k] << 29);
}

// cut_run over both runs on the device (see cut_next_kernel): the tile starts
// of [0, n_inner) then [n_inner, n_local) into tstart (+ the end n_local);
// returns the tile count, n_tiles_inner the inner run's
static size_t device_cut(const DBuf<uint8_t>& al, size_t n_inner, size_t n_local, uint32_t T, DBuf<uint32_t>& tstart,
                         size_t& n_tiles_inner, hipStream_t s) {
	DX_REQUIRE(T <= kCutMaxT, "tile size out of range for the device cut");
	const uint32_t n = uint32_t(n_local), lo = tile_lo(T);
	DBuf<uint32_t> next, ja, jb;
	next.alloc(size_t(n) + 1);
	const uint32_t runs[3] = {0u, uint32_t(n_inner), n};
	for (int r = 0; r < 2; r++) {
		const uint32_t r0 = runs[r], r1 = runs[r + 1];
		if (r1 > r0)
			cut_next_kernel<<<(r1 - r0 + kCutBlock - 1) / kCutBlock, kCutBlock, 0, s>>>(al.p, r0, r1, T, lo, next.p);
	}
	HIP_CHECK(hipGetLastError());
	HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(next.p + n), int(n), 1, s));  // terminal: next[n] = n
	// J64 = next^64
	ja.alloc(size_t(n) + 1);
	jb.alloc(size_t(n) + 1);
	const uint32_t* src = next.p;
	DBuf<uint32_t>* dst = &ja;
	for (int k = 0; k < 6; k++) {
		jump_double_kernel<<<grid_for(size_t(n) + 1, 256), 256, 0, s>>>(src, size_t(n) + 1, dst->p);
		HIP_CHECK(hipGetLastError());
		src = dst->p;
		dst = dst == &ja ? &jb : &ja;
	}
	// every tile but a run's last has at least lo slots: at most n / lo + 2
	// starts, + the terminal
	const uint32_t cap_anchor = uint32_t((size_t(n) / lo + 4) / 64 + 4);
	DBuf<uint32_t> anchors, cnt, starts;
	anchors.alloc(cap_anchor);
	cnt.alloc(1);
	chain_anchors_kernel<<<1, 64, 0, s>>>(src, n, anchors.p, cap_anchor, cnt.p);
	HIP_CHECK(hipGetLastError());
	starts.alloc(size_t(cap_anchor) * 64);
	HIP_CHECK(hipMemsetAsync(starts.p, 0xff, starts.n * 4, s));
	chain_expand_kernel<<<(cap_anchor + 63) / 64, 64, 0, s>>>(next.p, anchors.p, cnt.p, n, starts.p);
	HIP_CHECK(hipGetLastError());
	uint32_t na = 0;
	d2h_small(&na, cnt.p, 4, s);
	DX_REQUIRE(na >= 1 && na < cap_anchor, "internal error: tile chain longer than its bound");
	// the starts before the terminal: the sequence is increasing, so the
	// count of each run is a count of values below its end
	const std::vector<uint32_t> h = download(starts.p, size_t(na) * 64, s);
	size_t ntiles = 0, ni = 0;
	while (ntiles < h.size() && h[ntiles] < n) {
		ni += h[ntiles] < n_inner;
		ntiles++;
	}
	n_tiles_inner = ni;
	tstart.alloc(ntiles + 1);
	if (ntiles) HIP_CHECK(hipMemcpyAsync(tstart.p, starts.p, ntiles * 4, hipMemcpyDeviceToDevice, s));
	HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(tstart.p + ntiles), int(n), 1, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return ntiles;
}

TileBuild k_build_tiles(const uint32_t* face_ptr, const int32_t* face_ent, const uint64_t* slot_ids, const MapCtx& mc,
                        bool morton, size_t n_inner, size_t n_local, int tile, DBuf<uint32_t>& tstart,
                        DBuf<uint32_t>& tell, DBuf<uint32_t>& ext_ptr, DBuf<uint32_t>& ext, DBuf<uint32_t>& ext_pk,
                        DBuf<uint32_t>& fine_base, DBuf<uint32_t>& tfine, hipStream_t s) {
	DX_REQUIRE(tile > 0 && tile <= 4096, "tile size out of range");
	DX_REQUIRE(n_local < (size_t(1) << 29), "too many local cells for 29-bit tile slots");
	TileBuild out{};
	const uint32_t T = uint32_t(tile);
	DX_LAPS(s);
	DBuf<uint8_t> dal;
	if (morton && n_local) {
		dal.alloc(n_local);
		align_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(mc, slot_ids, uint32_t(n_local), dal.p);
		HIP_CHECK(hipGetLastError());
	}
	DX_LAP("tb.1_align");
	size_t ntiles = 0;
	if (morton && n_local) {
		ntiles = device_cut(dal, n_inner, n_local, T, tstart, out.n_tiles_inner, s);
		out.n_tiles_outer = ntiles - out.n_tiles_inner;
	} else {
		std::vector<uint32_t> hts;
		cut_run({}, 0, uint32_t(n_inner), T, hts);
		out.n_tiles_inner = hts.size();
		cut_run({}, uint32_t(n_inner), uint32_t(n_local), T, hts);
		out.n_tiles_outer = hts.size() - out.n_tiles_inner;
		ntiles = hts.size();
		hts.push_back(uint32_t(n_local));
		upload(tstart, hts, s);
	}
	TileGeom tg{tstart.p, uint32_t(ntiles), uint32_t(n_local)};
	DX_LAP("tb.2_cut");
	tell.alloc(3 * n_local + 3);
	ext_ptr.alloc(ntiles + 1);
	fine_base.alloc(ntiles + 1);
	if (n_local == 0) {
		HIP_CHECK(hipMemsetAsync(ext_ptr.p, 0, 4, s));
		HIP_CHECK(hipStreamSynchronize(s));
		ext.alloc(1);
		ext_pk.alloc(1);
		tfine.alloc(2);
		return out;
	}
	uint32_t n_ent = 0;
	d2h_small(&n_ent, face_ptr + n_local, 4, s);
	// (DCCRGX_TILE_GLOBAL=1: always the global build below, the fallback,
	// so that tests compare the two)
	if (T <= kXT && ntiles && !std::getenv("DCCRGX_TILE_GLOBAL")) {
		// per-tile build (tile_ext_kernel): each tile's lists at scratch places
		// first, then packed densely
		DBuf<uint32_t> en, fn, so, off, sext, sfine;
		DBuf<int> err;
		en.alloc(ntiles + 1);
		fn.alloc(ntiles + 1);
		so.alloc(ntiles + 1);
		err.alloc(1);
		HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
		sext.alloc(size_t(n_ent) + 1);
		sfine.alloc(2 * (size_t(n_ent) / 4 + 2));
		tile_ext_kernel<<<unsigned(ntiles), 512, 0, s>>>(tstart.p, T, face_ptr, face_ent, en.p, fn.p, so.p, sext.p, tell.p,
		                                                 n_local + 1, sfine.p, err.p);
		HIP_CHECK(hipGetLastError());
		int herr = 0;
		HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
		out.ext_n = download(en.p, ntiles, s);
		out.fine_n = download(fn.p, ntiles, s);
		if (herr == 0) {
			std::vector<uint32_t> ho(2 * ntiles);
			out.ext_off.resize(ntiles);
			out.fine_off.resize(ntiles);
			for (size_t t = 0; t < ntiles; t++) {
				out.ext_off[t] = ho[t] = uint32_t(out.total_ext);
				out.fine_off[t] = ho[ntiles + t] = uint32_t(out.n_fine);
				out.total_ext += out.ext_n[t];
				out.n_fine += out.fine_n[t];
				out.max_ext = std::max<size_t>(out.max_ext, out.ext_n[t]);
			}
			DX_REQUIRE(size_t(T) + out.max_ext < 0x8000u, "tile too large for 16-bit local indices");
			upload(off, ho, s);
			ext_pk.alloc(out.total_ext + 1);
			tfine.alloc(2 * out.n_fine + 2);
			tile_compact_kernel<<<unsigned(ntiles), 256, 0, s>>>(en.p, fn.p, so.p, off.p, uint32_t(ntiles), sext.p, sfine.p,
			                                                    ext_pk.p, tfine.p);
			HIP_CHECK(hipGetLastError());
			HIP_CHECK(hipStreamSynchronize(s));
			ext.alloc(1);
			DX_LAP("tb.3_ext_rows");
			return out;
		}
		DX_REQUIRE((herr & 2) != 0, "internal error: face neighbor missing from its tile's external list");
		// a tile beyond kXCap out-of-tile entries: the global build
	}
	// 1-3: per-tile distinct external neighbors: the out-of-tile entries'
	// keys compacted first (about an eighth of the face entries on config 3),
	// then sorted on the bits a (tile, slot) key uses
	DBuf<uint64_t> all, keys;
	all.alloc(size_t(n_ent) + 1);
	ext_keys_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(tg, face_ptr, face_ent, all.p);
	HIP_CHECK(hipGetLastError());
	keys.alloc(size_t(n_ent) + 1);
	size_t m0 = 0;
	{
		DBuf<unsigned long long> nsel;
		nsel.alloc(1);
		size_t bytes = 0;
		HIP_CHECK(hipcub::DeviceSelect::If(nullptr, bytes, all.p, keys.p, nsel.p, size_t(n_ent), OutOfTile(), s));
		DBuf<uint8_t> temp;
		temp.alloc(bytes + 1);
		HIP_CHECK(hipcub::DeviceSelect::If(temp.p, bytes, all.p, keys.p, nsel.p, size_t(n_ent), OutOfTile(), s));
		unsigned long long h = 0;
		d2h_small(&h, nsel.p, sizeof(h), s);
		m0 = size_t(h);
	}
	all.release();
	DX_LAP("tb.3_ext_keys_select");
	int end_bit = 32;
	while (end_bit < 64 && (uint64_t(ntiles) >> (end_bit - 32)) != 0) end_bit++;
	const size_t m = sort_unique_u64(keys.p, m0, s, end_bit);
	ext.alloc(m + 1);
	ext_ranges_kernel<<<grid_for(std::max(m, ntiles + 1), 256), 256, 0, s>>>(keys.p, m, uint32_t(ntiles), ext_ptr.p,
	                                                                         ext.p);
	HIP_CHECK(hipGetLastError());
	std::vector<uint32_t> hptr = download(ext_ptr.p, ntiles + 1, s);
	out.total_ext = m;
	for (size_t t = 0; t < ntiles; t++) out.max_ext = std::max<size_t>(out.max_ext, hptr[t + 1] - hptr[t]);
	DX_REQUIRE(size_t(T) + out.max_ext < 0x8000u, "tile too large for 16-bit local indices");
	DX_LAP("tb.4_sort_ranges");

	// 4: finer faces
	DBuf<uint32_t> cnt, fine_idx;
	cnt.alloc(n_local + 1);
	fine_idx.alloc(n_local + 1);
	fine_count_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(uint32_t(n_local), face_ptr, face_ent, cnt.p);
	HIP_CHECK(hipGetLastError());
	out.n_fine = scan_exclusive_u32(cnt.p, fine_idx.p, n_local, s);
	tfine.alloc(2 * out.n_fine + 2);
	fine_base_kernel<<<grid_for(ntiles, 256), 256, 0, s>>>(tg, fine_idx.p, fine_base.p);
	HIP_CHECK(hipGetLastError());

	DX_LAP("tb.5_fine");
	// 5: tile-local rows
	DBuf<int> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	DBuf<uint32_t> ext_ax;
	ext_ax.alloc(m + 1);
	HIP_CHECK(hipMemsetAsync(ext_ax.p, 0, (m + 1) * 4, s));
	tile_ell_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(tg, T, face_ptr, face_ent, ext_ptr.p, ext.p, fine_idx.p,
	                                                       fine_base.p, tell.p, tfine.p, ext_ax.p, err.p);
	HIP_CHECK(hipGetLastError());
	// ext slots with their axis mask in bits 29..31 (slots < 2^29)
	ext_pk.alloc(m + 1);
	pack_ext_kernel<<<grid_for(m, 256), 256, 0, s>>>(ext.p, ext_ax.p, m, ext_pk.p);
	HIP_CHECK(hipGetLastError());
	int herr = 0;
	d2h_small(&herr, err.p, 4, s);
	DX_REQUIRE(herr == 0, "internal error: face neighbor missing from its tile's external list");
	{
		const std::vector<uint32_t> fbh = download(fine_base.p, ntiles, s);
		out.ext_off.assign(hptr.begin(), hptr.begin() + ntiles);
		out.ext_n.resize(ntiles);
		out.fine_off = fbh;
		out.fine_n.resize(ntiles);
		for (size_t t = 0; t < ntiles; t++) {
			out.ext_n[t] = hptr[t + 1] - hptr[t];
			out.fine_n[t] = uint32_t((t + 1 < ntiles ? fbh[t + 1] : out.n_fine) - fbh[t]);
		}
	}
	DX_LAP("tb.6_tile_rows");
	return out;
}

// Regular / irregular split of the tiles of one layout (see
// classify_tiles_kernel): per-run lists of tile indices, and for regular
// tiles the six neighbor-box start slots.
__global__ void tile_first_ids_kernel(const uint32_t* __restrict__ tstart, const uint64_t* __restrict__ slot_ids,
                                      uint64_t* __restrict__ out, size_t nt) {
	const size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
	if (t < nt) out[t] = slot_ids[tstart[t]];
}

// 3-D Hilbert index of (x, y, z), b bits per axis (Skilling's transpose
// form, "Programming the Hilbert curve", AIP Conf. Proc. 707, 2004)
static uint64_t hilbert3(uint32_t x, uint32_t y, uint32_t z, int b) {
	uint32_t X[3] = {x, y, z};
	const uint32_t M = 1u << (b - 1);
	for (uint32_t Q = M; Q > 1; Q >>= 1) {
		const uint32_t P = Q - 1;
		for (int i = 0; i < 3; i++) {
			if (X[i] & Q) {
				X[0] ^= P;
			} else {
				const uint32_t t = (X[0] ^ X[i]) & P;
				X[0] ^= t;
				X[i] ^= t;
			}
		}
	}
	for (int i = 1; i < 3; i++) X[i] ^= X[i - 1];
	uint32_t t = 0;
	for (uint32_t Q = M; Q > 1; Q >>= 1)
		if (X[2] & Q) t ^= Q - 1;
	for (int i = 0; i < 3; i++) X[i] ^= t;
	uint64_t h = 0;
	for (int j = b - 1; j >= 0; j--)
		for (int i = 0; i < 3; i++) h = (h << 1) | ((X[i] >> j) & 1u);
	return h;
}

void k_classify_tiles(const MapCtx& m, const uint32_t* tstart, size_t n_tiles_inner, size_t n_tiles_outer,
                      const uint64_t* slot_ids, const int32_t* face_ell, DBuf<uint32_t>& lists, DBuf<int32_t>& tnb,
                      DBuf<RegTileMeta>& regmeta, size_t counts[4], hipStream_t s) {
	const size_t nt = n_tiles_inner + n_tiles_outer;
	tnb.alloc(6 * nt + 6);
	for (int k = 0; k < 4; k++) counts[k] = 0;
	lists.alloc(nt + 1);
	if (!nt) return;
	DBuf<uint32_t> treg;
	treg.alloc(nt);
	classify_tiles_kernel<<<unsigned(nt), 512, 0, s>>>(m, tstart, slot_ids, face_ell, treg.p, tnb.p);
	HIP_CHECK(hipGetLastError());
	const std::vector<uint32_t> h = download(treg.p, nt, s);
	if (std::getenv("DCCRGX_TILE_REASONS")) {  // diagnostics: why tiles are not regular
		std::map<uint32_t, size_t> hist;
		for (uint32_t v : h) hist[v]++;
		for (auto& kv : hist) std::fprintf(stderr, "[tiles] reason 0x%x: %zu tiles\n", kv.first, kv.second);
	}
	// layout: [regular inner | regular outer | irregular inner | irregular outer]
	std::vector<uint32_t> reg[2], irr[2];
	for (size_t t = 0; t < nt; t++) {
		const int run = t < n_tiles_inner ? 0 : 1;
		(h[t] == 1u ? reg[run] : irr[run]).push_back(uint32_t(t));
	}
	// experiment (DCCRGX_TILE_HILBERT=1): the regular tiles of each run in the
	// Hilbert order of their boxes' corners instead of Morton (slot) order;
	// the sweep is independent of the order (bitwise the same densities)
	// (=2: the irregular tiles too)
	const int hilbert = std::getenv("DCCRGX_TILE_HILBERT") ? std::atoi(std::getenv("DCCRGX_TILE_HILBERT")) : 0;
	if (hilbert > 0) {
		DBuf<uint64_t> fid;
		fid.alloc(nt);
		tile_first_ids_kernel<<<unsigned((nt + 255) / 256), 256, 0, s>>>(tstart, slot_ids, fid.p, nt);
		HIP_CHECK(hipGetLastError());
		const std::vector<uint64_t> ids = download(fid.p, nt, s);
		uint64_t gmax = std::max(m.glen[0], std::max(m.glen[1], m.glen[2])) >> 3;
		int b = 1;
		while (b < 21 && (uint64_t(1) << b) < gmax) b++;
		for (int k = 0; k < (hilbert > 1 ? 4 : 2); k++) {
			std::vector<uint32_t>& L = k < 2 ? reg[k] : irr[k - 2];
			std::vector<std::pair<uint64_t, uint32_t>> key;
			key.reserve(L.size());
			for (uint32_t t : L) {
				uint64_t x, y, z;
				map_indices(m, ids[t], x, y, z);
				key.push_back({hilbert3(uint32_t(x >> 3), uint32_t(y >> 3), uint32_t(z >> 3), b), t});
			}
			std::stable_sort(key.begin(), key.end(),
			                 [](const auto& a, const auto& c) { return a.first < c.first; });
			for (size_t i = 0; i < key.size(); i++) L[i] = key[i].second;
		}
	}
	std::vector<uint32_t> all;
	for (auto* v : {&reg[0], &reg[1], &irr[0], &irr[1]}) all.insert(all.end(), v->begin(), v->end());
	counts[0] = reg[0].size();
	counts[1] = reg[1].size();
	counts[2] = irr[0].size();
	counts[3] = irr[1].size();
	h2d(lists.p, all.data(), all.size() * 4, s);
	// per regular tile, in list order: start slot + neighbor-box starts
	const std::vector<uint32_t> hts = download(tstart, nt + 1, s);
	const std::vector<int32_t> hnb = download(tnb.p, 6 * nt, s);
	std::vector<RegTileMeta> meta;
	for (int run = 0; run < 2; run++)
		for (uint32_t t : reg[run]) {
			RegTileMeta r{};
			r.ts = hts[t];
			for (int d = 0; d < 6; d++) r.nst[d] = hnb[6 * size_t(t) + d];
			meta.push_back(r);
		}
	regmeta.alloc(meta.size() + 1);
	if (!meta.empty())
		h2d(regmeta.p, meta.data(), meta.size() * sizeof(RegTileMeta), s);
	HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace dccrgx
