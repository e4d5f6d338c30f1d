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

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

inline unsigned grid_for(size_t n, unsigned per_block, unsigned cap = 256u * 32u) {
	size_t g = (n + per_block - 1) / per_block;
	if (g > cap) g = cap;
	if (g == 0) g = 1;
	return unsigned(g);
}

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
                                uint32_t* __restrict__ tell, uint32_t* __restrict__ tfine, int* err) {
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
			if (k - e == 1) {
				code[d] = local_index(uint32_t(ent[e] >> 3), ts, te, T, ext, e0, e1, err);
			} else {
				uint32_t li[4];
				for (int i = 0; i < 4; i++) li[i] = local_index(uint32_t(ent[e + i] >> 3), ts, te, T, ext, e0, e1, err);
				tfine[2 * size_t(fk)] = li[0] | (li[1] << 16);
				tfine[2 * size_t(fk) + 1] = li[2] | (li[3] << 16);
				code[d] = 0x8000u | (fk - fine_base[gt]);
				fk++;
			}
			e = k;
		}
		tell[3 * size_t(r)] = code[0] | (code[1] << 16);
		tell[3 * size_t(r) + 1] = code[2] | (code[3] << 16);
		tell[3 * size_t(r) + 2] = code[4] | (code[5] << 16);
	}
}

}  // namespace

// Tile boundaries of one run [r0, r1): greedy, each tile ends at the
// best-aligned slot among the last three quarters of its allowed length
// (the latest one on ties), so that on
// Morton-ordered slots tiles coincide with aligned boxes wherever the mesh
// allows (fewer distinct out-of-tile neighbors than arbitrary cuts).
static void cut_run(const std::vector<uint8_t>& al, uint32_t r0, uint32_t r1, uint32_t T, std::vector<uint32_t>& out) {
	uint32_t a = r0;
	while (a < r1) {
		out.push_back(a);
		if (r1 - a <= T) break;
		uint32_t best = a + T;
		int best_al = -1;
		for (uint32_t b = a + T; b >= a + T / 4 && b > a; b--) {
			const int v = al.empty() ? 0 : int(al[b]);
			if (v > best_al) {
				best_al = v;
				best = b;
			}
		}
		a = best;
	}
}

TileBuild k_build_tiles(const uint32_t* face_ptr, const int32_t* face_ent, const uint64_t* slot_ids, const MapCtx& mc,
                        bool morton, size_t n_inner, size_t n_local, int tile, DBuf<uint32_t>& tstart,
                        DBuf<uint32_t>& tell, DBuf<uint32_t>& ext_ptr, DBuf<uint32_t>& ext,
                        DBuf<uint32_t>& fine_base, DBuf<uint32_t>& tfine, hipStream_t s) {
	DX_REQUIRE(tile > 0 && tile <= 4096, "tile size out of range");
	DX_REQUIRE(n_local < (size_t(1) << 31), "too many local cells for 32-bit slots");
	TileBuild out{};
	const uint32_t T = uint32_t(tile);
	std::vector<uint8_t> al;
	if (morton && n_local) {
		DBuf<uint8_t> dal;
		dal.alloc(n_local);
		align_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(mc, slot_ids, uint32_t(n_local), dal.p);
		HIP_CHECK(hipGetLastError());
		al = download(dal.p, n_local, s);
	}
	std::vector<uint32_t> hts;
	cut_run(al, 0, uint32_t(n_inner), T, hts);
	out.n_tiles_inner = hts.size();
	cut_run(al, uint32_t(n_inner), uint32_t(n_local), T, hts);
	out.n_tiles_outer = hts.size() - out.n_tiles_inner;
	const size_t ntiles = hts.size();
	hts.push_back(uint32_t(n_local));
	tstart.alloc(ntiles + 1);
	HIP_CHECK(hipMemcpyAsync(tstart.p, hts.data(), (ntiles + 1) * 4, hipMemcpyHostToDevice, s));
	TileGeom tg{tstart.p, uint32_t(ntiles), uint32_t(n_local)};
	tell.alloc(3 * n_local + 3);
	ext_ptr.alloc(ntiles + 1);
	fine_base.alloc(ntiles + 1);
	if (n_local == 0) {
		HIP_CHECK(hipMemsetAsync(ext_ptr.p, 0, 4, s));
		HIP_CHECK(hipStreamSynchronize(s));
		ext.alloc(1);
		tfine.alloc(2);
		return out;
	}
	uint32_t n_ent = 0;
	HIP_CHECK(hipMemcpyAsync(&n_ent, face_ptr + n_local, 4, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));

	// 1-3: per-tile distinct external neighbors
	DBuf<uint64_t> keys;
	keys.alloc(size_t(n_ent) + 1);
	ext_keys_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(tg, face_ptr, face_ent, keys.p);
	HIP_CHECK(hipGetLastError());
	size_t m = sort_unique_u64(keys.p, n_ent, s);
	if (m > 0) {
		uint64_t last = 0;
		HIP_CHECK(hipMemcpyAsync(&last, keys.p + m - 1, 8, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		if (last == ~0ull) m--;
	}
	ext.alloc(m + 1);
	ext_ranges_kernel<<<grid_for(std::max(m, ntiles + 1), 256), 256, 0, s>>>(keys.p, m, uint32_t(ntiles), ext_ptr.p,
	                                                                         ext.p);
	HIP_CHECK(hipGetLastError());
	std::vector<uint32_t> hptr = download(ext_ptr.p, ntiles + 1, s);
	out.total_ext = m;
	for (size_t t = 0; t < ntiles; t++) out.max_ext = std::max<size_t>(out.max_ext, hptr[t + 1] - hptr[t]);
	DX_REQUIRE(size_t(T) + out.max_ext < 0x8000u, "tile too large for 16-bit local indices");

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

	// 5: tile-local rows
	DBuf<int> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	tile_ell_kernel<<<grid_for(n_local, 256), 256, 0, s>>>(tg, T, face_ptr, face_ent, ext_ptr.p, ext.p, fine_idx.p,
	                                                       fine_base.p, tell.p, tfine.p, err.p);
	HIP_CHECK(hipGetLastError());
	int herr = 0;
	HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	DX_REQUIRE(herr == 0, "internal error: face neighbor missing from its tile's external list");
	return out;
}

}  // namespace dccrgx
