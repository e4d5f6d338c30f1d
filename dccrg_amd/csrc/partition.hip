// dccrgx: native repartitioner — recursive coordinate bisection of the leaves
// over the processes, weighted, computed on the device across ranks.
//
// It replaces the reference's default partitioner: balance_load(use_zoltan)
// -> make_new_partition (dccrg.hpp:8349-8376) -> Zoltan_LB_Balance with
// LB_METHOD "RCB" (7082), whose inputs are every local leaf, its weight
// (set_cell_weight 6210, unset = 1; fill_cell_list 11741-11783) and its center
// (fill_with_cell_coordinates 11682-11716).  Zoltan is third-party and absent
// here, so the cut rule is this file's own (parity unpinned against Zoltan):
//
//   * processes [lo, hi) holding a group of cells are split into
//     [lo, lo + P1) and [lo + P1, hi), P1 = (hi - lo) / 2;
//   * the cut axis is the longest side of the group's bounding box of cell
//     centers (ties: x before y before z);
//   * cells are ordered by (center along the axis, id) and the lower part
//     takes the longest prefix whose weight is <= floor(W * P1 / (hi - lo)).
//
// Centers are exact integers (2 x minimum index + length in indices), weights
// fixed point (2^-16), every sum an integer: the result is a pure function of
// the leaf set and the weights, bit-identical for any current distribution,
// rank count of the input or summation order.  The ordered cut is a radix
// select over the keys (center << id_bits | id; 64-bit when they fit, else
// 128-bit), 8 bits per pass from the highest occupied byte: one device
// histogram per pass and group, summed over ranks.
#include <algorithm>

#include "dccrgx_grid.hpp"

namespace dccrgx {
namespace {

constexpr int kBins = 256;
constexpr int kMaxGroupsLds = 16;  // groups whose histograms fit one block's LDS (32 KB)
constexpr double kWeightOne = 65536.0;

__global__ void rcb_init_kernel(MapCtx m, const uint64_t* ids, size_t n, uint32_t* c2, int32_t* lo, int32_t* hi,
                                uint64_t* w, int P) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		map_indices(m, ids[i], x, y, z);
		const uint64_t L = map_cell_len(m, ids[i]);
		c2[3 * i + 0] = uint32_t(2 * x + L);
		c2[3 * i + 1] = uint32_t(2 * y + L);
		c2[3 * i + 2] = uint32_t(2 * z + L);
		lo[i] = 0;
		hi[i] = P;
		w[i] = uint64_t(kWeightOne);
	}
}

__global__ void rcb_set_weights_kernel(const int32_t* slots, const uint64_t* wv, size_t n, uint64_t* w) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		w[slots[i]] = wv[i];
}

// per active group: min and max center along each axis (6 words; the
// minimum stored complemented so that every word is a max)
__global__ void rcb_bbox_kernel(const uint32_t* c2, const int32_t* lo, const int32_t* hi, size_t n,
                                const int32_t* group_of_lo, int G, unsigned int* box) {
	extern __shared__ unsigned int sbox[];
	for (int k = threadIdx.x; k < 6 * G; k += blockDim.x) sbox[k] = 0;
	__syncthreads();
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (hi[i] - lo[i] < 2) continue;
		const int gi = group_of_lo[lo[i]];
		for (int d = 0; d < 3; d++) {
			atomicMax(&sbox[6 * gi + d], ~c2[3 * i + d]);
			atomicMax(&sbox[6 * gi + 3 + d], c2[3 * i + d]);
		}
	}
	__syncthreads();
	for (int k = threadIdx.x; k < 6 * G; k += blockDim.x)
		if (sbox[k]) atomicMax(&box[k], sbox[k]);
}

// K: uint64_t when center and id bits fit 64, else unsigned __int128 (a grid
// at a refinement level near the id space's limit, set_maximum_refinement_
// level(-1) on a small grid)
template <class K>
__device__ __forceinline__ K rcb_key(const uint32_t* c2, const uint64_t* ids, size_t i, int axis, int id_bits) {
	return (K(c2[3 * i + axis]) << id_bits) | K(ids[i]);
}

// weight histogram of the next 8 key bits below `shift + 8` of the cells of
// every active group whose key agrees with the group's prefix above them
template <class K>
__global__ void rcb_hist_kernel(const uint32_t* c2, const uint64_t* ids, const uint64_t* w, const int32_t* lo,
                                const int32_t* hi, size_t n, const int32_t* group_of_lo, int G, const int32_t* axis,
                                const K* prefix, int shift, bool first, int id_bits, unsigned long long* hist) {
	extern __shared__ unsigned long long shist[];
	const bool lds = G <= kMaxGroupsLds;
	if (lds) {
		for (int k = threadIdx.x; k < G * kBins; k += blockDim.x) shist[k] = 0;
		__syncthreads();
	}
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		if (hi[i] - lo[i] < 2) continue;
		const int gi = group_of_lo[lo[i]];
		const K key = rcb_key<K>(c2, ids, i, axis[gi], id_bits);
		if (!first && (key >> (shift + 8)) != prefix[gi]) continue;
		const int b = int((key >> shift) & 0xff);
		if (lds) atomicAdd(&shist[gi * kBins + b], (unsigned long long)w[i]);
		else atomicAdd(&hist[gi * kBins + b], (unsigned long long)w[i]);
	}
	if (lds) {
		__syncthreads();
		for (int k = threadIdx.x; k < G * kBins; k += blockDim.x)
			if (shist[k]) atomicAdd(&hist[k], shist[k]);
	}
}

template <class K>
__global__ void rcb_assign_kernel(const uint32_t* c2, const uint64_t* ids, int32_t* lo, int32_t* hi, size_t n,
                                  const int32_t* group_of_lo, const int32_t* axis, const K* cut, int id_bits) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int32_t l = lo[i], h = hi[i];
		if (h - l < 2) continue;
		const int gi = group_of_lo[l];
		const int32_t mid = l + (h - l) / 2;
		if (rcb_key<K>(c2, ids, i, axis[gi], id_bits) < cut[gi]) hi[i] = mid;
		else lo[i] = mid;
	}
}

int bits_for(uint64_t v) {
	int b = 0;
	while (b < 64 && (v >> b)) b++;
	return b;
}

// element-wise sum / max over ranks of a host vector (through the grid's
// transport; every rank passes the same length)
void allreduce_u64(Grid& g, std::vector<uint64_t>& v, bool max) {
	if (g.size == 1) return;
	const auto all = comm_allgather_u64(g, v);
	std::fill(v.begin(), v.end(), 0);
	for (const auto& a : all) {
		DX_REQUIRE(a.size() == v.size(), "partitioner: ranks disagree on the group count");
		for (size_t k = 0; k < v.size(); k++) v[k] = max ? std::max(v[k], a[k]) : v[k] + a[k];
	}
}

// the bisection levels: every group's cut by a radix select over the keys
// (center << id_bits | id), 8 bits per pass from the highest occupied byte
template <class K>
void rcb_levels(Grid& g, size_t n, DBuf<uint32_t>& c2, DBuf<int32_t>& lo, DBuf<int32_t>& hi, DBuf<uint64_t>& w,
                int id_bits, int key_bits) {
	hipStream_t s = g.s_comp;
	const int P = g.size;
	const int top = ((key_bits + 7) / 8) * 8 - 8;
	// the process tree is known to every rank: groups of a level are the
	// ranges of size > 1 produced by halving the previous level's ranges
	std::vector<std::pair<int, int>> groups;
	if (P > 1) groups.push_back({0, P});
	DBuf<int32_t> d_group_of_lo, d_axis;
	DBuf<K> d_prefix, d_cut;
	DBuf<unsigned int> d_box;
	DBuf<unsigned long long> d_hist;
	d_group_of_lo.alloc(size_t(P) + 1);
	while (!groups.empty()) {
		const int G = int(groups.size());
		std::vector<int32_t> group_of_lo(size_t(P), -1);
		for (int k = 0; k < G; k++) group_of_lo[size_t(groups[size_t(k)].first)] = k;
		upload(d_group_of_lo, group_of_lo, s);

		// bounding boxes -> cut axis
		d_box.alloc(size_t(6 * G));
		HIP_CHECK(hipMemsetAsync(d_box.p, 0, size_t(6 * G) * 4, s));
		if (n) {
			rcb_bbox_kernel<<<grid_for(n, 256, 1024), 256, size_t(6 * G) * 4, s>>>(c2.p, lo.p, hi.p, n,
			                                                                     d_group_of_lo.p, G, d_box.p);
			HIP_CHECK(hipGetLastError());
		}
		std::vector<uint32_t> box32 = download(d_box.p, size_t(6 * G), s);
		std::vector<uint64_t> box(box32.begin(), box32.end());
		allreduce_u64(g, box, true);
		std::vector<int32_t> axis(size_t(G), 0);
		for (int k = 0; k < G; k++) {
			uint64_t best = 0;
			for (int d = 0; d < 3; d++) {
				const uint64_t mx = box[size_t(6 * k + 3 + d)], mn = ~uint32_t(box[size_t(6 * k + d)]);
				const uint64_t ext = mx >= mn ? mx - mn : 0;
				if (d == 0 || ext > best) {
					best = ext;
					axis[size_t(k)] = d;
				}
			}
		}
		upload(d_axis, axis, s);

		// radix select of every group's cut key, 8 bits per pass, high first
		std::vector<K> prefix(size_t(G), 0);
		std::vector<uint64_t> target(size_t(G), 0);
		d_hist.alloc(size_t(G) * kBins);
		for (int shift = top; shift >= 0; shift -= 8) {
			upload(d_prefix, prefix, s);
			HIP_CHECK(hipMemsetAsync(d_hist.p, 0, size_t(G) * kBins * 8, s));
			if (n) {
				const size_t lds = G <= kMaxGroupsLds ? size_t(G) * kBins * 8 : 0;
				rcb_hist_kernel<K><<<grid_for(n, 256, 1024), 256, lds, s>>>(c2.p, g.slot_ids.p, w.p, lo.p, hi.p, n,
				                                                           d_group_of_lo.p, G, d_axis.p, d_prefix.p,
				                                                           shift, shift == top, id_bits, d_hist.p);
				HIP_CHECK(hipGetLastError());
			}
			std::vector<unsigned long long> h64 = download(d_hist.p, size_t(G) * kBins, s);
			std::vector<uint64_t> hist(h64.begin(), h64.end());
			allreduce_u64(g, hist, false);
			for (int k = 0; k < G; k++) {
				const uint64_t* hk = hist.data() + size_t(k) * kBins;
				if (shift == top) {  // the group's total weight -> its target
					unsigned __int128 W = 0;
					for (int b = 0; b < kBins; b++) W += hk[b];
					const int gp = groups[size_t(k)].second - groups[size_t(k)].first;
					target[size_t(k)] = uint64_t(W * unsigned(gp / 2) / unsigned(gp));
				}
				// smallest bin whose inclusive prefix weight exceeds the target
				uint64_t cum = 0;
				int b = 0;
				for (; b < kBins - 1; b++) {
					if (cum + hk[b] > target[size_t(k)]) break;
					cum += hk[b];
				}
				target[size_t(k)] -= cum;
				prefix[size_t(k)] = (prefix[size_t(k)] << 8) | K(b);
			}
		}
		// prefix now holds each group's cut key K: keys < K go to the lower half
		upload(d_cut, prefix, s);
		if (n) {
			rcb_assign_kernel<K><<<grid_for(n, 256), 256, 0, s>>>(c2.p, g.slot_ids.p, lo.p, hi.p, n, d_group_of_lo.p,
			                                                      d_axis.p, d_cut.p, id_bits);
			HIP_CHECK(hipGetLastError());
		}
		std::vector<std::pair<int, int>> next;
		for (const auto& gr : groups) {
			const int mid = gr.first + (gr.second - gr.first) / 2;
			if (mid - gr.first > 1) next.push_back({gr.first, mid});
			if (gr.second - mid > 1) next.push_back({mid, gr.second});
		}
		groups.swap(next);
	}
}

}  // namespace

void rcb_partition(Grid& g, std::vector<uint64_t>& cells, std::vector<int32_t>& owners) {
	DX_REQUIRE(g.initialized, "not initialized");
	if (g.size > 1) comm_require(g, "balance_load");
	hipStream_t s = g.s_comp;
	const size_t n = g.n_local;
	const int P = g.size;
	const int id_bits = bits_for(g.m.last);
	uint64_t cmax = 0;
	for (int d = 0; d < 3; d++) cmax = std::max(cmax, 2 * g.m.glen[d]);
	DX_REQUIRE(cmax < (uint64_t(1) << 32), "grid too large for the partitioner's 32-bit centers");

	DBuf<uint32_t> c2;
	DBuf<int32_t> lo, hi;
	DBuf<uint64_t> w;
	c2.alloc(3 * n + 3);
	lo.alloc(n + 1);
	hi.alloc(n + 1);
	w.alloc(n + 1);
	if (n) {
		rcb_init_kernel<<<grid_for(n, 256), 256, 0, s>>>(g.m, g.slot_ids.p, n, c2.p, lo.p, hi.p, w.p, P);
		HIP_CHECK(hipGetLastError());
	}
	// user weights (set_cell_weight), fixed point
	if (!g.weights.empty()) {
		std::vector<int32_t> sl;
		std::vector<uint64_t> wv;
		for (const auto& kv : g.weights) {
			const int64_t sidx = host_slot_of(g, kv.first);
			if (sidx < 0 || size_t(sidx) >= n) continue;
			sl.push_back(int32_t(sidx));
			wv.push_back(uint64_t(std::llround(kv.second * kWeightOne)));
		}
		if (!sl.empty()) {
			DBuf<int32_t> dsl;
			DBuf<uint64_t> dwv;
			upload(dsl, sl, s);
			upload(dwv, wv, s);
			rcb_set_weights_kernel<<<grid_for(sl.size(), 256), 256, 0, s>>>(dsl.p, dwv.p, sl.size(), w.p);
			HIP_CHECK(hipGetLastError());
		}
	}

	const int key_bits = bits_for(cmax) + id_bits;
	if (key_bits <= 64) rcb_levels<uint64_t>(g, n, c2, lo, hi, w, id_bits, key_bits);
	else rcb_levels<unsigned __int128>(g, n, c2, lo, hi, w, id_bits, key_bits);
	HIP_CHECK(hipStreamSynchronize(s));
	// local cells ascending with their new owners
	const std::vector<uint64_t> ids = download(g.slot_ids.p, n, s);
	const std::vector<int32_t> own = download(lo.p, n, s);
	std::vector<size_t> order(n);
	for (size_t i = 0; i < n; i++) order[i] = i;
	std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return ids[a] < ids[b]; });
	cells.resize(n);
	owners.resize(n);
	for (size_t i = 0; i < n; i++) {
		cells[i] = ids[order[i]];
		owners[i] = P > 1 ? own[order[i]] : 0;
	}
}

}  // namespace dccrgx
