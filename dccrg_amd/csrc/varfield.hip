// Variable-size cell payloads (tests/variable_data_size/*: a Cell_Data whose
// get_mpi_datatype describes a different number of bytes per cell, e.g. a
// std::vector member, dccrg_get_cell_datatype.hpp:40-340).  A variable field
// is one byte pool over all slots with a byte offset per slot (voff, n_slots
// + 1 entries, the exclusive scan of the slot sizes): slot s owns bytes
// [voff[s], voff[s + 1]).  The halo, migrations and the removed-cell store
// move (sizes, concatenated bytes) pairs, so a receiver takes the sender's
// sizes (the reference requires the receiver to size its copies first,
// variable_neighbour_data.cpp:95-102; with that done the bytes are the same).
// Not a sweep path: copies are one wave per cell.
#include <hipcub/hipcub.hpp>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

// one wave copies one cell's bytes: 4-byte words when everything is aligned
__device__ __forceinline__ void wave_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t len,
                                          uint32_t lane) {
	if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | len) & 3u) == 0) {
		uint32_t* d = reinterpret_cast<uint32_t*>(dst);
		const uint32_t* q = reinterpret_cast<const uint32_t*>(src);
		for (uint64_t i = lane; i < len / 4; i += 64) d[i] = q[i];
	} else {
		for (uint64_t i = lane; i < len; i += 64) dst[i] = src[i];
	}
}

#define WAVE_LOOP(n)                                                                         \
	const uint32_t lane = threadIdx.x & 63u;                                                 \
	const size_t waves = size_t(gridDim.x) * (blockDim.x >> 6);                              \
	for (size_t i = blockIdx.x * size_t(blockDim.x >> 6) + (threadIdx.x >> 6); i < (n); i += waves)

__global__ void var_sizes_kernel(const uint64_t* __restrict__ voff, const int32_t* __restrict__ slots, size_t slot0,
                                 size_t n, uint64_t* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const size_t s = slots ? size_t(slots[i]) : slot0 + i;
		out[i] = voff[s + 1] - voff[s];
	}
}

// per slot the first min(old, new) bytes into the new layout (the rest was zeroed)
__global__ void var_resize_copy_kernel(const uint8_t* __restrict__ old_data, const uint64_t* __restrict__ ooff,
                                       uint8_t* __restrict__ new_data, const uint64_t* __restrict__ noff, size_t n) {
	WAVE_LOOP(n) {
		const uint64_t lo = ooff[i + 1] - ooff[i], ln = noff[i + 1] - noff[i];
		wave_copy(new_data + noff[i], old_data + ooff[i], lo < ln ? lo : ln, lane);
	}
}

// the cells at slots[i] into one buffer at out_off[i] (exclusive scan of their sizes)
__global__ void var_gather_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ voff,
                                  const int32_t* __restrict__ slots, size_t n, const uint64_t* __restrict__ out_off,
                                  uint8_t* __restrict__ out) {
	WAVE_LOOP(n) {
		const size_t s = size_t(slots[i]);
		wave_copy(out + out_off[i], data + voff[s], voff[s + 1] - voff[s], lane);
	}
}

// the concatenated payloads in (in_off) into the cells at slots[i] (already sized)
__global__ void var_scatter_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                                   const int32_t* __restrict__ slots, size_t n, uint8_t* __restrict__ data,
                                   const uint64_t* __restrict__ voff) {
	WAVE_LOOP(n) {
		const size_t s = size_t(slots[i]);
		wave_copy(data + voff[s], in + in_off[i], in_off[i + 1] - in_off[i], lane);
	}
}

__global__ void scatter_sizes_kernel(uint64_t* __restrict__ sizes, const int32_t* __restrict__ slots,
                                     const uint64_t* __restrict__ in, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		sizes[slots[i]] = in[i];
}

__global__ void differ_kernel(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, size_t n,
                              int32_t* __restrict__ flag) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		if (a[i] != b[i]) *flag = 1;
}

// after a rebuild: the old local slot of every new slot (-1: none)
__global__ void var_src_kernel(const uint64_t* __restrict__ old_ids, size_t n_old, DevMesh newM,
                               int32_t* __restrict__ src) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n_old; i += size_t(gridDim.x) * blockDim.x) {
		const int32_t s = dm_slot(newM, old_ids[i]);
		if (s >= 0) src[s] = int32_t(i);
	}
}

__global__ void var_src_sizes_kernel(const int32_t* __restrict__ src, const uint64_t* __restrict__ ooff, size_t n,
                                     uint64_t* __restrict__ sizes) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		sizes[i] = src[i] >= 0 ? ooff[src[i] + 1] - ooff[src[i]] : 0;
}

__global__ void var_src_copy_kernel(const uint8_t* __restrict__ old_data, const uint64_t* __restrict__ ooff,
                                    const int32_t* __restrict__ src, uint8_t* __restrict__ new_data,
                                    const uint64_t* __restrict__ noff, size_t n) {
	WAVE_LOOP(n) {
		if (src[i] < 0) continue;
		wave_copy(new_data + noff[i], old_data + ooff[src[i]], noff[i + 1] - noff[i], lane);
	}
}

unsigned wave_grid(size_t n) { return grid_for(n, 4, 8192); }  // 4 waves of 64 per 256-thread block

}  // namespace

uint64_t scan_exclusive_u64(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s) {
	// scans n + 1 entries (in[n] is ignored, out[n] = total)
	size_t bytes = 0;
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, n + 1, s));
	DBuf<uint8_t> temp;
	temp.alloc(bytes + 1);
	HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp.p, bytes, in, out, n + 1, s));
	uint64_t h = 0;
	d2h_small(&h, out + n, sizeof(h), s);
	return h;
}

void var_reset(Field& f, size_t n_slots, hipStream_t s) {
	f.voff.alloc(n_slots + 1);
	HIP_CHECK(hipMemsetAsync(f.voff.p, 0, (n_slots + 1) * 8, s));
	f.data.release();
	HIP_CHECK(hipStreamSynchronize(s));
}

uint64_t var_total(const Field& f, size_t n_slots, hipStream_t s) {
	uint64_t h = 0;
	d2h_small(&h, f.voff.p + n_slots, 8, s);
	return h;
}

void var_sizes(const Field& f, const int32_t* slots, size_t slot0, size_t n, uint64_t* out, hipStream_t s) {
	if (!n) return;
	var_sizes_kernel<<<grid_for(n, 256), 256, 0, s>>>(f.voff.p, slots, slot0, n, out);
	HIP_CHECK(hipGetLastError());
}

void var_resize(Field& f, size_t n_slots, const uint64_t* new_sizes, hipStream_t s) {
	DBuf<uint64_t> noff;
	noff.alloc(n_slots + 1);
	const uint64_t total = scan_exclusive_u64(new_sizes, noff.p, n_slots, s);
	DBuf<uint8_t> nd;
	nd.alloc(total + 1);
	HIP_CHECK(hipMemsetAsync(nd.p, 0, total + 1, s));
	if (n_slots && f.data.p) {
		var_resize_copy_kernel<<<wave_grid(n_slots), 256, 0, s>>>(f.data.p, f.voff.p, nd.p, noff.p, n_slots);
		HIP_CHECK(hipGetLastError());
	}
	HIP_CHECK(hipStreamSynchronize(s));
	f.data.swap(nd);
	f.voff.swap(noff);
}

size_t var_gather(const Field& f, const int32_t* slots, size_t n, DBuf<uint64_t>& sizes, DBuf<uint8_t>& bytes,
                  hipStream_t s) {
	sizes.alloc(n + 1);
	DBuf<uint64_t> off;
	off.alloc(n + 1);
	var_sizes(f, slots, 0, n, sizes.p, s);
	const uint64_t total = scan_exclusive_u64(sizes.p, off.p, n, s);
	bytes.alloc(total + 1);
	if (n && total) {
		var_gather_kernel<<<wave_grid(n), 256, 0, s>>>(f.data.p, f.voff.p, slots, n, off.p, bytes.p);
		HIP_CHECK(hipGetLastError());
	}
	HIP_CHECK(hipStreamSynchronize(s));
	return size_t(total);
}

uint64_t var_place(Field& f, size_t n_slots, const int32_t* slots, size_t n, const uint64_t* sizes,
                   const uint8_t* bytes, hipStream_t s) {
	if (!n) return 0;
	// the cells take the incoming sizes; the pool is relaid only when one changes
	DBuf<uint64_t> cur, want;
	cur.alloc(n_slots + 1);
	want.alloc(n_slots + 1);
	var_sizes(f, nullptr, 0, n_slots, cur.p, s);
	HIP_CHECK(hipMemcpyAsync(want.p, cur.p, n_slots * 8, hipMemcpyDeviceToDevice, s));
	scatter_sizes_kernel<<<grid_for(n, 256), 256, 0, s>>>(want.p, slots, sizes, n);
	HIP_CHECK(hipGetLastError());
	DBuf<int32_t> flag;
	flag.alloc(1);
	HIP_CHECK(hipMemsetAsync(flag.p, 0, 4, s));
	if (n_slots) {
		differ_kernel<<<grid_for(n_slots, 256), 256, 0, s>>>(cur.p, want.p, n_slots, flag.p);
		HIP_CHECK(hipGetLastError());
	}
	int32_t h = 0;
	d2h_small(&h, flag.p, 4, s);
	if (h) var_resize(f, n_slots, want.p, s);
	DBuf<uint64_t> in_off;
	in_off.alloc(n + 1);
	const uint64_t total = scan_exclusive_u64(sizes, in_off.p, n, s);
	if (total) {
		var_scatter_kernel<<<wave_grid(n), 256, 0, s>>>(bytes, in_off.p, slots, n, f.data.p, f.voff.p);
		HIP_CHECK(hipGetLastError());
	}
	HIP_CHECK(hipStreamSynchronize(s));
	return total;
}

void var_remap(Field& f, const uint64_t* old_ids, size_t n_old_local, const DevMesh& newM, size_t new_n_slots,
               hipStream_t s) {
	DBuf<int32_t> src;
	src.alloc(new_n_slots + 1);
	k_fill_i32(src.p, new_n_slots + 1, -1, s);
	if (n_old_local && f.voff.p) {
		var_src_kernel<<<grid_for(n_old_local, 256), 256, 0, s>>>(old_ids, n_old_local, newM, src.p);
		HIP_CHECK(hipGetLastError());
	}
	DBuf<uint64_t> sizes, noff;
	sizes.alloc(new_n_slots + 1);
	noff.alloc(new_n_slots + 1);
	if (new_n_slots) {
		if (f.voff.p) {
			var_src_sizes_kernel<<<grid_for(new_n_slots, 256), 256, 0, s>>>(src.p, f.voff.p, new_n_slots, sizes.p);
			HIP_CHECK(hipGetLastError());
		} else {
			HIP_CHECK(hipMemsetAsync(sizes.p, 0, new_n_slots * 8, s));
		}
	}
	const uint64_t total = scan_exclusive_u64(sizes.p, noff.p, new_n_slots, s);
	DBuf<uint8_t> nd;
	nd.alloc(total + 1);
	if (total && f.data.p) {
		var_src_copy_kernel<<<wave_grid(new_n_slots), 256, 0, s>>>(f.data.p, f.voff.p, src.p, nd.p, noff.p,
		                                                          new_n_slots);
		HIP_CHECK(hipGetLastError());
	}
	HIP_CHECK(hipStreamSynchronize(s));
	f.data.swap(nd);
	f.voff.swap(noff);
}

}  // namespace dccrgx
