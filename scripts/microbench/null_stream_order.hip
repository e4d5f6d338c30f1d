// Does a null-stream hipMemset order with a kernel queued afterwards on a
// non-blocking stream?  (The library's compute and comm streams are created
// with hipStreamNonBlocking; until a8c28ec, add_field and the Poisson solver's
// own fields were zeroed with hipMemset on the null stream, then written by
// kernels on the compute stream.)
//
// Per trial: hipMemset(buf, 0) on the null stream, then at once a kernel on a
// non-blocking stream that writes 1 into every element, then a device sync.
// If the two are unordered the memset may land after the kernel: the
// elements it clears after the kernel wrote them read 0.  Reports the trials
// with any such element, and the same with the kernel on a blocking stream
// (which the null stream orders) as the control.
//
//   hipcc --offload-arch=gfx950 -O2 null_stream_order.hip -o null_stream_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
	do {                                                                        \
		hipError_t e_ = (x);                                                    \
		if (e_ != hipSuccess) {                                                 \
			std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			std::exit(1);                                                       \
		}                                                                       \
	} while (0)

__global__ void fill_one(unsigned* p, size_t n) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = 1u;
}

__global__ void count_zero(const unsigned* p, size_t n, unsigned long long* z) {
	unsigned long long c = 0;
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) c += p[i] == 0u;
	if (c) atomicAdd(z, c);
}

static void run(const char* what, unsigned flags, size_t n, int trials) {
	hipStream_t s;
	CK(hipStreamCreateWithFlags(&s, flags));
	unsigned* buf;
	unsigned long long* z;
	CK(hipMalloc(&buf, n * 4));
	CK(hipMalloc(&z, 8));
	int bad = 0;
	unsigned long long worst = 0;
	for (int t = 0; t < trials; t++) {
		CK(hipDeviceSynchronize());
		CK(hipMemset(buf, 0, n * 4));                     // null stream
		fill_one<<<1024, 256, 0, s>>>(buf, n);            // the other stream, right away
		CK(hipGetLastError());
		CK(hipDeviceSynchronize());
		CK(hipMemset(z, 0, 8));
		count_zero<<<1024, 256>>>(buf, n, z);
		unsigned long long h = 0;
		CK(hipMemcpy(&h, z, 8, hipMemcpyDeviceToHost));
		if (h) {
			bad++;
			if (h > worst) worst = h;
		}
	}
	std::printf("{\"stream\": \"%s\", \"elements\": %zu, \"trials\": %d, \"trials_with_zeros\": %d, \"max_zeros\": %llu}\n",
	            what, n, trials, bad, worst);
	CK(hipFree(buf));
	CK(hipFree(z));
	CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
	const int trials = argc > 1 ? std::atoi(argv[1]) : 200;
	for (size_t n : {size_t(4096), size_t(1) << 16, size_t(1) << 22, size_t(1) << 26}) {
		run("non-blocking", hipStreamNonBlocking, n, trials);
		run("blocking (control)", hipStreamDefault, n, trials);
	}
	return 0;
}
