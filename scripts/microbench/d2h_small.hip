// Cost of a small device-to-host readback (a counter) after a kernel:
// pageable vs pinned destination, hipMemcpyAsync + hipStreamSynchronize.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void bump(unsigned long long* c) {
	if (threadIdx.x == 0 && blockIdx.x == 0) c[0] += 1;
}

int main() {
	unsigned long long* d = nullptr;
	if (hipMalloc(&d, 64) != hipSuccess) return 1;
	hipStream_t s;
	if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
	unsigned long long* pinned = nullptr;
	if (hipHostMalloc(&pinned, 64, 0) != hipSuccess) return 1;
	unsigned long long pageable[8] = {0};
	const int N = 2000;
	for (int mode = 0; mode < 3; mode++) {
		for (int rep = 0; rep < 2; rep++) {
			const auto t0 = std::chrono::steady_clock::now();
			for (int i = 0; i < N; i++) {
				bump<<<1, 64, 0, s>>>(d);
				if (mode == 0) {
					(void)hipMemcpyAsync(pageable, d, 8, hipMemcpyDeviceToHost, s);
					(void)hipStreamSynchronize(s);
				} else if (mode == 1) {
					(void)hipMemcpyAsync(pinned, d, 8, hipMemcpyDeviceToHost, s);
					(void)hipStreamSynchronize(s);
				} else {
					(void)hipStreamSynchronize(s);
				}
			}
			const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
			printf("%s: %.2f us per kernel + readback + sync\n",
			       mode == 0 ? "pageable" : (mode == 1 ? "pinned" : "sync only (no copy)"), us);
		}
	}
	(void)hipHostFree(pinned);
	(void)hipFree(d);
	return 0;
}
