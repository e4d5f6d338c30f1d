// Cost of host-to-device uploads of list-sized buffers before a kernel:
// pageable vs pinned source, per size (hipMemcpyAsync + kernel + sync).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void touch(const unsigned long long* d, unsigned long long* o) {
	if (threadIdx.x == 0 && blockIdx.x == 0) o[0] += d[0];
}

int main() {
	const size_t sizes[] = {8, 64 << 10, 400 << 10, 4 << 20};
	unsigned long long *d = nullptr, *o = nullptr;
	if (hipMalloc(&d, 4 << 20) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
	hipStream_t s;
	if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
	void* pinned = nullptr;
	if (hipHostMalloc(&pinned, 4 << 20, 0) != hipSuccess) return 1;
	std::vector<char> pageable(4 << 20, 1);
	for (size_t b : sizes) {
		for (int mode = 0; mode < 3; mode++) {
			const int N = 500;
			const auto t0 = std::chrono::steady_clock::now();
			for (int i = 0; i < N; i++) {
				if (mode == 0) (void)hipMemcpyAsync(d, pageable.data(), b, hipMemcpyHostToDevice, s);
				else if (mode == 1) (void)hipMemcpyAsync(d, pinned, b, hipMemcpyHostToDevice, s);
				else {
					std::memcpy(pinned, pageable.data(), b);  // staged through pinned memory
					(void)hipMemcpyAsync(d, pinned, b, hipMemcpyHostToDevice, s);
				}
				touch<<<1, 64, 0, s>>>(d, o);
				(void)hipStreamSynchronize(s);
			}
			const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / N;
			printf("%8zu B %-22s %.2f us per upload + kernel + sync\n", b,
			       mode == 0 ? "pageable" : (mode == 1 ? "pinned" : "memcpy + pinned"), us);
		}
	}
	return 0;
}
