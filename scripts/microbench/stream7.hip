// Calibration microbenchmark: the advection sweep's pure streaming part
// (7 fp64 arrays read, 1 written, n cells) in several access shapes, to
// know the achievable rate on this box before tuning the real kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

struct P7 { const double* p[7]; };

// one cell per thread, 8 B per lane per array
__global__ __launch_bounds__(256) void s8(P7 a, double* out, size_t n) {
	size_t i = blockIdx.x * size_t(256) + threadIdx.x;
	if (i >= n) return;
	double s = 0;
#pragma unroll
	for (int k = 0; k < 7; k++) s += a.p[k][i];
	out[i] = s;
}

// two cells per thread, 16 B per lane per array
__global__ __launch_bounds__(256) void s16(P7 a, double* out, size_t n) {
	size_t i = (blockIdx.x * size_t(256) + threadIdx.x) * 2;
	if (i + 1 >= n) return;
	double2 s = {0, 0};
#pragma unroll
	for (int k = 0; k < 7; k++) {
		const double2 v = *reinterpret_cast<const double2*>(a.p[k] + i);
		s.x += v.x;
		s.y += v.y;
	}
	*reinterpret_cast<double2*>(out + i) = s;
}

// persistent grid-stride, 16 B per lane, XCD-contiguous chunks
__global__ __launch_bounds__(256) void s16p(P7 a, double* out, size_t n) {
	const size_t nb = gridDim.x, b = blockIdx.x;
	const size_t lb = (b & 7) * (nb >> 3) + (b >> 3);
	const size_t per = (n / 2 + nb - 1) / nb;
	for (size_t q = lb * per + threadIdx.x; q < (lb + 1) * per && 2 * q + 1 < n; q += 256) {
		const size_t i = 2 * q;
		double2 s = {0, 0};
#pragma unroll
		for (int k = 0; k < 7; k++) {
			const double2 v = *reinterpret_cast<const double2*>(a.p[k] + i);
			s.x += v.x;
			s.y += v.y;
		}
		*reinterpret_cast<double2*>(out + i) = s;
	}
}

// 512-thread blocks, one cell per thread (the tile kernels' shape)
__global__ __launch_bounds__(512) void s8b512(P7 a, double* out, size_t n) {
	size_t i = blockIdx.x * size_t(512) + threadIdx.x;
	if (i >= n) return;
	double s = 0;
#pragma unroll
	for (int k = 0; k < 7; k++) s += a.p[k][i];
	out[i] = s;
}

int main() {
	const size_t n = 8870912;
	std::vector<double*> d(8);
	for (auto& p : d) {
		CK(hipMalloc(&p, n * 8));
		CK(hipMemset(p, 0, n * 8));
	}
	P7 a;
	for (int k = 0; k < 7; k++) a.p[k] = d[k];
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const double bytes = 64.0 * n;
	auto run = [&](const char* name, auto launch) {
		for (int w = 0; w < 3; w++) launch();
		CK(hipEventRecord(e0));
		const int it = 50;
		for (int w = 0; w < it; w++) launch();
		CK(hipEventRecord(e1));
		CK(hipEventSynchronize(e1));
		float ms = 0;
		CK(hipEventElapsedTime(&ms, e0, e1));
		printf("%-10s %.4f ms  %.2f TB/s\n", name, ms / it, bytes / (ms / it * 1e-3) / 1e12);
		return 0;
	};
	run("s8", [&] { s8<<<(n + 255) / 256, 256>>>(a, d[7], n); });
	run("s8b512", [&] { s8b512<<<(n + 511) / 512, 512>>>(a, d[7], n); });
	run("s16", [&] { s16<<<(n / 2 + 255) / 256, 256>>>(a, d[7], n); });
	for (int k : {1024, 2048, 4096})
		run(k == 1024 ? "s16p1k" : (k == 2048 ? "s16p2k" : "s16p4k"), [&] { s16p<<<k, 256>>>(a, d[7], n); });
	// a plain device copy of the same byte count for reference
	double *src, *dst;
	CK(hipMalloc(&src, n * 32));
	CK(hipMalloc(&dst, n * 32));
	run("memcpy", [&] { (void)hipMemcpyAsync(dst, src, n * 32, hipMemcpyDeviceToDevice, 0); });
	return 0;
}
