// Which XCD runs workgroup b?  Reads HW_REG_XCC_ID (gfx94x/gfx950 hwreg 20,
// bits 3:0) per workgroup, for the persistent tile sweeps' launch shape
// (512 threads, 62 KB dynamic LDS, 512 workgroups) and for a plain grid.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void xcc(int* out) {
	extern __shared__ double lds[];
	if (threadIdx.x == 0) {
		lds[0] = 1.0;
		out[blockIdx.x] = int(__builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)));
	}
}

int main() {
	for (int shape = 0; shape < 2; shape++) {
		const int nb = shape == 0 ? 512 : 4096;
		const size_t lds = shape == 0 ? 62 * 1024 : 0;
		int* d;
		(void)hipMalloc(&d, nb * sizeof(int));
		xcc<<<nb, 512, lds>>>(d);
		std::vector<int> h(nb);
		(void)hipMemcpy(h.data(), d, nb * sizeof(int), hipMemcpyDeviceToHost);
		int match = 0;
		for (int b = 0; b < nb; b++) match += (h[b] == b % 8);
		printf("shape %d: %d of %d workgroups on XCD b %% 8; first 16:", shape, match, nb);
		for (int b = 0; b < 16; b++) printf(" %d", h[b]);
		printf("\n");
		(void)hipFree(d);
	}
	return 0;
}
