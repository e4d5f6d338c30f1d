// Stencil sweeps over local cells and remote-neighbor copies, plus the halo
// pack.  These replace the user loops of the reference's tests/examples:
//   game of life  examples/game_of_life.cpp:54-79,
//                 tests/game_of_life/scalability3d.cpp:130-165
//   advection     tests/advection/solve.hpp:44-279 (calculate_fluxes +
//                 apply_fluxes fused: every cell gathers its own faces, so
//                 the reference's scatter into two cells becomes a race-free
//                 gather with no atomics)
// All bandwidth-bound; no MFMA.
#include <cstdlib>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

inline unsigned grid_for(size_t n, unsigned per_block, unsigned cap = 256u * 64u) {
	size_t g = (n + per_block - 1) / per_block;
	if (g > cap) g = cap;
	if (g == 0) g = 1;
	return unsigned(g);
}

// ---------------------------------------------------------------------------
template <class T>
__global__ void pack_kernel(const T* __restrict__ f, const int32_t* __restrict__ slots, size_t n, T* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = f[slots[i]];
}

__global__ void pack_bytes_kernel(const uint8_t* __restrict__ f, size_t elem, const int32_t* __restrict__ slots,
                                  size_t n, uint8_t* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n * elem; i += size_t(gridDim.x) * blockDim.x) {
		const size_t k = i / elem, b = i - k * elem;
		out[i] = f[size_t(slots[k]) * elem + b];
	}
}

// ---------------------------------------------------------------------------
// Game of life over the iterator neighbor list (deduplicated neighbors_of).
__global__ void gol_csr_kernel(const uint32_t* __restrict__ state, uint32_t* __restrict__ out,
                               const uint32_t* __restrict__ ptr, const int32_t* __restrict__ nb, size_t s0, size_t s1) {
	for (size_t s = s0 + blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < s1; s += size_t(gridDim.x) * blockDim.x) {
		uint32_t cnt = 0;
		for (uint32_t e = ptr[s]; e < ptr[s + 1]; e++) cnt += state[nb[e]] > 0 ? 1u : 0u;
		const uint32_t cur = state[s];
		out[s] = cnt == 3 ? 1u : (cnt == 2 ? cur : 0u);
	}
}

// Game of life, uniform grid (R = 0), one rank, neighborhood length 1: slot ==
// id - 1 == x + nx*(y + ny*z).  A workgroup owns a TX x TY column tile and
// marches up a z chunk; each plane is staged once into LDS with a one-cell
// ring, the 3x3 in-plane sums of three consecutive planes stay in registers,
// and count(z) = S(z-1) + S(z) + S(z+1) - state(z).
constexpr int GTX = 64, GTY = 8, GZC = 32;

__global__ __launch_bounds__(GTX* GTY) void gol_structured_kernel(const uint32_t* __restrict__ st,
                                                                   uint32_t* __restrict__ out, int nx, int ny, int nz,
                                                                   int px, int py, int pz) {
	__shared__ uint32_t tile[GTY + 2][GTX + 2];
	const int tx = threadIdx.x % GTX, ty = threadIdx.x / GTX;
	const int x0 = blockIdx.x * GTX, y0 = blockIdx.y * GTY, z0 = blockIdx.z * GZC;
	const int x = x0 + tx, y = y0 + ty;
	const int z1 = min(z0 + GZC, nz);
	const size_t plane = size_t(nx) * ny;

	auto load_plane = [&](int z) -> void {
		// returns via LDS; z may be outside [0, nz)
		bool zin = true;
		int zz = z;
		if (zz < 0 || zz >= nz) {
			if (pz) zz = (zz + nz) % nz;
			else zin = false;
		}
		for (int i = threadIdx.x; i < (GTX + 2) * (GTY + 2); i += GTX * GTY) {
			const int ly = i / (GTX + 2), lx = i % (GTX + 2);
			int gx = x0 + lx - 1, gy = y0 + ly - 1;
			bool in = zin;
			if (gx < 0 || gx >= nx) {
				if (px) gx = (gx + nx) % nx;
				else in = false;
			}
			if (gy < 0 || gy >= ny) {
				if (py) gy = (gy + ny) % ny;
				else in = false;
			}
			tile[ly][lx] = in ? (st[size_t(zz) * plane + size_t(gy) * nx + gx] > 0 ? 1u : 0u) : 0u;
		}
	};
	auto sum9 = [&]() -> uint32_t {
		uint32_t s = 0;
#pragma unroll
		for (int dy = 0; dy < 3; dy++)
#pragma unroll
			for (int dx = 0; dx < 3; dx++) s += tile[ty + dy][tx + dx];
		return s;
	};

	uint32_t s_prev, s_cur, c_cur;
	load_plane(z0 - 1);
	__syncthreads();
	s_prev = sum9();
	__syncthreads();
	load_plane(z0);
	__syncthreads();
	s_cur = sum9();
	c_cur = tile[ty + 1][tx + 1];
	__syncthreads();
	const bool active = x < nx && y < ny;
	for (int z = z0; z < z1; z++) {
		load_plane(z + 1);
		__syncthreads();
		const uint32_t s_next = sum9();
		const uint32_t c_next = tile[ty + 1][tx + 1];
		__syncthreads();
		if (active) {
			const uint32_t cnt = s_prev + s_cur + s_next - c_cur;
			const size_t idx = size_t(z) * plane + size_t(y) * nx + x;
			const uint32_t cur = st[idx];
			out[idx] = cnt == 3 ? 1u : (cnt == 2 ? cur : 0u);
		}
		s_prev = s_cur;
		s_cur = s_next;
		c_cur = c_next;
	}
}

// Barrier-free variant: a wavefront owns one x-run of 64 lanes (62 outputs,
// lanes 0 and 63 only feed their neighbors) on one y row and marches up z.
// Per plane each lane loads its column (y-1, y, y+1: three coalesced row
// loads, the outer two served from L1/L2 since neighboring waves load them
// as their own middle rows), the x-direction 3-sum comes from two lane
// shuffles, and the three in-plane sums of z-1, z, z+1 stay in registers.
constexpr int G2_OUT = 62, G2_ROWS = 4;

__global__ __launch_bounds__(64 * G2_ROWS) void gol_structured_v2(const uint32_t* __restrict__ st,
                                                                 uint32_t* __restrict__ out, int nx, int ny, int nz,
                                                                 int px, int py, int pz, int zc) {
	const int lane = threadIdx.x & 63;
	const int y = blockIdx.y * G2_ROWS + (threadIdx.x >> 6);
	if (y >= ny) return;  // wave-uniform
	const int x0 = blockIdx.x * G2_OUT;
	int x = x0 + lane - 1;
	bool xin = true;
	if (x < 0 || x >= nx) {
		if (px) x = ((x % nx) + nx) % nx;
		else xin = false;
	}
	int ym = y - 1, yp = y + 1;
	bool ymin = true, ypin = true;
	if (ym < 0) {
		if (py) ym += ny;
		else ymin = false;
	}
	if (yp >= ny) {
		if (py) yp -= ny;
		else ypin = false;
	}
	const size_t plane = size_t(nx) * ny;
	const size_t om = size_t(ym) * nx + x, oc = size_t(y) * nx + x, op = size_t(yp) * nx + x;
	// in-plane 3x3 sum at (x, y) of plane z and the raw center value
	auto plane_sum = [&](int z, uint32_t& center) -> uint32_t {
		bool zin = true;
		if (z < 0 || z >= nz) {
			if (pz) z = ((z % nz) + nz) % nz;
			else zin = false;
		}
		uint32_t c = 0;
		center = 0;
		if (zin && xin) {
			const uint32_t* p = st + size_t(z) * plane;
			center = p[oc];
			c = (center > 0) + (ymin ? (p[om] > 0) : 0u) + (ypin ? (p[op] > 0) : 0u);
		}
		const uint32_t l = __shfl_up(c, 1, 64), r = __shfl_down(c, 1, 64);
		return l + c + r;
	};
	const int z0 = blockIdx.z * zc;
	const int z1 = min(z0 + zc, nz);
	uint32_t dummy, cur;
	uint32_t s_prev = plane_sum(z0 - 1, dummy);
	uint32_t s_cur = plane_sum(z0, cur);
	const bool writer = lane >= 1 && lane <= G2_OUT && x0 + lane - 1 < nx;
	for (int z = z0; z < z1; z++) {
		uint32_t nxt;
		const uint32_t s_next = plane_sum(z + 1, nxt);
		if (writer) {
			const uint32_t cnt = s_prev + s_cur + s_next - (cur > 0 ? 1u : 0u);
			out[size_t(z) * plane + oc] = cnt == 3 ? 1u : (cnt == 2 ? cur : 0u);
		}
		s_prev = s_cur;
		s_cur = s_next;
		cur = nxt;
	}
}

// ---------------------------------------------------------------------------
// Advection (tests/advection/solve.hpp:44-279), fp64, fused flux + apply.
// Face entry = neighbor slot * 8 + dir (0..5 = -x,+x,-y,+y,-z,+z).  The flux
// through a face is evaluated with exactly the reference's expression and
// operand order (contraction off), so both sides of a face obtain bitwise
// the same value; only the order of the per-cell sum differs.
__global__ void advection_kernel(const double* __restrict__ rho, const double* __restrict__ vx,
                                 const double* __restrict__ vy, const double* __restrict__ vz,
                                 const double* __restrict__ lx, const double* __restrict__ ly,
                                 const double* __restrict__ lz, double* __restrict__ rho_out,
                                 const uint32_t* __restrict__ ptr, const int32_t* __restrict__ ent, size_t s0, size_t s1,
                                 double dt) {
#pragma clang fp contract(off)
	for (size_t s = s0 + blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < s1; s += size_t(gridDim.x) * blockDim.x) {
		const double cd = rho[s];
		const double clx = lx[s], cly = ly[s], clz = lz[s];
		const double cvx = vx[s], cvy = vy[s], cvz = vz[s];
		const double cv = clx * cly * clz;
		double acc = 0;
		const uint32_t e0 = ptr[s], e1 = ptr[s + 1];
		for (uint32_t e = e0; e < e1; e++) {
			const int32_t en = ent[e];
			const int32_t n = en >> 3;
			const int dir = en & 7;
			const double nd = rho[n];
			const double nlx = lx[n], nly = ly[n], nlz = lz[n];
			double min_area, v;
			if (dir < 2) {
				min_area = fmin(cly * clz, nly * nlz);
				v = (clx * vx[n] + nlx * cvx) / (clx + nlx);
			} else if (dir < 4) {
				min_area = fmin(clx * clz, nlx * nlz);
				v = (cly * vy[n] + nly * cvy) / (cly + nly);
			} else {
				min_area = fmin(clx * cly, nlx * nly);
				v = (clz * vz[n] + nlz * cvz) / (clz + nlz);
			}
			double flux;
			if (dir & 1) {  // positive direction
				flux = (v >= 0 ? cd : nd) * dt * v * min_area;
				acc -= flux / cv;
			} else {
				flux = (v >= 0 ? nd : cd) * dt * v * min_area;
				acc += flux / cv;
			}
		}
		rho_out[s] = cd + acc;
	}
}

// Same face flux, one thread per cell, no grid-stride: a workgroup maps to a
// contiguous run of slots, and the runs are dealt so that the 8 XCDs each
// sweep one contiguous eighth of the slot range (blocks b and b+8 share an
// XCD: logical block = (b % 8) * (nb / 8) + b / 8), keeping the z-neighbor
// planes of a chunk in that XCD's L2.  Faces are processed in batches of 4
// with all their gathers issued before any flux is evaluated, so a thread
// has up to 20 independent loads in flight instead of a dependent chain.
constexpr int ADV_BLOCK = 256;
constexpr int ADV_BATCH = 4;

__global__ __launch_bounds__(ADV_BLOCK) void advection_kernel_v1(
    const double* __restrict__ rho, const double* __restrict__ vx, const double* __restrict__ vy,
    const double* __restrict__ vz, const double* __restrict__ lx, const double* __restrict__ ly,
    const double* __restrict__ lz, double* __restrict__ rho_out, const uint32_t* __restrict__ ptr,
    const int32_t* __restrict__ ent, size_t s0, size_t s1, double dt, unsigned nb_real) {
#pragma clang fp contract(off)
	const unsigned nb = gridDim.x;  // multiple of 8
	const unsigned b = blockIdx.x;
	const unsigned lb = (b & 7u) * (nb >> 3) + (b >> 3);
	if (lb >= nb_real) return;
	const size_t s = s0 + size_t(lb) * ADV_BLOCK + threadIdx.x;
	if (s >= s1) return;
	const double cd = rho[s];
	const double clx = lx[s], cly = ly[s], clz = lz[s];
	const double cvx = vx[s], cvy = vy[s], cvz = vz[s];
	const double cv = clx * cly * clz;
	double acc = 0;
	const uint32_t e0 = ptr[s], e1 = ptr[s + 1];
	for (uint32_t e = e0; e < e1; e += ADV_BATCH) {
		int32_t en[ADV_BATCH];
		double nd[ADV_BATCH], nlx[ADV_BATCH], nly[ADV_BATCH], nlz[ADV_BATCH], nv[ADV_BATCH];
#pragma unroll
		for (int k = 0; k < ADV_BATCH; k++) en[k] = (e + k < e1) ? ent[e + k] : -1;
#pragma unroll
		for (int k = 0; k < ADV_BATCH; k++) {
			if (en[k] < 0) continue;
			const int32_t n = en[k] >> 3;
			const int dir = en[k] & 7;
			nd[k] = rho[n];
			nlx[k] = lx[n];
			nly[k] = ly[n];
			nlz[k] = lz[n];
			nv[k] = dir < 2 ? vx[n] : (dir < 4 ? vy[n] : vz[n]);
		}
#pragma unroll
		for (int k = 0; k < ADV_BATCH; k++) {
			if (en[k] < 0) continue;
			const int dir = en[k] & 7;
			double min_area, v;
			if (dir < 2) {
				min_area = fmin(cly * clz, nly[k] * nlz[k]);
				v = (clx * nv[k] + nlx[k] * cvx) / (clx + nlx[k]);
			} else if (dir < 4) {
				min_area = fmin(clx * clz, nlx[k] * nlz[k]);
				v = (cly * nv[k] + nly[k] * cvy) / (cly + nly[k]);
			} else {
				min_area = fmin(clx * cly, nlx[k] * nly[k]);
				v = (clz * nv[k] + nlz[k] * cvz) / (clz + nlz[k]);
			}
			double flux;
			if (dir & 1) {
				flux = (v >= 0 ? cd : nd[k]) * dt * v * min_area;
				acc -= flux / cv;
			} else {
				flux = (v >= 0 ? nd[k] : cd) * dt * v * min_area;
				acc += flux / cv;
			}
		}
	}
	rho_out[s] = cd + acc;
}

// Fixed-width face table (6 int32 per cell, see face_ell_kernel): the whole
// row is known after one load, so the 30 gathers of a cell's six regular
// faces are all issued before the first flux is evaluated (a missing face
// gathers the cell itself and is skipped).  Finer faces (4 cells) take a
// second dependent step through the overflow table.  Faces are accumulated
// in the reference's face order (dir -x,+x,-y,+y,-z,+z; the 4 finer cells in
// get_face_neighbors_of order), bitwise equal to advection_kernel.
__device__ __forceinline__ double adv_face(int dir, double cd, double clx, double cly, double clz, double cvx,
                                           double cvy, double cvz, double cv, double nd, double nlx, double nly,
                                           double nlz, double nv, double dt) {
#pragma clang fp contract(off)
	double min_area, v;
	if (dir < 2) {
		min_area = fmin(cly * clz, nly * nlz);
		v = (clx * nv + nlx * cvx) / (clx + nlx);
	} else if (dir < 4) {
		min_area = fmin(clx * clz, nlx * nlz);
		v = (cly * nv + nly * cvy) / (cly + nly);
	} else {
		min_area = fmin(clx * cly, nlx * nly);
		v = (clz * nv + nlz * cvz) / (clz + nlz);
	}
	if (dir & 1) return -(((v >= 0 ? cd : nd) * dt * v * min_area) / cv);
	return ((v >= 0 ? nd : cd) * dt * v * min_area) / cv;
}

__global__ __launch_bounds__(ADV_BLOCK) void advection_kernel_v2(
    const double* __restrict__ rho, const double* __restrict__ vx, const double* __restrict__ vy,
    const double* __restrict__ vz, const double* __restrict__ lx, const double* __restrict__ ly,
    const double* __restrict__ lz, double* __restrict__ rho_out, const int32_t* __restrict__ ell,
    const int32_t* __restrict__ fine, size_t s0, size_t s1, double dt, unsigned nb_real) {
#pragma clang fp contract(off)
	const unsigned nb = gridDim.x;
	const unsigned b = blockIdx.x;
	const unsigned lb = (b & 7u) * (nb >> 3) + (b >> 3);
	if (lb >= nb_real) return;
	const size_t s = s0 + size_t(lb) * ADV_BLOCK + threadIdx.x;
	if (s >= s1) return;
	int32_t row[6];
	{
		const int2* r2 = reinterpret_cast<const int2*>(ell + 6 * s);
		const int2 a = r2[0], bb = r2[1], c = r2[2];
		row[0] = a.x; row[1] = a.y; row[2] = bb.x; row[3] = bb.y; row[4] = c.x; row[5] = c.y;
	}
	const double cd = rho[s];
	const double clx = lx[s], cly = ly[s], clz = lz[s];
	const double cvx = vx[s], cvy = vy[s], cvz = vz[s];
	const double cv = clx * cly * clz;
	double nd[6], nlx[6], nly[6], nlz[6], nv[6];
#pragma unroll
	for (int d = 0; d < 6; d++) {
		const size_t n = row[d] >= 0 ? size_t(row[d]) : s;
		nd[d] = rho[n];
		nlx[d] = lx[n];
		nly[d] = ly[n];
		nlz[d] = lz[n];
		nv[d] = d < 2 ? vx[n] : (d < 4 ? vy[n] : vz[n]);
	}
	double acc = 0;
#pragma unroll
	for (int d = 0; d < 6; d++) {
		if (row[d] >= 0) {
			acc += adv_face(d, cd, clx, cly, clz, cvx, cvy, cvz, cv, nd[d], nlx[d], nly[d], nlz[d], nv[d], dt);
		} else if (row[d] <= -2) {
			const int4 q = reinterpret_cast<const int4*>(fine)[-2 - row[d]];
			const int32_t fs[4] = {q.x, q.y, q.z, q.w};
			double fd[4], fx[4], fy[4], fz[4], fv[4];
#pragma unroll
			for (int k = 0; k < 4; k++) {
				fd[k] = rho[fs[k]];
				fx[k] = lx[fs[k]];
				fy[k] = ly[fs[k]];
				fz[k] = lz[fs[k]];
				fv[k] = d < 2 ? vx[fs[k]] : (d < 4 ? vy[fs[k]] : vz[fs[k]]);
			}
#pragma unroll
			for (int k = 0; k < 4; k++)
				acc += adv_face(d, cd, clx, cly, clz, cvx, cvy, cvz, cv, fd[k], fx[k], fy[k], fz[k], fv[k], dt);
		}
	}
	rho_out[s] = cd + acc;
}

// LDS-staged variant: a workgroup sweeps ADV_TILE consecutive slots (a
// compact region of space: slots follow the Morton curve on refined grids)
// and first stages those cells' seven fields into LDS with coalesced loads
// (they are the cells' own reads, so no extra HBM traffic).  A face whose
// neighbor lies inside the tile is then served from LDS; only faces that
// leave the tile gather from L2/HBM.
template <int TILE, class F>
__device__ __forceinline__ void adv_fetch(size_t n, size_t base, size_t s1, const double (*sh)[TILE],
                                          const double* rho, const double* lx, const double* ly, const double* lz,
                                          const double* vdir, int dirv, double& nd, double& nlx, double& nly,
                                          double& nlz, double& nv, F) {
	const size_t k = n - base;
	if (k < size_t(TILE) && n < s1) {
		nd = sh[0][k];
		nlx = sh[4][k];
		nly = sh[5][k];
		nlz = sh[6][k];
		nv = sh[1 + dirv][k];
	} else {
		nd = rho[n];
		nlx = lx[n];
		nly = ly[n];
		nlz = lz[n];
		nv = vdir[n];
	}
}

template <int TILE, int MINW>
__global__ __launch_bounds__(TILE, MINW) void advection_kernel_v3(
    const double* __restrict__ rho, const double* __restrict__ vx, const double* __restrict__ vy,
    const double* __restrict__ vz, const double* __restrict__ lx, const double* __restrict__ ly,
    const double* __restrict__ lz, double* __restrict__ rho_out, const int32_t* __restrict__ ell,
    const int32_t* __restrict__ fine, size_t s0, size_t s1, double dt, unsigned nb_real) {
#pragma clang fp contract(off)
	__shared__ double sh[7][TILE];
	const unsigned nb = gridDim.x;
	const unsigned b = blockIdx.x;
	const unsigned lb = (b & 7u) * (nb >> 3) + (b >> 3);
	if (lb >= nb_real) return;  // block-uniform
	const size_t base = s0 + size_t(lb) * TILE;
	const size_t s = base + threadIdx.x;
	const bool valid = s < s1;
	double cd = 0, clx = 1, cly = 1, clz = 1, cvx = 0, cvy = 0, cvz = 0;
	int32_t row[6] = {-1, -1, -1, -1, -1, -1};
	if (valid) {
		const int2* r2 = reinterpret_cast<const int2*>(ell + 6 * s);
		const int2 a = r2[0], bb = r2[1], c = r2[2];
		row[0] = a.x; row[1] = a.y; row[2] = bb.x; row[3] = bb.y; row[4] = c.x; row[5] = c.y;
		cd = rho[s];
		cvx = vx[s];
		cvy = vy[s];
		cvz = vz[s];
		clx = lx[s];
		cly = ly[s];
		clz = lz[s];
	}
	sh[0][threadIdx.x] = cd;
	sh[1][threadIdx.x] = cvx;
	sh[2][threadIdx.x] = cvy;
	sh[3][threadIdx.x] = cvz;
	sh[4][threadIdx.x] = clx;
	sh[5][threadIdx.x] = cly;
	sh[6][threadIdx.x] = clz;
	__syncthreads();
	if (!valid) return;
	const double cv = clx * cly * clz;
	const double* vd[3] = {vx, vy, vz};
	double nd[6], nlx[6], nly[6], nlz[6], nv[6];
#pragma unroll
	for (int d = 0; d < 6; d++) {
		const size_t n = row[d] >= 0 ? size_t(row[d]) : s;
		adv_fetch(n, base, s1, sh, rho, lx, ly, lz, vd[d >> 1], d >> 1, nd[d], nlx[d], nly[d], nlz[d], nv[d], 0);
	}
	double acc = 0;
#pragma unroll
	for (int d = 0; d < 6; d++) {
		if (row[d] >= 0) {
			acc += adv_face(d, cd, clx, cly, clz, cvx, cvy, cvz, cv, nd[d], nlx[d], nly[d], nlz[d], nv[d], dt);
		} else if (row[d] <= -2) {
			const int4 q = reinterpret_cast<const int4*>(fine)[-2 - row[d]];
			const int32_t fs[4] = {q.x, q.y, q.z, q.w};
			double fd[4], fx[4], fy[4], fz[4], fv[4];
#pragma unroll
			for (int k = 0; k < 4; k++)
				adv_fetch(size_t(fs[k]), base, s1, sh, rho, lx, ly, lz, vd[d >> 1], d >> 1, fd[k], fx[k], fy[k], fz[k],
				          fv[k], 0);
#pragma unroll
			for (int k = 0; k < 4; k++)
				acc += adv_face(d, cd, clx, cly, clz, cvx, cvy, cvz, cv, fd[k], fx[k], fy[k], fz[k], fv[k], dt);
		}
	}
	rho_out[s] = cd + acc;
}

// max_time_step local part (solve.hpp:289-333): block minima
__global__ void adv_dt_kernel(const double* __restrict__ vx, const double* __restrict__ vy,
                              const double* __restrict__ vz, const double* __restrict__ lx,
                              const double* __restrict__ ly, const double* __restrict__ lz, size_t n,
                              double* partial) {
	__shared__ double red[256];
	double mn = 1.7976931348623157e308;
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const double a = lx[s] / fabs(vx[s]), b = ly[s] / fabs(vy[s]), c = lz[s] / fabs(vz[s]);
		if (__builtin_isnormal(a)) mn = fmin(mn, a);
		if (__builtin_isnormal(b)) mn = fmin(mn, b);
		if (__builtin_isnormal(c)) mn = fmin(mn, c);
	}
	red[threadIdx.x] = mn;
	__syncthreads();
	for (int k = blockDim.x / 2; k > 0; k >>= 1) {
		if (threadIdx.x < k) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + k]);
		__syncthreads();
	}
	if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// refine decisions of check_for_adaptation (tests/advection/adapter.hpp:47-178):
// max relative density difference over face neighbors whose transverse
// offsets are zero (adapter.hpp:74-96), threshold (lvl+1)*diff_increase
__global__ void adv_candidates_kernel(MapCtx m, const double* __restrict__ rho, const uint32_t* __restrict__ ptr,
                                      const int32_t* __restrict__ ent, const uint64_t* __restrict__ slot_ids, size_t n,
                                      double diff_increase, double diff_threshold, uint64_t* out,
                                      unsigned long long* counter) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		uint64_t c[3];
		const int lvl = map_indices(m, slot_ids[s], c[0], c[1], c[2]);
		const uint64_t len = uint64_t(1) << (m.R - lvl);
		double md = 0;
		const uint32_t e0 = ptr[s], e1 = ptr[s + 1];
		for (uint32_t e = e0; e < e1; e++) {
			const int32_t en = ent[e];
			const int32_t nsl = en >> 3;
			const int d = (en & 7) >> 1;
			const int nl = map_level(m, slot_ids[nsl]);
			bool zero = true;
			if (nl > lvl) {
				// finer: only the first of the four face cells sits at the cell's corner
				zero = (e == e0 || ((ent[e - 1] & 7) != (en & 7))) ;
			} else if (nl < lvl) {
				const uint64_t pl = len * 2;
				for (int k = 0; k < 3; k++)
					if (k != d && (c[k] & (pl - 1)) != 0) zero = false;
			}
			if (!zero) continue;
			const double a = rho[s], b = rho[nsl];
			const double diff = fabs(a - b) / (fmin(a, b) + diff_threshold);
			md = fmax(diff, md);
		}
		if (md > (lvl + 1) * diff_increase) out[atomicAdd(counter, 1ull)] = slot_ids[s];
	}
}

}  // namespace

// ===========================================================================
void k_pack(const uint8_t* field, size_t elem, const int32_t* slots, size_t n, uint8_t* out, hipStream_t s) {
	if (!n) return;
	if (elem == 4)
		pack_kernel<uint32_t><<<grid_for(n, 256), 256, 0, s>>>((const uint32_t*)field, slots, n, (uint32_t*)out);
	else if (elem == 8)
		pack_kernel<uint64_t><<<grid_for(n, 256), 256, 0, s>>>((const uint64_t*)field, slots, n, (uint64_t*)out);
	else
		pack_bytes_kernel<<<grid_for(n * elem, 256), 256, 0, s>>>(field, elem, slots, n, out);
	HIP_CHECK(hipGetLastError());
}

void k_gol_csr(const uint32_t* state, uint32_t* out, const uint32_t* it_ptr, const int32_t* it_slot, size_t s0,
               size_t s1, hipStream_t s) {
	if (s1 <= s0) return;
	gol_csr_kernel<<<grid_for(s1 - s0, 256), 256, 0, s>>>(state, out, it_ptr, it_slot, s0, s1);
	HIP_CHECK(hipGetLastError());
}

void k_gol_structured(const uint32_t* state, uint32_t* out, const uint64_t n[3], const int per[3], hipStream_t s) {
	static const int variant = [] {
		const char* e = getenv("DCCRGX_GOL_VARIANT");
		return e ? atoi(e) : 2;
	}();
	if (variant == 2) {
		const int zc = int(n[2] <= 64 ? n[2] : 64);
		dim3 g2(unsigned((n[0] + G2_OUT - 1) / G2_OUT), unsigned((n[1] + G2_ROWS - 1) / G2_ROWS),
		        unsigned((n[2] + zc - 1) / zc));
		gol_structured_v2<<<g2, 64 * G2_ROWS, 0, s>>>(state, out, int(n[0]), int(n[1]), int(n[2]), per[0], per[1],
		                                               per[2], zc);
		HIP_CHECK(hipGetLastError());
		return;
	}
	dim3 grid(unsigned((n[0] + GTX - 1) / GTX), unsigned((n[1] + GTY - 1) / GTY), unsigned((n[2] + GZC - 1) / GZC));
	gol_structured_kernel<<<grid, GTX * GTY, 0, s>>>(state, out, int(n[0]), int(n[1]), int(n[2]), per[0], per[1],
	                                                  per[2]);
	HIP_CHECK(hipGetLastError());
}

int adv_variant() {
	static int v = [] {
		const char* e = getenv("DCCRGX_ADV_VARIANT");
		return e ? atoi(e) : 3;
	}();
	return v;
}

void k_advection(const double* const f[7], double* rho_out, const uint32_t* face_ptr, const int32_t* face_ent,
                 const int32_t* face_ell, const int32_t* face_fine, size_t s0, size_t s1, double dt, hipStream_t s) {
	if (s1 <= s0) return;
	if (adv_variant() >= 3) {
		const int tile = adv_variant() == 4 ? 256 : 512;
		const size_t nb_real = (s1 - s0 + tile - 1) / tile;
		const size_t nb = (nb_real + 7) / 8 * 8;
		if (adv_variant() == 3)
			advection_kernel_v3<512, 4><<<unsigned(nb), 512, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out,
			                                                           face_ell, face_fine, s0, s1, dt, unsigned(nb_real));
		else if (adv_variant() == 4)
			advection_kernel_v3<256, 4><<<unsigned(nb), 256, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out,
			                                                           face_ell, face_fine, s0, s1, dt, unsigned(nb_real));
		else
			advection_kernel_v3<1024, 4><<<unsigned((( (s1 - s0 + 1023) / 1024) + 7) / 8 * 8), 1024, 0, s>>>(
			    f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out, face_ell, face_fine, s0, s1, dt,
			    unsigned((s1 - s0 + 1023) / 1024));
	} else if (adv_variant() == 2) {
		const size_t nb_real = (s1 - s0 + ADV_BLOCK - 1) / ADV_BLOCK;
		const size_t nb = (nb_real + 7) / 8 * 8;
		advection_kernel_v2<<<unsigned(nb), ADV_BLOCK, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out,
		                                                       face_ell, face_fine, s0, s1, dt, unsigned(nb_real));
	} else if (adv_variant() == 0) {
		advection_kernel<<<grid_for(s1 - s0, 256), 256, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out,
		                                                        face_ptr, face_ent, s0, s1, dt);
	} else {
		const size_t nb_real = (s1 - s0 + ADV_BLOCK - 1) / ADV_BLOCK;
		const size_t nb = (nb_real + 7) / 8 * 8;
		advection_kernel_v1<<<unsigned(nb), ADV_BLOCK, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out,
		                                                       face_ptr, face_ent, s0, s1, dt, unsigned(nb_real));
	}
	HIP_CHECK(hipGetLastError());
}

void k_adv_dt(const double* const f[7], size_t n, double* partial, size_t nblocks, hipStream_t s) {
	adv_dt_kernel<<<unsigned(nblocks), 256, 0, s>>>(f[1], f[2], f[3], f[4], f[5], f[6], n, partial);
	HIP_CHECK(hipGetLastError());
}

size_t k_adv_candidates(const MapCtx& m, const double* rho, const uint32_t* face_ptr, const int32_t* face_ent,
                        const uint64_t* slot_ids, size_t n, double diff_increase, double diff_threshold,
                        uint64_t* out, hipStream_t s) {
	if (!n) return 0;
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, sizeof(unsigned long long), s));
	adv_candidates_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, rho, face_ptr, face_ent, slot_ids, n, diff_increase,
	                                                       diff_threshold, out, ctr.p);
	HIP_CHECK(hipGetLastError());
	unsigned long long h = 0;
	HIP_CHECK(hipMemcpyAsync(&h, ctr.p, sizeof(h), hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
	return size_t(h);
}

}  // namespace dccrgx
