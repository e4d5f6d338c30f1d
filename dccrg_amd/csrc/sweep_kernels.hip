// Stencil sweeps over local cells and remote-neighbor copies, plus the halo
// pack.  These replace the user loops of the reference's tests/examples:
//   game of life  examples/game_of_life.cpp:54-79,
//                 tests/game_of_life/scalability3d.cpp:130-165
//   advection     tests/advection/solve.hpp:44-279 (calculate_fluxes +
//                 apply_fluxes fused: every cell gathers its own faces, so
//                 the reference's scatter into two cells becomes a race-free
//                 gather with no atomics)
// All bandwidth-bound; no MFMA.
#include <cstring>
#include <cstdlib>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

// ---------------------------------------------------------------------------
// halo pack / place: bytes [off, off + len) of the elements at `slots`
template <class T>
__global__ void pack_kernel(const T* __restrict__ f, const int32_t* __restrict__ slots, size_t n, T* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		out[i] = f[slots[i]];
}

template <class T>
__global__ void place_kernel(const T* __restrict__ in, const int32_t* __restrict__ slots, size_t n, T* __restrict__ f) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		f[slots[i]] = in[i];
}

__global__ void pack_bytes_kernel(const uint8_t* __restrict__ f, size_t elem, size_t off, size_t len,
                                  const int32_t* __restrict__ slots, size_t n, uint8_t* __restrict__ out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n * len; i += size_t(gridDim.x) * blockDim.x) {
		const size_t k = i / len, b = i - k * len;
		out[i] = f[size_t(slots[k]) * elem + off + b];
	}
}

__global__ void place_bytes_kernel(const uint8_t* __restrict__ in, size_t elem, size_t off, size_t len,
                                   const int32_t* __restrict__ slots, size_t n, uint8_t* __restrict__ f) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n * len; i += size_t(gridDim.x) * blockDim.x) {
		const size_t k = i / len, b = i - k * len;
		f[size_t(slots[k]) * elem + off + b] = in[i];
	}
}

// ---------------------------------------------------------------------------
// Game of life over the iterator neighbor list (deduplicated neighbors_of),
// for refined meshes and partitions the structured kernel cannot take.  One
// block per 256 consecutive rows: phase 1 reads the block's entries (one
// contiguous run of the CSR) coalesced, four per thread and word, and
// gathers their states eight in flight per thread into one LDS byte each;
// phase 2 sums each row from LDS (rows past the LDS window gather directly).
// Blocks are dealt XCD-contiguously (block b runs on XCD b % 8), so the rows
// whose states a block gathers were loaded into the same L2.
constexpr int kGolRows = 256;
__global__ __launch_bounds__(kGolRows) void gol_csr_kernel(const uint32_t* __restrict__ state,
                                                         uint32_t* __restrict__ out, const uint32_t* __restrict__ ptr,
                                                         const int32_t* __restrict__ nb, size_t s0, size_t s1) {
	constexpr uint32_t cap = 8192;  // entry bytes staged per block
	__shared__ uint32_t sp32[cap / 4];
	const uint32_t tid = threadIdx.x;
	const uint32_t lb = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
	const size_t r0 = s0 + size_t(lb) * kGolRows;
	if (r0 >= s1) return;  // block-uniform
	const size_t r1 = r0 + kGolRows < s1 ? r0 + kGolRows : s1;
	const uint32_t E0 = ptr[r0] & ~3u, E1 = ptr[r1];
	const uint32_t nB = E1 - E0 < cap ? E1 - E0 : cap;
	const uint32_t nw = (nB + 3) / 4;
	for (uint32_t w = tid; w < nw; w += 2 * kGolRows) {
		int32_t q[8];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const uint32_t e = E0 + 4 * (w + (k >> 2) * kGolRows) + (k & 3);
			q[k] = e >= E0 + 4 * nw || e >= E1 ? -1 : nb[e];
		}
		uint32_t v[8];
#pragma unroll
		for (int k = 0; k < 8; k++) v[k] = q[k] >= 0 && state[q[k]] > 0 ? 1u : 0u;
		sp32[w] = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
		if (w + kGolRows < nw) sp32[w + kGolRows] = v[4] | (v[5] << 8) | (v[6] << 16) | (v[7] << 24);
	}
	__syncthreads();
	const size_t s = r0 + tid;
	if (s >= r1) return;
	const uint8_t* sp8 = reinterpret_cast<const uint8_t*>(sp32);
	uint32_t cnt = 0;
	for (uint32_t j = ptr[s], e = ptr[s + 1]; j < e; j++)
		cnt += j - E0 < nB ? sp8[j - E0] : (state[nb[j]] > 0 ? 1u : 0u);
	const uint32_t cur = state[s];
	out[s] = cnt == 3 ? 1u : (cnt == 2 ? cur : 0u);
}

// Uniform 26-point game of life (nx a multiple of 256): a lane owns 4 consecutive x (16-B loads and
// stores), a wave one 256-x segment of one y row, a block G3_ROWS
// consecutive rows of the same segment; each wave marches a chunk of zc
// planes with the raw loads of the next DEPTH planes in flight while the
// current one is summed (8 B per cell-update, the y+-1 rows
// and the segment-edge columns are re-reads served by L2).  Blocks are
// dealt to XCDs in contiguous runs of the (x segment, y, z chunk) order, so
// the rows shared by vertically adjacent blocks stay in one XCD's L2.
#ifndef DCCRGX_G3_ROWS
#define DCCRGX_G3_ROWS 4
#endif
#ifndef DCCRGX_G3_DEPTH
#define DCCRGX_G3_DEPTH 3
#endif
constexpr int G3_ROWS = DCCRGX_G3_ROWS;

struct G3Plane {
	uint4 m, c, p;  // rows y-1, y, y+1 at this lane's 4 x
	uint32_t e[3];  // lane 0: column x0-1, lane 63: column x0+256 (rows y-1, y, y+1)
};

template <int DEPTH>
__global__ __launch_bounds__(64 * G3_ROWS) void gol_structured_v3(const uint32_t* __restrict__ st,
                                                                 uint32_t* __restrict__ out, int nx, int ny, int nz,
                                                                 int px, int py, int pz, int zc, unsigned nbx,
                                                                 unsigned nby, unsigned nb,
                                                                 const uint32_t* __restrict__ lo,
                                                                 const uint32_t* __restrict__ hi) {
	const unsigned per_xcd = gridDim.x >> 3;
	const unsigned L = (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3);
	if (L >= nb) return;  // block-uniform
	const unsigned bx = L % nbx, r = L / nbx, by = r % nby, bz = r / nby;
	const int lane = threadIdx.x & 63;
	const int y = int(by) * G3_ROWS + (threadIdx.x >> 6);
	if (y >= ny) return;  // wave-uniform
	const int x0 = int(bx) * 256;
	const int x = x0 + 4 * lane;
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
	// the edge column of lane 0 (left) / lane 63 (right), -1 when outside
	int xe = -1;
	if (lane == 0) xe = x0 > 0 ? x0 - 1 : (px ? nx - 1 : -1);
	if (lane == 63) xe = x0 + 256 < nx ? x0 + 256 : (px ? 0 : -1);
	const size_t plane = size_t(nx) * ny;
	const size_t om = size_t(ym) * nx, oc = size_t(y) * nx, op = size_t(yp) * nx;
	auto load = [&](int z, G3Plane& P) {
		P.m = P.c = P.p = make_uint4(0, 0, 0, 0);
		P.e[0] = P.e[1] = P.e[2] = 0;
		// planes z = -1 / nz: the lo / hi plane (another slab's copy), the
		// periodic wrap, or nothing
		const uint32_t* p;
		if (z < 0) p = lo ? lo : (pz ? st + size_t(z + nz) * plane : nullptr);
		else if (z >= nz) p = hi ? hi : (pz ? st + size_t(z - nz) * plane : nullptr);
		else p = st + size_t(z) * plane;
		if (!p) return;
		P.c = *reinterpret_cast<const uint4*>(p + oc + x);
		if (ymin) P.m = *reinterpret_cast<const uint4*>(p + om + x);
		if (ypin) P.p = *reinterpret_cast<const uint4*>(p + op + x);
		if (xe >= 0) {
			P.e[1] = p[oc + xe];
			if (ymin) P.e[0] = p[om + xe];
			if (ypin) P.e[2] = p[op + xe];
		}
	};
	// the in-plane 3x3 sums at this lane's 4 x
	auto psum = [&](const G3Plane& P, uint32_t s[4]) {
		const uint32_t c0 = (P.m.x > 0) + (P.c.x > 0) + (P.p.x > 0), c1 = (P.m.y > 0) + (P.c.y > 0) + (P.p.y > 0),
		               c2 = (P.m.z > 0) + (P.c.z > 0) + (P.p.z > 0), c3 = (P.m.w > 0) + (P.c.w > 0) + (P.p.w > 0);
		const uint32_t ce = (P.e[0] > 0) + (P.e[1] > 0) + (P.e[2] > 0);
		uint32_t l = __shfl_up(c3, 1, 64), rr = __shfl_down(c0, 1, 64);
		if (lane == 0) l = ce;
		if (lane == 63) rr = ce;
		s[0] = l + c0 + c1;
		s[1] = c0 + c1 + c2;
		s[2] = c1 + c2 + c3;
		s[3] = c2 + c3 + rr;
	};
	const int z0 = int(bz) * zc;
	const int z1 = min(z0 + zc, nz);
	// Q[i] holds the raw loads of plane z + 1 + i (DEPTH planes in flight)
	G3Plane A, B, Q[DEPTH];
	load(z0 - 1, A);
	load(z0, B);
#pragma unroll
	for (int i = 0; i < DEPTH; i++)
		if (z0 + 1 + i <= z1) load(z0 + 1 + i, Q[i]);
	uint32_t sp[4], sc[4], sn[4];
	psum(A, sp);
	psum(B, sc);
	uint4 cur = B.c;
	for (int z = z0; z < z1; z++) {
		G3Plane E = Q[DEPTH - 1];
		if (z + 1 + DEPTH <= z1) load(z + 1 + DEPTH, E);
		psum(Q[0], sn);
		uint4 o;
		uint32_t cnt;
		cnt = sp[0] + sc[0] + sn[0] - (cur.x > 0);
		o.x = cnt == 3 ? 1u : (cnt == 2 ? cur.x : 0u);
		cnt = sp[1] + sc[1] + sn[1] - (cur.y > 0);
		o.y = cnt == 3 ? 1u : (cnt == 2 ? cur.y : 0u);
		cnt = sp[2] + sc[2] + sn[2] - (cur.z > 0);
		o.z = cnt == 3 ? 1u : (cnt == 2 ? cur.z : 0u);
		cnt = sp[3] + sc[3] + sn[3] - (cur.w > 0);
		o.w = cnt == 3 ? 1u : (cnt == 2 ? cur.w : 0u);
		// streaming store: the next state is not read again in this sweep, so
		// keeping it out of L2 leaves room for the three planes in flight
		// (paired A/B on config 2: 0.113 -> 0.108 ms per sweep)
		{
			typedef unsigned int u4v __attribute__((ext_vector_type(4)));
			u4v ov = {o.x, o.y, o.z, o.w};
			__builtin_nontemporal_store(ov, reinterpret_cast<u4v*>(out + size_t(z) * plane + oc + x));
		}
#pragma unroll
		for (int i = 0; i < 4; i++) {
			sp[i] = sc[i];
			sc[i] = sn[i];
		}
		cur = Q[0].c;
#pragma unroll
		for (int i = 0; i + 1 < DEPTH; i++) Q[i] = Q[i + 1];
		Q[DEPTH - 1] = E;
	}
}

// gol_structured_v3 with YR consecutive y rows per wave (YR = 2 the default,
// DCCRGX_GOL_YR=4 / 1 for A/Bs): a plane's YR + 2 rows are loaded once per wave for YR output
// rows (v3: 3 row loads per output row), so the L2 reads of the y+-1 rows
// drop from 12 B to 4 (YR + 2) / YR B per cell.  Same sums, same states.
template <int DEPTH, int YR>
__global__ __launch_bounds__(64 * G3_ROWS) void gol_structured_yr(const uint32_t* __restrict__ st,
                                                                 uint32_t* __restrict__ out, int nx, int ny, int nz,
                                                                 int px, int py, int pz, int zc, unsigned nbx,
                                                                 unsigned nby, unsigned nb,
                                                                 const uint32_t* __restrict__ lo,
                                                                 const uint32_t* __restrict__ hi) {
	constexpr int NR = YR + 2;
	const unsigned per_xcd = gridDim.x >> 3;
	const unsigned L = (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3);
	if (L >= nb) return;  // block-uniform
	const unsigned bx = L % nbx, r = L / nbx, by = r % nby, bz = r / nby;
	const int lane = threadIdx.x & 63;
	const int y0 = (int(by) * G3_ROWS + int(threadIdx.x >> 6)) * YR;
	if (y0 >= ny) return;  // wave-uniform
	const int x0 = int(bx) * 256;
	const int x = x0 + 4 * lane;
	// row i of a plane is y0 - 1 + i, wrapped or absent (-1)
	size_t orow[NR];
	bool rin[NR];
#pragma unroll
	for (int i = 0; i < NR; i++) {
		int y = y0 - 1 + i;
		bool in = true;
		if (y < 0) {
			if (py) y += ny;
			else in = false;
		} else if (y >= ny) {
			if (py) y -= ny;
			else in = false;
		}
		rin[i] = in;
		orow[i] = in ? size_t(y) * nx : 0;
	}
	int xe = -1;
	if (lane == 0) xe = x0 > 0 ? x0 - 1 : (px ? nx - 1 : -1);
	if (lane == 63) xe = x0 + 256 < nx ? x0 + 256 : (px ? 0 : -1);
	const size_t plane = size_t(nx) * ny;
	struct P {
		uint4 v[NR];
		uint32_t e[NR];
	};
	auto load = [&](int z, P& Q) {
#pragma unroll
		for (int i = 0; i < NR; i++) {
			Q.v[i] = make_uint4(0, 0, 0, 0);
			Q.e[i] = 0;
		}
		const uint32_t* p;
		if (z < 0) p = lo ? lo : (pz ? st + size_t(z + nz) * plane : nullptr);
		else if (z >= nz) p = hi ? hi : (pz ? st + size_t(z - nz) * plane : nullptr);
		else p = st + size_t(z) * plane;
		if (!p) return;
#pragma unroll
		for (int i = 0; i < NR; i++)
			if (rin[i]) Q.v[i] = *reinterpret_cast<const uint4*>(p + orow[i] + x);
		if (xe >= 0) {
#pragma unroll
			for (int i = 0; i < NR; i++)
				if (rin[i]) Q.e[i] = p[orow[i] + xe];
		}
	};
	// per output row k the in-plane 3x3 sums at this lane's 4 x
	auto psum = [&](const P& Q, uint32_t s[YR][4]) {
		uint32_t c[NR][4], ce[NR];
#pragma unroll
		for (int i = 0; i < NR; i++) {
			c[i][0] = Q.v[i].x > 0;
			c[i][1] = Q.v[i].y > 0;
			c[i][2] = Q.v[i].z > 0;
			c[i][3] = Q.v[i].w > 0;
			ce[i] = Q.e[i] > 0;
		}
#pragma unroll
		for (int k = 0; k < YR; k++) {
			const uint32_t c0 = c[k][0] + c[k + 1][0] + c[k + 2][0], c1 = c[k][1] + c[k + 1][1] + c[k + 2][1],
			               c2 = c[k][2] + c[k + 1][2] + c[k + 2][2], c3 = c[k][3] + c[k + 1][3] + c[k + 2][3];
			const uint32_t cee = ce[k] + ce[k + 1] + ce[k + 2];
			uint32_t l = __shfl_up(c3, 1, 64), rr = __shfl_down(c0, 1, 64);
			if (lane == 0) l = cee;
			if (lane == 63) rr = cee;
			s[k][0] = l + c0 + c1;
			s[k][1] = c0 + c1 + c2;
			s[k][2] = c1 + c2 + c3;
			s[k][3] = c2 + c3 + rr;
		}
	};
	const int z0 = int(bz) * zc;
	const int z1 = min(z0 + zc, nz);
	P A, Q[DEPTH];
	uint32_t sp[YR][4], sc[YR][4], sn[YR][4];
	uint4 cur[YR];
	load(z0 - 1, A);
	psum(A, sp);
	load(z0, A);
	psum(A, sc);
#pragma unroll
	for (int k = 0; k < YR; k++) cur[k] = A.v[k + 1];
#pragma unroll
	for (int i = 0; i < DEPTH; i++)
		if (z0 + 1 + i <= z1) load(z0 + 1 + i, Q[i]);
	for (int z = z0; z < z1; z++) {
		P E = Q[DEPTH - 1];
		if (z + 1 + DEPTH <= z1) load(z + 1 + DEPTH, E);
		psum(Q[0], sn);
#pragma unroll
		for (int k = 0; k < YR; k++) {
			if (y0 + k >= ny) continue;
			uint4 o;
			uint32_t cnt;
			cnt = sp[k][0] + sc[k][0] + sn[k][0] - (cur[k].x > 0);
			o.x = cnt == 3 ? 1u : (cnt == 2 ? cur[k].x : 0u);
			cnt = sp[k][1] + sc[k][1] + sn[k][1] - (cur[k].y > 0);
			o.y = cnt == 3 ? 1u : (cnt == 2 ? cur[k].y : 0u);
			cnt = sp[k][2] + sc[k][2] + sn[k][2] - (cur[k].z > 0);
			o.z = cnt == 3 ? 1u : (cnt == 2 ? cur[k].z : 0u);
			cnt = sp[k][3] + sc[k][3] + sn[k][3] - (cur[k].w > 0);
			o.w = cnt == 3 ? 1u : (cnt == 2 ? cur[k].w : 0u);
			typedef unsigned int u4v __attribute__((ext_vector_type(4)));
			u4v ov = {o.x, o.y, o.z, o.w};
			__builtin_nontemporal_store(ov, reinterpret_cast<u4v*>(out + size_t(z) * plane + size_t(y0 + k) * nx + x));
		}
#pragma unroll
		for (int k = 0; k < YR; k++) {
#pragma unroll
			for (int i = 0; i < 4; i++) {
				sp[k][i] = sc[k][i];
				sc[k][i] = sn[k][i];
			}
			cur[k] = Q[0].v[k + 1];
		}
#pragma unroll
		for (int i = 0; i + 1 < DEPTH; i++) Q[i] = Q[i + 1];
		Q[DEPTH - 1] = E;
	}
}

// ---------------------------------------------------------------------------
// Face flux without the division by the cell volume (applied once per cell):
// the face velocity and the upwind flux keep the reference's expression
// (solve.hpp:169-225), so only the per-cell rounding of the sum differs.
__device__ __forceinline__ double adv_face_flux(int dir, double cd, double cl_a, double cl_b, double cl_c,
                                                double cvel, double nd, double nl_a, double nl_b, double nl_c,
                                                double nv, double dt) {
#pragma clang fp contract(off)
	// cl_a = the cell's length along the face normal, cl_b/cl_c transverse
	const double min_area = fmin(cl_b * cl_c, nl_b * nl_c);
	const double v = (cl_a * nv + nl_a * cvel) / (cl_a + nl_a);
	if (dir & 1) return -((v >= 0 ? cd : nd) * dt * v * min_area);
	return (v >= 0 ? nd : cd) * dt * v * min_area;
}

struct AdvNb {
	double d, lx, ly, lz, v;
};

__device__ __forceinline__ double adv_face_flux_d(int d, double cd, double clx, double cly, double clz, double cvx,
                                                  double cvy, double cvz, const AdvNb& n, double dt) {
	if (d < 2) return adv_face_flux(d, cd, clx, cly, clz, cvx, n.d, n.lx, n.ly, n.lz, n.v, dt);
	if (d < 4) return adv_face_flux(d, cd, cly, clx, clz, cvy, n.d, n.ly, n.lx, n.lz, n.v, dt);
	return adv_face_flux(d, cd, clz, clx, cly, cvz, n.d, n.lz, n.lx, n.ly, n.v, dt);
}

// Advection (tests/advection/solve.hpp:44-279), fp64, fused flux + apply,
// for runs the tile sweeps cannot take (tiles beyond the LDS capacity).
// Face entry = neighbor slot * 8 + dir (0..5 = -x,+x,-y,+y,-z,+z).  Every
// face flux is the tile sweeps' (the reference's expression and operand
// order, contraction off) and they are summed in the same face order and
// divided once by the cell volume, so a cell's new density is bitwise the
// same whichever sweep computes it.
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
		double acc = 0;
		const uint32_t e0 = ptr[s], e1 = ptr[s + 1];
		for (uint32_t e = e0; e < e1; e++) {
			const int32_t en = ent[e];
			const int32_t n = en >> 3;
			const int dir = en & 7;
			const double nv = dir < 2 ? vx[n] : (dir < 4 ? vy[n] : vz[n]);
			acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, AdvNb{rho[n], lx[n], ly[n], lz[n], nv}, dt);
		}
		rho_out[s] = cd + acc / (clx * cly * clz);
	}
}

// The same sweep over the fixed-width face table of ensure_face
// (face_table_kernel: ell[6 r + d] = the neighbor's slot, -1 none, -2 - f the
// four finer neighbors fine[4 f ..] in the reference's order): the sweep of a
// mesh that has just changed, before (and instead of) building its tiles.
// One thread per cell, the row's six codes as three 8-B loads, the same face
// fluxes summed in the same face order as advection_kernel and the tile
// sweeps, so the new density is bitwise theirs.
__global__ __launch_bounds__(256) void advection_ell_kernel(const double* __restrict__ rho, const double* __restrict__ vx,
                                                            const double* __restrict__ vy, const double* __restrict__ vz,
                                                            const double* __restrict__ lx, const double* __restrict__ ly,
                                                            const double* __restrict__ lz, double* __restrict__ rho_out,
                                                            const int32_t* __restrict__ ell,
                                                            const int32_t* __restrict__ fine, size_t s0, size_t s1,
                                                            double dt) {
#pragma clang fp contract(off)
	typedef int i2v __attribute__((ext_vector_type(2)));
	typedef int i4v __attribute__((ext_vector_type(4)));
	for (size_t s = s0 + blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < s1; s += size_t(gridDim.x) * blockDim.x) {
		const double cd = rho[s];
		const double clx = lx[s], cly = ly[s], clz = lz[s];
		const double cvx = vx[s], cvy = vy[s], cvz = vz[s];
		int32_t e6[6];
		const i2v* ev = reinterpret_cast<const i2v*>(ell + 6 * s);
#pragma unroll
		for (int j = 0; j < 3; j++) {
			const i2v v = ev[j];
			e6[2 * j] = v.x;
			e6[2 * j + 1] = v.y;
		}
		auto nb = [&](int32_t n, int dir) {
			const double nv = dir < 2 ? vx[n] : (dir < 4 ? vy[n] : vz[n]);
			return AdvNb{rho[n], lx[n], ly[n], lz[n], nv};
		};
		double acc = 0;
#pragma unroll
		for (int dir = 0; dir < 6; dir++) {
			const int32_t c = e6[dir];
			if (c == -1) continue;
			if (c >= 0) {
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(c, dir), dt);
			} else {
				const i4v q = *reinterpret_cast<const i4v*>(fine + 4 * size_t(-2 - c));
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.x, dir), dt);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.y, dir), dt);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.z, dir), dt);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.w, dir), dt);
			}
		}
		rho_out[s] = cd + acc / (clx * cly * clz);
	}
}

// advection_ell_kernel with the block's own 256 cells staged in LDS: a
// block sweeps 256 consecutive slots (Morton order: a compact box, where
// about five in six face neighbors are cells of the same block), reads its
// cells' seven values once, coalesced, and takes every neighbor inside the
// block from LDS; the others are gathered as before.  The same values in the
// same order: bitwise the densities of advection_ell_kernel.
// BANDS: check_for_adaptation's band of every swept cell as well (the
// densities it compares are the ones the sweep reads): adv_max_diff's
// comparisons in its order - a coarser single neighbor only from the corner
// of its face, of a finer face only the first cell - and adv_bands_kernel's
// thresholds, so the bytes are that kernel's.
template <bool BANDS>
__global__ __launch_bounds__(256) void advection_ell_lds_kernel(
    const double* __restrict__ rho, const double* __restrict__ vx, const double* __restrict__ vy,
    const double* __restrict__ vz, const double* __restrict__ lx, const double* __restrict__ ly,
    const double* __restrict__ lz, double* __restrict__ rho_out, const int32_t* __restrict__ ell,
    const int32_t* __restrict__ fine, size_t s0, size_t s1, double dt, BandArgs B) {
#pragma clang fp contract(off)
	typedef int i2v __attribute__((ext_vector_type(2)));
	typedef int i4v __attribute__((ext_vector_type(4)));
	__shared__ double sd[256], svx[256], svy[256], svz[256], slx[256], sly[256], slz[256];
	__shared__ uint8_t slv[BANDS ? 256 : 1];
	const unsigned t = threadIdx.x;
	for (size_t b0 = s0 + blockIdx.x * size_t(256); b0 < s1; b0 += size_t(gridDim.x) * 256) {
		const size_t s = b0 + t;
		const bool live = s < s1;
		const uint32_t nb_in = uint32_t(min(size_t(256), s1 - b0));
		double cd = 0, clx = 1, cly = 1, clz = 1, cvx = 0, cvy = 0, cvz = 0;
		int32_t e6[6] = {-1, -1, -1, -1, -1, -1};
		int lvl = 0;
		unsigned oct = 0;
		if (live) {
			cd = rho[s];
			clx = lx[s];
			cly = ly[s];
			clz = lz[s];
			cvx = vx[s];
			cvy = vy[s];
			cvz = vz[s];
			if (BANDS) {
				const unsigned v = B.lvl8[s];
				lvl = int(v & 31u);
				oct = v >> 5;
			}
			const i2v* ev = reinterpret_cast<const i2v*>(ell + 6 * s);
#pragma unroll
			for (int j = 0; j < 3; j++) {
				const i2v v = ev[j];
				e6[2 * j] = v.x;
				e6[2 * j + 1] = v.y;
			}
		}
		__syncthreads();  // the previous chunk's readers are done with LDS
		sd[t] = cd;
		svx[t] = cvx;
		svy[t] = cvy;
		svz[t] = cvz;
		slx[t] = clx;
		sly[t] = cly;
		slz[t] = clz;
		if (BANDS) slv[t] = uint8_t(lvl);
		__syncthreads();
		if (!live) continue;
		auto nb = [&](int32_t n, int dir) {
			const uint32_t k = uint32_t(int64_t(n) - int64_t(b0));
			if (k < nb_in) {
				const double nv = dir < 2 ? svx[k] : (dir < 4 ? svy[k] : svz[k]);
				return AdvNb{sd[k], slx[k], sly[k], slz[k], nv};
			}
			const double nv = dir < 2 ? vx[n] : (dir < 4 ? vy[n] : vz[n]);
			return AdvNb{rho[n], lx[n], ly[n], lz[n], nv};
		};
		double acc = 0, md = 0;
		auto band_cmp = [&](double b) {
			const double diff = fabs(cd - b) / (fmin(cd, b) + B.thr);
			md = fmax(diff, md);
		};
#pragma unroll
		for (int dir = 0; dir < 6; dir++) {
			const int32_t c = e6[dir];
			if (c == -1) continue;
			if (c >= 0) {
				const AdvNb q = nb(c, dir);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, q, dt);
				if (BANDS) {
					const uint32_t k = uint32_t(int64_t(c) - int64_t(b0));
					const int nl = k < nb_in ? int(slv[k]) : int(B.lvl8[c] & 31u);
					// coarser: only from the corner of its face, i.e. the
					// cell's octant bits across the face axis are zero
					if (nl >= lvl || (oct & ~(1u << (dir >> 1))) == 0) band_cmp(q.d);
				}
			} else {
				const i4v q = *reinterpret_cast<const i4v*>(fine + 4 * size_t(-2 - c));
				const AdvNb first = nb(q.x, dir);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, first, dt);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.y, dir), dt);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.z, dir), dt);
				acc += adv_face_flux_d(dir, cd, clx, cly, clz, cvx, cvy, cvz, nb(q.w, dir), dt);
				if (BANDS) band_cmp(first.d);
			}
		}
		rho_out[s] = cd + acc / (clx * cly * clz);
		if (BANDS) {
			const double refine_diff = (lvl + 1) * B.inc, unrefine_diff = B.uns * refine_diff;
			B.band[s] = md > refine_diff ? 2 : (md >= unrefine_diff ? 1 : 0);
		}
	}
}

// 32-bit byte offsets from a uniform base: global_load v, voff, s[base]
// (halves the address registers of a gather; slots < 2^29, checked on the host)
__device__ __forceinline__ double ldo(const double* __restrict__ p, uint32_t off) {
	return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(p) + off);
}

// density store of the tile sweeps: non-temporal (a streaming write that
// should not allocate over the face lines neighboring tiles re-read from
// L2; measured on config 3: 0.1960 -> 0.1945 ms per sweep.  The same hint on
// the own-field loads cost 12 %: those lines ARE the re-read face lines)
__device__ __forceinline__ void st_nt(double* __restrict__ p, uint32_t i, double v) {
	__builtin_nontemporal_store(v, p + i);
}

// Regular tiles (tile_build.hip classify_tiles_kernel): an aligned 8x8x8 box
// of same-level cells, slots ts..ts+511 in Morton order, whose face
// neighbors across each side are the same-level cells of one neighbor box
// starting at slot tnb[6 gt + d] (-1: no neighbor on that side).  Thread t
// owns the cell with local Morton index t.  Own fields are staged in LDS for
// the in-tile faces; the (at most three) out-of-tile face neighbors of a
// cell are each used by that cell alone, so they are read straight into
// registers, issued before the barrier.  No per-cell face rows are read.
__device__ __forceinline__ uint32_t m9(uint32_t x, uint32_t y, uint32_t z) {
	return (x & 1u) | ((y & 1u) << 1) | ((z & 1u) << 2) | ((x & 2u) << 2) | ((y & 2u) << 3) | ((z & 2u) << 4) |
	       ((x & 4u) << 4) | ((y & 4u) << 5) | ((z & 4u) << 6);
}

// the out-of-tile neighbors of a regular tile, flattened: k = (side * 5 +
// value) * 64 + face cell (value 0 rho, 1 lx, 2 ly, 3 lz, 4 the velocity
// along the side's axis): 30 (side, value) rows of 64, wave w loads rows w,
// w + 8, w + 16, w + 24, so side and value are wave-uniform (scalar pointer
// and neighbor-box start, no private-memory lookup tables)
struct AdvPtrs {
	const double* p[7];  // rho, lx, ly, lz, vx, vy, vz
};

// The upwind flux through one face with the cell `c` on its minus side and
// `n` on its plus side, along axis a (solve.hpp:136-225 for direction +a):
// the reference's expression and operand order.  The minus-side cell adds
// -G, the plus-side cell +G; evaluated from the plus side the reference
// computes the same products in swapped (commutative) order, so one
// evaluation per face is bitwise what each side would get.
__device__ __forceinline__ double adv_face_g(int a, double cd, double clx, double cly, double clz, double cv_a,
                                             const AdvNb& n, double dt) {
#pragma clang fp contract(off)
	double ca, cb, cc, na, nb, nc;
	if (a == 0) { ca = clx; cb = cly; cc = clz; na = n.lx; nb = n.ly; nc = n.lz; }
	else if (a == 1) { ca = cly; cb = clx; cc = clz; na = n.ly; nb = n.lx; nc = n.lz; }
	else { ca = clz; cb = clx; cc = cly; na = n.lz; nb = n.lx; nc = n.ly; }
	const double min_area = fmin(cb * cc, nb * nc);
	const double v = (ca * n.v + na * cv_a) / (ca + na);
	return (v >= 0 ? cd : n.d) * dt * v * min_area;
}

// Tile records (32 B) are read one tile ahead of their use by a vector load
// (lanes 0..7 one word each) and made uniform with readlane.  A scalar load
// issued that early would not help: the next LDS wait (lgkmcnt counts LDS and
// scalar memory alike) would wait for it, exposing its latency once per tile;
// the vector counter is in order, so waiting for the previous tile's fields
// does not wait for the record loaded after them.
__device__ __forceinline__ uint32_t tile_record_word(const void* meta, uint32_t tt, uint32_t lane) {
	return lane < 8u ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(meta) + 8u * tt + lane) : 0u;
}

__device__ __forceinline__ uint32_t word_of(uint32_t v, int k) {
	return uint32_t(__builtin_amdgcn_readlane(int(v), k));
}

// Static persistent schedule of the tile sweeps: block b runs on XCD b % 8
// (measured: scripts/microbench/xcd_map.hip); XCD x sweeps the x-th eighth
// of the tile list, its B blocks side by side (block j: tiles j, j + B, ...),
// so the tiles an XCD has in flight are Morton neighbors sharing L2 lines.
struct StaticTiles {
	uint32_t t0, t1, B;
	__device__ __forceinline__ explicit StaticTiles(uint32_t ntiles) {
		const uint32_t x = blockIdx.x & 7u;
		B = gridDim.x >> 3;
		t0 = uint32_t((uint64_t(x) * ntiles) >> 3);
		t1 = uint32_t((uint64_t(x + 1) * ntiles) >> 3);
	}
	__device__ __forceinline__ uint32_t first() const { return t0 + (blockIdx.x >> 3); }
	__device__ __forceinline__ uint32_t next(uint32_t t) const { return t + B; }
};

// Neighbor records (Grid::NbRecords): per axis a and slot s the 24-B record
// {l_a, l_b * l_c, v_a} at r[3 a n + 3 s], b < c the two other axes, the
// product formed as the reference forms a face's area (solve.hpp:142-161).
// An out-of-tile face neighbor across an a-face then costs its density and
// this record (one line or two) instead of its density, three lengths and
// v_a from five arrays.  The sweeps stage such a neighbor into LDS with its
// length along a in row l_a, the area in the row of the first transverse
// length (nb_area_row) and 1.0 in the other (nb_one_row): every flux
// expression then forms nb * nc = area * 1.0 = area exactly, so the fluxes
// are bitwise those from the fields.
__global__ void nbrec_kernel(const double* __restrict__ lx, const double* __restrict__ ly,
                             const double* __restrict__ lz, const double* __restrict__ vx,
                             const double* __restrict__ vy, const double* __restrict__ vz, size_t n,
                             double* __restrict__ r) {
#pragma clang fp contract(off)
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		const double x = lx[s], y = ly[s], z = lz[s];
		double* r0 = r + 3 * s;
		double* r1 = r + 3 * n + 3 * s;
		double* r2 = r + 6 * n + 3 * s;
		r0[0] = x;
		r0[1] = y * z;
		r0[2] = vx[s];
		r1[0] = y;
		r1[1] = x * z;
		r1[2] = vy[s];
		r2[0] = z;
		r2[1] = x * y;
		r2[2] = vz[s];
	}
}

// LDS / register rows (4 lx, 5 ly, 6 lz) of a record-staged neighbor across
// an a-face: the area in the row of nb, 1.0 in the row of nc, where
// adv_face_g / adv_face_flux take (nb, nc) = (ly, lz), (lx, lz), (lx, ly)
__device__ __forceinline__ uint32_t nb_area_row(uint32_t a) { return a == 0 ? 5u : 4u; }
__device__ __forceinline__ uint32_t nb_one_row(uint32_t a) { return a == 2 ? 5u : 6u; }

template <int MINW, bool REC>
__global__ __launch_bounds__(512, MINW) void advection_regular_pp_kernel(AdvPtrs P, double* __restrict__ rho_out,
                                                                         const RegTileMeta* __restrict__ meta,
                                                                         uint32_t ntiles, double dt,
                                                                         const double* __restrict__ R, size_t nrec) {
#pragma clang fp contract(off)
	// rows rho, vx, vy, vz, lx, ly, lz; columns 0..511 the tile's own cells,
	// 512 + 64 d + (face cell) the out-of-tile neighbor across side d (only
	// rows rho, lx, ly, lz and the velocity along d's axis are filled), so
	// every face reads its neighbor through one LDS index, whichever side
	constexpr uint32_t W = 512 + 6 * 64;
	__shared__ double shd[7][W];
	__shared__ double shg[3][512];  // flux through each cell's +x, +y, +z face
	__shared__ double shm[3][64];   // flux through the tile's -x, -y, -z boundary faces
	const StaticTiles tk(ntiles);
	const uint32_t t1 = tk.t1;
	uint32_t t = tk.first();
	if (t >= t1) return;  // block-uniform
	const uint32_t tid = threadIdx.x;
	const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
	const uint32_t l[3] = {(tid & 1u) | ((tid >> 2) & 2u) | ((tid >> 4) & 4u),
	                       ((tid >> 1) & 1u) | ((tid >> 3) & 2u) | ((tid >> 5) & 4u),
	                       ((tid >> 2) & 1u) | ((tid >> 4) & 2u) | ((tid >> 6) & 4u)};
	// index of this cell within a side of each axis (the two other coordinates)
	const uint32_t fi[3] = {l[1] + 8 * l[2], l[0] + 8 * l[2], l[0] + 8 * l[1]};
	// LDS column of the +a neighbor of this cell (inside the tile or across side 2a+1)
	uint32_t lp[3];
#pragma unroll
	for (int a = 0; a < 3; a++) {
		uint32_t q[3] = {l[0], l[1], l[2]};
		q[a] += 1;
		lp[a] = l[a] < 7 ? m9(q[0], q[1], q[2]) : 512u + 64u * uint32_t(2 * a + 1) + fi[a];
	}
	// boundary-face duty of waves 0..2: wave a evaluates the -a side face of
	// the cell at l[a] = 0 whose face index is the lane
	const uint32_t bu = lane & 7u, bv = lane >> 3;
	const uint32_t bcell = w == 0 ? m9(0, bu, bv) : (w == 1 ? m9(bu, 0, bv) : m9(bu, bv, 0));
	const double* __restrict__ rho = P.p[0];
	const double* __restrict__ lx = P.p[1];
	const double* __restrict__ ly = P.p[2];
	const double* __restrict__ lz = P.p[3];
	const double* __restrict__ vx = P.p[4];
	const double* __restrict__ vy = P.p[5];
	const double* __restrict__ vz = P.p[6];
	// LDS row of value `val` (0 rho, 1 lx, 2 ly, 3 lz, 4 velocity along a)
	auto vrow = [](uint32_t val, uint32_t a) -> uint32_t { return val == 0 ? 0u : (val == 4 ? 1u + a : val + 3u); };
	// a register set: a tile being loaded
	struct RegSet {
		double c[7], e[4];
	};
	// a tile record: its first slot, and the raw record words (lanes 0..7)
	// whose neighbor-box starts are read with a wave-uniform readlane (a
	// register array indexed by a run-time side would live in scratch)
	struct RM {
		uint32_t ts, rec;
		__device__ __forceinline__ int32_t nst(uint32_t d) const { return int32_t(word_of(rec, int(1 + d))); }
	};
	auto unpack = [&](uint32_t v) { return RM{word_of(v, 0), v}; };
	auto load = [&](const RM& mt, RegSet& r) {
		const uint32_t ts = mt.ts;
		const uint32_t o = (ts + tid) << 3;
		r.c[0] = ldo(rho, o); r.c[1] = ldo(vx, o); r.c[2] = ldo(vy, o);
		r.c[3] = ldo(vz, o); r.c[4] = ldo(lx, o); r.c[5] = ldo(ly, o);
		r.c[6] = ldo(lz, o);
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint32_t row = w + 8u * uint32_t(i);  // wave-uniform
			r.e[i] = 0;
			if (row >= (REC ? 24u : 30u)) continue;
			const uint32_t d = REC ? row >> 2 : row / 5u, val = REC ? row & 3u : row - 5u * d, a = d >> 1;
			const int32_t st = mt.nst(d);
			if (st < 0) continue;
			const uint32_t u = lane & 7u, v = lane >> 3, side = (d & 1u) ? 0u : 7u;
			const uint32_t q0 = a == 0 ? side : u, q1 = a == 1 ? side : (a == 0 ? u : v), q2 = a == 2 ? side : v;
			const uint32_t sl = uint32_t(st) + m9(q0, q1, q2);
			if (REC) {
				// rows (side, 0 rho | 1 l_a | 2 area | 3 v_a): the density from
				// its field, the rest from the side's axis record
				r.e[i] = val == 0 ? ldo(rho, sl << 3) : R[size_t(a) * 3 * nrec + 3 * size_t(sl) + (val - 1)];
			} else {
				r.e[i] = ldo(P.p[val == 4 ? 4 + a : val], sl << 3);
			}
		}
	};
	// a loaded tile into LDS (after the barrier that ends the previous tile's reads)
	auto stage = [&](const RegSet& r) {
#pragma unroll
		for (int k = 0; k < 7; k++) shd[k][tid] = r.c[k];
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint32_t row = w + 8u * uint32_t(i);
			if (REC) {
				if (row < 24u) {
					const uint32_t d = row >> 2, val = row & 3u, a = d >> 1, col = 512u + 64u * d + lane;
					const uint32_t k = val == 0 ? 0u : (val == 1 ? 4u + a : (val == 2 ? nb_area_row(a) : 1u + a));
					shd[k][col] = r.e[i];
					if (val == 2) shd[nb_one_row(a)][col] = 1.0;
				}
			} else if (row < 30u) {
				const uint32_t d = row / 5u, val = row - 5u * d;
				shd[vrow(val, d >> 1)][512u + 64u * d + lane] = r.e[i];
			}
		}
	};
	// the staged tile tc from LDS
	auto compute = [&](const RM& mc) {
		const uint32_t ts = mc.ts;
		const double cd = shd[0][tid], clx = shd[4][tid], cly = shd[5][tid], clz = shd[6][tid];
		const double cva[3] = {shd[1][tid], shd[2][tid], shd[3][tid]};
		// pass 1: the +x, +y, +z face of every cell, once per face, branch-free
		// (a missing face beyond a non-periodic boundary evaluates zeros and
		// is masked by a select)
#pragma unroll
		for (int a = 0; a < 3; a++) {
			const uint32_t li = lp[a];
			const double g = adv_face_g(a, cd, clx, cly, clz, cva[a],
			                            AdvNb{shd[0][li], shd[4][li], shd[5][li], shd[6][li], shd[1 + a][li]}, dt);
			const bool has = l[a] < 7 || mc.nst(2 * a + 1) >= 0;
			shg[a][tid] = has ? g : 0.0;
		}
		// the tile's -a boundary faces (minus cell outside): 192 faces on
		// waves 0..2, wave-uniform
		if (w < 3 && mc.nst(2 * w) >= 0) {
			const uint32_t k = 512u + 64u * (2u * w) + lane;
			const AdvNb self{shd[0][bcell], shd[4][bcell], shd[5][bcell], shd[6][bcell], shd[1 + w][bcell]};
			double gmv;
			if (w == 0) gmv = adv_face_g(0, shd[0][k], shd[4][k], shd[5][k], shd[6][k], shd[1][k], self, dt);
			else if (w == 1) gmv = adv_face_g(1, shd[0][k], shd[4][k], shd[5][k], shd[6][k], shd[2][k], self, dt);
			else gmv = adv_face_g(2, shd[0][k], shd[4][k], shd[5][k], shd[6][k], shd[3][k], self, dt);
			shm[w][lane] = gmv;
		}
		__syncthreads();
		// pass 2: sum in the reference's face order -x, +x, -y, +y, -z, +z
		double acc = 0;
#pragma unroll
		for (int a = 0; a < 3; a++) {
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] -= 1;
			double gm = 0;
			if (l[a] > 0) gm = shg[a][m9(q[0] & 7u, q[1] & 7u, q[2] & 7u)];
			else if (mc.nst(2 * a) >= 0) gm = shm[a][fi[a]];
			acc += gm;
			acc += -shg[a][tid];
		}
		st_nt(rho_out, ts + tid, cd + acc / (clx * cly * clz));
	};
#if DCCRGX_REG_DEPTH2
	// two tiles in flight per block: register sets ra / rb alternate; a set
	// is refilled with the tile after next as soon as it has been staged.
	// A tile's record is read before the loads of the tile before it, so the
	// in-order vector counter never makes a record wait for field loads
	// younger than the ones being staged.
	RegSet ra, rb;
	uint32_t tA = t;
	RM mA = unpack(tile_record_word(meta, tA, lane));
	uint32_t tB = tk.next(tA);
	uint32_t recB = tB < t1 ? tile_record_word(meta, tB, lane) : 0u;
	load(mA, ra);
	RM mB = mA;
	uint32_t tL = t1, recL = 0u;
	if (tB < t1) {
		mB = unpack(recB);
		tL = tk.next(tB);
		recL = tL < t1 ? tile_record_word(meta, tL, lane) : 0u;
		load(mB, rb);
	}
	// the tile held by S (meta mS, index tS < t1): staged, S refilled with
	// tile tL, then computed; tS becomes the refilled tile (t1: none)
	auto body = [&](RegSet& S, RM& mS, uint32_t& tS) {
		__syncthreads();  // the previous tile's faces have been read from LDS
		stage(S);
		__syncthreads();
		const RM mc = mS;
		if (tL < t1) {
			mS = unpack(recL);
			tS = tL;
			tL = tk.next(tL);
			recL = tL < t1 ? tile_record_word(meta, tL, lane) : 0u;
			load(mS, S);
		} else {
			tS = t1;
		}
		compute(mc);
	};
	for (;;) {
		body(ra, mA, tA);
		if (tB >= t1) break;
		body(rb, mB, tB);
		if (tA >= t1) break;
	}
#else
	RegSet ra;
	RM cur = unpack(tile_record_word(meta, t, lane));
	uint32_t tn = tk.next(t);
	load(cur, ra);
	uint32_t rec = tn < t1 ? tile_record_word(meta, tn, lane) : 0u;  // tile tn's record
	for (;;) {
		__syncthreads();  // the previous tile's faces have been read from LDS
		stage(ra);
		__syncthreads();
		const bool more = tn < t1;
		RM nxt = cur;
		if (more) {
			// the next tile's loads fly while this one is computed, then the
			// record of the tile after it
			nxt = unpack(rec);
			load(nxt, ra);
			const uint32_t tnn = tk.next(tn);
			rec = tnn < t1 ? tile_record_word(meta, tnn, lane) : 0u;
		}
		compute(cur);
		if (!more) break;
		cur = nxt;
		tn = tk.next(tn);
	}
#endif
}

// The regular sweep with a compact LDS footprint, three blocks per CU
// (VERDICT r04 lever (a): more tiles in flight per XCD at the same L2
// footprint).  Own fields 7 x 512, the out-of-tile layers only the five
// values each side's faces read (6 x 5 x 64), and the +x / +y / +z face
// fluxes written over the layers once pass 1 has read them (one more
// barrier): 45.5 KB per block instead of 64 KB, 80 VGPRs (6 waves per SIMD).
// Same faces, same expressions, same summation order: bitwise the kernel
// above.  Selected at run time (DCCRGX_REG3=1) for paired A/Bs.
template <int MINW>
__global__ __launch_bounds__(512, MINW) void advection_regular3_kernel(AdvPtrs P, double* __restrict__ rho_out,
                                                                       const RegTileMeta* __restrict__ meta,
                                                                       uint32_t ntiles, double dt) {
#pragma clang fp contract(off)
	constexpr uint32_t OWN = 0, EXT = 7 * 512, SHM = EXT + 6 * 5 * 64;  // double offsets
	__shared__ double sh[SHM + 3 * 64];
	const StaticTiles tk(ntiles);
	const uint32_t t1 = tk.t1;
	uint32_t t = tk.first();
	if (t >= t1) return;  // block-uniform
	const uint32_t tid = threadIdx.x;
	const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
	const uint32_t l[3] = {(tid & 1u) | ((tid >> 2) & 2u) | ((tid >> 4) & 4u),
	                       ((tid >> 1) & 1u) | ((tid >> 3) & 2u) | ((tid >> 5) & 4u),
	                       ((tid >> 2) & 1u) | ((tid >> 4) & 2u) | ((tid >> 6) & 4u)};
	const uint32_t fi[3] = {l[1] + 8 * l[2], l[0] + 8 * l[2], l[0] + 8 * l[1]};
	const uint32_t bu = lane & 7u, bv = lane >> 3;
	const uint32_t bcell = w == 0 ? m9(0, bu, bv) : (w == 1 ? m9(bu, 0, bv) : m9(bu, bv, 0));
	const double* __restrict__ rho = P.p[0];
	const double* __restrict__ lx = P.p[1];
	const double* __restrict__ ly = P.p[2];
	const double* __restrict__ lz = P.p[3];
	const double* __restrict__ vx = P.p[4];
	const double* __restrict__ vy = P.p[5];
	const double* __restrict__ vz = P.p[6];
	// own rows: 0 rho, 1 vx, 2 vy, 3 vz, 4 lx, 5 ly, 6 lz
	auto own = [&](uint32_t row, uint32_t c) -> double& { return sh[OWN + row * 512 + c]; };
	// layer of side d: values 0 rho, 1 lx, 2 ly, 3 lz, 4 the velocity along d's axis
	auto ext = [&](uint32_t d, uint32_t val, uint32_t c) -> double& { return sh[EXT + (d * 5 + val) * 64 + c]; };
	struct RegSet {
		double c[7], e[4];
	};
	struct RM {
		uint32_t ts, rec;
		__device__ __forceinline__ int32_t nst(uint32_t d) const { return int32_t(word_of(rec, int(1 + d))); }
	};
	auto unpack = [&](uint32_t v) { return RM{word_of(v, 0), v}; };
	auto load = [&](const RM& mt, RegSet& r) {
		const uint32_t o = (mt.ts + tid) << 3;
		r.c[0] = ldo(rho, o); r.c[1] = ldo(vx, o); r.c[2] = ldo(vy, o);
		r.c[3] = ldo(vz, o); r.c[4] = ldo(lx, o); r.c[5] = ldo(ly, o);
		r.c[6] = ldo(lz, o);
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint32_t row = w + 8u * uint32_t(i);  // wave-uniform
			r.e[i] = 0;
			if (row >= 30u) continue;
			const uint32_t d = row / 5u, val = row - 5u * d, a = d >> 1;
			const int32_t st = mt.nst(d);
			if (st < 0) continue;
			const uint32_t u = lane & 7u, v = lane >> 3, side = (d & 1u) ? 0u : 7u;
			const uint32_t q0 = a == 0 ? side : u, q1 = a == 1 ? side : (a == 0 ? u : v), q2 = a == 2 ? side : v;
			r.e[i] = ldo(P.p[val == 4 ? 4 + a : val], (uint32_t(st) + m9(q0, q1, q2)) << 3);
		}
	};
	auto stage = [&](const RegSet& r) {
#pragma unroll
		for (int k = 0; k < 7; k++) own(uint32_t(k), tid) = r.c[k];
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint32_t row = w + 8u * uint32_t(i);
			if (row < 30u) sh[EXT + row * 64 + lane] = r.e[i];  // row = d * 5 + val
		}
	};
	// the +a neighbor of this cell: inside the tile (its own column) or on
	// the +a layer; value `val` 0 rho, 1 lx, 2 ly, 3 lz, 4 velocity along a
	auto nbr = [&](int a) -> AdvNb {
		if (l[a] < 7) {
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] += 1;
			const uint32_t c = m9(q[0], q[1], q[2]);
			return AdvNb{own(0, c), own(4, c), own(5, c), own(6, c), own(1 + uint32_t(a), c)};
		}
		const uint32_t d = uint32_t(2 * a + 1);
		return AdvNb{ext(d, 0, fi[a]), ext(d, 1, fi[a]), ext(d, 2, fi[a]), ext(d, 3, fi[a]), ext(d, 4, fi[a])};
	};
	auto compute = [&](const RM& mc) {
		const uint32_t ts = mc.ts;
		const double cd = own(0, tid), clx = own(4, tid), cly = own(5, tid), clz = own(6, tid);
		const double cva[3] = {own(1, tid), own(2, tid), own(3, tid)};
		double g[3];
#pragma unroll
		for (int a = 0; a < 3; a++) {
			const double ga = adv_face_g(a, cd, clx, cly, clz, cva[a], nbr(a), dt);
			const bool has = l[a] < 7 || mc.nst(2 * a + 1) >= 0;
			g[a] = has ? ga : 0.0;
		}
		double gmv = 0;
		const bool bnd = w < 3 && mc.nst(2 * w) >= 0;  // wave-uniform
		if (bnd) {
			const uint32_t d = 2u * w;
			const AdvNb self{own(0, bcell), own(4, bcell), own(5, bcell), own(6, bcell), own(1 + w, bcell)};
			const double md = ext(d, 0, lane), mlx = ext(d, 1, lane), mly = ext(d, 2, lane), mlz = ext(d, 3, lane),
			             mv = ext(d, 4, lane);
			if (w == 0) gmv = adv_face_g(0, md, mlx, mly, mlz, mv, self, dt);
			else if (w == 1) gmv = adv_face_g(1, md, mlx, mly, mlz, mv, self, dt);
			else gmv = adv_face_g(2, md, mlx, mly, mlz, mv, self, dt);
		}
		__syncthreads();  // every layer value has been read: the fluxes go over them
		double* shg = sh + EXT;  // [3][512]
#pragma unroll
		for (int a = 0; a < 3; a++) shg[a * 512 + tid] = g[a];
		if (bnd) sh[SHM + w * 64 + lane] = gmv;
		__syncthreads();
		// nothing but indices stays live across the barriers: the fluxes and
		// the cell's own values are read back from LDS
		double acc = 0;
#pragma unroll
		for (int a = 0; a < 3; a++) {
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] -= 1;
			double gm = 0;
			if (l[a] > 0) gm = shg[a * 512 + m9(q[0] & 7u, q[1] & 7u, q[2] & 7u)];
			else if (mc.nst(2 * a) >= 0) gm = sh[SHM + a * 64 + fi[a]];
			acc += gm;
			acc += -shg[a * 512 + tid];
		}
		st_nt(rho_out, ts + tid, own(0, tid) + acc / (own(4, tid) * own(5, tid) * own(6, tid)));
	};
	// no register prefetch of the next tile (its 22 VGPRs would spill at 80):
	// with three blocks per CU the other blocks' loads overlap this one's
	// compute.  The next record is still read one tile ahead.
	RM cur = unpack(tile_record_word(meta, t, lane));
	uint32_t tn = tk.next(t);
	uint32_t rec = tn < t1 ? tile_record_word(meta, tn, lane) : 0u;
	for (;;) {
		{
			RegSet ra;
			load(cur, ra);
			__syncthreads();  // the previous tile's fluxes have been read from LDS
			stage(ra);
		}
		__syncthreads();
		const bool more = tn < t1;
		RM nxt = cur;
		if (more) {
			nxt = unpack(rec);
			const uint32_t tnn = tk.next(tn);
			rec = tnn < t1 ? tile_record_word(meta, tnn, lane) : 0u;
		}
		compute(cur);
		if (!more) break;
		cur = nxt;
		tn = tk.next(tn);
	}
}

// Persistent, software-pipelined form of advection_tiles_kernel for any tile
// (the tables of tile_build.hip): the same XCD-contiguous persistent schedule
// as advection_regular_pp_kernel; per tile one 32-B record; while a tile is
// computed from LDS, the next tile's own fields, face rows, ext cells (at
// most two per thread) and finer-face index pairs are in flight into
// registers, so the compute phase issues no global load.
struct TileMeta {
	uint32_t ts, n, e0, ne, fb, nf, pad0, pad1;
};

// ONCE: a face between two cells of the tile whose codes point at each other
// (a same-level pair: the minus cell's +a code is the plus cell, the plus
// cell's -a code the minus cell) is evaluated once, by its minus cell, into
// LDS (adv_face_g, as the regular kernel does), and the plus cell adds the
// stored value: the same product with the same operands (the expression is
// symmetric, see adv_face_g), so the densities are bitwise the two-sided
// form's.  Faces to ext cells, finer lists and coarser neighbors are still
// evaluated by each side.
template <int MINW, bool REC, bool ONCE>
__global__ __launch_bounds__(512, MINW) void advection_tiles_pp_kernel(
    AdvPtrs P, double* __restrict__ rho_out, const uint32_t* __restrict__ tell, uint32_t tplane,
    const uint32_t* __restrict__ ext, const uint32_t* __restrict__ tfine, const TileMeta* __restrict__ meta,
    uint32_t ntiles, uint32_t ecap, double dt, const double* __restrict__ R, size_t nrec) {
#pragma clang fp contract(off)
	constexpr uint32_t T = 512;
	// [7][T + ecap] doubles (rho vx vy vz lx ly lz); ONCE: 3 x T doubles of
	// +a face fluxes; 2 x T u32 finer-face pairs; ONCE: 3 x T flags
	extern __shared__ double shd[];
	const uint32_t W = T + ecap;
	double* shg = shd + 7 * W;
	uint32_t* shf = reinterpret_cast<uint32_t*>(shd + 7 * W + (ONCE ? 3 * T : 0));
	uint8_t* shok = reinterpret_cast<uint8_t*>(shf + 2 * T);
	const StaticTiles tk(ntiles);
	const uint32_t t1 = tk.t1;
	uint32_t t = tk.first();
	if (t >= t1) return;  // block-uniform
	const uint32_t tid = threadIdx.x;
	const double* const rho = P.p[0];
	const double* const lx = P.p[1];
	const double* const ly = P.p[2];
	const double* const lz = P.p[3];
	const double* const vx = P.p[4];
	const double* const vy = P.p[5];
	const double* const vz = P.p[6];
	// the register set of the tile being loaded (field order rho vx vy vz lx ly lz)
	double c[7], xa[7], xb[7];
	uint32_t row[3], fq[2];
	auto load7 = [&](uint32_t slot, double (&v)[7]) {
		const uint32_t o = slot << 3;
		v[0] = ldo(rho, o); v[1] = ldo(vx, o); v[2] = ldo(vy, o); v[3] = ldo(vz, o);
		v[4] = ldo(lx, o); v[5] = ldo(ly, o); v[6] = ldo(lz, o);
	};
	// ext = slot | axis mask << 29: density and lengths, and only the
	// velocity components along the axes its faces cross
	auto load5 = [&](uint32_t q, double (&v)[7]) {
		const uint32_t sl = q & 0x1fffffffu, o = sl << 3, ax = q >> 29;
		v[0] = ldo(rho, o);
		if (REC && (ax == 1u || ax == 2u || ax == 4u)) {
			// reached through faces of one axis (all but ~0.3 % on config 3):
			// its density and that axis' record, staged in the rows of
			// nb_area_row / nb_one_row (bitwise the same fluxes)
			const uint32_t a = ax >> 1;
			const double* r = R + size_t(a) * 3 * nrec + 3 * size_t(sl);
			const double la = r[0], ar = r[1], vv = r[2];
			v[4] = a == 0 ? la : ar;
			v[5] = a == 0 ? ar : (a == 1 ? la : 1.0);
			v[6] = a == 2 ? la : 1.0;
			v[1] = a == 0 ? vv : 0.0;
			v[2] = a == 1 ? vv : 0.0;
			v[3] = a == 2 ? vv : 0.0;
			return;
		}
		v[4] = ldo(lx, o); v[5] = ldo(ly, o); v[6] = ldo(lz, o);
		v[1] = (ax & 1u) ? ldo(vx, o) : 0.0;
		v[2] = (ax & 2u) ? ldo(vy, o) : 0.0;
		v[3] = (ax & 4u) ? ldo(vz, o) : 0.0;
	};
	const uint32_t lane = tid & 63u;
	struct GM {
		uint32_t ts, n, e0, ne, fb, nf;
	};
	auto unpack = [&](uint32_t v) { return GM{word_of(v, 0), word_of(v, 1), word_of(v, 2), word_of(v, 3), word_of(v, 4),
	                                          word_of(v, 5)}; };
	auto load = [&](const GM& mt) {
		const uint32_t ts = mt.ts, n = mt.n, e0 = mt.e0, ne = mt.ne, fb = mt.fb, nf = mt.nf;
		if (tid < n) {
			load7(ts + tid, c);
			// the tile's face codes, ext list and finer pairs are read once per
			// sweep: non-temporal, so they do not evict the field lines other
			// tiles re-read (paired A/B on config 3: 0.1915 -> 0.1865 ms/sweep)
			// (three planes of codes: one coalesced 4-B load per plane; the
			// interleaved 12-B records cost ~20 us per sweep on config 3)
			row[0] = __builtin_nontemporal_load(tell + (ts + tid));
			row[1] = __builtin_nontemporal_load(tell + tplane + (ts + tid));
			row[2] = __builtin_nontemporal_load(tell + 2 * tplane + (ts + tid));
		}
		if (tid < ne) load5(__builtin_nontemporal_load(ext + e0 + tid), xa);
		if (tid + T < ne) load5(__builtin_nontemporal_load(ext + e0 + tid + T), xb);
		if (tid < nf) {
			typedef unsigned int u2v __attribute__((ext_vector_type(2)));
			const u2v q = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(tfine) + (fb + tid));
			fq[0] = q.x;
			fq[1] = q.y;
		}
	};
	GM cur = unpack(tile_record_word(meta, t, lane));
	uint32_t tn = tk.next(t);
	load(cur);
	uint32_t rec = tn < t1 ? tile_record_word(meta, tn, lane) : 0u;  // tile tn's record
	for (;;) {
		const uint32_t n = cur.n, ne = cur.ne, nf = cur.nf, ts = cur.ts;
		__syncthreads();  // the previous tile's faces have been read from LDS
		if (tid < n)
#pragma unroll
			for (int k = 0; k < 7; k++) shd[k * W + tid] = c[k];
		if (tid < ne)
#pragma unroll
			for (int k = 0; k < 7; k++) shd[k * W + T + tid] = xa[k];
		if (tid + T < ne)
#pragma unroll
			for (int k = 0; k < 7; k++) shd[k * W + 2 * T + tid] = xb[k];
		if (tid < nf) {
			shf[2 * tid] = fq[0];
			shf[2 * tid + 1] = fq[1];
		}
		const uint32_t r0 = row[0], r1 = row[1], r2 = row[2];
		__syncthreads();
		const bool more = tn < t1;
		GM nxt = cur;
		if (more) {
			// the next tile's loads fly while this one is computed, then the
			// record of the tile after it
			nxt = unpack(rec);
			load(nxt);
			const uint32_t tnn = tk.next(tn);
			rec = tnn < t1 ? tile_record_word(meta, tnn, lane) : 0u;
		}
		const bool own = tid < n;
		double cd = 0, cvx = 0, cvy = 0, cvz = 0, clx = 1, cly = 1, clz = 1;
		if (own) {
			cd = shd[tid];
			cvx = shd[W + tid];
			cvy = shd[2 * W + tid];
			cvz = shd[3 * W + tid];
			clx = shd[4 * W + tid];
			cly = shd[5 * W + tid];
			clz = shd[6 * W + tid];
		}
		auto fetch = [&](uint32_t li, int d) -> AdvNb {
			return AdvNb{shd[li], shd[4 * W + li], shd[5 * W + li], shd[6 * W + li], shd[(1 + (d >> 1)) * W + li]};
		};
		const uint32_t rr[3] = {r0, r1, r2};
		// ONCE, pass 1: the +a faces to a cell of the tile (direct codes)
		double gp[3] = {0, 0, 0};
		bool hp[3] = {false, false, false};
		if (ONCE) {
			if (own) {
				const double cva[3] = {cvx, cvy, cvz};
#pragma unroll
				for (int a = 0; a < 3; a++) {
					const uint32_t code = rr[a] >> 16;
					hp[a] = code < n;  // (0xffff none and 0x8000 | k finer lists are >= n)
					if (hp[a]) {
						gp[a] = adv_face_g(a, cd, clx, cly, clz, cva[a], fetch(code, 2 * a + 1), dt);
						shg[a * T + tid] = gp[a];
					}
					shok[a * T + tid] = hp[a] ? 1 : 0;
				}
			}
			__syncthreads();
		}
		if (own) {
			double acc = 0;
#pragma unroll
			for (int d = 0; d < 6; d++) {
				const uint32_t code = (rr[d >> 1] >> (16 * (d & 1))) & 0xffffu;
				if (code == 0xffffu) continue;
				if (ONCE) {
					const int a = d >> 1;
					if ((d & 1) && hp[a]) {
						acc += -gp[a];
						continue;
					}
					if (!(d & 1) && code < n && shok[a * T + code]) {
						acc += shg[a * T + code];
						continue;
					}
				}
				if (code & 0x8000u) {
					const uint32_t fk = code & 0x7fffu;
					const uint32_t q0 = shf[2 * fk], q1 = shf[2 * fk + 1];
					const uint32_t li[4] = {q0 & 0xffffu, q0 >> 16, q1 & 0xffffu, q1 >> 16};
#pragma unroll
					for (int k = 0; k < 4; k++)
						acc += adv_face_flux_d(d, cd, clx, cly, clz, cvx, cvy, cvz, fetch(li[k], d), dt);
				} else {
					acc += adv_face_flux_d(d, cd, clx, cly, clz, cvx, cvy, cvz, fetch(code, d), dt);
				}
			}
			st_nt(rho_out, ts + tid, cd + acc / (clx * cly * clz));
		}
		if (!more) break;
		cur = nxt;
		tn = tk.next(tn);
	}
}
// Both kinds of tile in ONE persistent sweep, in tile order (the Morton
// order of the slots): the same XCD-contiguous static schedule, so the tiles
// an XCD has in flight are neighbors of both kinds and read each other's face
// lines from its L2, and one launch has one tail.  Per tile one 32-B record,
// word 7 its kind (1: a regular box, advection_regular_pp_kernel's record;
// 0: any other tile, advection_tiles_pp_kernel's); the LDS holds either
// layout, the registers of the tile in flight either register set (the
// regular one in c[] and xa[0..3]).  Each kind's face fluxes are its own
// kernel's expressions in its own order, so every density is bitwise that of
// the two-kernel sweep.
#if DCCRGX_FUSED_SWEEP
template <int MINW>
__global__ __launch_bounds__(512, MINW) void advection_fused_kernel(
    AdvPtrs P, double* __restrict__ rho_out, const uint32_t* __restrict__ tell, uint32_t tplane,
    const uint32_t* __restrict__ ext, const uint32_t* __restrict__ tfine, const uint32_t* __restrict__ meta,
    uint32_t ntiles, uint32_t ecap, double dt) {
#pragma clang fp contract(off)
	constexpr uint32_t T = 512;
	constexpr uint32_t WR = 512 + 6 * 64;  // regular layout: [7][WR] then [3][512] + [3][64] face fluxes
	extern __shared__ double shd[];
	const uint32_t W = T + ecap;  // general layout: [7][W] then 2 x T u32 finer-face pairs
	uint32_t* shf = reinterpret_cast<uint32_t*>(shd + 7 * W);
	double* shg = shd + 7 * WR;
	double* shm = shg + 3 * 512;
	const StaticTiles tk(ntiles);
	const uint32_t t1 = tk.t1;
	uint32_t t = tk.first();
	if (t >= t1) return;  // block-uniform
	const uint32_t tid = threadIdx.x;
	const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63u;
	const double* const rho = P.p[0];
	const double* const lx = P.p[1];
	const double* const ly = P.p[2];
	const double* const lz = P.p[3];
	const double* const vx = P.p[4];
	const double* const vy = P.p[5];
	const double* const vz = P.p[6];
	// the tile in flight: own fields (both kinds), regular out-of-tile rows
	// in xa[0..3] or general ext cells in xa (the rare ones beyond 512 are
	// loaded at staging), face codes, finer pairs
	double c[7], xa[7];
	uint32_t row[3], fq[2];
	auto load5 = [&](uint32_t q, double (&vv)[7]) {
		const uint32_t o = (q & 0x1fffffffu) << 3, ax = q >> 29;
		vv[0] = ldo(rho, o); vv[4] = ldo(lx, o); vv[5] = ldo(ly, o); vv[6] = ldo(lz, o);
		vv[1] = (ax & 1u) ? ldo(vx, o) : 0.0;
		vv[2] = (ax & 2u) ? ldo(vy, o) : 0.0;
		vv[3] = (ax & 4u) ? ldo(vz, o) : 0.0;
	};
	auto load7 = [&](uint32_t slot, double (&v)[7]) {
		const uint32_t o = slot << 3;
		v[0] = ldo(rho, o); v[1] = ldo(vx, o); v[2] = ldo(vy, o); v[3] = ldo(vz, o);
		v[4] = ldo(lx, o); v[5] = ldo(ly, o); v[6] = ldo(lz, o);
	};
	auto is_reg = [](uint32_t v) { return word_of(v, 7) != 0u; };
	// ---- regular tiles (advection_regular_pp_kernel) ----
	auto reg_l = [&](int a) -> uint32_t {
		return a == 0 ? ((tid & 1u) | ((tid >> 2) & 2u) | ((tid >> 4) & 4u))
		              : (a == 1 ? (((tid >> 1) & 1u) | ((tid >> 3) & 2u) | ((tid >> 5) & 4u))
		                        : (((tid >> 2) & 1u) | ((tid >> 4) & 2u) | ((tid >> 6) & 4u)));
	};
	auto vrow = [](uint32_t val, uint32_t a) -> uint32_t { return val == 0 ? 0u : (val == 4 ? 1u + a : val + 3u); };
	auto reg_load = [&](uint32_t v) {
		const uint32_t ts = word_of(v, 0);
		load7(ts + tid, c);
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint32_t rw = w + 8u * uint32_t(i);  // wave-uniform
			xa[i] = 0;
			if (rw >= 30u) continue;
			const uint32_t d = rw / 5u, val = rw - 5u * d, a = d >> 1;
			const int32_t st = int32_t(word_of(v, int(1 + d)));
			if (st < 0) continue;
			const uint32_t u = lane & 7u, vv = lane >> 3, side = (d & 1u) ? 0u : 7u;
			const uint32_t q0 = a == 0 ? side : u, q1 = a == 1 ? side : (a == 0 ? u : vv), q2 = a == 2 ? side : vv;
			xa[i] = ldo(P.p[val == 4 ? 4 + a : val], (uint32_t(st) + m9(q0, q1, q2)) << 3);
		}
	};
	auto reg_stage = [&]() {
		// own fields in the order rho vx vy vz lx ly lz (= the regular rows 0..6)
#pragma unroll
		for (int k = 0; k < 7; k++) shd[k * WR + tid] = c[k];
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint32_t rw = w + 8u * uint32_t(i);
			if (rw < 30u) {
				const uint32_t d = rw / 5u, val = rw - 5u * d;
				shd[vrow(val, d >> 1) * WR + 512u + 64u * d + lane] = xa[i];
			}
		}
	};
	auto reg_compute = [&](uint32_t v) {
		const uint32_t ts = word_of(v, 0);
		const uint32_t l[3] = {reg_l(0), reg_l(1), reg_l(2)};
		const uint32_t fi[3] = {l[1] + 8 * l[2], l[0] + 8 * l[2], l[0] + 8 * l[1]};
		auto nst = [&](uint32_t d) { return int32_t(word_of(v, int(1 + d))); };
		const double cd = shd[tid], clx = shd[4 * WR + tid], cly = shd[5 * WR + tid], clz = shd[6 * WR + tid];
		const double cva[3] = {shd[WR + tid], shd[2 * WR + tid], shd[3 * WR + tid]};
#pragma unroll
		for (int a = 0; a < 3; a++) {
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] += 1;
			const uint32_t li = l[a] < 7 ? m9(q[0], q[1], q[2]) : 512u + 64u * uint32_t(2 * a + 1) + fi[a];
			const double gg = adv_face_g(a, cd, clx, cly, clz, cva[a],
			                             AdvNb{shd[li], shd[4 * WR + li], shd[5 * WR + li], shd[6 * WR + li],
			                                   shd[(1 + a) * WR + li]},
			                             dt);
			const bool has = l[a] < 7 || nst(2 * a + 1) >= 0;
			shg[a * 512 + tid] = has ? gg : 0.0;
		}
		if (w < 3 && nst(2 * w) >= 0) {
			const uint32_t bu = lane & 7u, bv = lane >> 3;
			const uint32_t bcell = w == 0 ? m9(0, bu, bv) : (w == 1 ? m9(bu, 0, bv) : m9(bu, bv, 0));
			const uint32_t k = 512u + 64u * (2u * w) + lane;
			const AdvNb self{shd[bcell], shd[4 * WR + bcell], shd[5 * WR + bcell], shd[6 * WR + bcell],
			                 shd[(1 + w) * WR + bcell]};
			double gmv;
			if (w == 0) gmv = adv_face_g(0, shd[k], shd[4 * WR + k], shd[5 * WR + k], shd[6 * WR + k], shd[WR + k], self, dt);
			else if (w == 1)
				gmv = adv_face_g(1, shd[k], shd[4 * WR + k], shd[5 * WR + k], shd[6 * WR + k], shd[2 * WR + k], self, dt);
			else gmv = adv_face_g(2, shd[k], shd[4 * WR + k], shd[5 * WR + k], shd[6 * WR + k], shd[3 * WR + k], self, dt);
			shm[w * 64 + lane] = gmv;
		}
		__syncthreads();
		double acc = 0;
#pragma unroll
		for (int a = 0; a < 3; a++) {
			uint32_t q[3] = {l[0], l[1], l[2]};
			q[a] -= 1;
			double gm = 0;
			if (l[a] > 0) gm = shg[a * 512 + m9(q[0] & 7u, q[1] & 7u, q[2] & 7u)];
			else if (nst(2 * a) >= 0) gm = shm[a * 64 + fi[a]];
			acc += gm;
			acc += -shg[a * 512 + tid];
		}
		st_nt(rho_out, ts + tid, cd + acc / (clx * cly * clz));
	};
	// ---- other tiles (advection_tiles_pp_kernel) ----
	auto gen_load = [&](uint32_t v) {
		const uint32_t ts = word_of(v, 0), n = word_of(v, 1), e0 = word_of(v, 2), ne = word_of(v, 3),
		               fb = word_of(v, 4), nf = word_of(v, 5);
		if (tid < n) {
			load7(ts + tid, c);
			row[0] = __builtin_nontemporal_load(tell + (ts + tid));
			row[1] = __builtin_nontemporal_load(tell + tplane + (ts + tid));
			row[2] = __builtin_nontemporal_load(tell + 2 * tplane + (ts + tid));
		}
		if (tid < ne) load5(__builtin_nontemporal_load(ext + e0 + tid), xa);
		if (tid < nf) {
			typedef unsigned int u2v __attribute__((ext_vector_type(2)));
			const u2v q = __builtin_nontemporal_load(reinterpret_cast<const u2v*>(tfine) + (fb + tid));
			fq[0] = q.x;
			fq[1] = q.y;
		}
	};
	uint32_t rr[3] = {0, 0, 0};
	auto gen_stage = [&](uint32_t v) {
		const uint32_t n = word_of(v, 1), ne = word_of(v, 3), nf = word_of(v, 5);
		if (tid < n)
#pragma unroll
			for (int k = 0; k < 7; k++) shd[k * W + tid] = c[k];
		if (tid < ne)
#pragma unroll
			for (int k = 0; k < 7; k++) shd[k * W + T + tid] = xa[k];
		if (tid + T < ne) {  // ext cells beyond the first T: loaded here (rare)
			double xb[7];
			load5(__builtin_nontemporal_load(ext + word_of(v, 2) + tid + T), xb);
#pragma unroll
			for (int k = 0; k < 7; k++) shd[k * W + 2 * T + tid] = xb[k];
		}
		if (tid < nf) {
			shf[2 * tid] = fq[0];
			shf[2 * tid + 1] = fq[1];
		}
		rr[0] = row[0];
		rr[1] = row[1];
		rr[2] = row[2];
	};
	auto gen_compute = [&](uint32_t v) {
		const uint32_t ts = word_of(v, 0), n = word_of(v, 1);
		if (tid >= n) return;
		const double cd = shd[tid], cvx = shd[W + tid], cvy = shd[2 * W + tid], cvz = shd[3 * W + tid],
		             clx = shd[4 * W + tid], cly = shd[5 * W + tid], clz = shd[6 * W + tid];
		auto fetch = [&](uint32_t li, int d) -> AdvNb {
			return AdvNb{shd[li], shd[4 * W + li], shd[5 * W + li], shd[6 * W + li], shd[(1 + (d >> 1)) * W + li]};
		};
		double acc = 0;
#pragma unroll
		for (int d = 0; d < 6; d++) {
			const uint32_t code = (rr[d >> 1] >> (16 * (d & 1))) & 0xffffu;
			if (code == 0xffffu) continue;
			if (code & 0x8000u) {
				const uint32_t fk = code & 0x7fffu;
				const uint32_t q0 = shf[2 * fk], q1 = shf[2 * fk + 1];
				const uint32_t li[4] = {q0 & 0xffffu, q0 >> 16, q1 & 0xffffu, q1 >> 16};
#pragma unroll
				for (int k = 0; k < 4; k++) acc += adv_face_flux_d(d, cd, clx, cly, clz, cvx, cvy, cvz, fetch(li[k], d), dt);
			} else {
				acc += adv_face_flux_d(d, cd, clx, cly, clz, cvx, cvy, cvz, fetch(code, d), dt);
			}
		}
		st_nt(rho_out, ts + tid, cd + acc / (clx * cly * clz));
	};
	uint32_t cur = tile_record_word(meta, t, lane);
	if (is_reg(cur)) reg_load(cur);
	else gen_load(cur);
	uint32_t tn = tk.next(t);
	uint32_t rec = tn < t1 ? tile_record_word(meta, tn, lane) : 0u;  // tile tn's record
	for (;;) {
		__syncthreads();  // the previous tile's faces have been read from LDS
		const bool creg = is_reg(cur);
		if (creg) reg_stage();
		else gen_stage(cur);
		__syncthreads();
		const bool more = tn < t1;
		const uint32_t nxt = rec;
		if (more) {
			// the next tile's loads fly while this one is computed, then the
			// record of the tile after it
			if (is_reg(nxt)) reg_load(nxt);
			else gen_load(nxt);
			const uint32_t tnn = tk.next(tn);
			rec = tnn < t1 ? tile_record_word(meta, tnn, lane) : 0u;
		}
		if (creg) reg_compute(cur);
		else gen_compute(cur);
		if (!more) break;
		cur = nxt;
		tn = tk.next(tn);
	}
}

#endif

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
// max_diff of check_for_adaptation (tests/advection/adapter.hpp:74-121) of a
// local cell: the largest relative density difference over its face
// neighbors, counting a finer neighbor only at the cell's corner and a
// coarser one only when the cell sits at its corner (the x, y, z offset
// test of 84-102, the same from either side of a face)
// max_diff of one local cell (adapter.hpp:47-123) over the fixed-width face
// table: a same-size neighbor always counts, a coarser one only when the
// cell sits at the corner of the coarser cell's face, of four finer ones only
// the first (the one at the cell's corner); lvl8: the level of every slot
__device__ double adv_max_diff(MapCtx m, const double* __restrict__ rho, const int32_t* __restrict__ ell,
                               const int32_t* __restrict__ fine, const uint8_t* __restrict__ lvl8,
                               const uint64_t* __restrict__ slot_ids, size_t s, double diff_threshold, int& lvl) {
	typedef int i2v __attribute__((ext_vector_type(2)));
	const unsigned lv = lvl8[s];
	lvl = int(lv & 31u);
	const unsigned oct = lv >> 5;
	int32_t e6[6];
	const i2v* ev = reinterpret_cast<const i2v*>(ell + 6 * s);
#pragma unroll
	for (int j = 0; j < 3; j++) {
		const i2v v = ev[j];
		e6[2 * j] = v.x;
		e6[2 * j + 1] = v.y;
	}
	const double a = rho[s];
	double md = 0;
#pragma unroll
	for (int dir = 0; dir < 6; dir++) {
		const int32_t e = e6[dir];
		if (e == -1) continue;
		int32_t nsl;
		if (e >= 0) {
			nsl = e;
			// coarser: only when the cell sits at the corner of its face
			if (int(lvl8[e] & 31u) < lvl && (oct & ~(1u << (dir >> 1))) != 0) continue;
		} else {
			nsl = fine[4 * size_t(-2 - e)];
		}
		const double b = rho[nsl];
		const double diff = fabs(a - b) / (fmin(a, b) + diff_threshold);
		md = fmax(diff, md);
	}
	return md;
}

__global__ void adv_candidates_kernel(MapCtx m, const double* __restrict__ rho, const int32_t* __restrict__ ell,
                                      const int32_t* __restrict__ fine, const uint8_t* __restrict__ lvl8,
                                      const uint64_t* __restrict__ slot_ids, size_t n,
                                      double diff_increase, double diff_threshold, uint64_t* out,
                                      unsigned long long* counter) {
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		int lvl;
		const double md = adv_max_diff(m, rho, ell, fine, lvl8, slot_ids, s, diff_threshold, lvl);
		if (md > (lvl + 1) * diff_increase) out[atomicAdd(counter, 1ull)] = slot_ids[s];
	}
}

// the band of each local cell (adapter.hpp:124-176): 2 refine, 1 keep (no
// unrefine), 0 unrefine
__global__ void adv_bands_kernel(MapCtx m, const double* __restrict__ rho, const int32_t* __restrict__ ell,
                                 const int32_t* __restrict__ fine, const uint8_t* __restrict__ lvl8,
                                 const uint64_t* __restrict__ slot_ids, size_t n,
                                 double diff_increase, double diff_threshold, double unrefine_sensitivity,
                                 uint8_t* __restrict__ band) {
#pragma clang fp contract(off)
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		int lvl;
		const double md = adv_max_diff(m, rho, ell, fine, lvl8, slot_ids, s, diff_threshold, lvl);
		const double refine_diff = (lvl + 1) * diff_increase, unrefine_diff = unrefine_sensitivity * refine_diff;
		band[s] = md > refine_diff ? 2 : (md >= unrefine_diff ? 1 : 0);
	}
}

// the requests check_for_adaptation issues from the bands (adapter.hpp:
// 124-176), per local slot on Morton-ordered slots: a refine request for a
// band-2 leaf below the maximum level; per family (a run of consecutive slots
// with one parent, level > 0) headed at this slot: all 8 members here -> kept
// when any member's band is >= 1, else one unrefine request; fewer -> the
// run goes to the host, which merges the runs of a parent (families split
// between runs or processes).  Lists are appended through counters
// cnt[0] refines, cnt[1] unrefines, cnt[2] kept families, cnt[3] partial runs.
//
// Coalesced: a wave covers 64 x kJ consecutive slots, lane l taking slots
// base + 64 j + l (j < kJ) and the tail chunk base + 64 kJ + l (the runs that
// start in the last chunk reach up to 7 slots past it); the neighbors'
// parents and bands come from the other lanes by shuffles (slot + q is lane
// l + q of the same chunk, or of the next one past lane 63).  List positions
// are reserved per block (block_reserve4).  Every id and band load is issued
// before the parents are computed.  (Round 5: 282 -> 136 us a config-3 step,
// of which the per-block reservation took 277 -> 191, the solo shortcut
// 191 -> 165 and lane-uniform MapCtx reads the rest)
// Positions in the four request lists for a block of W waves: one atomic per
// block and list (per-wave atomics on the same four counters serialise at the
// device-coherent level - 4 x ~17000 of them a config-3 step).  c and the
// result in counter order: refine, unrefine, kept, partial.
template <int W>
__device__ __forceinline__ void block_reserve4(unsigned long long* __restrict__ cnt, const unsigned c[4],
                                               unsigned long long out[4]) {
	__shared__ unsigned tot[W][4];
	__shared__ unsigned long long at[W][4];
	const int lane = int(threadIdx.x & 63u), w = int(threadIdx.x >> 6);
	unsigned incl[4];
#pragma unroll
	for (int k = 0; k < 4; k++) {
		incl[k] = c[k];
#pragma unroll
		for (int d = 1; d < 64; d <<= 1) {
			const unsigned v = __shfl_up(incl[k], d, 64);
			if (lane >= d) incl[k] += v;
		}
		if (lane == 63) tot[w][k] = incl[k];
	}
	__syncthreads();
	if (threadIdx.x < 4) {
		const int k = int(threadIdx.x);
		unsigned run = 0;
		for (int v = 0; v < W; v++) run += tot[v][k];
		unsigned long long b = run ? atomicAdd(&cnt[k], static_cast<unsigned long long>(run)) : 0ull;
		for (int v = 0; v < W; v++) {
			at[v][k] = b;
			b += tot[v][k];
		}
	}
	__syncthreads();
#pragma unroll
	for (int k = 0; k < 4; k++) out[k] = at[w][k] + (incl[k] - c[k]);
}

// solo: every cell of the grid is local and the slots are in Morton order, so
// a family's leaves are one run and a partial run (k < 8) always has a
// sibling with children - no lookups needed to know it.
template <int BS>
__global__ __launch_bounds__(BS) void adv_requests_kernel(MapCtx m, DevMesh M, const uint64_t* __restrict__ ids,
                                                               const uint8_t* __restrict__ band, size_t n, bool solo,
                                                               int rank, uint64_t* __restrict__ ref, uint64_t* __restrict__ unref,
                                                               uint32_t* __restrict__ part,
                                                               unsigned long long* __restrict__ cnt) {
	constexpr int kJ = 8;
	constexpr int kSpan = BS * kJ;  // a block's slots: wave w takes [64 kJ w, 64 kJ (w + 1))
	// the parents (~0: level 0 or none) and bands of the block's slots, of
	// the slot before them and of the seven after them (entry i = slot
	// base0 + i - 1): a run head reads its run from here, every other slot
	// only its predecessor (round 5's form shuffled all seven neighbors of
	// every slot)
	__shared__ uint64_t sp[kSpan + 8];
	__shared__ uint8_t sb[kSpan + 8];
	const size_t base0 = size_t(blockIdx.x) * kSpan;
	for (int i = int(threadIdx.x); i < kSpan + 8; i += BS) {
		const bool ok = (base0 + size_t(i) >= 1) && base0 + size_t(i) - 1 < n;
		const uint64_t id = ok ? ids[base0 + size_t(i) - 1] : 0;
		sp[i] = map_level(m, id) > 0 ? map_parent(m, id) : ~uint64_t(0);
		sb[i] = ok ? band[base0 + size_t(i) - 1] : uint8_t(0);
	}
	__syncthreads();
	const int lane = int(threadIdx.x & 63u);
	const int w = int(threadIdx.x >> 6);
	uint32_t flags = 0;  // per j, 4 bits: 1 refine, 2 partial run head, 4 kept family head, 8 unrefine head
	uint32_t runk = 0;   // per j, 4 bits: the run length of a partial run head
	unsigned cr = 0, cp = 0, ck = 0, cu = 0;
#pragma unroll
	for (int j = 0; j < kJ; j++) {
		const int li = 64 * kJ * w + 64 * j + lane;  // block-local slot; its entries li + 1 (own), li (before)
		const size_t sj = base0 + size_t(li);
		if (sj >= n) continue;
		const uint64_t p = sp[li + 1];
		const uint64_t prev = sp[li];
		const uint32_t bj = sb[li + 1];
		const int lvl = p == ~uint64_t(0) ? 0 : map_level(m, p) + 1;
		uint32_t what = 0;
		if (bj == 2 && lvl < int(m.R)) {
			what |= 1;
			cr++;
		}
		if (lvl > 0 && prev != p) {
			uint32_t k = 1;
			bool keep = bj >= 1;
			for (int q = 1; q < 8; q++) {
				if (sp[li + 1 + q] != p) break;
				keep = keep || sb[li + 1 + q] >= 1;
				k++;
			}
			bool whole = !solo;  // every child of p is a leaf (some held elsewhere)
			// every child of p a local leaf (a family split between the inner
			// and outer runs): decided here, by the run headed by the first child
			// (-1: not local, 1: this run decides, 2: another run does)
			int local = 0;
			bool keep8 = false;
			if (k < 8 && whole) {
				// the slot just before or just after the run holding a child of a
				// sibling (a grandchild of p) settles it without lookups
				const uint64_t after = sp[li + 1 + int(k)];
				auto grandchild_of_p = [&](uint64_t par_of_slot) {
					return par_of_slot != ~uint64_t(0) && map_level(m, par_of_slot) > 0 && map_parent(m, par_of_slot) == p;
				};
				if (grandchild_of_p(prev) || grandchild_of_p(after)) whole = false;
			}
			if (k < 8 && whole) {
				uint64_t ch[8];
				map_all_children(m, p, ch);
				local = 1;
				for (int i = 0; i < 8; i++) {
					int32_t o = -1, sl = -1;
					if (!dm_lookup(M, ch[i], o, sl)) {
						whole = false;
						break;
					}
					if (o != rank || sl < 0 || size_t(sl) >= n) local = -1;
					else keep8 = keep8 || band[sl] >= 1;
				}
				if (local == 1 && ids[sj] != ch[0]) local = 2;
			}
			if (k < 8 && whole && local == 2) {
				// counted by the run of the first child
			} else if (k < 8 && whole && local == 1) {
				// 2679-2733 as decide() on the host: a kept family is counted, a
				// whole local family not kept is unrefined (its first child's id)
				if (keep8) ck++;
				else {
					what |= 8;
					cu++;
				}
			} else if (k < 8 && !whole) {
				// a sibling has children: the family cannot be unrefined in
				// this round (unrefine_completely refuses, a dont_unrefine mark
				// changes nothing), so the host never sees it; counted as the
				// host's decide() would count it
				if (keep) ck++;
			} else if (k < 8) {
				what |= 2;
				runk |= k << (4 * j);
				cp++;
			} else if (keep) {
				ck++;
			} else {
				what |= 8;
				cu++;
			}
		}
		flags |= what << (4 * j);
	}
	const unsigned c[4] = {cr, cu, ck, cp};
	unsigned long long b[4];
	block_reserve4<BS / 64>(cnt, c, b);
	unsigned long long ar = b[0], au = b[1], ap = b[3];
#pragma unroll
	for (int j = 0; j < kJ; j++) {
		const uint32_t what = (flags >> (4 * j)) & 15u;
		if (!what) continue;
		const size_t sj = base0 + size_t(64 * kJ * w + 64 * j + lane);
		if (what & 1) ref[ar++] = ids[sj];
		if (what & 2) part[ap++] = uint32_t(sj) | (((runk >> (4 * j)) & 15u) << 28);
		if (what & 8) unref[au++] = ids[sj];
	}
}

__global__ void gather_ids_bands_kernel(const uint64_t* __restrict__ ids, const uint8_t* __restrict__ band,
                                        const uint32_t* __restrict__ at, size_t n, uint64_t* __restrict__ oid,
                                        uint8_t* __restrict__ ob) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		oid[i] = ids[at[i]];
		ob[i] = band[at[i]];
	}
}

// adapt_grid (adapter.hpp:260-290): a merged parent's density is the sum of
// its removed children's densities / 8 (children in ascending id)
__global__ void adv_parent_density_kernel(double* __restrict__ rho, const int32_t* __restrict__ parent_slot,
                                          const int32_t* __restrict__ child_idx, const double* __restrict__ removed_rho,
                                          size_t np) {
#pragma clang fp contract(off)
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < np; i += size_t(gridDim.x) * blockDim.x) {
		double acc = 0;
		for (int k = 0; k < 8; k++) acc += removed_rho[child_idx[8 * i + k]] / 8;
		rho[parent_slot[i]] = acc;
	}
}

// merged families on the device: the parent of every removed child, and
// (after the parents are sorted and deduplicated) each child's place in its
// parent's row of eight, in map_all_children order (= ascending id)
__global__ void removed_parents_kernel(MapCtx m, const uint64_t* __restrict__ rm, size_t n, uint64_t* __restrict__ par) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		par[i] = map_parent(m, rm[i]);
}

__global__ void removed_rows_kernel(MapCtx m, const uint64_t* __restrict__ rm, size_t n,
                                    const uint64_t* __restrict__ parents, size_t np, int32_t* __restrict__ cidx,
                                    int* __restrict__ err) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t x, y, z;
		const int l = map_indices(m, rm[i], x, y, z);
		const uint64_t p = map_parent(m, rm[i]);
		size_t lo = 0, hi = np;
		while (lo < hi) {
			const size_t mid = (lo + hi) / 2;
			if (parents[mid] < p) lo = mid + 1;
			else hi = mid;
		}
		if (l <= 0 || lo >= np || parents[lo] != p) {
			atomicOr(err, 1);
			continue;
		}
		const uint64_t o = uint64_t(1) << (m.R - l);  // the child's length in indices
		const int k = int((x / o) & 1u) | int(((y / o) & 1u) << 1) | int(((z / o) & 1u) << 2);
		cidx[8 * lo + size_t(k)] = int32_t(i);
	}
}

__global__ void check_rows_kernel(const int32_t* __restrict__ cidx, const int32_t* __restrict__ pslot, size_t np,
                                  size_t n_local, int* __restrict__ err) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < np; i += size_t(gridDim.x) * blockDim.x) {
		if (pslot[i] < 0 || size_t(pslot[i]) >= n_local) atomicOr(err, 2);
		for (int k = 0; k < 8; k++)
			if (cidx[8 * i + k] < 0) atomicOr(err, 4);
	}
}

// adapt_grid (adapter.hpp:294-305): velocity (solve.hpp:336-342) and lengths
// (Cartesian_Geometry get_center / get_length, dccrg_cartesian_geometry.hpp:
// 282-362) of every local cell
// (+ the block minima of adv_dt_kernel's bound over the values written, when
// dt_partial is given: the next max_time_step needs no pass of its own)
__global__ __launch_bounds__(256) void adv_reset_kernel(MapCtx m, const uint64_t* __restrict__ slot_ids, size_t n,
                                                        double s0, double s1, double l00, double l01, double l02,
                                                        double* vx, double* vy, double* vz, double* lx, double* ly,
                                                        double* lz, double* dt_partial) {
#pragma clang fp contract(off)
	__shared__ double red[256];
	const double st[3] = {s0, s1, 0.0};
	const double l0[3] = {l00, l01, l02};
	double mn = 1.7976931348623157e308;
	for (size_t s = blockIdx.x * size_t(blockDim.x) + threadIdx.x; s < n; s += size_t(gridDim.x) * blockDim.x) {
		uint64_t ind[3];
		const int lvl = map_indices(m, slot_ids[s], ind[0], ind[1], ind[2]);
		const double sf = 1.0 / double(uint64_t(1) << lvl);
		double L[3], c[2];
		for (int d = 0; d < 3; d++) L[d] = l0[d] * sf;
		for (int d = 0; d < 2; d++) c[d] = st[d] + double(ind[d]) * l0[d] / double(uint64_t(1) << m.R) + L[d] / 2;
		const double v[3] = {-c[1] + 0.5, +c[0] - 0.5, 0.0};
		vx[s] = v[0];
		vy[s] = v[1];
		vz[s] = v[2];
		lx[s] = L[0];
		ly[s] = L[1];
		lz[s] = L[2];
		if (dt_partial) {
			// adv_dt_kernel's expression on the same values
			const double a = L[0] / fabs(v[0]), b = L[1] / fabs(v[1]), cc = L[2] / fabs(v[2]);
			if (__builtin_isnormal(a)) mn = fmin(mn, a);
			if (__builtin_isnormal(b)) mn = fmin(mn, b);
			if (__builtin_isnormal(cc)) mn = fmin(mn, cc);
		}
	}
	if (!dt_partial) return;  // grid-uniform
	red[threadIdx.x] = mn;
	__syncthreads();
	for (int k = blockDim.x / 2; k > 0; k >>= 1) {
		if (threadIdx.x < k) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + k]);
		__syncthreads();
	}
	if (threadIdx.x == 0) dt_partial[blockIdx.x] = red[0];
}

}  // namespace

// ===========================================================================
void k_pack(const uint8_t* field, size_t elem, size_t off, size_t len, const int32_t* slots, size_t n, uint8_t* out,
            hipStream_t s) {
	if (!n || !len) return;
	if (off == 0 && len == elem && elem == 4)
		pack_kernel<uint32_t><<<grid_for(n, 256), 256, 0, s>>>((const uint32_t*)field, slots, n, (uint32_t*)out);
	else if (off == 0 && len == elem && elem == 8)
		pack_kernel<uint64_t><<<grid_for(n, 256), 256, 0, s>>>((const uint64_t*)field, slots, n, (uint64_t*)out);
	else
		pack_bytes_kernel<<<grid_for(n * len, 256), 256, 0, s>>>(field, elem, off, len, slots, n, out);
	HIP_CHECK(hipGetLastError());
}

void k_place(const uint8_t* in, size_t elem, size_t off, size_t len, const int32_t* slots, size_t n, uint8_t* field,
             hipStream_t s) {
	if (!n || !len) return;
	if (off == 0 && len == elem && elem == 4)
		place_kernel<uint32_t><<<grid_for(n, 256), 256, 0, s>>>((const uint32_t*)in, slots, n, (uint32_t*)field);
	else if (off == 0 && len == elem && elem == 8)
		place_kernel<uint64_t><<<grid_for(n, 256), 256, 0, s>>>((const uint64_t*)in, slots, n, (uint64_t*)field);
	else
		place_bytes_kernel<<<grid_for(n * len, 256), 256, 0, s>>>(in, elem, off, len, slots, n, field);
	HIP_CHECK(hipGetLastError());
}

void k_gol_csr(const uint32_t* state, uint32_t* out, const uint32_t* it_ptr, const int32_t* it_slot, size_t s0,
               size_t s1, hipStream_t s) {
	if (s1 <= s0) return;
	const size_t nb = (s1 - s0 + kGolRows - 1) / kGolRows;
	gol_csr_kernel<<<unsigned((nb + 7) / 8 * 8), kGolRows, 0, s>>>(state, out, it_ptr, it_slot, s0, s1);
	HIP_CHECK(hipGetLastError());
}

// false when the box does not fit the structured kernel (nx % 256 != 0)
bool k_gol_structured(const uint32_t* state, uint32_t* out, const uint64_t n[3], const int per[3], const uint32_t* lo,
                      const uint32_t* hi, hipStream_t s) {
	if (n[0] % 256 != 0 || n[0] * n[1] * n[2] >= (uint64_t(1) << 32) || n[2] == 0) return false;
	// 64 planes per z chunk, 3 planes of loads in flight per wave (r01g/r01j
	// sweeps over zc and the depth on config 2)
	const int zc = int(std::min<uint64_t>(n[2], 64));
	// two rows per wave by default (paired A/B on config 2, profiles/r06ze_gol_yr_ab.txt:
	// 0.1118 -> 0.1083 ms per sweep; four rows: 185 VGPRs, slower); DCCRGX_GOL_YR=1: v3
	static const int yr = std::getenv("DCCRGX_GOL_YR") ? std::atoi(std::getenv("DCCRGX_GOL_YR")) : 2;
	static const int ydepth = std::getenv("DCCRGX_GOL_YDEPTH") ? std::atoi(std::getenv("DCCRGX_GOL_YDEPTH")) : 2;
	if (yr == 2 || yr == 4) {
		const unsigned rows = unsigned(G3_ROWS * yr);
		const unsigned nbx = unsigned(n[0] / 256), nby = unsigned((n[1] + rows - 1) / rows),
		               nbz = unsigned((n[2] + zc - 1) / zc);
		const size_t nb = size_t(nbx) * nby * nbz;
		const unsigned grid = unsigned((nb + 7) / 8 * 8);
#define DX_GOL_YR(D, Y)                                                                                                   \
	gol_structured_yr<D, Y><<<grid, 64 * G3_ROWS, 0, s>>>(state, out, int(n[0]), int(n[1]), int(n[2]), per[0], per[1], \
	                                                      per[2], zc, nbx, nby, unsigned(nb), lo, hi)
		if (yr == 2 && ydepth == 3) DX_GOL_YR(3, 2);
		else if (yr == 2) DX_GOL_YR(2, 2);
		else if (ydepth == 1) DX_GOL_YR(1, 4);
		else DX_GOL_YR(2, 4);
#undef DX_GOL_YR
		HIP_CHECK(hipGetLastError());
		return true;
	}
	const unsigned nbx = unsigned(n[0] / 256), nby = unsigned((n[1] + G3_ROWS - 1) / G3_ROWS),
	               nbz = unsigned((n[2] + zc - 1) / zc);
	const size_t nb = size_t(nbx) * nby * nbz;
	const unsigned grid = unsigned((nb + 7) / 8 * 8);
	gol_structured_v3<DCCRGX_G3_DEPTH><<<grid, 64 * G3_ROWS, 0, s>>>(state, out, int(n[0]), int(n[1]), int(n[2]), per[0], per[1],
	                                                    per[2], zc, nbx, nby, unsigned(nb), lo, hi);
	HIP_CHECK(hipGetLastError());
	return true;
}

void k_advection(const double* const f[7], double* rho_out, const uint32_t* face_ptr, const int32_t* face_ent,
                 size_t s0, size_t s1, double dt, hipStream_t s) {
	// the untiled gather over the face CSR: runs whose tiles exceed the
	// pipelined tile kernel's capacities
	if (s1 <= s0) return;
	advection_kernel<<<grid_for(s1 - s0, 256, 256u * 64u), 256, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5], f[6],
	                                                                    rho_out, face_ptr, face_ent, s0, s1, dt);
	HIP_CHECK(hipGetLastError());
}

// Tiled advection sweep of one run (0 inner, 1 outer): the regular tiles with
// advection_regular_pp_kernel, every other tile with advection_tiles_pp_kernel,
// both persistent with two blocks per CU (r01k: one / two tiles in flight per
// block, dynamic tickets and a second stream for the general sweep all tie
// or lose against this schedule).
void k_advection_ell(const double* const f[7], double* rho_out, const int32_t* ell, const int32_t* fine, size_t s0,
                     size_t s1, double dt, hipStream_t s, const BandArgs* bands) {
	if (s1 <= s0) return;
	static const bool plain = std::getenv("DCCRGX_ELL_LDS") && std::atoi(std::getenv("DCCRGX_ELL_LDS")) == 0;
	if (bands)
		advection_ell_lds_kernel<true><<<grid_for(s1 - s0, 256, 256u * 64u), 256, 0, s>>>(
		    f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out, ell, fine, s0, s1, dt, *bands);
	else if (plain)
		advection_ell_kernel<<<grid_for(s1 - s0, 256, 256u * 64u), 256, 0, s>>>(f[0], f[1], f[2], f[3], f[4], f[5],
		                                                                     f[6], rho_out, ell, fine, s0, s1, dt);
	else
		advection_ell_lds_kernel<false><<<grid_for(s1 - s0, 256, 256u * 64u), 256, 0, s>>>(
		    f[0], f[1], f[2], f[3], f[4], f[5], f[6], rho_out, ell, fine, s0, s1, dt, BandArgs{});
	HIP_CHECK(hipGetLastError());
}

void k_advection_tiles(const double* const f[7], double* rho_out, Grid& g, int run, double dt, hipStream_t s,
                       const double* nbrec) {
	const size_t n_reg = g.tcount[run], n_irr = g.tcount[2 + run];
	const AdvPtrs P{{f[0], f[4], f[5], f[6], f[1], f[2], f[3]}};
	if (n_irr && !g.tmeta.n) {
		// a tile beyond the pipelined kernel's capacities: the whole run untiled
		const size_t s0 = run == 0 ? 0 : g.n_inner, s1 = run == 0 ? g.n_inner : g.n_local;
		k_advection(f, rho_out, g.face_ptr.p, g.face_ent.p, s0, s1, dt, s);
		return;
	}
#if DCCRGX_FUSED_SWEEP
	if (g.tfused.n && g.tfused_n[run]) {
		const uint32_t* meta = g.tfused.p + 8 * (run == 0 ? 0 : g.tfused_n[0]);
		const size_t nt = g.tfused_n[run];
		const uint32_t ecap = uint32_t(g.max_ext);
		const size_t lgen = size_t(7) * (512 + ecap) * sizeof(double) + size_t(2) * 512 * sizeof(uint32_t);
		const size_t lreg = (size_t(7) * (512 + 6 * 64) + 3 * 512 + 3 * 64) * sizeof(double);
		const unsigned nblk = unsigned(std::min<size_t>(size_t(256) * 2, (nt + 7) / 8 * 8));
		advection_fused_kernel<4><<<nblk, 512, std::max(lgen, lreg), s>>>(
		    P, rho_out, g.tell.p, uint32_t(g.n_local + 1), g.ext_pk.p, g.tfine.p, meta, uint32_t(nt), ecap, dt);
		HIP_CHECK(hipGetLastError());
		return;
	}
#endif
	if (n_reg) {
		const RegTileMeta* meta = g.tregmeta.p + (run == 0 ? 0 : g.tcount[0]);
		static const bool reg3 = std::getenv("DCCRGX_REG3") && std::atoi(std::getenv("DCCRGX_REG3")) == 1;
		if (reg3) {
			const unsigned nblk = unsigned(std::min<size_t>(size_t(256) * 3, (n_reg + 7) / 8 * 8));
			advection_regular3_kernel<6><<<nblk, 512, 0, s>>>(P, rho_out, meta, uint32_t(n_reg), dt);
		} else {
			const unsigned nblk = unsigned(std::min<size_t>(size_t(256) * 2, (n_reg + 7) / 8 * 8));
			if (nbrec)
				advection_regular_pp_kernel<4, true><<<nblk, 512, 0, s>>>(P, rho_out, meta, uint32_t(n_reg), dt, nbrec,
				                                                          g.n_slots);
			else
				advection_regular_pp_kernel<4, false><<<nblk, 512, 0, s>>>(P, rho_out, meta, uint32_t(n_reg), dt, nullptr,
				                                                           0);
		}
		HIP_CHECK(hipGetLastError());
	}
	if (n_irr) {
		const TileMeta* meta = reinterpret_cast<const TileMeta*>(g.tmeta.p) + (run == 0 ? 0 : g.tcount[2]);
		const uint32_t ecap = uint32_t(g.max_ext);
		// DCCRGX_FACE_ONCE=1: in-tile same-level faces evaluated once (lost
		// its paired A/B: 0.184 -> 0.194 ms per sweep, the extra barrier costs
		// more than the halved flux arithmetic)
		static const char* fo = std::getenv("DCCRGX_FACE_ONCE");
		const bool once = fo && fo[0] == '1';
		const size_t lds = size_t(7) * (512 + ecap) * sizeof(double) + size_t(2) * 512 * sizeof(uint32_t) +
		                   (once ? size_t(3) * 512 * (sizeof(double) + 1) : 0);
		const unsigned nblk = unsigned(std::min<size_t>(size_t(256) * 2, (n_irr + 7) / 8 * 8));
		const uint32_t tp = uint32_t(g.n_local + 1);
		if (nbrec && once)
			advection_tiles_pp_kernel<4, true, true><<<nblk, 512, lds, s>>>(P, rho_out, g.tell.p, tp, g.ext_pk.p, g.tfine.p,
			                                                                meta, uint32_t(n_irr), ecap, dt, nbrec,
			                                                                g.n_slots);
		else if (nbrec)
			advection_tiles_pp_kernel<4, true, false><<<nblk, 512, lds, s>>>(P, rho_out, g.tell.p, tp, g.ext_pk.p,
			                                                                 g.tfine.p, meta, uint32_t(n_irr), ecap, dt,
			                                                                 nbrec, g.n_slots);
		else if (once)
			advection_tiles_pp_kernel<4, false, true><<<nblk, 512, lds, s>>>(P, rho_out, g.tell.p, tp, g.ext_pk.p,
			                                                                 g.tfine.p, meta, uint32_t(n_irr), ecap, dt,
			                                                                 nullptr, 0);
		else
			advection_tiles_pp_kernel<4, false, false><<<nblk, 512, lds, s>>>(P, rho_out, g.tell.p, tp, g.ext_pk.p,
			                                                                  g.tfine.p, meta, uint32_t(n_irr), ecap, dt,
			                                                                  nullptr, 0);
		HIP_CHECK(hipGetLastError());
	}
}

void k_nbrec(const double* const f[7], size_t n, double* r, hipStream_t s) {
	if (!n) return;
	nbrec_kernel<<<grid_for(n, 256), 256, 0, s>>>(f[4], f[5], f[6], f[1], f[2], f[3], n, r);
	HIP_CHECK(hipGetLastError());
}

void k_adv_dt(const double* const f[7], size_t n, double* partial, size_t nblocks, hipStream_t s) {
	adv_dt_kernel<<<unsigned(nblocks), 256, 0, s>>>(f[1], f[2], f[3], f[4], f[5], f[6], n, partial);
	HIP_CHECK(hipGetLastError());
}

namespace {
// the minimum of n partial minima into out[0] (one block; fmin is exact, so
// the order does not matter)
__global__ __launch_bounds__(256) void min_partials_kernel(const double* __restrict__ part, size_t n,
                                                           double* __restrict__ out) {
	__shared__ double red[256];
	double mn = 1.7976931348623157e308;
	for (size_t i = threadIdx.x; i < n; i += 256) mn = fmin(mn, part[i]);
	red[threadIdx.x] = mn;
	__syncthreads();
	for (int k = 128; k > 0; k >>= 1) {
		if (int(threadIdx.x) < k) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + k]);
		__syncthreads();
	}
	if (threadIdx.x == 0) out[0] = red[0];
}
}  // namespace

void k_min_partials(const double* partial, size_t n, double* out, hipStream_t s) {
	min_partials_kernel<<<1, 256, 0, s>>>(partial, n, out);
	HIP_CHECK(hipGetLastError());
}

void k_adv_bands(const MapCtx& m, const double* rho, const FaceView& F, const uint8_t* lvl8, size_t n,
                 double diff_increase, double diff_threshold, double unrefine_sensitivity, uint8_t* band,
                 hipStream_t s) {
	if (!n) return;
	adv_bands_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, rho, F.ell, F.fine, lvl8, F.slot_ids, n, diff_increase,
	                                                  diff_threshold, unrefine_sensitivity, band);
	HIP_CHECK(hipGetLastError());
}

// adapt_grid's merged parents (adapter.hpp:260-290) from the removed store's
// ids `rm` (store order): parents grouped, their eight children in ascending
// id, the parents' local slots, then the mean density
void k_adv_merge_parents(const MapCtx& m, const DevMesh& dm, size_t n_local, LazyIds& rm, double* rho,
                         const double* removed_rho, hipStream_t s, const uint64_t* parents, size_t np_given) {
	if (rm.empty()) return;
	const size_t n = rm.size();
	DBuf<uint64_t> up, par;
	const uint64_t* rm_dev = rm.dev();
	if (!rm_dev) {
		upload(up, rm.host(s), s);
		rm_dev = up.p;
	}
	size_t np = np_given;
	const uint64_t* parp = parents;
	if (!(parents && np * 8 == n)) {
		// the parents of the removed cells (the families' parents as
		// stop_refining merged them, when given: sorted and unique, and
		// removed_rows / check_rows below still verify every child maps to one)
		par.alloc(n);
		removed_parents_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, rm_dev, n, par.p);
		HIP_CHECK(hipGetLastError());
		np = sort_unique_u64(par.p, n, s, map_id_bits(m));
		parp = par.p;
	}
	DX_REQUIRE(np * 8 == n, "a merged family's removed children are incomplete");
	DBuf<int32_t> cidx, pslot;
	DBuf<int> err;
	cidx.alloc(8 * np);
	pslot.alloc(np);
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(cidx.p, 0xff, 8 * np * sizeof(int32_t), s));
	HIP_CHECK(hipMemsetAsync(err.p, 0, sizeof(int), s));
	removed_rows_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, rm_dev, n, parp, np, cidx.p, err.p);
	HIP_CHECK(hipGetLastError());
	k_lookup_slots(parp, np, dm, pslot.p, err.p, s);  // a missing parent sets err too
	check_rows_kernel<<<grid_for(np, 256), 256, 0, s>>>(cidx.p, pslot.p, np, n_local, err.p);
	HIP_CHECK(hipGetLastError());
	int h = 0;
	d2h_small(&h, err.p, sizeof(int), s);
	DX_REQUIRE(h == 0, "merged parent is not local or a removed child's payload is missing");
	k_adv_parent_density(rho, pslot.p, cidx.p, removed_rho, np, s);
}

void k_adv_parent_density(double* rho, const int32_t* parent_slot, const int32_t* child_idx, const double* removed_rho,
                          size_t np, hipStream_t s) {
	if (!np) return;
	adv_parent_density_kernel<<<grid_for(np, 256), 256, 0, s>>>(rho, parent_slot, child_idx, removed_rho, np);
	HIP_CHECK(hipGetLastError());
}

static void k_gather_ids_bands(const uint64_t* ids, const uint8_t* band, const uint32_t* at, size_t n, uint64_t* oid,
                               uint8_t* ob, hipStream_t s) {
	gather_ids_bands_kernel<<<grid_for(n, 256), 256, 0, s>>>(ids, band, at, n, oid, ob);
	HIP_CHECK(hipGetLastError());
}

AdvRequests k_adv_requests(const MapCtx& m, const DevMesh& dm, const uint64_t* slot_ids, const uint8_t* band, size_t n,
                           bool solo, int rank, hipStream_t s) {
	AdvRequests out;
	if (!n) return out;
	DX_REQUIRE(n < (size_t(1) << 28), "too many local cells for the request runs");
	DBuf<uint64_t> ref, unref;
	DBuf<uint32_t> part;
	DBuf<unsigned long long> cnt;
	ref.alloc(n);
	unref.alloc(n / 8 + 1);
	part.alloc(n);
	cnt.alloc(4);
	HIP_CHECK(hipMemsetAsync(cnt.p, 0, 4 * sizeof(unsigned long long), s));
	// 512 threads (4096 slots, 37 KB of LDS, four blocks per CU): a config-3
	// step's ~2100 blocks end in a shorter partial last round than 1024's
	// ~1050 two-per-CU blocks (122 -> 92 us; r06zj_requests_bs_ab.txt).
	// DCCRGX_REQ_BS=256 / 1024: the other sizes measured
	const char* rb = std::getenv("DCCRGX_REQ_BS");
	const int bs = rb && *rb ? std::atoi(rb) : 512;
	if (bs == 256)
		adv_requests_kernel<256><<<unsigned((n + 256 * 8 - 1) / (256 * 8)), 256, 0, s>>>(m, dm, slot_ids, band, n, solo,
		                                                                                rank, ref.p, unref.p, part.p, cnt.p);
	else if (bs == 512)
		adv_requests_kernel<512><<<unsigned((n + 512 * 8 - 1) / (512 * 8)), 512, 0, s>>>(m, dm, slot_ids, band, n, solo,
		                                                                                rank, ref.p, unref.p, part.p, cnt.p);
	else
		adv_requests_kernel<1024><<<unsigned((n + 1024 * 8 - 1) / (1024 * 8)), 1024, 0, s>>>(m, dm, slot_ids, band, n, solo,
		                                                                                    rank, ref.p, unref.p, part.p, cnt.p);
	HIP_CHECK(hipGetLastError());
	unsigned long long h[4];
	d2h_small(h, cnt.p, sizeof(h), s);
	// ascending ids (the lists the host merges and stop_refining sorts), sorted
	// here before they leave the device
	sort_u64(ref.p, size_t(h[0]), s, map_id_bits(m));
	sort_u64(unref.p, size_t(h[1]), s, map_id_bits(m));
	// the three lists gathered on the device and read at once
	const size_t b0 = 8 * size_t(h[0]), b1 = 8 * size_t(h[1]), b3 = 4 * size_t(h[3]);
	std::vector<uint32_t> runs(static_cast<size_t>(h[3]));
	out.refine.resize(size_t(h[0]));
	out.unrefine.resize(size_t(h[1]));
	if (b0 + b1 + b3) {
		DBuf<uint8_t> stage;
		stage.alloc(b0 + b1 + b3);
		if (b0) HIP_CHECK(hipMemcpyAsync(stage.p, ref.p, b0, hipMemcpyDeviceToDevice, s));
		if (b1) HIP_CHECK(hipMemcpyAsync(stage.p + b0, unref.p, b1, hipMemcpyDeviceToDevice, s));
		if (b3) HIP_CHECK(hipMemcpyAsync(stage.p + b0 + b1, part.p, b3, hipMemcpyDeviceToDevice, s));
		const std::vector<uint8_t> hb = download(stage.p, b0 + b1 + b3, s);
		if (b0) std::memcpy(out.refine.data(), hb.data(), b0);
		if (b1) std::memcpy(out.unrefine.data(), hb.data() + b0, b1);
		if (b3) std::memcpy(runs.data(), hb.data() + b0 + b1, b3);
	}
	out.refine_dev = std::move(ref);
	out.unrefine_dev = std::move(unref);
	out.kept = size_t(h[2]);
	// the partial runs' members: ids and bands
	for (uint32_t r : runs) {
		const size_t s0 = r & ((1u << 28) - 1u), k = r >> 28;
		out.part_slot.push_back(s0);
		out.part_len.push_back(uint32_t(k));
	}
	if (!runs.empty()) {
		std::vector<uint32_t> mem;
		for (size_t i = 0; i < out.part_slot.size(); i++)
			for (uint32_t j = 0; j < out.part_len[i]; j++) mem.push_back(uint32_t(out.part_slot[i] + j));
		DBuf<uint32_t> dm;
		upload(dm, mem, s);
		DBuf<uint64_t> gid;
		DBuf<uint8_t> gb;
		gid.alloc(mem.size());
		gb.alloc(mem.size());
		k_gather_ids_bands(slot_ids, band, dm.p, mem.size(), gid.p, gb.p, s);
		out.part_ids = download(gid.p, mem.size(), s);
		out.part_bands = download(gb.p, mem.size(), s);
	}
	return out;
}

size_t k_adv_reset(const MapCtx& m, const uint64_t* slot_ids, size_t n, const double start[3], const double l0[3],
                   double* const f[7], hipStream_t s, double* dt_partial) {
	if (!n) return 0;
	const unsigned nb = grid_for(n, 256, kDtPartials);
	adv_reset_kernel<<<nb, 256, 0, s>>>(m, slot_ids, n, start[0], start[1], l0[0], l0[1], l0[2], f[1], f[2], f[3], f[4],
	                                    f[5], f[6], dt_partial);
	HIP_CHECK(hipGetLastError());
	return nb;
}

size_t k_adv_candidates(const MapCtx& m, const double* rho, const FaceView& F, const uint8_t* lvl8, size_t n,
                        double diff_increase, double diff_threshold, uint64_t* out, hipStream_t s) {
	if (!n) return 0;
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, sizeof(unsigned long long), s));
	adv_candidates_kernel<<<grid_for(n, 256), 256, 0, s>>>(m, rho, F.ell, F.fine, lvl8, F.slot_ids, n, diff_increase,
	                                                       diff_threshold, out, ctr.p);
	HIP_CHECK(hipGetLastError());
	unsigned long long h = 0;
	d2h_small(&h, ctr.p, sizeof(h), s);
	return size_t(h);
}

}  // namespace dccrgx
