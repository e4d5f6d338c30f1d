// Poisson BiCG of the reference's tests/poisson/poisson_solve.hpp
// (Poisson_Solve::solve 251-522, solve_failsafe 531-634) on device-resident
// SoA fields.  Every per-cell loop of the reference is a grid-wide kernel over
// the local slots; the three global sums per iteration (p1.A.p0 and the
// residual, then r0.r1) are deterministic two-level reductions whose final
// stage also evaluates the reference's scalar control flow (alpha, beta,
// saving the best solution, the stop tests) on the device, so an iteration
// is a chain of kernels with no host round trip.  Bandwidth-bound; no MFMA.
//
// Per-cell arithmetic follows the reference expression by expression with
// contraction off, so per-cell results equal the reference's for the same
// inputs; only the global sums differ in summation order.
#include <cfloat>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

constexpr int PO_SOLVE = 0, PO_BOUNDARY = 1, PO_SKIP = 2;  // poisson_solve.hpp:146-150
constexpr int BS = 256;

// logical block of a launch whose blocks are dealt round-robin to the 8 XCDs:
// XCD x sweeps the contiguous x-th eighth of the slots, so the +-y / +-z
// neighbors a block gathers were loaded into the same XCD's L2 shortly before
__device__ __forceinline__ unsigned xcd_block() {
	const unsigned nb = gridDim.x, b = blockIdx.x;
	return (b & 7u) * (nb >> 3) + (b >> 3);
}

// block sum of up to two values in a fixed order (wave64 shuffles, then LDS)
template <int K>
__device__ __forceinline__ void block_sum_store(double (&v)[K], double* out) {
	__shared__ double red[K][BS / 64];
#pragma unroll
	for (int k = 0; k < K; k++)
		for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_down(v[k], o, 64);
	const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	if (lane == 0)
#pragma unroll
		for (int k = 0; k < K; k++) red[k][w] = v[k];
	__syncthreads();
	if (threadIdx.x == 0) {
#pragma unroll
		for (int k = 0; k < K; k++) {
			double s = 0;
			for (int i = 0; i < BS / 64; i++) s += red[k][i];
			out[K * blockIdx.x + k] = s;
		}
	}
}

// cache_system_info 827-971 + set_scaling_factor 696-819 for one local slot.
// cls: classification (0 solve, 1 boundary, 2 skip) of every slot (remote
// copies hold their owners' values); face_ell / face_fine: the unfiltered face
// table (dccrgx_internal.hpp); po_ell / po_fine: the same table with the
// entries the reference drops (skip neighbors, boundary-boundary pairs) set
// to -1.
__global__ void po_cache_kernel(MapCtx m, double l0x, double l0y, double l0z, const uint64_t* __restrict__ slot_ids,
                                const int32_t* __restrict__ cls, const int32_t* __restrict__ face_ell,
                                const int32_t* __restrict__ face_fine, size_t n, int32_t* __restrict__ po_ell,
                                int32_t* __restrict__ po_fine, int32_t* __restrict__ type, PoArrays a) {
#pragma clang fp contract(off)
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	if (s >= n) return;
	const int t = cls[s];
	int32_t row[6] = {-1, -1, -1, -1, -1, -1};
	const double l0[3] = {l0x, l0y, l0z};
	double f6[6] = {0, 0, 0, 0, 0, 0}, sf = 0;
	int out_type = t;
	if (t != PO_SKIP) {
		const int lvl = map_level(m, slot_ids[s]);
		const double sc = 1.0 / double(uint64_t(1) << lvl);  // Cartesian get_length (geometry 282-304)
		double ch[3];
		for (int d = 0; d < 3; d++) ch[d] = (l0[d] * sc) / 2.0;
		// offsets toward the +/- neighbor of each dimension (716-723)
		double pos[3], neg[3];
		for (int d = 0; d < 3; d++) {
			pos[d] = +2 * ch[d];
			neg[d] = -2 * ch[d];
		}
		auto keep = [&](int32_t nslot) {
			const int nt = cls[nslot];
			return nt != PO_SKIP && !(t == PO_BOUNDARY && nt == PO_BOUNDARY);  // 922-931
		};
		auto note = [&](int dir, int32_t nslot) {  // 725-762
			const int nl = map_level(m, slot_ids[nslot]);
			const double nsc = 1.0 / double(uint64_t(1) << nl);
			const int d = dir >> 1;
			const double nh = (l0[d] * nsc) / 2.0;
			if (dir & 1) pos[d] = ch[d] + nh;
			else neg[d] = -1.0 * (ch[d] + nh);
		};
		int count = 0;
		for (int dir = 0; dir < 6; dir++) {
			const int32_t e = face_ell[6 * s + dir];
			if (e >= 0) {
				if (keep(e)) {
					row[dir] = e;
					note(dir, e);
				}
			} else if (e < -1) {
				const size_t k = size_t(-2 - e);
				bool any = false;
				for (int j = 0; j < 4; j++) {
					const int32_t nsl = face_fine[4 * k + j];
					const bool kp = keep(nsl);
					po_fine[4 * k + j] = kp ? nsl : -1;
					if (kp) {
						any = true;
						note(dir, nsl);
					}
				}
				if (any) row[dir] = e;
			}
			if (row[dir] != -1) count++;
		}
		if (count == 0) {
			out_type = PO_SKIP;  // 953-957
		} else {
			double tot[3];
			for (int d = 0; d < 3; d++) tot[d] = pos[d] - neg[d];  // 764-767
			for (int dir = 0; dir < 6; dir++) {
				if (row[dir] == -1) continue;
				const int d = dir >> 1;
				if (dir & 1) f6[dir] = +2.0 / (pos[d] * tot[d]);
				else f6[dir] = -2.0 / (neg[d] * tot[d]);
			}
			// 809-816: - f_x_pos - f_x_neg - f_y_pos - f_y_neg - f_z_pos - f_z_neg
			sf = -f6[1] - f6[0] - f6[3] - f6[2] - f6[5] - f6[4];
		}
	}
	for (int dir = 0; dir < 6; dir++) po_ell[6 * s + dir] = row[dir];
	type[s] = out_type;
	a.sf[s] = sf;
	for (int dir = 0; dir < 6; dir++) a.f[dir][s] = f6[dir];
}

// A . x for one cell over its kept face neighbors, in the reference's face
// order; the neighbor factor is this cell's own f in the face direction, /4
// for a finer neighbor (332-337).  x is p0 (290-339) or the solution
// (initialize_solver 996-1036, which subtracts instead of adds).
template <bool SUBTRACT>
__device__ __forceinline__ double po_apply_row(const PoArrays& a, size_t s, double acc, const double* __restrict__ x) {
#pragma clang fp contract(off)
	// the six face entries, their factors and the same-size / coarser
	// neighbors' values are gathered together before the ordered sum
	int32_t ev[6];
	double fv[6], xv[6];
#pragma unroll
	for (int dir = 0; dir < 6; dir++) ev[dir] = a.ell[6 * s + dir];
#pragma unroll
	for (int dir = 0; dir < 6; dir++) {
		fv[dir] = ev[dir] != -1 ? a.f[dir][s] : 0.0;
		xv[dir] = ev[dir] >= 0 ? x[ev[dir]] : 0.0;
	}
#pragma unroll
	for (int dir = 0; dir < 6; dir++) {
		const int32_t e = ev[dir];
		if (e == -1) continue;
		double mul = fv[dir];
		if (e >= 0) {
			if (SUBTRACT) acc -= mul * xv[dir];
			else acc += mul * xv[dir];
		} else {
			mul /= 4.0;
			const size_t k = size_t(-2 - e);
			for (int j = 0; j < 4; j++) {
				const int32_t nsl = a.fine[4 * k + j];
				if (nsl < 0) continue;
				if (SUBTRACT) acc -= mul * x[nsl];
				else acc += mul * x[nsl];
			}
		}
	}
	return acc;
}

// initialize_solver 986-1051: r0 = rhs - A . solution; p0 = p1 = r1 = r0;
// partial r0 . r1
__global__ void po_init_kernel(PoArrays a, size_t n, double* part) {
#pragma clang fp contract(off)
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	double v[1] = {0};
	if (s < n && a.type[s] == PO_SOLVE) {
		double r0 = a.rhs[s] - a.sf[s] * a.sol[s];
		r0 = po_apply_row<true>(a, s, r0, a.sol);
		a.r0[s] = r0;
		a.p0[s] = r0;
		a.p1[s] = r0;
		a.r1[s] = r0;
		v[0] = r0 * r0;
	}
	block_sum_store<1>(v, part);
}

__device__ __forceinline__ bool po_idle(const PoScalars* st, unsigned max_it) {
	return st->done || st->iteration >= max_it;
}

// A . p0 (290-339), partial p1 . A.p0 (341-349) and partial residual
// sum |r0|^p over every cached cell (get_residual 677-687: the residual is
// taken from r0 before this iteration's update, so it is summed here)
__global__ void po_phase_a_kernel(PoArrays a, size_t n, double p_of_norm, unsigned max_it, const PoScalars* st,
                                  double* part) {
#pragma clang fp contract(off)
	if (po_idle(st, max_it)) return;  // grid-uniform
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	double v[2] = {0, 0};
	if (s < n) {
		const int t = a.type[s];
		if (t == PO_SOLVE) {
			const double p0 = a.p0[s];
			const double ap = po_apply_row<false>(a, s, a.sf[s] * p0, a.p0);
			a.ap0[s] = ap;
			v[0] = a.p1[s] * ap;
		}
		if (t != PO_SKIP) {
			const double r = fabs(a.r0[s]);
			v[1] = p_of_norm == 2.0 ? r * r : pow(r, p_of_norm);
		}
	}
	block_sum_store<2>(v, part);
}

// solution += alpha p0 (364-370), best = solution when the residual is the
// smallest so far (379-390); unless stopping: r0 -= alpha A.p0 (405-411),
// r1 -= alpha transpose(A).p1 (413-470, the neighbor's factor toward this
// cell), partial r0 . r1 (479-486)
__global__ void po_phase_b_kernel(PoArrays a, size_t n, const PoScalars* st, double* part) {
#pragma clang fp contract(off)
	if (st->done) return;  // grid-uniform
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	double v[1] = {0};
	if (s < n && a.type[s] == PO_SOLVE) {
		const double alpha = st->alpha;
		const double sol = a.sol[s] + alpha * a.p0[s];
		a.sol[s] = sol;
		if (st->save) a.best[s] = sol;
		if (!st->stop_b) {
			const double r0 = a.r0[s] - alpha * a.ap0[s];
			a.r0[s] = r0;
			double ap1 = a.sf[s] * a.p1[s];
			// as in po_apply_row: the six face entries, then the same-size /
			// coarser neighbors' factors (reversed direction) and p1 values
			// gathered together, then the ordered sum
			int32_t ev[6];
			double fv[6], pv[6];
#pragma unroll
			for (int dir = 0; dir < 6; dir++) ev[dir] = a.ell[6 * s + dir];
#pragma unroll
			for (int dir = 0; dir < 6; dir++) {
				fv[dir] = ev[dir] >= 0 ? (a.ft ? a.ft[size_t(dir) * n + s] : a.f[dir ^ 1][ev[dir]]) : 0.0;
				pv[dir] = ev[dir] >= 0 ? a.p1[ev[dir]] : 0.0;
			}
#pragma unroll
			for (int dir = 0; dir < 6; dir++) {
				const int32_t e = ev[dir];
				if (e == -1) continue;
				const double* __restrict__ fo = a.f[dir ^ 1];  // neighbor's factor, reversed direction
				if (e >= 0) {
					ap1 += fv[dir] * pv[dir];
				} else {
					const size_t k = size_t(-2 - e);
					for (int j = 0; j < 4; j++) {
						const int32_t nsl = a.fine[4 * k + j];
						if (nsl < 0) continue;
						double mul = fo[nsl];
						mul /= 4.0;
						ap1 += mul * a.p1[nsl];
					}
				}
			}
			const double r1 = a.r1[s] - alpha * ap1;
			a.r1[s] = r1;
			v[0] = r0 * r1;
		}
	}
	block_sum_store<1>(v, part);
}

// PoArrays::ft: per local cell and direction the single neighbor's factor in
// the reversed direction (0 where there is none or it is finer)
__global__ void po_transpose_kernel(PoArrays a, size_t n, double* __restrict__ ft) {
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	if (s >= n) return;
#pragma unroll
	for (int dir = 0; dir < 6; dir++) {
		const int32_t e = a.ell[6 * s + dir];
		ft[size_t(dir) * n + s] = e >= 0 ? a.f[dir ^ 1][e] : 0.0;
	}
}

// p0 = r0 + beta p0, p1 = r1 + beta p1 (497-504)
__global__ void po_phase_c_kernel(PoArrays a, size_t n, const PoScalars* st) {
#pragma clang fp contract(off)
	if (st->done) return;
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	if (s >= n || a.type[s] != PO_SOLVE) return;
	const double beta = st->beta;
	a.p0[s] = a.r0[s] + beta * a.p0[s];
	a.p1[s] = a.r1[s] + beta * a.p1[s];
}

// solution = best_solution (514-519)
__global__ void po_finish_kernel(PoArrays a, size_t n) {
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	if (s < n && a.type[s] == PO_SOLVE) a.sol[s] = a.best[s];
}

// solve_failsafe 555-613: next value into best_solution, partial |x - x'|
__global__ void po_jacobi_kernel(PoArrays a, size_t n, unsigned max_it, double stop_residual, const PoScalars* st,
                                 double* part) {
#pragma clang fp contract(off)
	if (st->done || st->iteration >= max_it || !(st->norm > stop_residual)) return;
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	double v[1] = {0};
	if (s < n && a.type[s] == PO_SOLVE) {
		const double inv = -1.0 / a.sf[s];
		double next = -inv * a.rhs[s];
		for (int dir = 0; dir < 6; dir++) {
			const int32_t e = a.ell[6 * s + dir];
			if (e == -1) continue;
			double mul = a.f[dir][s];
			if (e >= 0) {
				next += inv * mul * a.sol[e];
			} else {
				mul /= 4.0;
				const size_t k = size_t(-2 - e);
				for (int j = 0; j < 4; j++) {
					const int32_t nsl = a.fine[4 * k + j];
					if (nsl >= 0) next += inv * mul * a.sol[nsl];
				}
			}
		}
		a.best[s] = next;
		v[0] = fabs(a.sol[s] - next);
	}
	block_sum_store<1>(v, part);
}

// 621-626
__global__ void po_jacobi_copy_kernel(PoArrays a, size_t n, const PoScalars* st) {
	if (st->done) return;
	const size_t s = size_t(xcd_block()) * BS + threadIdx.x;
	if (s < n && a.type[s] == PO_SOLVE) a.sol[s] = a.best[s];
}

// second stage of every reduction: K sums over nb block partials in a fixed
// order -> red[0..K); then (scalar != 0, one GPU) the reference's control
// flow of that point of the iteration, or (scalar == 0) nothing: with
// several GPUs the sums are all-reduced first and po_scalar_kernel follows
constexpr int RB = 1024;  // threads of the second stage

template <int K>
__global__ __launch_bounds__(RB) void po_reduce_kernel(const double* __restrict__ part, unsigned nb, double* red,
                                                       PoScalars* st, PoParams prm, int stage, int scalar);

__device__ void po_scalar(PoScalars* st, const double* red, const PoParams& prm, int stage) {
	switch (stage) {
	case PO_STAGE_INIT:  // initialize_solver result, solve 267-272
		st->dot_r = red[0];
		st->residual_min = DBL_MAX;
		st->iteration = 0;
		st->done = 0;
		st->save = 0;
		st->stop_b = 0;
		break;
	case PO_STAGE_A: {  // 280-403
		if (st->done) return;
		if (st->iteration >= prm.max_it) {
			st->done = 1;
			return;
		}
		st->iteration++;
		const double dot_p = red[0];
		if (dot_p == 0) {  // 353-356
			st->done = 1;
			return;
		}
		st->alpha = st->dot_r / dot_p;
		const double residual = pow(red[1], 1.0 / prm.p_of_norm);
		st->residual = residual;
		st->save = st->residual_min > residual;
		if (st->save) st->residual_min = residual;
		const bool may_stop = st->iteration >= prm.min_it;
		st->stop_b = (residual <= prm.stop_residual && may_stop) ||
		             (residual >= prm.stop_increase * st->residual_min && may_stop);
		break;
	}
	case PO_STAGE_B: {  // 392-403, 472-494
		if (st->done) return;
		if (st->stop_b || st->dot_r == 0) {
			st->done = 1;
			return;
		}
		const double old = st->dot_r;
		st->dot_r = red[0];
		st->beta = st->dot_r / old;
		break;
	}
	case PO_STAGE_JACOBI_INIT:
		st->norm = DBL_MAX;
		st->iteration = 0;
		st->done = 0;
		break;
	case PO_STAGE_JACOBI: {  // 549, 615-616
		if (st->done) return;
		if (st->iteration >= prm.max_it || !(st->norm > prm.stop_residual)) {
			st->done = 1;
			return;
		}
		st->iteration++;
		st->norm = red[0];
		break;
	}
	}
}

// one block of RB threads: thread t sums partials t, t + RB, ... into four
// independent accumulators (their loads in flight together), then wave
// shuffles and the 16 wave sums in order - a fixed order for any run
template <int K>
__global__ __launch_bounds__(RB) void po_reduce_kernel(const double* __restrict__ part, unsigned nb, double* red,
                                                       PoScalars* st, PoParams prm, int stage, int scalar) {
#pragma clang fp contract(off)
	__shared__ double sh[K][RB / 64];
	double v[K];
#pragma unroll
	for (int k = 0; k < K; k++) {
		double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
		unsigned i = threadIdx.x;
		for (; i + 3 * RB < nb; i += 4 * RB) {
			a0 += part[K * i + k];
			a1 += part[K * (i + RB) + k];
			a2 += part[K * (i + 2 * RB) + k];
			a3 += part[K * (i + 3 * RB) + k];
		}
		for (; i < nb; i += RB) a0 += part[K * i + k];
		v[k] = (a0 + a1) + (a2 + a3);
		for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_down(v[k], o, 64);
	}
	const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	if (lane == 0)
#pragma unroll
		for (int k = 0; k < K; k++) sh[k][w] = v[k];
	__syncthreads();
	if (threadIdx.x == 0) {
		double r[2] = {0, 0};
		for (int k = 0; k < K; k++)
			for (int i = 0; i < RB / 64; i++) r[k] += sh[k][i];
		for (int k = 0; k < K; k++) red[k] = r[k];
		if (scalar) po_scalar(st, r, prm, stage);
	}
}

// all = P x k per-rank sums (rank-major, all-gathered): the global sums
// combined in rank order, as every rank does, then the scalar step
__global__ void po_scalar_kernel(const double* all, int P, int k, PoScalars* st, PoParams prm, int stage) {
#pragma clang fp contract(off)
	if (threadIdx.x != 0 || blockIdx.x != 0) return;
	double r[2] = {0, 0};
	for (int j = 0; j < k; j++) {
		double acc = all[j];
		for (int p = 1; p < P; p++) acc += all[p * k + j];
		r[j] = acc;
	}
	po_scalar(st, r, prm, stage);
}

inline unsigned po_blocks(size_t n) {
	size_t b = (n + BS - 1) / BS;
	b = (b + 7) / 8 * 8;  // whole rounds over the 8 XCDs (xcd_block is onto)
	return unsigned(b ? b : 8);
}

}  // namespace

unsigned k_po_blocks(size_t n) { return po_blocks(n); }

void k_po_cache(const MapCtx& m, const double l0[3], const uint64_t* slot_ids, const int32_t* cls,
                const int32_t* face_ell, const int32_t* face_fine, size_t n, int32_t* po_ell, int32_t* po_fine,
                int32_t* type, const PoArrays& a, hipStream_t s) {
	if (!n) return;
	po_cache_kernel<<<po_blocks(n), BS, 0, s>>>(m, l0[0], l0[1], l0[2], slot_ids, cls, face_ell, face_fine, n, po_ell,
	                                            po_fine, type, a);
	HIP_CHECK(hipGetLastError());
}

void k_po_transpose(const PoArrays& a, size_t n, double* ft, hipStream_t s) {
	if (!n) return;
	po_transpose_kernel<<<po_blocks(n), BS, 0, s>>>(a, n, ft);
	HIP_CHECK(hipGetLastError());
}

void k_po_phase(int phase, const PoArrays& a, size_t n, const PoParams& prm, const PoScalars* st, double* part,
                hipStream_t s) {
	const unsigned nb = po_blocks(n);
	switch (phase) {
	case PO_PHASE_INIT: po_init_kernel<<<nb, BS, 0, s>>>(a, n, part); break;
	case PO_PHASE_A: po_phase_a_kernel<<<nb, BS, 0, s>>>(a, n, prm.p_of_norm, prm.max_it, st, part); break;
	case PO_PHASE_B: po_phase_b_kernel<<<nb, BS, 0, s>>>(a, n, st, part); break;
	case PO_PHASE_C: po_phase_c_kernel<<<nb, BS, 0, s>>>(a, n, st); break;
	case PO_PHASE_FINISH: po_finish_kernel<<<nb, BS, 0, s>>>(a, n); break;
	case PO_PHASE_JACOBI: po_jacobi_kernel<<<nb, BS, 0, s>>>(a, n, prm.max_it, prm.stop_residual, st, part); break;
	case PO_PHASE_JACOBI_COPY: po_jacobi_copy_kernel<<<nb, BS, 0, s>>>(a, n, st); break;
	default: throw Error(DCCRGX_EINVAL, "invalid Poisson phase");
	}
	HIP_CHECK(hipGetLastError());
}

void k_po_reduce(int k, const double* part, unsigned nb, double* red, PoScalars* st, const PoParams& prm, int stage,
                 bool scalar, hipStream_t s) {
	if (k == 1) po_reduce_kernel<1><<<1, RB, 0, s>>>(part, nb, red, st, prm, stage, scalar ? 1 : 0);
	else po_reduce_kernel<2><<<1, RB, 0, s>>>(part, nb, red, st, prm, stage, scalar ? 1 : 0);
	HIP_CHECK(hipGetLastError());
}

void k_po_scalar(const double* all, int P, int k, PoScalars* st, const PoParams& prm, int stage, hipStream_t s) {
	po_scalar_kernel<<<1, 64, 0, s>>>(all, P, k, st, prm, stage);
	HIP_CHECK(hipGetLastError());
}

}  // namespace dccrgx
