// ORACLE — TEST INFRASTRUCTURE ONLY.  The reference's serial 1-D Poisson
// solver (tests/poisson/reference_poisson_solve.hpp, included unmodified from
// /root/reference by `make -C oracle ref`) on the cases of
// tests/poisson/poisson1d.cpp:150-160: n = 8, 16, ..., 32768 cells of length
// 2 pi / n, rhs(i) = sin((i + 0.5) * dx).  Prints per case "n" then per cell
// the solution and the rhs as solve() left it (offset to a zero total; the
// grids of poisson1d.cpp:225-236 take that rhs), %.17g (exact round trip);
// tests/golden/make_poisson_ref.py turns them into tests/golden/poisson1d_ref.npz.
#include <cmath>
#include <cstdio>

#include "reference_poisson_solve.hpp"

int main() {
	for (size_t n = 8; n <= 32768; n *= 2) {
		const double cell_length = 2 * M_PI / n;
		Reference_Poisson_Solve reference_solver(n, cell_length);
		for (size_t i = 0; i < n; i++) reference_solver.get_rhs(i) = std::sin((i + 0.5) * cell_length);
		reference_solver.solve();
		std::printf("%zu\n", n);
		for (size_t i = 0; i < n; i++)
			std::printf("%.17g %.17g\n", reference_solver.get_solution(i), reference_solver.get_rhs(i));
	}
	return 0;
}
