// The reference's 1-D Poisson test (tests/poisson/poisson1d.cpp: n periodic
// cells of length 2 pi / n along x, Poisson_Solve(10, 0, 1e-7, 2, 10) on
// every cell) through the facade's device members: the right-hand side and
// the solution are device fields, the solver is poisson_cache +
// poisson_solve.  The right-hand side is read from a file (n doubles in id
// order) and the solution written to one, so a test can compare it with the
// reference solver's.
//
// usage: mpiexec -n P poisson_device n rhs.bin solution.bin
//   prints on rank 0: "cells <n> iterations <I> residual <r>"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"

struct poisson_cell {  // the reference's cell (poisson_solve.hpp Poisson_Cell), unused on the device path
	double data[2] = {0, 0};
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)data, 2, MPI_DOUBLE); }
};

int main(int argc, char* argv[])
{
	MPI_Init(&argc, &argv);
	if (argc < 4) {
		std::fprintf(stderr, "usage: poisson_device n rhs.bin solution.bin\n");
		MPI_Abort(MPI_COMM_WORLD, 1);
	}
	const uint64_t n = std::strtoull(argv[1], nullptr, 10);
	std::vector<double> rhs_all(n), sol_all(n, 0.0);
	{
		FILE* f = std::fopen(argv[2], "rb");
		if (!f || std::fread(rhs_all.data(), 8, n, f) != n) MPI_Abort(MPI_COMM_WORLD, 1);
		std::fclose(f);
	}
	int rank = 0;
	dccrg::Poisson_Result res;
	{
		dccrg::Dccrg<poisson_cell, dccrg::Cartesian_Geometry> grid;
		grid.set_initial_length({n, 1, 1}).set_neighborhood_length(0).set_maximum_refinement_level(0);
		grid.set_periodic(true, true, true).set_host_staging(false);
		grid.initialize(MPI_COMM_WORLD);
		rank = grid.get_rank();
		dccrg::Cartesian_Geometry_Parameters geom;
		geom.level_0_cell_length = {{2 * M_PI / double(n), 1, 1}};
		grid.set_geometry(geom);
		const auto rhs = grid.add_field<double>("rhs", false);
		const auto sol = grid.add_field<double>("solution", true);
		const auto slots = grid.get_slot_ids();
		const size_t nl = grid.get_number_of_local_slots();
		std::vector<double> r(nl), zero(nl, 0.0);
		std::vector<uint64_t> cells(slots.begin(), slots.begin() + ptrdiff_t(nl));
		for (size_t s = 0; s < nl; s++) r[s] = rhs_all[slots[s] - 1];
		rhs.set(r);
		sol.set(zero);
		grid.poisson_cache(rhs, sol, cells);
		res = grid.poisson_solve(10, 0, 1e-7, 2, 10);  // poisson1d.cpp:164
		const auto x = sol.get(nl);
		std::vector<double> mine(n, 0.0);
		for (size_t s = 0; s < nl; s++) mine[slots[s] - 1] = x[s];
		MPI_Reduce(mine.data(), sol_all.data(), int(n), MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD);
	}
	if (rank == 0) {
		FILE* f = std::fopen(argv[3], "wb");
		if (!f || std::fwrite(sol_all.data(), 8, n, f) != n) MPI_Abort(MPI_COMM_WORLD, 1);
		std::fclose(f);
		std::printf("cells %llu iterations %u residual %.6e\n", (unsigned long long)n, res.iterations, res.residual);
	}
	MPI_Finalize();
	return 0;
}
