// The reference's adaptive advection test (tests/advection/2d.cpp, 3-D form
// of SURVEY config 3) written against the drop-in facade with every
// per-cell loop on the GPU through the facade's device members: the seven
// per-cell values are device fields (add_field<double>), initialize.hpp,
// solve.hpp and adapter.hpp are advection_initialize / advection_step /
// advection_check_adaptation + advection_adapt, the time step is
// advection_max_time_step (MIN over processes), and the remote neighbor
// update overlaps the inner sweep as in the reference.  No Cell_Data host
// staging (set_host_staging(false)), no native() / raw C calls.
//
// usage: mpiexec -n P advection_device [base] [steps]
//   prints on rank 0: "cells <N> steps <K> created <C> removed <R> mass0 <M0> mass <M> rate <cell-updates/s>"
#include <array>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"

struct advection_cell {  // the reference's cell (tests/advection/cell.hpp), unused on the device path
	double data[7] = {0, 0, 0, 0, 0, 0, 0};
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)data, 7, MPI_DOUBLE); }
};

using Grid = dccrg::Dccrg<advection_cell, dccrg::Cartesian_Geometry>;

// sum of density x volume over the local cells, reduced on rank 0
static double total_mass(Grid& grid, const Grid::Advection_Fields& f) {
	const size_t n = grid.get_number_of_local_slots();
	const auto rho = f[0].get(n), lx = f[4].get(n), ly = f[5].get(n), lz = f[6].get(n);
	double mine = 0, all = 0;
	for (size_t i = 0; i < n; i++) mine += rho[i] * (lx[i] * ly[i] * lz[i]);
	MPI_Reduce(&mine, &all, 1, MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD);
	return all;
}

int main(int argc, char* argv[])
{
	MPI_Init(&argc, &argv);
	const uint64_t base = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 16;
	const int steps = argc > 2 ? std::atoi(argv[2]) : 20;
	const int R = 2;
	const double diff_increase = 0.025 / R, diff_threshold = 0.25, unrefine_sensitivity = 0.5;  // 2d.cpp:92-103
	int rank = 0;
	uint64_t cells = 0, created = 0, removed = 0;
	double mass0 = 0, mass = 0, seconds = 0;
	{
		Grid grid;
		grid.set_initial_length({base, base, base}).set_neighborhood_length(0).set_maximum_refinement_level(R);
		grid.set_periodic(true, true, false).set_host_staging(false);
		grid.initialize(MPI_COMM_WORLD);
		rank = grid.get_rank();
		dccrg::Cartesian_Geometry_Parameters geom;
		geom.level_0_cell_length = {{1.0 / base, 1.0 / base, 1.0 / base}};
		grid.set_geometry(geom);
		// density first, then vx, vy, vz, lx, ly, lz (the library's field order)
		const char* names[7] = {"density", "vx", "vy", "vz", "length_x", "length_y", "length_z"};
		Grid::Advection_Fields f;
		for (int k = 0; k < 7; k++) f[size_t(k)] = grid.add_field<double>(names[k], k == 0);

		// pre-refinement around the hump (2d.cpp:260-285): initialize, adapt, repeat
		for (int i = 0; i < R; i++) {
			grid.advection_initialize(f);
			grid.advection_check_adaptation(f[0], diff_increase, diff_threshold, unrefine_sensitivity);
			grid.advection_adapt(f);
		}
		grid.advection_initialize(f);
		mass0 = total_mass(grid, f);

		MPI_Barrier(MPI_COMM_WORLD);
		const auto t0 = std::chrono::high_resolution_clock::now();
		for (int step = 0; step < steps; step++) {
			const double dt = 0.5 * grid.advection_max_time_step(f);  // cfl 0.5 (2d.cpp:121-123)
			cells += grid.get_number_of_local_slots();
			grid.start_remote_neighbor_copy_updates();
			grid.advection_step(f, dt, DCCRGX_REGION_INNER);
			grid.wait_remote_neighbor_copy_update_receives();
			grid.advection_step(f, dt, DCCRGX_REGION_OUTER);
			grid.wait_remote_neighbor_copy_update_sends();
			// adapt_n = 1 (2d.cpp:118-120): the check on the pre-step densities
			grid.advection_check_adaptation(f[0], diff_increase, diff_threshold, unrefine_sensitivity);
			grid.advection_commit(f[0]);
			const auto cr = grid.advection_adapt(f);
			created += cr[0];
			removed += cr[1];
		}
		grid.synchronize();
		MPI_Barrier(MPI_COMM_WORLD);
		seconds = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
		mass = total_mass(grid, f);
	}
	uint64_t all_cells = 0, all_created = 0, all_removed = 0;
	MPI_Reduce(&cells, &all_cells, 1, MPI_UINT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
	MPI_Reduce(&created, &all_created, 1, MPI_UINT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
	MPI_Reduce(&removed, &all_removed, 1, MPI_UINT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
	if (rank == 0)
		std::printf("cells %llu steps %d created %llu removed %llu mass0 %.17g mass %.17g rate %.4e\n",
		            (unsigned long long)all_cells, steps, (unsigned long long)all_created,
		            (unsigned long long)all_removed, mass0, mass, double(all_cells) / seconds);
	MPI_Finalize();
	return 0;
}
