// The reference's own advection solver run through the drop-in facade.
//
// A repo-owned main replicating tests/advection/2d.cpp:87-127 (defaults),
// 252-292 (initialize, balance at start, pre-refine to the maximum level,
// time step) and 321-350 + 390 (one step: start the halo, fluxes of inner
// cells, wait for receives, fluxes of outer cells, wait for sends, apply)
// with adapt_n = 0 (frozen mesh), on a 3-D base grid
// with x and y periodic.  The solver itself is the reference's code: this
// file is compiled with the reference's tests/advection directory on the
// include path and includes its cell.hpp, initialize.hpp, solve.hpp and
// adapter.hpp unmodified; their "dccrg.hpp" resolves to the facade
// (include/dccrg.hpp).  Nothing of the reference is copied into the repo;
// __graft_entry__.build_examples() compiles this only where /root/reference
// exists and only the binary (examples/bin/ref_advection) travels.
//
// usage: mpiexec -n P ref_advection nx ny nz max_ref_lvl steps out_prefix [balance]
//   writes <out_prefix>.prerefined.<rank> (after pre-refinement and the last
//   initialize) and <out_prefix>.final.<rank> (after `steps` steps): a header
//   {uint64 magic, uint64 n, double dt} then n records {uint64 id, double
//   data[9]} of the rank's local cells in ascending id.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <iomanip>
#include <sstream>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"
#include "cell.hpp"
#include "initialize.hpp"
#include "solve.hpp"
#include "adapter.hpp"

bool Cell::transfer_all_data = false;

using Grid = dccrg::Dccrg<Cell, dccrg::Cartesian_Geometry, std::tuple<Center>, std::tuple<Is_Local>>;

static void dump(const Grid& grid, const std::string& path, double dt) {
	std::vector<std::pair<uint64_t, const Cell*>> c;
	for (const auto& cell : grid.local_cells()) c.push_back({cell.id, cell.data});
	std::sort(c.begin(), c.end());
	FILE* f = std::fopen(path.c_str(), "wb");
	if (!f) {
		std::fprintf(stderr, "cannot write %s\n", path.c_str());
		std::abort();
	}
	const uint64_t magic = 0x6164766563746e31ull, n = c.size();
	std::fwrite(&magic, 8, 1, f);
	std::fwrite(&n, 8, 1, f);
	std::fwrite(&dt, 8, 1, f);
	for (const auto& e : c) {
		std::fwrite(&e.first, 8, 1, f);
		std::fwrite(e.second->data.data(), 8, 9, f);
	}
	std::fclose(f);
}

int main(int argc, char* argv[]) {
	if (MPI_Init(&argc, &argv) != MPI_SUCCESS) std::abort();
	if (argc < 7) {
		std::fprintf(stderr, "usage: %s nx ny nz max_ref_lvl steps out_prefix [balance]\n", argv[0]);
		MPI_Finalize();
		return EXIT_FAILURE;
	}
	MPI_Comm comm = MPI_COMM_WORLD;
	int rank = 0;
	MPI_Comm_rank(comm, &rank);
	const std::array<uint64_t, 3> length{{std::strtoull(argv[1], nullptr, 10), std::strtoull(argv[2], nullptr, 10),
	                                      std::strtoull(argv[3], nullptr, 10)}};
	const int max_ref_lvl = std::atoi(argv[4]);
	const int steps = std::atoi(argv[5]);
	const std::string out = argv[6];
	const bool balance = argc > 7 && std::atoi(argv[7]) != 0;

	// 2d.cpp:87-127 defaults
	const double relative_diff = 0.025, diff_threshold = 0.25, unrefine_sensitivity = 0.5, cfl = 0.5;
	{
		Grid grid;
		dccrg::Cartesian_Geometry::Parameters geom_params;
		grid.set_neighborhood_length(0).set_maximum_refinement_level(max_ref_lvl).set_load_balancing_method("RCB");
		grid.set_initial_length(length).set_periodic(true, true, false);
		for (int d = 0; d < 3; d++) {
			geom_params.start[size_t(d)] = 0;
			geom_params.level_0_cell_length[size_t(d)] = 1.0 / double(length[size_t(d)]);
		}
		grid.initialize(comm).set_geometry(geom_params);
		if (balance) grid.balance_load();

		// 2d.cpp:258-292
		Cell::transfer_all_data = true;
		initialize(grid);
		std::unordered_set<uint64_t> cells_to_refine, cells_not_to_unrefine, cells_to_unrefine;
		uint64_t created = 0, removed = 0;
		for (int ref_lvl = 0; ref_lvl < max_ref_lvl; ref_lvl++) {
			check_for_adaptation(relative_diff / grid.get_maximum_refinement_level(), diff_threshold,
			                     unrefine_sensitivity, cells_to_refine, cells_not_to_unrefine, cells_to_unrefine, grid);
			const auto adapted = adapt_grid(cells_to_refine, cells_not_to_unrefine, cells_to_unrefine, grid);
			created += adapted.first;
			removed += adapted.second;
			initialize(grid);
		}
		Cell::transfer_all_data = false;
		double dt = max_time_step(comm, grid);
		dump(grid, out + ".prerefined." + std::to_string(rank), dt);

		// 2d.cpp:321-350, 390 with adapt_n = 0
		for (int step = 0; step < steps; step++) {
			grid.start_remote_neighbor_copy_updates();
			calculate_fluxes(cfl * dt, true, grid);
			grid.wait_remote_neighbor_copy_update_receives();
			calculate_fluxes(cfl * dt, false, grid);
			grid.wait_remote_neighbor_copy_update_sends();
			apply_fluxes(grid);
		}
		dump(grid, out + ".final." + std::to_string(rank), dt);

		uint64_t n = 0, total = 0;
		for (const auto& cell : grid.local_cells()) (void)cell, n++;
		MPI_Reduce(&n, &total, 1, MPI_UINT64_T, MPI_SUM, 0, comm);
		if (rank == 0)
			std::printf("ref_advection cells %llu created %llu removed %llu steps %d dt %.17g\n",
			            (unsigned long long)total, (unsigned long long)created, (unsigned long long)removed, steps, dt);
	}
	MPI_Finalize();
	return EXIT_SUCCESS;
}
