// The reference's own refined game of life run through the drop-in facade.
//
// A repo-owned main in the shape of tests/game_of_life/unrefined2d.cpp:104-240
// (a 15 x 15 2-D grid with its normal along `direction`, neighborhood 1,
// maximum refinement level 1, the patterns of initialize.hpp, 25 turns; every
// turn: Refine::refine, balance_load, update_copies_of_remote_neighbors,
// get_live_neighbors on the refined grid and on an unrefined reference grid
// of the same game, whose states must agree per level-0 parent).  The game
// itself is the reference's code: this file is compiled with the reference's
// tests/game_of_life directory on the include path and includes its cell.hpp,
// initialize.hpp, refine.hpp and solve.hpp unmodified; their "dccrg.hpp"
// resolves to the facade (include/dccrg.hpp).  Nothing of the reference is
// copied into the repo; __graft_entry__.build_examples() compiles this only
// where /root/reference exists and only the binary travels.
//
// usage: mpiexec -n P ref_game_of_life_amr direction steps out_prefix
//   writes <out_prefix>.<step>.<rank> for every turn: {uint64 magic, uint64 n}
//   then n records {uint64 id, uint64 alive before the turn, uint64 alive
//   after it} of the rank's local cells in ascending id - the mesh and the
//   states get_live_neighbors (solve.hpp:37-170) saw and produced, which
//   tests/test_gpu_ref_gol_amr.py replays through the device kernels.
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"
#include "cell.hpp"
#include "initialize.hpp"
#include "refine.hpp"
#include "solve.hpp"

using Grid = dccrg::Dccrg<Cell, dccrg::Cartesian_Geometry>;

int main(int argc, char* argv[]) {
	if (MPI_Init(&argc, &argv) != MPI_SUCCESS) std::abort();
	if (argc < 4) {
		std::fprintf(stderr, "usage: %s direction steps out_prefix\n", argv[0]);
		MPI_Finalize();
		return EXIT_FAILURE;
	}
	MPI_Comm comm = MPI_COMM_WORLD;
	int rank = 0, comm_size = 1;
	MPI_Comm_rank(comm, &rank);
	MPI_Comm_size(comm, &comm_size);
	const char direction = argv[1][0];
	const int steps = std::atoi(argv[2]);
	const std::string out = argv[3];

	// unrefined2d.cpp:115-160
	const uint64_t base_length = 15;
	std::array<uint64_t, 3> grid_length{{base_length, base_length, base_length}};
	grid_length[direction == 'x' ? 0 : (direction == 'y' ? 1 : 2)] = 1;
	Grid grid, reference_grid;
	grid.set_initial_length(grid_length)
	    .set_neighborhood_length(1)
	    .set_maximum_refinement_level(1)
	    .set_load_balancing_method("RANDOM")
	    .initialize(comm);
	reference_grid.set_initial_length(grid_length)
	    .set_neighborhood_length(1)
	    .set_maximum_refinement_level(0)
	    .set_load_balancing_method("RANDOM")
	    .initialize(MPI_COMM_SELF);
	initialize(grid, grid_length[0]);
	initialize(reference_grid, grid_length[0]);

	for (int step = 0; step < steps; step++) {
		// unrefined2d.cpp:186-240
		Refine<dccrg::Cartesian_Geometry>::refine(grid, int(grid_length[0]), step, comm_size);
		grid.balance_load();
		grid.update_copies_of_remote_neighbors();
		std::vector<std::array<uint64_t, 3>> rec;
		for (const auto& cell : grid.local_cells()) rec.push_back({{cell.id, cell.data->data[0], 0}});
		get_live_neighbors(grid);
		get_live_neighbors(reference_grid);
		for (auto& r : rec) {
			const Cell* d = grid[r[0]];
			if (!d) {
				std::fprintf(stderr, "no data for cell %llu\n", (unsigned long long)r[0]);
				std::abort();
			}
			r[2] = d->data[0];
			const uint64_t ref_id = grid.get_refinement_level(r[0]) > 0 ? grid.mapping.get_parent(r[0]) : r[0];
			const Cell* rd = reference_grid[ref_id];
			if (!rd || rd->data[0] != r[2]) {
				std::fprintf(stderr, "cell %llu disagrees with the unrefined game at step %d\n",
				             (unsigned long long)r[0], step);
				std::abort();
			}
		}
		std::sort(rec.begin(), rec.end());
		const std::string path = out + "." + std::to_string(step) + "." + std::to_string(rank);
		FILE* f = std::fopen(path.c_str(), "wb");
		if (!f) {
			std::fprintf(stderr, "cannot write %s\n", path.c_str());
			std::abort();
		}
		const uint64_t magic = 0x676f6c616d723031ull, n = rec.size();
		std::fwrite(&magic, 8, 1, f);
		std::fwrite(&n, 8, 1, f);
		for (const auto& r : rec) std::fwrite(r.data(), 8, 3, f);
		std::fclose(f);
	}
	if (rank == 0) std::printf("PASSED %d turns\n", steps);
	MPI_Finalize();
	return EXIT_SUCCESS;
}
