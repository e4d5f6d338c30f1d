// Game of life on a 500 x 500 x 1 grid (BASELINE config 1's driver,
// reference examples/game_of_life.cpp), written against the drop-in facade
// include/dccrg.hpp: the same setters and start/wait halo pattern, with the
// per-cell loops replaced by the device sweep over inner/outer cells.
//
// build: hipcc -std=c++17 -I include examples/game_of_life.cpp \
//        -L dccrg_amd -ldccrgx -Wl,-rpath,$PWD/dccrg_amd -o gol
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "dccrg.hpp"

struct game_of_life_cell {
	uint32_t is_alive = 0, live_neighbor_count = 0;
};

int main(int argc, char* argv[])
{
	const int turns = argc > 1 ? std::atoi(argv[1]) : 100;
	dccrg::Dccrg<game_of_life_cell> grid;
	grid.set_initial_length({{500, 500, 1}})
		.set_neighborhood_length(1)
		.set_maximum_refinement_level(0)
		.initialize();

	// state as a device SoA field; seeded alive(id) rule
	const int state = grid.add_field<uint32_t>("is_alive", true);
	const auto cells = grid.local_cells();
	std::vector<uint32_t> alive(cells.size());
	for (size_t i = 0; i < cells.size(); i++) {
		uint64_t z = (cells[i] ^ 0x5DEECE66Dull) + 0x9E3779B97F4A7C15ull;
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
		z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
		z = z ^ (z >> 31);
		alive[i] = z < uint64_t(0.2 * 18446744073709551616.0) ? 1 : 0;
	}
	dccrg::detail::check(dccrgx_field_upload(grid.native(), state, 0, alive.size(), alive.data()));

	const auto t0 = std::chrono::high_resolution_clock::now();
	for (int turn = 0; turn < turns; turn++) {
		grid.start_remote_neighbor_copy_updates();
		dccrg::detail::check(dccrgx_gol_step(grid.native(), state, DCCRGX_REGION_INNER));
		grid.wait_remote_neighbor_copy_update_receives();
		dccrg::detail::check(dccrgx_gol_step(grid.native(), state, DCCRGX_REGION_OUTER));
		grid.wait_remote_neighbor_copy_update_sends();
		dccrg::detail::check(dccrgx_gol_commit(grid.native(), state));
	}
	dccrg::detail::check(dccrgx_synchronize(grid.native()));
	const double s = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();

	dccrg::detail::check(dccrgx_field_download(grid.native(), state, 0, alive.size(), alive.data()));
	uint64_t live = 0;
	for (auto a : alive) live += a;
	std::printf("cells %zu turns %d live %llu  %.3e cell-updates/s\n", cells.size(), turns,
	            (unsigned long long)live, double(cells.size()) * turns / s);
	return 0;
}
