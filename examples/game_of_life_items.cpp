// The reference's examples/game_of_life.cpp loop, unchanged in shape,
// against the facade's iteration items: per turn, update the remote copies,
// count live neighbors over cell.neighbors_of with neighbor.data, apply the
// rule (examples/game_of_life.cpp:54-79).  Cell_Data is the whole payload;
// the host loop reads the staging copy (download after the halo, upload
// after the rule).  Then the same game on the device sweep over a SoA
// field, and both must agree.
//
// usage: game_of_life_items [nx ny turns]; prints "live <n> idsum <s> agree <0|1>"
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dccrg.hpp"

struct game_of_life_cell {
	uint32_t is_alive = 0, live_neighbor_count = 0;
};

static bool alive0(uint64_t id) {  // SURVEY §8(d) seeded rule
	uint64_t z = (id ^ 0x5DEECE66Dull) + 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	z = z ^ (z >> 31);
	return z < uint64_t(0.2 * 18446744073709551616.0);
}

int main(int argc, char* argv[])
{
	const uint64_t nx = argc > 2 ? std::strtoull(argv[1], nullptr, 10) : 64;
	const uint64_t ny = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 64;
	const int turns = argc > 3 ? std::atoi(argv[3]) : 10;
	dccrg::Dccrg<game_of_life_cell> grid;
	grid.set_initial_length({{nx, ny, 1}}).set_neighborhood_length(1).set_maximum_refinement_level(0).initialize();

	grid.download();
	for (const auto& cell : grid.local_cells_items()) cell.data->is_alive = alive0(cell.id) ? 1 : 0;
	grid.upload();
	const int state = grid.add_field<uint32_t>("is_alive_soa", true);
	{
		const auto ids = grid.local_cells();
		std::vector<uint32_t> a(ids.size());
		for (size_t i = 0; i < ids.size(); i++) a[size_t(dccrgx_get_slot(grid.native(), ids[i]))] = alive0(ids[i]);
		dccrg::detail::check(dccrgx_field_upload(grid.native(), state, 0, a.size(), a.data()));
	}

	for (int turn = 0; turn < turns; turn++) {
		grid.update_copies_of_remote_neighbors();
		grid.download();
		const auto cells = grid.local_cells_items();
		for (const auto& cell : cells) {
			cell.data->live_neighbor_count = 0;
			for (const auto& neighbor : cell.neighbors_of)
				if (neighbor.data->is_alive > 0) cell.data->live_neighbor_count++;
		}
		for (const auto& cell : cells) {
			if (cell.data->live_neighbor_count == 3) cell.data->is_alive = 1;
			else if (cell.data->live_neighbor_count != 2) cell.data->is_alive = 0;
		}
		grid.upload();
		dccrg::detail::check(dccrgx_gol_step(grid.native(), state, DCCRGX_REGION_ALL));
		dccrg::detail::check(dccrgx_gol_commit(grid.native(), state));
	}
	grid.download();
	const auto ids = grid.local_cells();
	std::vector<uint32_t> dev(ids.size());
	dccrg::detail::check(dccrgx_field_download(grid.native(), state, 0, dev.size(), dev.data()));
	uint64_t live = 0, idsum = 0;
	bool agree = true;
	for (uint64_t id : ids) {
		const uint32_t h = grid[id]->is_alive;
		live += h;
		if (h) idsum += id;
		agree = agree && dev[size_t(dccrgx_get_slot(grid.native(), id))] == h;
	}
	std::printf("live %llu idsum %llu agree %d\n", (unsigned long long)live, (unsigned long long)idsum, agree ? 1 : 0);
	return agree ? 0 : 1;
}
