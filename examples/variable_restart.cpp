// Restart with a different amount of data per cell, the scenario of the
// reference's tests/restart/variable_cell_data.cpp written against the
// facade (include/dccrg.hpp): a 20 x 1 x 1 grid whose cells hold `id` ints
// (none when id % 4 == 0) behind a uint64 count.
//
//   variable_restart save FILE   the cells of every third process move to the
//                                next one, then save_grid_data
//   variable_restart load FILE   start_loading_grid_data, the counts
//                                (continue_loading_grid_data), the ints sized
//                                from them (continue again), finish; then a
//                                balance_load that moves the loaded payloads
//
// The file may be loaded by another number of processes than saved it.  Every
// process prints "PASS <rank> <cells>" or exits non-zero.
#include <array>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <tuple>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"

struct Cell {
	uint64_t data_size = 0;
	std::vector<int> data;

	// what get_mpi_datatype describes: everything (count + ints), the ints
	// only, or the count only
	enum Part { all, ints, count };
	static Part part;

	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() const {
		if (part == count) return std::make_tuple((void*)&data_size, 1, MPI_UINT64_T);
		if (part == ints) return std::make_tuple((void*)data.data(), int(data.size()), MPI_INT);
		int counts[2] = {1, int(data.size())};
		MPI_Aint disp[2] = {0, data.empty() ? 0 : MPI_Aint((const char*)data.data() - (const char*)&data_size)};
		MPI_Datatype types[2] = {MPI_UINT64_T, MPI_INT};
		MPI_Datatype t;
		MPI_Type_create_struct(2, counts, disp, types, &t);
		return std::make_tuple((void*)&data_size, 1, t);
	}
};
Cell::Part Cell::part = Cell::all;

using Grid = dccrg::Dccrg<Cell, dccrg::Cartesian_Geometry>;

static uint64_t expected_count(uint64_t id) { return id % 4 ? id : 0; }

static bool holds_its_data(Grid& grid, const char* when, int rank) {
	for (const auto& cell : grid.local_cells()) {
		const uint64_t n = expected_count(cell.id);
		bool ok = cell.data->data_size == n && cell.data->data.size() == n;
		for (uint64_t i = 0; ok && i < n; i++) ok = cell.data->data[i] == int(i);
		if (!ok) {
			std::fprintf(stderr, "rank %d %s: cell %llu holds %llu / %zu values, expected %llu\n", rank, when,
			             (unsigned long long)cell.id, (unsigned long long)cell.data->data_size, cell.data->data.size(),
			             (unsigned long long)n);
			return false;
		}
	}
	return true;
}

int main(int argc, char* argv[]) {
	MPI_Init(&argc, &argv);
	MPI_Comm comm = MPI_COMM_WORLD;
	int rank = 0, size = 1;
	MPI_Comm_rank(comm, &rank);
	MPI_Comm_size(comm, &size);
	if (argc != 3 || (std::string(argv[1]) != "save" && std::string(argv[1]) != "load")) {
		if (rank == 0) std::fprintf(stderr, "usage: %s save|load FILE\n", argv[0]);
		MPI_Finalize();
		return 2;
	}
	const std::string path = argv[2];
	std::tuple<void*, int, MPI_Datatype> header{nullptr, 0, MPI_INT};
	size_t cells = 0;
	{
		Grid grid;
		if (std::string(argv[1]) == "save") {
			dccrg::Cartesian_Geometry::Parameters geom;
			geom.start = {{0, 0, 0}};
			geom.level_0_cell_length = {{1, 1, 1}};
			grid.set_initial_length({{20, 1, 1}})
			    .set_neighborhood_length(1)
			    .set_maximum_refinement_level(-1)
			    .set_load_balancing_method("RANDOM")
			    .initialize(comm)
			    .set_geometry(geom);
			if (rank % 3 == 0 && rank + 1 < size)
				for (const auto& cell : grid.local_cells()) grid.pin(cell.id, rank + 1);
			grid.balance_load();
			grid.unpin_local_cells();
			for (const auto& cell : grid.local_cells()) {
				const uint64_t n = expected_count(cell.id);
				cell.data->data.resize(n);
				for (uint64_t i = 0; i < n; i++) cell.data->data[i] = int(i);
				cell.data->data_size = n;
			}
			if (!grid.save_grid_data(path, 0, header)) {
				std::fprintf(stderr, "rank %d: save_grid_data failed\n", rank);
				return 1;
			}
		} else {
			if (!grid.start_loading_grid_data(path, 0, header, comm, "RANDOM")) {
				std::fprintf(stderr, "rank %d: start_loading_grid_data failed\n", rank);
				return 1;
			}
			Cell::part = Cell::count;
			if (!grid.continue_loading_grid_data()) return 1;
			for (const auto& cell : grid.local_cells()) {
				if (cell.data->data_size != expected_count(cell.id) || !cell.data->data.empty()) {
					std::fprintf(stderr, "rank %d: cell %llu count %llu\n", rank, (unsigned long long)cell.id,
					             (unsigned long long)cell.data->data_size);
					return 1;
				}
				cell.data->data.resize(cell.data->data_size);
			}
			Cell::part = Cell::ints;
			if (!grid.continue_loading_grid_data()) return 1;
			if (!grid.finish_loading_grid_data()) return 1;
			if (!holds_its_data(grid, "loaded", rank)) return 1;
			// the loaded objects are the device payloads now: a balance moves
			// them (arrivals sized first, as variable_data_size.cpp:83-95)
			Cell::part = Cell::all;
			if (rank % 3 == 0 && rank + 1 < size)
				for (const auto& cell : grid.local_cells()) grid.pin(cell.id, rank + 1);
			grid.initialize_balance_load(true);
			for (const auto& sender : grid.get_cells_to_receive())
				for (const auto& item : sender.second) grid[item.first]->data.resize(expected_count(item.first));
			grid.continue_balance_load();
			grid.finish_balance_load();
			if (!holds_its_data(grid, "balanced", rank)) return 1;
		}
		for (const auto& cell : grid.local_cells()) {
			(void)cell;
			cells++;
		}
	}
	std::printf("PASS %d %zu\n", rank, cells);
	MPI_Finalize();
	return 0;
}
