// A grid with a Stretched_Cartesian_Geometry saved and loaded through the
// facade (include/dccrg.hpp, include/dccrg_stretched_cartesian_geometry.hpp):
// the file carries the stretched geometry's block (the reference's
// Stretched_Cartesian_Geometry::write / read,
// dccrg_stretched_cartesian_geometry.hpp:652-800) and the loaded grid has the
// same coordinates, cells, payloads and cell centers / lengths.  Unevenly
// spaced coordinates, some cells refined.
//
//   stretched_restart FILE     save, then load into a second grid, compare
//
// Every process prints "PASS <rank> <cells>" or exits non-zero.
#include <array>
#include <cstdio>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"
#include "dccrg_stretched_cartesian_geometry.hpp"

struct Cell {
	double v = 0;
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() const {
		return std::make_tuple((void*)&v, 1, MPI_DOUBLE);
	}
};

using Grid = dccrg::Dccrg<Cell, dccrg::Stretched_Cartesian_Geometry>;

int main(int argc, char* argv[]) {
	MPI_Init(&argc, &argv);
	MPI_Comm comm = MPI_COMM_WORLD;
	int rank = 0;
	MPI_Comm_rank(comm, &rank);
	if (argc != 2) {
		if (rank == 0) std::fprintf(stderr, "usage: %s FILE\n", argv[0]);
		MPI_Finalize();
		return 2;
	}
	const std::string path = argv[1];
	std::tuple<void*, int, MPI_Datatype> header{nullptr, 0, MPI_INT};
	dccrg::Stretched_Cartesian_Geometry::Parameters geom;
	geom.coordinates[0] = {0.0, 0.5, 1.5, 3.0, 5.0, 5.25};
	geom.coordinates[1] = {-2.0, -1.0, 0.25, 4.0, 4.5};
	geom.coordinates[2] = {10.0, 10.5, 12.0, 12.125};
	std::map<uint64_t, std::array<double, 7>> saved;  // own cells: value, center, length
	size_t cells = 0;
	{
		Grid grid;
		grid.set_initial_length({{5, 4, 3}}).set_neighborhood_length(1).set_maximum_refinement_level(1);
		grid.set_geometry(geom);
		grid.initialize(comm);
		for (const uint64_t c : {uint64_t(1), uint64_t(8), uint64_t(27), uint64_t(40)})
			if (grid.is_local(c)) grid.refine_completely(c);
		grid.stop_refining();
		for (const auto& cell : grid.local_cells()) {
			cell.data->v = 0.5 * double(cell.id);
			const auto c = grid.geometry.get_center(cell.id), L = grid.geometry.get_length(cell.id);
			saved[cell.id] = {{cell.data->v, c[0], c[1], c[2], L[0], L[1], L[2]}};
		}
		if (!grid.save_grid_data(path, 0, header)) {
			std::fprintf(stderr, "rank %d: save_grid_data failed\n", rank);
			return 1;
		}
	}
	MPI_Barrier(comm);
	{
		Grid grid;
		if (!grid.load_grid_data(path, 0, header, comm)) {
			std::fprintf(stderr, "rank %d: load_grid_data failed\n", rank);
			return 1;
		}
		const auto& got = grid.geometry.get().coordinates;
		for (size_t d = 0; d < 3; d++)
			if (got[d] != geom.coordinates[d]) {
				std::fprintf(stderr, "rank %d: coordinates of dimension %zu differ after loading\n", rank, d);
				return 1;
			}
		// every process checks the cells it owns now against the saved values
		// it can see: all of them on one process (the load balances anew)
		int size = 1;
		MPI_Comm_size(comm, &size);
		for (const auto& cell : grid.local_cells()) {
			cells++;
			const auto c = grid.geometry.get_center(cell.id), L = grid.geometry.get_length(cell.id);
			if (cell.data->v != 0.5 * double(cell.id)) {
				std::fprintf(stderr, "rank %d: cell %llu holds %g\n", rank, (unsigned long long)cell.id, cell.data->v);
				return 1;
			}
			const auto it = saved.find(cell.id);
			if (size == 1 && it == saved.end()) {
				std::fprintf(stderr, "rank %d: cell %llu was not saved\n", rank, (unsigned long long)cell.id);
				return 1;
			}
			if (it != saved.end())
				for (int k = 0; k < 3; k++)
					if (c[k] != it->second[1 + k] || L[k] != it->second[4 + k]) {
						std::fprintf(stderr, "rank %d: cell %llu geometry differs after loading\n", rank,
						             (unsigned long long)cell.id);
						return 1;
					}
		}
	}
	std::printf("PASS %d %zu\n", rank, cells);
	MPI_Finalize();
	return 0;
}
