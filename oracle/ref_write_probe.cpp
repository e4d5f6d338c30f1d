/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Writes the "internal grid data" block of a dccrg grid file the way the
 * reference's save_grid_data lays it out (dccrg.hpp:1104-1120, 1196-1258):
 * Mapping::write (dccrg_mapping.hpp:576), the neighborhood length as one
 * MPI_UNSIGNED, Grid_Topology::write (dccrg_topology.hpp:144) and
 * Cartesian_Geometry::write (dccrg_cartesian_geometry.hpp:618) — the three
 * writers are the reference's own headers compiled unmodified, driven
 * through MPI-IO (MPICH from /opt/conda).  Built by oracle/Makefile into
 * oracle/_ref/ref_write_probe; used only by tests/golden/make_golden.py.
 *
 * stdin: lx ly lz R hood px py pz sx sy sz l0x l0y l0z path
 * stdout: mapping_size topology_size geometry_size total_bytes
 */
#include <mpi.h>
#include <cstdio>
#include <iostream>
#include <limits>
#include <string>

#include "dccrg_mapping.hpp"
#include "dccrg_topology.hpp"
#include "dccrg_cartesian_geometry.hpp"

int main(int argc, char** argv)
{
	MPI_Init(&argc, &argv);
	unsigned long long lx, ly, lz;
	int R, px, py, pz;
	unsigned hood;
	double sx, sy, sz, l0x, l0y, l0z;
	std::string path;
	if (!(std::cin >> lx >> ly >> lz >> R >> hood >> px >> py >> pz >> sx >> sy >> sz >> l0x >> l0y >> l0z >> path))
		return 2;
	dccrg::Mapping mapping;
	if (!mapping.set_length({{lx, ly, lz}})) return 3;
	if (!mapping.set_maximum_refinement_level(R)) return 4;
	dccrg::Grid_Topology topology;
	topology.set_periodicity(0, px != 0);
	topology.set_periodicity(1, py != 0);
	topology.set_periodicity(2, pz != 0);
	dccrg::Cartesian_Geometry geometry(mapping.length, mapping, topology);
	dccrg::Cartesian_Geometry::Parameters params;
	params.start = {{sx, sy, sz}};
	params.level_0_cell_length = {{l0x, l0y, l0z}};
	if (!geometry.set(params)) return 5;

	MPI_File f;
	if (MPI_File_open(MPI_COMM_SELF, const_cast<char*>(path.c_str()), MPI_MODE_CREATE | MPI_MODE_WRONLY,
	                  MPI_INFO_NULL, &f) != MPI_SUCCESS)
		return 6;
	MPI_Offset off = 0;
	if (!mapping.write(f, off)) return 7;
	off += mapping.data_size();
	MPI_File_write_at(f, off, (void*)&hood, 1, MPI_UNSIGNED, MPI_STATUS_IGNORE);
	off += sizeof(unsigned);
	if (!topology.write(f, off)) return 8;
	off += topology.data_size();
	if (geometry.write(f, off) == 0) return 9;
	off += geometry.data_size();
	MPI_File_close(&f);
	std::cout << mapping.data_size() << ' ' << topology.data_size() << ' ' << geometry.data_size() << ' ' << off
	          << std::endl;
	MPI_Finalize();
	return 0;
}
