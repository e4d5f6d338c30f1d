/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Probe over the reference's own headers, compiled unmodified from where they
 * lie (/root/reference/dccrg_mapping.hpp, dccrg_topology.hpp,
 * dccrg_cartesian_geometry.hpp; their only external dependency is the MPI
 * header, which this image ships under /opt/conda/include).  Built by
 * oracle/Makefile into oracle/_ref/ref_probe and used only by
 * tests/golden/make_golden.py to generate the mapping/geometry golden vectors
 * that pin oracle/dccrg_oracle.cpp.  dccrg.hpp itself needs zoltan.h and Boost
 * (absent here) and is therefore NOT built.
 *
 * Protocol (stdin, whitespace separated):
 *   lx ly lz R  sx sy sz  l0x l0y l0z
 *   n  id_1 .. id_n
 *   m  (ix iy iz lvl) x m
 * Output (stdout): one line per id:
 *   id lvl ix iy iz clen parent child l0parent s0..s7 cx cy cz Lx Ly Lz
 * then one line per index query: cell
 * then: last_cell max_possible_level
 */
#include <cstdio>
#include <iostream>
#include <limits>  // dccrg_mpi_support.hpp uses std::numeric_limits without including it

#include "dccrg_mapping.hpp"
#include "dccrg_topology.hpp"
#include "dccrg_cartesian_geometry.hpp"

int main()
{
	unsigned long long lx, ly, lz;
	int R;
	double sx, sy, sz, l0x, l0y, l0z;
	if (!(std::cin >> lx >> ly >> lz >> R >> sx >> sy >> sz >> l0x >> l0y >> l0z)) return 2;

	dccrg::Mapping mapping;
	if (!mapping.set_length({{lx, ly, lz}})) return 3;
	if (!mapping.set_maximum_refinement_level(R)) return 4;
	dccrg::Grid_Topology topology;
	dccrg::Cartesian_Geometry geometry(mapping.length, mapping, topology);
	dccrg::Cartesian_Geometry::Parameters params;
	params.start = {{sx, sy, sz}};
	params.level_0_cell_length = {{l0x, l0y, l0z}};
	if (!geometry.set(params)) return 5;

	size_t n;
	std::cin >> n;
	std::cout.precision(17);
	for (size_t i = 0; i < n; i++) {
		uint64_t id;
		std::cin >> id;
		const auto ind = mapping.get_indices(id);
		const auto sib = mapping.get_siblings(id);
		std::cout << id << ' ' << mapping.get_refinement_level(id) << ' '
			<< ind[0] << ' ' << ind[1] << ' ' << ind[2] << ' '
			<< mapping.get_cell_length_in_indices(id) << ' '
			<< mapping.get_parent(id) << ' ' << mapping.get_child(id) << ' '
			<< mapping.get_level_0_parent(id);
		for (const auto s: sib) std::cout << ' ' << s;
		const int lvl = mapping.get_refinement_level(id);
		if (lvl >= 0) {
			const auto c = geometry.get_center(id);
			const auto l = geometry.get_length(id);
			std::cout << ' ' << c[0] << ' ' << c[1] << ' ' << c[2]
				<< ' ' << l[0] << ' ' << l[1] << ' ' << l[2];
		} else {
			std::cout << " nan nan nan nan nan nan";
		}
		std::cout << '\n';
	}
	size_t m;
	std::cin >> m;
	for (size_t i = 0; i < m; i++) {
		uint64_t ix, iy, iz;
		int lvl;
		std::cin >> ix >> iy >> iz >> lvl;
		std::cout << mapping.get_cell_from_indices({{ix, iy, iz}}, lvl) << '\n';
	}
	std::cout << mapping.get_last_cell() << ' ' << mapping.get_maximum_possible_refinement_level() << '\n';
	return 0;
}
