/*
 * dccrg_stretched_cartesian_geometry.hpp - the facade's
 * dccrg::Stretched_Cartesian_Geometry (reference
 * dccrg_stretched_cartesian_geometry.hpp:48-413): level-0 cell boundaries
 * given per dimension as a strictly increasing list of length + 1
 * coordinates; a refined cell divides its level-0 ancestor evenly.
 *
 * Host-side, like the facade's Cartesian_Geometry: a cell's refinement level
 * and indices come from the library's mapping (dccrgx_get_refinement_level /
 * dccrgx_get_indices), the arithmetic is the reference's, in its operand order
 * (get_length 298-337, get_center 346-403), so the doubles are the same.
 * Before the parameters are set (and after initialize without them) the
 * geometry is the reference's reset(): coordinates 0, 1, ..., length.
 * When every dimension's coordinates are evenly spaced (start + i * h, as
 * set(const Cartesian_Geometry&) makes them) the library's device geometry
 * gets that start and h too, so device-side consumers see the same cells;
 * uneven spacing stays host-side.
 * Grid files: save_grid_data writes this geometry's block (write 652-715,
 * file_block) in place of the Cartesian one and load_grid_data reads it back
 * (read 723-800, from_file_block), through dccrgx_set / get_geometry_block.
 */
#ifndef DCCRG_AMD_STRETCHED_CARTESIAN_GEOMETRY_HPP
#define DCCRG_AMD_STRETCHED_CARTESIAN_GEOMETRY_HPP

#include <cmath>
#include <cstring>
#include <vector>

#include "dccrg.hpp"

namespace dccrg {

class Stretched_Cartesian_Geometry_Parameters {  // 48-58
public:
	// per dimension: the start of the grid, then the end of each level-0 cell
	std::array<std::vector<double>, 3> coordinates;
};

class Stretched_Cartesian_Geometry : public No_Geometry {
public:
	static constexpr int geometry_id = 2;  // 78
	typedef Stretched_Cartesian_Geometry_Parameters Parameters;

	// 138-150: 0, 1, ..., length in each dimension
	void reset() {
		const auto L = grid_length();
		for (size_t d = 0; d < 3; d++) {
			p_.coordinates[d].resize(L[d] + 1);
			for (uint64_t i = 0; i <= L[d]; i++) p_.coordinates[d][i] = double(i);
		}
	}

	const Parameters& get() const {
		if (p_.coordinates[0].empty()) const_cast<Stretched_Cartesian_Geometry*>(this)->reset();
		return p_;
	}

	// 172-210: at least two strictly increasing values per dimension, length + 1
	// of them; returns false and changes nothing otherwise.  Empty parameters
	// (the facade's default before set_geometry) mean reset().
	bool set(const Parameters& given) {
		if (given.coordinates[0].empty() && given.coordinates[1].empty() && given.coordinates[2].empty()) {
			reset();
			push_device();
			return true;
		}
		const auto L = grid_length();
		for (size_t d = 0; d < 3; d++) {
			const auto& c = given.coordinates[d];
			if (c.size() < 2) {
				std::cerr << "At least two coordinates are required for grid cells in the " << d << " dimension"
				          << std::endl;
				return false;
			}
			if (c.size() != L[d] + 1) {
				std::cerr << "Number of values in dimension " << d << " must be length of the grid + 1 ("
				          << L[d] + 1 << ") but is " << c.size() << std::endl;
				return false;
			}
			for (size_t i = 0; i + 1 < c.size(); i++)
				if (c[i] >= c[i + 1]) {
					std::cerr << "Coordinates in the " << d << " dimension must be strictly increasing" << std::endl;
					return false;
				}
		}
		p_ = given;
		push_device();
		return true;
	}
	bool set(const Stretched_Cartesian_Geometry& other) { return set(other.get()); }  // 215

	std::array<double, 3> get_start() const {  // 261
		const auto& c = get().coordinates;
		return {{c[0][0], c[1][0], c[2][0]}};
	}
	std::array<double, 3> get_end() const {  // 279
		const auto& c = get().coordinates;
		return {{c[0].back(), c[1].back(), c[2].back()}};
	}

	// 298-337: the level-0 ancestor's extent divided by 2^level
	std::array<double, 3> get_length(const uint64_t cell) const {
		const int lvl = level(cell), R = max_level();
		if (cell == error_cell || lvl < 0 || lvl > R) return nan3();
		const auto s = get_level_0_cell_coord_start_index(cell);
		const auto& c = get().coordinates;
		const uint64_t len = uint64_t(1) << lvl;
		std::array<double, 3> r;
		for (size_t d = 0; d < 3; d++) r[d] = (c[d][s[d] + 1] - c[d][s[d]]) / len;
		return r;
	}

	// 346-403: start of the ancestor + index offset within it + half the cell
	std::array<double, 3> get_center(const uint64_t cell) const {
		const int lvl = level(cell), R = max_level();
		if (cell == error_cell || lvl < 0 || lvl > R) return nan3();
		const auto ind = indices(cell);
		const auto s = get_level_0_cell_coord_start_index(cell);
		const auto& c = get().coordinates;
		const uint64_t l0 = uint64_t(1) << R;
		const auto cl = get_length(cell);
		std::array<double, 3> r;
		for (size_t d = 0; d < 3; d++) {
			const double length_of_index = (c[d][s[d] + 1] - c[d][s[d]]) / l0;
			r[d] = c[d][s[d]] + length_of_index * (ind[d] - s[d] * l0) + cl[d] / 2;
		}
		return r;
	}
	std::array<double, 3> get_center(const Types<3>::indices_t ind, const int refinement_level) const {  // 464
		return get_center(g_ ? dccrgx_get_cell_from_indices(g_, ind.data(), refinement_level) : error_cell);
	}
	std::array<double, 3> get_min(const uint64_t cell) const {  // 417
		const auto c = get_center(cell), L = get_length(cell);
		return {{c[0] - L[0] / 2, c[1] - L[1] / 2, c[2] - L[2] / 2}};
	}
	std::array<double, 3> get_max(const uint64_t cell) const {  // 443
		const auto c = get_center(cell), L = get_length(cell);
		return {{c[0] + L[0] / 2, c[1] + L[1] / 2, c[2] + L[2] / 2}};
	}

	// 504-548: inside, or wrapped into the grid along periodic dimensions
	// (the grid's topology), else NaN
	std::array<double, 3> get_real_coordinate(const std::array<double, 3>& x) const {
		const auto start = get_start(), end = get_end();
		std::array<double, 3> r = nan3();
		for (size_t d = 0; d < 3; d++) {
			if (x[d] >= start[d] && x[d] <= end[d]) {
				r[d] = x[d];
			} else if (periodic(d)) {
				const double len = end[d] - start[d];
				r[d] = x[d] < start[d] ? x[d] + len * std::ceil((start[d] - x[d]) / len)
				                       : x[d] - len * std::ceil((x[d] - end[d]) / len);
			}
		}
		return r;
	}

	// 557-607: indices of a coordinate (error_index outside the grid)
	Types<3>::indices_t get_indices(const std::array<double, 3>& x) const {
		Types<3>::indices_t r{{error_index, error_index, error_index}};
		const auto start = get_start(), end = get_end();
		const uint64_t l0 = uint64_t(1) << max_level();
		const auto& c = get().coordinates;
		for (size_t d = 0; d < 3; d++) {
			if (!(x[d] >= start[d] && x[d] <= end[d])) continue;
			// the level-0 cell: the last boundary strictly below x (x at the
			// grid start belongs to the first cell)
			uint64_t i0 = uint64_t(std::lower_bound(c[d].begin(), c[d].end(), x[d]) - c[d].begin());
			i0 = i0 == 0 ? 0 : i0 - 1;
			const double li = (c[d][i0 + 1] - c[d][i0]) / double(l0);
			uint64_t k = 0;
			while (c[d][i0] + k * li < x[d]) k++;
			r[d] = i0 * l0 + (k == 0 ? 0 : k - 1);
		}
		return r;
	}
	// 478-490
	uint64_t get_cell(const int refinement_level, const std::array<double, 3>& x) const {
		if (refinement_level < 0 || refinement_level > max_level() || !g_) return error_cell;
		const auto ind = get_indices(x);
		return dccrgx_get_cell_from_indices(g_, ind.data(), refinement_level);
	}

	// 616-641: index of the level-0 ancestor's start in each coordinate list
	std::array<uint64_t, 3> get_level_0_cell_coord_start_index(const uint64_t cell) const {
		const int lvl = level(cell), R = max_level();
		if (cell == error_cell || lvl < 0 || lvl > R) return {{error_index, error_index, error_index}};
		const auto ind = indices(cell);
		return {{ind[0] / (uint64_t(1) << R), ind[1] / (uint64_t(1) << R), ind[2] / (uint64_t(1) << R)}};
	}

	// write 652-715: int id 2, 3 x uint64 coordinate counts, the coordinates
	std::vector<char> file_block() const {
		const auto& c = get().coordinates;
		std::vector<char> b(data_size());
		char* q = b.data();
		const int id = geometry_id;
		std::memcpy(q, &id, sizeof(int));
		q += sizeof(int);
		for (size_t d = 0; d < 3; d++) {
			const uint64_t n = c[d].size();
			std::memcpy(q, &n, sizeof(uint64_t));
			q += sizeof(uint64_t);
		}
		for (size_t d = 0; d < 3; d++) {
			std::memcpy(q, c[d].data(), c[d].size() * sizeof(double));
			q += c[d].size() * sizeof(double);
		}
		return b;
	}
	// read 723-800: the id must be this geometry's, then set() the coordinates
	bool from_file_block(const std::vector<char>& b) {
		int id = Cartesian_Geometry::geometry_id;
		if (b.size() >= sizeof(int)) std::memcpy(&id, b.data(), sizeof(int));
		if (b.empty() || id != geometry_id) {
			std::cerr << __FILE__ << ":" << __LINE__ << " Wrong geometry: " << id << ", should be " << geometry_id
			          << std::endl;
			return false;
		}
		uint64_t n[3] = {0, 0, 0};
		if (b.size() < sizeof(int) + sizeof(n)) return false;
		std::memcpy(n, b.data() + sizeof(int), sizeof(n));
		Parameters p;
		size_t at = sizeof(int) + sizeof(n);
		for (size_t d = 0; d < 3; d++) {
			if (at + n[d] * sizeof(double) > b.size()) return false;
			p.coordinates[d].resize(n[d]);
			std::memcpy(p.coordinates[d].data(), b.data() + at, n[d] * sizeof(double));
			at += n[d] * sizeof(double);
		}
		return set(p);
	}

	// 808-817: bytes of the geometry block the reference writes to a file
	size_t data_size() const {
		size_t r = sizeof(int) + 3 * sizeof(uint64_t);
		for (const auto& c : get().coordinates) r += c.size() * sizeof(double);
		return r;
	}

private:
	static std::array<double, 3> nan3() {
		const double n = std::numeric_limits<double>::quiet_NaN();
		return {{n, n, n}};
	}
	std::array<uint64_t, 3> grid_length() const { return length_ ? length_->get() : std::array<uint64_t, 3>{{1, 1, 1}}; }
	int level(uint64_t cell) const { return g_ ? dccrgx_get_refinement_level(g_, cell) : -1; }
	int max_level() const {
		int l = 0;
		if (g_) dccrgx_get_maximum_refinement_level(g_, &l);
		return l;
	}
	std::array<uint64_t, 3> indices(uint64_t cell) const {
		std::array<uint64_t, 3> r{{error_index, error_index, error_index}};
		if (g_) dccrgx_get_indices(g_, cell, r.data());
		return r;
	}
	bool periodic(size_t d) const { return topology_ && topology_->is_periodic(d); }
	// evenly spaced coordinates: the library's device geometry takes them too
	void push_device() const {
		if (!g_) return;
		double start[3], h[3];
		for (size_t d = 0; d < 3; d++) {
			const auto& c = p_.coordinates[d];
			if (c.size() < 2) return;
			start[d] = c[0];
			h[d] = c[1] - c[0];
			for (size_t i = 0; i < c.size(); i++)
				if (c[i] != c[0] + double(i) * h[d]) return;
		}
		dccrgx_set_geometry(g_, start, h);
	}

	Parameters p_;
};

}  // namespace dccrg

#endif
