/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's (lkotipal/dccrg @ 2024-10-24) hot-path
 * algorithms, used exclusively as the parity checker by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg.  Nothing in the
 * product (dccrg_amd/, include/) links, loads or calls this file.
 *
 * Every function restates the reference logic it cites (file:line into
 * /root/reference).  The data layout deliberately mirrors the reference:
 * hashed cell maps, a std::map-like face-neighbor cache and per-cell
 * neighbor vectors, walked one cell at a time.
 *
 * Parity pinning:
 *   - Mapping / Cartesian geometry: pinned against the reference headers
 *     compiled as-is (oracle/ref_probe.cpp -> oracle/_ref/ref_probe).
 *   - face cache / neighbor lists / GoL: pinned against the reference's own
 *     known-answer tests (tests/get_neighbors_/test1.cpp,
 *     tests/game_of_life/game_of_life_test.cpp, examples/simple_game_of_life.cpp,
 *     tests/user_neighborhood/neighbor_list_length.cpp) transcribed as
 *     fixtures in tests/golden/.
 *   - advection: the reference holds no known answer -> the
 *     advection restatement is "parity unpinned" against reference outputs.
 */
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace oracle {

static const uint64_t error_cell = 0;
static const uint64_t error_index = 0xFFFFFFFFFFFFFFFFull;

typedef std::array<uint64_t, 3> idx3;
typedef std::array<int, 3> off3;
typedef std::vector<std::pair<uint64_t, off3>> nlist;

/* ---------------------------------------------------------------------------
 * Mapping — dccrg_mapping.hpp:54-651
 * ------------------------------------------------------------------------- */
struct Mapping {
	uint64_t len[3] = {1, 1, 1};
	int R = 0;
	uint64_t last = 1;

	// dccrg_mapping.hpp:640-648
	void update_last() {
		const uint64_t g = len[0] * len[1] * len[2];
		last = 0;
		for (int i = 0; i <= R; i++) last += g * (uint64_t(1) << (i * 3));
	}

	// dccrg_mapping.hpp:316-329 (double-precision loop kept as-is)
	int max_possible_level() const {
		const uint64_t g = len[0] * len[1] * len[2];
		int lvl = 0;
		double cur = 0;
		while (cur <= double(~uint64_t(0))) {
			cur += double(g) * std::pow(8.0, double(lvl));
			lvl++;
		}
		return lvl - 2;
	}

	// dccrg_mapping.hpp:153-208
	uint64_t from_indices(const idx3& ind, int lvl) const {
		for (int d = 0; d < 3; d++)
			if (ind[d] >= len[d] * (uint64_t(1) << R)) return error_cell;
		if (lvl < 0 || lvl > R) return error_cell;
		uint64_t cell = 1;
		for (int i = 0; i < lvl; i++) cell += len[0] * len[1] * len[2] * (uint64_t(1) << (i * 3));
		const uint64_t sh = uint64_t(1) << (R - lvl);
		const uint64_t lx = len[0] * (uint64_t(1) << lvl), ly = len[1] * (uint64_t(1) << lvl);
		cell += ind[0] / sh + (ind[1] / sh) * lx + (ind[2] / sh) * lx * ly;
		return cell;
	}

	// dccrg_mapping.hpp:261-289
	int level(uint64_t cell) const {
		if (cell == error_cell || cell > last) return -1;
		int lvl = 0;
		uint64_t cur = 0;
		while (lvl <= R) {
			cur += len[0] * len[1] * len[2] * (uint64_t(1) << 3 * lvl);
			if (cell <= cur) break;
			lvl++;
		}
		if (lvl > R) return -1;
		return lvl;
	}

	// dccrg_mapping.hpp:217-253
	idx3 indices(uint64_t cell) const {
		if (cell == error_cell || cell > last) return {error_index, error_index, error_index};
		const int lvl = level(cell);
		for (int i = 0; i < lvl; i++) cell -= len[0] * len[1] * len[2] * (uint64_t(1) << (i * 3));
		cell -= 1;
		const uint64_t sh = uint64_t(1) << (R - lvl);
		const uint64_t lx = len[0] * (uint64_t(1) << lvl), ly = len[1] * (uint64_t(1) << lvl);
		return {(cell % lx) * sh, ((cell / lx) % ly) * sh,
		        (cell / (len[0] * len[1] * (uint64_t(1) << (2 * lvl)))) * sh};
	}

	// dccrg_mapping.hpp:297-310
	uint64_t cell_len(uint64_t cell) const {
		if (cell == error_cell) return error_index;
		const int lvl = level(cell);
		if (lvl < 0) return error_index;
		return uint64_t(1) << (R - lvl);
	}

	// dccrg_mapping.hpp:338-356
	uint64_t child(uint64_t cell) const {
		if (cell == error_cell || cell > last) return error_cell;
		const int lvl = level(cell);
		if (lvl >= R) return cell;
		return from_indices(indices(cell), lvl + 1);
	}

	// dccrg_mapping.hpp:367-383
	uint64_t parent(uint64_t cell) const {
		const int lvl = level(cell);
		if (lvl < 0 || lvl > R) return error_cell;
		if (lvl == 0) return cell;
		return from_indices(indices(cell), lvl - 1);
	}

	// dccrg_mapping.hpp:391-441 (z outer, y, x inner)
	std::array<uint64_t, 8> all_children(uint64_t cell) const {
		std::array<uint64_t, 8> ch;
		ch.fill(error_cell);
		if (cell == error_cell) return ch;
		int lvl = level(cell);
		if (lvl >= R) return ch;
		const idx3 ind = indices(cell);
		lvl++;
		const uint64_t o = uint64_t(1) << (R - lvl);
		size_t i = 0;
		for (uint64_t z = 0; z < 2 * o; z += o)
			for (uint64_t y = 0; y < 2 * o; y += o)
				for (uint64_t x = 0; x < 2 * o; x += o)
					ch[i++] = from_indices({ind[0] + x, ind[1] + y, ind[2] + z}, lvl);
		return ch;
	}

	// dccrg_mapping.hpp:449-470
	std::array<uint64_t, 8> siblings(uint64_t cell) const {
		std::array<uint64_t, 8> s;
		s.fill(error_cell);
		const int lvl = level(cell);
		if (lvl < 0 || lvl > R) return s;
		if (lvl == 0) {
			s[0] = cell;
			return s;
		}
		return all_children(parent(cell));
	}

	// dccrg_mapping.hpp:479-493
	uint64_t level0_parent(uint64_t cell) const {
		const int lvl = level(cell);
		if (lvl < 0 || lvl > R) return error_cell;
		if (lvl == 0) return cell;
		return from_indices(indices(cell), 0);
	}
};

/* ---------------------------------------------------------------------------
 * Grid — the single-address-space view of dccrg's global structures
 * (cell_process dccrg.hpp:7197, neighbors_ 7098-7109, neighbors_of/_to).
 * Every rank in the reference holds these for ALL cells (8243, 8898), so one
 * object here reproduces every rank's view.
 * ------------------------------------------------------------------------- */
struct Grid {
	Mapping m;
	bool periodic[3] = {false, false, false};
	unsigned hood_len = 1;
	int nprocs = 1;
	std::vector<off3> hood_of, hood_to;
	std::unordered_map<uint64_t, int> cell_process;
	std::unordered_map<uint64_t, std::array<uint64_t, 6>> neighbors_;
	std::unordered_map<uint64_t, nlist> nof, nto;
	// iterator lists are cached like the reference's update_cell_pointers
	// (11314-11628) caches them; cleared on every rebuild
	mutable std::unordered_map<uint64_t, nlist> it_cache;
	std::unordered_set<uint64_t> to_refine, to_unrefine, not_to_unrefine, not_to_refine;
	std::unordered_map<uint64_t, int> removed_to;  // cells removed by the last unrefine -> parent's process
	std::unordered_map<uint64_t, int> pins;
	// Cartesian geometry (dccrg_cartesian_geometry.hpp)
	double start[3] = {0, 0, 0}, l0[3] = {1, 1, 1};

	// dccrg.hpp:7895-7954
	void init_hoods() {
		hood_of.clear();
		hood_to.clear();
		if (hood_len == 0) {
			hood_of = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
		} else {
			const int L = int(hood_len);
			for (int z = -L; z <= L; z++)
				for (int y = -L; y <= L; y++)
					for (int x = -L; x <= L; x++) {
						if (x == 0 && y == 0 && z == 0) continue;
						hood_of.push_back({x, y, z});
					}
		}
		for (const auto& o : hood_of) hood_to.push_back({-o[0], -o[1], -o[2]});
	}

	// dccrg.hpp:7967-8013 (block partition, no SFC)
	void create_level_0_cells() {
		const uint64_t total = m.len[0] * m.len[1] * m.len[2];
		const uint64_t P = uint64_t(nprocs);
		uint64_t cpp;
		if (total < P) cpp = 1;
		else if (total % P > 0) cpp = total / P + 1;
		else cpp = total / P;
		const uint64_t fewer = cpp * P - total;
		uint64_t c = 1;
		for (uint64_t p = 0; p < P; p++) {
			const uint64_t n = (p < fewer) ? cpp - 1 : cpp;
			for (uint64_t i = 0; i < n; i++) cell_process[c++] = int(p);
		}
	}

	bool exists(uint64_t c) const { return cell_process.count(c) > 0; }

	// existence-aware get_child, dccrg.hpp:9555-9581
	uint64_t get_child_e(uint64_t cell) const {
		const int lvl = m.level(cell);
		if (lvl == m.R) return exists(cell) ? cell : error_cell;
		const uint64_t ch = m.from_indices(m.indices(cell), lvl + 1);
		if (exists(ch)) return ch;
		if (exists(cell)) return cell;
		return error_cell;
	}

	// existence-aware get_parent, dccrg.hpp:4157-4190
	uint64_t get_parent_e(uint64_t cell) const {
		if (m.level(cell) == 0) return exists(cell) ? cell : error_cell;
		const uint64_t par = m.from_indices(m.indices(cell), m.level(cell) - 1);
		if (exists(par)) return par;
		if (exists(cell)) return cell;
		return error_cell;
	}

	// dccrg.hpp:11275-11308
	uint64_t get_existing_cell(const idx3& ind, int minl, int maxl) const {
		for (int d = 0; d < 3; d++)
			if (ind[d] >= m.len[d] * (uint64_t(1) << m.R)) return error_cell;
		if (minl > maxl) return error_cell;
		for (int l = maxl; l >= minl; l--) {
			const uint64_t c = m.from_indices(ind, l);
			if (exists(c)) return c;
		}
		return error_cell;
	}

	// dccrg.hpp:9324-9458 (face-neighbor cache entry of one cell)
	void update_neighbors_(uint64_t cell) {
		if (cell == error_cell || !exists(cell) || cell != get_child_e(cell)) return;
		const idx3 ind = m.indices(cell);
		const uint64_t clen = m.cell_len(cell);
		std::array<idx3, 6> s{ind, ind, ind, ind, ind, ind};
		for (int dir : {0, 2, 4}) {
			const int d = dir / 2;
			if (s[dir][d] == 0) {
				s[dir][d] = periodic[d] ? m.len[d] * (uint64_t(1) << m.R) - 1 : error_index;
			} else {
				s[dir][d]--;
			}
		}
		for (int dir : {1, 3, 5}) {
			const int d = dir / 2;
			const uint64_t maxi = m.len[d] * (uint64_t(1) << m.R) - 1;
			if (maxi < clen || s[dir][d] > maxi - clen) {
				s[dir][d] = periodic[d] ? 0 : error_index;
			} else {
				s[dir][d] += clen;
			}
		}
		const int lvl = m.level(cell);
		const int lo = (lvl == 0) ? 0 : lvl - 1;
		const int hi = (lvl == m.R) ? m.R : lvl + 1;
		std::array<uint64_t, 6> nn;
		for (int i = 0; i < 6; i++) nn[i] = get_existing_cell(s[i], lo, hi);
		neighbors_[cell] = nn;
	}

	int len_int(uint64_t c) const { return int(m.cell_len(c)); }

	// offset from cell_ to its parent, dccrg.hpp:4384-4403
	off3 parent_offset(uint64_t c) const {
		off3 r{0, 0, 0};
		const uint64_t p = m.parent(c);
		if (p == error_cell || p == c) return r;
		const idx3 ci = m.indices(c), pi = m.indices(p);
		for (int d = 0; d < 3; d++) {
			if (pi[d] >= ci[d]) r[d] += int(pi[d] - ci[d]);
			else r[d] -= int(ci[d] - pi[d]);
		}
		return r;
	}

	// adjust_offset lambda, dccrg.hpp:4405-4527
	off3 adjust_offset(off3 o, uint64_t from, uint64_t to, int direction) const {
		const int fl = len_int(from), tl = len_int(to);
		const int d = std::abs(direction) - 1;
		const int sgn = direction > 0 ? 1 : -1;
		if (fl == tl) {
			o[d] += sgn * fl;
			return o;
		}
		if (fl < tl) {
			const off3 po = parent_offset(from);
			for (int k = 0; k < 3; k++) o[k] += po[k];
			o[d] += sgn * tl;  // -x: += par - to_len ; +x: += par + to_len
		} else {
			const off3 po = parent_offset(to);
			for (int k = 0; k < 3; k++) o[k] -= po[k];
			o[d] += sgn * fl;  // -x: -= par + from_len ; +x: -= par - from_len
		}
		return o;
	}

	// dccrg.hpp:4339-4680 — walk the face-neighbor graph to each stencil box
	nlist find_neighbors_of(uint64_t cell, const std::vector<off3>& hood) const {
		if (cell == error_cell || !exists(cell)) throw std::runtime_error("invalid cell");
		const int clen = len_int(cell);
		if (!neighbors_.count(cell)) throw std::runtime_error("no neighbors_");
		nlist ret;
		for (const auto& h : hood) {
			const off3 s{h[0] * clen, h[1] * clen, h[2] * clen};
			const off3 e{(h[0] + 1) * clen - 1, (h[1] + 1) * clen - 1, (h[2] + 1) * clen - 1};
			off3 o{0, 0, 0};
			uint64_t cur = cell;
			int cl = len_int(cur);
			while (o[0] + cl - 1 < s[0] || o[0] > e[0] || o[1] + cl - 1 < s[1] || o[1] > e[1] ||
			       o[2] + cl - 1 < s[2] || o[2] > e[2]) {
				const auto& nn = neighbors_.at(cur);
				int k = -1, dir = 0;
				if (o[0] > e[0]) { k = 0; dir = -1; }
				else if (o[0] + cl - 1 < s[0]) { k = 1; dir = +1; }
				else if (o[1] > e[1]) { k = 2; dir = -2; }
				else if (o[1] + cl - 1 < s[1]) { k = 3; dir = +2; }
				else if (o[2] > e[2]) { k = 4; dir = -3; }
				else if (o[2] + cl - 1 < s[2]) { k = 5; dir = +3; }
				else throw std::runtime_error("internal error");
				if (nn[k] != error_cell) o = adjust_offset(o, cur, nn[k], dir);
				cur = nn[k];
				if (cur == error_cell) break;
				cl = len_int(cur);
			}
			if (cur == error_cell) continue;  // 4634-4636
			cl = len_int(cur);
			if (cl >= clen) {
				ret.emplace_back(cur, o);
				continue;
			}
			// sibling expansion, 4644-4676
			const auto sib = m.siblings(cur);
			size_t ci = 0;
			for (; ci < sib.size(); ci++)
				if (cur == sib[ci]) break;
			if (ci == sib.size()) throw std::runtime_error("internal error (siblings)");
			if (ci % 2 > 0) o[0] -= cl;
			if (ci % 4 > 1) o[1] -= cl;
			if (ci > 3) o[2] -= cl;
			size_t i = 0;
			for (int oz : {0, cl})
				for (int oy : {0, cl})
					for (int ox : {0, cl}) ret.push_back({sib[i++], {o[0] + ox, o[1] + oy, o[2] + oz}});
		}
		return ret;
	}

	// dccrg.hpp:4200-4316
	std::vector<idx3> indices_from_neighborhood(const idx3& ind, uint64_t L, const std::vector<off3>& hood) const {
		std::vector<idx3> out;
		out.reserve(hood.size());
		const uint64_t gl[3] = {m.len[0] * (uint64_t(1) << m.R), m.len[1] * (uint64_t(1) << m.R),
		                        m.len[2] * (uint64_t(1) << m.R)};
		for (const auto& o : hood) {
			idx3 t = ind;
			for (int d = 0; d < 3; d++) {
				if (o[d] < 0) {
					if (periodic[d]) {
						for (int i = 0; i > o[d]; i--) {
							if (t[d] >= L) t[d] -= L;
							else t[d] = gl[d] - L;
						}
					} else {
						if (ind[d] < uint64_t(std::abs(o[d])) * L) {
							t = {error_index, error_index, error_index};
							break;
						}
						t[d] += int64_t(o[d]) * int64_t(L);
					}
				} else {
					if (periodic[d]) {
						for (int i = 0; i < o[d]; i++) {
							if (t[d] < gl[d] - L) t[d] += L;
							else t[d] = 0;
						}
					} else {
						if (ind[d] + uint64_t(o[d]) * L >= gl[d]) {
							t = {error_index, error_index, error_index};
							break;
						}
						t[d] += uint64_t(o[d]) * L;
					}
				}
			}
			out.push_back(t);
		}
		return out;
	}

	// dccrg.hpp:4708-4861 (returned unordered in the reference; sorted by id here)
	nlist find_neighbors_to(uint64_t cell, const std::vector<off3>& hood) const {
		if (cell == error_cell || cell > m.last || cell != get_child_e(cell))
			throw std::invalid_argument("find_neighbors_to: invalid cell");
		const int lvl = m.level(cell);
		std::set<uint64_t> uniq;
		if (lvl > 0) {
			const uint64_t par = m.parent(cell);
			for (const auto& si : indices_from_neighborhood(m.indices(par), m.cell_len(par), hood)) {
				if (si[0] == error_index) continue;
				const uint64_t f = m.from_indices(si, lvl - 1);
				if (f == get_child_e(f)) uniq.insert(f);
			}
		}
		if (lvl < m.R) {
			const auto ch = m.all_children(cell);
			const uint64_t L = m.cell_len(ch[0]);
			for (const auto c : ch) {
				for (const auto& si : indices_from_neighborhood(m.indices(c), L, hood)) {
					if (si[0] == error_index) continue;
					const uint64_t f = m.from_indices(si, lvl + 1);
					if (f == get_child_e(f)) uniq.insert(f);
				}
			}
		}
		for (const auto& si : indices_from_neighborhood(m.indices(cell), m.cell_len(cell), hood)) {
			if (si[0] == error_index) continue;
			const uint64_t f = m.from_indices(si, lvl);
			if (f == get_child_e(f)) uniq.insert(f);
		}
		nlist r;
		for (auto f : uniq) r.push_back({f, {0, 0, 0}});
		return r;
	}

	// dccrg.hpp:2806-2933
	std::vector<std::pair<uint64_t, int>> face_neighbors_of(uint64_t cell) const {
		std::vector<std::pair<uint64_t, int>> ret;
		const auto& nn = neighbors_.at(cell);
		const int lvl = m.level(cell);
		const int dirs[6] = {-1, +1, -2, +2, -3, +3};
		for (int i = 0; i < 6; i++) {
			const uint64_t n = nn[i];
			if (n == error_cell) continue;
			ret.emplace_back(n, dirs[i]);
			if (lvl >= m.level(n)) continue;
			const auto& n2 = neighbors_.at(n);
			int a, b;  // first/second in-face direction slots
			if (i < 2) { a = 3; b = 5; }
			else if (i < 4) { a = 1; b = 5; }
			else { a = 1; b = 3; }
			if (n2[a] != error_cell) ret.emplace_back(n2[a], dirs[i]);
			if (n2[b] != error_cell) {
				ret.emplace_back(n2[b], dirs[i]);
				const uint64_t x = neighbors_.at(n2[b])[a];
				if (x != error_cell) ret.emplace_back(x, dirs[i]);
			}
		}
		return ret;
	}

	// dccrg.hpp:9313-9319 then 8240-8289 / 8894-8963
	void rebuild() {
		it_cache.clear();
		neighbors_.clear();
		for (const auto& cp : cell_process) update_neighbors_(cp.first);
		nof.clear();
		nto.clear();
		for (const auto& cp : cell_process) {
			const uint64_t c = cp.first;
			if (c != get_child_e(c) || c != get_parent_e(c)) continue;
			nof[c] = find_neighbors_of(c, hood_of);
			nto[c] = find_neighbors_to(c, hood_to);
		}
	}

	// dccrg.hpp:2434-2520: at the maximum level dont_unrefine (2472-2475);
	// refused for a cell in cells_not_to_refine or with a coarser neighbor
	// there (2477-2491; the set persists between stop_refining calls)
	bool refine_completely(uint64_t c) {
		if (c == error_cell || !exists(c)) return false;
		if (m.level(c) == m.R) {
			dont_unrefine(c);
			return true;
		}
		if (not_to_refine.count(c)) return false;
		if (nof.count(c))
			for (const auto& n : nof.at(c))
				if (m.level(n.first) < m.level(c) && not_to_refine.count(n.first)) return false;
		to_refine.insert(c);
		return true;
	}

	// dccrg.hpp:9464-9544 and overlapping_indices 11225-11263
	bool is_neighbor(uint64_t c1, uint64_t c2) const {
		const idx3 i1 = m.indices(c1), i2 = m.indices(c2);
		const uint64_t l1 = m.cell_len(c1), l2 = m.cell_len(c2);
		uint64_t maxd = 0;
		int overlap = 0;
		for (int d = 0; d < 3; d++) {
			const uint64_t gl = m.len[d] * (uint64_t(1) << m.R);
			uint64_t dist;
			if (i1[d] <= i2[d]) {
				dist = (i2[d] <= i1[d] + l1) ? 0 : i2[d] - (i1[d] + l1);
				if (periodic[d]) dist = std::min(dist, i1[d] + (gl - (i2[d] + l2)));
			} else {
				dist = (i1[d] <= i2[d] + l2) ? 0 : i1[d] - (i2[d] + l2);
				if (periodic[d]) dist = std::min(dist, i2[d] + (gl - (i1[d] + l1)));
			}
			maxd = std::max(maxd, dist);
			if (i1[d] + l1 > i2[d] && i1[d] < i2[d] + l2) overlap++;
		}
		if (hood_len == 0) return maxd < l1 && overlap >= 2;
		return maxd < uint64_t(hood_len) * l1;
	}

	// dccrg.hpp:2560-2660; the neighbor test runs on get_parent(cell), which
	// is the cell itself because its parent does not exist (4157-4190)
	bool unrefine_completely(uint64_t cell) {
		if (cell == error_cell || !exists(cell)) return false;
		if (cell != get_child_e(cell)) return false;
		if (m.level(cell) == 0) return true;
		const auto sib = m.siblings(cell);
		for (const uint64_t s : sib) {
			if (s != get_child_e(s)) return false;
			if (to_refine.count(s) || not_to_unrefine.count(s)) return true;
		}
		const uint64_t parent = get_parent_e(cell);
		const int rl = m.level(parent);
		for (const auto& n : find_neighbors_of(parent, hood_of)) {
			const int nl = m.level(n.first);
			if (nl > rl + 1) return true;
			if (nl == rl + 1 && to_refine.count(n.first)) return true;
		}
		for (const uint64_t s : sib)
			if (to_unrefine.count(s)) return true;
		to_unrefine.insert(cell);
		return true;
	}

	// dccrg.hpp:2679-2733
	bool dont_unrefine(uint64_t cell) {
		if (cell == error_cell || !exists(cell)) return false;
		if (m.level(cell) == 0) return true;
		const auto sib = m.siblings(cell);
		for (const uint64_t s : sib)
			if (not_to_unrefine.count(s)) return true;
		for (const uint64_t s : sib) to_unrefine.erase(s);
		not_to_unrefine.insert(cell);
		return true;
	}

	// dccrg.hpp:2744-2784
	bool dont_refine(uint64_t cell) {
		if (cell == error_cell || !exists(cell)) return false;
		if (m.level(cell) == m.R) return true;
		to_refine.erase(cell);
		not_to_refine.insert(cell);
		return true;
	}

	// override_refines dccrg.hpp:9991-10038
	void override_refines() {
		std::unordered_set<uint64_t> new_donts, donts, old_donts;
		do {
			donts = new_donts;
			new_donts.clear();
			donts.insert(not_to_refine.begin(), not_to_refine.end());
			not_to_refine.clear();
			for (const uint64_t cell : donts) {
				std::set<uint64_t> all;
				if (nof.count(cell))
					for (const auto& n : nof.at(cell)) all.insert(n.first);
				if (nto.count(cell))
					for (const auto& n : nto.at(cell)) all.insert(n.first);
				const int rl = m.level(cell);
				for (const uint64_t n : all) {
					if (old_donts.count(n) || donts.count(n)) continue;
					if (m.level(n) > rl) new_donts.insert(n);
				}
			}
			old_donts.insert(donts.begin(), donts.end());
			donts.clear();
		} while (!new_donts.empty());
		not_to_refine = old_donts;  // 10039: kept for the next stop_refining
		for (const uint64_t c : old_donts) to_refine.erase(c);
	}

	// override_unrefines dccrg.hpp:9796-9898
	void override_unrefines() {
		std::unordered_set<uint64_t> final_unrefines;
		for (const uint64_t unrefined : to_unrefine) {
			bool can = true;
			const uint64_t parent = m.parent(unrefined);
			for (const uint64_t s : m.all_children(parent)) {
				if (s == error_cell) continue;
				if (to_refine.count(s) || not_to_unrefine.count(s)) {
					can = false;
					break;
				}
			}
			if (!can) continue;
			const int ul = m.level(unrefined);
			std::set<uint64_t> processed, process;
			for (const uint64_t n : neighbors_.at(unrefined)) process.insert(n);
			process.erase(error_cell);
			while (!process.empty()) {
				const uint64_t next = *process.begin();
				processed.insert(next);
				process.erase(next);
				for (const uint64_t n : neighbors_.at(next)) {
					if (n == error_cell || processed.count(n)) continue;
					if (is_neighbor(parent, n)) process.insert(n);
					else processed.insert(n);
				}
				const int rl = m.level(next);
				if (rl < ul) continue;
				if (rl == ul) {
					if (to_refine.count(next)) {
						can = false;
						break;
					}
					continue;
				}
				can = false;
				break;
			}
			if (can) final_unrefines.insert(unrefined);
		}
		to_unrefine = final_unrefines;
		not_to_unrefine.clear();
	}

	// override_refines, induce_refines dccrg.hpp:9591-9720 (single address
	// space: all processes' lists are the same global lists),
	// override_unrefines, then execute_refines 10104-10554
	std::vector<uint64_t> stop_refining() {
		override_refines();
		std::vector<uint64_t> fresh(to_refine.begin(), to_refine.end());
		while (!fresh.empty()) {
			std::unordered_set<uint64_t> induced;
			for (const uint64_t r : fresh) {
				const int rl = m.level(r);
				for (const auto* lst : {&nof.at(r), &nto.at(r)})
					for (const auto& n : *lst) {
						if (n.first == error_cell) continue;
						if (m.level(n.first) < rl && !to_refine.count(n.first)) induced.insert(n.first);
					}
			}
			fresh.assign(induced.begin(), induced.end());
			to_refine.insert(induced.begin(), induced.end());
		}
		override_unrefines();
		// unrefines 10282-10410: the parent is owned by the first child's owner
		removed_to.clear();
		for (const uint64_t u : to_unrefine) {
			const uint64_t parent = m.parent(u);
			const auto sib = m.all_children(parent);
			const int owner = cell_process.at(sib[0]);
			for (const uint64_t s : sib) {
				removed_to[s] = owner;
				cell_process.erase(s);
			}
			cell_process[parent] = owner;
		}
		to_unrefine.clear();
		std::vector<uint64_t> created;
		for (const uint64_t r : to_refine) {
			const int owner = cell_process.at(r);
			for (const auto ch : m.all_children(r)) {
				cell_process[ch] = owner;  // children inherit the parent's rank, 10228-10237
				created.push_back(ch);
			}
		}
		for (const uint64_t r : to_refine) cell_process.erase(r);  // 10498
		to_refine.clear();
		rebuild();
		std::sort(created.begin(), created.end());
		return created;
	}

	// Cartesian geometry, dccrg_cartesian_geometry.hpp:282-362
	std::array<double, 3> get_length(uint64_t c) const {
		const int lvl = m.level(c);
		const double s = 1.0 / double(uint64_t(1) << lvl);
		return {l0[0] * s, l0[1] * s, l0[2] * s};
	}
	std::array<double, 3> get_center(uint64_t c) const {
		const idx3 ind = m.indices(c);
		const auto cl = get_length(c);
		std::array<double, 3> r;
		for (int d = 0; d < 3; d++)
			r[d] = start[d] + double(ind[d]) * l0[d] / double(uint64_t(1) << m.R) + cl[d] / 2;
		return r;
	}

	/* -------------------- per-rank views -------------------- */
	struct RankView {
		std::vector<uint64_t> local, inner, outer;  // sorted ids
		std::set<uint64_t> local_bdy, remote_bdy;
		std::map<int, std::vector<uint64_t>> send, recv;  // sorted ascending
	};

	// update_remote_neighbor_info 8992-9095 + recalculate_..._lists 8590-8752
	RankView rank_view(int rank) const {
		RankView v;
		for (const auto& cp : cell_process)
			if (cp.second == rank) v.local.push_back(cp.first);
		std::sort(v.local.begin(), v.local.end());
		for (const uint64_t c : v.local) {
			for (const auto& n : nof.at(c)) {
				if (n.first == error_cell) continue;
				if (cell_process.at(n.first) != rank) {
					v.local_bdy.insert(c);
					v.remote_bdy.insert(n.first);
				}
			}
			for (const auto& n : nto.at(c)) {
				if (cell_process.at(n.first) != rank) {
					v.local_bdy.insert(c);
					v.remote_bdy.insert(n.first);
				}
			}
		}
		std::map<int, std::set<uint64_t>> us, ur;
		for (const uint64_t c : v.local_bdy) {
			for (const auto& n : nof.at(c)) {
				if (n.first == error_cell) continue;
				const int p = cell_process.at(n.first);
				if (p != rank) ur[p].insert(n.first);
			}
			for (const auto& n : nto.at(c)) {
				const int p = cell_process.at(n.first);
				if (p != rank) us[p].insert(c);
			}
		}
		for (auto& kv : us) v.send[kv.first].assign(kv.second.begin(), kv.second.end());
		for (auto& kv : ur) v.recv[kv.first].assign(kv.second.begin(), kv.second.end());
		for (const uint64_t c : v.local) (v.local_bdy.count(c) ? v.outer : v.inner).push_back(c);
		return v;
	}

	// iterator neighbor ranges, update_cell_pointers 11451-11500:
	// neighbors_of range = only_of (sorted set) followed by both (sorted set)
	const nlist& iter_of(uint64_t c) const {
		auto it = it_cache.find(c);
		if (it != it_cache.end()) return it->second;
		return it_cache.emplace(c, iterator_neighbors_of(c)).first->second;
	}

	nlist iterator_neighbors_of(uint64_t c) const {
		std::set<std::pair<uint64_t, off3>> ids_of, ids_to, only_of, both;
		for (const auto& n : nof.at(c))
			if (n.first != error_cell) ids_of.insert(n);
		for (const auto& n : nto.at(c))
			if (n.first != error_cell) ids_to.insert(n);
		for (const auto& n : ids_of) {
			auto t = n;
			t.second = {0, 0, 0};
			if (ids_to.count(t)) both.insert(n);
			else only_of.insert(n);
		}
		nlist r(only_of.begin(), only_of.end());
		r.insert(r.end(), both.begin(), both.end());
		return r;
	}
};

/* ---------------------------------------------------------------------------
 * Game of life — examples/game_of_life.cpp:54-79,
 * tests/game_of_life/scalability3d.cpp:130-165: count over the iterator's
 * cell.neighbors_of, then the rule.
 * ------------------------------------------------------------------------- */
static void gol_step(const Grid& g, std::unordered_map<uint64_t, uint32_t>& alive) {
	std::unordered_map<uint64_t, uint32_t> count;
	for (const auto& cp : g.cell_process) {
		uint32_t k = 0;
		for (const auto& n : g.iter_of(cp.first))
			if (alive.at(n.first) > 0) k++;
		count[cp.first] = k;
	}
	for (auto& a : alive) {
		const uint32_t k = count.at(a.first);
		if (k == 3) a.second = 1;
		else if (k != 2) a.second = 0;
	}
}

/* ---------------------------------------------------------------------------
 * Game of life on a refined grid emulating the unrefined game —
 * tests/game_of_life/solve.hpp:37-170 (get_live_neighbors), literally: the
 * collect loop (46-110), the halo (111; one process here), the in-place
 * spread among same-parent neighbors (113-150), the rule (152-167).  data[0]
 * is the state, data[1..8] the list of live level-0 neighbor parents.  The
 * reference loops in get_cells() (hash) order; ascending order here.
 * Aborts become exceptions with the reference's messages.
 * ------------------------------------------------------------------------- */
using GolAmrData = std::array<uint64_t, 9>;

static uint64_t level0_parent(const Mapping& m, uint64_t cell) {  // dccrg_mapping.hpp:479-493
	const int lvl = m.level(cell);
	if (lvl < 0 || lvl > m.R) return error_cell;
	if (lvl == 0) return cell;
	return m.from_indices(m.indices(cell), 0);
}

// the collect loop of get_live_neighbors (solve.hpp:45-109)
static void gol_amr_collect(const Grid& g, std::unordered_map<uint64_t, GolAmrData>& data,
                            const std::vector<uint64_t>& cells) {
	for (const uint64_t cell : cells) {
		GolAmrData& cd = data.at(cell);
		for (size_t i = 1; i < cd.size(); i++) cd[i] = 0;
		const uint64_t cp = level0_parent(g.m, cell);
		for (const auto& ni : g.nof.at(cell)) {
			const uint64_t nb = ni.first;
			if (nb == error_cell) continue;
			const uint64_t np = level0_parent(g.m, nb);
			if (np == cp) continue;
			const GolAmrData& nd = data.at(nb);
			if (nd[0] == 0) {
				for (size_t i = 1; i < cd.size(); i++)
					if (cd[i] == np) throw std::runtime_error("Neighbor should not be alive.");
			} else {
				for (size_t i = 1; i < cd.size(); i++) {
					if (cd[i] == np) break;
					else if (cd[i] == error_cell) {
						cd[i] = np;
						break;
					} else if (i == cd.size() - 1)
						throw std::runtime_error("No more room in live neighbor list.");
				}
			}
		}
	}
}

static void gol_amr_step(const Grid& g, std::unordered_map<uint64_t, GolAmrData>& data) {
	std::vector<uint64_t> cells;
	for (const auto& cp : g.cell_process) cells.push_back(cp.first);
	std::sort(cells.begin(), cells.end());
	gol_amr_collect(g, data, cells);
	for (const uint64_t cell : cells) {
		const uint64_t cp = level0_parent(g.m, cell);
		GolAmrData& cd = data.at(cell);
		for (const auto& ni : g.nof.at(cell)) {
			const uint64_t nb = ni.first;
			if (nb == error_cell) continue;
			if (cp != level0_parent(g.m, nb)) continue;
			const GolAmrData& nd = data.at(nb);
			for (size_t i = 1; i < nd.size(); i++) {
				if (nd[i] == error_cell) break;
				for (size_t j = 1; j < cd.size(); j++) {
					if (cd[j] == error_cell) {
						cd[j] = nd[i];
						break;
					} else if (cd[j] == nd[i]) break;
					else if (j == cd.size() - 1)
						throw std::runtime_error("No room in live neighbor list of cell");
				}
			}
		}
	}
	for (const uint64_t cell : cells) {
		GolAmrData& cd = data.at(cell);
		size_t live = 0;
		for (size_t i = 1; i < cd.size(); i++) {
			if (cd[i] != error_cell) live++;
			cd[i] = error_cell;
		}
		if (live == 3) cd[0] = 1;
		else if (live != 2) cd[0] = 0;
	}
}

/* ---------------------------------------------------------------------------
 * Advection — tests/advection/{initialize.hpp:36-82, solve.hpp:44-346}
 * ------------------------------------------------------------------------- */
struct AdvCell {
	double d[9];  // density, vx, vy, vz, flux, max_diff, lx, ly, lz (cell.hpp:38-49)
};

static double get_vx(double y) { return -y + 0.5; }  // solve.hpp:336-338
static double get_vy(double x) { return +x - 0.5; }  // solve.hpp:340-342

// initialize.hpp:36-82
static void adv_initialize(const Grid& g, std::unordered_map<uint64_t, AdvCell>& cells) {
	for (const auto& cp : g.cell_process) {
		AdvCell& c = cells[cp.first];
		for (int i = 0; i < 9; i++) c.d[i] = 0;
		const auto ctr = g.get_center(cp.first);
		const double radius = 0.15;
		c.d[1] = get_vx(ctr[1]);
		c.d[2] = get_vy(ctr[0]);
		c.d[3] = 0;
		const double hx = 0.25, hy = 0.5;
		const double hr = std::min(std::sqrt(std::pow(ctr[0] - hx, 2.0) + std::pow(ctr[1] - hy, 2.0)), radius) / radius;
		c.d[0] = 0.25 * (1 + std::cos(M_PI * hr));
		const auto L = g.get_length(cp.first);
		c.d[6] = L[0];
		c.d[7] = L[1];
		c.d[8] = L[2];
	}
}

// solve.hpp:44-266 for one cell: the flux scatter exactly as the reference
// does it; `is_local(n)` decides whether a local pair is solved from this side.
template <class IsLocal>
static void adv_cell_fluxes(const Grid& g, uint64_t cid, double dt, std::unordered_map<uint64_t, AdvCell>& cells,
                            const IsLocal& is_local) {
	AdvCell& cell = cells.at(cid);
	const double cd = cell.d[0];
	const double cv = cell.d[6] * cell.d[7] * cell.d[8];
	const int clen = int(g.m.cell_len(cid));
	for (const auto& nb : g.iter_of(cid)) {
		const int nlen = int(g.m.cell_len(nb.first));
		int overlaps = 0, direction = 0;
		const int x = nb.second[0], y = nb.second[1], z = nb.second[2];
		if (x < clen && x > -nlen) overlaps++;
		else if (x == clen) direction = 1;
		else if (x == -nlen) direction = -1;
		if (y < clen && y > -nlen) overlaps++;
		else if (y == clen) direction = 2;
		else if (y == -nlen) direction = -2;
		if (z < clen && z > -nlen) overlaps++;
		else if (z == clen) direction = 3;
		else if (z == -nlen) direction = -3;
		if (overlaps < 2) continue;
		if (overlaps > 2) throw std::runtime_error("advection: overlapping neighbor");
		if (direction == 0) continue;
		if (is_local(nb.first) && direction < 0) continue;
		AdvCell& nbc = cells.at(nb.first);
		const double nd = nbc.d[0];
		const double nv = nbc.d[6] * nbc.d[7] * nbc.d[8];
		double min_area = -1;
		switch (direction) {
		case -1: case +1: min_area = std::min(cell.d[7] * cell.d[8], nbc.d[7] * nbc.d[8]); break;
		case -2: case +2: min_area = std::min(cell.d[6] * cell.d[8], nbc.d[6] * nbc.d[8]); break;
		case -3: case +3: min_area = std::min(cell.d[6] * cell.d[7], nbc.d[6] * nbc.d[7]); break;
		}
		double flux = 0;
		const double vx = (cell.d[6] * nbc.d[1] + nbc.d[6] * cell.d[1]) / (cell.d[6] + nbc.d[6]);
		const double vy = (cell.d[7] * nbc.d[2] + nbc.d[7] * cell.d[2]) / (cell.d[7] + nbc.d[7]);
		const double vz = (cell.d[8] * nbc.d[3] + nbc.d[8] * cell.d[3]) / (cell.d[8] + nbc.d[8]);
		switch (direction) {
		case +1: flux = (vx >= 0 ? cd : nd) * dt * vx * min_area; break;
		case +2: flux = (vy >= 0 ? cd : nd) * dt * vy * min_area; break;
		case +3: flux = (vz >= 0 ? cd : nd) * dt * vz * min_area; break;
		case -1: flux = (vx >= 0 ? nd : cd) * dt * vx * min_area; break;
		case -2: flux = (vy >= 0 ? nd : cd) * dt * vy * min_area; break;
		case -3: flux = (vz >= 0 ? nd : cd) * dt * vz * min_area; break;
		}
		// the scatter into a remote neighbor lands in this rank's remote copy,
		// whose flux the reference never uses (solve.hpp:38): drop it here
		const bool nloc = is_local(nb.first);
		if (direction > 0) {
			cell.d[4] -= flux / cv;
			if (nloc) nbc.d[4] += flux / nv;
		} else {
			cell.d[4] += flux / cv;
			if (nloc) nbc.d[4] -= flux / nv;
		}
	}
}

// solve.hpp:289-333
static double adv_max_time_step(const std::unordered_map<uint64_t, AdvCell>& cells) {
	double mn = std::numeric_limits<double>::max();
	for (const auto& kv : cells) {
		const double* d = kv.second.d;
		const double s[3] = {d[6] / std::fabs(d[1]), d[7] / std::fabs(d[2]), d[8] / std::fabs(d[3])};
		for (int k = 0; k < 3; k++)
			if (std::isnormal(s[k])) mn = std::min(s[k], mn);
	}
	return mn;
}

// adapter.hpp:47-178, refine decisions only (unrefines are out of scope)
static std::vector<uint64_t> adv_refine_candidates(const Grid& g, std::unordered_map<uint64_t, AdvCell>& cells,
                                                    double diff_increase, double diff_threshold) {
	std::vector<uint64_t> ids;
	for (const auto& cp : g.cell_process) ids.push_back(cp.first);
	std::sort(ids.begin(), ids.end());
	for (auto id : ids) cells.at(id).d[5] = 0;
	for (auto id : ids) {
		AdvCell& c = cells.at(id);
		const int clen = int(g.m.cell_len(id));
		for (const auto& nb : g.iterator_neighbors_of(id)) {
			const int nlen = int(g.m.cell_len(nb.first));
			const int x = nb.second[0], y = nb.second[1], z = nb.second[2];
			bool face = false;
			if ((x == clen || x == -nlen) && y == 0 && z == 0) face = true;
			if ((y == clen || y == -nlen) && x == 0 && z == 0) face = true;
			if ((z == clen || z == -nlen) && x == 0 && y == 0) face = true;
			if (!face) continue;
			AdvCell& n = cells.at(nb.first);
			const double diff = std::fabs(c.d[0] - n.d[0]) / (std::min(c.d[0], n.d[0]) + diff_threshold);
			c.d[5] = std::max(diff, c.d[5]);
			n.d[5] = std::max(diff, n.d[5]);  // single address space: every neighbor is local
		}
	}
	std::vector<uint64_t> out;
	for (auto id : ids) {
		const int lvl = g.m.level(id);
		if (cells.at(id).d[5] > (lvl + 1) * diff_increase) out.push_back(id);
	}
	return out;
}

/* ---------------------------------------------------------------------------
 * Poisson BiCG — tests/poisson/poisson_solve.hpp:47-1054 (Poisson_Cell
 * 47-141, solve 251-522, solve_failsafe 531-634, get_residual 677-687,
 * set_scaling_factor 696-819, cache_system_info 827-971, initialize_solver
 * 979-1054).  Single address space: remote copies are the owners' objects,
 * which is what the reference's halo updates deliver before every use
 * (SOLVING before A.p0, GEOMETRY once after caching, INIT before the
 * initial residual).  Cells are visited in ascending id order; global sums
 * are taken in that order (the reference's order is hash order + the
 * MPI_Allreduce tree, so sums agree to rounding only).
 * ------------------------------------------------------------------------- */
enum { PO_SOLVE = 0, PO_BOUNDARY = 1, PO_SKIP = 2 };  // poisson_solve.hpp:146-150

struct PoissonCell {  // poisson_solve.hpp:51-86
	double rhs = 0, solution = 0, best_solution = 0, p0 = 0, p1 = 0, r0 = 0, r1 = 0, A_dot_p0 = 0, scaling_factor = 0;
	double f[6] = {0, 0, 0, 0, 0, 0};  // f_x_neg, f_x_pos, f_y_neg, f_y_pos, f_z_neg, f_z_pos
	int type = PO_BOUNDARY;
};

struct PoissonNb {
	uint64_t id;
	int direction;  // +-1..+-3
	int rel;        // relative refinement level (+1 finer, -1 coarser)
};

// direction (+-1..+-3) -> index into PoissonCell::f (-x,+x,-y,+y,-z,+z)
static inline int po_fi(int direction) { return 2 * (std::abs(direction) - 1) + (direction > 0 ? 1 : 0); }

struct PoissonSolver {
	unsigned max_iterations = 1000, min_iterations = 0;
	double stop_residual = 1e-15, p_of_norm = 2, stop_after_residual_increase = 10;
	std::vector<std::pair<uint64_t, std::vector<PoissonNb>>> cell_info;  // 647, 666
	std::unordered_map<uint64_t, PoissonCell> cells;
	unsigned iterations = 0;
	double residual_min = 0;
	bool reverse = false;

	PoissonCell& at(uint64_t c) { return cells.at(c); }

	// set_scaling_factor 696-819
	void set_scaling_factor(const Grid& g, uint64_t cell, const std::vector<std::pair<uint64_t, int>>& nbs) {
		PoissonCell& cd = at(cell);
		const auto cl = g.get_length(cell);
		const double chx = cl[0] / 2.0, chy = cl[1] / 2.0, chz = cl[2] / 2.0;
		double px = +2 * chx, nx = -2 * chx, py = +2 * chy, ny = -2 * chy, pz = +2 * chz, nz = -2 * chz;
		for (const auto& nb : nbs) {
			const auto nl = g.get_length(nb.first);
			const double hx = nl[0] / 2.0, hy = nl[1] / 2.0, hz = nl[2] / 2.0;
			switch (nb.second) {
			case +1: px = chx + hx; break;
			case -1: nx = -1.0 * (chx + hx); break;
			case +2: py = chy + hy; break;
			case -2: ny = -1.0 * (chy + hy); break;
			case +3: pz = chz + hz; break;
			case -3: nz = -1.0 * (chz + hz); break;
			default: throw std::runtime_error("poisson: invalid direction");
			}
		}
		const double tx = px - nx, ty = py - ny, tz = pz - nz;
		for (int k = 0; k < 6; k++) cd.f[k] = 0;
		for (const auto& nb : nbs) {
			switch (nb.second) {
			case +1: cd.f[1] = +2.0 / (px * tx); break;
			case -1: cd.f[0] = -2.0 / (nx * tx); break;
			case +2: cd.f[3] = +2.0 / (py * ty); break;
			case -2: cd.f[2] = -2.0 / (ny * ty); break;
			case +3: cd.f[5] = +2.0 / (pz * tz); break;
			case -3: cd.f[4] = -2.0 / (nz * tz); break;
			}
		}
		cd.scaling_factor = -cd.f[1] - cd.f[0] - cd.f[3] - cd.f[2] - cd.f[5] - cd.f[4];
	}

	// cache_system_info 827-971; types: per local cell (every leaf here)
	void cache_system_info(const Grid& g) {
		std::vector<uint64_t> all;
		for (const auto& cp : g.cell_process) all.push_back(cp.first);
		std::sort(all.begin(), all.end());
		// the reference walks get_cells() in hash order: any order is a faithful
		// restatement; `reverse` gives a second one to measure the order noise
		if (reverse) std::reverse(all.begin(), all.end());
		cell_info.clear();
		std::vector<uint64_t> newly_skipped;
		for (const uint64_t cell : all) {
			PoissonCell& cd = at(cell);
			if (cd.type == PO_SKIP) continue;
			const int clvl = g.m.level(cell);
			std::vector<std::pair<uint64_t, int>> face;
			std::vector<PoissonNb> info;
			for (const auto& fn : g.face_neighbors_of(cell)) {
				const PoissonCell& nd = at(fn.first);
				if (nd.type == PO_SKIP) continue;
				if (cd.type == PO_BOUNDARY && nd.type == PO_BOUNDARY) continue;
				face.push_back(fn);
				const int nlvl = g.m.level(fn.first);
				info.push_back({fn.first, fn.second, nlvl > clvl ? 1 : (nlvl < clvl ? -1 : 0)});
			}
			if (face.empty()) {
				// 953-957; applied after the loop, so every cell filters against
				// the classification it was given (the reference's outcome for a
				// neighbor converted here depends on its hash order)
				newly_skipped.push_back(cell);
				continue;
			}
			set_scaling_factor(g, cell, face);
			cell_info.push_back({cell, info});
		}
		for (const uint64_t c : newly_skipped) at(c).type = PO_SKIP;
	}

	// get_residual 677-687
	double get_residual() {
		double local = 0;
		for (const auto& ci : cell_info) local += std::pow(std::fabs(at(ci.first).r0), p_of_norm);
		return std::pow(local, 1.0 / p_of_norm);
	}

	// initialize_solver 979-1054
	double initialize_solver() {
		for (const auto& ci : cell_info) {
			PoissonCell& d = at(ci.first);
			if (d.type != PO_SOLVE) continue;
			d.r0 = d.rhs - d.scaling_factor * d.solution;
			for (const auto& nb : ci.second) {
				double mul = d.f[po_fi(nb.direction)];
				if (nb.rel > 0) mul /= 4.0;
				d.r0 -= mul * at(nb.id).solution;
			}
			d.p0 = d.p1 = d.r1 = d.r0;
		}
		double dot = 0;
		for (const auto& ci : cell_info) {
			const PoissonCell& d = at(ci.first);
			if (d.type == PO_SOLVE) dot += d.r0 * d.r1;
		}
		return dot;
	}

	// solve 251-522 (after cache_system_info)
	void solve() {
		double residual_min_ = std::numeric_limits<double>::max();
		double dot_r_g = initialize_solver();
		unsigned iteration = 0;
		do {
			iteration++;
			for (const auto& ci : cell_info) {  // A . p0 (290-339)
				PoissonCell& d = at(ci.first);
				if (d.type != PO_SOLVE) continue;
				d.A_dot_p0 = d.scaling_factor * d.p0;
				for (const auto& nb : ci.second) {
					double mul = d.f[po_fi(nb.direction)];
					if (nb.rel > 0) mul /= 4.0;
					d.A_dot_p0 += mul * at(nb.id).p0;
				}
			}
			double dot_p_g = 0;  // 341-349
			for (const auto& ci : cell_info) {
				const PoissonCell& d = at(ci.first);
				if (d.type == PO_SOLVE) dot_p_g += d.p1 * d.A_dot_p0;
			}
			if (dot_p_g == 0) break;
			const double alpha = dot_r_g / dot_p_g;
			for (const auto& ci : cell_info) {  // 364-370
				PoissonCell& d = at(ci.first);
				if (d.type == PO_SOLVE) d.solution += alpha * d.p0;
			}
			const double residual = get_residual();
			if (residual_min_ > residual) {  // 379-390
				residual_min_ = residual;
				for (const auto& ci : cell_info) {
					PoissonCell& d = at(ci.first);
					if (d.type == PO_SOLVE) d.best_solution = d.solution;
				}
			}
			if (residual <= stop_residual && iteration >= min_iterations) break;
			if (residual >= stop_after_residual_increase * residual_min_ && iteration >= min_iterations) break;
			for (const auto& ci : cell_info) {  // 405-411
				PoissonCell& d = at(ci.first);
				if (d.type == PO_SOLVE) d.r0 -= alpha * d.A_dot_p0;
			}
			for (const auto& ci : cell_info) {  // 413-470, transpose(A) . p1
				PoissonCell& d = at(ci.first);
				if (d.type != PO_SOLVE) continue;
				double A_dot_p1 = d.scaling_factor * d.p1;
				for (const auto& nb : ci.second) {
					const PoissonCell& n = at(nb.id);
					double mul = n.f[po_fi(-nb.direction)];
					if (nb.rel > 0) mul /= 4.0;
					A_dot_p1 += mul * n.p1;
				}
				d.r1 -= alpha * A_dot_p1;
			}
			if (dot_r_g == 0) break;
			const double old = dot_r_g;
			dot_r_g = 0;
			for (const auto& ci : cell_info) {
				const PoissonCell& d = at(ci.first);
				if (d.type == PO_SOLVE) dot_r_g += d.r0 * d.r1;
			}
			const double beta = dot_r_g / old;
			for (const auto& ci : cell_info) {  // 497-504
				PoissonCell& d = at(ci.first);
				if (d.type == PO_SOLVE) {
					d.p0 = d.r0 + beta * d.p0;
					d.p1 = d.r1 + beta * d.p1;
				}
			}
		} while (iteration < max_iterations);
		for (const auto& ci : cell_info) {
			PoissonCell& d = at(ci.first);
			if (d.type == PO_SOLVE) d.solution = d.best_solution;
		}
		iterations = iteration;
		residual_min = residual_min_;
	}

	// solve_failsafe 531-634 (Jacobi-like); best_solution holds the next value
	void solve_failsafe() {
		unsigned iteration = 0;
		double norm = std::numeric_limits<double>::max();
		while (iteration++ < max_iterations && norm > stop_residual) {
			norm = 0;
			for (const auto& ci : cell_info) {
				PoissonCell& d = at(ci.first);
				if (d.type != PO_SOLVE) continue;
				if (d.scaling_factor == 0) throw std::runtime_error("poisson: zero scaling factor");
				const double inv = -1.0 / d.scaling_factor;
				d.best_solution = -inv * d.rhs;
				for (const auto& nb : ci.second) {
					double mul = d.f[po_fi(nb.direction)];
					if (nb.rel > 0) mul /= 4.0;
					d.best_solution += inv * mul * at(nb.id).solution;
				}
				norm += std::fabs(d.solution - d.best_solution);
			}
			for (const auto& ci : cell_info) {
				PoissonCell& d = at(ci.first);
				if (d.type == PO_SOLVE) d.solution = d.best_solution;
			}
		}
		iterations = iteration - 1;  // loop bodies executed (the test post-increments)
		residual_min = norm;
	}
};

}  // namespace oracle

/* ===========================================================================
 * C ABI of the oracle (consumed by oracle/oracle.py through ctypes)
 * ========================================================================= */
using namespace oracle;

struct OracleHandle {
	Grid g;
	std::unordered_map<uint64_t, AdvCell> adv;
	std::set<uint64_t> adv_refine, adv_keep, adv_unrefine;  // check_for_adaptation's sets
	std::unordered_map<uint64_t, uint32_t> gol;
	std::unordered_map<uint64_t, GolAmrData> gola;
	PoissonSolver po;
	std::string err;
};

static thread_local std::string g_err;

#define OR_TRY(body)                        \
	try {                                   \
		body                                \
	} catch (const std::exception& e) {     \
		g_err = e.what();                   \
		return -1;                          \
	}

extern "C" {

const char* or_last_error() { return g_err.c_str(); }

/* mapping on a bare Mapping (no grid needed) */
static Mapping mk_map(const uint64_t* len, int R) {
	Mapping m;
	m.len[0] = len[0];
	m.len[1] = len[1];
	m.len[2] = len[2];
	m.R = R;
	m.update_last();
	return m;
}

uint64_t or_last_cell(const uint64_t* len, int R) { return mk_map(len, R).last; }
int or_max_possible_level(const uint64_t* len) { return mk_map(len, 0).max_possible_level(); }

/* batch mapping: for each id -> level, indices[3], cell length, parent, child,
   level0 parent, siblings[8] */
void or_map_batch(const uint64_t* len, int R, const uint64_t* ids, size_t n, int32_t* level, uint64_t* ind,
                  uint64_t* clen, uint64_t* parent, uint64_t* child, uint64_t* l0p, uint64_t* sib) {
	const Mapping m = mk_map(len, R);
	for (size_t i = 0; i < n; i++) {
		level[i] = m.level(ids[i]);
		const idx3 t = m.indices(ids[i]);
		for (int d = 0; d < 3; d++) ind[3 * i + d] = t[d];
		clen[i] = m.cell_len(ids[i]);
		parent[i] = m.parent(ids[i]);
		child[i] = m.child(ids[i]);
		l0p[i] = m.level0_parent(ids[i]);
		const auto s = m.siblings(ids[i]);
		for (int k = 0; k < 8; k++) sib[8 * i + k] = s[k];
	}
}

void or_from_indices_batch(const uint64_t* len, int R, const uint64_t* ind, const int32_t* lvl, size_t n,
                           uint64_t* out) {
	const Mapping m = mk_map(len, R);
	for (size_t i = 0; i < n; i++) out[i] = m.from_indices({ind[3 * i], ind[3 * i + 1], ind[3 * i + 2]}, lvl[i]);
}

void* or_grid_create(const uint64_t* len, int R, int px, int py, int pz, unsigned hood_len, int nprocs) {
	try {
		auto* h = new OracleHandle();
		Grid& g = h->g;
		g.m = mk_map(len, R);
		g.periodic[0] = px != 0;
		g.periodic[1] = py != 0;
		g.periodic[2] = pz != 0;
		g.hood_len = hood_len;
		g.nprocs = nprocs;
		g.init_hoods();
		g.create_level_0_cells();
		g.rebuild();
		return h;
	} catch (const std::exception& e) {
		g_err = e.what();
		return nullptr;
	}
}

void or_grid_destroy(void* h) { delete static_cast<OracleHandle*>(h); }

/* replace the leaf set wholesale (ids + owners) and rebuild: a repartition
 * (balance_load), which drops the pending requests and the dont sets
 * (dccrg.hpp:3808-3813) */
int or_grid_set_cells(void* hp, const uint64_t* ids, const int32_t* owners, size_t n) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		h->g.to_refine.clear();
		h->g.to_unrefine.clear();
		h->g.not_to_refine.clear();
		h->g.not_to_unrefine.clear();
		h->g.cell_process.clear();
		for (size_t i = 0; i < n; i++) h->g.cell_process[ids[i]] = owners[i];
		h->g.rebuild();
		return 0;
	})
}

size_t or_grid_num_cells(void* hp) { return static_cast<OracleHandle*>(hp)->g.cell_process.size(); }

/* sorted leaf ids and their owners */
void or_grid_cells(void* hp, uint64_t* ids, int32_t* owners) {
	auto* h = static_cast<OracleHandle*>(hp);
	std::vector<std::pair<uint64_t, int>> v(h->g.cell_process.begin(), h->g.cell_process.end());
	std::sort(v.begin(), v.end());
	for (size_t i = 0; i < v.size(); i++) {
		ids[i] = v[i].first;
		owners[i] = v[i].second;
	}
}

int or_refine_completely(void* hp, uint64_t c) { return static_cast<OracleHandle*>(hp)->g.refine_completely(c) ? 1 : 0; }
int or_unrefine_completely(void* hp, uint64_t c) {
	try {
		return static_cast<OracleHandle*>(hp)->g.unrefine_completely(c) ? 1 : 0;
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}
int or_dont_unrefine(void* hp, uint64_t c) { return static_cast<OracleHandle*>(hp)->g.dont_unrefine(c) ? 1 : 0; }
int or_dont_refine(void* hp, uint64_t c) { return static_cast<OracleHandle*>(hp)->g.dont_refine(c) ? 1 : 0; }
/* cells removed by the last stop_refining and their parent's process */
size_t or_removed(void* hp, uint64_t* ids, int32_t* owners) {
	auto* h = static_cast<OracleHandle*>(hp);
	std::vector<std::pair<uint64_t, int>> v(h->g.removed_to.begin(), h->g.removed_to.end());
	std::sort(v.begin(), v.end());
	if (ids)
		for (size_t i = 0; i < v.size(); i++) {
			ids[i] = v[i].first;
			owners[i] = v[i].second;
		}
	return v.size();
}

int64_t or_stop_refining(void* hp) {
	try {
		return int64_t(static_cast<OracleHandle*>(hp)->g.stop_refining().size());
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

/* face-neighbor cache entry (neighbors_[cell]) */
int or_neighbors_(void* hp, uint64_t c, uint64_t* out6) {
	auto* h = static_cast<OracleHandle*>(hp);
	auto it = h->g.neighbors_.find(c);
	if (it == h->g.neighbors_.end()) return -1;
	for (int i = 0; i < 6; i++) out6[i] = it->second[i];
	return 0;
}

/* kind: 0 = neighbors_of (stencil order), 1 = neighbors_to (sorted),
         2 = iterator cell.neighbors_of.  Returns count, fills up to cap. */
int64_t or_neighbors(void* hp, uint64_t c, int kind, uint64_t* ids, int32_t* offs, size_t cap) {
	auto* h = static_cast<OracleHandle*>(hp);
	try {
		const nlist* src = nullptr;
		nlist tmp;
		if (kind == 0) src = &h->g.nof.at(c);
		else if (kind == 1) src = &h->g.nto.at(c);
		else {
			tmp = h->g.iterator_neighbors_of(c);
			src = &tmp;
		}
		const size_t n = src->size();
		for (size_t i = 0; i < n && i < cap; i++) {
			ids[i] = (*src)[i].first;
			for (int d = 0; d < 3; d++) offs[3 * i + d] = (*src)[i].second[d];
		}
		return int64_t(n);
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

/* neighbors_of with a user-given neighborhood (find_neighbors_of with an
   arbitrary hood; add_neighborhood semantics dccrg.hpp:6383-6555) */
int64_t or_neighbors_of_hood(void* hp, uint64_t c, const int32_t* hood, size_t nh, uint64_t* ids, int32_t* offs,
                             size_t cap) {
	auto* h = static_cast<OracleHandle*>(hp);
	try {
		std::vector<off3> hv;
		for (size_t i = 0; i < nh; i++) hv.push_back({hood[3 * i], hood[3 * i + 1], hood[3 * i + 2]});
		const nlist r = h->g.find_neighbors_of(c, hv);
		for (size_t i = 0; i < r.size() && i < cap; i++) {
			ids[i] = r[i].first;
			for (int d = 0; d < 3; d++) offs[3 * i + d] = r[i].second[d];
		}
		return int64_t(r.size());
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

int64_t or_face_neighbors(void* hp, uint64_t c, uint64_t* ids, int32_t* dirs, size_t cap) {
	auto* h = static_cast<OracleHandle*>(hp);
	try {
		const auto r = h->g.face_neighbors_of(c);
		for (size_t i = 0; i < r.size() && i < cap; i++) {
			ids[i] = r[i].first;
			dirs[i] = r[i].second;
		}
		return int64_t(r.size());
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

/* per-rank view: what=0 local,1 inner,2 outer,3 local_bdy,4 remote_bdy;
   returns count */
int64_t or_rank_cells(void* hp, int rank, int what, uint64_t* out, size_t cap) {
	auto* h = static_cast<OracleHandle*>(hp);
	const auto v = h->g.rank_view(rank);
	std::vector<uint64_t> s;
	switch (what) {
	case 0: s = v.local; break;
	case 1: s = v.inner; break;
	case 2: s = v.outer; break;
	case 3: s.assign(v.local_bdy.begin(), v.local_bdy.end()); break;
	case 4: s.assign(v.remote_bdy.begin(), v.remote_bdy.end()); break;
	default: return -1;
	}
	for (size_t i = 0; i < s.size() && i < cap; i++) out[i] = s[i];
	return int64_t(s.size());
}

/* send (dir=0) or receive (dir=1) list of rank for peer; returns count */
int64_t or_rank_list(void* hp, int rank, int peer, int dir, uint64_t* out, size_t cap) {
	auto* h = static_cast<OracleHandle*>(hp);
	const auto v = h->g.rank_view(rank);
	const auto& mp = dir == 0 ? v.send : v.recv;
	auto it = mp.find(peer);
	if (it == mp.end()) return 0;
	for (size_t i = 0; i < it->second.size() && i < cap; i++) out[i] = it->second[i];
	return int64_t(it->second.size());
}

/* ---- game of life ---- */
int or_gol_set(void* hp, const uint64_t* ids, const uint32_t* alive, size_t n) {
	auto* h = static_cast<OracleHandle*>(hp);
	h->gol.clear();
	for (const auto& cp : h->g.cell_process) h->gol[cp.first] = 0;
	for (size_t i = 0; i < n; i++) h->gol[ids[i]] = alive[i];
	return 0;
}

int or_gol_steps(void* hp, int steps) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		for (int s = 0; s < steps; s++) gol_step(h->g, h->gol);
		return 0;
	})
}

int or_gol_get(void* hp, const uint64_t* ids, uint32_t* alive, size_t n) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		for (size_t i = 0; i < n; i++) alive[i] = h->gol.at(ids[i]);
		return 0;
	})
}

/* ---- game of life, refined (solve.hpp) ---- */
int or_gola_set(void* hp, const uint64_t* ids, const uint32_t* alive, size_t n) {
	auto* h = static_cast<OracleHandle*>(hp);
	h->gola.clear();
	for (const auto& cp : h->g.cell_process) h->gola[cp.first] = GolAmrData{};
	for (size_t i = 0; i < n; i++) h->gola[ids[i]][0] = alive[i];
	return 0;
}

int or_gola_steps(void* hp, int steps) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		for (int s = 0; s < steps; s++) gol_amr_step(h->g, h->gola);
		return 0;
	})
}

// only the collect loop; then the lists data[1..8] of the cells (8 per id)
int or_gola_collect(void* hp, const uint64_t* ids, uint64_t* lists, size_t n) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		std::vector<uint64_t> cells;
		for (const auto& cp : h->g.cell_process) cells.push_back(cp.first);
		std::sort(cells.begin(), cells.end());
		gol_amr_collect(h->g, h->gola, cells);
		for (size_t i = 0; i < n; i++)
			for (int k = 0; k < 8; k++) lists[8 * i + size_t(k)] = h->gola.at(ids[i])[size_t(k) + 1];
		return 0;
	})
}

int or_gola_get(void* hp, const uint64_t* ids, uint32_t* alive, size_t n) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		for (size_t i = 0; i < n; i++) alive[i] = uint32_t(h->gola.at(ids[i])[0]);
		return 0;
	})
}

/* ---- advection ---- */
void or_set_geometry(void* hp, const double* start, const double* l0) {
	auto* h = static_cast<OracleHandle*>(hp);
	for (int d = 0; d < 3; d++) {
		h->g.start[d] = start[d];
		h->g.l0[d] = l0[d];
	}
}

void or_geometry_batch(void* hp, const uint64_t* ids, size_t n, double* center, double* length) {
	auto* h = static_cast<OracleHandle*>(hp);
	for (size_t i = 0; i < n; i++) {
		const auto c = h->g.get_center(ids[i]);
		const auto l = h->g.get_length(ids[i]);
		for (int d = 0; d < 3; d++) {
			center[3 * i + d] = c[d];
			length[3 * i + d] = l[d];
		}
	}
}

int or_adv_initialize(void* hp) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		h->adv.clear();
		adv_initialize(h->g, h->adv);
		return 0;
	})
}

/* pre-refinement rounds as tests/advection/2d.cpp:260-285 (refines only) */
int64_t or_adv_prerefine(void* hp, double relative_diff, double diff_threshold) {
	try {
		auto* h = static_cast<OracleHandle*>(hp);
		int64_t total = 0;
		for (int lvl = 0; lvl < h->g.m.R; lvl++) {
			adv_initialize(h->g, h->adv);
			const auto cand = adv_refine_candidates(h->g, h->adv, relative_diff / h->g.m.R, diff_threshold);
			for (auto c : cand) h->g.refine_completely(c);
			total += int64_t(h->g.stop_refining().size());
			h->adv.clear();
		}
		adv_initialize(h->g, h->adv);
		return total;
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

double or_adv_max_time_step(void* hp) { return adv_max_time_step(static_cast<OracleHandle*>(hp)->adv); }

/* check_for_adaptation (tests/advection/adapter.hpp:47-178), single address
   space, cells in ascending id order: the three sets, kept for adapt */
int or_adv_check(void* hp, double diff_increase, double diff_threshold, double unrefine_sensitivity) {
	try {
		auto* h = static_cast<OracleHandle*>(hp);
		Grid& g = h->g;
		auto& cells = h->adv;
		std::set<uint64_t>& to_refine = h->adv_refine;
		std::set<uint64_t>& not_to_unrefine = h->adv_keep;
		std::set<uint64_t>& to_unrefine = h->adv_unrefine;
		to_refine.clear();
		not_to_unrefine.clear();
		to_unrefine.clear();
		if (g.m.R == 0) return 0;
		(void)adv_refine_candidates(g, cells, diff_increase, diff_threshold);  // max_diff of every cell (d[5])
		std::vector<uint64_t> ids;
		for (const auto& cp : g.cell_process) ids.push_back(cp.first);
		std::sort(ids.begin(), ids.end());
		for (const uint64_t id : ids) {  // 124-176
			const int lvl = g.m.level(id);
			const double refine_diff = (lvl + 1) * diff_increase, unrefine_diff = unrefine_sensitivity * refine_diff;
			const auto sib = g.m.siblings(id);
			const double diff = cells.at(id).d[5];
			if (diff > refine_diff) {
				to_refine.insert(id);
				for (const uint64_t s : sib) {
					to_unrefine.erase(s);
					not_to_unrefine.erase(s);
				}
			} else if (diff >= unrefine_diff) {
				bool dont = true;
				for (const uint64_t s : sib)
					if (to_refine.count(s) || not_to_unrefine.count(s)) {
						dont = false;
						break;
					}
				if (dont && lvl > 0) {
					not_to_unrefine.insert(id);
					for (const uint64_t s : sib) to_unrefine.erase(s);
				}
			} else {
				bool unref = true;
				for (const uint64_t s : sib)
					if (to_refine.count(s) || not_to_unrefine.count(s)) {
						unref = false;
						break;
					}
				if (unref && lvl > 0) to_unrefine.insert(id);
			}
		}
		return 0;
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

/* adapt_grid (adapter.hpp:187-309) with the sets of or_adv_check; the
   removed children's densities are summed in ascending id (the reference's
   get_removed_cells order is hash order).  out2: created, removed. */
int or_adv_adapt(void* hp, int64_t* out2) {
	try {
		auto* h = static_cast<OracleHandle*>(hp);
		Grid& g = h->g;
		auto& cells = h->adv;
		out2[0] = out2[1] = 0;
		if (g.m.R == 0) return 0;
		for (const uint64_t c : h->adv_refine) g.refine_completely(c);  // 200-231
		for (const uint64_t c : h->adv_keep) g.dont_unrefine(c);
		for (const uint64_t c : h->adv_unrefine) g.unrefine_completely(c);
		h->adv_refine.clear();
		h->adv_keep.clear();
		h->adv_unrefine.clear();
		const std::vector<uint64_t> created = g.stop_refining();
		for (const uint64_t c : created) {  // 236-250
			AdvCell a{};
			a.d[0] = cells.at(g.m.parent(c)).d[0];
			cells[c] = a;
		}
		std::vector<uint64_t> removed;
		for (const auto& kv : g.removed_to) removed.push_back(kv.first);
		std::sort(removed.begin(), removed.end());
		for (const uint64_t r : removed) {  // 252-275
			AdvCell& p = cells[g.m.parent(r)];
			for (int k = 0; k < 9; k++) p.d[k] = 0;
		}
		for (const uint64_t r : removed) cells[g.m.parent(r)].d[0] += cells.at(r).d[0] / 8;  // 276-290
		for (const uint64_t r : removed) cells.erase(r);
		for (auto it = cells.begin(); it != cells.end();) {  // refined parents
			if (!g.exists(it->first)) it = cells.erase(it);
			else ++it;
		}
		for (const auto& cp : g.cell_process) {  // 294-305
			AdvCell& c = cells.at(cp.first);
			const auto ctr = g.get_center(cp.first);
			c.d[1] = get_vx(ctr[1]);
			c.d[2] = get_vy(ctr[0]);
			c.d[3] = 0;
			const auto L = g.get_length(cp.first);
			c.d[6] = L[0];
			c.d[7] = L[1];
			c.d[8] = L[2];
		}
		out2[0] = int64_t(created.size());
		out2[1] = int64_t(removed.size());
		return 0;
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

/* `steps` time steps of calculate_fluxes(inner) + calculate_fluxes(outer) +
   apply_fluxes for every rank's cells (tests/advection/2d.cpp:327-395 with
   adapt_n = 0).  Cells of one rank are processed inner-then-outer in
   ascending id order; neighbor.is_local follows cell_process. */
int or_adv_steps(void* hp, int steps, double dt) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		Grid& g = h->g;
		std::vector<Grid::RankView> views;
		for (int r = 0; r < g.nprocs; r++) views.push_back(g.rank_view(r));
		for (int s = 0; s < steps; s++) {
			for (int r = 0; r < g.nprocs; r++) {
				// remote copies hold the owner's density of this step (densities
				// only change in apply_fluxes), so reading the owner's object is
				// what the halo-updated copy would hold
				auto is_local = [&](uint64_t n) { return g.cell_process.at(n) == r; };
				for (auto c : views[r].inner) adv_cell_fluxes(g, c, dt, h->adv, is_local);
				for (auto c : views[r].outer) adv_cell_fluxes(g, c, dt, h->adv, is_local);
			}
			for (auto& kv : h->adv) {
				kv.second.d[0] += kv.second.d[4];
				kv.second.d[4] = 0;
			}
		}
		return 0;
	})
}

int or_adv_get(void* hp, const uint64_t* ids, size_t n, double* out9) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		for (size_t i = 0; i < n; i++)
			for (int k = 0; k < 9; k++) out9[9 * i + k] = h->adv.at(ids[i]).d[k];
		return 0;
	})
}

/* ---- Poisson (tests/poisson/poisson_solve.hpp) ----
   cells: every leaf must be listed once; type 0 solve, 1 boundary, 2 skip
   (the reference's `cells` / default / `cells_to_skip`, 836-878) */
int or_po_set(void* hp, const uint64_t* ids, const double* rhs, const double* solution, const int32_t* type, size_t n) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		h->po.cells.clear();
		for (size_t i = 0; i < n; i++) {
			PoissonCell c;
			c.rhs = rhs[i];
			c.solution = solution[i];
			c.type = type[i];
			h->po.cells[ids[i]] = c;
		}
		for (const auto& cp : h->g.cell_process)
			if (!h->po.cells.count(cp.first)) throw std::runtime_error("poisson: leaf without data");
		return 0;
	})
}

/* solve (failsafe = 0) or solve_failsafe (1) with the given parameters
   (constructor 187-201), cells visited in ascending (reverse = 0) or
   descending id order; returns iterations, *residual = minimum residual
   (solve) or last norm (failsafe) */
int64_t or_po_solve(void* hp, unsigned max_it, unsigned min_it, double stop_residual, double p_of_norm,
                    double stop_increase, int failsafe, int reverse, double* residual) {
	try {
		auto* h = static_cast<OracleHandle*>(hp);
		PoissonSolver& s = h->po;
		s.max_iterations = max_it;
		s.min_iterations = min_it;
		s.stop_residual = stop_residual;
		s.p_of_norm = p_of_norm;
		s.stop_after_residual_increase = stop_increase;
		s.reverse = reverse != 0;
		s.cache_system_info(h->g);
		if (failsafe) s.solve_failsafe();
		else s.solve();
		*residual = s.residual_min;
		return int64_t(s.iterations);
	} catch (const std::exception& e) {
		g_err = e.what();
		return -1;
	}
}

/* per cell: solution, best_solution, p0, p1, r0, r1, A_dot_p0,
   scaling_factor, f[-x,+x,-y,+y,-z,+z], type (16 values) */
int or_po_get(void* hp, const uint64_t* ids, size_t n, double* out16) {
	OR_TRY({
		auto* h = static_cast<OracleHandle*>(hp);
		for (size_t i = 0; i < n; i++) {
			const PoissonCell& c = h->po.cells.at(ids[i]);
			double* o = out16 + 16 * i;
			o[0] = c.solution; o[1] = c.best_solution; o[2] = c.p0; o[3] = c.p1; o[4] = c.r0; o[5] = c.r1;
			o[6] = c.A_dot_p0; o[7] = c.scaling_factor;
			for (int k = 0; k < 6; k++) o[8 + k] = c.f[k];
			o[14] = double(c.type);
			o[15] = 0;
		}
		return 0;
	})
}

}  // extern "C"
