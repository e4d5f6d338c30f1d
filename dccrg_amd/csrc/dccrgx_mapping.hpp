// Cell-id <-> index <-> refinement-level math, usable from host and device.
//
// Replaces dccrg::Mapping (reference dccrg_mapping.hpp:54-651).  Semantics
// are identical (ids are 1-based, level-major, x fastest; indices are in
// units of the finest level; error_cell = 0, error_index = ~0), but the
// per-level cumulative offsets and shifts are precomputed once into a small
// POD (MapCtx) that is passed by value to kernels, so every query is a few
// shifts/adds and at most one 64-bit division pair instead of the
// reference's O(R) loop per call.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define DX_HD __host__ __device__ __forceinline__
#else
#define DX_HD inline
#endif

namespace dccrgx {

static constexpr uint64_t error_cell = 0;
static constexpr uint64_t error_index = 0xFFFFFFFFFFFFFFFFull;
static constexpr int kMaxLevels = 24;

struct MapCtx {
	uint64_t len[3];          // level-0 grid length
	int R;                    // maximum refinement level
	int periodic[3];
	uint64_t glen[3];         // grid length in finest-level indices: len << R
	uint64_t first[kMaxLevels + 1];  // first id of level l (first[R+1] = last_cell + 1)
	uint64_t last;            // last valid cell id
	int lg[2];                // log2 of len[0], len[1] when both are powers of two, else -1
};

DX_HD void map_init(MapCtx& m, const uint64_t len[3], int R, const int per[3]) {
	for (int d = 0; d < 3; d++) {
		m.len[d] = len[d];
		m.periodic[d] = per[d];
		m.glen[d] = len[d] << R;
	}
	m.R = R;
	m.lg[0] = m.lg[1] = -1;
	if (len[0] && len[1] && !(len[0] & (len[0] - 1)) && !(len[1] & (len[1] - 1))) {
		m.lg[0] = m.lg[1] = 0;
		while ((uint64_t(1) << m.lg[0]) < len[0]) m.lg[0]++;
		while ((uint64_t(1) << m.lg[1]) < len[1]) m.lg[1]++;
	}
	const uint64_t g = len[0] * len[1] * len[2];
	uint64_t c = 1;
	for (int l = 0; l <= R; l++) {
		m.first[l] = c;
		c += g << (3 * l);
	}
	m.first[R + 1] = c;
	m.last = c - 1;
	for (int l = R + 2; l <= kMaxLevels; l++) m.first[l] = c;
}

// dccrg_mapping.hpp:261-289.  first[] is read at lane-uniform indices only: in
// a kernel the MapCtx is a kernel argument, and an index that differs between
// lanes turns each read into a dependent global load (scalar loads otherwise)
DX_HD int map_level(const MapCtx& m, uint64_t cell) {
	if (cell == error_cell || cell > m.last) return -1;
	int l = 0;
	for (int k = 1; k <= m.R; k++) l += cell >= m.first[k] ? 1 : 0;
	return l;
}

// bits of the largest cell id: every id is < 2^map_id_bits (radix sorts of
// ids take only these bits)
DX_HD int map_id_bits(const MapCtx& m) {
	int b = 1;
	while (b < 64 && (m.last >> b) != 0) b++;
	return b;
}

// m.first[l] (0 <= l <= R + 1) by lane-uniform reads (see map_level)
DX_HD uint64_t map_first(const MapCtx& m, int l) {
	uint64_t f = m.first[0];
	for (int k = 1; k <= m.R + 1; k++) f = k <= l ? m.first[k] : f;
	return f;
}

// dccrg_mapping.hpp:297-310
DX_HD uint64_t map_cell_len(const MapCtx& m, uint64_t cell) {
	const int l = map_level(m, cell);
	if (l < 0) return error_index;
	return uint64_t(1) << (m.R - l);
}

// dccrg_mapping.hpp:153-208
DX_HD uint64_t map_from_indices(const MapCtx& m, uint64_t x, uint64_t y, uint64_t z, int lvl) {
	if (x >= m.glen[0] || y >= m.glen[1] || z >= m.glen[2]) return error_cell;
	if (lvl < 0 || lvl > m.R) return error_cell;
	const int sh = m.R - lvl;
	const uint64_t lx = m.len[0] << lvl, ly = m.len[1] << lvl;
	return map_first(m, lvl) + (x >> sh) + (y >> sh) * lx + (z >> sh) * lx * ly;
}

// dccrg_mapping.hpp:217-253; returns level (-1 on error) and fills indices
DX_HD int map_indices(const MapCtx& m, uint64_t cell, uint64_t& x, uint64_t& y, uint64_t& z) {
	const int l = map_level(m, cell);
	if (l < 0) {
		x = y = z = error_index;
		return -1;
	}
	uint64_t c = cell - map_first(m, l);
	const int sh = m.R - l;
	if (m.lg[0] >= 0) {
		// power-of-two x and y lengths: the divisions are shifts
		const int bx = m.lg[0] + l, by = m.lg[1] + l;
		x = (c & ((uint64_t(1) << bx) - 1)) << sh;
		const uint64_t q = c >> bx;
		y = (q & ((uint64_t(1) << by) - 1)) << sh;
		z = (q >> by) << sh;
		return l;
	}
	const uint64_t lx = m.len[0] << l, ly = m.len[1] << l;
	if (((c | lx | ly) >> 32) == 0) {
		// 32-bit division when the operands fit (exact, a fraction of the
		// instructions of the 64-bit expansion on the device)
		const uint32_t c32 = uint32_t(c), lx32 = uint32_t(lx), ly32 = uint32_t(ly);
		const uint32_t q = c32 / lx32, q2 = q / ly32;
		x = uint64_t(c32 - q * lx32) << sh;
		y = uint64_t(q - q2 * ly32) << sh;
		z = uint64_t(q2) << sh;
		return l;
	}
	const uint64_t q = c / lx;
	x = (c - q * lx) << sh;
	const uint64_t q2 = q / ly;
	y = (q - q2 * ly) << sh;
	z = q2 << sh;
	return l;
}

// dccrg_mapping.hpp:367-383
DX_HD uint64_t map_parent(const MapCtx& m, uint64_t cell) {
	uint64_t x, y, z;
	const int l = map_indices(m, cell, x, y, z);
	if (l < 0) return error_cell;
	if (l == 0) return cell;
	return map_from_indices(m, x, y, z, l - 1);
}

// dccrg_mapping.hpp:338-356
DX_HD uint64_t map_child(const MapCtx& m, uint64_t cell) {
	uint64_t x, y, z;
	const int l = map_indices(m, cell, x, y, z);
	if (l < 0) return error_cell;
	if (l >= m.R) return cell;
	return map_from_indices(m, x, y, z, l + 1);
}

// dccrg_mapping.hpp:391-441 — children in z-order (x fastest)
DX_HD void map_all_children(const MapCtx& m, uint64_t cell, uint64_t out[8]) {
	for (int i = 0; i < 8; i++) out[i] = error_cell;
	uint64_t x, y, z;
	const int l = map_indices(m, cell, x, y, z);
	if (l < 0 || l >= m.R) return;
	const uint64_t o = uint64_t(1) << (m.R - l - 1);
	for (int i = 0; i < 8; i++)
		out[i] = map_from_indices(m, x + (i & 1) * o, y + ((i >> 1) & 1) * o, z + ((i >> 2) & 1) * o, l + 1);
}

// dccrg_mapping.hpp:449-470
DX_HD void map_siblings(const MapCtx& m, uint64_t cell, uint64_t out[8]) {
	const int l = map_level(m, cell);
	for (int i = 0; i < 8; i++) out[i] = error_cell;
	if (l < 0) return;
	if (l == 0) {
		out[0] = cell;
		return;
	}
	map_all_children(m, map_parent(m, cell), out);
}

// dccrg_mapping.hpp:479-493
DX_HD uint64_t map_level0_parent(const MapCtx& m, uint64_t cell) {
	uint64_t x, y, z;
	const int l = map_indices(m, cell, x, y, z);
	if (l < 0) return error_cell;
	if (l == 0) return cell;
	return map_from_indices(m, x, y, z, 0);
}

// Wrap a signed finest-level coordinate into the grid along dimension d.
// Returns false when the coordinate falls outside a non-periodic dimension.
DX_HD bool map_wrap(const MapCtx& m, int d, int64_t v, uint64_t& out) {
	const int64_t G = int64_t(m.glen[d]);
	if (v >= 0 && v < G) {
		out = uint64_t(v);
		return true;
	}
	if (!m.periodic[d]) return false;
	int64_t r = v % G;
	if (r < 0) r += G;
	out = uint64_t(r);
	return true;
}

}  // namespace dccrgx
