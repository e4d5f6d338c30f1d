// Neighbor search primitives shared by the device build kernels and the host
// (refinement closure, single-cell queries).
//
// The reference finds neighbors_of by *walking* the face-neighbor cache from
// the cell to each stencil box (dccrg.hpp:4339-4680), one std::map probe per
// hop.  Under dccrg's own invariants (leaves tile the grid, refinement is
// aligned, and induce_refines 9591-9720 keeps every leaf in a stencil box
// within one level of the cell) the cell that walk lands on is fully
// determined by the box itself:
//
//   box min  b = cell_min + h * len (finest-level units, unwrapped)
//   - the level L+1 leaf at wrap(b) exists  -> the box is split: emit its 8
//     children in z-order with offsets h*len + {0,len/2}^3 (4644-4676)
//   - the level L   leaf at wrap(b) exists  -> emit (it, h*len)
//   - the level L-1 leaf containing wrap(b) -> emit (it, its unwrapped min
//     corner - cell_min) (what adjust_offset 4405-4527 accumulates)
//   - outside a non-periodic boundary / none -> dropped (4634-4636)
//
// so each stencil item costs <= 3 O(1) existence probes and the items are
// independent: one wavefront lane per item.  tests/test_gpu_neighbors.py
// checks this against the oracle's literal walk on random refined meshes.
#pragma once

#include "dccrgx_mapping.hpp"

namespace dccrgx {

// Result of one stencil item: up to 8 (id, offset) pairs.
struct ItemOut {
	int n;
	uint64_t id[8];
	int32_t off[8][3];
};

// The case of one stencil item (find_neighbors_of 4339-4460): 0 outside a
// non-periodic boundary or no leaf, 1 the eight finer leaves, 2 the
// same-size leaf, 3 the coarser one; w = the item's wrapped index.  Kernels
// take the case and form the ids from it (item_id) instead of an ItemOut in
// private memory.
template <class Exists>
DX_HD int nof_item_case(const MapCtx& m, const uint64_t c[3], int lvl, const int32_t h[3], const Exists& exists,
                        uint64_t w[3]) {
	const int64_t len = int64_t(1) << (m.R - lvl);
	for (int d = 0; d < 3; d++) {
		if (!map_wrap(m, d, int64_t(c[d]) + int64_t(h[d]) * len, w[d])) return 0;
	}
	if (lvl < m.R && exists(map_from_indices(m, w[0], w[1], w[2], lvl + 1))) return 1;
	if (exists(map_from_indices(m, w[0], w[1], w[2], lvl))) return 2;
	if (lvl > 0 && exists(map_from_indices(m, w[0], w[1], w[2], lvl - 1))) return 3;
	return 0;
}

DX_HD int item_count(int kind) { return kind == 1 ? 8 : (kind ? 1 : 0); }

// leaf i (< item_count) of an item's case and its offset (off may be null)
DX_HD uint64_t item_id(const MapCtx& m, int lvl, const int32_t h[3], int kind, const uint64_t w[3], int i,
                       int32_t* off) {
	const int64_t len = int64_t(1) << (m.R - lvl);
	if (kind == 1) {
		const int64_t hl = len / 2;
		const int dx = i & 1, dy = (i >> 1) & 1, dz = (i >> 2) & 1;
		if (off) {
			off[0] = int32_t(h[0] * len + dx * hl);
			off[1] = int32_t(h[1] * len + dy * hl);
			off[2] = int32_t(h[2] * len + dz * hl);
		}
		return map_from_indices(m, w[0] + dx * hl, w[1] + dy * hl, w[2] + dz * hl, lvl + 1);
	}
	if (kind == 2) {
		if (off)
			for (int d = 0; d < 3; d++) off[d] = int32_t(h[d] * len);
		return map_from_indices(m, w[0], w[1], w[2], lvl);
	}
	const uint64_t pl = uint64_t(len) * 2;
	if (off)
		for (int d = 0; d < 3; d++) off[d] = int32_t(h[d] * len - int64_t(w[d] & (pl - 1)));
	return map_from_indices(m, w[0], w[1], w[2], lvl - 1);
}

template <class Exists>
DX_HD void nof_item(const MapCtx& m, const uint64_t c[3], int lvl, const int32_t h[3], const Exists& exists,
                    ItemOut& o) {
	uint64_t w[3];
	const int kind = nof_item_case(m, c, lvl, h, exists, w);
	o.n = item_count(kind);
	for (int i = 0; i < o.n; i++) o.id[i] = item_id(m, lvl, h, kind, w, i, o.off[i]);
}

// indices_from_neighborhood (dccrg.hpp:4200-4316) for one hood item: the
// cell-sized step with periodic wrap; false if outside a non-periodic dim.
DX_HD bool hood_index(const MapCtx& m, const uint64_t ind[3], uint64_t L, const int32_t h[3], uint64_t out[3]) {
	for (int d = 0; d < 3; d++) {
		if (!map_wrap(m, d, int64_t(ind[d]) + int64_t(h[d]) * int64_t(L), out[d])) return false;
	}
	return true;
}

// Candidate k (0 <= k < 10*nh) of find_neighbors_to (dccrg.hpp:4708-4861):
//   [0, nh)      parent-level search around the parent   (lvl > 0)
//   [nh, 9nh)    child-level search around each of the 8 children (lvl < R)
//   [9nh, 10nh)  same-level search
// hood_to is the negated stencil.  Returns error_cell when the candidate does
// not exist as a leaf (found != get_child(found)).
template <class Exists>
DX_HD uint64_t nto_candidate(const MapCtx& m, const uint64_t c[3], int lvl, const int32_t* hood_to, int nh, int k,
                             const Exists& exists) {
	const uint64_t len = uint64_t(1) << (m.R - lvl);
	uint64_t base[3];
	uint64_t L;
	int tl;
	int item;
	if (k < nh) {
		if (lvl == 0) return error_cell;
		L = len * 2;
		for (int d = 0; d < 3; d++) base[d] = c[d] & ~(L - 1);
		tl = lvl - 1;
		item = k;
	} else if (k < 9 * nh) {
		if (lvl >= m.R) return error_cell;
		const int ch = (k - nh) / nh;
		item = (k - nh) % nh;
		L = len / 2;
		base[0] = c[0] + (ch & 1) * L;
		base[1] = c[1] + ((ch >> 1) & 1) * L;
		base[2] = c[2] + ((ch >> 2) & 1) * L;
		tl = lvl + 1;
	} else {
		L = len;
		for (int d = 0; d < 3; d++) base[d] = c[d];
		tl = lvl;
		item = k - 9 * nh;
	}
	uint64_t t[3];
	if (!hood_index(m, base, L, hood_to + 3 * item, t)) return error_cell;
	const uint64_t f = map_from_indices(m, t[0], t[1], t[2], tl);
	return exists(f) ? f : error_cell;
}

// Face neighbors in one direction (get_face_neighbors_of, dccrg.hpp:2806-2933,
// with the face cache update_neighbors_ 9324-9458 inlined): dir 0..5 =
// -x,+x,-y,+y,-z,+z.  Returns the count (0, 1 or 4) and their ids in the
// reference order: n0, n0+a, n0+b, n0+b+a with (a,b) the two in-face dims.
// The probe point of face direction `dir` (update_neighbors_ 9324-9381): the
// index just outside the cell's min corner across that face, wrapped; false
// outside a non-periodic boundary.
DX_HD bool face_probe(const MapCtx& m, const uint64_t c[3], int lvl, int dir, uint64_t p[3]) {
	const uint64_t len = uint64_t(1) << (m.R - lvl);
	const int d = dir >> 1;
	p[0] = c[0];
	p[1] = c[1];
	p[2] = c[2];
	const uint64_t maxi = m.glen[d] - 1;
	if ((dir & 1) == 0) {
		if (p[d] == 0) {
			if (!m.periodic[d]) return false;
			p[d] = maxi;
		} else {
			p[d]--;
		}
	} else {
		if (maxi < len || p[d] > maxi - len) {
			if (!m.periodic[d]) return false;
			p[d] = 0;
		} else {
			p[d] += len;
		}
	}
	return true;
}

template <class Exists>
DX_HD int face_dir(const MapCtx& m, const uint64_t c[3], int lvl, int dir, const Exists& exists, uint64_t out[4]) {
	const uint64_t len = uint64_t(1) << (m.R - lvl);
	const int d = dir >> 1;
	uint64_t p[3];
	if (!face_probe(m, c, lvl, dir, p)) return 0;
	// get_existing_cell over levels [lvl-1, lvl+1], finest first (11275-11308)
	const int lo = lvl == 0 ? 0 : lvl - 1;
	const int hi = lvl == m.R ? m.R : lvl + 1;
	for (int l = hi; l >= lo; l--) {
		const uint64_t f = map_from_indices(m, p[0], p[1], p[2], l);
		if (!exists(f)) continue;
		out[0] = f;
		if (l <= lvl) return 1;
		// finer: the other three cells of the box touching the face
		const int a = d == 0 ? 1 : 0;
		const int b = d == 2 ? 1 : 2;
		const uint64_t hl = len / 2;
		uint64_t q[3];
		for (int k = 0; k < 3; k++) q[k] = p[k] & ~(hl - 1);
		uint64_t qa[3] = {q[0], q[1], q[2]}, qb[3] = {q[0], q[1], q[2]}, qab[3] = {q[0], q[1], q[2]};
		qa[a] += hl;
		qb[b] += hl;
		qab[a] += hl;
		qab[b] += hl;
		out[1] = map_from_indices(m, qa[0], qa[1], qa[2], l);
		out[2] = map_from_indices(m, qb[0], qb[1], qb[2], l);
		out[3] = map_from_indices(m, qab[0], qab[1], qab[2], l);
		return 4;
	}
	return 0;
}

// Default neighborhood (initialize_neighborhoods, dccrg.hpp:7895-7954)
inline int default_hood(unsigned L, int32_t* out /* 3 * n */) {
	int n = 0;
	if (L == 0) {
		const int32_t f[6][3] = {{0, 0, -1}, {0, -1, 0}, {-1, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
		for (int i = 0; i < 6; i++)
			for (int d = 0; d < 3; d++) out[3 * i + d] = f[i][d];
		return 6;
	}
	const int l = int(L);
	for (int z = -l; z <= l; z++)
		for (int y = -l; y <= l; y++)
			for (int x = -l; x <= l; x++) {
				if (x == 0 && y == 0 && z == 0) continue;
				out[3 * n] = x;
				out[3 * n + 1] = y;
				out[3 * n + 2] = z;
				n++;
			}
	return n;
}

}  // namespace dccrgx
