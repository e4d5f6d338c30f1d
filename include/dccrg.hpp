/*
 * dccrg.hpp — C++ drop-in facade of dccrg::Dccrg<Cell_Data, Geometry> over
 * the MI355X-native C ABI (include/dccrgx.h, libdccrgx.so).
 *
 * Keeps the reference's namespace, class template, chainable setters and
 * query names (reference dccrg.hpp:145-7072).  Differences, by design:
 *   - the communicator is (rank, size, 128-byte RCCL id) instead of MPI_Comm
 *     (initialize 472-552); Dccrg::unique_id() makes the id on rank 0;
 *   - Cell_Data lives on the GPU as one AoS payload array over slots (local
 *     cells, then remote copies); the WHOLE struct is the halo payload
 *     (get_mpi_datatype 152-206 is not consulted).  operator[] returns a
 *     pointer into a host staging copy: call download() before reading and
 *     upload() after writing host-side, exactly where the reference would
 *     have touched cell data outside a device sweep;
 *   - device-side work uses SoA fields (add_field) and the built-in sweeps.
 */
#ifndef DCCRG_AMD_DCCRG_HPP
#define DCCRG_AMD_DCCRG_HPP

#include <algorithm>
#include <array>
#include <cstdint>
#include <tuple>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "dccrgx.h"

namespace dccrg {

static const uint64_t error_cell = 0;                     // dccrg_mapping.hpp:37
static const uint64_t error_index = 0xFFFFFFFFFFFFFFFFull;  // dccrg_mapping.hpp:40
static const int default_neighborhood_id = -0xDCC;        // dccrg.hpp:93

// dccrg_no_geometry.hpp / dccrg_cartesian_geometry.hpp parameter stand-ins
struct No_Geometry {
	struct Parameters {};
};
struct Cartesian_Geometry {
	struct Parameters {
		std::array<double, 3> start{{0, 0, 0}}, level_0_cell_length{{1, 1, 1}};
	};
};

namespace detail {
inline void check(int rc) {
	if (rc != DCCRGX_OK) throw std::runtime_error(std::string("dccrgx: ") + dccrgx_last_error());
}
}  // namespace detail

// Items of the iteration ranges (Neighbors_Item 7288-7340, Cells_Item
// 7364-7402): ids with data pointers into the host staging copy, so that a
// reference-style loop `for (const auto& cell: grid.local_cells_items())`
// `for (const auto& n: cell.neighbors_of) n.data->...` reads the payload
// downloaded last (the facade refreshes the items on download()).
template <class Cell_Data>
struct Neighbors_Item {
	uint64_t id;
	Cell_Data* data;
	int x, y, z;  // offset of the neighbor's min corner in index units
};
template <class Cell_Data>
struct Cells_Item {
	uint64_t id;
	Cell_Data* data;
	std::vector<Neighbors_Item<Cell_Data>> neighbors_of;  // sorted by (id, offset), no duplicates (11451-11500)
};

template <class Cell_Data, class Geometry = No_Geometry>
class Dccrg {
public:
	Dccrg() = default;
	Dccrg(const Dccrg&) = delete;
	Dccrg& operator=(const Dccrg&) = delete;
	~Dccrg() {
		if (g_) dccrgx_destroy(g_);
	}

	static std::array<char, 128> unique_id() {
		std::array<char, 128> id{};
		detail::check(dccrgx_get_unique_id(id.data()));
		return id;
	}

	// ---- setup (dccrg.hpp:8120-8230) ----------------------------------------
	Dccrg& set_initial_length(const std::array<uint64_t, 3>& l) {
		length_ = l;
		return *this;
	}
	Dccrg& set_maximum_refinement_level(const int l) {
		max_ref_ = l;
		return *this;
	}
	Dccrg& set_periodic(bool x, bool y, bool z) {
		periodic_ = {{x, y, z}};
		return *this;
	}
	Dccrg& set_neighborhood_length(unsigned n) {
		hood_ = n;
		return *this;
	}
	Dccrg& set_load_balancing_method(const std::string&) { return *this; }  // Zoltan: out of scope

	// initialize(comm) 472: comm = (rank, size, device, RCCL id or nullptr)
	Dccrg& initialize(int rank = 0, int size = 1, int device = 0, const void* rccl_id = nullptr) {
		detail::check(dccrgx_create(rank, size, device, rccl_id, &g_));
		detail::check(dccrgx_set_initial_length(g_, length_.data()));
		detail::check(dccrgx_set_maximum_refinement_level(g_, max_ref_));
		detail::check(dccrgx_set_periodic(g_, periodic_[0], periodic_[1], periodic_[2]));
		detail::check(dccrgx_set_neighborhood_length(g_, hood_));
		detail::check(dccrgx_initialize(g_));
		detail::check(dccrgx_add_field(g_, "Cell_Data", sizeof(Cell_Data), 1, &payload_));
		rank_ = rank;
		return *this;
	}

	Dccrg& set_geometry(const typename Geometry::Parameters& p) {
		set_geometry_impl(p);
		return *this;
	}

	dccrgx_grid* native() const { return g_; }
	int get_rank() const { return rank_; }

	// ---- mapping (dccrg_mapping.hpp) -----------------------------------------
	uint64_t get_cell_from_indices(const std::array<uint64_t, 3>& ind, int lvl) const {
		return dccrgx_get_cell_from_indices(g_, ind.data(), lvl);
	}
	std::array<uint64_t, 3> get_indices(uint64_t cell) const {
		std::array<uint64_t, 3> r{{error_index, error_index, error_index}};
		dccrgx_get_indices(g_, cell, r.data());
		return r;
	}
	int get_refinement_level(uint64_t cell) const { return dccrgx_get_refinement_level(g_, cell); }
	int get_maximum_refinement_level() const {
		int l = 0;
		detail::check(dccrgx_get_maximum_refinement_level(g_, &l));
		return l;
	}

	// ---- queries ----------------------------------------------------------------
	// get_cells (651), sorted ascending; selection instead of criteria
	std::vector<uint64_t> get_cells(int which = DCCRGX_CELLS_LOCAL) const {
		return fetch([&](uint64_t* o, size_t c, size_t* n) { return dccrgx_get_cells(g_, which, o, c, n); });
	}
	std::vector<uint64_t> local_cells() const { return get_cells(DCCRGX_CELLS_LOCAL); }
	std::vector<uint64_t> inner_cells() const { return get_cells(DCCRGX_CELLS_INNER); }
	std::vector<uint64_t> outer_cells() const { return get_cells(DCCRGX_CELLS_OUTER); }
	std::vector<uint64_t> remote_cells() const { return get_cells(DCCRGX_CELLS_REMOTE); }

	// get_neighbors_of (819): empty optional-like result (nullptr in the
	// reference) is signalled by `found == false`
	std::vector<std::pair<uint64_t, std::array<int, 3>>> get_neighbors_of(uint64_t cell, bool* found = nullptr) const {
		std::vector<std::pair<uint64_t, std::array<int, 3>>> r;
		size_t n = 0;
		int rc = dccrgx_get_neighbors_of(g_, cell, nullptr, nullptr, 0, &n);
		if (found) *found = rc != DCCRGX_ENOTFOUND;
		if (rc == DCCRGX_ENOTFOUND) return r;
		if (rc != DCCRGX_ERANGE) detail::check(rc);
		std::vector<uint64_t> ids(n);
		std::vector<int32_t> off(3 * n);
		detail::check(dccrgx_get_neighbors_of(g_, cell, ids.data(), off.data(), n, &n));
		for (size_t i = 0; i < n; i++) r.push_back({ids[i], {{off[3 * i], off[3 * i + 1], off[3 * i + 2]}}});
		return r;
	}
	std::vector<std::pair<uint64_t, std::array<int, 3>>> get_neighbors_to(uint64_t cell) const {
		std::vector<std::pair<uint64_t, std::array<int, 3>>> r;
		size_t n = 0;
		int rc = dccrgx_get_neighbors_to(g_, cell, nullptr, 0, &n);
		if (rc == DCCRGX_ENOTFOUND) return r;
		if (rc != DCCRGX_ERANGE) detail::check(rc);
		std::vector<uint64_t> ids(n);
		detail::check(dccrgx_get_neighbors_to(g_, cell, ids.data(), n, &n));
		for (auto i : ids) r.push_back({i, {{0, 0, 0}}});
		return r;
	}
	// get_neighbors_of / _to (819 / 883) for a user neighborhood id
	std::vector<std::pair<uint64_t, std::array<int, 3>>> get_neighbors_of(uint64_t cell, int neighborhood_id,
	                                                                      bool* found = nullptr) const {
		if (neighborhood_id == DCCRGX_DEFAULT_HOOD) return get_neighbors_of(cell, found);
		return user_neighbors(cell, neighborhood_id, 0, found);
	}
	std::vector<std::pair<uint64_t, std::array<int, 3>>> get_neighbors_to(uint64_t cell, int neighborhood_id) const {
		if (neighborhood_id == DCCRGX_DEFAULT_HOOD) return get_neighbors_to(cell);
		return user_neighbors(cell, neighborhood_id, 1, nullptr);
	}
	std::vector<std::pair<uint64_t, int>> get_face_neighbors_of(uint64_t cell) const {  // 2806
		std::vector<std::pair<uint64_t, int>> r;
		uint64_t ids[64];
		int32_t dirs[64];
		size_t n = 0;
		int rc = dccrgx_get_face_neighbors_of(g_, cell, ids, dirs, 64, &n);
		if (rc == DCCRGX_ENOTFOUND) return r;
		detail::check(rc);
		for (size_t i = 0; i < n; i++) r.push_back({ids[i], dirs[i]});
		return r;
	}
	bool is_local(uint64_t cell) const { return dccrgx_is_local(g_, cell) == 1; }  // 3270
	// the update lists of a neighborhood id (get_cells_to_send / _receive
	// 6900-6914 per id)
	std::vector<uint64_t> get_cells_to_send(int peer, int neighborhood_id = DCCRGX_DEFAULT_HOOD) const {
		if (neighborhood_id == DCCRGX_DEFAULT_HOOD)
			return fetch([&](uint64_t* o, size_t c, size_t* n) { return dccrgx_get_cells_to_send(g_, peer, o, c, n); });
		return fetch([&](uint64_t* o, size_t c, size_t* n) {
			return dccrgx_get_user_update_list(g_, neighborhood_id, peer, 0, o, c, n);
		});
	}
	std::vector<uint64_t> get_cells_to_receive(int peer, int neighborhood_id = DCCRGX_DEFAULT_HOOD) const {
		if (neighborhood_id == DCCRGX_DEFAULT_HOOD)
			return fetch([&](uint64_t* o, size_t c, size_t* n) { return dccrgx_get_cells_to_receive(g_, peer, o, c, n); });
		return fetch([&](uint64_t* o, size_t c, size_t* n) {
			return dccrgx_get_user_update_list(g_, neighborhood_id, peer, 1, o, c, n);
		});
	}

	// ---- user neighborhoods (add_neighborhood 6383, remove_neighborhood 6530) ----
	bool add_neighborhood(int neighborhood_id, const std::vector<std::array<int, 3>>& items) {
		std::vector<int32_t> o;
		for (const auto& it : items) o.insert(o.end(), it.begin(), it.end());
		return dccrgx_add_neighborhood(g_, neighborhood_id, o.data(), items.size()) == DCCRGX_OK;
	}
	Dccrg& remove_neighborhood(int neighborhood_id) {
		detail::check(dccrgx_remove_neighborhood(g_, neighborhood_id));
		return *this;
	}
	int get_process(uint64_t cell) const { return dccrgx_get_process(g_, cell); }   // 5807

	// ---- refinement / partition ----------------------------------------------
	bool refine_completely(uint64_t cell) { return dccrgx_refine_completely(g_, cell) == DCCRGX_OK; }
	std::vector<uint64_t> stop_refining() {
		size_t n = 0;
		detail::check(dccrgx_stop_refining(g_, nullptr, 0, &n));
		return fetch([&](uint64_t* o, size_t c, size_t* k) { return dccrgx_get_new_cells(g_, o, c, k); });
	}
	bool pin(uint64_t cell, int process) { return dccrgx_pin(g_, cell, process) == DCCRGX_OK; }
	bool unpin(uint64_t cell) { return dccrgx_unpin(g_, cell) == DCCRGX_OK; }
	Dccrg& balance_load(bool /*use_zoltan*/ = true) {
		detail::check(dccrgx_balance_load(g_));
		return *this;
	}
	// balance_load to an explicit partition: one owner per leaf, leaves ascending
	Dccrg& balance_load(const std::vector<uint64_t>& leaves, const std::vector<int32_t>& owners) {
		detail::check(dccrgx_balance_load_to(g_, leaves.data(), owners.data(), leaves.size()));
		return *this;
	}

	// ---- grid files (save_grid_data 1089, load_grid_data 1742) ------------------
	// the header is raw bytes (the reference takes (void*, count, MPI_Datatype))
	bool save_grid_data(const std::string& name, uint64_t offset, const void* header = nullptr,
	                    size_t header_bytes = 0) {
		upload();
		return dccrgx_save_grid_data(g_, name.c_str(), offset, header, header_bytes) == DCCRGX_OK;
	}
	// replaces initialize(): every setting comes from the file
	bool load_grid_data(const std::string& name, uint64_t offset, size_t header_bytes, int rank = 0, int size = 1,
	                    int device = 0, const void* rccl_id = nullptr) {
		detail::check(dccrgx_create(rank, size, device, rccl_id, &g_));
		detail::check(dccrgx_add_field(g_, "Cell_Data", sizeof(Cell_Data), 1, &payload_));
		rank_ = rank;
		if (dccrgx_load_grid_data(g_, name.c_str(), offset, header_bytes) != DCCRGX_OK) return false;
		download();
		return true;
	}

	// ---- Cell_Data payload (host staging) -----------------------------------
	void download() {
		size_t ns = 0;
		detail::check(dccrgx_get_counts(g_, nullptr, nullptr, nullptr, &ns));
		host_.resize(ns);
		ids_ = fetch([&](uint64_t* o, size_t c, size_t* n) { return dccrgx_get_slot_ids(g_, o, c, n); });
		if (ns) detail::check(dccrgx_field_download(g_, payload_, 0, ns, host_.data()));
	}
	void upload() {
		if (!host_.empty()) detail::check(dccrgx_field_upload(g_, payload_, 0, host_.size(), host_.data()));
	}
	// operator[] (756): local cell or remote copy in the host staging copy
	Cell_Data* operator[](uint64_t cell) {
		const int64_t s = dccrgx_get_slot(g_, cell);
		if (s < 0 || size_t(s) >= host_.size()) return nullptr;
		return &host_[size_t(s)];
	}

	// ---- iteration (inner_cells / outer_cells / local_cells 7478-7602) ------------
	// items of a selection, ascending id, each with its iterator neighbors_of;
	// data pointers are valid until the next download() or structural change
	std::vector<Cells_Item<Cell_Data>> cells_items(int which = DCCRGX_CELLS_LOCAL) {
		if (host_.empty()) download();
		size_t nl = 0, ns = 0;
		detail::check(dccrgx_get_counts(g_, nullptr, nullptr, nullptr, &ns));
		{
			size_t ni = 0, no = 0;
			detail::check(dccrgx_get_counts(g_, &ni, &no, nullptr, nullptr));
			nl = ni + no;
		}
		std::vector<uint32_t> ptr(nl + 1);
		size_t ne = 0;
		int rc = dccrgx_download_csr(g_, 0, ptr.data(), nullptr, nullptr, 0, &ne);
		if (rc != DCCRGX_OK && rc != DCCRGX_ERANGE) detail::check(rc);
		std::vector<uint64_t> nid(ne + 1);
		std::vector<int32_t> off(3 * ne + 3);
		detail::check(dccrgx_download_csr(g_, 0, ptr.data(), nid.data(), off.data(), ne, &ne));
		std::vector<Cells_Item<Cell_Data>> out;
		for (uint64_t id : get_cells(which)) {
			const int64_t s = dccrgx_get_slot(g_, id);
			Cells_Item<Cell_Data> it{id, &host_[size_t(s)], {}};
			for (uint32_t j = ptr[size_t(s)]; j < ptr[size_t(s) + 1]; j++) {
				const int64_t ns2 = dccrgx_get_slot(g_, nid[j]);
				it.neighbors_of.push_back({nid[j], ns2 >= 0 ? &host_[size_t(ns2)] : nullptr, off[3 * j], off[3 * j + 1],
				                           off[3 * j + 2]});
			}
			std::sort(it.neighbors_of.begin(), it.neighbors_of.end(), [](const auto& a, const auto& b) {
				return std::tie(a.id, a.x, a.y, a.z) < std::tie(b.id, b.x, b.y, b.z);
			});
			it.neighbors_of.erase(std::unique(it.neighbors_of.begin(), it.neighbors_of.end(),
			                                  [](const auto& a, const auto& b) {
				                                  return a.id == b.id && a.x == b.x && a.y == b.y && a.z == b.z;
			                                  }),
			                      it.neighbors_of.end());
			out.push_back(std::move(it));
		}
		return out;
	}
	std::vector<Cells_Item<Cell_Data>> local_cells_items() { return cells_items(DCCRGX_CELLS_LOCAL); }
	std::vector<Cells_Item<Cell_Data>> inner_cells_items() { return cells_items(DCCRGX_CELLS_INNER); }
	std::vector<Cells_Item<Cell_Data>> outer_cells_items() { return cells_items(DCCRGX_CELLS_OUTER); }

	// ---- halo (966, 5010-5367) -------------------------------------------------
	bool update_copies_of_remote_neighbors() { return dccrgx_update_copies_of_remote_neighbors(g_) == DCCRGX_OK; }
	bool start_remote_neighbor_copy_updates() { return dccrgx_start_remote_neighbor_copy_updates(g_) == DCCRGX_OK; }
	bool wait_remote_neighbor_copy_update_receives() {
		return dccrgx_wait_remote_neighbor_copy_update_receives(g_) == DCCRGX_OK;
	}
	bool wait_remote_neighbor_copy_update_sends() {
		return dccrgx_wait_remote_neighbor_copy_update_sends(g_) == DCCRGX_OK;
	}
	bool wait_remote_neighbor_copy_updates() { return dccrgx_wait_remote_neighbor_copy_updates(g_) == DCCRGX_OK; }
	bool update_copies_of_remote_neighbors(int neighborhood_id) {  // 966 with an id
		return dccrgx_update_copies_of_remote_neighbors_hood(g_, neighborhood_id) == DCCRGX_OK;
	}

	// ---- device SoA fields ------------------------------------------------------
	template <class T>
	int add_field(const std::string& name, bool transfer) {
		int id = -1;
		detail::check(dccrgx_add_field(g_, name.c_str(), sizeof(T), transfer ? 1 : 0, &id));
		return id;
	}
	int payload_field() const { return payload_; }

private:
	template <class F>
	static std::vector<uint64_t> fetch(F&& f) {
		size_t n = 0;
		int rc = f(nullptr, 0, &n);
		if (rc != DCCRGX_OK && rc != DCCRGX_ERANGE) detail::check(rc);
		std::vector<uint64_t> v(n);
		if (n) detail::check(f(v.data(), n, &n));
		return v;
	}
	std::vector<std::pair<uint64_t, std::array<int, 3>>> user_neighbors(uint64_t cell, int id, int kind,
	                                                                    bool* found) const {
		std::vector<std::pair<uint64_t, std::array<int, 3>>> r;
		size_t n = 0;
		int rc = dccrgx_get_user_neighbors(g_, id, cell, kind, nullptr, nullptr, 0, &n);
		if (found) *found = rc != DCCRGX_ENOTFOUND;
		if (rc == DCCRGX_ENOTFOUND) return r;
		if (rc != DCCRGX_ERANGE) detail::check(rc);
		std::vector<uint64_t> ids(n);
		std::vector<int32_t> off(3 * n);
		detail::check(dccrgx_get_user_neighbors(g_, id, cell, kind, ids.data(), off.data(), n, &n));
		for (size_t i = 0; i < n; i++)
			r.push_back({ids[i], kind == 0 ? std::array<int, 3>{{off[3 * i], off[3 * i + 1], off[3 * i + 2]}}
			                               : std::array<int, 3>{{0, 0, 0}}});
		return r;
	}
	void set_geometry_impl(const No_Geometry::Parameters&) {}
	void set_geometry_impl(const Cartesian_Geometry::Parameters& p) {
		detail::check(dccrgx_set_geometry(g_, p.start.data(), p.level_0_cell_length.data()));
	}

	dccrgx_grid* g_ = nullptr;
	int rank_ = 0, payload_ = -1;
	std::array<uint64_t, 3> length_{{1, 1, 1}};
	int max_ref_ = 0;
	std::array<bool, 3> periodic_{{false, false, false}};
	unsigned hood_ = 1;
	std::vector<Cell_Data> host_;
	std::vector<uint64_t> ids_;
};

}  // namespace dccrg

#endif
