/*
 * dccrg.hpp - C++ drop-in facade of dccrg::Dccrg<Cell_Data, Geometry,
 * Additional_Cell_Items, Additional_Neighbor_Items> (reference dccrg.hpp:
 * 143-7072) over the MI355X-native C ABI (include/dccrgx.h, libdccrgx.so).
 *
 * A program written against the reference compiles against this header
 * unchanged except for the include line (examples/game_of_life.cpp of the
 * reference: tests/test_facade_cpu.py builds it, tests/test_gpu_facade.py
 * runs it at 1 and 2 MPI ranks).  Kept from the reference: the namespace,
 * the class template and its defaults, initialize(const MPI_Comm&) and the
 * chainable setters, the public mapping / topology / length / geometry
 * members, get_cells(criteria, exact_match, neighborhood_id, sorted),
 * operator[], get_neighbors_of / _to returning a pointer (nullptr for
 * unknown cells or neighborhoods), the iteration ranges inner_cells() /
 * outer_cells() / local_cells() / remote_cells() / all_cells() of Cells_Item
 * {id, data, neighbors_of, neighbors_to, all_neighbors} with Neighbors_Item
 * {id, data, x, y, z}, the Additional_*_Items update hooks, the halo
 * (update_copies_of_remote_neighbors and its start / wait split), the
 * process-boundary and update-count getters, refinement, pins and
 * balance_load, save / load_grid_data.
 *
 * How it works: Cell_Data lives in host memory for the user's loops, one
 * element per slot (local cells, then copies of remote neighbors), and is
 * mirrored in a device field of the library.  The halo moves exactly the
 * bytes Cell_Data::get_mpi_datatype() describes (dccrg_get_cell_datatype.hpp:
 * 40-340): local payloads go up, the library packs / exchanges / places them
 * on the device, the received bytes come back into the host copies.  Ranks
 * use RCCL when every rank of a node has its own GPU, otherwise the
 * library's host exchange over the caller's MPI communicator
 * (DCCRGX_TRANSPORT=host forces the latter).  Device-side sweeps use the
 * library directly (dccrgx_* calls on native()).
 *
 * Build: -I include -I <mpi include> ... -L dccrg_amd -ldccrgx -lmpi
 */
#ifndef DCCRG_AMD_DCCRG_HPP
#define DCCRG_AMD_DCCRG_HPP

#include <mpi.h>

// the standard headers the reference's dccrg.hpp and its helpers pull in
// (dccrg.hpp:20-56), which programs written against it rely on
#include <algorithm>
#include <array>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <iterator>
#include <limits>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "dccrg_get_cell_datatype.hpp"
#include "dccrgx.h"

namespace dccrg {

static const uint64_t error_cell = 0;                      // dccrg_mapping.hpp:37
static const uint64_t error_index = 0xFFFFFFFFFFFFFFFFull;  // dccrg_mapping.hpp:40
static const int default_neighborhood_id = DCCRGX_DEFAULT_HOOD;  // dccrg.hpp:93

// neighbor types of get_cells (dccrg.hpp:95-142)
static const int has_no_neighbor = 0, has_local_neighbor_of = (1 << 0), has_local_neighbor_to = (1 << 1),
                 has_remote_neighbor_of = (1 << 2), has_remote_neighbor_to = (1 << 3),
                 has_local_neighbor_both = has_local_neighbor_of | has_local_neighbor_to,
                 has_remote_neighbor_both = has_remote_neighbor_of | has_remote_neighbor_to;

namespace detail {
inline void check(int rc) {
	if (rc != DCCRGX_OK) throw std::runtime_error(std::string("dccrgx: ") + dccrgx_last_error());
}

template <class F>
std::vector<uint64_t> fetch_u64(F&& f) {
	size_t n = 0;
	int rc = f(nullptr, 0, &n);
	if (rc != DCCRGX_OK && rc != DCCRGX_ERANGE) check(rc);
	std::vector<uint64_t> v(n);
	if (n) check(f(v.data(), n, &n));
	return v;
}

// get_mpi_datatype dispatch: the reference's get_cell_mpi_datatype
// (include/dccrg_get_cell_datatype.hpp): a five-argument member before a
// zero-argument one, a named MPI type for arithmetic cells, else the bytes
template <class T>
mpi_transfer_t call_datatype(T& c, int) {
	return get_cell_mpi_datatype(c, error_cell, 0, 0, false, default_neighborhood_id);
}

// the datatype of one cell for a transfer (the five-argument member gets the
// cell, the processes and the direction, dccrg_get_cell_datatype.hpp:68-340)
template <class T>
mpi_transfer_t cell_datatype(T& c, uint64_t cell, int sender, int receiver, bool receiving, int hood, int) {
	return get_cell_mpi_datatype(c, cell, sender, receiver, receiving, hood);
}

inline bool is_named_datatype(MPI_Datatype t) {
	int ni = 0, na = 0, nd = 0, comb = 0;
	MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);
	return comb == MPI_COMBINER_NAMED;
}

// a Cell_Data that is not trivially copyable (e.g. std::vector members,
// tests/variable_data_size) is serialized with MPI_Pack over the datatype
// it describes and lives on the device as a variable-size field.  Limit: a
// cell is packed once, with sender == receiver == this rank, and that one
// byte string goes to every peer (the reference asks get_mpi_datatype per
// destination); a Cell_Data whose datatype depends on the peer is not
// supported.
template <class T>
void pack_cell(T& c, uint64_t cell, int sender, int receiver, int hood, MPI_Comm comm, std::vector<char>& out) {
	auto dt = cell_datatype(c, cell, sender, receiver, false, hood, 0);
	MPI_Datatype t = std::get<2>(dt);
	const bool named = is_named_datatype(t);
	if (!named) MPI_Type_commit(&t);
	int bound = 0;
	MPI_Pack_size(std::get<1>(dt), t, comm, &bound);
	const size_t at = out.size();
	out.resize(at + size_t(bound));
	int pos = 0;
	if (bound) MPI_Pack(std::get<0>(dt), std::get<1>(dt), t, out.data() + at, bound, &pos, comm);
	out.resize(at + size_t(pos));
	if (!named) MPI_Type_free(&t);
}

template <class T>
void unpack_cell(T& c, uint64_t cell, int sender, int receiver, int hood, MPI_Comm comm, const char* in, size_t bytes) {
	auto dt = cell_datatype(c, cell, sender, receiver, true, hood, 0);
	MPI_Datatype t = std::get<2>(dt);
	const bool named = is_named_datatype(t);
	if (!named) MPI_Type_commit(&t);
	int need = 0;
	MPI_Pack_size(std::get<1>(dt), t, comm, &need);
	if (size_t(need) < bytes) {
		if (!named) MPI_Type_free(&t);
		throw std::runtime_error("dccrg: received " + std::to_string(bytes) + " bytes for cell " + std::to_string(cell) +
		                         " whose datatype holds " + std::to_string(need) + " (size its data first)");
	}
	int pos = 0;
	if (bytes && size_t(need) > bytes) {
		// a shorter message than the receiving datatype describes: the
		// reference's MPI_Irecv fills only the bytes that arrived and leaves the
		// rest of the object as it was, so the object's own packed bytes are
		// overlaid with what arrived and unpacked whole
		std::vector<char> full(static_cast<size_t>(need));
		int at = 0;
		MPI_Pack(std::get<0>(dt), std::get<1>(dt), t, full.data(), need, &at, comm);
		std::memcpy(full.data(), in, bytes);
		MPI_Unpack(full.data(), at, &pos, std::get<0>(dt), std::get<1>(dt), t, comm);
	} else if (bytes) {
		MPI_Unpack(const_cast<char*>(in), int(bytes), &pos, std::get<0>(dt), std::get<1>(dt), t, comm);
	}
	if (!named) MPI_Type_free(&t);
}

// the halo window [offset, offset + bytes) of a Cell_Data: one contiguous
// run inside the object (a non-contiguous or out-of-object datatype sends
// the whole object)
template <class T>
std::pair<size_t, size_t> datatype_window() {
	T c{};
	const auto dt = call_datatype(c, 0);
	int sz = 0;
	MPI_Type_size(std::get<2>(dt), &sz);
	MPI_Aint lb = 0, extent = 0;
	MPI_Type_get_true_extent(std::get<2>(dt), &lb, &extent);
	const size_t bytes = size_t(std::get<1>(dt)) * size_t(sz);
	const char* base = reinterpret_cast<const char*>(&c);
	const char* p = static_cast<const char*>(std::get<0>(dt));
	const bool inside = p >= base && p + bytes <= base + sizeof(T);
	if (!inside || bytes == 0 || MPI_Aint(sz) != extent || lb != 0) return {0, sizeof(T)};
	return {size_t(p - base), bytes};
}

// the library's host exchange over MPI point-to-point (one message per peer
// each way, chunked below INT_MAX bytes)
inline int mpi_exchange(void* ctx, const void* const* send, const size_t* sb, void* const* recv, const size_t* rb) {
	MPI_Comm comm = *static_cast<MPI_Comm*>(ctx);
	int size = 0;
	MPI_Comm_size(comm, &size);
	const size_t chunk = size_t(1) << 30;
	std::vector<MPI_Request> req;
	for (int p = 0; p < size; p++)
		for (size_t o = 0; o < rb[p]; o += chunk) {
			req.emplace_back();
			MPI_Irecv(static_cast<char*>(recv[p]) + o, int(std::min(chunk, rb[p] - o)), MPI_BYTE, p, 0x7dc, comm,
			          &req.back());
		}
	for (int p = 0; p < size; p++)
		for (size_t o = 0; o < sb[p]; o += chunk) {
			req.emplace_back();
			MPI_Isend(static_cast<const char*>(send[p]) + o, int(std::min(chunk, sb[p] - o)), MPI_BYTE, p, 0x7dc, comm,
			          &req.back());
		}
	return MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE) == MPI_SUCCESS ? 0 : -1;
}
}  // namespace detail

// ---- value types (dccrg_types.hpp:34-86, dccrg_length.hpp, dccrg_topology.hpp,
// dccrg_mapping.hpp) --------------------------------------------------------
template <unsigned int Dimensions>
class Types {
public:
	// a cell's indices in units of the finest cells, x first
	typedef std::array<uint64_t, Dimensions> indices_t;
	// one neighborhood item: an offset in units of the cell's own size
	typedef std::array<int, Dimensions> neighborhood_item_t;
};

class Grid_Length {
public:
	std::array<uint64_t, 3> get() const { return l_; }
	bool set(const std::array<uint64_t, 3>& l) {
		if (l[0] == 0 || l[1] == 0 || l[2] == 0) return false;
		l_ = l;
		return true;
	}

private:
	std::array<uint64_t, 3> l_{{1, 1, 1}};
};

class Grid_Topology {
public:
	bool is_periodic(size_t d) const { return d < 3 && p_[d]; }
	bool set_periodicity(size_t d, bool v) {
		if (d > 2) return false;
		p_[d] = v;
		return true;
	}

private:
	std::array<bool, 3> p_{{false, false, false}};
};

// Mapping (dccrg_mapping.hpp:54-651) of the grid, answered by the library
class Mapping {
public:
	Grid_Length length;
	uint64_t get_cell_from_indices(const std::array<uint64_t, 3>& ind, int lvl) const {
		return g_ ? dccrgx_get_cell_from_indices(g_, ind.data(), lvl) : error_cell;
	}
	std::array<uint64_t, 3> get_indices(uint64_t cell) const {
		std::array<uint64_t, 3> r{{error_index, error_index, error_index}};
		if (g_) dccrgx_get_indices(g_, cell, r.data());
		return r;
	}
	int get_refinement_level(uint64_t cell) const { return g_ ? dccrgx_get_refinement_level(g_, cell) : -1; }
	int get_maximum_refinement_level() const {
		int l = 0;
		if (g_) dccrgx_get_maximum_refinement_level(g_, &l);
		return l;
	}
	uint64_t get_last_cell() const { return g_ ? dccrgx_get_last_cell(g_) : 0; }
	uint64_t get_cell_length_in_indices(uint64_t cell) const {
		const int l = get_refinement_level(cell);
		if (l < 0) return error_index;
		return uint64_t(1) << (get_maximum_refinement_level() - l);
	}
	uint64_t get_parent(uint64_t cell) const {
		const int l = get_refinement_level(cell);
		if (l < 0) return error_cell;
		if (l == 0) return cell;
		return get_cell_from_indices(get_indices(cell), l - 1);
	}
	uint64_t get_level_0_parent(uint64_t cell) const {
		const int l = get_refinement_level(cell);
		if (l < 0) return error_cell;
		return get_cell_from_indices(get_indices(cell), 0);
	}
	uint64_t get_child(uint64_t cell) const {
		const int l = get_refinement_level(cell);
		if (l < 0) return error_cell;
		if (l >= get_maximum_refinement_level()) return cell;
		return get_cell_from_indices(get_indices(cell), l + 1);
	}
	std::array<uint64_t, 8> get_all_children(uint64_t cell) const {
		std::array<uint64_t, 8> r;
		r.fill(error_cell);
		const int l = get_refinement_level(cell);
		if (l < 0 || l >= get_maximum_refinement_level()) return r;
		const auto ind = get_indices(cell);
		const uint64_t h = get_cell_length_in_indices(cell) / 2;
		for (int i = 0; i < 8; i++)
			r[size_t(i)] = get_cell_from_indices(
			    {{ind[0] + (i & 1) * h, ind[1] + ((i >> 1) & 1) * h, ind[2] + ((i >> 2) & 1) * h}}, l + 1);
		return r;
	}
	std::array<uint64_t, 8> get_siblings(uint64_t cell) const {
		std::array<uint64_t, 8> r;
		r.fill(error_cell);
		const int l = get_refinement_level(cell);
		if (l < 0) return r;
		if (l == 0) {
			r[0] = cell;
			return r;
		}
		return get_all_children(get_parent(cell));
	}
	void attach(dccrgx_grid* g) { g_ = g; }

private:
	dccrgx_grid* g_ = nullptr;
};

// ---- geometries (dccrg_no_geometry.hpp, dccrg_cartesian_geometry.hpp) ----
class No_Geometry {
public:
	struct Parameters {};
	static constexpr int geometry_id = 0;
	void attach(dccrgx_grid* g) { g_ = g; }
	Parameters get() const { return {}; }
	// parameters the library read from a grid file (load_grid_data)
	void sync_from_library() {}
	// the grid's length in level-0 cells and its periodicity, for geometries
	// that size their parameters by them (Stretched_Cartesian_Geometry, whose
	// parameters may be set before initialize)
	void attach_parts(const Grid_Length* l, const Grid_Topology* t) {
		length_ = l;
		topology_ = t;
	}
	bool set(const Parameters&) { return true; }
	// the geometry block save_grid_data writes (empty: the library's
	// Cartesian block) and the check of the block a load found (empty: a
	// Cartesian file), the reference's write / read of each geometry
	std::vector<char> file_block() const { return {}; }
	bool from_file_block(const std::vector<char>& b) {
		if (b.empty()) return true;
		std::cerr << "Wrong geometry: 2 (Stretched_Cartesian_Geometry) in the grid file" << std::endl;
		return false;
	}
	std::array<double, 3> get_length(uint64_t cell) const { return batch(cell, false); }
	std::array<double, 3> get_center(uint64_t cell) const { return batch(cell, true); }

protected:
	std::array<double, 3> batch(uint64_t cell, bool center) const {
		std::array<double, 3> c{{0, 0, 0}}, L{{0, 0, 0}};
		if (g_) dccrgx_geometry_batch(g_, &cell, 1, c.data(), L.data());
		return center ? c : L;
	}
	dccrgx_grid* g_ = nullptr;
	const Grid_Length* length_ = nullptr;
	const Grid_Topology* topology_ = nullptr;
};

struct Cartesian_Geometry_Parameters {
	std::array<double, 3> start{{0, 0, 0}}, level_0_cell_length{{1, 1, 1}};
};

class Cartesian_Geometry : public No_Geometry {
public:
	using Parameters = Cartesian_Geometry_Parameters;
	static constexpr int geometry_id = 1;
	bool set(const Parameters& p) {
		p_ = p;
		return !g_ || dccrgx_set_geometry(g_, p.start.data(), p.level_0_cell_length.data()) == DCCRGX_OK;
	}
	const Parameters& get() const { return p_; }
	void sync_from_library() {
		if (g_) dccrgx_get_geometry(g_, p_.start.data(), p_.level_0_cell_length.data());
	}
	std::array<double, 3> get_start() const { return p_.start; }
	std::array<double, 3> get_level_0_cell_length() const { return p_.level_0_cell_length; }
	std::array<double, 3> get_min(uint64_t cell) const {
		const auto c = get_center(cell), L = get_length(cell);
		return {{c[0] - L[0] / 2, c[1] - L[1] / 2, c[2] - L[2] / 2}};
	}
	std::array<double, 3> get_max(uint64_t cell) const {
		const auto c = get_center(cell), L = get_length(cell);
		return {{c[0] + L[0] / 2, c[1] + L[1] / 2, c[2] + L[2] / 2}};
	}

private:
	Parameters p_;
};

template <class T>
struct Iterator_Storage {  // dccrg.hpp:7279-7285
	typename std::vector<T>::const_iterator begin_, end_;
	typename std::vector<T>::const_iterator begin() const { return begin_; }
	typename std::vector<T>::const_iterator cbegin() const { return begin_; }
	typename std::vector<T>::const_iterator end() const { return end_; }
	typename std::vector<T>::const_iterator cend() const { return end_; }
};

// A device-resident SoA field of the library (one T per slot: local cells in
// slot order, then the copies of remote neighbors), the form the device
// sweeps read and write.  Handles are cheap values; the array itself moves
// on a structural change (refinement, balance_load), so data() asks the
// library each time.  Converts to the field id of the C ABI.
template <class T>
class Device_Field {
public:
	Device_Field() = default;
	Device_Field(dccrgx_grid* g, int id) : g_(g), id_(id) {}
	int id() const { return id_; }
	operator int() const { return id_; }
	// the device array (valid until the next structural change)
	T* data() const {
		void* p = nullptr;
		detail::check(dccrgx_field_device_ptr(g_, id_, &p));
		return static_cast<T*>(p);
	}
	// slots [slot0, slot0 + n) to / from the host
	void upload(const T* host, size_t n, size_t slot0 = 0) const {
		detail::check(dccrgx_field_upload(g_, id_, slot0, n, host));
	}
	void download(T* host, size_t n, size_t slot0 = 0) const {
		detail::check(dccrgx_field_download(g_, id_, slot0, n, host));
	}
	void set(const std::vector<T>& v, size_t slot0 = 0) const { upload(v.data(), v.size(), slot0); }
	std::vector<T> get(size_t n, size_t slot0 = 0) const {
		std::vector<T> v(n);
		if (n) download(v.data(), n, slot0);
		return v;
	}

private:
	dccrgx_grid* g_ = nullptr;
	int id_ = -1;
};

// dccrgx_poisson_solve's outcome (Poisson_Solve::solve, poisson_solve.hpp:251-522)
struct Poisson_Result {
	unsigned iterations = 0;
	double residual = 0;
};

template <class Cell_Data, class Geometry = No_Geometry, class Additional_Cell_Items = std::tuple<>,
          class Additional_Neighbor_Items = std::tuple<>>
class Dccrg;

template <class Cell_Data, class Geometry, class... Additional_Cell_Items, class... Additional_Neighbor_Items>
class Dccrg<Cell_Data, Geometry, std::tuple<Additional_Cell_Items...>, std::tuple<Additional_Neighbor_Items...>> {
	// a trivially copyable Cell_Data is mirrored byte for byte in a device
	// field; any other one (std::vector members, tests/variable_data_size) is
	// serialized over its get_mpi_datatype into a variable-size device field
	static constexpr bool serialized_ = !std::is_trivially_copyable<Cell_Data>::value;

public:
	using cell_data_type = Cell_Data;
	using geometry_type = Geometry;
	using neighbor_list_t = std::vector<std::pair<uint64_t, std::array<int, 3>>>;

	// Neighbors_Item / Cells_Item (7288-7402)
	struct Neighbors_Item : Additional_Neighbor_Items... {
		uint64_t id;
		Cell_Data* data;
		int x, y, z;
		template <class Grid, class Cell_Item>
		void update_caller(const Grid&, const Cell_Item&, const int&) {}
		template <class Grid, class Cell_Item, class A, class... B>
		void update_caller(const Grid& grid, const Cell_Item& cell, const int& hood, const A& a, const B&... b) {
			A::update(grid, cell, *this, hood, a);
			update_caller(grid, cell, hood, b...);
		}
	};
	struct Cells_Item : Additional_Cell_Items... {
		uint64_t id = error_cell;
		Cell_Data* data = nullptr;
		Iterator_Storage<Neighbors_Item> neighbors_of, neighbors_to, all_neighbors;
		friend bool operator<(const Cells_Item& a, const Cells_Item& b) { return a.id < b.id; }
		template <class Grid>
		void update_caller(const Grid&) {}
		template <class Grid, class A, class... B>
		void update_caller(const Grid& grid, const A& a, const B&... b) {
			A::update(grid, *this, a);
			update_caller(grid, b...);
		}
	};

	// public read-only members (235-279)
	const Grid_Topology& topology = topology_rw;
	const Mapping& mapping = mapping_rw;
	const Grid_Length& length = mapping_rw.length;
	const Geometry& geometry = geometry_rw;
	const std::vector<Cells_Item>& cells = cells_rw;
	const std::vector<Neighbors_Item>& neighbors = neighbors_rw;

	Dccrg() { geometry_rw.attach_parts(&mapping_rw.length, &topology_rw); }
	Dccrg(const Dccrg&) = delete;
	Dccrg& operator=(const Dccrg&) = delete;
	~Dccrg() {
		dump_cells("final");
		if (g_) dccrgx_destroy(g_);
		if (comm_ != MPI_COMM_NULL) {
			int fin = 0;
			MPI_Finalized(&fin);
			if (!fin) MPI_Comm_free(&comm_);
		}
	}

	// ---- setup (8120-8230), chainable ----------------------------------------
	Dccrg& set_initial_length(const std::array<uint64_t, 3>& l) {
		if (!mapping_rw.length.set(l)) throw std::invalid_argument("dccrg: grid length must be > 0");
		return *this;
	}
	Dccrg& set_maximum_refinement_level(const int l) {
		max_ref_ = l;
		return *this;
	}
	Dccrg& set_periodic(bool x, bool y, bool z) {
		topology_rw.set_periodicity(0, x);
		topology_rw.set_periodicity(1, y);
		topology_rw.set_periodicity(2, z);
		return *this;
	}
	Dccrg& set_neighborhood_length(unsigned n) {
		hood_ = n;
		return *this;
	}
	// 8223: the native partitioner is recursive coordinate bisection (Zoltan's
	// "RCB", the reference default); "NONE" keeps the partition; any other
	// Zoltan method name also partitions with RCB (Zoltan is not available)
	Dccrg& set_load_balancing_method(const std::string& m) {
		lb_method_ = m;
		if (g_) detail::check(dccrgx_set_load_balancing_method(g_, m == "NONE" ? "NONE" : "RCB"));
		return *this;
	}
	const std::string& get_load_balancing_method() const { return lb_method_; }  // 8228
	// set / get_send_single_cells (6658-6681): on, remote neighbor updates
	// send each cell's fixed-size payload as its own message (dccrgx.h)
	Dccrg& set_send_single_cells(const bool given) {
		send_single_cells_ = given;
		if (g_) detail::check(dccrgx_set_send_single_cells(g_, given ? 1 : 0));
		return *this;
	}
	bool get_send_single_cells() const { return send_single_cells_; }

	// initialize (472-552)
	Dccrg& initialize(const MPI_Comm& comm, const uint64_t /*sfc_caching_batches*/ = 1) {
		if (g_) throw std::invalid_argument("dccrg: already initialized");
		create(comm);
		const auto L = mapping_rw.length.get();
		detail::check(dccrgx_set_initial_length(g_, L.data()));
		detail::check(dccrgx_set_maximum_refinement_level(g_, max_ref_));
		detail::check(dccrgx_set_periodic(g_, topology_rw.is_periodic(0), topology_rw.is_periodic(1),
		                                  topology_rw.is_periodic(2)));
		detail::check(dccrgx_set_neighborhood_length(g_, hood_));
		detail::check(dccrgx_set_load_balancing_method(g_, lb_method_ == "NONE" ? "NONE" : "RCB"));
		detail::check(dccrgx_initialize(g_));
		add_payload_field();
		refresh();
		return *this;
	}

	Dccrg& set_geometry(const typename Geometry::Parameters& p) {  // 576
		if (!geometry_rw.set(p)) throw std::invalid_argument("dccrg: couldn't set geometry");
		refresh_items();
		return *this;
	}

	dccrgx_grid* native() const { return g_; }
	int get_rank() const { return rank_; }
	int get_comm_size() const { return size_; }
	unsigned int get_neighborhood_length() const { return hood_; }
	int get_maximum_refinement_level() const { return mapping_rw.get_maximum_refinement_level(); }
	int get_refinement_level(const uint64_t cell) const { return mapping_rw.get_refinement_level(cell); }  // 1050
	MPI_Comm get_communicator() const { return comm_; }
	// 4157-4190: the parent if it exists as a cell of the grid, else the cell
	// itself if it exists, else error_cell (existence as known to this rank:
	// its own and ghost leaves)
	uint64_t get_parent(const uint64_t cell) const {
		const int l = mapping_rw.get_refinement_level(cell);
		if (l < 0) return error_cell;
		const bool cell_exists = dccrgx_get_process(g_, cell) >= 0;
		if (l == 0) return cell_exists ? cell : error_cell;
		const uint64_t parent = mapping_rw.get_parent(cell);
		if (dccrgx_get_process(g_, parent) >= 0) return parent;
		return cell_exists ? cell : error_cell;
	}

	// 11275-11308: the smallest cell known to exist at the indices between the
	// two refinement levels (finest first); error_cell outside the grid
	uint64_t get_existing_cell(const Types<3>::indices_t& indices, const int minimum_refinement_level,
	                           const int maximum_refinement_level) const {
		const auto L = mapping_rw.length.get();
		const int R = mapping_rw.get_maximum_refinement_level();
		for (size_t d = 0; d < 3; d++)
			if (indices[d] >= L[d] * (uint64_t(1) << R)) return error_cell;
		for (int l = maximum_refinement_level; l >= minimum_refinement_level; l--) {
			const uint64_t c = mapping_rw.get_cell_from_indices(indices, l);
			if (c != error_cell && dccrgx_get_process(g_, c) >= 0) return c;
		}
		return error_cell;
	}

	// ---- queries ----------------------------------------------------------------
	// get_cells (651-739) with is_neighbor_type_match (2946-3053)
	std::vector<uint64_t> get_cells(const std::vector<int>& criteria = std::vector<int>(), const bool exact_match = false,
	                                const int neighborhood_id = default_neighborhood_id,
	                                const bool /*sorted*/ = false) const {
		std::vector<int32_t> c(criteria.begin(), criteria.end());
		return detail::fetch_u64([&](uint64_t* o, size_t cap, size_t* n) {
			return dccrgx_get_cells_by_criteria(g_, c.data(), c.size(), exact_match, neighborhood_id, o, cap, n);
		});
	}
	Cell_Data* operator[](const uint64_t cell) const {  // 756: local cells, remote copies, removed cells (764)
		if (balancing_) {  // cells arriving in the balance_load in progress (3855)
			const auto it = pending_.find(cell);
			if (it != pending_.end()) return const_cast<Cell_Data*>(&it->second);
		}
		int64_t s = -1;
		if (g_) dccrgx_get_slots(g_, &cell, 1, &s);
		if (s >= 0 && size_t(s) < host_.size()) return const_cast<Cell_Data*>(&host_[size_t(s)]);
		const auto rf = refined_.find(cell);  // refined_cell_data (762)
		if (rf != refined_.end()) return const_cast<Cell_Data*>(&rf->second);
		const auto it = removed_index_.find(cell);
		if (it != removed_index_.end()) return const_cast<Cell_Data*>(&removed_[it->second]);
		return nullptr;
	}
	std::array<double, 3> get_center(const uint64_t cell) const { return geometry_rw.get_center(cell); }  // 771

	// get_neighbors_of / _to (819 / 883): nullptr for a cell that is not local
	// or a neighborhood that does not exist; valid until the next structural change
	const neighbor_list_t* get_neighbors_of(const uint64_t cell,
	                                        const int neighborhood_id = default_neighborhood_id) const {
		return neighbor_list(cell, neighborhood_id, 0);
	}
	const neighbor_list_t* get_neighbors_to(const uint64_t cell,
	                                        const int neighborhood_id = default_neighborhood_id) const {
		return neighbor_list(cell, neighborhood_id, 1);
	}
	std::vector<std::pair<uint64_t, int>> get_face_neighbors_of(const uint64_t cell) const {  // 2806
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
	bool is_local(const uint64_t cell) const { return dccrgx_is_local(g_, cell) == 1; }  // 3270
	int get_process(const uint64_t cell) const { return dccrgx_get_process(g_, cell); }  // 5807
	bool is_neighbor_type_match(const uint64_t cell, const std::vector<int>& criteria, const bool exact_match,
	                            const int neighborhood_id) const {  // 2946
		const auto c = get_cells(criteria, exact_match, neighborhood_id);
		return std::binary_search(c.begin(), c.end(), cell);
	}

	// process boundaries (6050-6206)
	std::vector<uint64_t> get_local_cells_on_process_boundary(const int neighborhood_id = default_neighborhood_id,
	                                                          const bool sorted = false) const {
		return get_cells({has_remote_neighbor_of, has_remote_neighbor_to}, false, neighborhood_id, sorted);
	}
	std::vector<uint64_t> get_local_cells_not_on_process_boundary(const int neighborhood_id = default_neighborhood_id,
	                                                              const bool sorted = false) const {
		return get_cells({has_no_neighbor, has_local_neighbor_of, has_local_neighbor_to, has_local_neighbor_both}, true,
		                 neighborhood_id, sorted);
	}
	std::vector<uint64_t> get_remote_cells_on_process_boundary(const int neighborhood_id = default_neighborhood_id,
	                                                           const bool /*sorted*/ = false) const {
		if (neighborhood_id == default_neighborhood_id)
			return detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) {
				return dccrgx_get_cells(g_, DCCRGX_CELLS_REMOTE, o, c, n);
			});
		std::vector<uint64_t> r;
		for (const auto& kv : cells_to_receive(neighborhood_id))
			for (const auto& c : kv.second) r.push_back(c.first);
		std::sort(r.begin(), r.end());
		r.erase(std::unique(r.begin(), r.end()), r.end());
		return r;
	}
	// update counts (5382-5490); max uint64 for an unknown neighborhood
	uint64_t get_number_of_update_send_cells(const int neighborhood_id = default_neighborhood_id) const {
		return count_updates(neighborhood_id, false);
	}
	uint64_t get_number_of_update_receive_cells(const int neighborhood_id = default_neighborhood_id) const {
		return count_updates(neighborhood_id, true);
	}
	// cells_to_send / cells_to_receive (6900-6914): per process the ids in
	// ascending order with their message tags 1..n (8662-8748)
	const std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>& get_cells_to_send(
	    const int neighborhood_id = default_neighborhood_id) const {
		return cells_to_send_map(neighborhood_id);
	}
	const std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>& get_cells_to_receive(
	    const int neighborhood_id = default_neighborhood_id) const {
		return cells_to_receive(neighborhood_id);
	}

	// ---- iteration (7478-7602) ----------------------------------------------------
	const Iterator_Storage<Cells_Item>& inner_cells(const int neighborhood_id = default_neighborhood_id) const {
		return range(neighborhood_id, 0);
	}
	const Iterator_Storage<Cells_Item>& outer_cells(const int neighborhood_id = default_neighborhood_id) const {
		return range(neighborhood_id, 1);
	}
	const Iterator_Storage<Cells_Item>& local_cells(const int neighborhood_id = default_neighborhood_id) const {
		return range(neighborhood_id, 2);
	}
	const Iterator_Storage<Cells_Item>& remote_cells(const int neighborhood_id = default_neighborhood_id) const {
		return range(neighborhood_id, 3);
	}
	const Iterator_Storage<Cells_Item>& all_cells(const int neighborhood_id = default_neighborhood_id) const {
		return range(neighborhood_id, 4);
	}

	// ---- halo (966-1000, 5010-5367) -------------------------------------------------
	bool update_copies_of_remote_neighbors(const int neighborhood_id = default_neighborhood_id) {
		stage_up();
		if (dccrgx_update_copies_of_remote_neighbors_hood(g_, neighborhood_id) != DCCRGX_OK) return false;
		if (staging_) download_remote();
		return true;
	}
	bool start_remote_neighbor_copy_updates(const int neighborhood_id = default_neighborhood_id) {
		if (neighborhood_id != default_neighborhood_id) return update_copies_of_remote_neighbors(neighborhood_id);
		stage_up();
		return dccrgx_start_remote_neighbor_copy_updates(g_) == DCCRGX_OK;
	}
	bool start_remote_neighbor_copy_receives(const int neighborhood_id = default_neighborhood_id) {
		return start_remote_neighbor_copy_updates(neighborhood_id);
	}
	bool start_remote_neighbor_copy_sends(const int = default_neighborhood_id) { return true; }
	bool wait_remote_neighbor_copy_update_receives(const int = default_neighborhood_id) {
		if (dccrgx_wait_remote_neighbor_copy_update_receives(g_) != DCCRGX_OK) return false;
		if (staging_) download_remote();
		return true;
	}
	// The halo calls stage the host Cell_Data (every local payload up, the
	// received copies down; default on, the reference's semantics).  A
	// program whose per-cell state lives in device fields turns it off: the
	// halo then moves only the transferred device fields, with no host copy.
	Dccrg& set_host_staging(const bool on) {
		staging_ = on;
		if (g_ && payload_ >= 0) detail::check(dccrgx_set_field_transfer(g_, payload_, on ? 1 : 0));
		return *this;
	}
	bool get_host_staging() const { return staging_; }
	bool wait_remote_neighbor_copy_update_sends(const int = default_neighborhood_id) {
		return dccrgx_wait_remote_neighbor_copy_update_sends(g_) == DCCRGX_OK;
	}
	bool wait_remote_neighbor_copy_updates(const int neighborhood_id = default_neighborhood_id) {
		return wait_remote_neighbor_copy_update_receives(neighborhood_id) &&
		       wait_remote_neighbor_copy_update_sends(neighborhood_id);
	}

	// the default neighborhood and its opposite (6738 / 6748, initialize_neighborhoods
	// 7895-7954): length 0 = the six face offsets, otherwise the cube without
	// (0, 0, 0), z outermost, x innermost
	const std::vector<Types<3>::neighborhood_item_t>& get_neighborhood_of() const {
		default_hoods();
		return hood_of_;
	}
	const std::vector<Types<3>::neighborhood_item_t>& get_neighborhood_to() const {
		default_hoods();
		return hood_to_;
	}
	// the user neighborhoods (6755-6775)
	const std::unordered_map<int, std::vector<Types<3>::neighborhood_item_t>>& get_user_hood_of() const {
		return user_hood_of_;
	}
	const std::unordered_map<int, std::vector<Types<3>::neighborhood_item_t>>& get_user_hood_to() const {
		return user_hood_to_;
	}
	// 4339-4680: the neighbors of a cell for any neighborhood, in item order
	// (a finer box as its eight cells); throws for a cell this process does
	// not know.  For a local cell the items must stay within the process's
	// ghost region (max(neighborhood length, 1) level-0 cells); for a remote
	// cell the list may be incomplete, as the reference documents (4327).
	neighbor_list_t find_neighbors_of(const uint64_t cell,
	                                  const std::vector<Types<3>::neighborhood_item_t>& neighborhood) const {
		std::vector<int32_t> items;
		for (const auto& it : neighborhood) items.insert(items.end(), it.begin(), it.end());
		size_t n = 0;
		int rc = dccrgx_find_neighbors_of(g_, cell, items.data(), neighborhood.size(), nullptr, nullptr, 0, &n);
		if (rc == DCCRGX_ENOTFOUND) throw std::runtime_error("dccrg: invalid cell: " + std::to_string(cell));
		if (rc != DCCRGX_ERANGE) detail::check(rc);
		std::vector<uint64_t> ids(n);
		std::vector<int32_t> off(3 * n);
		detail::check(dccrgx_find_neighbors_of(g_, cell, items.data(), neighborhood.size(), ids.data(), off.data(), n, &n));
		neighbor_list_t r;
		r.reserve(n);
		for (size_t i = 0; i < n; i++) r.push_back({ids[i], {{off[3 * i], off[3 * i + 1], off[3 * i + 2]}}});
		return r;
	}
	// 7107: the face-neighbor cache, per leaf the cell just across each face
	// at the min corner (-x, +x, -y, +y, -z, +z; error_cell where none).  The
	// reference holds every leaf of the grid; here the leaves this process can
	// resolve: all local ones and the ghosts within its ghost region.  Valid
	// until the next structural change.
	const std::map<uint64_t, std::array<uint64_t, 6>>& get_neighbors_() const {
		if (!face_cache_valid_) {
			size_t n = 0;
			int rc = dccrgx_get_face_cache(g_, nullptr, nullptr, 0, &n);
			if (rc != DCCRGX_ERANGE) detail::check(rc);
			std::vector<uint64_t> ids(n), nb(6 * n);
			detail::check(dccrgx_get_face_cache(g_, ids.data(), nb.data(), n, &n));
			face_cache_.clear();
			for (size_t i = 0; i < n; i++)
				face_cache_[ids[i]] = {{nb[6 * i], nb[6 * i + 1], nb[6 * i + 2], nb[6 * i + 3], nb[6 * i + 4], nb[6 * i + 5]}};
			face_cache_valid_ = true;
		}
		return face_cache_;
	}

	// ---- user neighborhoods (6383-6603) -----------------------------------------------
	bool add_neighborhood(const int neighborhood_id, const std::vector<std::array<int, 3>>& items) {
		std::vector<int32_t> o;
		for (const auto& it : items) o.insert(o.end(), it.begin(), it.end());
		const bool ok = dccrgx_add_neighborhood(g_, neighborhood_id, o.data(), items.size()) == DCCRGX_OK;
		if (ok) {
			user_hood_of_[neighborhood_id] = items;
			auto& to = user_hood_to_[neighborhood_id];
			to.clear();
			for (const auto& it : items) to.push_back({{-it[0], -it[1], -it[2]}});
			refresh_items();
		}
		return ok;
	}
	void remove_neighborhood(const int neighborhood_id) {
		detail::check(dccrgx_remove_neighborhood(g_, neighborhood_id));
		user_hood_of_.erase(neighborhood_id);
		user_hood_to_.erase(neighborhood_id);
		refresh_items();
	}

	// ---- refinement (2434, 3461) ------------------------------------------------------
	bool refine_completely(const uint64_t cell) { return dccrgx_refine_completely(g_, cell) == DCCRGX_OK; }
	bool unrefine_completely(const uint64_t cell) { return dccrgx_unrefine_completely(g_, cell) == DCCRGX_OK; }  // 2560
	bool dont_unrefine(const uint64_t cell) { return dccrgx_dont_unrefine(g_, cell) == DCCRGX_OK; }  // 2679
	bool dont_refine(const uint64_t cell) { return dccrgx_dont_refine(g_, cell) == DCCRGX_OK; }  // 2744
	std::vector<uint64_t> stop_refining(const bool sorted = false) {
		upload_local();
		size_t n = 0;
		detail::check(dccrgx_stop_refining(g_, nullptr, 0, &n));
		std::unordered_map<uint64_t, Cell_Data> gone;
		// the refined local parents' data before the change (the parents of
		// the new cells), for refined_cell_data below
		std::unordered_map<uint64_t, Cell_Data> before;
		if constexpr (!serialized_) {
			const auto created =
			    detail::fetch_u64([&](uint64_t* o, size_t c, size_t* k) { return dccrgx_get_new_cells(g_, o, c, k); });
			std::unordered_set<uint64_t> parents;
			for (const uint64_t c : created) parents.insert(mapping_rw.get_parent(c));
			for (size_t s = 0; s < n_local_ && s < slot_ids_.size() && s < host_.size() && !parents.empty(); s++)
				if (parents.count(slot_ids_[s])) before.emplace(slot_ids_[s], host_[s]);
		}
		refresh(&gone);
		if constexpr (serialized_) before = gone;
		// removed cells' payloads on the parent's process (unrefined_cell_data 7250)
		removed_ids_ = detail::fetch_u64([&](uint64_t* o, size_t c, size_t* k) { return dccrgx_get_removed_cells(g_, o, c, k); });
		removed_.clear();
		removed_.resize(removed_ids_.size());
		removed_index_.clear();
		for (size_t i = 0; i < removed_ids_.size(); i++) removed_index_[removed_ids_[i]] = i;
		if (serialized_) {
			// the removed children that were local here keep their objects
			for (size_t i = 0; i < removed_ids_.size(); i++) {
				auto it = gone.find(removed_ids_[i]);
				if (it != gone.end()) removed_[i] = std::move(it->second);
			}
		} else if (!removed_.empty()) {
			removed_download(removed_.data(), removed_.size() * sizeof(Cell_Data));
		}
		auto out = detail::fetch_u64([&](uint64_t* o, size_t c, size_t* k) { return dccrgx_get_new_cells(g_, o, c, k); });
		// refined_cell_data (10215-10219): the refined local parents' data
		// stay reachable through operator[] until the next structural change
		refined_.clear();
		for (const uint64_t c : out) {
			const uint64_t p = mapping_rw.get_parent(c);
			if (refined_.count(p)) continue;
			auto it = before.find(p);
			if (it != before.end()) refined_.emplace(p, it->second);
		}
		if (sorted) std::sort(out.begin(), out.end());
		return out;
	}
	// 5504
	Dccrg& clear_refined_unrefined_data() {
		clear_removed();
		return *this;
	}
	// 3497: cells removed by the last stop_refining whose parent is local
	std::vector<uint64_t> get_removed_cells(const bool sorted = false) const {
		std::vector<uint64_t> r = removed_ids_;
		if (sorted) std::sort(r.begin(), r.end());
		return r;
	}

	// ---- partition (1024, 5832-5909) ---------------------------------------------------
	bool pin(const uint64_t cell) { return pin(cell, rank_); }
	bool pin(const uint64_t cell, const int process) { return dccrgx_pin(g_, cell, process) == DCCRGX_OK; }
	bool unpin(const uint64_t cell) { return dccrgx_unpin(g_, cell) == DCCRGX_OK; }
	// 6017: every pin is dropped (call on every process)
	Dccrg& unpin_all_cells() {
		detail::check(dccrgx_unpin_all_cells(g_));
		return *this;
	}
	// 5952: unpin every local cell
	bool unpin_local_cells() {
		bool ok = true;
		for (size_t s = 0; s < n_local_ && s < slot_ids_.size(); s++) ok = unpin(slot_ids_[s]) && ok;
		return ok;
	}
	Dccrg& balance_load(const bool use_zoltan = true) {
		initialize_balance_load(use_zoltan);
		continue_balance_load();
		finish_balance_load();
		return *this;
	}
	// split form (3746, 3899, 3942): the payloads move in continue; in
	// between, get_cells_to_receive() lists the arriving cells and
	// operator[] gives their (default-constructed) data, which a program
	// with variable-size data sizes before continue (variable_data_size.cpp:83-95)
	void initialize_balance_load(const bool use_zoltan) {
		clear_removed();
		upload_local();
		detail::check(dccrgx_initialize_balance_load(g_, use_zoltan ? 1 : 0, nullptr, nullptr, 0));
		begin_balancing();
	}
	void continue_balance_load() { detail::check(dccrgx_continue_balance_load(g_)); }
	void finish_balance_load() {
		detail::check(dccrgx_finish_balance_load(g_));
		end_balancing();
	}
	// 6210 / 6244
	bool set_cell_weight(const uint64_t cell, const double weight) {
		return dccrgx_set_cell_weight(g_, cell, weight) == DCCRGX_OK;
	}
	double get_cell_weight(const uint64_t cell) const { return dccrgx_get_cell_weight(g_, cell); }
	// a partitioner's export list: local cells and their new processes
	Dccrg& balance_load(const std::vector<uint64_t>& cells_out, const std::vector<int>& processes) {
		clear_removed();
		upload_local();
		std::vector<int32_t> p(processes.begin(), processes.end());
		detail::check(dccrgx_initialize_balance_load(g_, 0, cells_out.data(), p.data(), cells_out.size()));
		begin_balancing();
		continue_balance_load();
		finish_balance_load();
		return *this;
	}
	// allocate_copies_of_remote_neighbors (1054-1074): the copies exist (default
	// constructed) after every structural change
	void allocate_copies_of_remote_neighbors(const int = default_neighborhood_id) {}

	// ---- grid files (1089, 1742, 1795, 2112, 2380) --------------------------------------
	// raw-byte header form
	bool save_grid_data(const std::string& name, const uint64_t offset, const void* header = nullptr,
	                    const size_t header_bytes = 0) {
		sync_window();  // the bytes get_mpi_datatype describes now
		upload_local();
		const std::vector<char> geo = geometry_rw.file_block();  // Geometry::write's bytes (empty: Cartesian)
		if (dccrgx_set_geometry_block(g_, geo.empty() ? nullptr : geo.data(), geo.size()) != DCCRGX_OK) return false;
		return dccrgx_save_grid_data(g_, name.c_str(), offset, header, header_bytes) == DCCRGX_OK;
	}
	// the reference's form: the header is (address, count, datatype), written
	// by process 0 as MPI packs it (native layout, no padding)
	bool save_grid_data(const std::string& name, const MPI_Offset offset, std::tuple<void*, int, MPI_Datatype> header) {
		const std::vector<char> h = pack_header(header);
		return save_grid_data(name, uint64_t(offset), h.data(), h.size());
	}
	// replaces initialize(): every setting comes from the file
	bool load_grid_data(const std::string& name, const uint64_t offset, const MPI_Comm& comm,
	                    const size_t header_bytes = 0) {
		if (!start_loading(name, offset, comm, header_bytes)) return false;
		if (!continue_loading_grid_data()) return false;
		return finish_loading_grid_data();
	}
	bool load_grid_data(const std::string& name, const MPI_Offset offset, std::tuple<void*, int, MPI_Datatype> header,
	                    const MPI_Comm& comm, const char* const load_balancing_method = "RCB",
	                    const uint64_t = 1, const uint64_t = ~uint64_t(0)) {
		if (!start_loading_grid_data(name, offset, header, comm, load_balancing_method)) return false;
		if (!continue_loading_grid_data()) return false;
		return finish_loading_grid_data();
	}
	// start_loading_grid_data (1795): the grid, its cells and the header; the
	// cells' data come with continue_loading_grid_data
	bool start_loading_grid_data(const std::string& name, const MPI_Offset offset,
	                             std::tuple<void*, int, MPI_Datatype> header, const MPI_Comm& comm,
	                             const char* const load_balancing_method = "RCB", const uint64_t = 1,
	                             const uint64_t = ~uint64_t(0)) {
		const size_t hb = pack_header(header).size();
		if (!start_loading(name, uint64_t(offset), comm, hb)) return false;
		if (load_balancing_method) set_load_balancing_method(load_balancing_method);
		if (hb) {
			// the header as process 0 wrote it, into the caller's object
			std::vector<char> h(hb);
			std::FILE* f = std::fopen(name.c_str(), "rb");
			const bool ok = f && std::fseek(f, long(offset), SEEK_SET) == 0 && std::fread(h.data(), 1, hb, f) == hb;
			if (f) std::fclose(f);
			if (!ok) return false;
			MPI_Datatype t = std::get<2>(header);
			int pos = 0;
			MPI_Unpack(h.data(), int(hb), &pos, std::get<0>(header), std::get<1>(header), t, comm_);
		}
		return true;
	}
	// continue_loading_grid_data (2112): for every local cell the bytes its
	// get_mpi_datatype describes now (receiving, from process -1), read from
	// where the previous call stopped
	bool continue_loading_grid_data() {
		const size_t nl = n_local_;
		if constexpr (serialized_) {
			std::vector<uint64_t> sizes(nl);
			for (size_t s = 0; s < nl; s++) {
				auto dt = detail::cell_datatype(host_[s], slot_ids_[s], -1, rank_, true, -1, 0);
				int sz = 0;
				MPI_Type_size(std::get<2>(dt), &sz);
				sizes[s] = uint64_t(std::get<1>(dt)) * uint64_t(sz);
				if (!detail::is_named_datatype(std::get<2>(dt))) {
					MPI_Datatype t = std::get<2>(dt);
					MPI_Type_free(&t);
				}
			}
			if (dccrgx_continue_loading_grid_data(g_, payload_, sizes.data()) != DCCRGX_OK) return false;
			for (size_t s = 0; s < nl; s++) {
				uint64_t sz = 0;
				detail::check(dccrgx_variable_field_sizes(g_, payload_, s, 1, &sz));
				std::vector<char> bytes(size_t(sz) + 1);
				size_t got = 0;
				detail::check(dccrgx_variable_field_download(g_, payload_, s, 1, bytes.data(), bytes.size(), &got));
				detail::unpack_cell(host_[s], slot_ids_[s], -1, rank_, -1, comm_, bytes.data(), got);
			}
			return true;
		}
		sync_window();
		if (dccrgx_continue_loading_grid_data(g_, payload_, nullptr) != DCCRGX_OK) return false;
		if (nl) {
			std::vector<Cell_Data> tmp(nl);
			detail::check(dccrgx_field_download(g_, payload_, 0, nl, tmp.data()));
			for (size_t s = 0; s < nl; s++)
				std::memcpy(reinterpret_cast<char*>(&host_[s]) + window_.first,
				            reinterpret_cast<const char*>(&tmp[s]) + window_.first, window_.second);
		}
		return true;
	}
	// finish_loading_grid_data (2380): the device payloads take the loaded objects
	bool finish_loading_grid_data() {
		if (dccrgx_finish_loading_grid_data(g_) != DCCRGX_OK) return false;
		upload_local();
		return true;
	}

	// ---- device SoA fields and the device sweeps -------------------------------------------
	// The host-staged Cell_Data path above moves every local payload to the
	// device and back at each halo; a program whose per-cell loops run on the
	// GPU keeps its state in device fields instead and calls the sweeps below
	// (no native() or raw C calls needed).  A transferred field takes part in
	// every halo of the default neighborhood.
	template <class T>
	Device_Field<T> add_field(const std::string& name, bool transfer) {
		int id = -1;
		detail::check(dccrgx_add_field(g_, name.c_str(), sizeof(T), transfer ? 1 : 0, &id));
		return Device_Field<T>(g_, id);
	}
	int payload_field() const { return payload_; }
	// host Cell_Data <-> device payload field
	void upload() { upload_all(); }
	void download() { download_all(); }
	// slot -> cell id of every slot (local cells first, in slot order)
	std::vector<uint64_t> get_slot_ids() const {
		return detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) { return dccrgx_get_slot_ids(g_, o, c, n); });
	}
	size_t get_number_of_local_slots() const { return n_local_; }
	// the compute stream's work done
	void synchronize() const { detail::check(dccrgx_synchronize(g_)); }

	// game of life over cell.neighbors_of (examples/game_of_life.cpp:54-79):
	// `region` DCCRGX_REGION_ALL / _INNER / _OUTER; commit makes the new
	// states current
	void gol_step(const Device_Field<uint32_t>& state, const int region = DCCRGX_REGION_ALL) {
		detail::check(dccrgx_gol_step(g_, state.id(), region));
	}
	void gol_commit(const Device_Field<uint32_t>& state) { detail::check(dccrgx_gol_commit(g_, state.id())); }
	// one turn of the refined game (tests/game_of_life/solve.hpp:37-170);
	// list: 8 x uint64 per cell (Cell_Data::data[1..8])
	void get_live_neighbors(const Device_Field<uint32_t>& state, const Device_Field<std::array<uint64_t, 8>>& list) {
		detail::check(dccrgx_get_live_neighbors(g_, state.id(), list.id()));
	}

	// advection (tests/advection): fields density, vx, vy, vz, lx, ly, lz
	using Advection_Fields = std::array<Device_Field<double>, 7>;
	void advection_initialize(const Advection_Fields& f) {  // initialize.hpp:36-82
		const auto id = ids(f);
		detail::check(dccrgx_advection_initialize(g_, id.data()));
	}
	double advection_max_time_step(const Advection_Fields& f) {  // solve.hpp:289-333, MIN over processes
		const auto id = ids(f);
		double v = 0;
		detail::check(dccrgx_advection_max_time_step(g_, id.data(), &v));
		detail::check(dccrgx_allreduce_f64(g_, &v, 1, 1));
		return v;
	}
	// the same into device memory, stream-ordered (no host round trip over RCCL)
	void advection_max_time_step(const Advection_Fields& f, double* device_out) {
		const auto id = ids(f);
		detail::check(dccrgx_advection_max_time_step_device(g_, id.data(), device_out));
	}
	void advection_step(const Advection_Fields& f, const double dt, const int region = DCCRGX_REGION_ALL) {
		const auto id = ids(f);  // calculate_fluxes + apply_fluxes (solve.hpp:44-279)
		detail::check(dccrgx_advection_step(g_, id.data(), dt, region));
	}
	void advection_commit(const Device_Field<double>& density) {
		detail::check(dccrgx_advection_commit(g_, density.id()));
	}
	// check_for_adaptation + adapt_grid (adapter.hpp:47-309); returns the
	// accepted (refines, dont_unrefines, unrefines) and (created, removed)
	std::array<uint64_t, 3> advection_check_adaptation(const Device_Field<double>& density, const double diff_increase,
	                                                   const double diff_threshold = 0.25,
	                                                   const double unrefine_sensitivity = 0.5) {
		std::array<uint64_t, 3> c{{0, 0, 0}};
		detail::check(dccrgx_advection_check_adaptation(g_, density.id(), diff_increase, diff_threshold,
		                                                unrefine_sensitivity, c.data()));
		return c;
	}
	std::array<uint64_t, 2> advection_adapt(const Advection_Fields& f) {
		const auto id = ids(f);
		std::array<uint64_t, 2> out{{0, 0}};
		detail::check(dccrgx_advection_adapt(g_, id.data(), out.data()));
		after_device_change();
		return out;
	}

	// Poisson (tests/poisson/poisson_solve.hpp): cache_system_info (827-971)
	// for the given cells, then solve (251-522) or solve_failsafe (531-634)
	void poisson_cache(const Device_Field<double>& rhs, const Device_Field<double>& solution,
	                   const std::vector<uint64_t>& solve_cells, const std::vector<uint64_t>& skip_cells = {}) {
		detail::check(dccrgx_poisson_cache(g_, rhs.id(), solution.id(), solve_cells.data(), solve_cells.size(),
		                                   skip_cells.data(), skip_cells.size()));
	}
	Poisson_Result poisson_solve(const unsigned max_iterations = 1000, const unsigned min_iterations = 0,
	                             const double stop_residual = 1e-15, const double p_of_norm = 2,
	                             const double stop_after_residual_increase = 10, const bool failsafe = false) {
		Poisson_Result r;
		detail::check(dccrgx_poisson_solve(g_, max_iterations, min_iterations, stop_residual, p_of_norm,
		                                   stop_after_residual_increase, failsafe ? 1 : 0, &r.iterations, &r.residual));
		return r;
	}

private:
	void stage_up() {
		if (!staging_) return;
		dump_initial();
		sync_window();
		upload_local();
	}
	static std::array<int, 7> ids(const std::array<Device_Field<double>, 7>& f) {
		std::array<int, 7> r;
		for (size_t k = 0; k < 7; k++) r[k] = f[k].id();
		return r;
	}
	// the mesh changed under a device call (adaptation): the host side follows
	void after_device_change() {
		clear_removed();
		refresh();
	}
	// DCCRGX_DUMP_CELLS=<path>: every rank writes its local cells (uint64 id +
	// Cell_Data bytes, ascending id) to <path>.initial.<rank> at the first
	// remote neighbor update and to <path>.final.<rank> when the grid is
	// destroyed (verification of unmodified reference programs,
	// tests/test_gpu_facade.py)
	void dump_cells(const char* when) const {
		const char* base = std::getenv("DCCRGX_DUMP_CELLS");
		if (!base || !g_ || serialized_) return;
		const std::string path = std::string(base) + "." + when + "." + std::to_string(rank_);
		std::vector<std::pair<uint64_t, size_t>> c;
		for (size_t s = 0; s < n_local_ && s < slot_ids_.size(); s++) c.push_back({slot_ids_[s], s});
		std::sort(c.begin(), c.end());
		if (FILE* f = std::fopen(path.c_str(), "wb")) {
			for (const auto& e : c) {
				std::fwrite(&e.first, 8, 1, f);
				std::fwrite(&host_[e.second], sizeof(Cell_Data), 1, f);
			}
			std::fclose(f);
		}
	}

	std::vector<char> pack_header(std::tuple<void*, int, MPI_Datatype> header) const {
		std::vector<char> out;
		MPI_Datatype t = std::get<2>(header);
		int sz = 0;
		MPI_Type_size(t, &sz);
		const size_t bytes = size_t(std::get<1>(header)) * size_t(sz);
		if (!bytes) return out;
		int bound = 0;
		MPI_Pack_size(std::get<1>(header), t, comm_, &bound);
		out.resize(size_t(bound));
		int pos = 0;
		MPI_Pack(std::get<0>(header), std::get<1>(header), t, out.data(), bound, &pos, comm_);
		out.resize(size_t(pos));
		return out;
	}
	bool start_loading(const std::string& name, const uint64_t offset, const MPI_Comm& comm, const size_t header_bytes) {
		if (g_) throw std::invalid_argument("dccrg: already initialized");
		create(comm);
		add_payload_field();
		if (dccrgx_start_loading_grid_data(g_, name.c_str(), offset, header_bytes) != DCCRGX_OK) return false;
		int R = 0;
		detail::check(dccrgx_get_maximum_refinement_level(g_, &R));
		max_ref_ = R;
		// the neighborhood length stored in the file: the
		// default neighborhood's offsets follow it
		unsigned L = 0;
		detail::check(dccrgx_get_neighborhood_length(g_, &L));
		hood_ = L;
		hood_set_ = ~0u;
		{
			int per[3] = {0, 0, 0};
			detail::check(dccrgx_get_periodic(g_, per));
			for (size_t d = 0; d < 3; d++) topology_rw.set_periodicity(d, per[d] != 0);
			uint64_t len[3] = {1, 1, 1};
			detail::check(dccrgx_get_initial_length(g_, len));
			mapping_rw.length.set({{len[0], len[1], len[2]}});
		}
		geometry_rw.sync_from_library();
		{
			// Geometry::read: the file's geometry block (none for a Cartesian file)
			size_t n = 0;
			detail::check(dccrgx_get_geometry_block(g_, nullptr, 0, &n));
			std::vector<char> geo(n);
			if (n) detail::check(dccrgx_get_geometry_block(g_, geo.data(), n, &n));
			if (!geometry_rw.from_file_block(geo)) return false;
		}
		refresh();
		return true;
	}
	void create(const MPI_Comm& comm) {
		MPI_Comm_dup(comm, &comm_);
		MPI_Comm_rank(comm_, &rank_);
		MPI_Comm_size(comm_, &size_);
		MPI_Comm node;
		MPI_Comm_split_type(comm_, MPI_COMM_TYPE_SHARED, rank_, MPI_INFO_NULL, &node);
		int lrank = 0, lsize = 1;
		MPI_Comm_rank(node, &lrank);
		MPI_Comm_size(node, &lsize);
		MPI_Comm_free(&node);
		int ndev = 1;
		detail::check(dccrgx_device_count(&ndev));
		if (ndev < 1) throw std::runtime_error("dccrg: no GPU visible");
		const int device = lrank % ndev;
		// processes sharing a GPU split the library's device-memory cache
		if (lsize > ndev && !std::getenv("DCCRGX_POOL_MAX_MB")) {
			const int per_dev = (lsize + ndev - 1) / ndev;
			setenv("DCCRGX_POOL_MAX_MB", std::to_string(16384 / per_dev).c_str(), 0);
		}
		const char* env = std::getenv("DCCRGX_TRANSPORT");
		const bool host = env && std::string(env) == "host";
		if (size_ == 1) {
			detail::check(dccrgx_create(0, 1, device, nullptr, &g_));
		} else if (!host && lsize <= ndev) {
			std::array<char, 128> id{};
			if (rank_ == 0) detail::check(dccrgx_get_unique_id(id.data()));
			MPI_Bcast(id.data(), 128, MPI_BYTE, 0, comm_);
			detail::check(dccrgx_create(rank_, size_, device, id.data(), &g_));
		} else {
			detail::check(dccrgx_create_with_exchange(rank_, size_, device, &detail::mpi_exchange, &comm_, &g_));
		}
		mapping_rw.attach(g_);
		if (send_single_cells_) detail::check(dccrgx_set_send_single_cells(g_, 1));
		geometry_rw.attach(g_);
		geometry_rw.set(geometry_rw.get_params_or_default());
	}
	void add_payload_field() {
		if constexpr (serialized_) {
			detail::check(dccrgx_add_variable_field(g_, "Cell_Data", staging_ ? 1 : 0, &payload_));
			return;
		}
		detail::check(dccrgx_add_field(g_, "Cell_Data", sizeof(Cell_Data), staging_ ? 1 : 0, &payload_));
		const auto w = detail::datatype_window<Cell_Data>();
		detail::check(dccrgx_set_field_window(g_, payload_, w.first, w.second));
		window_ = w;
	}
	// the reference asks get_mpi_datatype at every transfer, so the bytes a
	// halo moves may change between calls (tests/advection/cell.hpp:47-55,
	// Cell::transfer_all_data): re-read the window before each exchange
	void sync_window() {
		if constexpr (!serialized_) {
			const auto w = detail::datatype_window<Cell_Data>();
			if (w != window_) {
				detail::check(dccrgx_set_field_window(g_, payload_, w.first, w.second));
				window_ = w;
			}
		}
	}

	size_t n_local() const {
		size_t ni = 0, no = 0;
		detail::check(dccrgx_get_counts(g_, &ni, &no, nullptr, nullptr));
		return ni + no;
	}
	void clear_removed() {
		refined_.clear();
		removed_ids_.clear();
		removed_.clear();
		removed_index_.clear();
	}
	void dump_initial() {
		if (!dumped_initial_) {
			dumped_initial_ = true;
			dump_cells("initial");
		}
	}
	// serialized Cell_Data: slots [s0, s0 + n) packed into the device field
	void pack_range(size_t s0, size_t n) {
		std::vector<char> bytes;
		std::vector<uint64_t> sizes(n);
		for (size_t i = 0; i < n; i++) {
			const size_t at = bytes.size();
			detail::pack_cell(host_[s0 + i], slot_ids_[s0 + i], rank_, rank_, default_neighborhood_id, comm_, bytes);
			sizes[i] = bytes.size() - at;
		}
		if (!n) return;
		detail::check(dccrgx_variable_field_resize(g_, payload_, s0, n, sizes.data()));
		detail::check(dccrgx_variable_field_upload(g_, payload_, s0, n, bytes.data(), bytes.size()));
	}
	// ... and back (receiving side: the objects' own datatypes decide the layout)
	void unpack_slot(size_t s, int sender) {
		uint64_t sz = 0;
		detail::check(dccrgx_variable_field_sizes(g_, payload_, s, 1, &sz));
		std::vector<char> bytes(size_t(sz) + 1);
		size_t got = 0;
		detail::check(dccrgx_variable_field_download(g_, payload_, s, 1, bytes.data(), bytes.size(), &got));
		detail::unpack_cell(host_[s], slot_ids_[s], sender, rank_, default_neighborhood_id, comm_, bytes.data(), got);
	}
	void upload_local() {
		const size_t nl = std::min(n_local_, host_.size());
		if constexpr (serialized_) {
			pack_range(0, nl);
			return;
		}
		if (nl) detail::check(dccrgx_field_upload(g_, payload_, 0, nl, host_.data()));
	}
	void upload_all() {
		if constexpr (serialized_) {
			pack_range(0, host_.size());
			return;
		}
		if (!host_.empty()) detail::check(dccrgx_field_upload(g_, payload_, 0, host_.size(), host_.data()));
	}
	void download_all() {
		if constexpr (serialized_) {
			for (size_t s = 0; s < host_.size(); s++) unpack_slot(s, s < n_local_ ? rank_ : dccrgx_get_process(g_, slot_ids_[s]));
			return;
		}
		if (!host_.empty()) detail::check(dccrgx_field_download(g_, payload_, 0, host_.size(), host_.data()));
	}
	// received bytes into the host copies of remote neighbors
	void download_remote() {
		const size_t nr = host_.size() - n_local_;
		if (!nr) return;
		if constexpr (serialized_) {
			size_t nrecv = 0;
			detail::check(dccrgx_get_counts(g_, nullptr, nullptr, &nrecv, nullptr));
			for (size_t s = n_local_; s < n_local_ + nrecv; s++) unpack_slot(s, dccrgx_get_process(g_, slot_ids_[s]));
			return;
		}
		std::vector<Cell_Data> tmp(nr);
		detail::check(dccrgx_field_download(g_, payload_, n_local_, nr, tmp.data()));
		for (size_t i = 0; i < nr; i++)
			std::memcpy(reinterpret_cast<char*>(&host_[n_local_ + i]) + window_.first,
			            reinterpret_cast<const char*>(&tmp[i]) + window_.first, window_.second);
	}

	// after a structural change: slots, host payloads, items, caches
	void refresh(std::unordered_map<uint64_t, Cell_Data>* gone = nullptr) {
		size_t ns = 0;
		detail::check(dccrgx_get_counts(g_, nullptr, nullptr, nullptr, &ns));
		const size_t old_nl = n_local_;
		n_local_ = n_local();
		std::vector<uint64_t> old_ids = std::move(slot_ids_);
		slot_ids_ = detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) { return dccrgx_get_slot_ids(g_, o, c, n); });
		if constexpr (serialized_) {
			// the host objects are the data: a local cell keeps its object,
			// arrivals take the objects sized during the balance, new cells and
			// every remote copy start default-constructed (the reference clears
			// remote_neighbors at a balance and at a refinement, 3807, 10124)
			std::unordered_map<uint64_t, Cell_Data> old;
			for (size_t s = 0; s < old_ids.size() && s < host_.size() && s < old_nl; s++)
				old.emplace(old_ids[s], std::move(host_[s]));
			host_.clear();
			host_.resize(ns);
			arrived_.clear();
			for (size_t s = 0; s < ns; s++) {
				const uint64_t id = slot_ids_[s];
				auto it = old.find(id);
				if (it != old.end() && s < n_local_) {
					host_[s] = std::move(it->second);
					old.erase(it);
					continue;
				}
				auto pt = pending_.find(id);
				if (pt != pending_.end() && s < n_local_) {
					host_[s] = std::move(pt->second);
					arrived_.push_back(s);
					continue;
				}
				if (s < n_local_) arrived_.push_back(s);
			}
			if (gone) *gone = std::move(old);
		} else {
			(void)old_nl;
			(void)gone;
			host_.assign(ns, Cell_Data{});
			download_all();
		}
		refresh_items();
	}

	// initialize_balance_load done: the migration lists and the arriving cells' objects
	void begin_balancing() {
		balancing_ = true;
		pending_.clear();
		bal_send_.clear();
		bal_recv_.clear();
		for (int p = 0; p < size_; p++) {
			if (p == rank_) continue;
			for (int in = 0; in < 2; in++) {
				const auto v = detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) {
					return dccrgx_get_migration_cells(g_, p, in, o, c, n);
				});
				if (v.empty()) continue;
				auto& dst = (in ? bal_recv_ : bal_send_)[p];
				for (size_t i = 0; i < v.size(); i++) {
					dst.push_back({v[i], int(i + 1)});
					if (in) pending_[v[i]];
				}
			}
		}
	}
	void end_balancing() {
		balancing_ = false;
		refresh();
		pending_.clear();
		bal_send_.clear();
		bal_recv_.clear();
		if constexpr (serialized_) {
			// the arrived cells' bytes into their objects (sized by the program
			// between initialize_ and continue_balance_load, as in the reference)
			for (size_t s : arrived_) unpack_slot(s, dccrgx_get_process(g_, slot_ids_[s]));
		}
		arrived_.clear();
	}
	void removed_download(Cell_Data* out, size_t bytes) {
		if constexpr (!serialized_) detail::check(dccrgx_removed_field_download(g_, payload_, out, bytes));
	}

	void default_hoods() const {
		if (hood_set_ == hood_) return;
		hood_of_.clear();
		hood_to_.clear();
		const int L = int(hood_);
		if (L == 0) {
			hood_of_ = {{{0, 0, -1}}, {{0, -1, 0}}, {{-1, 0, 0}}, {{1, 0, 0}}, {{0, 1, 0}}, {{0, 0, 1}}};
		} else {
			for (int z = -L; z <= L; z++)
				for (int y = -L; y <= L; y++)
					for (int x = -L; x <= L; x++)
						if (x || y || z) hood_of_.push_back({{x, y, z}});
		}
		for (const auto& it : hood_of_) hood_to_.push_back({{-it[0], -it[1], -it[2]}});
		hood_set_ = hood_;
	}

	void refresh_items() {
		if (!g_) return;
		face_cache_valid_ = false;
		lists_.clear();
		send_maps_.clear();
		recv_maps_.clear();
		user_ranges_.clear();
		user_cells_.clear();
		user_neighbors_.clear();
		build_items(default_neighborhood_id, cells_rw, neighbors_rw, ranges_);
	}

	int64_t slot_of(uint64_t id) const {
		int64_t s = -1;
		dccrgx_get_slots(g_, &id, 1, &s);
		return s;
	}

	// neighbors_of / neighbors_to CSR of a neighborhood (slot order)
	void csr(int hood, int kind, std::vector<uint32_t>& ptr, std::vector<uint64_t>& ids,
	         std::vector<int32_t>& off) const {
		ptr.assign(n_local_ + 1, 0);
		size_t n = 0;
		auto call = [&](uint64_t* i, int32_t* o, size_t cap) {
			return hood == default_neighborhood_id ? dccrgx_download_csr(g_, kind, ptr.data(), i, o, cap, &n)
			                                       : dccrgx_download_user_csr(g_, hood, kind, ptr.data(), i, o, cap, &n);
		};
		int rc = call(nullptr, nullptr, 0);
		if (rc != DCCRGX_OK && rc != DCCRGX_ERANGE) detail::check(rc);
		ids.assign(n, 0);
		off.assign(3 * n, 0);
		if (n) detail::check(call(ids.data(), off.data(), n));
	}

	// update_cell_pointers (11314-11628): Cells_Item for inner, outer, remote
	// cells; per cell [only_of | both | only_to] neighbor items, each part in
	// (id, offset) order; ranges of / to / all into it
	void build_items(int hood, std::vector<Cells_Item>& items, std::vector<Neighbors_Item>& nbrs,
	                 std::array<Iterator_Storage<Cells_Item>, 5>& rg) {
		items.clear();
		nbrs.clear();
		std::vector<uint32_t> op, tp;
		std::vector<uint64_t> oi, ti;
		std::vector<int32_t> oo, to;
		csr(hood, 0, op, oi, oo);
		csr(hood, 1, tp, ti, to);
		const size_t nl = n_local_;
		std::vector<uint64_t> all_ids(oi);
		all_ids.insert(all_ids.end(), ti.begin(), ti.end());
		std::vector<int64_t> slots(all_ids.size());
		if (!all_ids.empty()) detail::check(dccrgx_get_slots(g_, all_ids.data(), all_ids.size(), slots.data()));
		auto dptr = [&](int64_t s) -> Cell_Data* { return s >= 0 && size_t(s) < host_.size() ? &host_[size_t(s)] : nullptr; };
		struct Part {
			size_t b, m1, m2, e;  // [b, m1) only_of, [m1, m2) both, [m2, e) only_to
		};
		std::vector<Part> parts(nl);
		std::vector<char> outer(nl, 0);
		using Key = std::pair<uint64_t, std::array<int, 3>>;
		for (size_t r = 0; r < nl; r++) {
			std::vector<std::pair<Key, int64_t>> of_items, to_items;
			for (uint32_t e = op[r]; e < op[r + 1]; e++)
				if (oi[e] != error_cell) of_items.push_back({{oi[e], {{oo[3 * e], oo[3 * e + 1], oo[3 * e + 2]}}}, slots[e]});
			for (uint32_t e = tp[r]; e < tp[r + 1]; e++)
				if (ti[e] != error_cell) to_items.push_back({{ti[e], {{0, 0, 0}}}, slots[oi.size() + e]});
			auto by_key = [](const std::pair<Key, int64_t>& a, const std::pair<Key, int64_t>& b) { return a.first < b.first; };
			auto same = [](const std::pair<Key, int64_t>& a, const std::pair<Key, int64_t>& b) { return a.first == b.first; };
			std::sort(of_items.begin(), of_items.end(), by_key);
			of_items.erase(std::unique(of_items.begin(), of_items.end(), same), of_items.end());
			std::sort(to_items.begin(), to_items.end(), by_key);
			to_items.erase(std::unique(to_items.begin(), to_items.end(), same), to_items.end());
			std::vector<uint64_t> to_ids;
			for (const auto& t : to_items) to_ids.push_back(t.first.first);
			std::vector<uint64_t> of_ids;
			for (const auto& t : of_items) of_ids.push_back(t.first.first);
			std::sort(of_ids.begin(), of_ids.end());
			std::vector<std::pair<Key, int64_t>> only_of, both, only_to;
			for (const auto& t : of_items)
				(std::binary_search(to_ids.begin(), to_ids.end(), t.first.first) ? both : only_of).push_back(t);
			for (const auto& t : to_items)
				if (!std::binary_search(of_ids.begin(), of_ids.end(), t.first.first)) only_to.push_back(t);
			Part& P = parts[r];
			P.b = nbrs.size();
			for (auto* v : {&only_of, &both, &only_to}) {
				if (v == &both) P.m1 = nbrs.size();
				if (v == &only_to) P.m2 = nbrs.size();
				for (const auto& t : *v) {
					Neighbors_Item it{};
					it.id = t.first.first;
					it.data = dptr(t.second);
					it.x = t.first.second[0];
					it.y = t.first.second[1];
					it.z = t.first.second[2];
					nbrs.push_back(it);
					if (t.second < 0 || size_t(t.second) >= nl) outer[r] = 1;
				}
			}
			P.e = nbrs.size();
		}
		// cells: inner, outer, remote (slot order within each)
		const size_t ns = host_.size();
		std::vector<size_t> order;
		for (size_t r = 0; r < nl; r++)
			if (!outer[r]) order.push_back(r);
		const size_t n_inner = order.size();
		for (size_t r = 0; r < nl; r++)
			if (outer[r]) order.push_back(r);
		items.reserve(ns);
		for (size_t r : order) {
			Cells_Item c{};
			c.id = slot_ids_[r];
			c.data = &host_[r];
			items.push_back(c);
		}
		for (size_t s = nl; s < ns; s++) {
			Cells_Item c{};
			c.id = slot_ids_[s];
			c.data = &host_[s];
			items.push_back(c);
		}
		for (size_t k = 0; k < nl; k++) {
			const Part& P = parts[order[k]];
			auto at = [&](size_t i) { return nbrs.cbegin() + ptrdiff_t(i); };
			items[k].neighbors_of = {at(P.b), at(P.m2)};
			items[k].neighbors_to = {at(P.m1), at(P.e)};
			items[k].all_neighbors = {at(P.b), at(P.e)};
		}
		for (size_t k = nl; k < ns; k++)
			items[k].neighbors_of = items[k].neighbors_to = items[k].all_neighbors = {nbrs.cend(), nbrs.cend()};
		auto cat = [&](size_t i) { return items.cbegin() + ptrdiff_t(i); };
		rg[0] = {cat(0), cat(n_inner)};
		rg[1] = {cat(n_inner), cat(nl)};
		rg[2] = {cat(0), cat(nl)};
		rg[3] = {cat(nl), cat(ns)};
		rg[4] = {cat(0), cat(ns)};
		// Additional_*_Items hooks (7318-7339, 7387-7401), for every item the
		// reference builds one for (local and remote cells, 11405-11409, and
		// each neighbor item, 11504-11516), with default-constructed arguments
		for (size_t k = 0; k < ns; k++) {
			Cells_Item& c = items[k];
			c.update_caller(*this, Additional_Cell_Items()...);
			for (size_t i = size_t(c.all_neighbors.begin_ - nbrs.cbegin()); i < size_t(c.all_neighbors.end_ - nbrs.cbegin());
			     i++)
				nbrs[i].update_caller(*this, c, hood, Additional_Neighbor_Items()...);
		}
	}

	const Iterator_Storage<Cells_Item>& range(int hood, int which) const {
		if (hood == default_neighborhood_id) return ranges_[size_t(which)];
		auto it = user_ranges_.find(hood);
		if (it == user_ranges_.end()) {
			auto* self = const_cast<Dccrg*>(this);
			size_t n = 0;
			int rc = dccrgx_download_user_csr(g_, hood, 0, nullptr, nullptr, nullptr, 0, &n);
			if (rc == DCCRGX_ENOTFOUND)
				throw std::runtime_error("dccrg: neighborhood id " + std::to_string(hood) + " doesn't exist");
			self->build_items(hood, self->user_cells_[hood], self->user_neighbors_[hood], self->user_ranges_[hood]);
			it = user_ranges_.find(hood);
		}
		return it->second[size_t(which)];
	}

	const neighbor_list_t* neighbor_list(uint64_t cell, int hood, int kind) const {
		const auto key = std::make_tuple(cell, hood, kind);
		auto it = lists_.find(key);
		if (it != lists_.end()) return &it->second;
		std::vector<uint64_t> ids(8192);
		std::vector<int32_t> off(3 * 8192);
		size_t n = 0;
		int rc;
		if (hood == default_neighborhood_id)
			rc = kind == 0 ? dccrgx_get_neighbors_of(g_, cell, ids.data(), off.data(), ids.size(), &n)
			               : dccrgx_get_neighbors_to(g_, cell, ids.data(), ids.size(), &n);
		else
			rc = dccrgx_get_user_neighbors(g_, hood, cell, kind, ids.data(), off.data(), ids.size(), &n);
		if (rc == DCCRGX_ENOTFOUND) return nullptr;
		detail::check(rc);
		neighbor_list_t v;
		for (size_t i = 0; i < n; i++)
			v.push_back({ids[i], kind == 0 ? std::array<int, 3>{{off[3 * i], off[3 * i + 1], off[3 * i + 2]}}
			                               : std::array<int, 3>{{0, 0, 0}}});
		return &(lists_[key] = std::move(v));
	}

	using list_map = std::unordered_map<int, std::vector<std::pair<uint64_t, int>>>;
	const list_map& lists_for(int hood, bool receive) const {
		if (balancing_) return receive ? bal_recv_ : bal_send_;  // the migration lists (3746-3884)
		auto& cache = receive ? recv_maps_ : send_maps_;
		auto it = cache.find(hood);
		if (it != cache.end()) return it->second;
		list_map m;
		std::vector<int32_t> peers(size_t(std::max(size_, 1)));
		size_t np = 0;
		detail::check(dccrgx_get_peers(g_, peers.data(), peers.size(), &np));
		for (int p = 0; p < size_; p++) {
			if (p == rank_) continue;
			std::vector<uint64_t> v;
			if (hood == default_neighborhood_id)
				v = detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) {
					return receive ? dccrgx_get_cells_to_receive(g_, p, o, c, n) : dccrgx_get_cells_to_send(g_, p, o, c, n);
				});
			else
				v = detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) {
					return dccrgx_get_user_update_list(g_, hood, p, receive ? 1 : 0, o, c, n);
				});
			if (v.empty()) continue;
			auto& dst = m[p];
			for (size_t i = 0; i < v.size(); i++) dst.push_back({v[i], int(i + 1)});
		}
		return cache[hood] = std::move(m);
	}
	const list_map& cells_to_send_map(int hood) const { return lists_for(hood, false); }
	const list_map& cells_to_receive(int hood) const { return lists_for(hood, true); }
	uint64_t count_updates(int hood, bool receive) const {
		if (hood != default_neighborhood_id) {
			size_t n = 0;
			if (dccrgx_download_user_csr(g_, hood, 0, nullptr, nullptr, nullptr, 0, &n) == DCCRGX_ENOTFOUND)
				return ~uint64_t(0);
		}
		uint64_t t = 0;
		for (const auto& kv : lists_for(hood, receive)) t += kv.second.size();
		return t;
	}

	// geometry parameters survive create() (set_geometry may come first)
	struct GeometryHolder : Geometry {
		typename Geometry::Parameters get_params_or_default() const { return params_; }
		void sync_from_library() {
			Geometry::sync_from_library();
			params_ = Geometry::get();
		}
		bool from_file_block(const std::vector<char>& b) {
			if (!Geometry::from_file_block(b)) return false;
			params_ = Geometry::get();
			return true;
		}
		bool set(const typename Geometry::Parameters& p) {
			params_ = p;
			return Geometry::set(p);
		}
		typename Geometry::Parameters params_{};
	};

	dccrgx_grid* g_ = nullptr;
	MPI_Comm comm_ = MPI_COMM_NULL;
	int rank_ = 0, size_ = 1, payload_ = -1;
	int max_ref_ = 0;
	unsigned hood_ = 1;
	std::string lb_method_ = "RCB";
	bool send_single_cells_ = false;
	bool staging_ = true;  // set_host_staging
	std::pair<size_t, size_t> window_{0, sizeof(Cell_Data)};
	Grid_Topology topology_rw;
	Mapping mapping_rw;
	GeometryHolder geometry_rw;
	size_t n_local_ = 0;
	bool dumped_initial_ = false;
	std::vector<uint64_t> removed_ids_;
	std::unordered_map<uint64_t, Cell_Data> refined_;
	std::vector<Cell_Data> removed_;
	std::unordered_map<uint64_t, size_t> removed_index_;
	std::vector<uint64_t> slot_ids_;
	std::vector<Cell_Data> host_;
	// a balance_load in progress: migration lists and the arriving cells' objects
	bool balancing_ = false;
	list_map bal_send_, bal_recv_;
	std::unordered_map<uint64_t, Cell_Data> pending_;
	std::vector<size_t> arrived_;  // serialized Cell_Data: local slots whose bytes came from elsewhere
	std::vector<Cells_Item> cells_rw;
	std::vector<Neighbors_Item> neighbors_rw;
	std::array<Iterator_Storage<Cells_Item>, 5> ranges_{};
	std::map<int, std::vector<Cells_Item>> user_cells_;
	std::map<int, std::vector<Neighbors_Item>> user_neighbors_;
	std::map<int, std::array<Iterator_Storage<Cells_Item>, 5>> user_ranges_;
	mutable std::map<std::tuple<uint64_t, int, int>, neighbor_list_t> lists_;
	mutable std::map<int, list_map> send_maps_, recv_maps_;
	mutable std::vector<Types<3>::neighborhood_item_t> hood_of_, hood_to_;
	mutable unsigned hood_set_ = ~0u;
	std::unordered_map<int, std::vector<Types<3>::neighborhood_item_t>> user_hood_of_, user_hood_to_;
	mutable std::map<uint64_t, std::array<uint64_t, 6>> face_cache_;
	mutable bool face_cache_valid_ = false;
};

}  // namespace dccrg

#endif
