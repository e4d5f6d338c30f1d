// Internal state of one dccrgx grid (one per process / GPU).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdint>
#include <deque>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/dccrgx.h"
#include "dccrgx_mapping.hpp"
#include "dccrgx_mesh.hpp"
#include "dccrgx_neighbors.hpp"

namespace dccrgx {

struct Error : std::runtime_error {
	int code;
	Error(int c, const std::string& s) : std::runtime_error(s), code(c) {}
};

#define DX_STR2(x) #x
#define DX_STR(x) DX_STR2(x)
#define HIP_CHECK(expr)                                                                                        \
	do {                                                                                                       \
		hipError_t e_ = (expr);                                                                                \
		if (e_ != hipSuccess)                                                                                  \
			throw ::dccrgx::Error(DCCRGX_EHIP, std::string(__FILE__ ":" DX_STR(__LINE__) " ") + #expr + ": " + \
			                                       hipGetErrorString(e_));                                     \
	} while (0)
#define NCCL_CHECK(expr)                                                                                        \
	do {                                                                                                        \
		ncclResult_t r_ = (expr);                                                                               \
		if (r_ != ncclSuccess)                                                                                  \
			throw ::dccrgx::Error(DCCRGX_ECOMM, std::string(__FILE__ ":" DX_STR(__LINE__) " ") + #expr + ": " + \
			                                        ncclGetErrorString(r_));                                    \
	} while (0)
#define DX_REQUIRE(cond, msg)                                                     \
	do {                                                                          \
		if (!(cond)) throw ::dccrgx::Error(DCCRGX_EINVAL, std::string(msg)); \
	} while (0)

// Host phase timing of an analysis build (-DDCCRGX_PHASE_TIMING=1, never the
// product build): DX_PHASE("name", stream) times the enclosing scope, the
// stream drained at its end; the totals go to stderr at exit.
#if DCCRGX_PHASE_TIMING
void phase_add(const char* name, double seconds);
void phase_reset();
// seconds spent in the transport's byte mover so far (comm.hip), so that a
// lap can book its time without the transport under "<name>.net"
double& phase_comm_total();
struct PhaseScope {
	const char* name;
	hipStream_t s;
	double t0;
	bool comm;
	static double now();
	PhaseScope(const char* n, hipStream_t st, bool is_comm = false) : name(n), s(st), t0(now()), comm(is_comm) {}
	~PhaseScope() {
		(void)hipStreamSynchronize(s);
		const double d = now() - t0;
		phase_add(name, d);
		if (comm) phase_comm_total() += d;
	}
};
// laps: DX_LAPS(stream) starts a lap clock in this scope, DX_LAP("name")
// books the time since the previous lap (stream drained) under name, and
// that time less the transport's inside it under "name.net"
// stream syncs of the library since start (the pt build counts every
// hipStreamSynchronize below this header's end; the laps' own drains not)
long& phase_sync_count();
struct PhaseLaps {
	hipStream_t s;
	double t, c;
	long k;
	explicit PhaseLaps(hipStream_t st) : s(st), t(PhaseScope::now()), c(phase_comm_total()), k(phase_sync_count()) {}
	void lap(const char* name) {
		(void)hipStreamSynchronize(s);
		const double n = PhaseScope::now(), cn = phase_comm_total();
		phase_add(name, n - t);
		if (cn > c) phase_add((std::string(name) + ".net").c_str(), (n - t) - (cn - c));
		// "<name>.syncs": the stream syncs inside the lap, booked as 1 ms each
		// (the table's ms column is then the count)
		const long kn = phase_sync_count();
		if (kn > k) phase_add((std::string(name) + ".syncs").c_str(), 1e-3 * double(kn - k));
		t = n;
		c = cn;
		k = kn;
	}
};
#define DX_PHASE_CAT2(a, b) a##b
#define DX_PHASE_CAT(a, b) DX_PHASE_CAT2(a, b)
#define DX_PHASE(name, s) ::dccrgx::PhaseScope DX_PHASE_CAT(dx_phase_, __LINE__)(name, s)
#define DX_PHASE_COMM(name, s) ::dccrgx::PhaseScope DX_PHASE_CAT(dx_phase_, __LINE__)(name, s, true)
#define DX_LAPS(s) ::dccrgx::PhaseLaps dx_laps_(s)
#define DX_LAP(name) dx_laps_.lap(name)
#else
#define DX_PHASE(name, s) \
	do {                  \
	} while (0)
#define DX_PHASE_COMM(name, s) \
	do {                       \
	} while (0)
#define DX_LAPS(s) \
	do {           \
	} while (0)
#define DX_LAP(name) \
	do {             \
	} while (0)
#endif

// Owning device buffer.  Buffers of 1 MiB and more start at a rotating skew
// (1..31 x 4352 B, a multiple of 256 B) past the allocator's 2-MiB-aligned
// base, so the same element index of different field arrays does not fall on
// the same DRAM channel / L2 set alignment: paired A/B on config 3 (three
// boxes) 0.1893 / 0.1884 / 0.1904 -> 0.1870 / 0.1864 / 0.1866 ms per sweep.
inline unsigned alloc_skew_next() {
	static std::atomic<unsigned> k{0};
	return (k.fetch_add(1u) * 7u) % 31u + 1u;
}
// Device memory of every DBuf comes from a process-wide caching pool
// (pool.hip): a released block is kept and handed to a later allocation of a
// similar size instead of hipFree (which drains the whole device: ~0.08 ms per
// call, ~2.5 K calls in 20 adaptive steps of config 3).  A block released
// while work that uses it may still be queued is only reused after a device
// synchronisation, the same ordering hipFree gave.  `bytes` is the block's
// capacity (what pool_free must be given back).
void* pool_alloc(size_t bytes, size_t& capacity);
void pool_free(void* raw, size_t capacity);

template <class T>
struct DBuf {
	T* p = nullptr;
	size_t n = 0;
	void* raw = nullptr;
	size_t cap = 0;
	DBuf() = default;
	DBuf(const DBuf&) = delete;
	DBuf& operator=(const DBuf&) = delete;
	DBuf(DBuf&& o) noexcept : p(o.p), n(o.n), raw(o.raw), cap(o.cap) {
		o.p = nullptr;
		o.n = 0;
		o.raw = nullptr;
		o.cap = 0;
	}
	DBuf& operator=(DBuf&& o) noexcept {
		if (this != &o) {
			release();
			p = o.p;
			n = o.n;
			raw = o.raw;
			cap = o.cap;
			o.p = nullptr;
			o.n = 0;
			o.raw = nullptr;
			o.cap = 0;
		}
		return *this;
	}
	~DBuf() { release(); }
	void release() {
		if (raw) pool_free(raw, cap);
		p = nullptr;
		n = 0;
		raw = nullptr;
		cap = 0;
	}
	void alloc(size_t count) {
		if (count == n && p) return;
		release();
		if (count) {
			const size_t skew = count * sizeof(T) >= (size_t(1) << 20) ? size_t(alloc_skew_next()) * 4352u : 0;
			raw = pool_alloc(count * sizeof(T) + skew, cap);
			p = reinterpret_cast<T*>(static_cast<char*>(raw) + skew);
		}
		n = count;
	}
	// grow-only (keeps the allocation when it is large enough)
	void reserve(size_t count) {
		if (count > n) alloc(count);
	}
	void swap(DBuf& o) {
		std::swap(p, o.p);
		std::swap(n, o.n);
		std::swap(raw, o.raw);
		std::swap(cap, o.cap);
	}
};

// bytes from the device into host memory, s drained first (copy + sync);
// reads of up to kSmallRead bytes go through a pinned staging buffer
// (round 6: 4 MiB, the adaptive step's request lists of ~200 KB took 45-65 us
// each through pageable memory)
constexpr size_t kSmallRead = 4 * 1024 * 1024;
void d2h_small(void* host, const void* dev, size_t bytes, hipStream_t s);
// bytes from host memory to the device on s (list-sized ones staged through
// pinned memory and completed on return); the host buffer may be reused on
// return
constexpr size_t kStageUp = 256 * 1024;
void h2d(void* dev, const void* host, size_t bytes, hipStream_t s);

// an id list made on the device, read on the host only when asked (the
// adaptive step never reads its created / removed cells on the host)
struct LazyIds {
	DBuf<uint64_t> d;
	std::vector<uint64_t> h;
	size_t n = 0;
	bool host_valid = true;
	bool unsorted = false;  // the device list is sorted on the first host read
	void clear() {
		d.release();
		h.clear();
		n = 0;
		host_valid = true;
		unsorted = false;
	}
	void set_host(std::vector<uint64_t> v) {
		d.release();
		h = std::move(v);
		n = h.size();
		host_valid = true;
		unsorted = false;
	}
	void set_device(DBuf<uint64_t>&& buf, size_t count, bool sorted = true) {
		h.clear();
		d = std::move(buf);
		n = count;
		host_valid = count == 0;
		unsorted = !sorted && count > 1;
	}
	size_t size() const { return n; }
	bool empty() const { return n == 0; }
	const uint64_t* dev() const { return n && d.n >= n ? d.p : nullptr; }
	inline const std::vector<uint64_t>& host(hipStream_t s);
};

template <class T>
inline void upload(DBuf<T>& d, const std::vector<T>& h, hipStream_t s) {
	d.alloc(h.size());
	if (!h.empty()) h2d(d.p, h.data(), h.size() * sizeof(T), s);
}

template <class T>
inline std::vector<T> download(const T* d, size_t n, hipStream_t s) {
	std::vector<T> h(n);
	if (n) d2h_small(h.data(), d, n * sizeof(T), s);
	return h;
}

void sort_u64(uint64_t* keys, size_t n, hipStream_t s, int end_bit);  // (declared with its default below)

inline const std::vector<uint64_t>& LazyIds::host(hipStream_t s) {
	if (!host_valid) {
		if (unsorted) sort_u64(d.p, n, s, 64);
		unsorted = false;
		h = download(d.p, n, s);
		host_valid = true;
	}
	return h;
}

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// Stream compaction: every lane of a FULL wave (no lane may have exited)
// reserves `c` consecutive output positions from *ctr; one atomic per wave.
// Appending one element per lane per atomic (even wave-aggregated, which the
// compiler already does) serialises on the counter's address: ~140 K wave
// atomics take ~1.5 ms for 8.87 M elements, so callers give each lane a run
// of elements (kAppendRun) and reserve once for all of them.
constexpr int kAppendRun = 16;
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* ctr, unsigned c) {
	const int lane = int(threadIdx.x & 63u);
	unsigned incl = c;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const unsigned v = __shfl_up(incl, d, 64);
		if (lane >= d) incl += v;
	}
	const unsigned total = __shfl(incl, 63, 64);
	unsigned long long base = 0;
	if (lane == 63 && total) base = atomicAdd(ctr, static_cast<unsigned long long>(total));
	base = __shfl(base, 63, 64);
	return base + (incl - c);
}
#endif

inline unsigned grid_for(size_t n, unsigned per_block, unsigned cap = 256u * 32u) {
	size_t g = (n + per_block - 1) / per_block;
	if (g > cap) g = cap;
	if (g == 0) g = 1;
	return unsigned(g);
}

// A field: one SoA array over all slots.  The halo carries bytes
// [win_off, win_off + win_len) of every element (the part a Cell_Data's
// get_mpi_datatype describes, dccrg_get_cell_datatype.hpp:40-340); the whole
// element by default.
struct Field {
	std::string name;
	size_t elem = 0;
	bool transfer = false;
	size_t win_off = 0, win_len = 0;
	DBuf<uint8_t> data;     // n_slots * elem
	DBuf<uint8_t> scratch;  // double buffer for sweeps (allocated on demand)
	// payloads of the cells removed by the last stop_refining whose parent is
	// local (unrefined_cell_data 7250), in the order of Grid::removed_ids
	DBuf<uint8_t> removed;
	// variable-size payloads (varfield.hip): elem == 0, `data` is a byte pool
	// and slot s owns [voff[s], voff[s + 1]); the removed store likewise
	// (rm_off, one entry per removed cell + 1)
	bool var = false;
	DBuf<uint64_t> voff, rm_off;
	// every local element known to be all-zero bytes (set by the refined game
	// of life turn, which leaves each local list error_cell-cleared as the
	// reference does; dropped by anything that may write local payloads)
	bool local_zero = false;
	// the next rebuild does not carry this field's payloads (its caller
	// rewrites every local element right after, e.g. advection_adapt's
	// velocity / length reset): the local part is left unwritten, the rest
	// zeroed; the flag is dropped by that rebuild
	bool no_carry = false;
	// write tracking for caches derived from the payloads (the advection
	// sweep's neighbor records, NbRecords): `epoch` goes up with every write
	// the library makes or is asked to make (field_written); `external` is set
	// once the device pointer was handed out (writes then untracked, so no
	// cache is built from the field until the next structural change moves
	// the array and voids that pointer)
	uint64_t epoch = 0;
	// writes of local slots only (epoch counts remote-copy writes too): a
	// cache over the inner cells, which read no remote copy, checks this one
	uint64_t local_epoch = 0;
	bool external = false;
	bool full_window() const { return win_off == 0 && win_len == elem; }
};

inline void field_written(Field& f) {
	f.epoch++;
	f.local_epoch++;
}
// a write of the field's remote copies only (halo receives)
inline void field_halo_written(Field& f) { f.epoch++; }

// ---- Poisson BiCG (tests/poisson/poisson_solve.hpp) ------------------------
// device pointers of one solve: user fields rhs / solution, the solver's own
// per-slot fields and the filtered face table (see poisson_kernels.hip)
struct PoArrays {
	const int32_t* ell;   // 6 per local slot: slot, -1, or -2-k -> fine[4k..4k+3] (-1 = dropped)
	const int32_t* fine;
	const int32_t* type;  // 0 solve, 1 boundary, 2 skip
	const double* rhs;
	double *sol, *best, *p0, *p1, *r0, *r1, *ap0, *sf;
	double* f[6];  // f_x_neg, f_x_pos, f_y_neg, f_y_pos, f_z_neg, f_z_pos
	// ft[dir * n + s]: the same-size / coarser neighbor's factor toward s
	// (f[dir ^ 1][ell[6 s + dir]]), gathered once per cache pass for phase B's
	// transpose product (null: phase B gathers it)
	const double* ft;
};

struct PoParams {  // Poisson_Solve constructor, poisson_solve.hpp:187-201
	unsigned max_it, min_it;
	double stop_residual, p_of_norm, stop_increase;
};

// the solver's scalars, resident on the device (host reads them only to
// detect termination)
struct PoScalars {
	double dot_r, alpha, beta, residual, residual_min, norm;
	unsigned iteration, done, save, stop_b;
};

enum { PO_PHASE_INIT, PO_PHASE_A, PO_PHASE_B, PO_PHASE_C, PO_PHASE_FINISH, PO_PHASE_JACOBI, PO_PHASE_JACOBI_COPY };
enum { PO_STAGE_INIT, PO_STAGE_A, PO_STAGE_B, PO_STAGE_JACOBI_INIT, PO_STAGE_JACOBI };

struct PoissonState {
	bool valid = false;        // cache_system_info done for the current mesh
	int rhs = -1, sol = -1;    // user fields
	int type = -1;             // int32 field: classification / final type
	int p0 = -1, p1 = -1, r0 = -1, r1 = -1, ap0 = -1, best = -1, sf = -1, f[6] = {-1, -1, -1, -1, -1, -1};
	DBuf<int32_t> ell, fine;
	DBuf<double> ft;               // PoArrays::ft
	DBuf<double> part, red, gath;  // gath: P x 2 all-gathered per-rank sums
	DBuf<PoScalars> st;
	size_t n_cached = 0;       // local cells in cell_info
};

// one regular advection tile (tile_build.hip): first slot and the start slot
// of the same-level neighbor box across each side (-1: none)
struct RegTileMeta {
	uint32_t ts;
	int32_t nst[6];
	uint32_t pad;
};

// Send / receive lists of one neighborhood (recalculate_neighbor_update_
// send_receive_lists 8590-8752): per peer the ids in ascending order (= the
// wire order of update_copies_of_remote_neighbors), their slots flattened
// peer by peer, and staging buffers.  For the default neighborhood the
// receive slots of a peer are one contiguous run of halo slots.
struct HaloPlan {
	std::map<int, std::vector<uint64_t>> send_ids, recv_ids;
	std::map<int, size_t> send_off, recv_off;  // cell offsets into send_slots / recv_slots
	size_t n_send = 0, n_recv = 0;
	DBuf<int32_t> send_slots, recv_slots;
	DBuf<uint8_t> sendbuf, recvbuf;
	std::vector<int> peers() const;
};

// A user neighborhood (add_neighborhood, dccrg.hpp:6383-6520): its offsets,
// neighbors_of / neighbors_to CSR of the local cells (built lazily after
// every structural change, update_user_neighbors 8974-8980) and its halo plan.
struct UserHood {
	std::vector<int32_t> of, to;  // 3 per item; to = -of
	DBuf<int32_t> d_of, d_to;
	bool valid = false;
	DBuf<uint32_t> nof_ptr, nto_ptr;
	DBuf<uint64_t> nof_id, nto_id;
	DBuf<int32_t> nof_off;
	HaloPlan plan;
};

// The leaves this rank knows (dccrgx_mesh.hpp): implicit (initial level-0
// grid, block partition) or an explicit list of own + ghost leaves.
struct Mesh {
	bool implicit = true;
	DBuf<uint64_t> kid;   // explicit: known leaves, any order
	DBuf<int32_t> kown;   // their owners
	size_t n_known = 0;
	// when > 0 (explicit meshes on Morton slots): kid[0, n_prefix) are the own
	// leaves, kid[0, prefix_run1) and kid[prefix_run1, n_prefix) each in Morton
	// order (set by rebuild, carried through refinement by k_apply_refines)
	size_t n_prefix = 0, prefix_run1 = 0;
	// per own leaf of the prefix, the old slot its payload comes from (-1
	// none), when k_apply_refines made this mesh from one whose prefix was
	// the old slot order; used (and released) by rebuild's carry step
	DBuf<int32_t> carry;
	DBuf<HashEntry> tab;
	uint64_t mask = 0;
	uint32_t shift = 63;
	// the range map instead of `tab` (dccrgx_mesh.hpp DevMesh::rmap)
	DBuf<int2> rmap;
	RangeLevel rl[kRangeLevels] = {};
	int rlev = 0;
	// the grid's persistent full-level map (Grid::rmap_full) instead of an
	// owned one: not freed with the mesh, cleared entry by entry by the next
	// rebuild
	const int2* rmap_shared = nullptr;
	BlockPart bp;
	DevMesh dev(uint64_t last) const {
		DevMesh d{};
		d.tab = tab.p;
		d.mask = mask;
		d.shift = shift;
		d.implicit = implicit ? 1 : 0;
		d.bp = bp;
		d.last = last;
		d.rmap = rmap_shared ? rmap_shared : rmap.p;
		d.rlev = d.rmap ? rlev : 0;
		for (int L = 0; L < d.rlev; L++) d.rl[L] = rl[L];
		return d;
	}
};

// Gathered variable-size payloads of the cells of a send list (sizes on the
// device and the host, concatenated bytes) and what arrived for a receive
// list (varfield.hip, grid.hip)
struct VarMsg {
	DBuf<uint64_t> ssz, rsz;
	DBuf<uint8_t> sbytes, rbytes;
	std::vector<uint64_t> hs;
};

// A balance_load in progress (initialize_balance_load 3746 / continue 3899 /
// finish 3942): per peer the cells leaving / arriving (ascending id), the
// payloads of every field packed peer by peer (per peer: field 0 of every
// cell, field 1 of every cell, ...).
struct Migration {
	bool active = false, transferred = false;
	std::map<int, std::vector<uint64_t>> out, in;
	std::map<int, size_t> out_off, in_off;  // byte offsets into the buffers
	std::vector<uint64_t> in_pinned;        // arriving cells that stay pinned here
	DBuf<uint8_t> sendbuf, recvbuf;
	size_t bytes_per_cell = 0;
	std::vector<VarMsg> var;  // per variable-size field (field order)
};

// a box of whole z-planes of the uniform grid in slot order (slot0 first
// slot, nz planes) and the slots of its z-1 / z+1 planes (-2: outside the
// grid, -3: the box wraps onto itself periodically)
// refined game of life per mesh: level-0 parent of every slot (bit 31 set
// on level-0 leaves), the per-call packed (parent << 1 | alive), the groups
// of slots sharing a refined level-0 parent (gptr / gslot) and the local
// level-0 leaves
// Mask path (neighborhood length <= 1, small enough grids): every neighbor's
// level-0 parent is one of the 27 level-0 cells around the row's own, so a
// neighbor entry carries that position (code 0..26, 13 = the own parent)
// next to its slot (ent = slot | code << 27) and the distinct live parents
// of a leaf are a 27-bit mask (mask, per slot); l0c = packed level-0
// coordinates (x | y << bx | z << (bx + by)) of every slot
struct GolAmrTables {
	bool valid = false;
	DBuf<uint32_t> l0, pack, gptr, gslot, lvl0;
	size_t ng = 0, n_lvl0 = 0;
	bool mask_path = false;
	DBuf<uint32_t> l0c, ent, mask;
	size_t n_ent = 0;
	uint32_t bx = 0, by = 0, lx = 0, ly = 0, lz = 0;
	// geometric collect (maximum refinement level <= 1, mask path): per local
	// slot its child octant (bit 7: a level-0 leaf); per level-0 cell of the
	// known region's bounding box a byte (bit 0: a known leaf there alive,
	// bit 1: one dead)
	bool geo = false;
	bool lg_layout = false;  // every family eight consecutive slots (the level-0 game)
	DBuf<uint32_t> lg_rows;  // its rows: level-0 leaves' and families' first slots, ascending
	size_t n_lg_rows = 0;
	DBuf<uint8_t> corner, l0tab;
	uint32_t box0[3] = {0, 0, 0}, boxn[3] = {0, 0, 0};
	uint32_t geo_lb[3] = {0, 0, 0}, geo_bstride[3] = {1, 1, 1}, geo_istride[3] = {1, 1, 1};  // table blocks
	int per[3] = {0, 0, 0};
};

struct GolBox {
	uint64_t slot0, nz;
	int64_t lo, hi;
};

struct Grid {
	// communicator: RCCL (nccl != nullptr), a caller-provided host exchange
	// (xfn), or none (a detached view: structures only, no collectives)
	int rank = 0, size = 1, device = 0;
	ncclComm_t nccl = nullptr;
	dccrgx_exchange_fn xfn = nullptr;
	void* xctx = nullptr;
	hipStream_t s_comp = nullptr, s_comm = nullptr;
	hipEvent_t ev_comp = nullptr, ev_halo = nullptr;
	bool halo_in_flight = false;
	bool send_single_cells = false;  // set_send_single_cells (6677): halo messages one cell at a time

	// setup (dccrg.hpp:8120-8230)
	uint64_t len[3] = {1, 1, 1};
	int R = 0;
	int per[3] = {0, 0, 0};
	unsigned hood_len = 1;
	bool initialized = false;
	MapCtx m{};
	std::vector<int32_t> hood;     // neighborhood_of, 3 per item
	std::vector<int32_t> hood_to;  // neighborhood_to (negated)
	double start[3] = {0, 0, 0}, l0[3] = {1, 1, 1};
	// a grid file's geometry block other than the Cartesian one (the bytes
	// Stretched_Cartesian_Geometry::write makes, id 2): written by
	// save_grid_data instead of start / l0, read back by load_grid_data
	// (dccrgx_set_geometry_block / dccrgx_get_geometry_block); empty: Cartesian
	std::vector<uint8_t> geo_block;

	Mesh mesh;
	std::unordered_map<uint64_t, int> pins;  // local cells pinned to a process (pin 5832-5909)
	std::unordered_map<uint64_t, double> weights;  // set_cell_weight (6210), cleared by balance_load
	std::string lb_method = "RCB";                 // set_load_balancing_method (8223); default 7082
	std::unordered_set<uint64_t> refine_requests;      // refine_completely 2434
	std::unordered_set<uint64_t> unrefine_requests;    // unrefine_completely 2560 (one sibling per family)
	// requests made in bulk by the device check_for_adaptation: plain lists,
	// merged into the sets above by flush_bulk_requests() before any call
	// that consults the sets, and read directly by stop_refining
	std::vector<uint64_t> refine_bulk, unrefine_bulk;
	// refine_bulk's device copy when it is exactly one device request list
	// (check_for_adaptation's, sorted and unique) and nothing else was
	// requested: stop_refining then skips its uploads of that list
	DBuf<uint64_t> refine_dev;
	bool refine_dev_valid = false;
	// the same for unrefine_bulk: check_for_adaptation's whole-family heads
	// on one process (octant-0 children, ascending: their parents ascend too)
	DBuf<uint64_t> unrefine_dev;
	bool unrefine_dev_valid = false;
	// the last stop_refining's merged parents on the device (one process:
	// every removed cell's parent, sorted), for adapt_grid's parent means
	DBuf<uint64_t> merged_dev;
	size_t n_merged = 0;
	// a grid file being loaded in parts (start / continue / finish_loading_
	// grid_data 1795-2400): per local slot the next unread byte of the cell's
	// record and the record's end
	struct FileLoad {
		bool active = false;
		std::string path;
		std::vector<uint64_t> pos, end;
	} load;
	std::unordered_set<uint64_t> dont_unrefine_cells;  // dont_unrefine 2679
	std::unordered_set<uint64_t> dont_refine_cells;    // dont_refine 2744
	LazyIds removed_ids;  // get_removed_cells 3497 (order of Field::removed)
	LazyIds new_cells;    // local cells created by the last stop_refining (ascending on the host)
	Migration mig;
	// the range map over the full id range of every level (one process,
	// Morton-ordered own leaves: rebuild's "direct" mode), kept across
	// rebuilds: each rebuild clears the previous mesh's entries and writes its
	// own instead of clearing the whole map
	DBuf<int2> rmap_full;
	bool rmap_full_clean = true;  // every entry {-1, -1}
	// a cleared per-level range map (every entry {-1, -1}) over rmap_spare_rl:
	// the previous explicit mesh's map, its entries cleared one by one at the
	// end of rebuild, taken by the next mesh whose level ranges it covers (no
	// memset of the ranges; slabs of several processes)
	DBuf<int2> rmap_spare;
	RangeLevel rmap_spare_rl[kRangeLevels] = {};
	int rmap_spare_rlev = 0;
	DBuf<double> red_all;  // P x count all-gathered values of comm_allreduce_f64_dev (s_comp only)
	// pinned host staging of the host-exchange transport (comm.hip
	// move_bytes), grow-only, freed with the grid: the device <-> host legs
	// then run on the copy engines instead of the runtime's pageable path
	uint8_t* pin_stage = nullptr;
	size_t pin_stage_cap = 0;
	DBuf<double> dt_part;  // block minima of the advection time step (dt_cache)
	// the block minima in dt_part are those of the velocity / length fields
	// fid with these write epochs over n_local cells (nb of them): the time
	// step of advection_adapt's reset pass (fused into it), or of the last
	// max_time_step, reused until one of the fields is written again
	struct DtCache {
		bool valid = false;
		int fid[6] = {-1, -1, -1, -1, -1, -1};
		uint64_t epoch[6] = {0, 0, 0, 0, 0, 0};
		size_t n_local = 0, nb = 0;
	} dt_cache;
	// check_for_adaptation's bands computed by the face-table sweep
	// (advection_ell_lds_kernel<true>) with the parameters of the last check
	// call, per run (0 inner, 1 outer): valid for the check that follows when
	// the face table, the density array and its writes since are the ones the
	// sweep saw (DCCRGX_BAND_CACHE=0: always the separate bands kernel)
	DBuf<uint8_t> band_cache;
	struct BandRec {
		bool valid = false;
		uint64_t face_gen = 0, epoch = 0, local_epoch = 0;
		const void* rho = nullptr;
	} band_rec[2];
	bool band_params_valid = false;
	double band_inc = 0, band_thr = 0, band_uns = 0;
	uint64_t face_gen = 0;  // bumped by every face table build (ensure_face)

	// local layout
	size_t n_inner = 0, n_outer = 0, n_local = 0, n_recv = 0, n_slots = 0;
	std::vector<int> peers;           // union of send/recv peers, ascending
	HaloPlan halo;                    // default neighborhood
	std::vector<uint64_t> extra_remote;  // remote neighbors_to-only cells
	std::vector<uint64_t> slot_ids_h;    // host mirror of slot -> id
	bool slot_ids_h_valid = false;
	// host index of the slotted ids (ascending) and their slots, for per-cell
	// queries (is_local, operator[], refine_completely) without a device trip
	std::vector<uint64_t> index_ids_h;
	std::vector<int32_t> index_slots_h;
	bool index_h_valid = false;

	DBuf<uint64_t> slot_ids;  // n_slots
	DBuf<int32_t> d_hood, d_hood_to;
	// full CSR (built lazily): neighbors_of (stencil order), neighbors_to (ascending)
	bool csr_valid = false;
	DBuf<uint32_t> nof_ptr, nto_ptr, it_ptr;
	DBuf<uint64_t> nof_id, nto_id;
	DBuf<int32_t> nof_off, nof_slot, it_slot, it_off;
	// face table (built lazily, ensure_face) and its CSR form (built from the
	// table when a consumer needs it, ensure_face_csr): entry = slot * 8 + dir
	// (dir 0..5 = -x,+x,-y,+y,-z,+z)
	bool face_valid = false, face_csr_valid = false;
	// advection sweeps committed on the current mesh (rebuild resets it): the
	// first step on a new mesh sweeps the face table, tiles are built for the
	// second (a mesh that changes every step never pays for them)
	unsigned adv_commits_on_mesh = 0;
	DBuf<uint32_t> face_ptr;
	DBuf<int32_t> face_ent;
	DBuf<int32_t> face_ell, face_fine;  // fixed-width form used by the advection sweep
	DBuf<uint8_t> slot_lvl;             // refinement level of every slot (with the face table)
	size_t n_fine_faces = 0;
	// face tiles (built lazily from the face CSR): the inner and the outer run
	// of slots are cut into tiles of at most `tile` consecutive slots
	// (boundaries `tstart`, on aligned Morton boxes where possible); per tile the
	// distinct out-of-tile face neighbors (`ext`, ascending slot) and per cell
	// six 16-bit tile-local neighbor indices (< tile: a slot of the tile,
	// tile + k: ext[k] of the tile, 0x8000 | j: finer face j of the tile whose
	// four tile-local indices are in `tfine`, 0xffff: no face neighbor)
	bool tiles_valid = false;
	int tile = 512;
	size_t n_tiles_inner = 0, n_tiles_outer = 0, max_ext = 0, total_ext = 0;
	DBuf<uint32_t> tstart;     // n_tiles + 1
	DBuf<uint32_t> tell;       // 3 x u32 per local slot (6 x u16)
	DBuf<uint32_t> ext_ptr;    // n_tiles + 1
	DBuf<uint32_t> ext;        // total_ext slots
	DBuf<uint32_t> ext_pk;     // ext slots | axis mask << 29 (axes through which a face reaches the cell)
	DBuf<uint32_t> fine_base;  // n_tiles: index of the tile's first finer face
	DBuf<uint32_t> tfine;      // 2 x u32 per finer face (4 x u16)
	// regular tiles (aligned uniform 8x8x8 boxes, see tile_build.hip) are swept
	// without face rows; tlists = [regular inner | regular outer | irregular
	// inner | irregular outer] tile indices, tcount = the four lengths,
	// tnb = per tile the six neighbor-box start slots (-1: none)
	DBuf<uint32_t> tlists;
	DBuf<int32_t> tnb;
	size_t tcount[4] = {0, 0, 0, 0};
	DBuf<RegTileMeta> tregmeta;  // per regular tile (list order): start slot + neighbor-box starts
	// per irregular tile (list order), 8 x u32: first slot, slots, first ext,
	// ext count, first finer face, finer faces; empty when some tile exceeds
	// the pipelined kernel's capacities (> 1024 ext cells or > 512 finer
	// faces): the run is then swept by the untiled face-CSR kernel
	DBuf<uint32_t> tmeta;
	// both kinds in tile order per run (advection_fused_kernel), 8 x u32 per
	// tile, word 7 = 1 for a regular tile (then RegTileMeta's words), 0 for
	// another (then tmeta's); empty with tmeta
	DBuf<uint32_t> tfused;
	size_t tfused_n[2] = {0, 0};
	uint64_t tiles_gen = 0;  // bumped by every tile build
	// Neighbor records of the tile sweeps (sweep_kernels.hip, built by
	// ensure_nbrec): per axis a and slot s one 24-B record {l_a, l_b * l_c,
	// v_a} (b < c the other two axes, the product as the reference forms the
	// face area) at r[(3 a n_slots + 3 s) ..], so an out-of-tile face neighbor
	// costs its density and one record instead of five field lines.  Built
	// from the velocity / length fields of the sweep, kept while their ids,
	// epochs and arrays and the tiles are unchanged.
	struct NbRecords {
		DBuf<double> r;
		int fid[6] = {-1, -1, -1, -1, -1, -1};
		uint64_t epoch[6] = {0, 0, 0, 0, 0, 0};
		const void* ptr[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
		uint64_t tiles_gen = 0;
		size_t n_slots = 0;
		bool valid = false;
	} nbrec;
	std::vector<int> halo_fields;  // fixed-size fields of the halo in flight (written again when it lands)
	std::map<int, UserHood> uhoods;  // add_neighborhood ids
	GolAmrTables gola;  // refined game of life: per-mesh tables (gol_amr.hip)
	// uniform game of life: the regions as plane boxes (gol_slab_plan), built lazily
	bool gol_plan_valid = false, gol_plan_ok = false;
	std::vector<GolBox> gol_inner, gol_outer;

	std::vector<Field> fields;

	// timing of sweep kernels (HIP events on s_comp)
	bool timing = false;
	double timed_ms = 0;
	int64_t timed_count = 0;
	std::deque<std::pair<hipEvent_t, hipEvent_t>> pending_events;

	// slot order inside the inner and outer runs: 0 = ascending id (raster,
	// needed by the structured uniform kernels), 1 = Morton order of the min
	// corners (locality for refined meshes)
	int slot_order = -1;  // -1: Morton when R > 0, else id
	bool morton_slots = false;  // the order in effect

	PoissonState po;

	DevMesh dm() const { return mesh.dev(m.last); }
	bool uniform() const { return R == 0; }
	bool has_collectives() const { return size == 1 || nccl != nullptr || xfn != nullptr; }
};

// --- comm.hip: collectives and point-to-point transfers -----------------------
// Every rank calls these in the same order (as the reference's MPI calls).
// exchange: send[p] to rank p, receive what rank p sends (any sizes)
std::vector<std::vector<uint8_t>> comm_exchange(Grid& g, const std::vector<std::vector<uint8_t>>& send);
std::vector<std::vector<uint64_t>> comm_allgather_u64(Grid& g, const std::vector<uint64_t>& mine);
std::vector<std::vector<uint64_t>> comm_alltoall_u64(Grid& g, const std::vector<std::vector<uint64_t>>& send);
void comm_allreduce_f64(Grid& g, double* v, int count, int op);  // 0 sum, 1 min, 2 max
// the same on device values, queued on s (stream-ordered over RCCL)
void comm_allreduce_f64_dev(Grid& g, const double* d_in, double* d_out, int count, int op, hipStream_t s);
uint64_t comm_allreduce_max_u64(Grid& g, uint64_t v);
// device payloads: per peer one message of known size each way.  cell > 0:
// the message is a run of cells of `cell` bytes each way, which
// send_single_cells (6677) puts on the wire one cell at a time (comm.hip)
struct DevMsg {
	int peer;
	const uint8_t* send;
	size_t send_bytes;
	uint8_t* recv;
	size_t recv_bytes;
	size_t cell = 0;
};
// one grouped point-to-point round of device messages (the same message list
// for every transport; see comm.hip)
void comm_device_transfer(Grid& g, const std::vector<DevMsg>& msgs, hipStream_t s);
void comm_loopback(Grid& g, const void* send, void* recv, size_t bytes, size_t cell, hipStream_t s);
// every rank's `bytes` at `mine` into all[p * bytes] on the device (own slot included)
void comm_allgather_dev(Grid& g, const void* mine, size_t bytes, uint8_t* all, hipStream_t s);
// P x count values, rank-major, combined in rank order (op 0 sum, 1 min, 2 max)
void rank_ordered_combine(const double* all, int P, int count, int op, double* out);
void comm_require(const Grid& g, const char* what);

// --- mesh.hip: knowledge, hash table, structures --------------------------------
void mesh_init_implicit(Grid& g);
// from a global leaf list (every leaf, ascending, owners): keep own + ghost
void mesh_from_global(Grid& g, Mesh& out, const std::vector<uint64_t>& ids, const std::vector<int32_t>& owners);
// explicit own + ghost list of the current mesh (materializes an implicit mesh)
void mesh_materialize(Grid& g, Mesh& out);
// after a repartition: own leaves known, ghosts fetched from their owners
void mesh_from_local(Grid& g, Mesh& out, DBuf<uint64_t>& local, size_t n_local);
// (entries i < slot_upto get slot i, the others -1)
void mesh_build_range(Grid& g, Mesh& M, const uint64_t* ids, const int32_t* owners, size_t n, hipStream_t s,
                      size_t slot_upto);
bool k_level_ranges(const MapCtx& m, const uint64_t* ids, size_t n, uint64_t* lo, uint64_t* hi, hipStream_t s);
void k_range_insert(int2* rmap, const DevMesh& M, const uint64_t* ids, const int32_t* owners, size_t n, size_t slot_upto,
                    hipStream_t s);
void k_range_clear(int2* rmap, const DevMesh& M, const uint64_t* ids, size_t n, hipStream_t s);
void mesh_build_hash(Mesh& M, const uint64_t* ids, const int32_t* owners, size_t n, hipStream_t s,
                     size_t slot_upto = 0);
void rebuild(Grid& g, Mesh& new_mesh);  // new_mesh is moved into g.mesh
void ensure_csr(Grid& g);
void ensure_face(Grid& g);
void ensure_face_csr(Grid& g);  // ensure_face + face_ptr / face_ent
void ensure_tiles(Grid& g);
const std::vector<uint64_t>& slot_ids_host(Grid& g);
// batch lookups of known leaves: owner (-1 unknown) and slot (-1 none)
void lookup_batch(Grid& g, const uint64_t* ids, size_t n, int32_t* owner, int32_t* slot);
int32_t lookup_owner(Grid& g, uint64_t id);
bool is_local_cell(Grid& g, uint64_t id);
int64_t lookup_slot(Grid& g, uint64_t id);
// all known leaves (own + ghost) ascending
void known_leaves(Grid& g, std::vector<uint64_t>& ids, std::vector<int32_t>& owners);
// local leaf ids on the device (slot order)
inline const uint64_t* local_ids_dev(const Grid& g) { return g.slot_ids.p; }

// the face table of the local rows (ensure_face): per row and direction the
// neighbor's slot (same size or coarser), -1, or -2 - k for the finer face k
// (its 4 slots at fine[4 k ..]), in reference order
struct FaceView {
	const int32_t* ell;
	const int32_t* fine;
	const uint64_t* slot_ids;
	size_t n_local;
};

// --- launchers implemented in build_kernels.hip -----------------------------
void k_fill_i32(int32_t* p, size_t n, int32_t v, hipStream_t s);
void k_iota_u64(uint64_t* out, uint64_t first, size_t n, hipStream_t s);
void k_hash_insert(HashEntry* tab, uint64_t mask, uint32_t shift, const uint64_t* ids, const int32_t* owners,
                   int32_t owner_const, size_t n, hipStream_t s, size_t slot_upto = 0);
void k_hash_set_slots(const DevMesh& M, const uint64_t* slot_ids, size_t n, int32_t* err, hipStream_t s);
void k_lookup(const DevMesh& M, const uint64_t* ids, size_t n, int32_t* owner, int32_t* slot, hipStream_t s);
// flag local cells that have a remote neighbors_of / neighbors_to entry;
// with `near` (a byte per level-0 id in [near_lo, near_lo + near_n), see
// k_level0_near) only cells whose level-0 parent is marked are examined, the
// others are inner
void k_remote_flags(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const DevMesh& M, int rank,
                    const uint64_t* cells, size_t n, uint32_t* flag, hipStream_t s, const uint8_t* near = nullptr,
                    uint64_t near_lo = 0, size_t near_n = 0);
// Level-0 cells within `radius` level-0 cells of a ghost leaf's level-0
// parent, marked in a byte map over the level-0 span of the known leaves
// (every neighbors_of / neighbors_to entry of a leaf lies under the level-0
// cells within that radius of its level-0 parent, so a leaf under an
// unmarked level-0 cell has no remote neighbor).  False when the span is too
// sparse for a map (then no filter).
bool k_level0_near(const MapCtx& m, const uint64_t* kid, const int32_t* kown, size_t n_known, int rank, int radius,
                   DBuf<uint8_t>& near, uint64_t& near_lo, hipStream_t s);
// local ids -> slots: inner first, outer second, both in the input order
void k_assign_slots2(const uint32_t* flag, const uint32_t* scan_outer, size_t n, size_t n_inner, const uint64_t* cells,
                     uint64_t* slot_ids, hipStream_t s);
void k_fill_neighbors_of(const MapCtx& m, const int32_t* hood, int nh, const DevMesh& M, const uint64_t* slot_ids,
                         size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids, int32_t* offs, hipStream_t s);
void k_fill_neighbors_to(const MapCtx& m, const int32_t* hood_to, int nh, const DevMesh& M, const uint64_t* slot_ids,
                         size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids, hipStream_t s);
void k_count_rows(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const DevMesh& M,
                  const uint64_t* slot_ids, size_t row0, size_t nrows, uint32_t* nof_cnt, uint32_t* nto_cnt,
                  hipStream_t s);
int max_hood_items();  // largest stencil the neighbors_to dedupe can hold in LDS
// the entries of an id array owned by another process, grouped by owner
// (each group ascending, unique); device sorts of owner * (last + 1) + id
// keys, or of (owner, id) pairs when the ids leave no room for the owner
// remote ids of `ids` grouped by owner, each group ascending; `keep` (when
// given) receives the sorted unique (owner * (last + 1) + id) keys on the
// device and `keep_n` their count (0 and no keys when the keys would overflow)
void k_remote_by_owner(const uint64_t* ids, size_t n, const DevMesh& M, int rank, int size,
                       std::map<int, std::vector<uint64_t>>& out, hipStream_t s, DBuf<uint64_t>* keep = nullptr,
                       size_t* keep_n = nullptr);
// Rebuild step 3 in one device pass and two reads (the pair-free case): the
// receive lists (remote neighbors_of), the send lists (local cells in whose
// neighbors_to a remote cell appears) grouped by peer, ascending, the remote
// neighbors_to-only ids, and both lists' ids on the device in wire order
struct HaloLists {
	std::map<int, std::vector<uint64_t>> recv, send;
	std::vector<uint64_t> extra;
	DBuf<uint64_t> recv_keys, send_keys, recv_ids, send_ids;
	size_t n_recv = 0, n_send = 0;
};
bool k_halo_lists(const uint64_t* of_id, size_t t_of, const uint64_t* to_id, const uint32_t* p_to, size_t t_to,
                  const uint64_t* slot_ids, size_t row0, size_t nrows, const DevMesh& M, int rank, int size,
                  HaloLists& out, hipStream_t s);
void k_iota_i32(int32_t* out, size_t n, int32_t first, hipStream_t s);
// the remote ids of `ids` whose key is not among `of_keys` (kept by
// k_remote_by_owner), ascending; false when keys would overflow
bool k_remote_extra(const uint64_t* ids, size_t n, const DevMesh& M, int rank, int size, const uint64_t* of_keys,
                    size_t n_of, std::vector<uint64_t>& out, hipStream_t s);
// the send side: for each neighbors_to entry (n_entries in all) with a remote
// owner, the row's own id under that owner
void k_send_by_owner(const uint64_t* nto_id, const uint32_t* nto_ptr, size_t n_entries, const uint64_t* slot_ids,
                     size_t row0, size_t nrows, const DevMesh& M, int rank, int size,
                     std::map<int, std::vector<uint64_t>>& out, hipStream_t s);
size_t sort_unique_u64(uint64_t* keys, size_t n, hipStream_t s, int end_bit = 64);  // in place; keys < 2^end_bit
void sort_u64(uint64_t* keys, size_t n, hipStream_t s, int end_bit = 64);  // in place; keys < 2^end_bit
void host_sort_u64(std::vector<uint64_t>& v, bool unique, hipStream_t s);  // host list, device radix sort when large
// (id, slot) of every slot sorted by id
void k_sorted_slot_index(const uint64_t* slot_ids, size_t n, std::vector<uint64_t>& ids, std::vector<int32_t>& slots,
                         hipStream_t s);
void k_morton_merge2(const MapCtx& m, uint64_t* ids, size_t n, size_t run1, hipStream_t s);
void k_morton_sort(const MapCtx& m, uint64_t* ids, size_t n, hipStream_t s);
uint32_t scan_exclusive_u32(const uint32_t* in, uint32_t* out, size_t n, hipStream_t s);  // returns total
// two scans of n + 1 entries (the same temp storage size), both totals in one read
void scan_exclusive_u32_pair(const uint32_t* in1, uint32_t* out1, const uint32_t* in2, uint32_t* out2, size_t n,
                             hipStream_t s, size_t& t1, size_t& t2);
// the same, and out[at[j]] (j < k <= 3) into vals, all in one device read
uint32_t scan_exclusive_u32_at(const uint32_t* in, uint32_t* out, size_t n, hipStream_t s, const size_t* at, int k,
                               uint32_t* vals);
void k_lookup_slots(const uint64_t* ids, size_t n, const DevMesh& M, int32_t* out, int32_t* err_flag, hipStream_t s);
// iterator ranges cell.neighbors_of (update_cell_pointers 11451-11500): pass
// 0 classifies the neighbors_of entries into cls (one byte per entry) and
// counts, pass 1 fills slots (+ offsets when it_off != nullptr)
void k_iterator_lists(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                      const int32_t* nof_slot, const uint32_t* nto_ptr, const uint64_t* nto_id, size_t nrows,
                      uint8_t* cls, uint32_t* it_cnt, const uint32_t* it_ptr, int32_t* it_slot, int32_t* it_off,
                      int pass, hipStream_t s);
void k_slot_levels(const MapCtx& m, const uint64_t* slot_ids, size_t n, uint8_t* lvl, hipStream_t s);
// the fixed-width face table of rows [0, nrows) (ensure_face); fine is
// allocated here; returns the number of finer faces
size_t k_face_table(const MapCtx& m, const DevMesh& M, const uint64_t* slot_ids, size_t nrows, size_t run1,
                    bool morton, int32_t* ell, DBuf<int32_t>& fine, int32_t* err, hipStream_t s);
// its CSR rows (ensure_face_csr)
void k_face_csr(const int32_t* ell, const int32_t* fine, size_t nrows, DBuf<uint32_t>& ptr, DBuf<int32_t>& ent,
                hipStream_t s);
void k_carry_src(const uint64_t* slot_ids, size_t n_slots, size_t nl, const MapCtx& m, const DevMesh& oldM,
                 size_t old_n_local, int32_t* src, hipStream_t s);
void k_gather_rows(const uint8_t* old_data, const int32_t* src, size_t n, size_t elem, uint8_t* out, hipStream_t s);
// ghost region: the level-0 cells within `radius` of the level-0 parent of a
// local cell that are not wholly owned here (sorted, unique)
std::vector<uint64_t> k_ghost_level0(const MapCtx& m, const DevMesh& M, int rank, const uint64_t* local, size_t n,
                                     int radius, hipStream_t s);
// local cells whose level-0 parent is in `l0` (sorted)
std::vector<uint64_t> k_cells_under(const MapCtx& m, const uint64_t* local, size_t n, const std::vector<uint64_t>& l0,
                                    hipStream_t s);
// refinement closure (induce_refines 9591-9720): coarser neighbors_of /
// neighbors_to entries of the requested local cells; finer: the finer ones
// (the dont_refine spread of override_refines 9991-10038)
std::vector<uint64_t> k_induced_refines(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh,
                                        const DevMesh& M, int rank, const std::vector<uint64_t>& req, hipStream_t s,
                                        bool finer = false, const uint64_t* dreq_given = nullptr);
// override_unrefines (9796-9898) on the device: the requested cells'
// parents (sorted, unique) whose families may merge given the final refine
// set S (sorted): none of the children refined or marked dont_unrefine (DU,
// sorted), and no finer leaf or refined same-level leaf in the parent's
// neighborhood (unrefine_check_kernel)
// (stop_refining's sets S and F are sorted host lists; dS / dF, when given,
// are their device copies, uploaded once by the caller)
std::vector<uint64_t> k_unrefine_families(const MapCtx& m, const int32_t* hood, int nh, const DevMesh& M,
                                          const std::vector<uint64_t>& req, const std::vector<uint64_t>& S,
                                          const std::vector<uint64_t>& DU, hipStream_t s,
                                          const uint64_t* dS = nullptr, const uint64_t* dreq_heads = nullptr);
// the children of the refined cells S owned by `rank`, ascending, into out;
// returns their count
size_t k_created_children(const MapCtx& m, const DevMesh& M, int rank, const std::vector<uint64_t>& S,
                          DBuf<uint64_t>& out, hipStream_t s, const uint64_t* dS = nullptr, bool sorted = true);
// the children of the merged families F staying on `rank` (owned here, like
// the family's first child), ascending, into ids with their slots; returns
// their count
// all_local: every child of every family is a local leaf (one process):
// ordered by ranks within octant streams instead of a sort
size_t k_kept_children(const MapCtx& m, const DevMesh& M, int rank, const std::vector<uint64_t>& F,
                       DBuf<uint64_t>& ids, DBuf<int32_t>& slots, hipStream_t s, const uint64_t* dF = nullptr,
                       bool all_local = false);
// known list after refining the sorted set S and merging the families under
// the sorted parents F: every known leaf in S is replaced by its 8 children
// (same owner), the children of a parent in F by the parent (owner of the
// first child)
void k_apply_refines(const MapCtx& m, const uint64_t* kid, const int32_t* kown, size_t n, const std::vector<uint64_t>& S,
                     const std::vector<uint64_t>& F, DBuf<uint64_t>& out_id, DBuf<int32_t>& out_own, size_t& n_out,
                     hipStream_t s, const size_t* at = nullptr, size_t* pos_at = nullptr, int n_at = 0,
                     size_t n_prefix = 0, const DevMesh* dm = nullptr, DBuf<int32_t>* src = nullptr,
                     const uint64_t* dS = nullptr, const uint64_t* dF = nullptr);

// --- launchers implemented in tile_build.hip --------------------------------
struct TileBuild {
	size_t n_tiles_inner = 0, n_tiles_outer = 0, max_ext = 0, total_ext = 0, n_fine = 0;
	// per tile: first ext entry (of ext_pk) and count, first finer face (of
	// tfine, 2 words each) and count
	std::vector<uint32_t> ext_off, ext_n, fine_off, fine_n;
};
TileBuild k_build_tiles(const uint32_t* face_ptr, const int32_t* face_ent, const uint64_t* slot_ids, const MapCtx& m,
                        bool morton, size_t n_inner, size_t n_local, int tile, DBuf<uint32_t>& tstart,
                        DBuf<uint32_t>& tell, DBuf<uint32_t>& ext_ptr, DBuf<uint32_t>& ext, DBuf<uint32_t>& ext_pk,
                        DBuf<uint32_t>& fine_base, DBuf<uint32_t>& tfine, hipStream_t s);

void k_classify_tiles(const MapCtx& m, const uint32_t* tstart, size_t n_tiles_inner, size_t n_tiles_outer,
                      const uint64_t* slot_ids, const int32_t* face_ell, DBuf<uint32_t>& lists, DBuf<int32_t>& tnb,
                      DBuf<RegTileMeta>& regmeta, size_t counts[4], hipStream_t s);

// --- launchers implemented in sweep_kernels.hip -----------------------------
// gather bytes [off, off + len) of the elements at `slots` into `out`
void k_pack(const uint8_t* field, size_t elem, size_t off, size_t len, const int32_t* slots, size_t n, uint8_t* out,
            hipStream_t s);
// scatter: inverse of k_pack
void k_place(const uint8_t* in, size_t elem, size_t off, size_t len, const int32_t* slots, size_t n, uint8_t* field,
             hipStream_t s);
void k_gol_csr(const uint32_t* state, uint32_t* out, const uint32_t* it_ptr, const int32_t* it_slot, size_t s0,
               size_t s1, hipStream_t s);
// uniform 26-point game of life on a box of nx x ny x nz cells stored in
// raster order; planes z = -1 and z = nz come from lo / hi (nullptr: outside)
bool k_gol_structured(const uint32_t* state, uint32_t* out, const uint64_t n[3], const int per[3], const uint32_t* lo,
                      const uint32_t* hi, hipStream_t s);
void k_advection(const double* const f[7], double* rho_out, const uint32_t* face_ptr, const int32_t* face_ent,
                 size_t s0, size_t s1, double dt, hipStream_t s);
// tiled advection sweep over the regular and the irregular tiles of one run
// (run 0 inner, 1 outer: tiles never straddle the two)
void k_advection_tiles(const double* const f[7], double* rho_out, Grid& g, int run, double dt, hipStream_t s,
                       const double* nbrec = nullptr);
// the neighbor records for the sweep of fields fids (rho vx vy vz lx ly lz),
// rebuilt when stale; nullptr when a velocity / length field is external
// (or DCCRGX_NBREC=0): the sweeps then read the fields
const double* ensure_nbrec(Grid& g, const int fids[7]);
void k_nbrec(const double* const f[7], size_t n, double* r, hipStream_t s);
// the bands of check_for_adaptation (adv_bands_kernel) written by the sweep
// as well, for rows [s0, s1) of `band`
struct BandArgs {
	MapCtx m;
	const uint8_t* lvl8;
	const uint64_t* slot_ids;
	double inc, thr, uns;
	uint8_t* band;
};
void k_advection_ell(const double* const f[7], double* rho_out, const int32_t* ell, const int32_t* fine, size_t s0,
                     size_t s1, double dt, hipStream_t s, const BandArgs* bands = nullptr);
void k_adv_dt(const double* const f[7], size_t n, double* partial, size_t nblocks, hipStream_t s);
void k_min_partials(const double* partial, size_t n, double* out, hipStream_t s);
size_t k_adv_candidates(const MapCtx& m, const double* rho, const FaceView& F, const uint8_t* lvl8, size_t n,
                        double diff_increase, double diff_threshold, uint64_t* out, hipStream_t s);
// adaptation of tests/advection/adapter.hpp: per local cell band (2 refine,
// 1 keep, 0 unrefine), merged parents' densities, velocity + length reset
// check_for_adaptation's requests computed on the device (sweep_kernels.hip
// adv_requests_kernel): refine ids, unrefine ids of whole local families,
// the number of kept whole families, and the partial runs (first slot,
// length, members' ids and bands) for the host to merge by parent
struct AdvRequests {
	std::vector<uint64_t> refine, unrefine;
	DBuf<uint64_t> refine_dev;  // `refine` on the device (sorted, unique)
	DBuf<uint64_t> unrefine_dev;  // `unrefine` on the device (sorted; one process: octant-0 heads)
	size_t kept = 0;
	std::vector<size_t> part_slot;
	std::vector<uint32_t> part_len;
	std::vector<uint64_t> part_ids;
	std::vector<uint8_t> part_bands;
};
AdvRequests k_adv_requests(const MapCtx& m, const DevMesh& dm, const uint64_t* slot_ids, const uint8_t* band, size_t n,
                           bool solo, int rank, hipStream_t s);
void k_adv_bands(const MapCtx& m, const double* rho, const FaceView& F, const uint8_t* lvl8, size_t n,
                 double diff_increase, double diff_threshold, double unrefine_sensitivity, uint8_t* band,
                 hipStream_t s);
// rm: the removed cells (on the device when it holds them, else uploaded)
// (parents, np: the merged parents on the device, sorted, when known - one
// process: exactly the removed cells' parents; used when 8 np removed cells)
void k_adv_merge_parents(const MapCtx& m, const DevMesh& dm, size_t n_local, LazyIds& rm, double* rho,
                         const double* removed_rho, hipStream_t s, const uint64_t* parents = nullptr, size_t np = 0);
void k_adv_parent_density(double* rho, const int32_t* parent_slot, const int32_t* child_idx, const double* removed_rho,
                          size_t np, hipStream_t s);
// (dt_partial: when given, the block minima of the time-step bound of the
// values written, as k_adv_dt computes them; returns their count)
constexpr unsigned kDtPartials = 2048;  // block minima a reset pass leaves at most
size_t k_adv_reset(const MapCtx& m, const uint64_t* slot_ids, size_t n, const double start[3], const double l0[3],
                   double* const f[7], hipStream_t s, double* dt_partial = nullptr);
void k_time_begin(Grid& g);
void k_time_end(Grid& g);

// --- variable-size fields (varfield.hip) ----------------------------------
uint64_t scan_exclusive_u64(const uint64_t* in, uint64_t* out, size_t n, hipStream_t s);  // returns total
void var_reset(Field& f, size_t n_slots, hipStream_t s);  // every slot empty
uint64_t var_total(const Field& f, size_t n_slots, hipStream_t s);
// sizes of slots[i] (slots != nullptr) or of slot0 + i, into out (device)
void var_sizes(const Field& f, const int32_t* slots, size_t slot0, size_t n, uint64_t* out, hipStream_t s);
// new sizes for every slot (device): each keeps its first min(old, new) bytes, the rest zero
void var_resize(Field& f, size_t n_slots, const uint64_t* new_sizes, hipStream_t s);
// the payloads of slots[0..n): sizes and concatenated bytes; returns the byte total
size_t var_gather(const Field& f, const int32_t* slots, size_t n, DBuf<uint64_t>& sizes, DBuf<uint8_t>& bytes,
                  hipStream_t s);
// payloads into slots[0..n) (sizes and concatenated bytes on the device); returns the byte total
uint64_t var_place(Field& f, size_t n_slots, const int32_t* slots, size_t n, const uint64_t* sizes,
                   const uint8_t* bytes, hipStream_t s);
// after a rebuild: cells that stayed local keep their payload, every other slot is empty
void var_remap(Field& f, const uint64_t* old_ids, size_t n_old_local, const DevMesh& newM, size_t new_n_slots,
               hipStream_t s);

// --- launchers implemented in gol_amr.hip ----------------------------------
// refined game of life (gol_amr.hip): per-mesh tables, then one phase
void k_gol_amr_tables(const MapCtx& m, const uint64_t* slot_ids, size_t n_slots, size_t n_local, unsigned hood_len,
                      const uint32_t* ptr, const int32_t* nslot, GolAmrTables& T, hipStream_t s);
// the geometric collect of one turn (gol_amr.hip): level-0 cell states from
// the known leaves, then every local row's live level-0 parents as a mask
// (lists written for rows >= list_from); err bits 1 (over 8), 4 (a family's
// leaves disagree) and 8 (a reached level-0 cell unknown): with 4 or 8 the
// caller runs the exact collect instead
void k_gol_amr_geo(GolAmrTables& T, const int32_t* hood, int nh, const uint32_t* state, size_t n_local, size_t n_state,
                   uint64_t* lst, size_t list_from, int* err, hipStream_t s);
void k_gol_amr_level0_game(GolAmrTables& T, const int32_t* hood, int nh, uint32_t* state, size_t n_local, int* err,
                           hipStream_t s);
void k_gol_amr(int phase, GolAmrTables& T, size_t n_slots, size_t n_local, uint32_t* state, uint64_t* lst, const uint32_t* ptr,
               const int32_t* nslot, size_t s0, size_t s1, int* err, hipStream_t s, size_t list_from = 0,
               const int* gate = nullptr);

// --- launchers implemented in poisson_kernels.hip ---------------------------
unsigned k_po_blocks(size_t n);  // blocks (= partials) of a phase launch over n slots
void k_po_transpose(const PoArrays& a, size_t n, double* ft, hipStream_t s);
void k_po_cache(const MapCtx& m, const double l0[3], const uint64_t* slot_ids, const int32_t* cls,
                const int32_t* face_ell, const int32_t* face_fine, size_t n, int32_t* po_ell, int32_t* po_fine,
                int32_t* type, const PoArrays& a, hipStream_t s);
void k_po_phase(int phase, const PoArrays& a, size_t n, const PoParams& prm, const PoScalars* st, double* part,
                hipStream_t s);
void k_po_reduce(int k, const double* part, unsigned nb, double* red, PoScalars* st, const PoParams& prm, int stage,
                 bool scalar, hipStream_t s);
// all: P x k all-gathered per-rank sums, combined in rank order
void k_po_scalar(const double* all, int P, int k, PoScalars* st, const PoParams& prm, int stage, hipStream_t s);

}  // namespace dccrgx

#if DCCRGX_PHASE_TIMING
// the analysis build counts the library's stream syncs (PhaseLaps "<lap>.syncs")
namespace dccrgx {
inline hipError_t dx_counted_stream_sync(hipStream_t s) {
	phase_sync_count()++;
	return (hipStreamSynchronize)(s);
}
}  // namespace dccrgx
#define hipStreamSynchronize(s) ::dccrgx::dx_counted_stream_sync(s)
#endif
