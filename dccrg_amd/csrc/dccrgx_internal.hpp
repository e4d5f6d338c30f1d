// Internal state of one dccrgx grid (one per process / GPU).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dccrgx.h"
#include "dccrgx_mapping.hpp"
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

// Owning device buffer.
template <class T>
struct DBuf {
	T* p = nullptr;
	size_t n = 0;
	DBuf() = default;
	DBuf(const DBuf&) = delete;
	DBuf& operator=(const DBuf&) = delete;
	DBuf(DBuf&& o) noexcept : p(o.p), n(o.n) {
		o.p = nullptr;
		o.n = 0;
	}
	DBuf& operator=(DBuf&& o) noexcept {
		if (this != &o) {
			release();
			p = o.p;
			n = o.n;
			o.p = nullptr;
			o.n = 0;
		}
		return *this;
	}
	~DBuf() { release(); }
	void release() {
		if (p) (void)hipFree(p);
		p = nullptr;
		n = 0;
	}
	void alloc(size_t count) {
		if (count == n && p) return;
		release();
		if (count) HIP_CHECK(hipMalloc(&p, count * sizeof(T)));
		n = count;
	}
	void swap(DBuf& o) {
		std::swap(p, o.p);
		std::swap(n, o.n);
	}
};

template <class T>
inline void upload(DBuf<T>& d, const std::vector<T>& h, hipStream_t s) {
	d.alloc(h.size());
	if (!h.empty()) HIP_CHECK(hipMemcpyAsync(d.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
}

template <class T>
inline std::vector<T> download(const T* d, size_t n, hipStream_t s) {
	std::vector<T> h(n);
	if (n) {
		HIP_CHECK(hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
	}
	return h;
}

struct Field {
	std::string name;
	size_t elem = 0;
	bool transfer = false;
	DBuf<uint8_t> data;     // n_slots * elem
	DBuf<uint8_t> scratch;  // double buffer for sweeps (allocated on demand)
};

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
	DBuf<double> part, red;
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

// A user neighborhood (add_neighborhood, dccrg.hpp:6383-6520): its offsets,
// neighbors_of / neighbors_to CSR of the local cells (built lazily after
// every structural change, update_user_neighbors 8974-8980) and its
// per-peer send / receive lists (recalculate_neighbor_update_send_receive_lists
// for the id, 8590-8752), with their slots for the halo over this hood only.
struct UserHood {
	std::vector<int32_t> of, to;  // 3 per item; to = -of
	DBuf<int32_t> d_of, d_to;
	bool valid = false;
	DBuf<uint32_t> nof_ptr, nto_ptr;
	DBuf<uint64_t> nof_id, nto_id;
	DBuf<int32_t> nof_off;
	std::map<int, std::vector<uint64_t>> send_ids, recv_ids;
	std::map<int, size_t> send_off, recv_off;
	size_t n_send = 0, n_recv = 0;
	DBuf<int32_t> send_slots, recv_slots;
	DBuf<uint8_t> sendbuf, recvbuf;
};

struct Grid {
	// communicator
	int rank = 0, size = 1, device = 0;
	ncclComm_t comm = nullptr;
	hipStream_t s_comp = nullptr, s_comm = nullptr;
	hipEvent_t ev_comp = nullptr, ev_halo = nullptr;
	bool halo_in_flight = false;

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

	// global leaves (like cell_process, dccrg.hpp:7197): sorted ids + owners
	std::vector<uint64_t> leaves;
	std::vector<int32_t> owners;
	std::unordered_map<uint64_t, int> pins;
	std::vector<uint64_t> refine_requests;
	std::vector<uint64_t> last_new_cells;  // local cells created by the last stop_refining

	// local layout
	size_t n_inner = 0, n_outer = 0, n_local = 0, n_recv = 0, n_slots = 0;
	std::vector<int> peers;                                     // union of send/recv peers, ascending
	std::map<int, std::vector<uint64_t>> send_ids, recv_ids;    // ascending ids per peer
	std::map<int, size_t> recv_slot0;                           // first halo slot per peer
	std::map<int, size_t> send_off;                             // offset into send_slots per peer
	size_t n_send_total = 0;
	std::vector<uint64_t> extra_remote;                         // remote neighbors_to-only cells
	std::vector<uint64_t> slot_ids_h;                           // host mirror of slot -> id
	bool slot_ids_h_valid = false;

	// device structures
	DBuf<int32_t> owner_by_id;  // last_cell + 1 entries, -1 = not a leaf
	DBuf<int32_t> slot_by_id;   // last_cell + 1 entries, -1 = no slot on this rank
	DBuf<uint64_t> slot_ids;    // n_slots
	DBuf<int32_t> d_hood, d_hood_to;
	// full CSR (built lazily): neighbors_of (stencil order), neighbors_to (ascending)
	bool csr_valid = false;
	DBuf<uint32_t> nof_ptr, nto_ptr, it_ptr;
	DBuf<uint64_t> nof_id, nto_id;
	DBuf<int32_t> nof_off, nof_slot, it_slot;
	// face CSR (built lazily): entry = slot * 8 + dir (dir 0..5 = -x,+x,-y,+y,-z,+z)
	bool face_valid = false;
	DBuf<uint32_t> face_ptr;
	DBuf<int32_t> face_ent;
	DBuf<int32_t> face_ell, face_fine;  // fixed-width form used by the advection sweep
	size_t n_fine_faces = 0;
	// face tiles (built lazily from the face CSR): the inner and the outer run
	// of slots are cut into tiles of at most `tile` consecutive slots
	// (boundaries `tstart`, on aligned Morton boxes where possible); per tile the
	// distinct out-of-tile face neighbors (`ext`, ascending slot) and per cell
	// six 16-bit tile-local neighbor indices (< tile: a slot of the tile,
	// tile + k: ext[k] of the tile, 0x8000 | j: finer face j of the tile whose
	// four tile-local indices are in `tfine`, 0xffff: no face neighbor)
	bool tiles_valid = false;
	int tile = 0;
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
	// the pipelined kernel's capacities (> 1024 ext cells or > 512 finer faces)
	DBuf<uint32_t> tmeta;
	// per tile (all tiles, slot order), 16 u32: ts, n, e0, ne, fb, nf,
	// nst[6] (regular: neighbor-box starts), kind (1 regular), pad; for the
	// fused sweep over both kinds (empty when a tile exceeds its limits)
	DBuf<uint32_t> tfmeta;
	// work tickets of the persistent advection kernels: [kernel (0 regular,
	// 1 general)][set][XCD][32] (one 128-B line per counter); a launch draws
	// from set adv_par[kernel] and
	// zeroes the other set for the next launch of that kernel
	DBuf<uint32_t> adv_ctr;
	uint32_t adv_par[2] = {0, 0};
	// second compute stream: the general-tile sweep runs beside the regular one
	hipStream_t s_adv2 = nullptr;
	hipEvent_t ev_fork = nullptr, ev_join = nullptr;
	std::map<int, UserHood> uhoods;  // add_neighborhood ids
	DBuf<uint64_t> gol_l0p;  // refined game of life: level-0 parent per slot (scratch)
	// halo
	DBuf<int32_t> send_slots;
	DBuf<uint8_t> sendbuf;

	std::vector<Field> fields;

	// timing of sweep kernels (HIP events on s_comp)
	bool timing = false;
	double timed_ms = 0;
	int64_t timed_count = 0;
	std::vector<std::pair<hipEvent_t, hipEvent_t>> pending_events;

	// slot order inside the inner and outer runs: 0 = ascending id (raster,
	// needed by the structured uniform kernels), 1 = Morton order of the min
	// corners (locality for refined meshes)
	int slot_order = -1;  // -1: Morton when R > 0, else id
	bool morton_slots = false;  // the order in effect

	PoissonState po;

	bool uniform() const { return R == 0; }
};

// --- launchers implemented in build_kernels.hip -----------------------------
void k_fill_i32(int32_t* p, size_t n, int32_t v, hipStream_t s);
void k_scatter_owner(int32_t* owner_by_id, const uint64_t* ids, const int32_t* owners, size_t n, hipStream_t s);
void k_scatter_slots(int32_t* slot_by_id, const uint64_t* slot_ids, size_t n, hipStream_t s);
// flag local cells that have a remote neighbors_of / neighbors_to entry
void k_remote_flags(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                    int rank, const uint64_t* cells, size_t n, uint32_t* flag, hipStream_t s);
// local ids -> slots: inner first, outer second, both ascending
void k_assign_slots2(const uint32_t* flag, const uint32_t* scan_outer, size_t n, size_t n_inner, const uint64_t* cells,
                     uint64_t* slot_ids, hipStream_t s);
void k_fill_neighbors_of(const MapCtx& m, const int32_t* hood, int nh, const int32_t* owner_by_id,
                         const uint64_t* slot_ids, size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids,
                         int32_t* offs, hipStream_t s);
void k_fill_neighbors_to(const MapCtx& m, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                         const uint64_t* slot_ids, size_t row0, size_t nrows, const uint32_t* ptr, uint64_t* ids,
                         hipStream_t s);
void k_count_rows(const MapCtx& m, const int32_t* hood, const int32_t* hood_to, int nh, const int32_t* owner_by_id,
                  const uint64_t* slot_ids, size_t row0, size_t nrows, uint32_t* nof_cnt, uint32_t* nto_cnt,
                  hipStream_t s);
// remote (owner != rank) entries of an id array as composite keys owner*(last+1)+id
size_t k_extract_remote(const uint64_t* ids, size_t n, const int32_t* owner_by_id, int rank, uint64_t stride,
                        uint64_t* keys_out, hipStream_t s);
// keys for the send side: for each neighbors_to entry with a remote owner,
// owner*(last+1) + the row's own id
size_t k_extract_send(const uint64_t* nto_id, const uint32_t* nto_ptr, const uint64_t* slot_ids, size_t row0,
                      size_t nrows, const int32_t* owner_by_id, int rank, uint64_t stride, uint64_t* keys_out,
                      hipStream_t s);
size_t sort_unique_u64(uint64_t* keys, size_t n, hipStream_t s);  // in place
void k_morton_sort(const MapCtx& m, uint64_t* ids, size_t n, hipStream_t s);
size_t k_face_ell(const uint32_t* ptr, const int32_t* ent, size_t nrows, int32_t* ell, int32_t* fine, hipStream_t s);
uint32_t scan_exclusive_u32(const uint32_t* in, uint32_t* out, size_t n, hipStream_t s);  // returns total
void k_lookup_slots(const uint64_t* ids, size_t n, const int32_t* slot_by_id, int32_t* out, int32_t* err_flag,
                    hipStream_t s);
void k_iterator_lists(const uint32_t* nof_ptr, const uint64_t* nof_id, const int32_t* nof_off,
                      const int32_t* nof_slot, size_t nrows, uint32_t* it_cnt, const uint32_t* it_ptr,
                      int32_t* it_slot, int pass, hipStream_t s);
void k_face_lists(const MapCtx& m, const int32_t* owner_by_id, const int32_t* slot_by_id, const uint64_t* slot_ids,
                  size_t nrows, uint32_t* cnt, const uint32_t* ptr, int32_t* ent, int32_t* err_flag, int pass,
                  hipStream_t s);
void k_remap_field2(const uint8_t* old_data, const uint64_t* old_ids, size_t n_old, const int32_t* new_slot_by_id,
                    uint64_t last, uint8_t* new_data, size_t elem, hipStream_t s);
void k_parent_fill(uint8_t* data, const uint64_t* slot_ids, size_t n, const int32_t* slot_by_id, const MapCtx& m,
                   const uint8_t* old_data, const int32_t* old_slot_by_id, size_t elem, hipStream_t s);

// --- launchers implemented in tile_build.hip --------------------------------
struct TileBuild {
	size_t n_tiles_inner, n_tiles_outer, max_ext, total_ext, n_fine;
};
TileBuild k_build_tiles(const uint32_t* face_ptr, const int32_t* face_ent, const uint64_t* slot_ids, const MapCtx& m,
                        bool morton, size_t n_inner, size_t n_local, int tile, DBuf<uint32_t>& tstart,
                        DBuf<uint32_t>& tell, DBuf<uint32_t>& ext_ptr, DBuf<uint32_t>& ext, DBuf<uint32_t>& ext_pk,
                        DBuf<uint32_t>& fine_base, DBuf<uint32_t>& tfine, hipStream_t s);

void k_classify_tiles(const MapCtx& m, const uint32_t* tstart, size_t n_tiles_inner, size_t n_tiles_outer,
                      const uint64_t* slot_ids, const int32_t* face_ell, DBuf<uint32_t>& lists, DBuf<int32_t>& tnb,
                      DBuf<RegTileMeta>& regmeta, size_t counts[4], hipStream_t s);

// --- launchers implemented in sweep_kernels.hip -----------------------------
void k_pack(const uint8_t* field, size_t elem, const int32_t* slots, size_t n, uint8_t* out, hipStream_t s);
void k_gol_csr(const uint32_t* state, uint32_t* out, const uint32_t* it_ptr, const int32_t* it_slot, size_t s0,
               size_t s1, hipStream_t s);
void k_gol_structured(const uint32_t* state, uint32_t* out, const uint64_t n[3], const int per[3], hipStream_t s);
void k_advection(const double* const f[7], double* rho_out, const uint32_t* face_ptr, const int32_t* face_ent,
                 const int32_t* face_ell, const int32_t* face_fine, size_t s0, size_t s1, double dt, hipStream_t s);
// tiled advection sweep over the regular and the irregular tiles of one run
// (run 0 inner, 1 outer: tiles never straddle the two)
void k_advection_tiles(const double* const f[7], double* rho_out, Grid& g, int run, double dt, hipStream_t s);
int adv_variant();  // DCCRGX_ADV_VARIANT (11 = tiled, the default)
void k_adv_dt(const double* const f[7], size_t n, double* partial, size_t nblocks, hipStream_t s);
size_t k_adv_candidates(const MapCtx& m, const double* rho, const uint32_t* face_ptr, const int32_t* face_ent,
                        const uint64_t* slot_ids, size_t n, double diff_increase, double diff_threshold,
                        uint64_t* out, hipStream_t s);
void k_time_begin(Grid& g);
void k_time_end(Grid& g);

// --- launchers implemented in gol_amr.hip ----------------------------------
void k_gol_amr(int phase, const MapCtx& m, const uint64_t* slot_ids, size_t n_slots, uint64_t* l0p, uint32_t* state,
               uint64_t* lst, const uint32_t* ptr, const int32_t* nslot, size_t s0, size_t s1, int* err,
               hipStream_t s);

// --- launchers implemented in poisson_kernels.hip ---------------------------
unsigned k_po_blocks(size_t n);  // blocks (= partials) of a phase launch over n slots
void k_po_cache(const MapCtx& m, const double l0[3], const uint64_t* slot_ids, const int32_t* cls,
                const int32_t* face_ell, const int32_t* face_fine, size_t n, int32_t* po_ell, int32_t* po_fine,
                int32_t* type, const PoArrays& a, hipStream_t s);
void k_po_phase(int phase, const PoArrays& a, size_t n, const PoParams& prm, const PoScalars* st, double* part,
                hipStream_t s);
void k_po_reduce(int k, const double* part, unsigned nb, double* red, PoScalars* st, const PoParams& prm, int stage,
                 bool scalar, hipStream_t s);
void k_po_scalar(const double* red, PoScalars* st, const PoParams& prm, int stage, hipStream_t s);

}  // namespace dccrgx
