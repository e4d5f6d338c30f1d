// dccrgx C ABI (include/dccrgx.h): every entry point wraps the host driver
// in an exception guard and returns a status code.
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <numeric>

#include <fcntl.h>
#include <unistd.h>

#include "dccrgx_grid.hpp"

namespace dccrgx {

static thread_local std::string g_last_error;

template <class F>
static int guard(F&& f) {
	try {
		return f();
	} catch (const Error& e) {
		g_last_error = e.what();
		return e.code;
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return DCCRGX_EINVAL;
	}
}

static int copy_out_u64(const std::vector<uint64_t>& v, uint64_t* out, size_t cap, size_t* n) {
	if (n) *n = v.size();
	if (v.size() > cap || (!out && !v.empty())) return DCCRGX_ERANGE;
	if (!v.empty()) std::memcpy(out, v.data(), v.size() * 8);
	return DCCRGX_OK;
}

// dccrg_mapping.hpp:316-329: the largest level whose ids fit in 64 bits
static int max_possible_level(const uint64_t len[3]) {
	const double gl = double(len[0]) * double(len[1]) * double(len[2]);
	int lvl = 0;
	double cur = 0;
	while (cur <= double(~uint64_t(0))) {
		cur += gl * std::pow(8.0, double(lvl));
		lvl++;
	}
	return lvl - 2;
}

// the largest neighborhood length whose neighbors_to dedupe fits in LDS
static unsigned max_hood_length() {
	unsigned L = 0;
	while (true) {
		const unsigned n = (2 * (L + 1) + 1) * (2 * (L + 1) + 1) * (2 * (L + 1) + 1) - 1;
		if (int(n) > max_hood_items()) return L;
		L++;
	}
}

static void init_impl(Grid& g) {
	DX_REQUIRE(!g.initialized, "already initialized");
	map_init(g.m, g.len, g.R, g.per);
	const unsigned L = g.hood_len;
	const size_t cube = size_t(2 * L + 1) * (2 * L + 1) * (2 * L + 1);
	std::vector<int32_t> h(3 * std::max<size_t>(cube, 6));
	const int nh = default_hood(g.hood_len, h.data());
	g.hood.assign(h.begin(), h.begin() + 3 * nh);
	g.hood_to.resize(g.hood.size());
	for (size_t i = 0; i < g.hood.size(); i++) g.hood_to[i] = -g.hood[i];
	upload(g.d_hood, g.hood, g.s_comp);
	upload(g.d_hood_to, g.hood_to, g.s_comp);
	Mesh nm;
	nm.implicit = true;
	nm.bp.init(g.m.first[1] - 1, uint64_t(g.size));
	rebuild(g, nm);
	g.initialized = true;
}

// --------------------------------------------------------------------------- Poisson
// Poisson_Solve (tests/poisson/poisson_solve.hpp:156-1056) over device fields.

// halo update of exactly the given fields (the reference's
// Poisson_Cell::transfer_switch, 92-140)
static void halo_only(Grid& g, const std::vector<int>& fids) {
	if (g.size == 1 || g.peers.empty()) return;
	std::vector<char> saved(g.fields.size());
	for (size_t i = 0; i < g.fields.size(); i++) {
		saved[i] = g.fields[i].transfer;
		g.fields[i].transfer = false;
	}
	for (int f : fids) field(g, f).transfer = true;
	try {
		halo_start(g);
	} catch (...) {
		for (size_t i = 0; i < g.fields.size(); i++) g.fields[i].transfer = saved[i];
		throw;
	}
	for (size_t i = 0; i < g.fields.size(); i++) g.fields[i].transfer = saved[i];
	halo_wait(g);
}

__global__ void po_classify_kernel(int32_t* cls, DevMesh M, const uint64_t* ids, size_t n, size_t n_local,
                                   int32_t value) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		const int32_t sl = dm_slot(M, ids[i]);
		if (sl >= 0 && size_t(sl) < n_local) cls[sl] = value;  // only local cells (is_local, 839-878)
	}
}

static int po_field(Grid& g, const char* name, size_t elem) {
	Field f;
	f.name = name;
	f.elem = elem;
	f.win_len = elem;
	f.transfer = false;
	g.fields.push_back(std::move(f));
	Field& nf = g.fields.back();
	nf.data.alloc(g.n_slots * elem);
	if (nf.data.n) HIP_CHECK(hipMemsetAsync(nf.data.p, 0, nf.data.n, g.s_comp));
	return int(g.fields.size() - 1);
}

static void po_ensure_fields(Grid& g) {
	PoissonState& P = g.po;
	if (P.type >= 0) return;
	P.type = po_field(g, "poisson.type", 4);
	P.p0 = po_field(g, "poisson.p0", 8);
	P.p1 = po_field(g, "poisson.p1", 8);
	P.r0 = po_field(g, "poisson.r0", 8);
	P.r1 = po_field(g, "poisson.r1", 8);
	P.ap0 = po_field(g, "poisson.A_dot_p0", 8);
	P.best = po_field(g, "poisson.best_solution", 8);
	P.sf = po_field(g, "poisson.scaling_factor", 8);
	static const char* fn[6] = {"poisson.f_x_neg", "poisson.f_x_pos", "poisson.f_y_neg",
	                            "poisson.f_y_pos", "poisson.f_z_neg", "poisson.f_z_pos"};
	for (int k = 0; k < 6; k++) P.f[k] = po_field(g, fn[k], 8);
}

static PoArrays po_arrays(Grid& g) {
	PoissonState& P = g.po;
	auto d = [&](int f) { return (double*)field(g, f).data.p; };
	PoArrays a{};
	a.ell = P.ell.p;
	a.fine = P.fine.p;
	a.type = (const int32_t*)field(g, P.type).data.p;
	a.rhs = d(P.rhs);
	a.sol = d(P.sol);
	a.best = d(P.best);
	a.p0 = d(P.p0);
	a.p1 = d(P.p1);
	a.r0 = d(P.r0);
	a.r1 = d(P.r1);
	a.ap0 = d(P.ap0);
	a.sf = d(P.sf);
	for (int k = 0; k < 6; k++) a.f[k] = d(P.f[k]);
	a.ft = P.valid && P.ft.p ? P.ft.p : nullptr;
	return a;
}

// the fields a solve or a cache pass writes: the solution and the solver's own
static void po_written(Grid& g) {
	const PoissonState& P = g.po;
	for (int id : {P.sol, P.type, P.best, P.p0, P.p1, P.r0, P.r1, P.ap0, P.sf})
		if (id >= 0 && size_t(id) < g.fields.size()) field_written(g.fields[size_t(id)]);
	for (int k = 0; k < 6; k++)
		if (P.f[k] >= 0 && size_t(P.f[k]) < g.fields.size()) field_written(g.fields[size_t(P.f[k])]);
}

// cache_system_info 827-971
static void po_cache(Grid& g, int rhs, int sol, const uint64_t* solve, size_t ns, const uint64_t* skip, size_t nk) {
	DX_REQUIRE(field(g, rhs).elem == 8 && field(g, sol).elem == 8, "rhs and solution must be fp64 fields");
	po_ensure_fields(g);
	PoissonState& P = g.po;
	P.rhs = rhs;
	P.sol = sol;
	po_written(g);
	ensure_face(g);
	hipStream_t s = g.s_comp;
	const size_t nl = g.n_local;
	int32_t* type = (int32_t*)field(g, P.type).data.p;
	// classify: local cells boundary, then skip, then solve (836-878)
	k_fill_i32(type, nl, 1, s);
	for (int pass = 0; pass < 2; pass++) {
		const uint64_t* ids = pass == 0 ? skip : solve;
		const size_t n = pass == 0 ? nk : ns;
		if (!n) continue;
		DBuf<uint64_t> d;
		d.alloc(n);
		h2d(d.p, ids, n * 8, s);
		po_classify_kernel<<<grid_for(n, 256), 256, 0, s>>>(type, g.dm(), d.p, n, nl, pass == 0 ? 2 : 0);
		HIP_CHECK(hipGetLastError());
		HIP_CHECK(hipStreamSynchronize(s));
	}
	halo_only(g, {P.type});  // TYPE (880-881)
	DBuf<int32_t> cls;
	cls.alloc(g.n_slots + 1);
	if (g.n_slots) HIP_CHECK(hipMemcpyAsync(cls.p, type, g.n_slots * 4, hipMemcpyDeviceToDevice, s));
	P.ell.alloc(6 * nl + 6);
	P.fine.alloc(g.face_fine.n);
	const PoArrays a = po_arrays(g);
	k_po_cache(g.m, g.l0, g.slot_ids.p, cls.p, g.face_ell.p, g.face_fine.p, nl, P.ell.p, P.fine.p, type, a, s);
	HIP_CHECK(hipStreamSynchronize(s));
	std::vector<int> geo{P.sf};  // GEOMETRY (969-970)
	for (int k = 0; k < 6; k++) geo.push_back(P.f[k]);
	halo_only(g, geo);
	// the neighbors' factors toward each cell, once per cache pass (phase B
	// reads them coalesced instead of gathering them every iteration;
	// DCCRGX_PO_FT=0 keeps the gathers)
	const char* ftv = std::getenv("DCCRGX_PO_FT");
	if (!(ftv && ftv[0] == '0') && nl) {
		P.ft.alloc(6 * nl);
		k_po_transpose(po_arrays(g), nl, P.ft.p, s);
	} else {
		P.ft.release();
	}
	HIP_CHECK(hipStreamSynchronize(s));
	P.valid = true;
}

// sums of the last phase -> (all ranks) -> scalar control flow
static void po_reduce(Grid& g, int k, unsigned nb, const PoParams& prm, int stage) {
	PoissonState& P = g.po;
	const bool one = g.size == 1;
	k_po_reduce(k, P.part.p, nb, P.red.p, P.st.p, prm, stage, one, g.s_comp);
	if (one) return;
	// MPI_Allreduce SUM (poisson_solve.hpp:349, 486, 684): the ranks' sums
	// all-gathered and added in rank order on every rank (the same result
	// over RCCL and the host exchange)
	comm_require(g, "Poisson solve");
	P.gath.reserve(size_t(g.size) * 2);
	comm_allgather_dev(g, P.red.p, size_t(k) * 8, reinterpret_cast<uint8_t*>(P.gath.p), g.s_comp);
	k_po_scalar(P.gath.p, g.size, k, P.st.p, prm, stage, g.s_comp);
}

static PoScalars po_read_scalars(Grid& g) {
	PoScalars h{};
	d2h_small(&h, g.po.st.p, sizeof(h), g.s_comp);
	return h;
}

// solve 251-522 / solve_failsafe 531-634 after po_cache; the host only
// enqueues kernels and polls the device's `done` flag every few iterations.
// Timed (dccrgx_kernel_timing): from the first phase of an iteration to its
// last, the reductions included, the halo excluded.
static PoScalars po_solve(Grid& g, const PoParams& prm, bool failsafe) {
	PoissonState& P = g.po;
	DX_REQUIRE(P.valid, "Poisson system not cached for the current mesh");
	po_written(g);
	hipStream_t s = g.s_comp;
	const size_t n = g.n_local;
	const unsigned nb = k_po_blocks(n);
	if (P.part.n < 2 * size_t(nb)) P.part.alloc(2 * size_t(nb));
	P.red.alloc(2);
	P.st.alloc(1);
	const PoArrays a = po_arrays(g);
	const int poll = 8;
	if (!failsafe) {
		halo_only(g, {P.sol});  // INIT (983-984)
		k_po_phase(PO_PHASE_INIT, a, n, prm, P.st.p, P.part.p, s);
		po_reduce(g, 1, nb, prm, PO_STAGE_INIT);
		for (unsigned it = 0; it < prm.max_it; it++) {
			halo_only(g, {P.p0, P.p1});  // SOLVING (283-284)
			k_time_begin(g);
			k_po_phase(PO_PHASE_A, a, n, prm, P.st.p, P.part.p, s);
			po_reduce(g, 2, nb, prm, PO_STAGE_A);
			k_po_phase(PO_PHASE_B, a, n, prm, P.st.p, P.part.p, s);
			po_reduce(g, 1, nb, prm, PO_STAGE_B);
			k_po_phase(PO_PHASE_C, a, n, prm, P.st.p, P.part.p, s);
			k_time_end(g);
			if ((it + 1) % poll == 0 && po_read_scalars(g).done) break;
		}
		k_po_phase(PO_PHASE_FINISH, a, n, prm, P.st.p, P.part.p, s);
	} else {
		k_po_reduce(1, P.part.p, 0, P.red.p, P.st.p, prm, PO_STAGE_JACOBI_INIT, true, s);
		for (unsigned it = 0; it < prm.max_it; it++) {
			halo_only(g, {P.sol});  // INIT (545, 551)
			k_time_begin(g);
			k_po_phase(PO_PHASE_JACOBI, a, n, prm, P.st.p, P.part.p, s);
			po_reduce(g, 1, nb, prm, PO_STAGE_JACOBI);
			k_po_phase(PO_PHASE_JACOBI_COPY, a, n, prm, P.st.p, P.part.p, s);
			k_time_end(g);
			if ((it + 1) % poll == 0 && po_read_scalars(g).done) break;
		}
	}
	return po_read_scalars(g);
}

// --------------------------------------------------------------------------- grid files
// save_grid_data / load_grid_data (dccrg.hpp:1089-1740, 1742-2425), file
// layout 1104-1120: `offset` bytes left alone, the caller's header, uint64
// 0x1234567890abcdef, the grid block (Mapping::write dccrg_mapping.hpp:576 =
// 3 x uint64 length + int max_ref_lvl; the neighborhood length as unsigned;
// Grid_Topology::write dccrg_topology.hpp:144 = 3 x uint8 periodic;
// Cartesian_Geometry::write dccrg_cartesian_geometry.hpp:618 = int id 1 +
// 3 x double start + 3 x double level-0 length), uint64 total cells, per
// cell (uint64 id, uint64 absolute byte offset of its data) rank by rank,
// then the cell data in the same order.  A cell's data = the payload of
// every transferred field, in field order (the reference writes what
// get_mpi_datatype describes at save time: a fixed-size field's window, a
// variable-size field's bytes of the cell).  Cells of a rank in ascending id
// (the reference: get_cells() order).  Every rank writes its own records with
// pwrite at offsets derived from the all-gathered per-rank cell counts.
static constexpr uint64_t kEndianCheck = 0x1234567890abcdefULL;
static constexpr int kCartesianGeometryId = 1;
static constexpr int kStretchedGeometryId = 2;

// bytes of a Stretched_Cartesian_Geometry block (write 652-715: int id 2, 3 x
// uint64 coordinate counts, then each dimension's coordinates as doubles)
// given its first 28 bytes; 0 when they are no such block
static size_t stretched_block_bytes(const uint8_t* head) {
	int32_t id = 0;
	uint64_t cnt[3];
	std::memcpy(&id, head, 4);
	std::memcpy(cnt, head + 4, 24);
	if (id != kStretchedGeometryId) return 0;
	uint64_t tot = 0;
	for (int d = 0; d < 3; d++) {
		if (cnt[d] < 2 || cnt[d] > (uint64_t(1) << 40)) return 0;  // the reference's set() needs two per dimension
		tot += cnt[d];
	}
	return 28 + size_t(8 * tot);
}

static std::vector<uint8_t> grid_block(const Grid& g) {
	std::vector<uint8_t> b;
	auto put = [&b](const void* p, size_t n) {
		const uint8_t* q = static_cast<const uint8_t*>(p);
		b.insert(b.end(), q, q + n);
	};
	put(g.len, 24);
	const int32_t R = g.R;
	put(&R, 4);
	const uint32_t hood = g.hood_len;
	put(&hood, 4);
	const uint8_t per[3] = {uint8_t(g.per[0] != 0), uint8_t(g.per[1] != 0), uint8_t(g.per[2] != 0)};
	put(per, 3);
	if (!g.geo_block.empty()) {
		put(g.geo_block.data(), g.geo_block.size());  // the stretched geometry's block
		return b;
	}
	const int32_t gid = kCartesianGeometryId;
	put(&gid, 4);
	put(g.start, 24);
	put(g.l0, 24);
	return b;
}

static void pwrite_all(int fd, const void* p, size_t n, uint64_t off) {
	const uint8_t* q = static_cast<const uint8_t*>(p);
	while (n) {
		const ssize_t w = ::pwrite(fd, q, n, off_t(off));
		DX_REQUIRE(w > 0, "grid file write failed");
		q += w;
		n -= size_t(w);
		off += uint64_t(w);
	}
}

static void pread_all(int fd, void* p, size_t n, uint64_t off) {
	uint8_t* q = static_cast<uint8_t*>(p);
	while (n) {
		const ssize_t r = ::pread(fd, q, n, off_t(off));
		DX_REQUIRE(r > 0, "grid file truncated");
		q += r;
		n -= size_t(r);
		off += uint64_t(r);
	}
}

struct Closer {
	int fd;
	~Closer() { ::close(fd); }
};

// The bytes a field adds to one cell's record: a fixed-size field the window
// its get_mpi_datatype describes (the whole element by default), a
// variable-size field the cell's own bytes (save_grid_data writes what each
// cell's datatype describes, 1521-1540; padding is not written, 1529).
static void save_grid_impl(Grid& g, const char* path, uint64_t offset, const void* header, size_t header_bytes) {
	DX_REQUIRE(g.initialized, "not initialized");
	const std::vector<Field*> tf = transfer_fields(g);
	const size_t nl = g.n_local;
	// the local slots' payloads on the host, and each cell's record length
	std::vector<std::vector<uint8_t>> host(tf.size());
	std::vector<std::vector<uint64_t>> voff(tf.size());
	std::vector<uint64_t> rec(nl, 0);
	for (size_t k = 0; k < tf.size(); k++) {
		const Field* f = tf[k];
		if (f->var) {
			voff[k] = download(f->voff.p, nl + 1, g.s_comp);
			host[k] = download(f->data.p + voff[k][0], voff[k][nl] - voff[k][0], g.s_comp);
			for (size_t s = 0; s < nl; s++) rec[s] += voff[k][s + 1] - voff[k][s];
		} else {
			host[k] = download(f->data.p, nl * f->elem, g.s_comp);
			for (size_t s = 0; s < nl; s++) rec[s] += f->win_len;
		}
	}
	const uint64_t mine = std::accumulate(rec.begin(), rec.end(), uint64_t(0));
	const auto cnt = comm_allgather_u64(g, {uint64_t(nl), mine});
	uint64_t total = 0, before = 0, bytes_before = 0, bytes_total = 0;
	for (int p = 0; p < g.size; p++) {
		const auto& c = cnt[size_t(p)];
		DX_REQUIRE(c.size() == 2, "grid file: inconsistent cell counts");
		if (p < g.rank) {
			before += c[0];
			bytes_before += c[1];
		}
		total += c[0];
		bytes_total += c[1];
	}
	const int fd = ::open(path, O_CREAT | O_WRONLY, 0644);
	DX_REQUIRE(fd >= 0, std::string("cannot open grid file ") + path);
	Closer closer{fd};
	uint64_t off = offset;
	if (g.rank == 0 && header_bytes) pwrite_all(fd, header, header_bytes, off);
	off += header_bytes;
	if (g.rank == 0) pwrite_all(fd, &kEndianCheck, 8, off);
	off += 8;
	const std::vector<uint8_t> block = grid_block(g);
	if (g.rank == 0) pwrite_all(fd, block.data(), block.size(), off);
	off += block.size();
	if (g.rank == 0) pwrite_all(fd, &total, 8, off);
	off += 8;
	const uint64_t list0 = off, data0 = off + 16 * total + bytes_before;
	// local cells ascending, with their slots
	const auto& sid = slot_ids_host(g);
	std::vector<uint32_t> order(nl);
	std::iota(order.begin(), order.end(), 0u);
	std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return sid[a] < sid[b]; });
	std::vector<uint64_t> list(2 * nl);
	std::vector<uint8_t> data(mine);
	uint64_t at = 0;
	for (size_t i = 0; i < nl; i++) {
		const size_t s = order[i];
		list[2 * i] = sid[s];
		list[2 * i + 1] = data0 + at;
		for (size_t k = 0; k < tf.size(); k++) {
			const Field* f = tf[k];
			if (f->var) {
				const uint64_t a = voff[k][s] - voff[k][0], n = voff[k][s + 1] - voff[k][s];
				if (n) std::memcpy(&data[at], &host[k][a], n);
				at += n;
			} else {
				if (f->win_len) std::memcpy(&data[at], &host[k][s * f->elem + f->win_off], f->win_len);
				at += f->win_len;
			}
		}
	}
	if (nl) pwrite_all(fd, list.data(), 16 * nl, list0 + 16 * before);
	if (mine) pwrite_all(fd, data.data(), data.size(), data0);
	// Like the reference (MPI_MODE_CREATE | MPI_MODE_WRONLY, dccrg.hpp:1131)
	// bytes already in the file past the grid data stay - except
	// when a variable-size field is saved: the one-shot load_grid_data takes
	// such a field's bytes up to the record's end, and the last record ends at
	// the end of the file, so stale bytes of an older, longer file there would
	// become the last cell's payload.  Then rank 0 cuts the file at
	// the end of the grid data (every rank's records lie before it).
	const uint64_t data_end = list0 + 16 * total + bytes_total;
	if (g.rank == 0 && !var_transfer_fields(g).empty()) {
		const off_t cur = ::lseek(fd, 0, SEEK_END);
		DX_REQUIRE(cur >= 0, "grid file size unknown");
		if (uint64_t(cur) > data_end) DX_REQUIRE(::ftruncate(fd, off_t(data_end)) == 0, "grid file: truncate failed");
	}
}

// start_loading_grid_data (1795-2083): the grid block and the cell list; every
// local cell's record position, none of its payload
static void start_load_impl(Grid& g, const char* path, uint64_t offset, size_t header_bytes) {
	DX_REQUIRE(!g.initialized, "load_grid_data initializes the grid: call it instead of initialize");
	const int fd = ::open(path, O_RDONLY);
	DX_REQUIRE(fd >= 0, std::string("cannot open grid file ") + path);
	Closer closer{fd};
	const off_t file_end = ::lseek(fd, 0, SEEK_END);
	DX_REQUIRE(file_end >= 0, "grid file size unknown");
	uint64_t off = offset + header_bytes, endian = 0;
	pread_all(fd, &endian, 8, off);
	DX_REQUIRE(endian == kEndianCheck, "grid file endianness check failed");
	off += 8;
	// mapping + neighborhood length + topology (35 B), then the geometry block:
	// Cartesian (id 1, 52 B) or stretched (id 2, 28 B + the coordinates)
	uint8_t blk[87];
	pread_all(fd, blk, 63, off);
	uint64_t len[3];
	int32_t R, gid;
	uint32_t hood;
	double start[3], l0[3];
	std::memcpy(len, blk, 24);
	std::memcpy(&R, blk + 24, 4);
	std::memcpy(&hood, blk + 28, 4);
	std::memcpy(&gid, blk + 35, 4);
	std::vector<uint8_t> geo;
	if (gid == kStretchedGeometryId) {
		const size_t nb = stretched_block_bytes(blk + 35);
		DX_REQUIRE(nb > 0 && nb <= uint64_t(file_end) - (off + 35), "grid file: invalid stretched geometry block");
		geo.resize(nb);
		pread_all(fd, geo.data(), nb, off + 35);
		uint64_t cnt[3];
		std::memcpy(cnt, geo.data() + 4, 24);
		std::vector<double> c(size_t(cnt[0] + cnt[1] + cnt[2]));
		std::memcpy(c.data(), geo.data() + 28, c.size() * 8);
		// the library's device geometry: each dimension's start and first
		// level-0 cell length (exact for evenly spaced coordinates; uneven
		// spacing stays with the facade's host-side geometry)
		size_t at = 0;
		for (int d = 0; d < 3; d++) {
			start[d] = c[at];
			l0[d] = c[at + 1] - c[at];
			at += size_t(cnt[d]);
		}
		off += 35 + nb;
	} else {
		DX_REQUIRE(gid == kCartesianGeometryId,
		           "grid file geometry is neither Cartesian_Geometry nor Stretched_Cartesian_Geometry");
		pread_all(fd, blk + 63, 24, off + 63);
		std::memcpy(start, blk + 39, 24);
		std::memcpy(l0, blk + 63, 24);
		off += sizeof(blk);
	}
	// the same checks as the setters (a foreign or corrupt file must not
	// reach the builders)
	for (int d = 0; d < 3; d++) DX_REQUIRE(len[d] > 0, "grid file: grid length must be > 0");
	DX_REQUIRE(R >= 0 && R <= max_possible_level(len) && R < kMaxLevels, "grid file: invalid refinement level");
	DX_REQUIRE(hood <= max_hood_length(), "grid file: neighborhood length not supported");
	for (int d = 0; d < 3; d++) DX_REQUIRE(l0[d] > 0, "grid file: cell length must be > 0");
	for (int d = 0; d < 3; d++) {
		g.len[d] = len[d];
		g.per[d] = blk[32 + d] != 0;
		g.start[d] = start[d];
		g.l0[d] = l0[d];
	}
	g.R = R;
	g.hood_len = hood;
	g.geo_block = std::move(geo);
	init_impl(g);
	uint64_t total = 0;
	pread_all(fd, &total, 8, off);
	off += 8;
	DX_REQUIRE(total <= (uint64_t(file_end) - off) / 16, "grid file truncated");
	std::vector<uint64_t> list(2 * total);
	if (total) pread_all(fd, list.data(), 16 * total, off);
	const uint64_t data_start = off + 16 * total;
	// a record ends where the next one starts, the last at the end of the
	// file: in list order when the offsets never decrease along the list (the
	// files save_grid_data writes, rank by rank, each rank's cells in the
	// order of their data; empty records then stay empty), else in the order
	// of the offsets
	bool monotone = true;
	for (size_t i = 0; i < total; i++) {
		const uint64_t p = list[2 * i + 1];
		DX_REQUIRE(p >= data_start && p <= uint64_t(file_end), "grid file: cell data out of range");
		if (i && p < list[2 * i - 1]) monotone = false;
	}
	std::vector<uint64_t> starts(total);
	for (size_t i = 0; i < total; i++) starts[i] = list[2 * i + 1];
	std::sort(starts.begin(), starts.end());
	struct Rec {
		uint64_t id, pos, end;
		bool operator<(const Rec& o) const { return id < o.id; }
	};
	std::vector<Rec> cells(total);
	for (size_t i = 0; i < total; i++) {
		const uint64_t p = list[2 * i + 1];
		uint64_t e = uint64_t(file_end);
		if (monotone) {
			if (i + 1 < total) e = list[2 * i + 3];
		} else {
			auto nx = std::upper_bound(starts.begin(), starts.end(), p);
			if (nx != starts.end()) e = *nx;
		}
		cells[i] = {list[2 * i], p, e};
	}
	if (!monotone) {
		// records sharing a start: only the last of them in list order holds
		// bytes, the others are empty (as a writer lays out an empty record
		// followed by a full one at the same position)
		std::unordered_map<uint64_t, size_t> last;
		for (size_t i = 0; i < total; i++) last[list[2 * i + 1]] = i;
		for (size_t i = 0; i < total; i++)
			if (last[list[2 * i + 1]] != i) cells[i].end = cells[i].pos;
	}
	std::sort(cells.begin(), cells.end());
	// owners as load_cells (3647) produces them: the level-0 block
	// partition (create_level_0_cells), refined cells inherit it
	std::vector<uint64_t> ids(total);
	std::vector<int32_t> own(total);
	for (size_t i = 0; i < total; i++) {
		ids[i] = cells[i].id;
		DX_REQUIRE(i == 0 || ids[i] > ids[i - 1], "grid file lists a cell twice");
		const uint64_t l0p = map_level0_parent(g.m, ids[i]);
		DX_REQUIRE(l0p != error_cell, "grid file lists an invalid cell");
		own[i] = g.mesh.bp.owner(l0p);
	}
	Mesh nm;
	mesh_from_global(g, nm, ids, own);
	rebuild(g, nm);
	const size_t nl = g.n_local;
	const auto& sid = slot_ids_host(g);
	g.load.pos.assign(nl, 0);
	g.load.end.assign(nl, 0);
	for (size_t i = 0; i < nl; i++) {
		auto it = std::lower_bound(cells.begin(), cells.end(), Rec{sid[i], 0, 0});
		DX_REQUIRE(it != cells.end() && it->id == sid[i], "local cell missing from grid file");
		g.load.pos[i] = it->pos;
		g.load.end[i] = it->end;
	}
	g.load.path = path;
	g.load.active = true;
}

// continue_loading_grid_data (2112-2378): the next bytes of every local
// cell's record into one field, from the cell's position on, which then
// advances past them.  bytes[s]: the count for local slot s (a fixed-size
// field: its window).  Reads coalesce records that lie close together.
static void continue_load_impl(Grid& g, int fid, const uint64_t* sizes) {
	DX_REQUIRE(g.load.active, "no grid file being loaded (start_loading_grid_data first)");
	Field& f = field(g, fid);
	const size_t nl = g.n_local;
	DX_REQUIRE(g.load.pos.size() == nl, "the grid changed while loading a grid file");
	DX_REQUIRE(!f.var || sizes || !nl, "a variable-size field needs the byte count of every local cell");
	std::vector<uint64_t> bytes(nl);
	for (size_t s = 0; s < nl; s++) {
		bytes[s] = f.var ? sizes[s] : f.win_len;
		DX_REQUIRE(bytes[s] <= g.load.end[s] - g.load.pos[s],
		           "grid file: cell " + std::to_string(slot_ids_host(g)[s]) + " has fewer bytes left than requested");
	}
	const int fd = ::open(g.load.path.c_str(), O_RDONLY);
	DX_REQUIRE(fd >= 0, "cannot open grid file " + g.load.path);
	Closer closer{fd};
	// slot order -> file order, then runs with gaps under 64 KiB read at once
	std::vector<uint32_t> by_pos(nl);
	std::iota(by_pos.begin(), by_pos.end(), 0u);
	std::sort(by_pos.begin(), by_pos.end(), [&](uint32_t a, uint32_t b) { return g.load.pos[a] < g.load.pos[b]; });
	std::vector<uint64_t> at(nl + 1, 0);  // the slot's bytes in `got` (slot order)
	for (size_t s = 0; s < nl; s++) at[s + 1] = at[s] + bytes[s];
	std::vector<uint8_t> got(at[nl]);
	std::vector<uint8_t> run;
	for (size_t i = 0; i < nl;) {
		const uint64_t lo = g.load.pos[by_pos[i]];
		uint64_t hi = lo + bytes[by_pos[i]];
		size_t j = i + 1;
		while (j < nl && g.load.pos[by_pos[j]] <= hi + 65536 && g.load.pos[by_pos[j]] - lo < (uint64_t(1) << 30)) {
			hi = std::max(hi, g.load.pos[by_pos[j]] + bytes[by_pos[j]]);
			j++;
		}
		if (hi > lo) {
			run.resize(hi - lo);
			pread_all(fd, run.data(), run.size(), lo);
			for (size_t k = i; k < j; k++) {
				const uint32_t s = by_pos[k];
				if (bytes[s]) std::memcpy(&got[at[s]], &run[g.load.pos[s] - lo], bytes[s]);
			}
		}
		i = j;
	}
	if (f.var) {
		DBuf<uint64_t> all;
		all.alloc(g.n_slots + 1);
		var_sizes(f, nullptr, 0, g.n_slots, all.p, g.s_comp);
		if (nl) h2d(all.p, bytes.data(), nl * 8, g.s_comp);
		var_resize(f, g.n_slots, all.p, g.s_comp);
		if (at[nl]) {
			HIP_CHECK(hipMemcpyAsync(f.data.p, got.data(), got.size(), hipMemcpyHostToDevice, g.s_comp));
			HIP_CHECK(hipStreamSynchronize(g.s_comp));
		}
	} else if (nl && f.win_len) {
		// the window of every element; the rest of it keeps its bytes
		std::vector<uint8_t> h = download(f.data.p, nl * f.elem, g.s_comp);
		for (size_t s = 0; s < nl; s++) std::memcpy(&h[s * f.elem + f.win_off], &got[at[s]], f.win_len);
		{
			HIP_CHECK(hipMemcpyAsync(f.data.p, h.data(), h.size(), hipMemcpyHostToDevice, g.s_comp));
			HIP_CHECK(hipStreamSynchronize(g.s_comp));
		}
	}
	for (size_t s = 0; s < nl; s++) g.load.pos[s] += bytes[s];
	field_written(f);
}

// finish_loading_grid_data (2380-2400)
static void finish_load_impl(Grid& g) {
	g.load = Grid::FileLoad{};
}

// load_grid_data (1742-1790) = start, one continue over the transferred
// fields in field order, finish.  A variable-size field takes what is left of
// each record after the fixed-size fields that follow it, so at most one
// variable-size field can be read this way (more need the split load with
// the caller's byte counts, as the reference's multi-pass example
// tests/restart/variable_cell_data.cpp does).
static void load_grid_impl(Grid& g, const char* path, uint64_t offset, size_t header_bytes) {
	DX_REQUIRE(var_transfer_fields(g).size() <= 1,
	           "several variable-size fields: load with start / continue / finish_loading_grid_data");
	start_load_impl(g, path, offset, header_bytes);
	const std::vector<Field*> tf = transfer_fields(g);
	for (size_t k = 0; k < tf.size(); k++) {
		Field* f = tf[k];
		if (!f->var) {
			continue_load_impl(g, int(f - g.fields.data()), nullptr);
			continue;
		}
		uint64_t after = 0;
		for (size_t j = k + 1; j < tf.size(); j++) after += tf[j]->win_len;
		std::vector<uint64_t> sz(g.n_local);
		for (size_t s = 0; s < g.n_local; s++) {
			const uint64_t left = g.load.end[s] - g.load.pos[s];
			DX_REQUIRE(left >= after, "grid file: a cell's record is shorter than its fixed-size fields");
			sz[s] = left - after;
		}
		continue_load_impl(g, int(f - g.fields.data()), sz.data());
	}
	finish_load_impl(g);
}

static void adv_fields(Grid& g, const int fids[7], const double* f[7]) {
	for (int k = 0; k < 7; k++) {
		Field& F = field(g, fids[k]);
		DX_REQUIRE(F.elem == 8, "advection fields must be fp64");
		f[k] = (const double*)F.data.p;
	}
}

// the block minima now in g.dt_part (nb of them) belong to fields fids as
// they are now (Grid::DtCache)
static void dt_cache_set(Grid& g, const int fids[7], size_t nb) {
	Grid::DtCache& C = g.dt_cache;
	for (int k = 1; k < 7; k++) {
		C.fid[k - 1] = fids[k];
		C.epoch[k - 1] = field(g, fids[k]).epoch;
	}
	C.n_local = g.n_local;
	C.nb = nb;
	C.valid = nb > 0;
}

// The neighbor records of the tile sweeps (Grid::NbRecords) for the fields
// fids: kept while the six velocity / length fields are the same fields with
// the same write epochs and arrays and the tiles are the same; rebuilt
// otherwise (one pass over the slots, 48 B read + 72 B written per slot, on
// the compute stream, so it follows every queued write of those fields).
// nullptr - the sweeps read the fields - when one of them is external (its
// device pointer is out), when the slots exceed the records' 32-bit indexing,
// and unless DCCRGX_NBREC=1: the records are an experiment that lost (paired
// A/B, DESIGN §5: the record lines are touched by neighbor reads alone, so
// they miss where the field lines hit because the neighbor tile's own reads
// brought them into L2: 0.182 -> 0.235 ms of sweep kernels on config 3).
const double* ensure_nbrec(Grid& g, const int fids[7]) {
	const char* env = std::getenv("DCCRGX_NBREC");  // read per call: tests switch it
	const bool off = !(env && std::atoi(env) == 1);
	Grid::NbRecords& R = g.nbrec;
	if (off || g.n_slots == 0 || g.n_slots >= (size_t(1) << 29)) return nullptr;
	for (int k = 1; k < 7; k++)
		if (field(g, fids[k]).external) return nullptr;
	bool ok = R.valid && R.tiles_gen == g.tiles_gen && R.n_slots == g.n_slots;
	for (int k = 1; k < 7 && ok; k++) {
		const Field& F = field(g, fids[k]);
		ok = R.fid[k - 1] == fids[k] && R.epoch[k - 1] == F.epoch && R.ptr[k - 1] == F.data.p;
	}
	if (ok) return R.r.p;
	const double* f[7];
	adv_fields(g, fids, f);
	R.r.alloc(9 * g.n_slots);
	k_nbrec(f, g.n_slots, R.r.p, g.s_comp);
	for (int k = 1; k < 7; k++) {
		const Field& F = field(g, fids[k]);
		R.fid[k - 1] = fids[k];
		R.epoch[k - 1] = F.epoch;
		R.ptr[k - 1] = F.data.p;
	}
	R.tiles_gen = g.tiles_gen;
	R.n_slots = g.n_slots;
	R.valid = true;
	return R.r.p;
}

static void gol_step_impl(Grid& g, Field& f, int region) {
	size_t s0, s1;
	region_range(g, region, s0, s1);
	if (s1 <= s0) return;
	if (!g.gol_plan_valid) {
		g.gol_plan_ok = gol_slab_plan(g, g.gol_inner, g.gol_outer);
		g.gol_plan_valid = true;
	}
	const uint32_t* st = (const uint32_t*)f.data.p;
	uint32_t* out = (uint32_t*)f.scratch.p;
	k_time_begin(g);
	bool done = false;
	if (g.gol_plan_ok) {
		done = true;
		const uint64_t plane = g.len[0] * g.len[1];
		for (int r = 0; r < 2 && done; r++) {
			if (r == 0 && region == DCCRGX_REGION_OUTER) continue;
			if (r == 1 && region == DCCRGX_REGION_INNER) continue;
			for (const GolBox& b : r == 0 ? g.gol_inner : g.gol_outer) {
				const uint64_t n[3] = {g.len[0], g.len[1], b.nz};
				const int per[3] = {g.per[0], g.per[1], b.lo == -3 ? g.per[2] : 0};
				const uint32_t* lo = b.lo >= 0 ? st + uint64_t(b.lo) : nullptr;
				const uint32_t* hi = b.hi >= 0 ? st + uint64_t(b.hi) : nullptr;
				(void)plane;
				if (!k_gol_structured(st + b.slot0, out + b.slot0, n, per, lo, hi, g.s_comp)) {
					done = false;
					break;
				}
			}
		}
	}
	if (!done) {
		ensure_csr(g);
		k_gol_csr(st, out, g.it_ptr.p, g.it_slot.p, s0, s1, g.s_comp);
	}
	k_time_end(g);
}


#if DCCRGX_PHASE_TIMING
namespace {
struct PhaseTable {
	std::map<std::string, std::pair<double, long>> t;
	~PhaseTable() {
		const char* r = std::getenv("RANK");
		for (auto& kv : t)
			std::fprintf(stderr, "[phase r%s] %-28s %10.3f ms total %7ld calls %9.3f ms/call\n", r ? r : "0",
			             kv.first.c_str(), kv.second.first * 1e3, kv.second.second,
			             kv.second.first * 1e3 / double(kv.second.second));
	}
};
PhaseTable& phase_table() {
	static PhaseTable pt;
	return pt;
}
}  // namespace
double PhaseScope::now() {
	return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void phase_add(const char* name, double seconds) {
	auto& e = phase_table().t[name];
	e.first += seconds;
	e.second += 1;
}
void phase_reset() { phase_table().t.clear(); }
double& phase_comm_total() {
	static double t = 0;
	return t;
}
long& phase_sync_count() {
	static long k = 0;
	return k;
}
#endif

}  // namespace dccrgx

// ============================================================================
// C ABI
// ============================================================================
using namespace dccrgx;

struct dccrgx_grid {
	Grid g;
};

#define GRID_OR_FAIL(gp) \
	if (!(gp)) throw Error(DCCRGX_EINVAL, "null grid"); \
	Grid& g = (gp)->g

static dccrgx_grid* new_grid(int rank, int size, int device) {
	DX_REQUIRE(size >= 1 && rank >= 0 && rank < size, "invalid rank/size");
	HIP_CHECK(hipSetDevice(device));
	auto* h = new dccrgx_grid();
	Grid& g = h->g;
	g.rank = rank;
	g.size = size;
	g.device = device;
	HIP_CHECK(hipStreamCreateWithFlags(&g.s_comp, hipStreamNonBlocking));
	HIP_CHECK(hipStreamCreateWithFlags(&g.s_comm, hipStreamNonBlocking));
	HIP_CHECK(hipEventCreateWithFlags(&g.ev_comp, hipEventDisableTiming));
	HIP_CHECK(hipEventCreateWithFlags(&g.ev_halo, hipEventDisableTiming));
	mesh_init_implicit(g);
	return h;
}

extern "C" {

#if DCCRGX_PHASE_TIMING
// analysis build only: forget the phase totals so far (e.g. after a warm-up)
void dccrgx_phase_reset(void) { phase_reset(); }
#endif

const char* dccrgx_last_error(void) { return g_last_error.c_str(); }
int dccrgx_abi_version(void) { return DCCRGX_ABI_VERSION; }

int dccrgx_get_unique_id(void* out) {
	return guard([&] {
		ncclUniqueId id;
		NCCL_CHECK(ncclGetUniqueId(&id));
		std::memcpy(out, &id, sizeof(id));
		return 0;
	});
}

int dccrgx_create(int rank, int size, int device, const void* nccl_id, dccrgx_grid** out) {
	return guard([&] {
		DX_REQUIRE(out, "null output");
		dccrgx_grid* h = new_grid(rank, size, device);
		if (nccl_id) {  // without an id: a detached view of one rank (no transport)
			ncclUniqueId id;
			std::memcpy(&id, nccl_id, sizeof(id));
			const ncclResult_t r = ncclCommInitRank(&h->g.nccl, size, id, rank);
			if (r != ncclSuccess) {
				delete h;
				throw Error(DCCRGX_ECOMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
			}
		}
		*out = h;
		return 0;
	});
}

int dccrgx_create_with_exchange(int rank, int size, int device, dccrgx_exchange_fn fn, void* ctx, dccrgx_grid** out) {
	return guard([&] {
		DX_REQUIRE(out && fn, "null output or exchange function");
		dccrgx_grid* h = new_grid(rank, size, device);
		h->g.xfn = fn;
		h->g.xctx = ctx;
		*out = h;
		return 0;
	});
}

int dccrgx_device_count(int* n) {
	return guard([&] {
		DX_REQUIRE(n, "null output");
		HIP_CHECK(hipGetDeviceCount(n));
		return 0;
	});
}

int dccrgx_get_cells_by_criteria(dccrgx_grid* gp, const int32_t* criteria, size_t nc, int exact_match, int hood,
                                 uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		DX_REQUIRE(criteria || !nc, "null criteria");
		if (hood != DCCRGX_DEFAULT_HOOD && !g.uhoods.count(hood)) return copy_out_u64({}, out, cap, n);
		return copy_out_u64(cells_by_criteria(g, criteria, nc, exact_match != 0, hood), out, cap, n);
	});
}

int dccrgx_get_slots(dccrgx_grid* gp, const uint64_t* ids, size_t n, int64_t* slots) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE((ids && slots) || !n, "null argument");
		for (size_t i = 0; i < n; i++) slots[i] = lookup_slot(g, ids[i]);
		return 0;
	});
}

int dccrgx_download_user_csr(dccrgx_grid* gp, int hood, int kind, uint32_t* ptr, uint64_t* ids, int32_t* offs,
                             size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (!g.uhoods.count(hood)) return DCCRGX_ENOTFOUND;
		DX_REQUIRE(kind == 0 || kind == 1, "invalid CSR kind");
		UserHood& h = ensure_uhood(g, hood);
		const size_t nl = g.n_local;
		const std::vector<uint32_t> hp = download(kind == 0 ? h.nof_ptr.p : h.nto_ptr.p, nl + 1, g.s_comp);
		const size_t tot = hp[nl];
		if (n) *n = tot;
		if (tot > cap) return DCCRGX_ERANGE;
		std::memcpy(ptr, hp.data(), (nl + 1) * 4);
		if (!tot) return 0;
		d2h_small(ids, kind == 0 ? h.nof_id.p : h.nto_id.p, tot * 8, g.s_comp);
		if (offs && kind == 0) d2h_small(offs, h.nof_off.p, tot * 12, g.s_comp);
		return 0;
	});
}

int dccrgx_destroy(dccrgx_grid* gp) {
	return guard([&] {
		if (!gp) return 0;
		Grid& g = gp->g;
		(void)hipDeviceSynchronize();
		drain_timing(g);
		if (g.nccl) ncclCommDestroy(g.nccl);
		if (g.pin_stage) (void)hipHostFree(g.pin_stage);
		if (g.ev_comp) (void)hipEventDestroy(g.ev_comp);
		if (g.ev_halo) (void)hipEventDestroy(g.ev_halo);
		if (g.s_comp) (void)hipStreamDestroy(g.s_comp);
		if (g.s_comm) (void)hipStreamDestroy(g.s_comm);
		delete gp;
		return 0;
	});
}

int dccrgx_set_initial_length(dccrgx_grid* gp, const uint64_t length[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_initial_length after initialize");
		for (int d = 0; d < 3; d++) DX_REQUIRE(length[d] > 0, "grid length must be > 0");
		for (int d = 0; d < 3; d++) g.len[d] = length[d];
		return 0;
	});
}

int dccrgx_get_initial_length(dccrgx_grid* gp, uint64_t length[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (int d = 0; d < 3; d++) length[d] = g.len[d];
		return 0;
	});
}

int dccrgx_get_periodic(dccrgx_grid* gp, int periodic[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (int d = 0; d < 3; d++) periodic[d] = g.per[d] ? 1 : 0;
		return 0;
	});
}

int dccrgx_set_maximum_refinement_level(dccrgx_grid* gp, int level) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_maximum_refinement_level after initialize");
		const int maxpos = max_possible_level(g.len);
		if (level < 0) level = maxpos;
		DX_REQUIRE(level <= maxpos && level < kMaxLevels, "refinement level too large for the grid");
		g.R = level;
		return 0;
	});
}

int dccrgx_get_maximum_refinement_level(dccrgx_grid* gp, int* level) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		*level = g.R;
		return 0;
	});
}

int dccrgx_get_neighborhood_length(dccrgx_grid* gp, unsigned* length) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(length != nullptr, "null output");
		*length = g.hood_len;
		return 0;
	});
}

int dccrgx_set_periodic(dccrgx_grid* gp, int x, int y, int z) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_periodic after initialize");
		g.per[0] = x != 0;
		g.per[1] = y != 0;
		g.per[2] = z != 0;
		return 0;
	});
}

int dccrgx_set_neighborhood_length(dccrgx_grid* gp, unsigned length) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(!g.initialized, "set_neighborhood_length after initialize");
		DX_REQUIRE(length <= max_hood_length(),
		           "neighborhood length > " + std::to_string(max_hood_length()) + " not supported");
		g.hood_len = length;
		return 0;
	});
}

int dccrgx_initialize(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		init_impl(g);
		return 0;
	});
}

int dccrgx_set_geometry(dccrgx_grid* gp, const double start[3], const double l0[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (int d = 0; d < 3; d++) DX_REQUIRE(l0[d] > 0, "cell length must be > 0");
		for (int d = 0; d < 3; d++) {
			g.start[d] = start[d];
			g.l0[d] = l0[d];
		}
		return 0;
	});
}

int dccrgx_get_geometry(dccrgx_grid* gp, double start[3], double l0[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (int d = 0; d < 3; d++) {
			if (start) start[d] = g.start[d];
			if (l0) l0[d] = g.l0[d];
		}
		return 0;
	});
}

int dccrgx_set_geometry_block(dccrgx_grid* gp, const void* bytes, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (n == 0) {
			g.geo_block.clear();
			return 0;
		}
		DX_REQUIRE(bytes != nullptr && n >= 28, "geometry block too short");
		const uint8_t* b = static_cast<const uint8_t*>(bytes);
		DX_REQUIRE(stretched_block_bytes(b) == n, "not a Stretched_Cartesian_Geometry block (id 2, counts, coordinates)");
		g.geo_block.assign(b, b + n);
		return 0;
	});
}

int dccrgx_get_geometry_block(dccrgx_grid* gp, void* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(n != nullptr, "null count");
		*n = g.geo_block.size();
		if (!out) return 0;
		DX_REQUIRE(cap >= g.geo_block.size(), "buffer too small for the geometry block");
		if (!g.geo_block.empty()) std::memcpy(out, g.geo_block.data(), g.geo_block.size());
		return 0;
	});
}

int dccrgx_geometry_batch(dccrgx_grid* gp, const uint64_t* ids, size_t n, double* center, double* length) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(ids || !n, "null ids");
		MapCtx m;
		map_init(m, g.len, g.R, g.per);
		const double nan = std::numeric_limits<double>::quiet_NaN();
		for (size_t i = 0; i < n; i++) {
			uint64_t ind[3];
			const int lvl = map_indices(m, ids[i], ind[0], ind[1], ind[2]);
			for (int d = 0; d < 3; d++) {
				double L = nan, c = nan;
				if (lvl >= 0) {  // dccrg_cartesian_geometry.hpp:299-303, 334-359
					L = g.l0[d] * (1.0 / double(uint64_t(1) << lvl));
					c = g.start[d] + double(ind[d]) * g.l0[d] / double(uint64_t(1) << g.R) + L / 2;
				}
				if (length) length[3 * i + d] = L;
				if (center) center[3 * i + d] = c;
			}
		}
		return 0;
	});
}

uint64_t dccrgx_get_cell_from_indices(dccrgx_grid* gp, const uint64_t ind[3], int level) {
	if (!gp) return error_cell;
	MapCtx m;
	map_init(m, gp->g.len, gp->g.R, gp->g.per);
	return map_from_indices(m, ind[0], ind[1], ind[2], level);
}

namespace {
// the device id math every build and sweep kernel uses (dccrgx_mapping.hpp),
// evaluated for a batch of ids: 15 words per id (indices x3, length in
// indices, parent, first child, level-0 parent, siblings x8)
__global__ void mapping_batch_kernel(MapCtx m, const uint64_t* ids, size_t n, int32_t* level, uint64_t* out) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t* o = out + 15 * i;
		uint64_t x = 0, y = 0, z = 0;
		const int l = map_indices(m, ids[i], x, y, z);
		level[i] = l;
		for (int k = 0; k < 15; k++) o[k] = error_cell;
		if (l < 0) continue;
		o[0] = x;
		o[1] = y;
		o[2] = z;
		o[3] = map_cell_len(m, ids[i]);
		o[4] = map_parent(m, ids[i]);
		o[5] = map_child(m, ids[i]);
		o[6] = map_level0_parent(m, ids[i]);
		map_siblings(m, ids[i], o + 7);
	}
}
}  // namespace

int dccrgx_mapping_batch(dccrgx_grid* gp, const uint64_t* ids, size_t n, int32_t* level, uint64_t* out) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE((ids && level && out) || !n, "null argument");
		if (!n) return 0;
		MapCtx m;
		map_init(m, g.len, g.R, g.per);
		DBuf<uint64_t> d_ids, d_out;
		DBuf<int32_t> d_lvl;
		d_ids.alloc(n);
		d_out.alloc(15 * n);
		d_lvl.alloc(n);
		h2d(d_ids.p, ids, n * 8, g.s_comp);
		mapping_batch_kernel<<<grid_for(n, 256), 256, 0, g.s_comp>>>(m, d_ids.p, n, d_lvl.p, d_out.p);
		HIP_CHECK(hipGetLastError());
		HIP_CHECK(hipMemcpyAsync(level, d_lvl.p, n * 4, hipMemcpyDeviceToHost, g.s_comp));
		d2h_small(out, d_out.p, 15 * n * 8, g.s_comp);
		return 0;
	});
}

int dccrgx_get_indices(dccrgx_grid* gp, uint64_t cell, uint64_t ind[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		MapCtx m;
		map_init(m, g.len, g.R, g.per);
		const int l = map_indices(m, cell, ind[0], ind[1], ind[2]);
		return l < 0 ? DCCRGX_ENOTFOUND : 0;
	});
}

int dccrgx_get_refinement_level(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return -1;
	MapCtx m;
	map_init(m, gp->g.len, gp->g.R, gp->g.per);
	return map_level(m, cell);
}

uint64_t dccrgx_get_last_cell(dccrgx_grid* gp) {
	if (!gp) return 0;
	MapCtx m;
	map_init(m, gp->g.len, gp->g.R, gp->g.per);
	return m.last;
}

int dccrgx_get_counts(dccrgx_grid* gp, size_t* ni, size_t* no, size_t* nr, size_t* ns) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (ni) *ni = g.n_inner;
		if (no) *no = g.n_outer;
		if (nr) *nr = g.n_recv;
		if (ns) *ns = g.n_slots;
		return 0;
	});
}

int dccrgx_get_cells(dccrgx_grid* gp, int which, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		const auto& ids = slot_ids_host(g);
		std::vector<uint64_t> v;
		switch (which) {
		case DCCRGX_CELLS_LOCAL: v.assign(ids.begin(), ids.begin() + ptrdiff_t(g.n_local)); break;
		case DCCRGX_CELLS_INNER: v.assign(ids.begin(), ids.begin() + ptrdiff_t(g.n_inner)); break;
		case DCCRGX_CELLS_OUTER: v.assign(ids.begin() + ptrdiff_t(g.n_inner), ids.begin() + ptrdiff_t(g.n_local)); break;
		case DCCRGX_CELLS_REMOTE: v.assign(ids.begin() + ptrdiff_t(g.n_local), ids.end()); break;
		case DCCRGX_CELLS_ALL: v = ids; break;
		default: throw Error(DCCRGX_EINVAL, "invalid selection");
		}
		std::sort(v.begin(), v.end());
		return copy_out_u64(v, out, cap, n);
	});
}

int dccrgx_get_slot_ids(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		return copy_out_u64(slot_ids_host(g), out, cap, n);
	});
}

int dccrgx_get_neighbors_of(dccrgx_grid* gp, uint64_t cell, uint64_t* ids, int32_t* offs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const int64_t s = lookup_slot(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		ensure_csr(g);
		uint32_t be[2];
		d2h_small(be, g.nof_ptr.p + s, 8, g.s_comp);
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		if (k) {
			d2h_small(ids, g.nof_id.p + be[0], k * 8, g.s_comp);
			if (offs) d2h_small(offs, g.nof_off.p + 3 * size_t(be[0]), k * 12, g.s_comp);
		}
		return 0;
	});
}

int dccrgx_get_neighbors_to(dccrgx_grid* gp, uint64_t cell, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const int64_t s = lookup_slot(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		ensure_csr(g);
		uint32_t be[2];
		d2h_small(be, g.nto_ptr.p + s, 8, g.s_comp);
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		if (k) d2h_small(ids, g.nto_id.p + be[0], k * 8, g.s_comp);
		return 0;
	});
}

int dccrgx_get_face_neighbors_of(dccrgx_grid* gp, uint64_t cell, uint64_t* ids, int32_t* dirs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		static const int dmap[6] = {-1, +1, -2, +2, -3, +3};
		const int64_t s = lookup_slot(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) {
			// a remote cell this process knows (e.g. a copy in all_cells()): its
			// faces from the known leaves, probed at every level at each face's
			// probe point (the leaf there must be known, else the face lies
			// beyond the ghost region and the cell is not answered)
			if (lookup_owner(g, cell) < 0) return DCCRGX_ENOTFOUND;
			const MapCtx& m = g.m;
			uint64_t c[3], p[3];
			const int lvl = map_indices(m, cell, c[0], c[1], c[2]);
			std::vector<uint64_t> cand;
			for (int dir = 0; dir < 6; dir++)
				if (face_probe(m, c, lvl, dir, p))
					for (int l = 0; l <= m.R; l++) cand.push_back(map_from_indices(m, p[0], p[1], p[2], l));
			std::sort(cand.begin(), cand.end());
			cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
			std::vector<int32_t> own(cand.size());
			lookup_batch(g, cand.data(), cand.size(), own.data(), nullptr);
			const auto exists = [&](uint64_t id) {
				const auto it = std::lower_bound(cand.begin(), cand.end(), id);
				return it != cand.end() && *it == id && own[size_t(it - cand.begin())] >= 0;
			};
			std::vector<std::pair<uint64_t, int>> out;
			for (int dir = 0; dir < 6; dir++) {
				if (!face_probe(m, c, lvl, dir, p)) continue;
				bool any = false;
				for (int l = 0; l <= m.R && !any; l++) any = exists(map_from_indices(m, p[0], p[1], p[2], l));
				if (!any) throw Error(DCCRGX_ENOTFOUND, "a face of this remote cell lies beyond the ghost region");
				uint64_t f[4];
				const int k = face_dir(m, c, lvl, dir, exists, f);
				for (int i = 0; i < k; i++) out.push_back({f[i], dmap[dir]});
			}
			if (n) *n = out.size();
			if (out.size() > cap) return DCCRGX_ERANGE;
			for (size_t i = 0; i < out.size(); i++) {
				ids[i] = out[i].first;
				if (dirs) dirs[i] = out[i].second;
			}
			return 0;
		}
		ensure_face_csr(g);
		uint32_t be[2];
		d2h_small(be, g.face_ptr.p + s, 8, g.s_comp);
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		std::vector<int32_t> ent(k);
		if (k) d2h_small(ent.data(), g.face_ent.p + be[0], k * 4, g.s_comp);
		const auto& sid = slot_ids_host(g);
		for (size_t i = 0; i < k; i++) {
			ids[i] = sid[size_t(ent[i] >> 3)];
			if (dirs) dirs[i] = dmap[ent[i] & 7];
		}
		return 0;
	});
}

int dccrgx_download_csr(dccrgx_grid* gp, int kind, uint32_t* ptr, uint64_t* ids, int32_t* aux, size_t cap,
                        size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(kind >= 0 && kind <= 3, "invalid CSR kind");
		const size_t nl = g.n_local;
		const uint32_t* dptr = nullptr;
		if (kind == 2) {
			ensure_face_csr(g);
			dptr = g.face_ptr.p;
		} else {
			ensure_csr(g);
			dptr = kind == 0 ? g.nof_ptr.p : kind == 1 ? g.nto_ptr.p : g.it_ptr.p;
		}
		std::vector<uint32_t> hp = download(dptr, nl + 1, g.s_comp);
		const size_t tot = hp[nl];
		if (n) *n = tot;
		if (tot > cap) return DCCRGX_ERANGE;
		std::memcpy(ptr, hp.data(), (nl + 1) * 4);
		if (!tot) return 0;
		const auto& sid = slot_ids_host(g);
		if (kind == 0) {
			d2h_small(ids, g.nof_id.p, tot * 8, g.s_comp);
			if (aux) d2h_small(aux, g.nof_off.p, tot * 12, g.s_comp);
		} else if (kind == 1) {
			d2h_small(ids, g.nto_id.p, tot * 8, g.s_comp);
		} else if (kind == 2) {
			std::vector<int32_t> ent = download(g.face_ent.p, tot, g.s_comp);
			static const int dmap[6] = {-1, +1, -2, +2, -3, +3};
			for (size_t i = 0; i < tot; i++) {
				ids[i] = sid[size_t(ent[i] >> 3)];
				if (aux) aux[i] = dmap[ent[i] & 7];
			}
		} else {
			std::vector<int32_t> sl = download(g.it_slot.p, tot, g.s_comp);
			for (size_t i = 0; i < tot; i++) ids[i] = sid[size_t(sl[i])];
			if (aux) d2h_small(aux, g.it_off.p, tot * 12, g.s_comp);
		}
		return 0;
	});
}

int dccrgx_is_local(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return 0;
	try {
		return is_local_cell(gp->g, cell) ? 1 : 0;
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return 0;
	}
}

int dccrgx_get_process(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return -1;
	try {
		return lookup_owner(gp->g, cell);
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return -1;
	}
}

int64_t dccrgx_get_slot(dccrgx_grid* gp, uint64_t cell) {
	if (!gp) return -1;
	try {
		return lookup_slot(gp->g, cell);
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return -1;
	}
}

int dccrgx_get_peers(dccrgx_grid* gp, int32_t* peers, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (n) *n = g.peers.size();
		if (g.peers.size() > cap) return DCCRGX_ERANGE;
		for (size_t i = 0; i < g.peers.size(); i++) peers[i] = g.peers[i];
		return 0;
	});
}

int dccrgx_get_cells_to_send(dccrgx_grid* gp, int peer, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		auto it = g.halo.send_ids.find(peer);
		static const std::vector<uint64_t> empty;
		return copy_out_u64(it == g.halo.send_ids.end() ? empty : it->second, ids, cap, n);
	});
}

int dccrgx_get_cells_to_receive(dccrgx_grid* gp, int peer, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		auto it = g.halo.recv_ids.find(peer);
		static const std::vector<uint64_t> empty;
		return copy_out_u64(it == g.halo.recv_ids.end() ? empty : it->second, ids, cap, n);
	});
}

int dccrgx_get_cell_process(dccrgx_grid* gp, uint64_t* ids, int32_t* owners, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		std::vector<uint64_t> k;
		std::vector<int32_t> o;
		known_leaves(g, k, o);
		if (n) *n = k.size();
		if (!ids) return 0;
		if (cap < k.size()) return int(DCCRGX_ERANGE);
		std::copy(k.begin(), k.end(), ids);
		if (owners) std::copy(o.begin(), o.end(), owners);
		return 0;
	});
}

static int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

int dccrgx_find_neighbors_of(dccrgx_grid* gp, uint64_t cell, const int32_t* items, size_t n_items, uint64_t* ids,
                             int32_t* offs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		DX_REQUIRE(items || !n_items, "null neighborhood");
		const MapCtx& m = g.m;
		if (lookup_owner(g, cell) < 0) return DCCRGX_ENOTFOUND;  // 4354-4362: unknown cell
		uint64_t c[3];
		const int lvl = map_indices(m, cell, c[0], c[1], c[2]);
		const bool local = is_local_cell(g, cell);
		const int64_t len = int64_t(1) << (m.R - lvl), l0 = int64_t(1) << m.R;
		const int64_t r = std::max(1, int(g.hood_len));
		// the three cells an item's box can resolve to (nof_item): finer,
		// same size and coarser, all probed in one device lookup
		std::vector<uint64_t> cand;
		for (size_t i = 0; i < n_items; i++) {
			const int32_t* h = items + 3 * i;
			uint64_t w[3];
			bool inside = true;
			for (int d = 0; d < 3; d++) {
				const int64_t lo = int64_t(c[d]) + int64_t(h[d]) * len;
				// a local cell's box must lie in the level-0 cells this rank
				// knows (its ghost region); a remote cell's list may be
				// incomplete, as the reference documents (4327-4328)
				if (local) {
					const int64_t own = int64_t(c[d]) / l0;
					if (std::abs(floor_div(lo, l0) - own) > r || std::abs(floor_div(lo + len - 1, l0) - own) > r)
						throw Error(DCCRGX_EINVAL, "neighborhood item beyond the ghost region of this process");
				}
				inside = inside && map_wrap(m, d, lo, w[d]);
			}
			if (!inside) continue;
			for (int l = std::max(0, lvl - 1); l <= std::min(m.R, lvl + 1); l++)
				cand.push_back(map_from_indices(m, w[0], w[1], w[2], l));
		}
		std::sort(cand.begin(), cand.end());
		cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
		std::vector<int32_t> own(cand.size());
		lookup_batch(g, cand.data(), cand.size(), own.data(), nullptr);
		const auto exists = [&](uint64_t id) {
			const auto it = std::lower_bound(cand.begin(), cand.end(), id);
			return it != cand.end() && *it == id && own[size_t(it - cand.begin())] >= 0;
		};
		std::vector<uint64_t> oi;
		std::vector<int32_t> oo;
		ItemOut o;
		for (size_t i = 0; i < n_items; i++) {
			nof_item(m, c, lvl, items + 3 * i, exists, o);
			for (int k = 0; k < o.n; k++) {
				oi.push_back(o.id[k]);
				oo.insert(oo.end(), o.off[k], o.off[k] + 3);
			}
		}
		if (n) *n = oi.size();
		if (oi.size() > cap || (!ids && !oi.empty())) return DCCRGX_ERANGE;
		std::copy(oi.begin(), oi.end(), ids);
		if (offs) std::copy(oo.begin(), oo.end(), offs);
		return 0;
	});
}

int dccrgx_get_face_cache(dccrgx_grid* gp, uint64_t* ids, uint64_t* nbrs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		const MapCtx& m = g.m;
		std::vector<uint64_t> k;
		std::vector<int32_t> o;
		known_leaves(g, k, o);
		// every leaf under a known level-0 cell is known (own + ghost region)
		std::vector<uint64_t> l0;
		for (uint64_t id : k) l0.push_back(map_level0_parent(m, id));
		std::sort(l0.begin(), l0.end());
		l0.erase(std::unique(l0.begin(), l0.end()), l0.end());
		const auto exists = [&](uint64_t id) { return std::binary_search(k.begin(), k.end(), id); };
		std::vector<uint64_t> oi, on;
		for (uint64_t id : k) {
			uint64_t c[3];
			const int lvl = map_indices(m, id, c[0], c[1], c[2]);
			std::array<uint64_t, 6> e;
			bool known = true;
			for (int dir = 0; dir < 6 && known; dir++) {
				uint64_t p[3], f[4];
				e[size_t(dir)] = error_cell;
				if (!face_probe(m, c, lvl, dir, p)) continue;
				// the probe's level-0 cell must be known for the entry to be exact
				known = std::binary_search(l0.begin(), l0.end(), map_from_indices(m, p[0], p[1], p[2], 0));
				if (known && face_dir(m, c, lvl, dir, exists, f) > 0) e[size_t(dir)] = f[0];
			}
			if (!known) continue;
			oi.push_back(id);
			on.insert(on.end(), e.begin(), e.end());
		}
		if (n) *n = oi.size();
		if (oi.size() > cap || (!ids && !oi.empty())) return DCCRGX_ERANGE;
		std::copy(oi.begin(), oi.end(), ids);
		if (nbrs) std::copy(on.begin(), on.end(), nbrs);
		return 0;
	});
}

int dccrgx_unpin_all_cells(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		g.pins.clear();
		return 0;
	});
}

int dccrgx_get_number_of_update_cells(dccrgx_grid* gp, uint64_t* ns, uint64_t* nr) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (ns) *ns = g.halo.n_send;
		if (nr) *nr = g.halo.n_recv;
		return 0;
	});
}

static void flush_bulk_requests(Grid& g) {
	g.refine_dev_valid = false;
	g.refine_dev.release();
	g.unrefine_dev_valid = false;
	g.unrefine_dev.release();
	g.refine_requests.insert(g.refine_bulk.begin(), g.refine_bulk.end());
	g.unrefine_requests.insert(g.unrefine_bulk.begin(), g.unrefine_bulk.end());
	g.refine_bulk.clear();
	g.unrefine_bulk.clear();
}


// refine_completely (2434-2530): only local leaves; at the maximum level it
// is dont_unrefine (2472-2475); refused (false) when the cell, or a coarser
// neighbor of it, is in the dont_refine set that persists from the last
// stop_refining (2477-2491)
int dccrgx_refine_completely(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		flush_bulk_requests(g);
		if (!is_local_cell(g, cell)) return DCCRGX_ENOTFOUND;  // 2449-2459: only local cells
		const int lvl = map_level(g.m, cell);
		if (lvl >= g.R) {
			// 2472-2475: dont_unrefine (2679-2733) and true
			if (lvl == 0) return 0;
			uint64_t sib[8];
			map_siblings(g.m, cell, sib);
			for (uint64_t s : sib)
				if (g.dont_unrefine_cells.count(s)) return 0;
			for (uint64_t s : sib) g.unrefine_requests.erase(s);
			g.dont_unrefine_cells.insert(cell);
			return 0;
		}
		if (!g.dont_refine_cells.empty()) {
			if (g.dont_refine_cells.count(cell)) return DCCRGX_ENOTFOUND;
			// a coarser neighbors_of entry in the set (2480-2490): per hood item
			// the level lvl - 1 leaf holding the item box's min corner (nof_item:
			// the coarser neighbor of a 2:1-balanced mesh), tested against the
			// set first and looked up only when it is in it (not a
			// walk of the whole set per call)
			if (lvl > 0) {
				uint64_t c[3];
				map_indices(g.m, cell, c[0], c[1], c[2]);
				const int64_t len = int64_t(1) << (g.R - lvl);
				for (size_t k = 0; k + 2 < g.hood.size(); k += 3) {
					uint64_t w[3];
					bool inside = true;
					for (int a = 0; a < 3 && inside; a++)
						inside = map_wrap(g.m, a, int64_t(c[a]) + int64_t(g.hood[k + size_t(a)]) * len, w[a]);
					if (!inside) continue;
					const uint64_t pl = uint64_t(len) * 2;
					const uint64_t p = map_from_indices(g.m, w[0] & ~(pl - 1), w[1] & ~(pl - 1), w[2] & ~(pl - 1), lvl - 1);
					if (g.dont_refine_cells.count(p) && lookup_owner(g, p) >= 0) return DCCRGX_ENOTFOUND;
				}
			}
		}
		g.refine_requests.insert(cell);
		return 0;
	});
}

// unrefine_completely (2560-2660): local leaves only; level 0 is a no-op;
// false (ENOTFOUND) when a sibling has children; a family marked by a
// refine or dont_unrefine of a sibling, or already requested, is a no-op.
// The neighborhood test happens in stop_refining (override_unrefines).
int dccrgx_unrefine_completely(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		if (!is_local_cell(g, cell)) return DCCRGX_ENOTFOUND;
		if (map_level(g.m, cell) == 0) return 0;
		flush_bulk_requests(g);
		uint64_t sib[8];
		map_siblings(g.m, cell, sib);
		auto has = [](const std::unordered_set<uint64_t>& v, uint64_t x) { return v.count(x) > 0; };
		for (uint64_t s : sib) {  // 2596-2607, sibling by sibling
			if (lookup_owner(g, s) < 0) return DCCRGX_ENOTFOUND;  // the sibling has children
			if (has(g.refine_requests, s) || has(g.dont_unrefine_cells, s)) return 0;
		}
		for (uint64_t s : sib)
			if (has(g.unrefine_requests, s)) return 0;  // 2636-2641
		g.unrefine_requests.insert(cell);
		return 0;
	});
}

// dont_unrefine (2679-2733): the family of a local leaf is not merged by the
// next stop_refining (local requests of its siblings are dropped now)
int dccrgx_dont_unrefine(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		if (!is_local_cell(g, cell)) return DCCRGX_ENOTFOUND;
		if (map_level(g.m, cell) == 0) return 0;
		flush_bulk_requests(g);
		uint64_t sib[8];
		map_siblings(g.m, cell, sib);
		for (uint64_t s : sib)
			if (g.dont_unrefine_cells.count(s)) return 0;
		for (uint64_t s : sib) g.unrefine_requests.erase(s);
		g.dont_unrefine_cells.insert(cell);
		return 0;
	});
}

// dont_refine (2744-2784): the local leaf and, in stop_refining, its finer
// neighbors (override_refines) are not refined by request; the spread set
// persists after stop_refining (10039) until balance_load clears it (3812)
int dccrgx_dont_refine(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		if (!is_local_cell(g, cell)) return DCCRGX_ENOTFOUND;
		if (map_level(g.m, cell) >= g.R) return 0;
		flush_bulk_requests(g);
		g.refine_requests.erase(cell);
		g.dont_refine_cells.insert(cell);
		return 0;
	});
}

int dccrgx_get_removed_cells(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		return copy_out_u64(g.removed_ids.host(g.s_comp), out, cap, n);
	});
}

int dccrgx_removed_field_download(dccrgx_grid* gp, int fid, void* host, size_t cap_bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = fixed_field(g, fid);
		const size_t bytes = g.removed_ids.size() * f.elem;
		DX_REQUIRE(cap_bytes >= bytes, "buffer too small for the removed cells' payloads");
		if (bytes) d2h_small(host, f.removed.p, bytes, g.s_comp);
		return 0;
	});
}

int dccrgx_removed_field_device_ptr(dccrgx_grid* gp, int fid, void** ptr) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(ptr, "null pointer");
		*ptr = g.removed_ids.empty() ? nullptr : fixed_field(g, fid).removed.p;
		return 0;
	});
}

int dccrgx_stop_refining(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		stop_refining_impl(g);
		if (!out) {
			if (n) *n = g.new_cells.size();
			return 0;
		}
		return copy_out_u64(g.new_cells.host(g.s_comp), out, cap, n);
	});
}

int dccrgx_get_new_cells(dccrgx_grid* gp, uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		return copy_out_u64(g.new_cells.host(g.s_comp), out, cap, n);
	});
}

int dccrgx_set_cells(dccrgx_grid* gp, const uint64_t* ids, const int32_t* owners, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		DX_REQUIRE(!g.mig.active, "balance_load in progress");
		std::vector<uint64_t> L(ids, ids + n);
		std::vector<int32_t> O(owners, owners + n);
		for (size_t i = 0; i < n; i++) {
			DX_REQUIRE(L[i] != error_cell && L[i] <= g.m.last, "invalid cell id");
			DX_REQUIRE(i == 0 || L[i] > L[i - 1], "cell ids must be strictly ascending");
			DX_REQUIRE(O[i] >= 0 && O[i] < g.size, "invalid owner");
		}
		Mesh nm;
		mesh_from_global(g, nm, L, O);
		rebuild(g, nm);
		g.pins.clear();
		return 0;
	});
}

int dccrgx_pin(dccrgx_grid* gp, uint64_t cell, int process) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(process >= 0 && process < g.size, "invalid process");
		if (!is_local_cell(g, cell)) return DCCRGX_ENOTFOUND;  // 5877-5887: local leaves only
		g.pins[cell] = process;
		return 0;
	});
}

int dccrgx_unpin(dccrgx_grid* gp, uint64_t cell) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		g.pins.erase(cell);
		return 0;
	});
}

int dccrgx_add_neighborhood(dccrgx_grid* gp, int id, const int32_t* offsets, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		// add_neighborhood 6383-6520: the reference returns false for these
		DX_REQUIRE(id != DCCRGX_DEFAULT_HOOD, "neighborhood id is the default id");
		DX_REQUIRE(!g.uhoods.count(id), "neighborhood id already exists");
		for (size_t i = 0; i < n; i++) {
			const int32_t* o = offsets + 3 * i;
			if (g.hood_len > 0) {
				for (int d = 0; d < 3; d++)
					DX_REQUIRE(unsigned(std::abs(o[d])) <= g.hood_len, "offset outside the default neighborhood");
				DX_REQUIRE(o[0] || o[1] || o[2], "offset (0, 0, 0)");
			} else {
				int zeros = 0;
				for (int d = 0; d < 3; d++) {
					zeros += o[d] == 0;
					DX_REQUIRE(std::abs(o[d]) <= 1, "offset outside the face neighborhood");
				}
				DX_REQUIRE(zeros == 2, "face neighborhood offsets must be unit face offsets");
			}
		}
		UserHood& h = g.uhoods[id];
		h.of.assign(offsets, offsets + 3 * n);
		h.to.resize(h.of.size());
		for (size_t i = 0; i < h.of.size(); i++) h.to[i] = -h.of[i];
		upload(h.d_of, h.of, g.s_comp);
		upload(h.d_to, h.to, g.s_comp);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		ensure_uhood(g, id);
		return 0;
	});
}

int dccrgx_remove_neighborhood(dccrgx_grid* gp, int id) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		g.uhoods.erase(id);
		return 0;
	});
}

int dccrgx_get_user_neighbors(dccrgx_grid* gp, int id, uint64_t cell, int kind, uint64_t* ids, int32_t* offs,
                              size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (!g.uhoods.count(id)) return DCCRGX_ENOTFOUND;
		const int64_t s = lookup_slot(g, cell);
		if (s < 0 || size_t(s) >= g.n_local) return DCCRGX_ENOTFOUND;
		UserHood& h = ensure_uhood(g, id);
		const DBuf<uint32_t>& ptr = kind == 0 ? h.nof_ptr : h.nto_ptr;
		uint32_t be[2];
		d2h_small(be, ptr.p + s, 8, g.s_comp);
		const size_t k = be[1] - be[0];
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		if (k) {
			d2h_small(ids, (kind == 0 ? h.nof_id.p : h.nto_id.p) + be[0], k * 8, g.s_comp);
			if (offs && kind == 0)
				d2h_small(offs, h.nof_off.p + 3 * size_t(be[0]), k * 12, g.s_comp);
		}
		return 0;
	});
}

int dccrgx_get_user_update_list(dccrgx_grid* gp, int id, int peer, int receive, uint64_t* ids, size_t cap,
                                size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (!g.uhoods.count(id)) return DCCRGX_ENOTFOUND;
		UserHood& h = ensure_uhood(g, id);
		const auto& mp = receive ? h.plan.recv_ids : h.plan.send_ids;
		auto it = mp.find(peer);
		static const std::vector<uint64_t> empty;
		return copy_out_u64(it == mp.end() ? empty : it->second, ids, cap, n);
	});
}

int dccrgx_update_copies_of_remote_neighbors_hood(dccrgx_grid* gp, int id) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		if (id == DCCRGX_DEFAULT_HOOD) {
			halo_start(g);
			halo_wait(g);
		} else {
			uhood_halo(g, id);
		}
		return 0;
	});
}

int dccrgx_halo_message_size(dccrgx_grid* gp, int hood, int peer, size_t* sb, size_t* rb) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		size_t a = 0, b = 0;
		halo_message_size(g, hood, peer, a, b);
		if (sb) *sb = a;
		if (rb) *rb = b;
		return 0;
	});
}

int dccrgx_halo_pack(dccrgx_grid* gp, int hood, int peer, void* buf, size_t cap) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_pack_peer(g, hood, peer, static_cast<uint8_t*>(buf), cap);
		return 0;
	});
}

int dccrgx_halo_place(dccrgx_grid* gp, int hood, int peer, const void* buf, size_t bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_place_peer(g, hood, peer, static_cast<const uint8_t*>(buf), bytes);
		return 0;
	});
}

int dccrgx_balance_load(dccrgx_grid* gp, int use_partitioner) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		initialize_balance_load_impl(g, use_partitioner != 0, nullptr, nullptr, 0);
		continue_balance_load_impl(g);
		finish_balance_load_impl(g);
		return 0;
	});
}

int dccrgx_balance_load_to(dccrgx_grid* gp, const uint64_t* cells, const int32_t* procs, size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		DX_REQUIRE((cells && procs) || !n, "null export list");
		initialize_balance_load_impl(g, false, cells, procs, n);
		continue_balance_load_impl(g);
		finish_balance_load_impl(g);
		return 0;
	});
}

int dccrgx_initialize_balance_load(dccrgx_grid* gp, int use_partitioner, const uint64_t* cells, const int32_t* procs,
                                   size_t n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE((cells && procs) || !n, "null export list");
		initialize_balance_load_impl(g, use_partitioner != 0, cells, procs, n);
		return 0;
	});
}

int dccrgx_make_new_partition(dccrgx_grid* gp, uint64_t* cells, int32_t* procs, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		std::vector<uint64_t> c;
		std::vector<int32_t> o;
		rcb_partition(g, c, o);
		if (n) *n = c.size();
		if (c.size() > cap) return DCCRGX_ERANGE;
		if (!c.empty()) {
			std::copy(c.begin(), c.end(), cells);
			std::copy(o.begin(), o.end(), procs);
		}
		return 0;
	});
}

int dccrgx_set_load_balancing_method(dccrgx_grid* gp, const char* method) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(method, "null method");
		const std::string m(method);
		// the native partitioner is RCB; "NONE" keeps the partition (pins only)
		if (m != "RCB" && m != "NONE") return DCCRGX_EINVAL;
		g.lb_method = m;
		return 0;
	});
}

int dccrgx_get_load_balancing_method(dccrgx_grid* gp, char* out, size_t cap) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(out && cap > g.lb_method.size(), "buffer too small");
		std::memcpy(out, g.lb_method.c_str(), g.lb_method.size() + 1);
		return 0;
	});
}

int dccrgx_set_cell_weight(dccrgx_grid* gp, uint64_t cell, double weight) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		if (!is_local_cell(g, cell)) return DCCRGX_ENOTFOUND;  // 6225-6235: local leaves only
		// the native partitioner cuts on fixed-point weights: a negative or
		// non-finite weight has no meaning there
		DX_REQUIRE(std::isfinite(weight) && weight >= 0 && weight * 65536.0 < 9.2e18,
		           "cell weight must be finite and non-negative");
		g.weights[cell] = weight;
		return 0;
	});
}

double dccrgx_get_cell_weight(dccrgx_grid* gp, uint64_t cell) {
	const double nan = std::numeric_limits<double>::quiet_NaN();
	if (!gp || !gp->g.initialized) return nan;
	Grid& g = gp->g;
	try {
		if (!is_local_cell(g, cell)) return nan;
	} catch (...) {
		return nan;
	}
	auto it = g.weights.find(cell);
	return it == g.weights.end() ? 1.0 : it->second;
}

int dccrgx_continue_balance_load(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		continue_balance_load_impl(g);
		return 0;
	});
}

int dccrgx_finish_balance_load(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		finish_balance_load_impl(g);
		return 0;
	});
}

int dccrgx_migration_message_size(dccrgx_grid* gp, int peer, size_t* sb, size_t* rb) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		size_t a = 0, b = 0;
		migration_message_size(g, peer, a, b);
		if (sb) *sb = a;
		if (rb) *rb = b;
		return 0;
	});
}

int dccrgx_migration_pack(dccrgx_grid* gp, int peer, void* buf, size_t cap) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		migration_pack_peer(g, peer, static_cast<uint8_t*>(buf), cap);
		return 0;
	});
}

int dccrgx_migration_place(dccrgx_grid* gp, int peer, const void* buf, size_t bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (auto& f : g.fields) f.local_zero = false;
		migration_place_peer(g, peer, static_cast<const uint8_t*>(buf), bytes);
		return 0;
	});
}

int dccrgx_save_grid_data(dccrgx_grid* gp, const char* path, uint64_t offset, const void* header,
                          size_t header_bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		save_grid_impl(g, path, offset, header, header_bytes);
		return 0;
	});
}

int dccrgx_load_grid_data(dccrgx_grid* gp, const char* path, uint64_t offset, size_t header_bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		load_grid_impl(g, path, offset, header_bytes);
		return 0;
	});
}

int dccrgx_start_loading_grid_data(dccrgx_grid* gp, const char* path, uint64_t offset, size_t header_bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		start_load_impl(g, path, offset, header_bytes);
		return 0;
	});
}

int dccrgx_continue_loading_grid_data(dccrgx_grid* gp, int field_id, const uint64_t* sizes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		for (auto& f : g.fields) f.local_zero = false;
		continue_load_impl(g, field_id, sizes);
		return 0;
	});
}

int dccrgx_finish_loading_grid_data(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.load.active, "no grid file being loaded");
		finish_load_impl(g);
		return 0;
	});
}

int dccrgx_grid_file_bytes_left(dccrgx_grid* gp, uint64_t* bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.load.active, "no grid file being loaded");
		DX_REQUIRE(bytes || !g.n_local, "null pointer");
		for (size_t s = 0; s < g.n_local; s++) bytes[s] = g.load.end[s] - g.load.pos[s];
		return 0;
	});
}

int dccrgx_add_field(dccrgx_grid* gp, const char* name, size_t elem, int transfer, int* fid) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(elem > 0, "element size must be > 0");
		Field f;
		f.name = name ? name : "";
		f.elem = elem;
		f.win_len = elem;
		f.transfer = transfer != 0;
		g.fields.push_back(std::move(f));
		Field& nf = g.fields.back();
		if (g.initialized) {
			nf.data.alloc(g.n_slots * elem);
			if (nf.data.n) HIP_CHECK(hipMemsetAsync(nf.data.p, 0, nf.data.n, g.s_comp));
		}
		*fid = int(g.fields.size() - 1);
		return 0;
	});
}

// ---- variable-size fields (tests/variable_data_size; varfield.hip) ----------
int dccrgx_add_variable_field(dccrgx_grid* gp, const char* name, int transfer, int* fid) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(fid, "null pointer");
		Field f;
		f.name = name ? name : "";
		f.var = true;
		f.transfer = transfer != 0;
		g.fields.push_back(std::move(f));
		if (g.initialized) var_reset(g.fields.back(), g.n_slots, g.s_comp);
		*fid = int(g.fields.size() - 1);
		return 0;
	});
}

static Field& var_field(Grid& g, int fid, size_t slot0, size_t n) {
	Field& f = field(g, fid);
	DX_REQUIRE(f.var, "not a variable-size field");
	DX_REQUIRE(g.initialized, "not initialized");
	DX_REQUIRE(slot0 + n <= g.n_slots, "slot range out of bounds");
	return f;
}

int dccrgx_variable_field_sizes(dccrgx_grid* gp, int fid, size_t slot0, size_t n, uint64_t* sizes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = var_field(g, fid, slot0, n);
		DX_REQUIRE(sizes || !n, "null pointer");
		const std::vector<uint64_t> o = download(f.voff.p + slot0, n + 1, g.s_comp);
		for (size_t i = 0; i < n; i++) sizes[i] = o[i + 1] - o[i];
		return 0;
	});
}

int dccrgx_variable_field_resize(dccrgx_grid* gp, int fid, size_t slot0, size_t n, const uint64_t* sizes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = var_field(g, fid, slot0, n);
		DX_REQUIRE(sizes || !n, "null pointer");
		DBuf<uint64_t> all;
		all.alloc(g.n_slots + 1);
		var_sizes(f, nullptr, 0, g.n_slots, all.p, g.s_comp);
		if (n) h2d(all.p + slot0, sizes, n * 8, g.s_comp);
		var_resize(f, g.n_slots, all.p, g.s_comp);
		return 0;
	});
}

int dccrgx_variable_field_upload(dccrgx_grid* gp, int fid, size_t slot0, size_t n, const void* bytes, size_t nbytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = var_field(g, fid, slot0, n);
		uint64_t a = 0, b = 0;
		HIP_CHECK(hipMemcpyAsync(&a, f.voff.p + slot0, 8, hipMemcpyDeviceToHost, g.s_comp));
		d2h_small(&b, f.voff.p + slot0 + n, 8, g.s_comp);
		DX_REQUIRE(nbytes == b - a, "byte count differs from the cells' sizes (resize them first)");
		if (nbytes) {
			HIP_CHECK(hipMemcpyAsync(f.data.p + a, bytes, nbytes, hipMemcpyHostToDevice, g.s_comp));
			HIP_CHECK(hipStreamSynchronize(g.s_comp));
		}
		return 0;
	});
}

int dccrgx_variable_field_download(dccrgx_grid* gp, int fid, size_t slot0, size_t n, void* bytes, size_t cap,
                                   size_t* nbytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = var_field(g, fid, slot0, n);
		uint64_t a = 0, b = 0;
		HIP_CHECK(hipMemcpyAsync(&a, f.voff.p + slot0, 8, hipMemcpyDeviceToHost, g.s_comp));
		d2h_small(&b, f.voff.p + slot0 + n, 8, g.s_comp);
		if (nbytes) *nbytes = size_t(b - a);
		if (b - a > cap) return DCCRGX_ERANGE;
		if (b > a) d2h_small(bytes, f.data.p + a, b - a, g.s_comp);
		return 0;
	});
}

int dccrgx_variable_field_device_ptr(dccrgx_grid* gp, int fid, void** data, const uint64_t** offsets) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = var_field(g, fid, 0, 0);
		if (data) *data = f.data.p;
		if (offsets) *offsets = f.voff.p;
		return 0;
	});
}

int dccrgx_removed_variable_field_download(dccrgx_grid* gp, int fid, uint64_t* sizes, void* bytes, size_t cap,
                                           size_t* nbytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = field(g, fid);
		DX_REQUIRE(f.var, "not a variable-size field");
		const size_t n = g.removed_ids.size();
		if (!n || !f.rm_off.p) {
			if (nbytes) *nbytes = 0;
			return 0;
		}
		const std::vector<uint64_t> o = download(f.rm_off.p, n + 1, g.s_comp);
		if (nbytes) *nbytes = size_t(o[n]);
		if (sizes)
			for (size_t i = 0; i < n; i++) sizes[i] = o[i + 1] - o[i];
		if (o[n] > cap) return DCCRGX_ERANGE;
		if (o[n] && bytes) d2h_small(bytes, f.removed.p, o[n], g.s_comp);
		return 0;
	});
}

// cells_to_send / cells_to_receive while a balance_load is in progress
// (initialize_balance_load fills them with the migration lists, 3746-3884)
int dccrgx_get_migration_cells(dccrgx_grid* gp, int peer, int incoming, uint64_t* ids, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.mig.active, "no balance_load in progress");
		const auto& m = incoming ? g.mig.in : g.mig.out;
		const auto it = m.find(peer);
		const size_t k = it == m.end() ? 0 : it->second.size();
		if (n) *n = k;
		if (k > cap) return DCCRGX_ERANGE;
		for (size_t i = 0; i < k; i++) ids[i] = it->second[i];
		return 0;
	});
}

// set_send_single_cells 6677 / get_send_single_cells 6684: on, the halo's
// fixed-size payloads go on the wire one cell at a time (comm.hip
// wire_pieces); the received payloads are the same either way
int dccrgx_set_send_single_cells(dccrgx_grid* gp, int on) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		g.send_single_cells = on != 0;
		return 0;
	});
}

int dccrgx_get_send_single_cells(dccrgx_grid* gp, int* on) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(on, "null pointer");
		*on = g.send_single_cells ? 1 : 0;
		return 0;
	});
}

int dccrgx_set_field_transfer(dccrgx_grid* gp, int fid, int transfer) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		field(g, fid).transfer = transfer != 0;
		return 0;
	});
}

int dccrgx_set_field_window(dccrgx_grid* gp, int fid, size_t offset, size_t bytes) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = fixed_field(g, fid);
		DX_REQUIRE(offset + bytes <= f.elem && bytes > 0, "window outside the element");
		f.win_off = offset;
		f.win_len = bytes;
		return 0;
	});
}

int dccrgx_field_device_ptr(dccrgx_grid* gp, int fid, void** ptr) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		field(g, fid).local_zero = false;
		Field& f = fixed_field(g, fid);
		field_written(f);
		f.external = true;  // writes through the pointer are not seen
		*ptr = f.data.p;
		return 0;
	});
}

int dccrgx_field_upload(dccrgx_grid* gp, int fid, size_t slot0, size_t n, const void* host) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		field(g, fid).local_zero = false;
		Field& f = fixed_field(g, fid);
		DX_REQUIRE(slot0 + n <= g.n_slots, "slot range out of bounds");
		field_written(f);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		if (n) {
			HIP_CHECK(hipMemcpyAsync(f.data.p + slot0 * f.elem, host, n * f.elem, hipMemcpyHostToDevice, g.s_comp));
			HIP_CHECK(hipStreamSynchronize(g.s_comp));
		}
		return 0;
	});
}

int dccrgx_field_download(dccrgx_grid* gp, int fid, size_t slot0, size_t n, void* host) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = fixed_field(g, fid);
		DX_REQUIRE(slot0 + n <= g.n_slots, "slot range out of bounds");
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		if (n) d2h_small(host, f.data.p + slot0 * f.elem, n * f.elem, g.s_comp);
		return 0;
	});
}

int dccrgx_update_copies_of_remote_neighbors(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_start(g);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_start_remote_neighbor_copy_updates(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_start(g);
		return 0;
	});
}

int dccrgx_wait_remote_neighbor_copy_update_receives(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_wait_remote_neighbor_copy_update_sends(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_wait_remote_neighbor_copy_updates(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		halo_wait(g);
		return 0;
	});
}

int dccrgx_gol_step(dccrgx_grid* gp, int sf, int region) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& f = field(g, sf);
		DX_REQUIRE(f.elem == 4, "game of life state must be a 4-byte field");
		ensure_scratch(g, f);
		gol_step_impl(g, f, region);
		return 0;
	});
}

int dccrgx_gol_commit(dccrgx_grid* gp, int sf) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		commit(g, field(g, sf));
		return 0;
	});
}

// get_live_neighbors of tests/game_of_life/solve.hpp:37-170, split at its
// halo: phase 0 = the collect loop (46-110), phase 1 = spread + rule
// (113-167); see gol_amr.hip
int dccrgx_gol_amr(dccrgx_grid* gp, int phase, int sf, int lf, int region) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(phase == 0 || phase == 1, "phase must be 0 (collect) or 1 (spread)");
		Field& st = field(g, sf);
		Field& ls = field(g, lf);
		DX_REQUIRE(st.elem == 4, "game of life state must be a 4-byte field");
		field_written(st);
		field_written(ls);
		DX_REQUIRE(ls.elem == 64, "live level-0 neighbor list must be a 64-byte field (8 x uint64)");
		size_t s0, s1;
		region_range(g, region, s0, s1);
		if (s1 <= s0) return 0;
		ensure_csr(g);
		DBuf<int> err;
		err.alloc(1);
		HIP_CHECK(hipMemsetAsync(err.p, 0, sizeof(int), g.s_comp));
		if (!g.gola.valid)
			k_gol_amr_tables(g.m, g.slot_ids.p, g.n_slots, g.n_local, g.hood_len, g.nof_ptr.p, g.nof_slot.p, g.gola,
			                 g.s_comp);
		k_time_begin(g);
		k_gol_amr(phase, g.gola, g.n_slots, g.n_local, (uint32_t*)st.data.p, (uint64_t*)ls.data.p, g.nof_ptr.p, g.nof_slot.p, s0,
		          s1, err.p, g.s_comp);
		k_time_end(g);
		if (phase == 0) ls.local_zero = false;
		int h = 0;
		d2h_small(&h, err.p, sizeof(int), g.s_comp);
		DX_REQUIRE(!(h & 1), "No more room in live neighbor list (more than 8 live level-0 neighbors)");
		DX_REQUIRE(!(h & 2), "a dead neighbor's level-0 parent was recorded alive (siblings disagree)");
		return 0;
	});
}

// One turn of get_live_neighbors (tests/game_of_life/solve.hpp:37-170):
// collect, the halo, spread + rule, and every local list error_cell-cleared
// at the end as the reference's rule loop leaves it (163).  Collected lists
// stay in the kernels' per-cell masks; only the cells other processes read
// (the outer run) write theirs into list_field for the halo, then clear them.
// the whole turn's error words: err[0] the collect (the geometric one's,
// replaced by err[1], the exact one's, when that had to run: err[0] bits 4 |
// 8), err[2] the spread - in the order the reference would have aborted
static void check_gol_turn_err(Grid& g, DBuf<int>& err) {
	int h[3] = {0, 0, 0};
	d2h_small(h, err.p, sizeof(h), g.s_comp);
	const int collect = (h[0] & (4 | 8)) ? h[1] : h[0];
	for (int e : {collect, h[2]}) {
		DX_REQUIRE(!(e & 1), "No more room in live neighbor list (more than 8 live level-0 neighbors)");
		DX_REQUIRE(!(e & 2), "a dead neighbor's level-0 parent was recorded alive (siblings disagree)");
	}
}

int dccrgx_get_live_neighbors(dccrgx_grid* gp, int sf, int lf) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		Field& st = field(g, sf);
		Field& ls = field(g, lf);
		DX_REQUIRE(st.elem == 4, "game of life state must be a 4-byte field");
		field_written(st);
		field_written(ls);
		DX_REQUIRE(ls.elem == 64, "live level-0 neighbor list must be a 64-byte field (8 x uint64)");
		const size_t nl = g.n_local;
		if (!nl && g.size == 1) return 0;
		ensure_csr(g);
		// err[0] the (geometric) collect, err[1] the exact collect, err[2]
		// the spread: one host read per turn, at its end
		DBuf<int> err;
		err.alloc(3);
		HIP_CHECK(hipMemsetAsync(err.p, 0, 3 * sizeof(int), g.s_comp));
		if (!g.gola.valid)
			k_gol_amr_tables(g.m, g.slot_ids.p, g.n_slots, g.n_local, g.hood_len, g.nof_ptr.p, g.nof_slot.p, g.gola,
			                 g.s_comp);
		uint64_t* L = reinterpret_cast<uint64_t*>(ls.data.p);
		uint32_t* S = reinterpret_cast<uint32_t*>(st.data.p);
		// the inner cells' lists are never written by the turn: clear them once
		const bool lean = g.gola.mask_path;
		if (lean && !ls.local_zero && g.n_inner) HIP_CHECK(hipMemsetAsync(L, 0, g.n_inner * 64, g.s_comp));
		k_time_begin(g);
		// one process: the level-0 game (gol_amr.hip), the exact collect and
		// spread only behind it (gated on the device) when a family disagrees
		const bool level0_game = lean && g.gola.geo && g.gola.lg_layout && g.size == 1 && g.n_slots == nl &&
		                         g.n_inner == nl && !std::getenv("DCCRGX_GOL_NO_L0GAME");
		if (level0_game) {
			k_gol_amr_level0_game(g.gola, g.d_hood.p, int(g.hood.size() / 3), S, nl, err.p, g.s_comp);
			k_time_end(g);
			int h[3] = {0, 0, 0};
			d2h_small(h, err.p, sizeof(h), g.s_comp);
			// every level-0 cell of a one-process grid has a known leaf
			DX_REQUIRE(!(h[0] & 8), "internal error: the level-0 game met a level-0 cell without a known leaf");
			if (h[0] & 4) {
				// a family's leaves disagree (the game pass did not run): the
				// exact collect and spread, whose abort order is the reference's
				k_time_begin(g);
				k_gol_amr(0, g.gola, g.n_slots, nl, S, L, g.nof_ptr.p, g.nof_slot.p, 0, nl, err.p + 1, g.s_comp,
				          g.n_inner);
				k_gol_amr(1, g.gola, g.n_slots, nl, S, L, g.nof_ptr.p, g.nof_slot.p, 0, nl, err.p + 2, g.s_comp, 0);
				k_time_end(g);
				d2h_small(h, err.p, sizeof(h), g.s_comp);
			}
			const int collect = (h[0] & 4) ? h[1] : h[0];
			for (int e : {collect, h[2]}) {
				DX_REQUIRE(!(e & 1), "No more room in live neighbor list (more than 8 live level-0 neighbors)");
				DX_REQUIRE(!(e & 2), "a dead neighbor's level-0 parent was recorded alive (siblings disagree)");
			}
			ls.local_zero = true;
			return 0;
		}
		if (lean && g.gola.geo) {
			// the geometric collect; the exact per-entry one (gated on the
			// device) when a family's leaves disagree or a reached level-0 cell
			// is unknown - the reference's abort conditions then depend on the
			// entry order
			k_gol_amr_geo(g.gola, g.d_hood.p, int(g.hood.size() / 3), S, nl, nl + g.n_recv, L, g.n_inner, err.p,
			              g.s_comp);
			k_gol_amr(0, g.gola, g.n_slots, nl, S, L, g.nof_ptr.p, g.nof_slot.p, 0, nl, err.p + 1, g.s_comp, g.n_inner,
			          err.p);
		} else {
			k_gol_amr(0, g.gola, g.n_slots, nl, S, L, g.nof_ptr.p, g.nof_slot.p, 0, nl, err.p, g.s_comp,
			          lean ? g.n_inner : 0);
		}
		k_time_end(g);
		halo_start(g);  // update_copies_of_remote_neighbors (solve.hpp:111)
		halo_wait(g);
		k_time_begin(g);
		k_gol_amr(1, g.gola, g.n_slots, nl, S, L, g.nof_ptr.p, g.nof_slot.p, 0, nl, err.p + 2, g.s_comp);
		k_time_end(g);
		const size_t c0 = lean ? g.n_inner : 0;
		if (nl > c0) HIP_CHECK(hipMemsetAsync(L + c0 * 8, 0, (nl - c0) * 64, g.s_comp));
		check_gol_turn_err(g, err);
		ls.local_zero = true;
		return 0;
	});
}

int dccrgx_advection_step(dccrgx_grid* gp, const int fids[7], double dt, int region) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const double* f[7];
		adv_fields(g, fids, f);
		Field& rho = field(g, fids[0]);
		ensure_scratch(g, rho);
		size_t s0, s1;
		region_range(g, region, s0, s1);
		if (s1 <= s0) return 0;
		DX_LAPS(g.s_comp);
		// tiles for a mesh already swept once (DCCRGX_TILES=always / never
		// overrides): building them costs ~10 sweeps, so the first step on a
		// freshly adapted mesh sweeps the face table (bitwise the same
		// densities)
		static const char* tp = std::getenv("DCCRGX_TILES");
		const bool tiles = g.tiles_valid || (tp && std::strcmp(tp, "always") == 0) ||
		                   (!(tp && std::strcmp(tp, "never") == 0) && g.adv_commits_on_mesh > 0);
		if (tiles) ensure_tiles(g);
		else ensure_face(g);
		DX_LAP("step.0_ensure_tiles");
		if (tiles) {
			// (outside the timed interval: a rebuild happens once per mesh or
			// field change, not per step)
			const double* rec = ensure_nbrec(g, fids);
			DX_LAP("step.0_nbrec");
			k_time_begin(g);
			// tiles never straddle the inner / outer runs
			if (s0 < g.n_inner) k_advection_tiles(f, (double*)rho.scratch.p, g, 0, dt, g.s_comp, rec);
			if (s1 > g.n_inner) k_advection_tiles(f, (double*)rho.scratch.p, g, 1, dt, g.s_comp, rec);
		} else {
			// the bands of the check that follows computed by the sweep (with the
			// last check's parameters), recorded per run for band_cache_ok
			const char* bc = std::getenv("DCCRGX_BAND_CACHE");  // read per call: tests switch it
			const bool bands = g.band_params_valid && !(bc && bc[0] == '0') && !rho.external;
			BandArgs B{};
			if (bands) {
				if (g.band_cache.n < g.n_local + 1) {
					g.band_cache.alloc(g.n_local + 1);
					g.band_rec[0].valid = g.band_rec[1].valid = false;
				}
				B = BandArgs{g.m, g.slot_lvl.p, g.slot_ids.p, g.band_inc, g.band_thr, g.band_uns, g.band_cache.p};
				for (int run = 0; run < 2; run++) {
					const size_t r0 = run == 0 ? 0 : g.n_inner, r1 = run == 0 ? g.n_inner : g.n_local;
					if (r1 > r0 && s0 <= r0 && s1 >= r1)
						g.band_rec[run] = Grid::BandRec{true, g.face_gen, rho.epoch, rho.local_epoch, rho.data.p};
				}
			}
			k_time_begin(g);
			k_advection_ell(f, (double*)rho.scratch.p, g.face_ell.p, g.face_fine.p, s0, s1, dt, g.s_comp,
			                bands ? &B : nullptr);
		}
		k_time_end(g);
		DX_LAP("step.1_sweep");
		return 0;
	});
}

int dccrgx_advection_layout(dccrgx_grid* gp, uint64_t out[12]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(out, "null output");
		ensure_tiles(g);
		const uint64_t nt = g.n_tiles_inner + g.n_tiles_outer;
		uint32_t entries = 0;
		d2h_small(&entries, g.face_ptr.p + g.n_local, 4, g.s_comp);
		const uint64_t n = g.n_local;
		out[0] = uint64_t(g.tile);
		out[1] = nt;
		out[2] = g.total_ext;
		out[3] = g.max_ext;
		out[4] = g.n_fine_faces;
		out[5] = entries;
		// 64 B per cell (7 fp64 fields read, density written) +
		// the face CSR (4 B per entry + 4 B row pointer)
		out[6] = 64 * n + 4 * (n + 1) + 4 * uint64_t(entries);
		out[7] = 64 * n;
		const size_t nreg = g.tcount[0] + g.tcount[1];
		out[8] = nreg;
		out[9] = 512 * nreg;
		uint64_t ext_reg = 0;
		if (nreg) {
			std::vector<RegTileMeta> rm(nreg);
			d2h_small(rm.data(), g.tregmeta.p, nreg * sizeof(RegTileMeta), g.s_comp);
			for (const auto& r : rm)
				for (int d = 0; d < 6; d++) ext_reg += r.nst[d] >= 0 ? 64 : 0;
		}
		out[10] = ext_reg;
		// 40 B per out-of-tile neighbor from the fields (density, three
		// lengths, the velocity along the face); 32 B with the records
		// (DCCRGX_NBREC=1, ensure_nbrec)
		const char* env = std::getenv("DCCRGX_NBREC");
		const bool rec_off = !(env && std::atoi(env) == 1);
		const uint64_t per_ext = rec_off ? 40 : 32;
		const uint64_t n_irr_cells = n - out[9], ext_irr = g.total_ext - ext_reg;
		out[11] = 64 * n + 12 * n_irr_cells + (per_ext + 4) * ext_irr + per_ext * ext_reg + 8 * uint64_t(g.n_fine_faces) +
		          32 * nt;
		return 0;
	});
}

int dccrgx_advection_commit(dccrgx_grid* gp, int df) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		commit(g, field(g, df));
		g.adv_commits_on_mesh++;
		return 0;
	});
}

// tests/advection/initialize.hpp:36-82 + Cartesian_Geometry get_center /
// get_length (dccrg_cartesian_geometry.hpp:282-362), evaluated on the host
// with the reference's expression order so the initial state is bitwise the
// reference's.
int dccrgx_advection_initialize(dccrgx_grid* gp, const int fids[7]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		// local cells and remote copies alike: the analytic initial state of a
		// remote copy is what initialize() + update_copies_of_remote_neighbors()
		// with transfer_all_data = true would deliver (initialize.hpp:80)
		const auto& ids = slot_ids_host(g);
		const size_t n = g.n_slots;
		std::vector<double> a[7];
		for (auto& v : a) v.resize(n);
		for (size_t i = 0; i < n; i++) {
			uint64_t ind[3];
			const int lvl = map_indices(g.m, ids[i], ind[0], ind[1], ind[2]);
			const double sf = 1.0 / double(uint64_t(1) << lvl);
			double L[3], c[3];
			for (int d = 0; d < 3; d++) L[d] = g.l0[d] * sf;
			for (int d = 0; d < 3; d++)
				c[d] = g.start[d] + double(ind[d]) * g.l0[d] / double(uint64_t(1) << g.R) + L[d] / 2;
			const double radius = 0.15;
			const double hr = std::min(std::sqrt(std::pow(c[0] - 0.25, 2.0) + std::pow(c[1] - 0.5, 2.0)), radius) / radius;
			a[0][i] = 0.25 * (1 + std::cos(M_PI * hr));
			a[1][i] = -c[1] + 0.5;
			a[2][i] = +c[0] - 0.5;
			a[3][i] = 0;
			a[4][i] = L[0];
			a[5][i] = L[1];
			a[6][i] = L[2];
		}
		for (int k = 0; k < 7; k++) {
			Field& F = field(g, fids[k]);
			DX_REQUIRE(F.elem == 8, "advection fields must be fp64");
			field_written(F);
			if (n) {
				HIP_CHECK(hipMemcpyAsync(F.data.p, a[k].data(), n * 8, hipMemcpyHostToDevice, g.s_comp));
				HIP_CHECK(hipStreamSynchronize(g.s_comp));
			}
		}
		return 0;
	});
}

// the block minima of the time-step bound of fields fids in g.dt_part (their
// count): the cached ones while the six velocity / length fields are
// unwritten since (advection_adapt's reset pass leaves them), else one pass
static size_t dt_partials(Grid& g, const int fids[7]) {
	const double* f[7];
	adv_fields(g, fids, f);
	Grid::DtCache& C = g.dt_cache;
	bool ok = C.valid && C.n_local == g.n_local && C.nb > 0;
	for (int k = 1; k < 7 && ok; k++) ok = C.fid[k - 1] == fids[k] && C.epoch[k - 1] == field(g, fids[k]).epoch;
	if (ok) return C.nb;
	const size_t nb = 512;
	g.dt_part.reserve(kDtPartials);
	k_adv_dt(f, g.n_local, g.dt_part.p, nb, g.s_comp);
	dt_cache_set(g, fids, nb);
	return nb;
}

int dccrgx_advection_max_time_step(dccrgx_grid* gp, const int fids[7], double* out) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		const size_t nb = dt_partials(g, fids);
		auto h = download(g.dt_part.p, nb, g.s_comp);
		*out = *std::min_element(h.begin(), h.end());
		return 0;
	});
}

int dccrgx_advection_max_time_step_device(dccrgx_grid* gp, const int fids[7], double* d_out) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(d_out != nullptr, "null device pointer");
		const size_t nb = dt_partials(g, fids);
		k_min_partials(g.dt_part.p, nb, d_out, g.s_comp);
		comm_allreduce_f64_dev(g, d_out, d_out, 1, 1, g.s_comp);
		return 0;
	});
}

int dccrgx_advection_refine_candidates(dccrgx_grid* gp, int df, double diff_increase, double diff_threshold,
                                       uint64_t* out, size_t cap, size_t* n) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		ensure_face(g);
		Field& F = field(g, df);
		DBuf<uint64_t> d;
		d.alloc(g.n_local + 1);
		const FaceView fv{g.face_ell.p, g.face_fine.p, g.slot_ids.p, g.n_local};
		const size_t k = k_adv_candidates(g.m, (const double*)F.data.p, fv, g.slot_lvl.p, g.n_local, diff_increase,
		                                  diff_threshold, d.p, g.s_comp);
		auto v = download(d.p, k, g.s_comp);
		std::sort(v.begin(), v.end());
		return copy_out_u64(v, out, cap, n);
	});
}

// The sweep's bands (advection_step) stand for adv_bands_kernel's when the
// same parameters were given, the face table is the one swept, and the
// density array has not been written since: the inner run reads no remote
// copy, so only local writes matter there; the outer run's rows read the
// copies the halo placed before it.
static bool band_cache_ok(Grid& g, const Field& F, double inc, double thr, double uns) {
	if (!g.band_params_valid || g.band_inc != inc || g.band_thr != thr || g.band_uns != uns || F.external) return false;
	if (g.band_cache.n < g.n_local + 1 || !g.face_valid) return false;
	for (int run = 0; run < 2; run++) {
		const size_t r0 = run == 0 ? 0 : g.n_inner, r1 = run == 0 ? g.n_inner : g.n_local;
		if (r1 <= r0) continue;
		const Grid::BandRec& R = g.band_rec[run];
		if (!R.valid || R.face_gen != g.face_gen || R.rho != F.data.p || R.local_epoch != F.local_epoch) return false;
		if (run == 1 && R.epoch != F.epoch) return false;
	}
	return true;
}

// check_for_adaptation (tests/advection/adapter.hpp:47-178) + the requests
// adapt_grid makes from its sets (187-231): per local cell the band of its
// max_diff; band-2 cells are refined, a family with a band-1 member is kept
// (dont_unrefine), a family whose local members are all band 0 is unrefined.
// The reference builds the sets in local-cell order with sibling erasures;
// their outcome per family is the one above, whatever the order.  A family
// with a band-2 member is also marked kept: on one process the reference's
// sibling erasure keeps it even when that member is at the maximum level
// (whose refine request is a no-op); marking it makes every partition give
// that one-process outcome.
int dccrgx_advection_check_adaptation(dccrgx_grid* gp, int df, double diff_increase, double diff_threshold,
                                      double unrefine_sensitivity, uint64_t counts[3]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		Field& F = field(g, df);
		DX_REQUIRE(F.elem == 8, "advection fields must be fp64");
		if (counts) counts[0] = counts[1] = counts[2] = 0;
		if (g.R == 0) return 0;  // 61-63
		DX_LAPS(g.s_comp);
		ensure_face(g);
		DX_LAP("chk.0_face");
		const size_t n = g.n_local;
		DBuf<uint8_t> band_own;
		const uint8_t* band = nullptr;
		if (band_cache_ok(g, F, diff_increase, diff_threshold, unrefine_sensitivity)) {
			band = g.band_cache.p;  // the sweep's (advection_step)
		} else {
			band_own.alloc(n + 1);
			const FaceView fv{g.face_ell.p, g.face_fine.p, g.slot_ids.p, g.n_local};
			k_adv_bands(g.m, (const double*)F.data.p, fv, g.slot_lvl.p, n, diff_increase, diff_threshold,
			            unrefine_sensitivity, band_own.p, g.s_comp);
			band = band_own.p;
		}
		g.band_rec[0].valid = g.band_rec[1].valid = false;
		g.band_params_valid = true;  // the next sweeps compute the bands with these
		g.band_inc = diff_increase;
		g.band_thr = diff_threshold;
		g.band_uns = unrefine_sensitivity;
		DX_LAP("chk.1_bands");
		uint64_t nref = 0, nkeep = 0, nunref = 0;
		// decide one family from its local members (bands bb, ids ii, k of
		// them): dont_unrefine (2679-2733) when any member is kept or refined,
		// else unrefine it
		auto decide = [&](const uint8_t* bb, const uint64_t* ii, size_t k) {
			size_t first2 = k, first1 = k;
			for (size_t i = 0; i < k; i++) {
				if (bb[i] == 2 && first2 == k) first2 = i;
				if (bb[i] == 1 && first1 == k) first1 = i;
			}
			if (first2 != k || first1 != k) {
				// the mark can only cancel an unrefine request of this family: one
				// from another process (a family split across processes, k < 8)
				// or one made earlier here; a whole local family without a pending
				// request needs no mark (the outcome of stop_refining is the same)
				bool pending = k < 8;
				for (size_t i = 0; i < k && !pending && !g.unrefine_requests.empty(); i++)
					pending = g.unrefine_requests.count(ii[i]) != 0;
				if (pending) g.dont_unrefine_cells.insert(ii[first2 != k ? first2 : first1]);
				nkeep++;
			} else if (k == 8) {  // the whole family is local: every sibling a leaf here
				g.unrefine_requests.insert(ii[0]);
				nunref++;
			} else if (dccrgx_unrefine_completely(gp, ii[0]) == DCCRGX_OK) {
				nunref++;
			}
		};
		// families: the local members of a parent are consecutive slots on
		// Morton-ordered meshes (a run of 8 is a whole family); shorter runs
		// (a family split between the inner and outer runs, or with members
		// elsewhere) are merged by parent
		std::unordered_map<uint64_t, std::pair<std::vector<uint8_t>, std::vector<uint64_t>>> partial;
		auto add_partial = [&](uint64_t parent, uint8_t band_v, uint64_t id) {
			auto& pr = partial[parent];
			pr.first.push_back(band_v);
			pr.second.push_back(id);
		};
		flush_bulk_requests(g);
		if (g.unrefine_requests.empty() && n < (size_t(1) << 28)) {
			// on the device: refine requests, whole-family decisions, partial runs
			// one process with Morton-ordered slots: each family's leaves are one run
			const bool solo = g.size == 1 && g.morton_slots;
			AdvRequests q = k_adv_requests(g.m, g.dm(), g.slot_ids.p, band, n, solo, g.rank, g.s_comp);
			DX_LAP("chk.2a_device_requests");
			// 2434-2520 (bulk lists: no set hashing of ~20 K ids per step)
			g.refine_bulk.insert(g.refine_bulk.end(), q.refine.begin(), q.refine.end());
			if (g.refine_requests.empty() && !q.refine.empty()) {
				// the whole refine request set: its device copy stays for stop_refining
				g.refine_dev = std::move(q.refine_dev);
				g.refine_dev_valid = true;
			}
			if (g.unrefine_requests.empty() && !q.unrefine.empty()) {
				g.unrefine_dev = std::move(q.unrefine_dev);
				g.unrefine_dev_valid = true;
			}
			nref = q.refine.size();
			nkeep = q.kept;
			g.unrefine_bulk.insert(g.unrefine_bulk.end(), q.unrefine.begin(), q.unrefine.end());
			nunref = q.unrefine.size();
			size_t at = 0;
			for (size_t r = 0; r < q.part_slot.size(); r++) {
				const uint64_t parent = map_parent(g.m, q.part_ids[at]);
				for (uint32_t j = 0; j < q.part_len[r]; j++, at++) add_partial(parent, q.part_bands[at], q.part_ids[at]);
			}
		} else {
			// unrefine requests pending from before (or more local cells than
			// the device runs encode): the same walk on the host
			const std::vector<uint8_t> b = download(band, n, g.s_comp);
			const auto& ids = slot_ids_host(g);
			std::vector<uint8_t> rb;
			std::vector<uint64_t> ri;
			uint64_t run_parent = error_cell;
			auto flush = [&] {
				if (ri.empty()) return;
				if (ri.size() == 8) decide(rb.data(), ri.data(), 8);
				else
					for (size_t i = 0; i < ri.size(); i++) add_partial(run_parent, rb[i], ri[i]);
				rb.clear();
				ri.clear();
			};
			for (size_t s = 0; s < n; s++) {
				const int lvl = map_level(g.m, ids[s]);
				if (b[s] == 2 && lvl < g.R) {
					g.refine_requests.insert(ids[s]);  // 2434-2520: a local leaf below the maximum level
					nref++;
				}
				if (lvl == 0) {
					flush();
					run_parent = error_cell;
					continue;
				}
				const uint64_t p = map_parent(g.m, ids[s]);
				if (p != run_parent) {
					flush();
					run_parent = p;
				}
				rb.push_back(b[s]);
				ri.push_back(ids[s]);
			}
			flush();
		}
		DX_LAP("chk.2_requests");
		for (auto& kv : partial) decide(kv.second.first.data(), kv.second.second.data(), kv.second.first.size());
		DX_LAP("chk.3_partial_families");
		if (counts) {
			counts[0] = nref;
			counts[1] = nkeep;
			counts[2] = nunref;
		}
		return 0;
	});
}

// adapt_grid (tests/advection/adapter.hpp:232-309): stop_refining, the new
// children carry their parent's payload (density = parent's, 247), a merged
// parent's density = its removed children's / 8 (260-290), velocities and
// lengths of every local cell reset (294-305), then a halo of all seven
// fields (transfer_all_data, 2d.cpp:400-407).  out: created, removed cells.
int dccrgx_advection_adapt(dccrgx_grid* gp, const int fids[7], uint64_t out[2]) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "not initialized");
		const double* cf[7];
		adv_fields(g, fids, cf);
		DX_LAPS(g.s_comp);
		// velocities and lengths are reset for every local cell below
		// (adapter.hpp:292-309): the rebuild need not carry them (the removed
		// store still gets them, packed before the rebuild)
		for (int k = 1; k < 7; k++)
			if (fids[k] != fids[0]) field(g, fids[k]).no_carry = true;
		try {
			stop_refining_impl(g);
		} catch (...) {
			for (int k = 1; k < 7; k++) field(g, fids[k]).no_carry = false;
			throw;
		}
		for (int k = 1; k < 7; k++) field(g, fids[k]).no_carry = false;  // no rebuild ran (nothing changed)
		DX_LAP("adapt.1_stop_refining");
		hipStream_t s = g.s_comp;
		double* f[7];
		for (int k = 0; k < 7; k++) {
			f[k] = (double*)field(g, fids[k]).data.p;
			field_written(field(g, fids[k]));
		}
		// merged parents (adapter.hpp:260-290): the removed children grouped by
		// parent on the device, each parent's mean of its eight children
		k_adv_merge_parents(g.m, g.dm(), g.n_local, g.removed_ids, f[0], (const double*)field(g, fids[0]).removed.p, s,
		                    g.merged_dev.p, g.n_merged);
		DX_LAP("adapt.2_parents");
		// the reset pass also leaves the next time step's block minima
		g.dt_part.reserve(kDtPartials);
		const size_t nb = k_adv_reset(g.m, g.slot_ids.p, g.n_local, g.start, g.l0, f, s, g.dt_part.p);
		dt_cache_set(g, fids, nb);
		HIP_CHECK(hipStreamSynchronize(s));
		DX_LAP("adapt.3_reset");
		// transfer_all_data: every field of the seven in this halo
		bool saved[7];
		for (int k = 0; k < 7; k++) {
			Field& F = field(g, fids[k]);
			saved[k] = F.transfer;
			F.transfer = true;
		}
		try {
			halo_start(g);
			halo_wait(g);
		} catch (...) {
			for (int k = 0; k < 7; k++) field(g, fids[k]).transfer = saved[k];
			throw;
		}
		for (int k = 0; k < 7; k++) field(g, fids[k]).transfer = saved[k];
		DX_LAP("adapt.4_halo");
		if (out) {
			out[0] = g.new_cells.size();
			out[1] = g.removed_ids.size();
		}
		return 0;
	});
}

int dccrgx_allreduce_f64(dccrgx_grid* gp, double* v, int count, int op) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		comm_allreduce_f64(g, v, count, op);
		return 0;
	});
}

int dccrgx_allreduce_f64_device(dccrgx_grid* gp, const double* d_in, double* d_out, int count, int op) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(count >= 0 && (count == 0 || (d_in && d_out)), "allreduce: null device buffer");
		comm_allreduce_f64_dev(g, d_in, d_out, count, op, g.s_comp);
		return 0;
	});
}

int dccrgx_barrier(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		double z = 0;
		comm_allreduce_f64(g, &z, 1, 0);
		return 0;
	});
}

int dccrgx_get_transport(dccrgx_grid* gp, int* kind, int* comm_ranks) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		int k = DCCRGX_TRANSPORT_NONE, n = 1;
		if (g.xfn) {
			k = DCCRGX_TRANSPORT_HOST;
			n = g.size;
		} else if (g.nccl) {
			k = DCCRGX_TRANSPORT_RCCL;
			NCCL_CHECK(ncclCommCount(g.nccl, &n));
		}
		if (kind) *kind = k;
		if (comm_ranks) *comm_ranks = n;
		return 0;
	});
}

int dccrgx_comm_loopback(dccrgx_grid* gp, int field_id, size_t slot0, size_t n, size_t dst_slot0) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.nccl && !g.xfn, "loopback needs the RCCL transport");
		Field& f = field(g, field_id);
		DX_REQUIRE(!f.var, "loopback of a variable-size field");
		DX_REQUIRE(slot0 + n <= g.n_slots && dst_slot0 + n <= g.n_slots, "slot range beyond the field");
		DX_REQUIRE(slot0 + n <= dst_slot0 || dst_slot0 + n <= slot0, "overlapping slot ranges");
		f.local_zero = false;  // the receive may land in local slots
		field_written(f);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));  // the field's producers
		comm_loopback(g, f.data.p + slot0 * f.elem, f.data.p + dst_slot0 * f.elem, n * f.elem,
		              g.send_single_cells ? f.elem : 0, g.s_comm);
		HIP_CHECK(hipStreamSynchronize(g.s_comm));
		return 0;
	});
}

int dccrgx_synchronize(dccrgx_grid* gp) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		HIP_CHECK(hipStreamSynchronize(g.s_comm));
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		return 0;
	});
}

void* dccrgx_compute_stream(dccrgx_grid* gp) { return gp ? (void*)gp->g.s_comp : nullptr; }

int dccrgx_kernel_timing(dccrgx_grid* gp, int enable, double* total_ms, int64_t* count) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		drain_timing(g);
		if (total_ms) *total_ms = g.timed_ms;
		if (count) *count = g.timed_count;
		if (enable == 1) {
			g.timing = true;
			g.timed_ms = 0;
			g.timed_count = 0;
		} else if (enable == 0) {
			g.timing = false;
		}
		return 0;
	});
}

// ---- Poisson (tests/poisson/poisson_solve.hpp) ----------------------------
int dccrgx_poisson_cache(dccrgx_grid* gp, int rhs_field, int solution_field, const uint64_t* solve_cells,
                         size_t n_solve, const uint64_t* skip_cells, size_t n_skip) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(g.initialized, "grid not initialized");
		DX_REQUIRE((solve_cells || !n_solve) && (skip_cells || !n_skip), "null cell list");
		po_cache(g, rhs_field, solution_field, solve_cells, n_solve, skip_cells, n_skip);
		return 0;
	});
}

int dccrgx_poisson_solve(dccrgx_grid* gp, unsigned max_iterations, unsigned min_iterations, double stop_residual,
                         double p_of_norm, double stop_after_residual_increase, int failsafe, unsigned* iterations,
                         double* residual) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(p_of_norm > 0, "p_of_norm must be > 0");
		// solve() is a do-while (279-506): at least one iteration
		const unsigned max_it = failsafe ? max_iterations : std::max(1u, max_iterations);
		const PoParams prm{max_it, min_iterations, stop_residual, p_of_norm, stop_after_residual_increase};
		const PoScalars st = po_solve(g, prm, failsafe != 0);
		if (iterations) *iterations = st.iteration;
		if (residual) *residual = failsafe ? st.norm : st.residual_min;
		return 0;
	});
}

int dccrgx_poisson_field(dccrgx_grid* gp, const char* name, int* fid) {
	return guard([&] {
		GRID_OR_FAIL(gp);
		DX_REQUIRE(name && fid, "null argument");
		DX_REQUIRE(g.po.type >= 0, "Poisson system not cached yet");
		const std::string want = std::string("poisson.") + name;
		for (size_t i = 0; i < g.fields.size(); i++)
			if (g.fields[i].name == want) {
				*fid = int(i);
				return 0;
			}
		throw Error(DCCRGX_ENOTFOUND, "no Poisson field " + std::string(name));
	});
}

}  // extern "C"
