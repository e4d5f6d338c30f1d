// Collectives and point-to-point transfers of one grid.
//
// The reference talks MPI: Allgather(v) / Allreduce for the control plane
// (dccrg_mpi_support.hpp:98-275), Isend / Irecv of derived datatypes for
// payloads (start_user_data_transfers, dccrg.hpp:10564-10997).  Here every
// transfer is a list of device-buffer messages (DevMsg: peer, send pointer
// and size, receive pointer and size), built by the same code whatever the
// transport, and handed to one byte mover (`move_bytes`), the only place
// the transports differ:
//   - RCCL (the grid was created with a bootstrap id): one grouped
//     ncclSend / ncclRecv per message over xGMI, device to device;
//   - a caller-provided host exchange (dccrgx_create_with_exchange): the
//     messages of a peer are staged through one host buffer each way and
//     moved by one grouped point-to-point exchange (MPI in the C++ facade
//     when ranks share a GPU, torch.distributed in tests).
// The collectives are message lists too: sizes, all-to-all and all-gather
// go through move_bytes; reductions all-gather the per-rank values and
// combine them in rank order on every rank, so results do not depend on the
// transport (no ncclAllReduce, whose summation order is RCCL's own).
#include <algorithm>
#include <cstring>

#include "dccrgx_internal.hpp"

namespace dccrgx {

void comm_require(const Grid& g, const char* what) {
	if (!g.has_collectives())
		throw Error(DCCRGX_EINVAL, std::string(what) +
		                               " needs a communicator (grid created without an RCCL id or an exchange function)");
}

// The wire: per direction a list of (peer, pointer, bytes) pieces.  A
// message is one piece each way, except under send_single_cells (6658-6681,
// start_user_data_transfers 10613-10692: one MPI message per cell, in the
// cells' order): then the consecutive messages of a peer that are runs of
// cells (DevMsg::cell) go out cell by cell, each cell's pieces in message
// (field) order, so the wire carries the reference's per-cell sequence.  The
// pieces land where their messages point, so the bytes placed are the same
// either way.
struct Piece {
	int peer;
	uint8_t* p;
	size_t n;
};

static void wire_pieces(const std::vector<DevMsg>& msgs, bool single, std::vector<Piece>& snd, std::vector<Piece>& rcv) {
	for (size_t i = 0; i < msgs.size();) {
		size_t j = i;
		while (j < msgs.size() && msgs[j].peer == msgs[i].peer) j++;
		for (int dir = 0; dir < 2; dir++) {
			auto bytes = [&](const DevMsg& m) { return dir == 0 ? m.send_bytes : m.recv_bytes; };
			auto ptr = [&](const DevMsg& m) {
				return dir == 0 ? const_cast<uint8_t*>(m.send) : m.recv;
			};
			std::vector<Piece>& out = dir == 0 ? snd : rcv;
			// cells per message of the run, when every message is a run of as many
			size_t cells = 0;
			bool split = single;
			for (size_t k = i; k < j && split; k++) {
				const DevMsg& m = msgs[k];
				split = m.cell > 0 && bytes(m) % m.cell == 0 && (k == i || bytes(m) / m.cell == cells);
				if (split) cells = bytes(m) / m.cell;
			}
			if (split) {
				for (size_t c = 0; c < cells; c++)
					for (size_t k = i; k < j; k++) out.push_back({msgs[k].peer, ptr(msgs[k]) + c * msgs[k].cell, msgs[k].cell});
			} else {
				for (size_t k = i; k < j; k++)
					if (bytes(msgs[k])) out.push_back({msgs[k].peer, ptr(msgs[k]), bytes(msgs[k])});
			}
		}
		i = j;
	}
}

// Pieces per peer and direction in one RCCL group.  Under send_single_cells
// a config-5 face plane is ~10^6 pieces per peer; one group of that many
// ncclSend / ncclRecv is past what RCCL is built for, so the pieces go out in
// rounds: round j holds, for every peer and direction, that peer's pieces
// [j K, (j + 1) K).  A pair's sends of round j are the peer's receives of round
// j (both sides build the same wire), so every round completes on its own
// and the posting order of a pair - the per-cell wire order - is kept.
constexpr size_t kPiecesPerGroup = 4096;

// consecutive pieces to one peer that continue each other in memory become
// one piece (same bytes, same order)
static void coalesce(std::vector<Piece>& v) {
	size_t o = 0;
	for (size_t i = 0; i < v.size(); i++) {
		if (o && v[o - 1].peer == v[i].peer && v[o - 1].p + v[o - 1].n == v[i].p) {
			v[o - 1].n += v[i].n;
		} else {
			v[o++] = v[i];
		}
	}
	v.resize(o);
}

// The byte mover.  Pieces to / from one peer keep their order (the wire
// order): RCCL matches a pair's sends and receives in posting order, the host
// exchange concatenates them in that order.  Returns with the transfer
// queued on `s` (RCCL) or completed (host exchange).
static void move_bytes(Grid& g, const std::vector<DevMsg>& msgs, hipStream_t s) {
	std::vector<Piece> snd, rcv;
	wire_pieces(msgs, g.send_single_cells, snd, rcv);
	if (g.nccl && !g.xfn) {
		// each piece's index among its peer's pieces of its direction
		auto rank_in_peer = [&](const std::vector<Piece>& v, std::vector<size_t>& idx) {
			std::vector<size_t> cnt(size_t(g.size), 0);
			idx.resize(v.size());
			size_t most = 0;
			for (size_t i = 0; i < v.size(); i++) {
				idx[i] = cnt[size_t(v[i].peer)]++;
				most = std::max(most, idx[i] + 1);
			}
			return most;
		};
		std::vector<size_t> si, ri;
		const size_t rounds = (std::max(rank_in_peer(snd, si), rank_in_peer(rcv, ri)) + kPiecesPerGroup - 1) /
		                      kPiecesPerGroup;
		if (rounds <= 1) {
			NCCL_CHECK(ncclGroupStart());
			for (const auto& m : snd) NCCL_CHECK(ncclSend(m.p, m.n, ncclUint8, m.peer, g.nccl, s));
			for (const auto& m : rcv) NCCL_CHECK(ncclRecv(m.p, m.n, ncclUint8, m.peer, g.nccl, s));
			NCCL_CHECK(ncclGroupEnd());
			return;
		}
		for (size_t j = 0; j < rounds; j++) {
			const size_t lo = j * kPiecesPerGroup, hi = lo + kPiecesPerGroup;
			NCCL_CHECK(ncclGroupStart());
			for (size_t i = 0; i < snd.size(); i++)
				if (si[i] >= lo && si[i] < hi) NCCL_CHECK(ncclSend(snd[i].p, snd[i].n, ncclUint8, snd[i].peer, g.nccl, s));
			for (size_t i = 0; i < rcv.size(); i++)
				if (ri[i] >= lo && ri[i] < hi) NCCL_CHECK(ncclRecv(rcv[i].p, rcv[i].n, ncclUint8, rcv[i].peer, g.nccl, s));
			NCCL_CHECK(ncclGroupEnd());
		}
		return;
	}
	// the host exchange carries one byte stream per peer and direction, so
	// piece boundaries are this side's own business: contiguous pieces are
	// copied at once (a single-field halo under send_single_cells is one copy
	// per peer, not one per cell)
	DX_PHASE_COMM("comm.host_move_bytes", s);
	coalesce(snd);
	coalesce(rcv);
	const size_t P = size_t(g.size);
	std::vector<size_t> sb(P, 0), rb(P, 0);
	for (const auto& m : msgs) DX_REQUIRE(m.peer >= 0 && m.peer < g.size && m.peer != g.rank, "message to an invalid peer");
	for (const auto& m : snd) sb[size_t(m.peer)] += m.n;
	for (const auto& m : rcv) rb[size_t(m.peer)] += m.n;
	// one pinned staging area: the send bytes of every peer, then the
	// receive bytes (grow-only, kept by the grid)
	std::vector<size_t> sbase(P, 0), rbase(P, 0);
	size_t tot = 0;
	for (size_t p = 0; p < P; p++) {
		sbase[p] = tot;
		tot += sb[p];
	}
	for (size_t p = 0; p < P; p++) {
		rbase[p] = tot;
		tot += rb[p];
	}
	if (tot > g.pin_stage_cap) {
		HIP_CHECK(hipStreamSynchronize(s));
		if (g.pin_stage) HIP_CHECK(hipHostFree(g.pin_stage));
		g.pin_stage = nullptr;
		g.pin_stage_cap = 0;
		const size_t cap = std::max(tot + tot / 4, size_t(1) << 20);
		HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&g.pin_stage), cap, hipHostMallocDefault));
		g.pin_stage_cap = cap;
	}
	uint8_t* const pin = g.pin_stage;
	std::vector<size_t> so(P, 0), ro(P, 0);
	HIP_CHECK(hipStreamSynchronize(s));  // the send buffers are complete
	for (const auto& m : snd) {
		const size_t p = size_t(m.peer);
		HIP_CHECK(hipMemcpyAsync(pin + sbase[p] + so[p], m.p, m.n, hipMemcpyDefault, s));
		so[p] += m.n;
	}
	HIP_CHECK(hipStreamSynchronize(s));
	std::vector<const void*> sp(P, nullptr);
	std::vector<void*> rp(P, nullptr);
	for (size_t p = 0; p < P; p++) {
		sp[p] = pin + sbase[p];
		rp[p] = pin + rbase[p];
	}
#if DCCRGX_PHASE_TIMING
	const double tx0 = PhaseScope::now();
#endif
	DX_REQUIRE(g.xfn(g.xctx, sp.data(), sb.data(), rp.data(), rb.data()) == 0, "exchange function failed");
#if DCCRGX_PHASE_TIMING
	phase_add("comm.xfn_wait", PhaseScope::now() - tx0);
#endif
	for (const auto& m : rcv) {
		const size_t p = size_t(m.peer);
		HIP_CHECK(hipMemcpyAsync(m.p, pin + rbase[p] + ro[p], m.n, hipMemcpyDefault, s));
		ro[p] += m.n;
	}
	HIP_CHECK(hipStreamSynchronize(s));
}

void comm_device_transfer(Grid& g, const std::vector<DevMsg>& msgs, hipStream_t s) {
	if (g.size == 1) return;
	comm_require(g, "payload transfer");
	move_bytes(g, msgs, s);
}

// one message to this rank itself through the RCCL branch of the byte mover
// (a grouped ncclSend / ncclRecv pair; a host exchange has no self peer);
// `cell` > 0: a run of cells of that many bytes each, which send_single_cells
// puts on the wire cell by cell
void comm_loopback(Grid& g, const void* send, void* recv, size_t bytes, size_t cell, hipStream_t s) {
	DX_REQUIRE(g.nccl && !g.xfn, "loopback needs the RCCL transport");
	move_bytes(g, {DevMsg{g.rank, static_cast<const uint8_t*>(send), bytes, static_cast<uint8_t*>(recv), bytes, cell}},
	           s);
}

// every rank's `bytes` bytes at `mine` into all[p * bytes] (device), own
// slot included; queued on s
void comm_allgather_dev(Grid& g, const void* mine, size_t bytes, uint8_t* all, hipStream_t s) {
	HIP_CHECK(hipMemcpyAsync(all + size_t(g.rank) * bytes, mine, bytes, hipMemcpyDefault, s));
	if (g.size == 1 || bytes == 0) return;
	comm_require(g, "all-gather");
	std::vector<DevMsg> msgs;
	for (int p = 0; p < g.size; p++)
		if (p != g.rank)
			msgs.push_back({p, static_cast<const uint8_t*>(mine), bytes, all + size_t(p) * bytes, bytes});
	move_bytes(g, msgs, s);
}

// host exchange of arbitrary byte buffers: sizes first (one 8-byte message
// each way per peer), then the payloads, both through move_bytes
std::vector<std::vector<uint8_t>> comm_exchange(Grid& g, const std::vector<std::vector<uint8_t>>& send) {
	const int P = g.size;
	std::vector<std::vector<uint8_t>> recv(static_cast<size_t>(P));
	DX_REQUIRE(send.size() == size_t(P), "exchange: one buffer per rank");
	if (P == 1) return recv;
	comm_require(g, "this operation");
	hipStream_t s = g.s_comm;
	std::vector<uint64_t> ssz(size_t(P), 0);
	for (int p = 0; p < P; p++) ssz[size_t(p)] = p == g.rank ? 0 : send[size_t(p)].size();
	if (g.xfn) {
		// the host exchange moves host bytes: the lists go to it as they are
		// (no device staging), the sizes first
		DX_PHASE_COMM("comm.host_exchange_lists", s);
		static uint64_t none = 0;
		std::vector<uint64_t> rsz(size_t(P), 0);
		std::vector<const void*> sp(size_t(P), &none);
		std::vector<void*> rp(size_t(P), &none);
		std::vector<size_t> sb(size_t(P), 0), rb(size_t(P), 0);
		for (int p = 0; p < P; p++) {
			if (p == g.rank) continue;
			sp[size_t(p)] = &ssz[size_t(p)];
			rp[size_t(p)] = &rsz[size_t(p)];
			sb[size_t(p)] = rb[size_t(p)] = 8;
		}
		DX_REQUIRE(g.xfn(g.xctx, sp.data(), sb.data(), rp.data(), rb.data()) == 0, "exchange function failed");
		for (int p = 0; p < P; p++) {
			if (p == g.rank) continue;
			recv[size_t(p)].resize(size_t(rsz[size_t(p)]));
			sp[size_t(p)] = ssz[size_t(p)] ? static_cast<const void*>(send[size_t(p)].data()) : &none;
			rp[size_t(p)] = rsz[size_t(p)] ? static_cast<void*>(recv[size_t(p)].data()) : &none;
			sb[size_t(p)] = size_t(ssz[size_t(p)]);
			rb[size_t(p)] = size_t(rsz[size_t(p)]);
		}
		DX_REQUIRE(g.xfn(g.xctx, sp.data(), sb.data(), rp.data(), rb.data()) == 0, "exchange function failed");
		return recv;
	}
	DBuf<uint64_t> dsz, drsz;
	upload(dsz, ssz, s);
	drsz.alloc(size_t(P));
	std::vector<DevMsg> msgs;
	for (int p = 0; p < P; p++)
		if (p != g.rank)
			msgs.push_back({p, reinterpret_cast<const uint8_t*>(dsz.p + p), 8, reinterpret_cast<uint8_t*>(drsz.p + p), 8});
	move_bytes(g, msgs, s);
	std::vector<uint64_t> rsz = download(drsz.p, size_t(P), s);
	rsz[size_t(g.rank)] = 0;
	size_t stot = 0, rtot = 0;
	std::vector<size_t> soff(static_cast<size_t>(P)), roff(static_cast<size_t>(P));
	for (int p = 0; p < P; p++) {
		soff[size_t(p)] = stot;
		roff[size_t(p)] = rtot;
		stot += size_t(ssz[size_t(p)]);
		rtot += size_t(rsz[size_t(p)]);
	}
	std::vector<uint8_t> hs(stot);
	for (int p = 0; p < P; p++)
		if (ssz[size_t(p)]) std::memcpy(hs.data() + soff[size_t(p)], send[size_t(p)].data(), size_t(ssz[size_t(p)]));
	DBuf<uint8_t> ds, dr;
	ds.alloc(stot + 1);
	dr.alloc(rtot + 1);
	if (stot) h2d(ds.p, hs.data(), stot, s);
	msgs.clear();
	for (int p = 0; p < P; p++)
		if (ssz[size_t(p)] || rsz[size_t(p)])
			msgs.push_back({p, ds.p + soff[size_t(p)], size_t(ssz[size_t(p)]), dr.p + roff[size_t(p)], size_t(rsz[size_t(p)])});
	move_bytes(g, msgs, s);
	const std::vector<uint8_t> hr = download(dr.p, rtot, s);
	for (int p = 0; p < P; p++)
		recv[size_t(p)].assign(hr.begin() + ptrdiff_t(roff[size_t(p)]),
		                       hr.begin() + ptrdiff_t(roff[size_t(p)] + size_t(rsz[size_t(p)])));
	return recv;
}

static std::vector<uint8_t> as_bytes(const std::vector<uint64_t>& v) {
	std::vector<uint8_t> b(v.size() * 8);
	if (!v.empty()) std::memcpy(b.data(), v.data(), b.size());
	return b;
}

static std::vector<uint64_t> as_u64(const std::vector<uint8_t>& b) {
	std::vector<uint64_t> v(b.size() / 8);
	if (!v.empty()) std::memcpy(v.data(), b.data(), v.size() * 8);
	return v;
}

std::vector<std::vector<uint64_t>> comm_alltoall_u64(Grid& g, const std::vector<std::vector<uint64_t>>& send) {
	std::vector<std::vector<uint8_t>> sb(size_t(g.size));
	for (int p = 0; p < g.size; p++) sb[size_t(p)] = as_bytes(send[size_t(p)]);
	const auto rb = comm_exchange(g, sb);
	std::vector<std::vector<uint64_t>> out(size_t(g.size));
	for (int p = 0; p < g.size; p++) out[size_t(p)] = p == g.rank ? send[size_t(p)] : as_u64(rb[size_t(p)]);
	return out;
}

// All_Gather (dccrg_mpi_support.hpp:98-235): everyone's list, by rank
std::vector<std::vector<uint64_t>> comm_allgather_u64(Grid& g, const std::vector<uint64_t>& mine) {
	std::vector<std::vector<uint64_t>> send(size_t(g.size), mine);
	return comm_alltoall_u64(g, send);
}

// combine P x count values (rank-major) in rank order: value of rank 0 first
void rank_ordered_combine(const double* all, int P, int count, int op, double* out) {
	for (int k = 0; k < count; k++) {
		double acc = all[k];
		for (int p = 1; p < P; p++) {
			const double x = all[size_t(p) * size_t(count) + size_t(k)];
			if (op == 0) acc += x;
			else if (op == 1) acc = std::min(acc, x);
			else acc = std::max(acc, x);
		}
		out[k] = acc;
	}
}

namespace {
// the same rank-ordered combine on the device: one thread per value (the
// host form above, operation for operation - std::min / std::max are the
// two comparisons below, which keep the first operand on NaN and on +-0 where
// fmin / fmax would not - so both give the same bits)
__global__ void rank_combine_kernel(const double* __restrict__ all, int P, int count, int op, double* __restrict__ out) {
#pragma clang fp contract(off)
	const int k = int(blockIdx.x * blockDim.x + threadIdx.x);
	if (k >= count) return;
	double acc = all[k];
	for (int p = 1; p < P; p++) {
		const double x = all[size_t(p) * size_t(count) + size_t(k)];
		if (op == 0) acc += x;
		else if (op == 1) acc = (x < acc) ? x : acc;
		else acc = (acc < x) ? x : acc;
	}
	out[k] = acc;
}

// all-gather of count doubles into `gather` (P x count, rank-major) and the
// rank-ordered combine into d_out, all queued on s
void allreduce_through(Grid& g, double* gather, const double* d_in, double* d_out, int count, int op, hipStream_t s) {
	comm_allgather_dev(g, d_in, size_t(count) * 8, reinterpret_cast<uint8_t*>(gather), s);
	rank_combine_kernel<<<unsigned((count + 63) / 64), 64, 0, s>>>(gather, g.size, count, op, d_out);
	HIP_CHECK(hipGetLastError());
}
}  // namespace

// MPI_Allreduce on device doubles, queued on `s`: the ranks' values
// all-gathered into a device buffer, then combined in rank order by one small
// kernel on every rank.  Over RCCL nothing waits on the host (the reduction
// is stream-ordered and can sit between two kernels of an iteration); the
// host exchange has to stage through the host and returns with the result
// on the device.  d_in and d_out may be the same buffer.
//
// The gather buffer g.red_all belongs to the compute stream: only this
// function writes it and callers pass s_comp (the combine kernel may still be
// reading it when this returns).  The host form below runs on s_comm and
// gathers into a buffer of its own, so a host allreduce (dccrgx_barrier,
// dccrgx_allreduce_f64) right after a device one cannot overwrite the values
// the device form's pending combine has yet to read.  A grow of red_all under
// a pending reader is safe: the old block goes to the pool's pending list,
// reused only after a device synchronisation (pool.hip).
void comm_allreduce_f64_dev(Grid& g, const double* d_in, double* d_out, int count, int op, hipStream_t s) {
	if (count <= 0) return;
	const size_t bytes = size_t(count) * 8;
	if (g.size == 1) {
		if (d_in != d_out) HIP_CHECK(hipMemcpyAsync(d_out, d_in, bytes, hipMemcpyDeviceToDevice, s));
		return;
	}
	comm_require(g, "allreduce");
	DX_REQUIRE(op >= 0 && op <= 2, "allreduce: op must be 0 (sum), 1 (min) or 2 (max)");
	DX_REQUIRE(s == g.s_comp, "device allreduce: the compute stream owns the gather buffer");
	g.red_all.reserve(size_t(count) * size_t(g.size));
	allreduce_through(g, g.red_all.p, d_in, d_out, count, op, s);
}

// MPI_Allreduce on host doubles (advection dt MIN, solve.hpp:317; sums): up,
// gathered and combined on s_comm in a buffer of this call (value slot +
// P x count gather), down
void comm_allreduce_f64(Grid& g, double* v, int count, int op) {
	if (g.size == 1 || count <= 0) return;
	comm_require(g, "allreduce");
	DX_REQUIRE(op >= 0 && op <= 2, "allreduce: op must be 0 (sum), 1 (min) or 2 (max)");
	hipStream_t s = g.s_comm;
	DBuf<double> d;
	d.alloc(size_t(count) * size_t(g.size + 1));
	h2d(d.p, v, size_t(count) * 8, s);
	allreduce_through(g, d.p + count, d.p, d.p, count, op, s);
	d2h_small(v, d.p, size_t(count) * 8, s);
}

uint64_t comm_allreduce_max_u64(Grid& g, uint64_t v) {
	const auto all = comm_allgather_u64(g, {v});
	uint64_t m = v;
	for (const auto& a : all)
		if (!a.empty()) m = std::max(m, a[0]);
	return m;
}

}  // namespace dccrgx
