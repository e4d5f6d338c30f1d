// Collectives and point-to-point transfers of one grid.
//
// The reference talks MPI: Allgather(v) / Allreduce for the control plane
// (dccrg_mpi_support.hpp:98-275), Isend / Irecv of derived datatypes for
// payloads (start_user_data_transfers, dccrg.hpp:10564-10997).  Here every
// exchange goes through one of two transports:
//   - RCCL (the grid was created with a bootstrap id): payloads move
//     device-to-device with grouped ncclSend / ncclRecv over xGMI, control
//     data through small device staging buffers;
//   - a caller-provided host exchange (dccrgx_create_with_exchange): one
//     grouped point-to-point exchange of host buffers with every rank (MPI
//     in the C++ facade when ranks share a GPU, torch.distributed in tests);
//     payloads are staged through the host.
// Every collective is built on the single primitive `exchange`; reductions
// combine the per-rank values in rank order, so results do not depend on
// the transport.
#include <algorithm>
#include <cstring>

#include "dccrgx_internal.hpp"

namespace dccrgx {

void comm_require(const Grid& g, const char* what) {
	if (!g.has_collectives())
		throw Error(DCCRGX_EINVAL, std::string(what) +
		                               " needs a communicator (grid created without an RCCL id or an exchange function)");
}

// host exchange of arbitrary byte buffers; sizes first (8 bytes to every rank)
std::vector<std::vector<uint8_t>> comm_exchange(Grid& g, const std::vector<std::vector<uint8_t>>& send) {
	const int P = g.size;
	std::vector<std::vector<uint8_t>> recv(static_cast<size_t>(P));
	DX_REQUIRE(send.size() == size_t(P), "exchange: one buffer per rank");
	if (P == 1) return recv;
	comm_require(g, "this operation");
	std::vector<uint64_t> ssz(size_t(P), 0), rsz(size_t(P), 0);
	for (int p = 0; p < P; p++) ssz[size_t(p)] = p == g.rank ? 0 : send[size_t(p)].size();
	if (g.xfn) {
		// sizes
		std::vector<const void*> sp(static_cast<size_t>(P));
		std::vector<void*> rp(static_cast<size_t>(P));
		std::vector<size_t> sb(size_t(P), 8), rb(size_t(P), 8);
		for (int p = 0; p < P; p++) {
			sp[size_t(p)] = &ssz[size_t(p)];
			rp[size_t(p)] = &rsz[size_t(p)];
		}
		sb[size_t(g.rank)] = rb[size_t(g.rank)] = 0;
		DX_REQUIRE(g.xfn(g.xctx, sp.data(), sb.data(), rp.data(), rb.data()) == 0, "exchange function failed");
		for (int p = 0; p < P; p++) {
			recv[size_t(p)].resize(p == g.rank ? 0 : size_t(rsz[size_t(p)]));
			sp[size_t(p)] = send[size_t(p)].data();
			sb[size_t(p)] = size_t(ssz[size_t(p)]);
			rp[size_t(p)] = recv[size_t(p)].data();
			rb[size_t(p)] = recv[size_t(p)].size();
		}
		DX_REQUIRE(g.xfn(g.xctx, sp.data(), sb.data(), rp.data(), rb.data()) == 0, "exchange function failed");
		return recv;
	}
	// RCCL: all-gather the P x P size matrix, then grouped send / recv
	hipStream_t s = g.s_comm;
	DBuf<uint64_t> dsz, dall;
	dsz.alloc(static_cast<size_t>(P));
	dall.alloc(size_t(P) * size_t(P));
	HIP_CHECK(hipMemcpyAsync(dsz.p, ssz.data(), size_t(P) * 8, hipMemcpyHostToDevice, s));
	NCCL_CHECK(ncclAllGather(dsz.p, dall.p, size_t(P), ncclUint64, g.nccl, s));
	const std::vector<uint64_t> all = download(dall.p, size_t(P) * size_t(P), s);
	size_t stot = 0, rtot = 0;
	std::vector<size_t> soff(static_cast<size_t>(P)), roff(static_cast<size_t>(P));
	for (int p = 0; p < P; p++) {
		rsz[size_t(p)] = p == g.rank ? 0 : all[size_t(p) * size_t(P) + size_t(g.rank)];
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
	if (stot) HIP_CHECK(hipMemcpyAsync(ds.p, hs.data(), stot, hipMemcpyHostToDevice, s));
	NCCL_CHECK(ncclGroupStart());
	for (int p = 0; p < P; p++) {
		if (ssz[size_t(p)]) NCCL_CHECK(ncclSend(ds.p + soff[size_t(p)], size_t(ssz[size_t(p)]), ncclUint8, p, g.nccl, s));
		if (rsz[size_t(p)]) NCCL_CHECK(ncclRecv(dr.p + roff[size_t(p)], size_t(rsz[size_t(p)]), ncclUint8, p, g.nccl, s));
	}
	NCCL_CHECK(ncclGroupEnd());
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

// MPI_Allreduce on doubles; combined in rank order on every rank
void comm_allreduce_f64(Grid& g, double* v, int count, int op) {
	if (g.size == 1 || count <= 0) return;
	comm_require(g, "allreduce");
	if (g.nccl && !g.xfn) {
		DBuf<double> d;
		d.alloc(size_t(count));
		HIP_CHECK(hipMemcpyAsync(d.p, v, size_t(count) * 8, hipMemcpyHostToDevice, g.s_comm));
		const ncclRedOp_t rop = op == 0 ? ncclSum : (op == 1 ? ncclMin : ncclMax);
		NCCL_CHECK(ncclAllReduce(d.p, d.p, size_t(count), ncclFloat64, rop, g.nccl, g.s_comm));
		HIP_CHECK(hipMemcpyAsync(v, d.p, size_t(count) * 8, hipMemcpyDeviceToHost, g.s_comm));
		HIP_CHECK(hipStreamSynchronize(g.s_comm));
		return;
	}
	std::vector<uint8_t> mine(size_t(count) * 8);
	std::memcpy(mine.data(), v, mine.size());
	const auto all = comm_exchange(g, std::vector<std::vector<uint8_t>>(size_t(g.size), mine));
	for (int k = 0; k < count; k++) {
		double acc = 0;
		for (int p = 0; p < g.size; p++) {
			double x;
			std::memcpy(&x, p == g.rank ? mine.data() + 8 * k : all[size_t(p)].data() + 8 * k, 8);
			if (p == 0) acc = x;
			else if (op == 0) acc += x;
			else if (op == 1) acc = std::min(acc, x);
			else acc = std::max(acc, x);
		}
		v[k] = acc;
	}
}

uint64_t comm_allreduce_max_u64(Grid& g, uint64_t v) {
	const auto all = comm_allgather_u64(g, {v});
	uint64_t m = v;
	for (const auto& a : all)
		if (!a.empty()) m = std::max(m, a[0]);
	return m;
}

// payload messages between device buffers (migration, user-hood halos)
void comm_device_transfer(Grid& g, const std::vector<DevMsg>& msgs, hipStream_t s) {
	if (g.size == 1) return;
	comm_require(g, "payload transfer");
	if (g.nccl && !g.xfn) {
		NCCL_CHECK(ncclGroupStart());
		for (const auto& m : msgs) {
			if (m.send_bytes) NCCL_CHECK(ncclSend(m.send, m.send_bytes, ncclUint8, m.peer, g.nccl, s));
			if (m.recv_bytes) NCCL_CHECK(ncclRecv(m.recv, m.recv_bytes, ncclUint8, m.peer, g.nccl, s));
		}
		NCCL_CHECK(ncclGroupEnd());
		return;
	}
	// host exchange: device -> host, exchange, host -> device
	std::vector<std::vector<uint8_t>> hs(size_t(g.size)), hr(size_t(g.size));
	for (const auto& m : msgs) {
		hs[size_t(m.peer)].resize(m.send_bytes);
		if (m.send_bytes) HIP_CHECK(hipMemcpyAsync(hs[size_t(m.peer)].data(), m.send, m.send_bytes, hipMemcpyDefault, s));
	}
	HIP_CHECK(hipStreamSynchronize(s));
	std::vector<const void*> sp(size_t(g.size), nullptr);
	std::vector<void*> rp(size_t(g.size), nullptr);
	std::vector<size_t> sb(size_t(g.size), 0), rb(size_t(g.size), 0);
	for (const auto& m : msgs) {
		hr[size_t(m.peer)].resize(m.recv_bytes);
		sp[size_t(m.peer)] = hs[size_t(m.peer)].data();
		sb[size_t(m.peer)] = m.send_bytes;
		rp[size_t(m.peer)] = hr[size_t(m.peer)].data();
		rb[size_t(m.peer)] = m.recv_bytes;
	}
	DX_REQUIRE(g.xfn(g.xctx, sp.data(), sb.data(), rp.data(), rb.data()) == 0, "exchange function failed");
	for (const auto& m : msgs)
		if (m.recv_bytes) HIP_CHECK(hipMemcpyAsync(m.recv, hr[size_t(m.peer)].data(), m.recv_bytes, hipMemcpyDefault, s));
	HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace dccrgx
