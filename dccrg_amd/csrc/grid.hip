// dccrgx: host side of the MI355X-native dccrg hot path.  Drives the halo
// exchange, the refinement closure, the repartition / migration and the
// built-in sweeps over the structures of mesh.hip; the C ABI
// (include/dccrgx.h) is in api.hip.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>
#include <set>

#include "dccrgx_grid.hpp"

namespace dccrgx {

std::vector<Field*> transfer_fields(Grid& g) {
	std::vector<Field*> tf;
	for (auto& f : g.fields)
		if (f.transfer) tf.push_back(&f);
	return tf;
}

// the fixed-size / variable-size ones among them
static std::vector<Field*> fixed_transfer_fields(Grid& g) {
	std::vector<Field*> tf;
	for (auto& f : g.fields)
		if (f.transfer && !f.var) tf.push_back(&f);
	return tf;
}

std::vector<Field*> var_transfer_fields(Grid& g) {
	std::vector<Field*> tf;
	for (auto& f : g.fields)
		if (f.transfer && f.var) tf.push_back(&f);
	return tf;
}

// --------------------------------------------------------------------------- variable-size payloads
// Per peer (ascending) the runs of a transfer: cells [soff, soff + sn) of the
// send list and [roff, roff + rn) of the receive list.
struct PeerRuns {
	std::vector<int> peer;
	std::vector<size_t> soff, sn, roff, rn;
	void add(int p, size_t so, size_t ns, size_t ro, size_t nr) {
		peer.push_back(p);
		soff.push_back(so);
		sn.push_back(ns);
		roff.push_back(ro);
		rn.push_back(nr);
	}
};

static void var_pack(const Field& f, const int32_t* slots, size_t n, VarMsg& M, hipStream_t s) {
	var_gather(f, slots, n, M.ssz, M.sbytes, s);
	M.hs = download(M.ssz.p, n, s);
}

// the two exchanges of a variable-size transfer: the sizes (their counts are
// known to both sides), then the bytes (known from the sizes)
static void var_transfer(Grid& g, VarMsg& M, const PeerRuns& R, size_t n_recv, hipStream_t s) {
	M.rsz.alloc(n_recv + 1);
	std::vector<DevMsg> m1;
	for (size_t i = 0; i < R.peer.size(); i++)
		if (R.sn[i] || R.rn[i])
			m1.push_back(DevMsg{R.peer[i], reinterpret_cast<const uint8_t*>(M.ssz.p + R.soff[i]), R.sn[i] * 8,
			                    reinterpret_cast<uint8_t*>(M.rsz.p + R.roff[i]), R.rn[i] * 8});
	comm_device_transfer(g, m1, s);
	HIP_CHECK(hipStreamSynchronize(s));
	const std::vector<uint64_t> hr = download(M.rsz.p, n_recv, s);
	auto sum = [](const std::vector<uint64_t>& v, size_t a, size_t b) {
		uint64_t t = 0;
		for (size_t i = a; i < b; i++) t += v[i];
		return t;
	};
	const uint64_t rtotal = sum(hr, 0, n_recv);
	M.rbytes.alloc(rtotal + 1);
	std::vector<DevMsg> m2;
	for (size_t i = 0; i < R.peer.size(); i++) {
		const uint64_t sbo = sum(M.hs, 0, R.soff[i]), sbl = sum(M.hs, R.soff[i], R.soff[i] + R.sn[i]);
		const uint64_t rbo = sum(hr, 0, R.roff[i]), rbl = sum(hr, R.roff[i], R.roff[i] + R.rn[i]);
		if (sbl || rbl) m2.push_back(DevMsg{R.peer[i], M.sbytes.p + sbo, sbl, M.rbytes.p + rbo, rbl});
	}
	comm_device_transfer(g, m2, s);
	HIP_CHECK(hipStreamSynchronize(s));
}

Field& field(Grid& g, int fid) {
	DX_REQUIRE(fid >= 0 && size_t(fid) < g.fields.size(), "invalid field id");
	return g.fields[size_t(fid)];
}

Field& fixed_field(Grid& g, int fid) {
	Field& f = field(g, fid);
	DX_REQUIRE(!f.var, "a variable-size field has no fixed element layout (use the dccrgx_variable_field_* calls)");
	return f;
}

void ensure_scratch(Grid& g, Field& f) {
	(void)g;
	if (f.scratch.n != f.data.n) f.scratch.alloc(f.data.n);
}

// commit a double-buffered sweep: swap, and carry the current remote copies
// over so they hold the last received values (as the reference's copies do)
void commit(Grid& g, Field& f) {
	DX_REQUIRE(f.scratch.n == f.data.n && f.data.p, "nothing to commit");
	const size_t halo = (g.n_slots - g.n_local) * f.elem;
	if (halo)
		HIP_CHECK(hipMemcpyAsync(f.scratch.p + g.n_local * f.elem, f.data.p + g.n_local * f.elem, halo,
		                         hipMemcpyDeviceToDevice, g.s_comp));
	f.data.swap(f.scratch);
	field_written(f);
}

void region_range(const Grid& g, int region, size_t& s0, size_t& s1) {
	switch (region) {
	case DCCRGX_REGION_ALL: s0 = 0; s1 = g.n_local; break;
	case DCCRGX_REGION_INNER: s0 = 0; s1 = g.n_inner; break;
	case DCCRGX_REGION_OUTER: s0 = g.n_inner; s1 = g.n_local; break;
	default: throw Error(DCCRGX_EINVAL, "invalid region");
	}
}

void k_time_begin(Grid& g) {
	if (!g.timing) return;
	hipEvent_t a, b;
	if (!g.pending_events.empty() && hipEventQuery(g.pending_events.front().second) == hipSuccess) {
		// the oldest pair has completed: its time is taken now and its events
		// are reused (no event creation per timed launch)
		const auto ab = g.pending_events.front();
		g.pending_events.pop_front();
		float ms = 0;
		HIP_CHECK(hipEventElapsedTime(&ms, ab.first, ab.second));
		g.timed_ms += ms;
		g.timed_count++;
		a = ab.first;
		b = ab.second;
	} else {
		HIP_CHECK(hipEventCreate(&a));
		HIP_CHECK(hipEventCreate(&b));
	}
	HIP_CHECK(hipEventRecord(a, g.s_comp));
	g.pending_events.push_back({a, b});
}

void k_time_end(Grid& g) {
	if (!g.timing) return;
	HIP_CHECK(hipEventRecord(g.pending_events.back().second, g.s_comp));
}

void drain_timing(Grid& g) {
	for (auto& ab : g.pending_events) {
		HIP_CHECK(hipEventSynchronize(ab.second));
		float ms = 0;
		HIP_CHECK(hipEventElapsedTime(&ms, ab.first, ab.second));
		g.timed_ms += ms;
		g.timed_count++;
		(void)hipEventDestroy(ab.first);
		(void)hipEventDestroy(ab.second);
	}
	g.pending_events.clear();
}

// --------------------------------------------------------------------------- halo
// The wire message of a neighborhood to / from one peer: for each transferred
// field (field order) the window bytes of each listed cell in ascending id.
// The send buffer holds the packed payloads field by field over all peers
// (field k: n_send cells x window), the receive buffer likewise.
struct PlanLayout {
	std::vector<size_t> sfo, rfo;  // per field: start of its segment in sendbuf / recvbuf
	size_t sbytes = 0, rbytes = 0, bpc = 0;
};

static PlanLayout plan_layout(const HaloPlan& H, const std::vector<Field*>& tf) {
	PlanLayout L;
	for (Field* f : tf) {
		L.sfo.push_back(L.sbytes);
		L.rfo.push_back(L.rbytes);
		L.sbytes += H.n_send * f->win_len;
		L.rbytes += H.n_recv * f->win_len;
		L.bpc += f->win_len;
	}
	return L;
}

static void pack_plan(HaloPlan& H, const std::vector<Field*>& tf, const PlanLayout& L, hipStream_t s) {
	H.sendbuf.reserve(L.sbytes + 1);
	H.recvbuf.reserve(L.rbytes + 1);
	for (size_t k = 0; k < tf.size(); k++)
		k_pack(tf[k]->data.p, tf[k]->elem, tf[k]->win_off, tf[k]->win_len, H.send_slots.p, H.n_send,
		       H.sendbuf.p + L.sfo[k], s);
}

static size_t count_of(const std::map<int, std::vector<uint64_t>>& m, int p) {
	auto it = m.find(p);
	return it == m.end() ? 0 : it->second.size();
}

static size_t off_of(const std::map<int, size_t>& m, int p) {
	auto it = m.find(p);
	return it == m.end() ? 0 : it->second;
}

// start the exchange of a plan on s_comm (after the work queued on s_comp);
// `direct`: the plan's receive slots of a peer are one contiguous run of
// halo slots, so full-element fields are received in place
static void var_halo(Grid& g, HaloPlan& H, hipStream_t s) {
	const std::vector<Field*> vf = var_transfer_fields(g);
	if (vf.empty()) return;
	PeerRuns R;
	for (int p : H.peers()) R.add(p, off_of(H.send_off, p), count_of(H.send_ids, p), off_of(H.recv_off, p), count_of(H.recv_ids, p));
	for (Field* f : vf) {
		VarMsg M;
		var_pack(*f, H.send_slots.p, H.n_send, M, s);
		var_transfer(g, M, R, H.n_recv, s);
		var_place(*f, g.n_slots, H.recv_slots.p, H.n_recv, M.rsz.p, M.rbytes.p, s);
	}
}

static void plan_start(Grid& g, HaloPlan& H, bool direct) {
	if (transfer_fields(g).empty()) return;
	// every transferred field is written by this exchange (its remote
	// copies), now and again when it lands (halo_wait): a cache built from a
	// field while its copies are in flight is rebuilt after
	g.halo_fields.clear();
	for (Field* f : transfer_fields(g)) {
		field_halo_written(*f);
		g.halo_fields.push_back(int(f - g.fields.data()));
	}
	const std::vector<Field*> tf = fixed_transfer_fields(g);
	if (tf.empty()) {
		// variable-size payloads only: synchronous (their byte counts travel first)
		HIP_CHECK(hipEventRecord(g.ev_comp, g.s_comp));
		HIP_CHECK(hipStreamWaitEvent(g.s_comm, g.ev_comp, 0));
		var_halo(g, H, g.s_comm);
		HIP_CHECK(hipEventRecord(g.ev_halo, g.s_comm));
		return;
	}
	const PlanLayout L = plan_layout(H, tf);
	HIP_CHECK(hipEventRecord(g.ev_comp, g.s_comp));
	HIP_CHECK(hipStreamWaitEvent(g.s_comm, g.ev_comp, 0));
	hipStream_t s = g.s_comm;
	pack_plan(H, tf, L, s);
	// one message per peer and field (field order): the send slice of the
	// packed buffer, received straight into the peer's run of halo slots for
	// a whole-element field of a direct plan, else into the receive buffer
	// and placed; the same list for RCCL and the host exchange (cell by cell
	// on the wire under send_single_cells, comm.hip)
	std::vector<DevMsg> msgs;
	for (int p : H.peers()) {
		const size_t ns = count_of(H.send_ids, p), nr = count_of(H.recv_ids, p);
		const size_t so = off_of(H.send_off, p), ro = off_of(H.recv_off, p);
		for (size_t k = 0; k < tf.size(); k++) {
			Field* f = tf[k];
			uint8_t* dst = direct && f->full_window() ? f->data.p + (g.n_local + ro) * f->elem
			                                          : H.recvbuf.p + L.rfo[k] + ro * f->win_len;
			msgs.push_back({p, H.sendbuf.p + L.sfo[k] + so * f->win_len, ns * f->win_len, dst, nr * f->win_len,
			                f->win_len});
		}
	}
	comm_device_transfer(g, msgs, s);
	for (size_t k = 0; k < tf.size(); k++)
		if (!(direct && tf[k]->full_window()))
			k_place(H.recvbuf.p + L.rfo[k], tf[k]->elem, tf[k]->win_off, tf[k]->win_len, H.recv_slots.p, H.n_recv,
			        tf[k]->data.p, s);
	var_halo(g, H, s);
	HIP_CHECK(hipEventRecord(g.ev_halo, s));
}

void halo_start(Grid& g) {
	if (g.size == 1 || g.peers.empty()) return;
	comm_require(g, "update_copies_of_remote_neighbors");
	DX_REQUIRE(!g.halo_in_flight, "remote neighbor update already in flight");
	if (transfer_fields(g).empty()) return;
	plan_start(g, g.halo, true);
	g.halo_in_flight = true;
}

void halo_wait(Grid& g) {
	if (!g.halo_in_flight) return;
	HIP_CHECK(hipStreamWaitEvent(g.s_comp, g.ev_halo, 0));
	g.halo_in_flight = false;
	for (int fid : g.halo_fields)
		if (fid >= 0 && size_t(fid) < g.fields.size()) field_halo_written(g.fields[size_t(fid)]);
	g.halo_fields.clear();
}

// --------------------------------------------------------------------------- user neighborhoods
// neighbors of / to every local cell for hood id (find_neighbors_of /
// find_neighbors_to with user_hood_of / user_hood_to, 8974-8980), then the
// send / receive lists of the id: receive from p = the cells of p in the
// neighbors_of of local cells, send to p = the local cells in whose
// neighbors_to a cell of p appears, both ascending (the wire order)
UserHood& ensure_uhood(Grid& g, int id) {
	auto it = g.uhoods.find(id);
	DX_REQUIRE(it != g.uhoods.end(), "no such neighborhood id");
	UserHood& h = it->second;
	if (h.valid) return h;
	hipStream_t s = g.s_comp;
	const int nh = int(h.of.size() / 3);
	const size_t nl = g.n_local;
	const DevMesh dm = g.dm();
	DBuf<uint32_t> c_of, c_to;
	c_of.alloc(nl + 1);
	c_to.alloc(nl + 1);
	h.nof_ptr.alloc(nl + 1);
	h.nto_ptr.alloc(nl + 1);
	k_count_rows(g.m, h.d_of.p, h.d_to.p, nh, dm, g.slot_ids.p, 0, nl, c_of.p, c_to.p, s);
	const size_t t_of = scan_exclusive_u32(c_of.p, h.nof_ptr.p, nl, s);
	const size_t t_to = scan_exclusive_u32(c_to.p, h.nto_ptr.p, nl, s);
	h.nof_id.alloc(t_of + 1);
	h.nof_off.alloc(3 * t_of + 3);
	h.nto_id.alloc(t_to + 1);
	k_fill_neighbors_of(g.m, h.d_of.p, nh, dm, g.slot_ids.p, 0, nl, h.nof_ptr.p, h.nof_id.p, h.nof_off.p, s);
	k_fill_neighbors_to(g.m, h.d_to.p, nh, dm, g.slot_ids.p, 0, nl, h.nto_ptr.p, h.nto_id.p, s);
	HaloPlan& P = h.plan;
	P.send_ids.clear();
	P.recv_ids.clear();
	if (g.size > 1) {
		k_remote_by_owner(h.nof_id.p, t_of, dm, g.rank, g.size, P.recv_ids, s);
		k_send_by_owner(h.nto_id.p, h.nto_ptr.p, t_to, g.slot_ids.p, 0, nl, dm, g.rank, g.size, P.send_ids, s);
	}
	std::vector<uint64_t> sall, rall;
	P.send_off.clear();
	P.recv_off.clear();
	for (auto& kv : P.send_ids) {
		P.send_off[kv.first] = sall.size();
		sall.insert(sall.end(), kv.second.begin(), kv.second.end());
	}
	for (auto& kv : P.recv_ids) {
		P.recv_off[kv.first] = rall.size();
		rall.insert(rall.end(), kv.second.begin(), kv.second.end());
	}
	P.n_send = sall.size();
	P.n_recv = rall.size();
	DBuf<int32_t> err;
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
	P.send_slots.alloc(P.n_send + 1);
	P.recv_slots.alloc(P.n_recv + 1);
	DBuf<uint64_t> d1, d2;
	upload(d1, sall, s);
	upload(d2, rall, s);
	k_lookup_slots(d1.p, P.n_send, dm, P.send_slots.p, err.p, s);
	k_lookup_slots(d2.p, P.n_recv, dm, P.recv_slots.p, err.p, s);
	int herr = 0;
	d2h_small(&herr, err.p, 4, s);
	DX_REQUIRE(herr == 0, "user neighborhood references a cell without a local slot or remote copy");
	h.valid = true;
	return h;
}

HaloPlan& plan_of(Grid& g, int hood) {
	if (hood == DCCRGX_DEFAULT_HOOD) return g.halo;
	return ensure_uhood(g, hood).plan;
}

// update_copies_of_remote_neighbors(id) (966-1000 with a user id)
void uhood_halo(Grid& g, int id) {
	UserHood& h = ensure_uhood(g, id);
	if (g.size == 1 || (h.plan.send_ids.empty() && h.plan.recv_ids.empty())) return;
	comm_require(g, "update_copies_of_remote_neighbors");
	DX_REQUIRE(!g.halo_in_flight, "remote neighbor update already in flight");
	if (transfer_fields(g).empty()) return;
	plan_start(g, h.plan, false);
	HIP_CHECK(hipStreamWaitEvent(g.s_comp, g.ev_halo, 0));
}

// the explicit transport of one plan (dccrgx_halo_pack / _place)
static void no_var_transfer(Grid& g, const char* what) {
	DX_REQUIRE(var_transfer_fields(g).empty(),
	           std::string(what) + ": variable-size fields move only with the library's own transport");
}

size_t halo_pack_peer(Grid& g, int hood, int peer, uint8_t* buf, size_t cap) {
	no_var_transfer(g, "halo_pack");
	HaloPlan& H = plan_of(g, hood);
	const std::vector<Field*> tf = fixed_transfer_fields(g);
	const PlanLayout L = plan_layout(H, tf);
	const size_t ns = count_of(H.send_ids, peer), so = off_of(H.send_off, peer);
	DX_REQUIRE(cap >= ns * L.bpc, "buffer too small for the halo message");
	pack_plan(H, tf, L, g.s_comp);
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
	size_t o = 0;
	for (size_t k = 0; k < tf.size(); k++) {
		const size_t b = ns * tf[k]->win_len;
		if (b)
			HIP_CHECK(hipMemcpyAsync(buf + o, H.sendbuf.p + L.sfo[k] + so * tf[k]->win_len, b, hipMemcpyDefault, g.s_comp));
		o += b;
	}
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
	return o;
}

void halo_place_peer(Grid& g, int hood, int peer, const uint8_t* buf, size_t bytes) {
	no_var_transfer(g, "halo_place");
	HaloPlan& H = plan_of(g, hood);
	const std::vector<Field*> tf = fixed_transfer_fields(g);
	const PlanLayout L = plan_layout(H, tf);
	const size_t nr = count_of(H.recv_ids, peer), ro = off_of(H.recv_off, peer);
	DX_REQUIRE(bytes == nr * L.bpc, "halo message has the wrong size");
	H.recvbuf.reserve(L.rbytes + 1);
	size_t o = 0;
	for (size_t k = 0; k < tf.size(); k++) {
		const size_t b = nr * tf[k]->win_len;
		if (b)
			HIP_CHECK(hipMemcpyAsync(H.recvbuf.p + L.rfo[k] + ro * tf[k]->win_len, buf + o, b, hipMemcpyDefault, g.s_comp));
		k_place(H.recvbuf.p + L.rfo[k] + ro * tf[k]->win_len, tf[k]->elem, tf[k]->win_off, tf[k]->win_len,
		        H.recv_slots.p + ro, nr, tf[k]->data.p, g.s_comp);
		field_halo_written(*tf[k]);
		o += b;
	}
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
}

void halo_message_size(Grid& g, int hood, int peer, size_t& sb, size_t& rb) {
	no_var_transfer(g, "halo_message_size");
	HaloPlan& H = plan_of(g, hood);
	const PlanLayout L = plan_layout(H, fixed_transfer_fields(g));
	sb = count_of(H.send_ids, peer) * L.bpc;
	rb = count_of(H.recv_ids, peer) * L.bpc;
}

// --------------------------------------------------------------------------- refinement
static std::vector<uint64_t> union_sorted(Grid& g, const std::vector<std::vector<uint64_t>>& all) {
	// every rank's list ascending (as gather_union's callers give them): merged
	// pairwise on the host, O(n log P), no device round trip
	bool sorted = true;
	for (const auto& v : all) sorted = sorted && std::is_sorted(v.begin(), v.end());
	if (sorted) {
		std::vector<std::vector<uint64_t>> parts(all.begin(), all.end());
		while (parts.size() > 1) {
			std::vector<std::vector<uint64_t>> next;
			for (size_t i = 0; i + 1 < parts.size(); i += 2) {
				std::vector<uint64_t> mg;
				mg.reserve(parts[i].size() + parts[i + 1].size());
				std::merge(parts[i].begin(), parts[i].end(), parts[i + 1].begin(), parts[i + 1].end(), std::back_inserter(mg));
				next.push_back(std::move(mg));
			}
			if (parts.size() % 2) next.push_back(std::move(parts.back()));
			parts.swap(next);
		}
		std::vector<uint64_t> u = parts.empty() ? std::vector<uint64_t>{} : std::move(parts[0]);
		u.erase(std::unique(u.begin(), u.end()), u.end());
		return u;
	}
	std::vector<uint64_t> u;
	for (const auto& v : all) u.insert(u.end(), v.begin(), v.end());
	host_sort_u64(u, true, g.s_comp);
	return u;
}

// every rank's sorted list merged (All_Gather + union); one process: its own
// list, without the copies of the exchange
static std::vector<uint64_t> gather_union(Grid& g, std::vector<uint64_t> mine) {
	if (g.size == 1) {
		host_sort_u64(mine, true, g.s_comp);  // a no-op for the sorted lists given here
		return mine;
	}
	return union_sorted(g, comm_allgather_u64(g, mine));
}

static DBuf<int32_t> slots_of(Grid& g, const std::vector<uint64_t>& ids);

static std::vector<uint64_t> sorted_unique(Grid& g, std::vector<uint64_t> v) {
	host_sort_u64(v, true, g.s_comp);
	return v;
}

static bool sorted_contains(const std::vector<uint64_t>& v, uint64_t x) {
	return std::binary_search(v.begin(), v.end(), x);
}

// closure of a sorted set under a rule every rank evaluates for its own
// cells in `fresh`, the new cells all-gathered each round (the loops of
// induce_refines 9591-9720 and of override_refines 9991-10038).  dS: S on
// the device (the first round reads it there); returns whether S grew
static bool close_set(Grid& g, std::vector<uint64_t>& S, bool finer, const uint64_t* dS = nullptr) {
	const int nh = int(g.hood.size() / 3);
	std::vector<uint64_t> fresh = S;
	bool grew = false;
	while (true) {
		DX_PHASE("cs.round", g.s_comp);
		std::vector<uint64_t> found;
		{
			DX_PHASE("cs.induced", g.s_comp);
			found = k_induced_refines(g.m, g.d_hood.p, g.d_hood_to.p, nh, g.dm(), g.rank, fresh, g.s_comp, finer,
			                          grew ? nullptr : dS);
		}
		std::vector<uint64_t> mine_new;
		std::set_difference(found.begin(), found.end(), S.begin(), S.end(), std::back_inserter(mine_new));
		std::vector<uint64_t> all;
		{
			DX_PHASE("cs.gather", g.s_comp);
			all = gather_union(g, std::move(mine_new));
		}
		fresh.clear();
		std::set_difference(all.begin(), all.end(), S.begin(), S.end(), std::back_inserter(fresh));
		if (fresh.empty()) break;
		std::vector<uint64_t> merged;
		std::merge(S.begin(), S.end(), fresh.begin(), fresh.end(), std::back_inserter(merged));
		S.swap(merged);
		grew = true;
	}
	return grew;
}

// Children of the merged families F that change process (10360-10410): one
// thread per family looks up its eight children's owners; a child of this
// rank whose parent goes to another (child 0's owner) is sent there, a child
// of another rank whose parent stays here is received from it.  Only those
// (the families on process boundaries) are appended, as (id, peer * 2 +
// 0 send / 1 receive); everything else stays on the device.
__global__ void moving_children_kernel(MapCtx m, DevMesh M, const uint64_t* __restrict__ F, size_t nf, int rank,
                                       uint64_t* __restrict__ out_id, int32_t* __restrict__ out_peer,
                                       unsigned long long* __restrict__ cnt, unsigned long long cap) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < nf; i += size_t(gridDim.x) * blockDim.x) {
		uint64_t ch[8];
		map_all_children(m, F[i], ch);
		int32_t o[8];
		for (int k = 0; k < 8; k++) o[k] = dm_owner(M, ch[k]);
		const int32_t po = o[0];
		for (int k = 0; k < 8; k++) {
			int32_t peer = -1, kind = 0;
			if (o[k] == rank && po != rank) {
				peer = po;
			} else if (o[k] != rank && po == rank && o[k] >= 0) {
				peer = o[k];
				kind = 1;
			}
			if (peer < 0) continue;
			const unsigned long long at = atomicAdd(cnt, 1ull);
			if (at < cap) {
				out_id[at] = ch[k];
				out_peer[at] = peer * 2 + kind;
			}
		}
	}
}

static void k_moving_children(Grid& g, const uint64_t* dF, size_t nf, std::map<int, std::vector<uint64_t>>& send_ids,
                              std::map<int, std::vector<uint64_t>>& recv_ids, hipStream_t s) {
	if (!nf) return;
	DBuf<unsigned long long> cnt;
	cnt.alloc(1);
	size_t cap = std::max<size_t>(4096, nf);  // most families do not straddle ranks; once more when short
	for (int pass = 0; pass < 2; pass++) {
		DBuf<uint64_t> id;
		DBuf<int32_t> peer;
		id.alloc(cap);
		peer.alloc(cap);
		HIP_CHECK(hipMemsetAsync(cnt.p, 0, 8, s));
		moving_children_kernel<<<grid_for(nf, 256), 256, 0, s>>>(g.m, g.dm(), dF, nf, g.rank, id.p, peer.p, cnt.p,
		                                                        (unsigned long long)cap);
		HIP_CHECK(hipGetLastError());
		unsigned long long n = 0;
		d2h_small(&n, cnt.p, 8, s);
		if (n > cap) {
			cap = size_t(n);
			continue;
		}
		const std::vector<uint64_t> hi = download(id.p, size_t(n), s);
		const std::vector<int32_t> hp = download(peer.p, size_t(n), s);
		for (size_t k = 0; k < size_t(n); k++) (hp[k] & 1 ? recv_ids : send_ids)[hp[k] >> 1].push_back(hi[k]);
		return;
	}
	DX_REQUIRE(false, "internal error: moving children beyond their count");
}

// stop_refining (3461-3485) = override_refines, induce_refines,
// override_unrefines, execute_refines, distributed:
//  * override_refines (9991-10038): dont_refine cells spread to their finer
//    neighbors_of / neighbors_to entries until closed; refine requests of
//    those cells are dropped; every rank's requests are all-gathered;
//  * induce_refines (9591-9720): a neighbors_of / neighbors_to entry coarser
//    than a refined cell is refined too - every rank evaluates the rule for
//    its own cells, the induced ones are all-gathered each round;
//  * override_unrefines (9796-9898): a requested family merges unless a
//    sibling is refined or marked dont_unrefine, or its parent's
//    neighborhood holds a finer leaf or a same-level one being refined
//    (evaluated by the requesting rank, which knows that region);
//  * execute_refines (10104-10554): on the device the known leaves in S are
//    replaced by their children (the owner's, 10228-10237) and every merged
//    family by its parent (owned by the first child's owner, 10298); the
//    removed children's payloads go to the parent's process (10360-10410,
//    get_removed_cells 3497), the parents start zeroed (cell_data[parent],
//    10475) and every structure is rebuilt.
// The local cells created by refinement go to Grid::new_cells.
void stop_refining_impl(Grid& g) {
	if (g.size > 1) comm_require(g, "stop_refining");
	const int nh = int(g.hood.size() / 3);
	hipStream_t s = g.s_comp;
	DX_LAPS(s);
	for (auto& f : g.fields) {
		f.removed.release();
		f.rm_off.release();
	}
	g.removed_ids.clear();
	g.new_cells.clear();
	g.merged_dev.release();
	g.n_merged = 0;

	auto vec = [](const std::unordered_set<uint64_t>& s) { return std::vector<uint64_t>(s.begin(), s.end()); };
	std::vector<uint64_t> D = gather_union(g, sorted_unique(g, vec(g.dont_refine_cells)));
	if (!D.empty()) close_set(g, D, true);
	// cells_not_to_refine = old_donts (10039-10040): the spread set, the same
	// on every rank, stays for the next stop_refining and refine_completely
	// (2477-2491) until balance_load (3812)
	// (clear() of an unordered_set costs its bucket count even when empty, and
	// the request sets keep the buckets of their largest size: cleared only
	// when they hold something)
	if (!D.empty()) g.dont_refine_cells = std::unordered_set<uint64_t>(D.begin(), D.end());
	else if (!g.dont_refine_cells.empty()) g.dont_refine_cells.clear();
	DX_LAP("sr.1_override_refines");
	// the request set is exactly check_for_adaptation's device list: S starts
	// as it, on the device as well
	DBuf<uint64_t> dS;
	const bool dev_rq = g.refine_dev_valid && g.refine_requests.empty() && D.empty() && g.size == 1;
	if (dev_rq) dS = std::move(g.refine_dev);
	g.refine_dev_valid = false;
	g.refine_dev.release();
	std::vector<uint64_t> mine;
	{
		std::vector<uint64_t> rq = vec(g.refine_requests);
		rq.insert(rq.end(), g.refine_bulk.begin(), g.refine_bulk.end());
		rq = sorted_unique(g, std::move(rq));
		if (D.empty()) mine = std::move(rq);
		else std::set_difference(rq.begin(), rq.end(), D.begin(), D.end(), std::back_inserter(mine));
	}
	if (!g.refine_requests.empty()) g.refine_requests.clear();
	g.refine_bulk.clear();
	DX_LAP("sr.2a_mine");
	std::vector<uint64_t> S = gather_union(g, std::move(mine));
	DX_LAP("sr.2b_gather_S");
	bool s_on_dev = dev_rq && !S.empty();
	if (!S.empty() && close_set(g, S, false, s_on_dev ? dS.p : nullptr)) s_on_dev = false;
	DX_LAP("sr.2_induce_refines");

	// unrefines: one family per requested parent, unless one of its children
	// is refined or marked dont_unrefine, or its neighborhood forbids it (on
	// the device)
	// (the requests exactly check_for_adaptation's device list of family
	// heads: read there, no upload, no sort of their parents)
	DBuf<uint64_t> dUR;
	const bool dev_ur = g.unrefine_dev_valid && g.unrefine_requests.empty();
	if (dev_ur) dUR = std::move(g.unrefine_dev);
	g.unrefine_dev_valid = false;
	g.unrefine_dev.release();
	std::vector<uint64_t> req(g.unrefine_requests.begin(), g.unrefine_requests.end());
	req.insert(req.end(), g.unrefine_bulk.begin(), g.unrefine_bulk.end());
	if (!g.unrefine_requests.empty()) g.unrefine_requests.clear();
	g.unrefine_bulk.clear();
	const std::vector<uint64_t> DU = gather_union(g, sorted_unique(g, vec(g.dont_unrefine_cells)));
	if (!g.dont_unrefine_cells.empty()) g.dont_unrefine_cells.clear();
	DX_LAP("sr.3a_requests");
	// S is final: one device copy for the passes below
	if (!s_on_dev) upload(dS, S, s);
	DX_LAP("sr.3b_upload_S");
	const std::vector<uint64_t> fmine =
	    k_unrefine_families(g.m, g.d_hood.p, nh, g.dm(), req, S, DU, s, dS.p, dev_ur ? dUR.p : nullptr);
	DX_LAP("sr.3c_families");
	const std::vector<uint64_t> F = gather_union(g, fmine);
	DBuf<uint64_t> dF;
	upload(dF, F, s);
	DX_LAP("sr.3_override_unrefines");
	if (S.empty() && F.empty()) return;

	// local refined cells -> the new local cells (on the device, read on the
	// host only when asked); weights and pins follow (6199-6200, 10239-10251)
	{
		DBuf<uint64_t> created;
		// ascending on the first host read (new_cells has no device reader)
		const size_t nc = k_created_children(g.m, g.dm(), g.rank, S, created, s, dS.p, false);
		g.new_cells.set_device(std::move(created), nc, false);
	}
	if (!g.weights.empty() || !g.pins.empty()) {
		std::vector<int32_t> own(S.size());
		lookup_batch(g, S.data(), S.size(), own.data(), nullptr);
		for (size_t i = 0; i < S.size(); i++) {
			if (own[i] != g.rank) continue;
			uint64_t ch[8];
			map_all_children(g.m, S[i], ch);
			auto w = g.weights.find(S[i]);
			if (w != g.weights.end()) {
				const double wv = w->second;
				g.weights.erase(w);
				for (uint64_t c : ch) g.weights[c] = wv;
			}
			// children inherit their parent's pin (10239-10251)
			auto pn = g.pins.find(S[i]);
			if (pn != g.pins.end()) {
				const int pv = pn->second;
				g.pins.erase(pn);
				for (uint64_t c : ch) g.pins[c] = pv;
			}
		}
	}
	DX_LAP("sr.4_created");

	// merged families: the children's payloads to the parent's new process
	std::map<int, std::vector<uint64_t>> send_ids, recv_ids;
	DBuf<uint64_t> keep_ids;  // removed children staying on this rank (device, ascending)
	DBuf<int32_t> ksl;        // and their slots
	size_t n_keep = 0;
	if (!F.empty()) {
		n_keep = k_kept_children(g.m, g.dm(), g.rank, F, keep_ids, ksl, s, dF.p,
		                         g.size == 1 && !std::getenv("DCCRGX_KEPT_SORT"));
		DX_LAP("sr.5a_kept");
		const bool attrs = !g.weights.empty() || !g.pins.empty();
		if (g.size > 1 && !attrs) {
			// the device scan of the children that change process
			k_moving_children(g, dF.p, F.size(), send_ids, recv_ids, s);
			for (auto* mp : {&send_ids, &recv_ids})
				for (auto& kv : *mp) std::sort(kv.second.begin(), kv.second.end());
		} else if (attrs) {
			// the children leaving / arriving, and the weights / pins of the
			// removed local ones
			std::vector<uint64_t> ch_all(8 * F.size());
			for (size_t i = 0; i < F.size(); i++) map_all_children(g.m, F[i], ch_all.data() + 8 * i);
			std::vector<int32_t> ch_own(ch_all.size());
			lookup_batch(g, ch_all.data(), ch_all.size(), ch_own.data(), nullptr);
			for (size_t i = 0; i < F.size(); i++) {
				const int parent_owner = ch_own[8 * i];
				for (int k = 0; k < 8; k++) {
					const uint64_t c = ch_all[8 * i + k];
					const int o = ch_own[8 * i + k];
					if (o == g.rank && attrs) {
						g.weights.erase(c);
						g.pins.erase(c);
					}
					if (o == g.rank && parent_owner != g.rank) send_ids[parent_owner].push_back(c);
					else if (o != g.rank && parent_owner == g.rank && o >= 0) recv_ids[o].push_back(c);
				}
			}
			for (auto* mp : {&send_ids, &recv_ids})
				for (auto& kv : *mp) std::sort(kv.second.begin(), kv.second.end());
		}
		DX_LAP("sr.5b_moving");
	}
	size_t bpc = 0;
	for (auto& f : g.fields) bpc += f.elem;
	const size_t n_recv = [&] {
		size_t k = 0;
		for (auto& kv : recv_ids) k += kv.second.size();
		return k;
	}();
	const size_t n_rm = n_keep + n_recv;
	// every rank takes part when any family merges (the host transport's
	// exchanges are collective)
	if (!F.empty()) {
		// removed store order: the kept children ascending, then per source
		// process (ascending rank) its children ascending
		for (auto& f : g.fields) {
			if (f.var) continue;
			f.removed.alloc(n_rm * f.elem + 1);
			if (n_keep) k_pack(f.data.p, f.elem, 0, f.elem, ksl.p, n_keep, f.removed.p, s);
		}
		std::vector<size_t> soff, roff;
		size_t so = 0, ro = 0;
		for (auto& kv : send_ids) {
			soff.push_back(so);
			so += kv.second.size() * bpc;
		}
		for (auto& kv : recv_ids) {
			roff.push_back(ro);
			ro += kv.second.size() * bpc;
		}
		if (recv_ids.empty()) {
			g.removed_ids.set_device(std::move(keep_ids), n_keep);
		} else {
			// the kept children, then the received ones per source process
			std::vector<uint64_t> all = download(keep_ids.p, n_keep, s);
			for (auto& kv : recv_ids) all.insert(all.end(), kv.second.begin(), kv.second.end());
			g.removed_ids.set_host(std::move(all));
		}
		DBuf<uint8_t> sbuf, rbuf;
		sbuf.alloc(so + 1);
		rbuf.alloc(ro + 1);
		size_t i = 0;
		for (auto& kv : send_ids) {
			const DBuf<int32_t> sl = slots_of(g, kv.second);
			size_t o = soff[i++];
			for (auto& f : g.fields) {
				if (f.var) continue;
				k_pack(f.data.p, f.elem, 0, f.elem, sl.p, kv.second.size(), sbuf.p + o, s);
				o += kv.second.size() * f.elem;
			}
		}
		if (!send_ids.empty()) HIP_CHECK(hipStreamSynchronize(s));  // (the slot lists' host vectors)
		std::vector<DevMsg> msgs;
		i = 0;
		size_t j = 0;
		for (int p = 0; p < g.size; p++) {
			if (p == g.rank) continue;
			DevMsg m{p, sbuf.p, 0, rbuf.p, 0};
			if (send_ids.count(p)) {
				m.send = sbuf.p + soff[i++];
				m.send_bytes = send_ids[p].size() * bpc;
			}
			if (recv_ids.count(p)) {
				m.recv = rbuf.p + roff[j++];
				m.recv_bytes = recv_ids[p].size() * bpc;
			}
			if (m.send_bytes || m.recv_bytes) msgs.push_back(m);
		}
		if (g.size > 1) comm_device_transfer(g, msgs, s);
		// field-major messages -> the removed store after the kept children
		j = 0;
		size_t at = n_keep;
		for (auto& kv : recv_ids) {
			size_t o = roff[j++];
			for (auto& f : g.fields) {
				if (f.var) continue;
				HIP_CHECK(hipMemcpyAsync(f.removed.p + at * f.elem, rbuf.p + o, kv.second.size() * f.elem,
				                         hipMemcpyDeviceToDevice, s));
				o += kv.second.size() * f.elem;
			}
			at += kv.second.size();
		}
		if (g.size > 1) HIP_CHECK(hipStreamSynchronize(s));  // the messages' buffers end with this scope
		// variable-size payloads: the kept children's, then the received ones
		if (std::any_of(g.fields.begin(), g.fields.end(), [](const Field& f) { return f.var; })) {
			std::vector<uint64_t> out_all;
			PeerRuns R;
			size_t so2 = 0, ro2 = 0;
			for (int p = 0; p < g.size; p++) {
				if (p == g.rank) continue;
				const size_t ns = count_of(send_ids, p), nr = count_of(recv_ids, p);
				if (ns) out_all.insert(out_all.end(), send_ids[p].begin(), send_ids[p].end());
				R.add(p, so2, ns, ro2, nr);
				so2 += ns;
				ro2 += nr;
			}
			const DBuf<int32_t> osl = slots_of(g, out_all);
			for (auto& f : g.fields) {
				if (!f.var) continue;
				VarMsg K, X;
				var_pack(f, ksl.p, n_keep, K, s);
				var_pack(f, osl.p, out_all.size(), X, s);
				if (g.size > 1) var_transfer(g, X, R, ro2, s);
				const size_t nk = n_keep;
				DBuf<uint64_t> sizes;
				sizes.alloc(n_rm + 1);
				if (nk) HIP_CHECK(hipMemcpyAsync(sizes.p, K.ssz.p, nk * 8, hipMemcpyDeviceToDevice, s));
				if (ro2) HIP_CHECK(hipMemcpyAsync(sizes.p + nk, X.rsz.p, ro2 * 8, hipMemcpyDeviceToDevice, s));
				f.rm_off.alloc(n_rm + 1);
				const uint64_t tot = scan_exclusive_u64(sizes.p, f.rm_off.p, n_rm, s);
				const uint64_t kb = std::accumulate(K.hs.begin(), K.hs.end(), uint64_t(0));
				f.removed.alloc(tot + 1);
				if (kb) HIP_CHECK(hipMemcpyAsync(f.removed.p, K.sbytes.p, kb, hipMemcpyDeviceToDevice, s));
				if (tot > kb) HIP_CHECK(hipMemcpyAsync(f.removed.p + kb, X.rbytes.p, tot - kb, hipMemcpyDeviceToDevice, s));
				HIP_CHECK(hipStreamSynchronize(s));
			}
		}
	}

	DX_LAP("sr.5_removed_payloads");
	// the known leaves: the current explicit list itself (read only), or the
	// implicit initial mesh written out
	Mesh materialized, nm;
	if (g.mesh.implicit) mesh_materialize(g, materialized);
	const Mesh& known = g.mesh.implicit ? materialized : g.mesh;
	nm.implicit = false;
	nm.bp = known.bp;
	{
		// the own leaves stay kid's prefix: refined ones expand in place into
		// their children (Morton order), a merged family's first child becomes
		// its parent, the other children drop out
		const size_t at[2] = {known.prefix_run1, known.n_prefix};
		size_t pos_at[2] = {0, 0};
		const DevMesh dm = g.dm();
		k_apply_refines(g.m, known.kid.p, known.kown.p, known.n_known, S, F, nm.kid, nm.kown, nm.n_known, s, at, pos_at,
		                known.n_prefix ? 2 : 0, known.n_prefix, &dm, g.size == 1 && known.n_prefix ? &nm.carry : nullptr,
		                dS.p, dF.p);
		nm.prefix_run1 = pos_at[0];
		nm.n_prefix = pos_at[1];
	}
	DX_LAP("sr.6_apply");
	rebuild(g, nm);
	DX_LAP("sr.7_rebuild");
	if (g.size == 1 && !F.empty()) {
		g.merged_dev = std::move(dF);
		g.n_merged = F.size();
	}
}

// --------------------------------------------------------------------------- load balance
__global__ void flag_slots_kernel(const int32_t* slots, size_t n, uint8_t* flag) {
	for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
		if (slots[i] >= 0) flag[slots[i]] = 1;
}

__global__ void keep_unflagged_kernel(const uint64_t* ids, const uint8_t* flag, size_t n, uint64_t* out,
                                      unsigned long long* counter) {
	// each lane a run of kAppendRun ids, one counter atomic per wave
	const size_t i0 = (blockIdx.x * size_t(blockDim.x) + threadIdx.x) * kAppendRun;
	unsigned c = 0;
	for (int k = 0; k < kAppendRun; k++)
		if (i0 + k < n && !flag[i0 + k]) c++;
	unsigned long long at = wave_reserve(counter, c);
	for (int k = 0; k < kAppendRun && c; k++)
		if (i0 + k < n && !flag[i0 + k]) {
			out[at++] = ids[i0 + k];
			c--;
		}
}

static DBuf<int32_t> slots_of(Grid& g, const std::vector<uint64_t>& ids) {
	DBuf<uint64_t> d;
	upload(d, ids, g.s_comp);
	DBuf<int32_t> sl, err;
	sl.alloc(ids.size() + 1);
	err.alloc(1);
	HIP_CHECK(hipMemsetAsync(err.p, 0, 4, g.s_comp));
	k_lookup_slots(d.p, ids.size(), g.dm(), sl.p, err.p, g.s_comp);
	int32_t h = 0;
	d2h_small(&h, err.p, 4, g.s_comp);
	DX_REQUIRE(h == 0, "migrating cell without a slot");
	return sl;
}

// initialize_balance_load (3746-3884) with make_new_partition's decisions
// (8349-8581): the partitioner's (use_partitioner, LB method not "NONE":
// rcb_partition in partition.hip), overridden by an export list of local
// cells given as data, overridden by the pins (8426-8518, they win).  The id
// lists go to their new owners (ascending id, the order make_new_partition
// sorts its receive lists in, 8482-8493) and the payloads of every field are
// packed per destination.  Cell weights are dropped (1011-1018).
void initialize_balance_load_impl(Grid& g, bool use_partitioner, const uint64_t* cells, const int32_t* procs,
                                  size_t n) {
	DX_REQUIRE(!g.mig.active, "balance_load already in progress");
	DX_REQUIRE(g.initialized, "not initialized");
	if (g.size > 1) comm_require(g, "balance_load");
	Migration& M = g.mig;
	M = Migration{};
	std::map<uint64_t, int> dest;
	if (use_partitioner && g.lb_method != "NONE") {
		std::vector<uint64_t> pc;
		std::vector<int32_t> po;
		rcb_partition(g, pc, po);
		for (size_t i = 0; i < pc.size(); i++)
			if (po[i] != g.rank) dest[pc[i]] = po[i];
	}
	g.weights.clear();
	g.refine_bulk.clear();
	g.refine_dev_valid = false;
	g.refine_dev.release();
	g.unrefine_dev_valid = false;
	g.unrefine_dev.release();
	g.unrefine_bulk.clear();
	g.refine_requests.clear();      // cells_to_refine (3808)
	g.unrefine_requests.clear();    // cells_to_unrefine (3810)
	g.dont_refine_cells.clear();    // cells_not_to_refine (3812)
	g.dont_unrefine_cells.clear();  // cells_not_to_unrefine (3813)
	g.removed_ids.clear();  // unrefined_cell_data (3811)
	for (auto& f : g.fields) {
		f.removed.release();
		f.rm_off.release();
	}
	if (n) {
		std::vector<int32_t> own(n);
		lookup_batch(g, cells, n, own.data(), nullptr);
		for (size_t i = 0; i < n; i++) {
			DX_REQUIRE(procs[i] >= 0 && procs[i] < g.size, "new process out of range");
			DX_REQUIRE(own[i] == g.rank, "balance_load: only local cells can be exported");
			if (procs[i] != g.rank) dest[cells[i]] = procs[i];
			else dest.erase(cells[i]);
		}
	}
	std::vector<uint64_t> pinned_out;
	for (auto& kv : g.pins) {
		if (kv.second != g.rank) dest[kv.first] = kv.second;
		else dest.erase(kv.first);
	}
	std::vector<std::vector<uint64_t>> out(size_t(g.size)), pin_out(size_t(g.size));
	for (auto& kv : dest) {
		out[size_t(kv.second)].push_back(kv.first);  // ascending (map order)
		if (g.pins.count(kv.first)) pin_out[size_t(kv.second)].push_back(kv.first);
	}
	const auto in = comm_alltoall_u64(g, out);
	const auto pin_in = comm_alltoall_u64(g, pin_out);
	for (auto& kv : dest) g.pins.erase(kv.first);
	for (int p = 0; p < g.size; p++) {
		if (p == g.rank) continue;
		if (!out[size_t(p)].empty()) M.out[p] = out[size_t(p)];
		if (!in[size_t(p)].empty()) M.in[p] = in[size_t(p)];
		M.in_pinned.insert(M.in_pinned.end(), pin_in[size_t(p)].begin(), pin_in[size_t(p)].end());
	}
	for (auto& f : g.fields) M.bytes_per_cell += f.elem;
	size_t so = 0, ro = 0;
	for (auto& kv : M.out) {
		M.out_off[kv.first] = so;
		so += kv.second.size() * M.bytes_per_cell;
	}
	for (auto& kv : M.in) {
		M.in_off[kv.first] = ro;
		ro += kv.second.size() * M.bytes_per_cell;
	}
	M.sendbuf.alloc(so + 1);
	M.recvbuf.alloc(ro + 1);
	for (auto& kv : M.out) {
		const DBuf<int32_t> sl = slots_of(g, kv.second);
		size_t o = M.out_off[kv.first];
		for (auto& f : g.fields) {
			if (f.var) continue;
			k_pack(f.data.p, f.elem, 0, f.elem, sl.p, kv.second.size(), M.sendbuf.p + o, g.s_comp);
			o += kv.second.size() * f.elem;
		}
	}
	// variable-size payloads of the leaving cells (peer by peer, ascending id)
	std::vector<uint64_t> leaving;
	for (auto& kv : M.out) leaving.insert(leaving.end(), kv.second.begin(), kv.second.end());
	const DBuf<int32_t> lsl = slots_of(g, leaving);
	for (auto& f : g.fields) {
		if (!f.var) continue;
		M.var.emplace_back();
		var_pack(f, lsl.p, leaving.size(), M.var.back(), g.s_comp);
	}
	HIP_CHECK(hipStreamSynchronize(g.s_comp));
	M.active = true;
}

// the runs of a migration's leaving / arriving cells per peer
static PeerRuns migration_runs(const Grid& g, const Migration& M, size_t& n_in) {
	PeerRuns R;
	size_t so = 0, ro = 0;
	for (int p = 0; p < g.size; p++) {
		if (p == g.rank) continue;
		const size_t ns = count_of(M.out, p), nr = count_of(M.in, p);
		R.add(p, so, ns, ro, nr);
		so += ns;
		ro += nr;
	}
	n_in = ro;
	return R;
}

// continue_balance_load (3899-3934): the payloads move
void continue_balance_load_impl(Grid& g) {
	Migration& M = g.mig;
	DX_REQUIRE(M.active, "continue_balance_load without initialize_balance_load");
	if (g.size > 1) {
		std::vector<DevMsg> msgs;
		for (int p = 0; p < g.size; p++) {
			if (p == g.rank) continue;
			const size_t sb = count_of(M.out, p) * M.bytes_per_cell, rb = count_of(M.in, p) * M.bytes_per_cell;
			msgs.push_back(DevMsg{p, M.sendbuf.p + off_of(M.out_off, p), sb, M.recvbuf.p + off_of(M.in_off, p), rb});
		}
		comm_device_transfer(g, msgs, g.s_comp);
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
		size_t n_in = 0;
		const PeerRuns R = migration_runs(g, M, n_in);
		for (VarMsg& vm : M.var) var_transfer(g, vm, R, n_in, g.s_comp);
	}
	M.transferred = true;
}

// finish_balance_load (3942-4147): the new own leaves, the ghost leaves
// fetched from their owners, every structure rebuilt, arrived payloads placed
void finish_balance_load_impl(Grid& g) {
	Migration& M = g.mig;
	DX_REQUIRE(M.active && M.transferred, "finish_balance_load before the payloads moved");
	hipStream_t s = g.s_comp;
	const size_t nl = g.n_local;
	std::vector<uint64_t> gone, arrived;
	for (auto& kv : M.out) gone.insert(gone.end(), kv.second.begin(), kv.second.end());
	for (auto& kv : M.in) arrived.insert(arrived.end(), kv.second.begin(), kv.second.end());
	DBuf<uint8_t> flag;
	flag.alloc(nl + 1);
	HIP_CHECK(hipMemsetAsync(flag.p, 0, nl + 1, s));
	if (!gone.empty()) {
		const DBuf<int32_t> sl = slots_of(g, gone);
		flag_slots_kernel<<<grid_for(gone.size(), 256), 256, 0, s>>>(sl.p, gone.size(), flag.p);
		HIP_CHECK(hipGetLastError());
	}
	DBuf<uint64_t> local;
	local.alloc(nl + arrived.size() + 1);
	DBuf<unsigned long long> ctr;
	ctr.alloc(1);
	HIP_CHECK(hipMemsetAsync(ctr.p, 0, 8, s));
	if (nl) {
		keep_unflagged_kernel<<<unsigned((nl + 256 * kAppendRun - 1) / (256 * kAppendRun)), 256, 0, s>>>(
		    g.slot_ids.p, flag.p, nl, local.p, ctr.p);
		HIP_CHECK(hipGetLastError());
	}
	unsigned long long kept = 0;
	d2h_small(&kept, ctr.p, 8, s);
	if (!arrived.empty())
		h2d(local.p + kept, arrived.data(), arrived.size() * 8, s);
	const size_t n_new = size_t(kept) + arrived.size();
	Mesh nm;
	mesh_from_local(g, nm, local, n_new);
	rebuild(g, nm);
	for (auto& kv : M.in) {
		const DBuf<int32_t> sl = slots_of(g, kv.second);
		size_t o = M.in_off[kv.first];
		for (auto& f : g.fields) {
			if (f.var) continue;
			k_place(M.recvbuf.p + o, f.elem, 0, f.elem, sl.p, kv.second.size(), f.data.p, s);
			field_written(f);
			o += kv.second.size() * f.elem;
		}
	}
	if (!arrived.empty() && !M.var.empty()) {
		const DBuf<int32_t> asl = slots_of(g, arrived);
		size_t k = 0;
		for (auto& f : g.fields) {
			if (!f.var) continue;
			VarMsg& vm = M.var[k++];
			var_place(f, g.n_slots, asl.p, arrived.size(), vm.rsz.p, vm.rbytes.p, s);
		}
	}
	HIP_CHECK(hipStreamSynchronize(s));
	for (uint64_t c : M.in_pinned) g.pins[c] = g.rank;
	g.mig = Migration{};
}

void migration_message_size(Grid& g, int peer, size_t& sb, size_t& rb) {
	const Migration& M = g.mig;
	DX_REQUIRE(M.active, "no balance_load in progress");
	DX_REQUIRE(M.var.empty(), "migration messages: variable-size fields move only with continue_balance_load");
	sb = count_of(M.out, peer) * M.bytes_per_cell;
	rb = count_of(M.in, peer) * M.bytes_per_cell;
}

void migration_pack_peer(Grid& g, int peer, uint8_t* buf, size_t cap) {
	Migration& M = g.mig;
	size_t sb, rb;
	migration_message_size(g, peer, sb, rb);
	DX_REQUIRE(cap >= sb, "buffer too small for the migration message");
	if (sb) {
		HIP_CHECK(hipMemcpyAsync(buf, M.sendbuf.p + off_of(M.out_off, peer), sb, hipMemcpyDefault, g.s_comp));
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
	}
}

void migration_place_peer(Grid& g, int peer, const uint8_t* buf, size_t bytes) {
	Migration& M = g.mig;
	size_t sb, rb;
	migration_message_size(g, peer, sb, rb);
	DX_REQUIRE(bytes == rb, "migration message has the wrong size");
	if (rb) {
		HIP_CHECK(hipMemcpyAsync(M.recvbuf.p + off_of(M.in_off, peer), buf, rb, hipMemcpyDefault, g.s_comp));
		HIP_CHECK(hipStreamSynchronize(g.s_comp));
	}
	M.transferred = true;
}

// --------------------------------------------------------------------------- game of life, slab planes
// The structured 26-point sweep needs the cells of a box in raster order.
// On a uniform level-0 grid whose ranks hold whole z-planes (the block
// partition, or any repartition into z-planes) a rank holds its planes in
// slot order [inner planes | outer planes] and receives each neighbor plane as
// one contiguous run of halo slots, so every region is a set of boxes whose
// z-1 / z+1 planes are other runs.
static int64_t plane_slot(Grid& g, int64_t z) {
	const int64_t nz = int64_t(g.len[2]);
	if (z < 0 || z >= nz) {
		if (!g.per[2]) return -2;  // outside the grid
		z = (z % nz + nz) % nz;
	}
	const uint64_t plane = g.len[0] * g.len[1];
	const uint64_t first = 1 + uint64_t(z) * plane, last = first + plane - 1;
	const int64_t a = lookup_slot(g, first), b = lookup_slot(g, last);
	if (a < 0 || b != a + int64_t(plane) - 1) return -1;  // not one contiguous run
	return a;
}

bool gol_slab_plan(Grid& g, std::vector<GolBox>& inner, std::vector<GolBox>& outer) {
	inner.clear();
	outer.clear();
	if (g.R != 0 || g.hood_len != 1 || g.len[0] % 256 != 0) return false;
	const uint64_t plane = g.len[0] * g.len[1];
	const int64_t nz = int64_t(g.len[2]);
	if (!g.n_local || g.n_local % plane != 0) return false;
	if (g.size == 1 && g.n_outer == 0 && g.n_slots == g.n_local && g.n_local == plane * uint64_t(nz)) {
		inner.push_back(GolBox{0, uint64_t(nz), -3, -3});  // -3: the kernel's own periodic wrap
		return true;
	}
	// the own cells must be whole planes, each one run of local slots of one
	// class (inner or outer); any number of z runs (e.g. a rank holding two
	// slabs after a repartition)
	std::vector<int64_t> own(size_t(nz), -1);
	uint64_t owned = 0;
	for (int64_t z = 0; z < nz; z++) {
		const int64_t s0 = plane_slot(g, z);
		if (s0 < 0 || uint64_t(s0) + plane > g.n_local) continue;
		if ((uint64_t(s0) < g.n_inner) != (uint64_t(s0) + plane - 1 < g.n_inner)) return false;
		own[size_t(z)] = s0;
		owned++;
	}
	if (owned * plane != g.n_local) return false;
	auto slot = [&](int64_t z) -> int64_t {
		return (z >= 0 && z < nz && own[size_t(z)] >= 0) ? own[size_t(z)] : plane_slot(g, z);
	};
	// boxes: runs of inner planes consecutive in z and in slots; every outer
	// plane alone; z-1 / z+1 of a box: another run (local or halo) or nothing
	for (int64_t z = 0; z < nz;) {
		if (own[size_t(z)] < 0) {
			z++;
			continue;
		}
		const bool in = uint64_t(own[size_t(z)]) < g.n_inner;
		int64_t e = z + 1;
		while (in && e < nz && own[size_t(e)] >= 0 && uint64_t(own[size_t(e)]) < g.n_inner &&
		       own[size_t(e)] == own[size_t(e - 1)] + int64_t(plane))
			e++;
		const int64_t lo = slot(z - 1), hi = slot(e);
		if (lo == -1 || hi == -1) return false;  // a neighbor plane not held as one run
		(in ? inner : outer).push_back(GolBox{uint64_t(own[size_t(z)]), uint64_t(e - z), lo, hi});
		z = e;
	}
	return true;
}

// --------------------------------------------------------------------------- get_cells(criteria)
// is_neighbor_type_match (dccrg.hpp:2946-3053) for every local row of a CSR pair
__global__ void neighbor_types_kernel(DevMesh M, int rank, const uint32_t* of_ptr, const uint64_t* of_id,
                                      const uint32_t* to_ptr, const uint64_t* to_id, size_t n, int32_t* types) {
	for (size_t r = blockIdx.x * size_t(blockDim.x) + threadIdx.x; r < n; r += size_t(gridDim.x) * blockDim.x) {
		int32_t t = 0;
		for (uint32_t e = of_ptr[r]; e < of_ptr[r + 1]; e++) {
			if (of_id[e] == error_cell) continue;
			t |= dm_owner(M, of_id[e]) == rank ? 1 : 4;
		}
		for (uint32_t e = to_ptr[r]; e < to_ptr[r + 1]; e++) {
			if (to_id[e] == error_cell) continue;
			t |= dm_owner(M, to_id[e]) == rank ? 2 : 8;
		}
		types[r] = t;
	}
}

std::vector<uint64_t> cells_by_criteria(Grid& g, const int32_t* crit, size_t nc, bool exact, int hood) {
	const size_t nl = g.n_local;
	const auto& sid = slot_ids_host(g);
	std::vector<uint64_t> out;
	if (nc == 0) {
		out.assign(sid.begin(), sid.begin() + ptrdiff_t(nl));
	} else {
		const uint32_t *op, *tp;
		const uint64_t *oi, *ti;
		if (hood == DCCRGX_DEFAULT_HOOD) {
			ensure_csr(g);
			op = g.nof_ptr.p;
			oi = g.nof_id.p;
			tp = g.nto_ptr.p;
			ti = g.nto_id.p;
		} else {
			UserHood& h = ensure_uhood(g, hood);
			op = h.nof_ptr.p;
			oi = h.nof_id.p;
			tp = h.nto_ptr.p;
			ti = h.nto_id.p;
		}
		DBuf<int32_t> t;
		t.alloc(nl + 1);
		if (nl) {
			neighbor_types_kernel<<<grid_for(nl, 256), 256, 0, g.s_comp>>>(g.dm(), g.rank, op, oi, tp, ti, nl, t.p);
			HIP_CHECK(hipGetLastError());
		}
		const std::vector<int32_t> ht = download(t.p, nl, g.s_comp);
		int32_t merged = 0;
		for (size_t k = 0; k < nc; k++) merged |= crit[k];
		for (size_t r = 0; r < nl; r++) {
			bool match = false;
			if (exact) {
				for (size_t k = 0; k < nc && !match; k++) match = ht[r] == crit[k];
			} else {
				match = (ht[r] & merged) != 0;
			}
			if (match) out.push_back(sid[r]);
		}
	}
	std::sort(out.begin(), out.end());
	return out;
}

}  // namespace dccrgx
