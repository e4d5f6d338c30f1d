// Process-wide caching pool of device memory behind every DBuf
// (dccrgx_internal.hpp).  hipFree synchronises the whole device and unmaps
// the block (~0.08 ms a call; an adaptive advection step of config 3 made
// ~120 of them), so released blocks are kept and handed to later requests of
// a similar size.
//
// Ordering: a block released while queued work may still use it goes to
// `pending`; it becomes reusable only after a device synchronisation, done on
// demand when a request finds no ready block but a pending one - the same
// guarantee hipFree gave, paid once for every block pending at that moment.
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "dccrgx_internal.hpp"

namespace dccrgx {

namespace {

// cached bytes kept at most (the rest is hipFree'd): 16 GiB, or
// DCCRGX_POOL_MAX_MB (processes sharing one GPU - the host transport - each
// take their share; the facade sets it from the ranks per device)
size_t max_held() {
	static const size_t v = [] {
		const char* e = std::getenv("DCCRGX_POOL_MAX_MB");
		return e && *e ? size_t(std::strtoull(e, nullptr, 10)) << 20 : size_t(16) << 30;
	}();
	return v;
}
constexpr size_t kBig = size_t(1) << 20;

struct Pool {
	std::mutex mu;
	std::multimap<size_t, void*> ready;    // reusable now
	std::multimap<size_t, void*> pending;  // released, reusable after a device synchronisation
	size_t held = 0;                       // bytes in ready + pending
};

// never destroyed: blocks outlive static destruction and go with the process
Pool& pool() {
	static Pool* p = new Pool();
	return *p;
}

// size classes: powers of two up to 1 MiB, 2-MiB multiples above
size_t size_class(size_t b) {
	if (b <= kBig) {
		size_t r = 256;
		while (r < b) r <<= 1;
		return r;
	}
	const size_t g = size_t(2) << 20;
	return (b + g - 1) / g * g;
}

// a block of at least `want` bytes and at most a quarter more (exact class
// for small blocks)
bool take(Pool& P, std::multimap<size_t, void*>& m, size_t want, void*& out, size_t& cap) {
	auto it = m.lower_bound(want);
	if (it == m.end()) return false;
	if (want <= kBig ? it->first != want : it->first > want + want / 4) return false;
	out = it->second;
	cap = it->first;
	P.held -= cap;
	m.erase(it);
	return true;
}

void retire_pending(Pool& P) {
#if DCCRGX_PHASE_TIMING
	const double t0 = PhaseScope::now();
	HIP_CHECK(hipDeviceSynchronize());
	phase_add("pool.sync", PhaseScope::now() - t0);
#else
	HIP_CHECK(hipDeviceSynchronize());
#endif
	P.ready.insert(P.pending.begin(), P.pending.end());
	P.pending.clear();
}

void free_all(Pool& P) {
	(void)hipDeviceSynchronize();
	for (auto* m : {&P.ready, &P.pending}) {
		for (auto& kv : *m) (void)hipFree(kv.second);
		m->clear();
	}
	P.held = 0;
}

}  // namespace

void* pool_alloc(size_t bytes, size_t& cap) {
	const size_t want = size_class(bytes);
	Pool& P = pool();
	std::lock_guard<std::mutex> lock(P.mu);
	void* out = nullptr;
	if (take(P, P.ready, want, out, cap)) return out;
	{
		auto it = P.pending.lower_bound(want);
		if (it != P.pending.end() && (want <= kBig ? it->first == want : it->first <= want + want / 4)) {
			retire_pending(P);
			if (take(P, P.ready, want, out, cap)) return out;
		}
	}
#if DCCRGX_PHASE_TIMING
	const double t0 = PhaseScope::now();
	hipError_t e = hipMalloc(&out, want);
	phase_add("pool.hipMalloc", PhaseScope::now() - t0);
#else
	hipError_t e = hipMalloc(&out, want);
#endif
	if (e != hipSuccess) {  // out of memory: give the cached blocks back and retry once
		(void)hipGetLastError();
		free_all(P);
		e = hipMalloc(&out, want);
	}
	if (e != hipSuccess) {
		(void)hipGetLastError();
		throw Error(DCCRGX_EHIP, "device allocation of " + std::to_string(want) + " bytes failed: " +
		                             hipGetErrorString(e));
	}
	cap = want;
	return out;
}

void pool_free(void* raw, size_t cap) {
	if (!raw) return;
	Pool& P = pool();
	std::lock_guard<std::mutex> lock(P.mu);
	if (P.held + cap > max_held()) {
		(void)hipFree(raw);
		return;
	}
	P.pending.insert({cap, raw});
	P.held += cap;
}

// Device -> host reads of up to kSmallRead bytes (counters, totals, error
// flags, the adaptive step's lists) through a pinned staging buffer per host
// thread: a pageable destination costs ~15 us more per small read than a
// pinned one on MI355X (scripts/microbench/d2h_small.hip: 27 vs 15 us per
// kernel + read + sync, 12 for the sync alone), and list-sized reads (~200
// KB) 45-65 us through pageable memory in the adaptive step's HIP trace
// (r06m).  The buffer is kept for the thread's life (never freed: a
// thread_local destructor may run after the HIP runtime is gone).
void d2h_small(void* host, const void* dev, size_t bytes, hipStream_t s) {
	if (!bytes) return;
	thread_local void* stage = nullptr;
	if (bytes <= kSmallRead) {
		if (!stage) HIP_CHECK(hipHostMalloc(&stage, kSmallRead, hipHostMallocDefault));
		HIP_CHECK(hipMemcpyAsync(stage, dev, bytes, hipMemcpyDeviceToHost, s));
		HIP_CHECK(hipStreamSynchronize(s));
		std::memcpy(host, stage, bytes);
		return;
	}
	HIP_CHECK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s));
	HIP_CHECK(hipStreamSynchronize(s));
}

// Host -> device copies of list-sized buffers (256 B .. 256 KiB) through a
// pinned staging buffer per host thread: a pageable 64-KiB upload costs
// 85 us against 21 from pinned memory on MI355X, the stream sync included
// (scripts/microbench/h2d_small.hip); smaller and larger ones go directly
// (pageable is as fast there).  The staged copy is waited for before
// returning (the buffer is reused by the next upload; an event per staging
// slot instead is unsafe here: grids destroy their streams, and HIP refuses
// to wait on an event last recorded on a destroyed stream).
void h2d(void* dev, const void* host, size_t bytes, hipStream_t s) {
	if (!bytes) return;
	if (bytes < 256 || bytes > kStageUp) {
		HIP_CHECK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
		return;
	}
	thread_local void* stage = nullptr;
	if (!stage) HIP_CHECK(hipHostMalloc(&stage, kStageUp, hipHostMallocDefault));
	std::memcpy(stage, host, bytes);
	HIP_CHECK(hipMemcpyAsync(dev, stage, bytes, hipMemcpyHostToDevice, s));
	HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace dccrgx
