// profiler.hip — event pool + per-phase accumulation behind ngp_profiler_* (include/ngp_engine.h).
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ngp_engine.h"
#include "profiler.h"

namespace ngp {

namespace {
struct Pending { std::string name; hipEvent_t a, b; };
struct Stat { uint64_t calls = 0; double ms = 0.0; };
std::mutex mu;
bool enabled = false;
std::vector<hipEvent_t> pool;
std::vector<Pending> pending;
std::map<std::string, Stat> stats;

void drain() {
	for (auto& p : pending) {
		(void)hipEventSynchronize(p.b);
		float ms = 0.f;
		(void)hipEventElapsedTime(&ms, p.a, p.b);
		auto& s = stats[p.name];
		s.calls++;
		s.ms += ms;
		pool.push_back(p.a);
		pool.push_back(p.b);
	}
	pending.clear();
}
}  // namespace

bool profiler_enabled() { return enabled; }

hipEvent_t profiler_event() {
	std::lock_guard<std::mutex> l(mu);
	if (pool.empty()) {
		hipEvent_t e;
		NGP_HIP(hipEventCreateWithFlags(&e, hipEventDefault));
		return e;
	}
	hipEvent_t e = pool.back();
	pool.pop_back();
	return e;
}

void profiler_record(const char* name, hipEvent_t a, hipEvent_t b) {
	std::lock_guard<std::mutex> l(mu);
	pending.push_back({name, a, b});
	if (pending.size() > 4096) drain();
}

}  // namespace ngp

extern "C" {

int ngp_profiler_enable(int enable) {
	std::lock_guard<std::mutex> l(ngp::mu);
	ngp::enabled = enable != 0;
	// events are created up front: creating them while a stream is being captured into a graph fails
	while (ngp::enabled && ngp::pool.size() < 8192) {
		hipEvent_t e;
		if (hipEventCreateWithFlags(&e, hipEventDefault) != hipSuccess) return NGP_ERROR;
		ngp::pool.push_back(e);
	}
	return NGP_OK;
}

int ngp_profiler_reset(void) {
	std::lock_guard<std::mutex> l(ngp::mu);
	ngp::drain();
	ngp::stats.clear();
	return NGP_OK;
}

// JSON object {"phase": {"calls": n, "ms": total}, ...}; returns the needed length (incl. NUL)
int ngp_profiler_read(char* buf, size_t len) {
	std::lock_guard<std::mutex> l(ngp::mu);
	ngp::drain();
	std::string s = "{";
	bool first = true;
	for (auto& kv : ngp::stats) {
		if (!first) s += ", ";
		first = false;
		s += "\"" + kv.first + "\": {\"calls\": " + std::to_string(kv.second.calls) + ", \"ms\": " + std::to_string(kv.second.ms) + "}";
	}
	s += "}";
	if (buf && len) {
		size_t n = std::min(len - 1, s.size());
		memcpy(buf, s.data(), n);
		buf[n] = 0;
	}
	return (int)s.size() + 1;
}

}  // extern "C"
