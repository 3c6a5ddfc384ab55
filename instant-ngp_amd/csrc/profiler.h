// profiler.h — optional per-phase HIP-event timing on the stream each kernel is launched on.
// Disabled by default (zero cost); bench.py enables it over its timed region (ngp_profiler_*).
#pragma once
#include "common.h"

namespace ngp {

bool profiler_enabled();
void profiler_record(const char* name, hipEvent_t start, hipEvent_t stop);
hipEvent_t profiler_event();

struct ProfScope {
	const char* name;
	hipStream_t stream;
	hipEvent_t a = nullptr, b = nullptr;
	ProfScope(const char* n, hipStream_t s) : name(n), stream(s) {
		if (profiler_enabled()) {
			a = profiler_event();
			b = profiler_event();
			NGP_HIP(hipEventRecord(a, s));
		}
	}
	~ProfScope() {
		if (a) {
			(void)hipEventRecord(b, stream);
			profiler_record(name, a, b);
		}
	}
};

}  // namespace ngp
