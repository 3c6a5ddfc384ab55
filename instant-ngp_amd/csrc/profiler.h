// profiler.h — optional per-phase HIP-event timing on the stream each kernel is launched on.
// Disabled by default (zero cost); bench.py enables it over its timed region (ngp_profiler_*).
#pragma once
#include "common.h"

namespace ngp {

bool profiler_enabled();
void profiler_record(const char* name, hipEvent_t start, hipEvent_t stop);
hipEvent_t profiler_event();

// Scopes are not timed while their stream is being captured into a graph: external event-record
// nodes are rejected by the HIP runtime PyTorch ships (ROCm 7.0), so graph-mode timing is taken from
// an eager replay instead (bench.py).
inline bool stream_capturing(hipStream_t s) {
	hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
	(void)hipStreamIsCapturing(s, &st);
	return st == hipStreamCaptureStatusActive;
}

struct ProfScope {
	const char* name;
	hipStream_t stream;
	hipEvent_t a = nullptr, b = nullptr;
	ProfScope(const char* n, hipStream_t s) : name(n), stream(s) {
		if (profiler_enabled() && !stream_capturing(s)) {
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
