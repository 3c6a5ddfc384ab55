// What a cross-queue dependency costs on the GPU timeline (the NeRF step shows ~11 us between the
// sampler's last kernel and the inference that waits for it). Kernels stamp the 100-MHz wall clock at their start
// and end; the gap is (start of the kernel after the dependency) - (end of the kernel before it), median of 30.
//   S0  one queue: K1 (spin) then K2, no wait                                  (in-queue launch gap)
//   S1  queue B: K1 (spin), wait on an event of queue A that completed long ago, K2
//   S2  queue B: K1 (spin 200 us), wait on an event recorded on A after a 100-us spin (satisfied at K1's end), K2
//   S3  as S2, A's work a captured HIP graph (the NeRF step's training pass) and the event recorded after it
//   S4  queue B: K1 (spin) and an event after it; queue A (idle) waits on it, then K2   (pending dependency)
//   S5  as S1 with a timing event (hipEventDefault) instead of hipEventDisableTiming
//   S6  as S1 with hipStreamWriteValue32 on A and hipStreamWaitValue32 on B (signal memory) instead of the event
//   S7  as S4 with the write / wait value pair (the NeRF step's sampler -> inference handoff since round 6)
// Build: hipcc --offload-arch=gfx950 -O2 -o queue_handoff queue_handoff.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(err_)); exit(1); } } while (0)

// one wave: stamps its start in out[0], spins `ticks` of the wall clock, stamps its end in out[1] (vector stores)
__global__ void k_spin(unsigned long long ticks, unsigned long long* out) {
	const unsigned long long t0 = wall_clock64();
	while (wall_clock64() - t0 < ticks) {}
	const unsigned long long t1 = wall_clock64();
	if (threadIdx.x == 0) { out[0] = t0; out[1] = t1; }
}

static double median(std::vector<double> v) {
	std::sort(v.begin(), v.end());
	return v[v.size() / 2];
}

int main() {
	int rate_khz = 0;
	CHECK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
	const double us_per_tick = 1e3 / rate_khz;
	const unsigned long long T100 = (unsigned long long)(100.0 / us_per_tick), T200 = 2 * T100, T5 = T100 / 20;
	unsigned long long* d;
	CHECK(hipMalloc(&d, 64 * 8));
	hipStream_t A, B;
	CHECK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
	CHECK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
	hipEvent_t ev, evt;
	CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
	CHECK(hipEventCreateWithFlags(&evt, hipEventDefault));
	// the graph of S3: one 100-us spin captured on A
	hipGraph_t g;
	hipGraphExec_t ge;
	CHECK(hipStreamBeginCapture(A, hipStreamCaptureModeThreadLocal));
	k_spin<<<1, 64, 0, A>>>(T100, d + 8);
	CHECK(hipStreamEndCapture(A, &g));
	CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
	void* sig = nullptr;
	CHECK(hipExtMallocWithFlags(&sig, 8, hipMallocSignalMemory));
	CHECK(hipMemset(sig, 0, 8));
	uint32_t seq = 0;
	const char* names[8] = {"S0 in-queue", "S1 wait, long done", "S2 wait, done at K1 end", "S3 wait on graph, done",
	                        "S4 pending dependency", "S5 as S1, timing event", "S6 as S1, wait value",
	                        "S7 as S4, write / wait value"};
	for (int sc = 0; sc < 8; ++sc) {
		std::vector<double> gaps;
		for (int rep = 0; rep < 31; ++rep) {
			CHECK(hipDeviceSynchronize());
			hipStream_t q2 = B;  // the queue K2 runs on
			switch (sc) {
			case 0:
				k_spin<<<1, 64, 0, B>>>(T200, d);
				break;
			case 1: case 5: {
				hipEvent_t e = sc == 5 ? evt : ev;
				k_spin<<<1, 64, 0, A>>>(T5, d + 8);
				CHECK(hipEventRecord(e, A));
				CHECK(hipStreamSynchronize(A));
				k_spin<<<1, 64, 0, B>>>(T200, d);
				CHECK(hipStreamWaitEvent(B, e, 0));
				break;
			}
			case 2:
				k_spin<<<1, 64, 0, A>>>(T100, d + 8);
				CHECK(hipEventRecord(ev, A));
				k_spin<<<1, 64, 0, B>>>(T200, d);
				CHECK(hipStreamWaitEvent(B, ev, 0));
				break;
			case 3:
				CHECK(hipGraphLaunch(ge, A));
				CHECK(hipEventRecord(ev, A));
				k_spin<<<1, 64, 0, B>>>(T200, d);
				CHECK(hipStreamWaitEvent(B, ev, 0));
				break;
			case 6:
				k_spin<<<1, 64, 0, A>>>(T5, d + 8);
				CHECK(hipStreamWriteValue32(A, sig, ++seq, 0));
				CHECK(hipStreamSynchronize(A));
				k_spin<<<1, 64, 0, B>>>(T200, d);
				CHECK(hipStreamWaitValue32(B, sig, seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
				break;
			case 7:
				k_spin<<<1, 64, 0, B>>>(T200, d);
				CHECK(hipStreamWriteValue32(B, sig, ++seq, 0));
				CHECK(hipStreamWaitValue32(A, sig, seq, hipStreamWaitValueGte, 0xFFFFFFFFu));
				q2 = A;
				break;
			case 4:
				k_spin<<<1, 64, 0, B>>>(T200, d);
				CHECK(hipEventRecord(ev, B));
				CHECK(hipStreamWaitEvent(A, ev, 0));
				q2 = A;
				break;
			}
			k_spin<<<1, 64, 0, q2>>>(T5, d + 2);
			CHECK(hipDeviceSynchronize());
			unsigned long long h[4];
			CHECK(hipMemcpy(h, d, 32, hipMemcpyDeviceToHost));
			if (rep) gaps.push_back((double)(h[2] - h[1]) * us_per_tick);
		}
		printf("{\"scenario\": \"%s\", \"gap_us_median\": %.2f, \"gap_us_min\": %.2f, \"gap_us_max\": %.2f}\n", names[sc], median(gaps),
		       *std::min_element(gaps.begin(), gaps.end()), *std::max_element(gaps.begin(), gaps.end()));
	}
	return 0;
}
