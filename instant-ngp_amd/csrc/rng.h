// rng.h — tcnn::pcg32 on the device (PCG-XSH-RR 64/32, random_val.cuh:26-43 via tcnn's pcg32.h;
// restated, tcnn absent: SURVEY F1). Works on any struct with uint64_t state, inc.
#pragma once
#include "common.h"

namespace ngp {

struct Pcg32Dev { uint64_t state, inc; };

template <typename R>
__device__ __forceinline__ uint32_t pcg_next(R& r) {
	const uint64_t old = r.state;
	r.state = old * 0x5851f42d4c957f2dULL + r.inc;
	const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u), rot = (uint32_t)(old >> 59u);
	return (xs >> rot) | (xs << ((~rot + 1u) & 31));
}
// next_float: bits (u >> 9 | 0x3f800000) - 1 (random_val.cuh:150-153)
template <typename R>
__device__ __forceinline__ float pcg_float(R& r) { return __uint_as_float((pcg_next(r) >> 9) | 0x3f800000u) - 1.0f; }
// log-time jump ahead by delta draws
template <typename R>
__device__ __forceinline__ void pcg_advance(R& r, uint64_t delta) {
	uint64_t cm = 0x5851f42d4c957f2dULL, cp = r.inc, am = 1u, ap = 0u;
	while (delta > 0) {
		if (delta & 1) { am *= cm; ap = ap * cm + cp; }
		cp = (cm + 1) * cp; cm *= cm; delta /= 2;
	}
	r.state = am * r.state + ap;
}

// host mirror (Testbed::m_rng lives on the host; kernels get it by value)
struct HostPcg32 {
	uint64_t state, inc;
	void advance(uint64_t delta) {
		uint64_t cm = 0x5851f42d4c957f2dULL, cp = inc, am = 1u, ap = 0u;
		while (delta > 0) {
			if (delta & 1) { am *= cm; ap = ap * cm + cp; }
			cp = (cm + 1) * cp; cm *= cm; delta /= 2;
		}
		state = am * state + ap;
	}
};

}  // namespace ngp
