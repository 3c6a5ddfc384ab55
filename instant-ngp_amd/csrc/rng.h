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
// Log-time jump ahead by delta draws. The classic loop squares the step map once per bit of delta:
// after k squarings the multiplier is m_k = M^(2^k) and the increment is inc * s_k with s_0 = 1,
// s_{k+1} = (m_k + 1) s_k (mod 2^64), both independent of the state. They are tabulated at compile time,
// so a bit costs the composition alone (bit k: am *= m_k, ap = ap m_k + inc s_k); the result is the
// same integer as the classic loop's (HostPcg32::advance).
struct PcgJumpTable { uint64_t m[64], s[64]; };
constexpr PcgJumpTable make_pcg_jump_table() {
	PcgJumpTable t{};
	uint64_t cm = 0x5851f42d4c957f2dULL, s = 1u;
	for (int k = 0; k < 64; ++k) {
		t.m[k] = cm;
		t.s[k] = s;
		s = (cm + 1) * s;
		cm *= cm;
	}
	return t;
}
static __constant__ PcgJumpTable c_pcg_jump = make_pcg_jump_table();
constexpr uint64_t pcg_advance_classic(uint64_t state, uint64_t inc, uint64_t delta) {
	uint64_t cm = 0x5851f42d4c957f2dULL, cp = inc, am = 1u, ap = 0u;
	for (; delta; delta /= 2) {
		if (delta & 1) { am *= cm; ap = ap * cm + cp; }
		cp = (cm + 1) * cp; cm *= cm;
	}
	return am * state + ap;
}
constexpr uint64_t pcg_advance_tabulated(uint64_t state, uint64_t inc, uint64_t delta) {
	const PcgJumpTable t = make_pcg_jump_table();
	uint64_t am = 1u, ap = 0u;
	for (uint32_t k = 0; delta; ++k, delta >>= 1)
		if (delta & 1) { am *= t.m[k]; ap = ap * t.m[k] + inc * t.s[k]; }
	return am * state + ap;
}
static_assert(pcg_advance_tabulated(0x853c49e6748fea9bULL, 0xda3e39cb94b95bdbULL, 0x3fffff0ULL) ==
              pcg_advance_classic(0x853c49e6748fea9bULL, 0xda3e39cb94b95bdbULL, 0x3fffff0ULL), "pcg jump table");
static_assert(pcg_advance_tabulated(12345u, 54321u | 1u, 0xfedcba9876543210ULL) ==
              pcg_advance_classic(12345u, 54321u | 1u, 0xfedcba9876543210ULL), "pcg jump table");

template <typename R>
__device__ __forceinline__ void pcg_advance(R& r, uint64_t delta) {
	uint64_t am = 1u, ap = 0u;
	for (uint32_t k = 0; delta; ++k, delta >>= 1) {  // k is the same in every lane: scalar table loads
		if (delta & 1) {
			const uint64_t m = c_pcg_jump.m[k];
			am *= m;
			ap = ap * m + r.inc * c_pcg_jump.s[k];
		}
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
