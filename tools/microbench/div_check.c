// Exhaustive checks of the sampler's divisions against the IEEE quotient, for every non-negative
// finite float t (negative t: both forms are odd in t):
//  - by MIN_CONE_STEPSIZE (nerf.hip div_min_stepsize): q = t * RN(1/c); q' = fma(fma(-q, c, t), RN(1/c), q);
//    prints the largest failing t below 1 and the smallest failing t above 1;
//  - by log(1 + cone) (ngp_math.h ngp_div_rc, the stepping space's exponential segment) at the
//    default cone 1/256: counts mismatches over the range ngp_div_rc refines (2^-100 .. 2^100).
// Build: gcc -O2 -ffp-contract=off -I instant-ngp_amd/csrc -o /tmp/div_check tools/microbench/div_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "ngp_math.h"

int main(void) {
	const float c = 1.73205080757f / 1024;  // MIN_CONE_STEPSIZE (testbed_nerf.cu:65-71)
	volatile float cv = c;
	const float r = 1.0f / cv;
	int64_t last_small = -1, first_big = -1, bad = 0;
	for (int64_t u = 0; u < 0x7f800000LL; ++u) {
		const uint32_t b = (uint32_t)u;
		float t;
		memcpy(&t, &b, 4);
		const float ref = t / cv, q = t * r, q2 = fmaf(fmaf(-q, c, t), r, q);
		if (memcmp(&ref, &q2, 4) != 0) {
			++bad;
			if (t < 1.0f) last_small = u;
			else if (first_big < 0) first_big = u;
		}
	}
	float a, z;
	const uint32_t x = (uint32_t)last_small, y = (uint32_t)first_big;
	memcpy(&a, &x, 4);
	memcpy(&z, &y, 4);
	printf("MIN_CONE_STEPSIZE: mismatches %lld; largest failing t < 1: %g; smallest failing t > 1: %g\n", (long long)bad, a, z);

	volatile float cone = 1.0f / 256;
	const float l = ngp_logf(1.0f + cone), rl = 1.0f / l;
	int64_t bad2 = 0, n2 = 0;
	for (int64_t u = 0x0d800000LL; u <= 0x71800000LL; ++u) {  // 2^-100 .. 2^100
		const uint32_t b = (uint32_t)u;
		float t;
		memcpy(&t, &b, 4);
		volatile float lv = l;
		const float ref = t / lv, q2 = ngp_div_rc(t, l, rl);
		++n2;
		if (memcmp(&ref, &q2, 4) != 0) ++bad2;
	}
	printf("log(1 + 1/256) = %.9g: ngp_div_rc mismatches %lld of %lld\n", l, (long long)bad2, (long long)n2);
	return bad2 != 0;
}
