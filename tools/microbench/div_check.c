// Exhaustive check of the sampler's division by MIN_CONE_STEPSIZE (nerf.hip div_min_stepsize):
// q = t * RN(1/c); q' = fma(fma(-q, c, t), RN(1/c), q) against the IEEE quotient t / c for every
// non-negative finite float t. Prints the largest failing t below 1 and the smallest failing t above 1.
// Build: gcc -O2 -ffp-contract=off -o /tmp/div_check tools/microbench/div_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

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
	printf("mismatches %lld; largest failing t < 1: %g; smallest failing t > 1: %g\n", (long long)bad, a, z);
	return 0;
}
