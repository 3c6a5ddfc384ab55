/* ngp_math.h — the single expf/logf used wherever a transcendental decides an integer result.
 *
 * The reference computes the cone-angle stepping (to/from_stepping_space, src/testbed_nerf.cu:114-184)
 * with logf/expf and the compositing weights of the loss pass (:1740-1760, network_to_density :357-365)
 * with __expf. Those floats decide integers: the number of steps of every ray (and so every sample
 * index of the batch) and where a ray's compositing terminates (and so the compacted sample count and
 * the compacted base of every ray). Two libm implementations that differ by one ulp move those
 * integers, so the engine's device kernels and the CPU oracle (oracle/ngp_nerf_oracle.c) both include
 * this header and evaluate the same instruction sequence: +, -, *, fmaf (fused, one rounding on both
 * sides), one IEEE division, floorf and exponent bit manipulation. Both sides compile with
 * -ffp-contract=off, so nothing else is fused.
 *
 * Accuracy (tests/test_oracle.py::test_shared_math_accuracy, against float64 numpy): measured
 * < 1 ulp for both over random normal inputs and all positive float bit patterns sampled; the test
 * bounds them at 1 ulp. The reference's own logf/expf/__expf are CUDA libdevice
 * approximations of the same ulp class, so this costs nothing against the reference.
 *
 * Plain C99 and HIP C++: NGP_MATH_FN adds __host__ __device__ under hipcc.
 */
#ifndef NGP_MATH_H
#define NGP_MATH_H

#include <stdint.h>

#ifndef NGP_LOGF_FASTDIV
#define NGP_LOGF_FASTDIV 1  /* device: the logf's f / (2 + f) without the IEEE division sequence (ngp_div_2pf) */
#endif

#if defined(__HIPCC__)
#define NGP_MATH_FN static __host__ __device__ __forceinline__
#define NGP_FMAF(a, b, c) __builtin_fmaf((a), (b), (c))
#define NGP_FLOORF(x) __builtin_floorf(x)
#else
#include <math.h>
#define NGP_MATH_FN static inline
#define NGP_FMAF(a, b, c) fmaf((a), (b), (c))
#define NGP_FLOORF(x) floorf(x)
#endif

NGP_MATH_FN uint32_t ngp_math_f2u(float f) {
	union { float f; uint32_t u; } v;
	v.f = f;
	return v.u;
}
NGP_MATH_FN float ngp_math_u2f(uint32_t u) {
	union { float f; uint32_t u; } v;
	v.u = u;
	return v.f;
}

/* e^x: x = k ln2 + r (Cody-Waite two-part ln2, |r| <= 0.35), e^r by a degree-7 Taylor polynomial in
 * Horner form (truncation 5e-9 relative), scaled by 2^k through the exponent bits (two factors when
 * the result is subnormal). */
/* the polynomial e^r and k of x (x finite, no overflow/underflow checks) */
NGP_MATH_FN float ngp_expf_poly(float x, float* kout) {
	const float k = NGP_FLOORF(NGP_FMAF(x, 1.44269502162933349609375f, 0.5f));
	float r = NGP_FMAF(-k, 0.693145751953125f, x);
	r = NGP_FMAF(-k, 1.428606765330187045e-06f, r);
	float p = 1.98412701138295233249664306640625e-4f; /* 1/5040 */
	p = NGP_FMAF(p, r, 1.38888892251998186111450195312500e-3f); /* 1/720 */
	p = NGP_FMAF(p, r, 8.33333376795053482055664062500000e-3f); /* 1/120 */
	p = NGP_FMAF(p, r, 4.16666679084300994873046875000000e-2f); /* 1/24 */
	p = NGP_FMAF(p, r, 1.66666671633720397949218750000000e-1f); /* 1/6 */
	p = NGP_FMAF(p, r, 0.5f);
	p = NGP_FMAF(p, r, 1.0f);
	p = NGP_FMAF(p, r, 1.0f);
	*kout = k;
	return p;
}
/* e^x for |x| <= 80 (normal result: the scale 2^k is one normal factor): same operations and value as
 * ngp_expf there, without its range checks (the stepping space's exponential segment) */
NGP_MATH_FN float ngp_expf_mid(float x) {
	float k;
	const float p = ngp_expf_poly(x, &k);
	return p * ngp_math_u2f((uint32_t)((int)k + 127) << 23);
}
NGP_MATH_FN float ngp_expf(float x);
/* ngp_expf with the common case |x| <= 80 first (no further checks there; NaN and the rest take the
 * full path): same value as ngp_expf for every x */
NGP_MATH_FN float ngp_expf_fast(float x) {
	const float ax = x < 0.0f ? -x : x;
	if (ax <= 80.0f) return ngp_expf_mid(x);
	return ngp_expf(x);
}
NGP_MATH_FN float ngp_expf(float x) {
	if (x != x) return x;
	if (x > 88.72283935546875f) return ngp_math_u2f(0x7f800000u);
	if (x < -103.97208404541015625f) return 0.0f;
	float k;
	const float p = ngp_expf_poly(x, &k);
	const int ki = (int)k;
	if (ki >= -126 && ki <= 127) return p * ngp_math_u2f((uint32_t)(ki + 127) << 23);
	/* ki in [-150, -127] or 128: split the scale so both factors are normal */
	const int k1 = ki < 0 ? -100 : 64;
	return (p * ngp_math_u2f((uint32_t)(k1 + 127) << 23)) * ngp_math_u2f((uint32_t)(ki - k1 + 127) << 23);
}

/* ln x (FreeBSD e_logf.c algorithm): x = 2^e m with m in [sqrt(2)/2, sqrt(2)), f = m - 1,
 * s = f / (2 + f), log(1+f) = f - f^2/2 + s (f^2/2 + R(s^2)), e ln2 added in two parts.
 * The polynomial constants Lg1..Lg4 and the ln2 hi/lo split below are those of fdlibm's e_logf.c,
 * which carries this notice:
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this software is freely granted,
 *   provided that this notice is preserved. */
/* f / (2 + f) for the reduced argument of ngp_logf_core, f = m - 1 with m in [sqrt(2)/2, sqrt(2)) (2^23
 * values): the IEEE quotient. On the device it is a reciprocal, one Newton step and one fused residual
 * step (six dependent operations instead of the eleven of the IEEE division sequence), which equals the
 * IEEE quotient for every one of those f: ngp_debug_math_check compares the two over the whole range on
 * the GPU (tests/test_gpu_math.py). The host keeps the division. */
NGP_MATH_FN float ngp_div_2pf(float f) {
#if defined(__HIP_DEVICE_COMPILE__) && NGP_LOGF_FASTDIV
	const float b = 2.0f + f;
	float r = __builtin_amdgcn_rcpf(b);
	r = NGP_FMAF(NGP_FMAF(-b, r, 1.0f), r, r);
	const float q = f * r;
	return NGP_FMAF(NGP_FMAF(-b, q, f), r, q);
#else
	return f / (2.0f + f);
#endif
}
/* ln x for x = 2^(e0) m already reduced to ix = its bits (positive, normal) */
NGP_MATH_FN float ngp_logf_core(uint32_t ix, int e);
NGP_MATH_FN float ngp_logf(float x) {
	uint32_t ix = ngp_math_f2u(x);
	if (x != x) return x;
	if (x < 0.0f) return ngp_math_u2f(0x7fc00000u);
	if (x == 0.0f) return ngp_math_u2f(0xff800000u);
	if (ix == 0x7f800000u) return x;
	int e = 0;
	if (ix < 0x00800000u) { /* subnormal: scale by 2^25 */
		x *= 33554432.0f;
		ix = ngp_math_f2u(x);
		e = -25;
	}
	return ngp_logf_core(ix, e);
}
/* ln x for positive normal finite x: same operations and value as ngp_logf there, without its
 * special-case checks (the stepping space's logarithmic segment) */
NGP_MATH_FN float ngp_logf_pos(float x) { return ngp_logf_core(ngp_math_f2u(x), 0); }
NGP_MATH_FN float ngp_logf_core(uint32_t ix, int e) {
	/* m in [sqrt(2)/2, sqrt(2)): bias the mantissa by (1 - sqrt(2)/2) so the exponent step falls there */
	ix += 0x3f800000u - 0x3f3504f3u;
	e += (int)(ix >> 23) - 127;
	ix = (ix & 0x007fffffu) + 0x3f3504f3u;
	const float f = ngp_math_u2f(ix) - 1.0f;
	const float s = ngp_div_2pf(f);
	const float z = s * s, w = z * z;
	const float t1 = w * NGP_FMAF(w, 0.24279078841f, 0.40000972152f);
	const float t2 = z * NGP_FMAF(w, 0.28498786688f, 0.66666662693f);
	const float R = t2 + t1;
	const float hfsq = 0.5f * f * f;
	const float dk = (float)e;
	/* ln2 = 6.9313812256e-01 (hi: dk * hi is exact) + 9.0580006145e-06 (lo) */
	return dk * 6.9313812256e-01f - ((hfsq - (s * (hfsq + R) + dk * 9.0580006145e-06f)) - f);
}

/* x / c given rc = RN(1/c) (computed once with an IEEE division): q = x rc refined by one fused
 * residual step (Markstein), three dependent operations instead of the IEEE division sequence. Used for
 * the stepping-space division by log(1 + cone) (testbed_nerf.cu:114-184), on both sides. Equal to the
 * IEEE quotient for every x at the default cone 1/256 (tools/microbench/div_check.c, exhaustive over
 * the range below); outside 2^-100 <= |x| <= 2^100 it is the IEEE division. */
NGP_MATH_FN float ngp_div_rc(float x, float c, float rc) {
	const float ax = x < 0.0f ? -x : x;
	if (ax >= 7.88860905221011805e-31f && ax <= 1.26765060022822940e30f) {
		const float q = x * rc;
		return NGP_FMAF(NGP_FMAF(-q, c, x), rc, q);
	}
	return x / c;
}

#endif /* NGP_MATH_H */
