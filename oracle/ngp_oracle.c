/*
 * ngp_oracle.c — CPU restatement of the instant-ngp training hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker (or the timed CPU baseline). The product path
 * (instant-ngp_amd/csrc) never links or calls it.
 *
 * Parity status:
 *   - pcg32: PINNED by the published PCG known-answer vector (pcg32 seeded (42, 54)), tests/golden/.
 *   - sRGB, morton3D, NeRF stepping / warps / activations: restated from code present in the reference
 *     (file:line cited per function), exact float formulas.
 *   - hash-grid encoding, fully-fused MLP, SH encoding, Adam/EMA: the arithmetic lives in tiny-cuda-nn,
 *     which is ABSENT from /root/reference (pinned version unrecoverable, API era ~2023).
 *     These are restated from tcnn's published algorithm and are "parity unpinned" against the
 *     reference: no golden vector for them exists in the reference.
 *
 * Conventions shared with the C-ABI (include/ngp_engine.h):
 *   - half values are passed as uint16_t IEEE binary16 bit patterns;
 *   - positions: element (i, d) at pos[i * stride + d] (tcnn "CM"/AoS NerfCoordinate convention);
 *   - encoding / network activations: AoS, element (i, f) at x[i * width + f].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------------
 * IEEE binary16 <-> binary32 (round to nearest even), matches v_cvt_f16_f32 / v_cvt_f32_f16.
 * ---------------------------------------------------------------------------------------------- */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

EXPORT uint16_t orc_f32_to_f16(float f) {
	uint32_t x = f2u(f);
	uint32_t sign = (x >> 16) & 0x8000u;
	uint32_t ax = x & 0x7fffffffu;
	if (ax >= 0x7f800000u) { /* inf / nan */
		return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u | ((ax >> 13) & 0x3ffu) : 0));
	}
	if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520 -> inf */
	if (ax < 0x38800000u) { /* subnormal half (or zero) */
		if (ax < 0x33000000u) return (uint16_t)sign; /* < 2^-25 rounds to 0 (ties to even at 2^-25 -> 0) */
		uint32_t e = ax >> 23;
		uint32_t m = (ax & 0x7fffffu) | 0x800000u;
		uint32_t shift = 126 - e; /* value = m * 2^(e-150); in half-subnormal units (2^-24): m >> (126-e) */
		uint32_t r = m >> shift;
		uint32_t rem = m & ((1u << shift) - 1);
		uint32_t halfway = 1u << (shift - 1);
		if (rem > halfway || (rem == halfway && (r & 1))) r++;
		return (uint16_t)(sign | r);
	}
	uint32_t r = ax + 0xc8000000u; /* rebias exponent: (e-112) << 23 */
	uint32_t lsb = (r >> 13) & 1u;
	r += 0xfffu + lsb;
	return (uint16_t)(sign | (r >> 13));
}

EXPORT float orc_f16_to_f32(uint16_t h) {
	uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
	uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
	if (e == 0) {
		if (m == 0) return u2f(sign);
		float v = (float)m * (1.0f / 16777216.0f);
		return sign ? -v : v;
	}
	if (e == 31) return u2f(sign | 0x7f800000u | (m << 13));
	return u2f(sign | ((e + 112) << 23) | (m << 13));
}

static inline float hf(uint16_t h) { return orc_f16_to_f32(h); }
static inline uint16_t fh(float f) { return orc_f32_to_f16(f); }
static inline float rh(float f) { return hf(fh(f)); } /* round through half */

EXPORT void orc_f32_to_f16_array(const float* in, uint16_t* out, size_t n) {
	for (size_t i = 0; i < n; ++i) out[i] = fh(in[i]);
}
EXPORT void orc_f16_to_f32_array(const uint16_t* in, float* out, size_t n) {
	for (size_t i = 0; i < n; ++i) out[i] = hf(in[i]);
}

/* ------------------------------------------------------------------------------------------------
 * pcg32 — tcnn::pcg32 (= Wenzel Jakob's pcg32.h, PCG-XSH-RR 64/32), used by the reference as
 * default_rng_t (include/neural-graphics-primitives/random_val.cuh:26-43, 150-153; seeds
 * src/testbed.cu:3906,3919). Pinned by the PCG reference known-answer vector.
 * ---------------------------------------------------------------------------------------------- */
#define PCG32_DEFAULT_STATE 0x853c49e6748fea9bULL
#define PCG32_DEFAULT_STREAM 0xda3e39cb94b95bdbULL
#define PCG32_MULT 0x5851f42d4c957f2dULL

typedef struct { uint64_t state, inc; } orc_pcg32;

EXPORT uint32_t orc_pcg32_next_uint(orc_pcg32* r) {
	uint64_t old = r->state;
	r->state = old * PCG32_MULT + r->inc;
	uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
	uint32_t rot = (uint32_t)(old >> 59u);
	return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
}
EXPORT void orc_pcg32_seed(orc_pcg32* r, uint64_t initstate, uint64_t initseq) {
	r->state = 0u;
	r->inc = (initseq << 1u) | 1u;
	orc_pcg32_next_uint(r);
	r->state += initstate;
	orc_pcg32_next_uint(r);
}
EXPORT void orc_pcg32_default(orc_pcg32* r) { r->state = PCG32_DEFAULT_STATE; r->inc = PCG32_DEFAULT_STREAM; }
EXPORT float orc_pcg32_next_float(orc_pcg32* r) {
	return u2f((orc_pcg32_next_uint(r) >> 9) | 0x3f800000u) - 1.0f;
}
EXPORT void orc_pcg32_advance(orc_pcg32* r, int64_t delta_) {
	uint64_t cur_mult = PCG32_MULT, cur_plus = r->inc, acc_mult = 1u, acc_plus = 0u;
	uint64_t delta = (uint64_t)delta_;
	while (delta > 0) {
		if (delta & 1) { acc_mult *= cur_mult; acc_plus = acc_plus * cur_mult + cur_plus; }
		cur_plus = (cur_mult + 1) * cur_plus;
		cur_mult *= cur_mult;
		delta /= 2;
	}
	r->state = acc_mult * r->state + acc_plus;
}

/* tcnn generate_random_uniform (restated, unpinned): element idx = i*4 + j is drawn by the generator
 * advanced by i*4 then j further draws; the caller's rng advances by n afterwards.
 * Equivalent closed form: element k uses draw number k of the stream. */
EXPORT void orc_generate_random_uniform(orc_pcg32* rng, size_t n, float* out, float lo, float hi) {
	orc_pcg32 r = *rng;
	for (size_t k = 0; k < n; ++k) out[k] = orc_pcg32_next_float(&r) * (hi - lo) + lo;
	orc_pcg32_advance(rng, (int64_t)n);
}

/* ------------------------------------------------------------------------------------------------
 * Multiresolution hash-grid encoding (tcnn GridEncodingTemplated).
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
	uint32_t n_dims;          /* D: 2 or 3 */
	uint32_t n_levels;        /* L */
	uint32_t n_features;      /* F per level */
	uint32_t log2_hashmap;    /* log2 T */
	uint32_t base_resolution; /* N_min */
	float per_level_scale;    /* b (the fork forces 2.0: src/testbed.cu:3991) */
	uint32_t offsets[33];     /* entry offset per level, offsets[L] = total entries */
	float scale[32];          /* per-level scale = exp2f(l*log2 b)*N_min - 1 */
	uint32_t resolution[32];  /* ceilf(scale)+1 */
} orc_grid;

static uint32_t powu(uint32_t b, uint32_t e) { uint32_t r = 1; while (e--) r *= b; return r; }

/* Offset table: dense level size rounded up to a multiple of 8, clamped to T for hash grids. */
EXPORT uint32_t orc_grid_init(orc_grid* g, uint32_t D, uint32_t L, uint32_t F, uint32_t log2T, uint32_t Nmin, float b) {
	g->n_dims = D; g->n_levels = L; g->n_features = F; g->log2_hashmap = log2T;
	g->base_resolution = Nmin; g->per_level_scale = b;
	float log2b = log2f(b);
	uint32_t off = 0;
	for (uint32_t l = 0; l < L; ++l) {
		float s = exp2f((float)l * log2b) * (float)Nmin - 1.0f;
		uint32_t res = (uint32_t)ceilf(s) + 1u;
		g->scale[l] = s; g->resolution[l] = res;
		uint32_t max_params = 0xffffffffu / 2;
		uint32_t n = powf((float)res, (float)D) > (float)max_params ? max_params : powu(res, D);
		n = (n + 7u) / 8u * 8u;
		if (n > (1u << log2T)) n = 1u << log2T;
		g->offsets[l] = off;
		off += n;
	}
	g->offsets[L] = off;
	return off; /* total entries; params = off * F */
}

static inline uint32_t grid_index(const orc_grid* g, uint32_t l, const uint32_t* p) {
	static const uint32_t primes[3] = {1u, 2654435761u, 805459861u};
	uint32_t T = g->offsets[l + 1] - g->offsets[l];
	uint32_t res = g->resolution[l];
	uint32_t stride = 1, index = 0;
	for (uint32_t d = 0; d < g->n_dims && stride <= T; ++d) {
		index += p[d] * stride;
		stride *= res;
	}
	if (T < stride) {
		index = 0;
		for (uint32_t d = 0; d < g->n_dims; ++d) index ^= p[d] * primes[d];
	}
	return index % T;
}

/* Per-sample, per-level corner setup shared by forward and backward. */
static inline void grid_corner_setup(const orc_grid* g, uint32_t l, const float* x, float* frac, uint32_t* base) {
	for (uint32_t d = 0; d < g->n_dims; ++d) {
		float p = fmaf(g->scale[l], x[d], 0.5f);
		float t = floorf(p);
		base[d] = (uint32_t)(int)t;
		frac[d] = p - t;
	}
}

static inline float corner_weight(const orc_grid* g, uint32_t c, const float* frac, const uint32_t* base, uint32_t* p) {
	float w = 1.0f;
	for (uint32_t d = 0; d < g->n_dims; ++d) {
		if ((c & (1u << d)) == 0) { w *= 1.0f - frac[d]; p[d] = base[d]; }
		else { w *= frac[d]; p[d] = base[d] + 1u; }
	}
	return w;
}

/* Forward. out: AoS float [n x L*F] (the value before the final fp16 rounding; callers round).
 * Accumulation: fp32 in corner order c = 0..2^D-1 (our kernel's contract; tcnn accumulates in the
 * table precision). Levels >= max_level*L (+1e-3) are zeroed (set_max_level). */
EXPORT void orc_grid_forward(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride,
                             const uint16_t* table, float max_level, const float* max_level_per_sample, float* out) {
	const uint32_t L = g->n_levels, F = g->n_features;
	#pragma omp parallel for schedule(static)
	for (size_t i = 0; i < n; ++i) {
		const float* x = pos + i * pos_stride;
		float ml = (max_level_per_sample ? max_level_per_sample[i] : max_level) * (float)L;
		for (uint32_t l = 0; l < L; ++l) {
			float* o = out + i * (size_t)(L * F) + l * F;
			if ((float)l >= ml + 1e-3f) { for (uint32_t f = 0; f < F; ++f) o[f] = 0.f; continue; }
			float frac[4]; uint32_t base[4], p[4];
			grid_corner_setup(g, l, x, frac, base);
			float acc[8] = {0};
			for (uint32_t c = 0; c < (1u << g->n_dims); ++c) {
				float w = corner_weight(g, c, frac, base, p);
				size_t e = (size_t)g->offsets[l] + grid_index(g, l, p);
				for (uint32_t f = 0; f < F; ++f) acc[f] = fmaf(w, hf(table[e * F + f]), acc[f]);
			}
			for (uint32_t f = 0; f < F; ++f) o[f] = acc[f];
		}
	}
}

/* Backward: grad[e*F+f] += w * dL_dy[i, l*F+f] (double accumulation; the kernel accumulates in fp16
 * atomics like tcnn's half2 atomicAdd, so comparisons use a tolerance). dL_dy AoS float [n x L*F]. */
EXPORT void orc_grid_backward(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride,
                              const float* dL_dy, float max_level, const float* max_level_per_sample, double* grad) {
	const uint32_t L = g->n_levels, F = g->n_features;
	for (size_t i = 0; i < n; ++i) {
		const float* x = pos + i * pos_stride;
		float ml = (max_level_per_sample ? max_level_per_sample[i] : max_level) * (float)L;
		for (uint32_t l = 0; l < L; ++l) {
			if ((float)l > ml + 1e-3f) continue;
			const float* gy = dL_dy + i * (size_t)(L * F) + l * F;
			float frac[4]; uint32_t base[4], p[4];
			grid_corner_setup(g, l, x, frac, base);
			for (uint32_t c = 0; c < (1u << g->n_dims); ++c) {
				float w = corner_weight(g, c, frac, base, p);
				size_t e = (size_t)g->offsets[l] + grid_index(g, l, p);
				for (uint32_t f = 0; f < F; ++f) grad[e * F + f] += (double)w * (double)gy[f];
			}
		}
	}
}

/* Backward, contribution-exact: tcnn's kernel_grid_backward rounds every contribution w * dL/dy to the
 * table precision before its half2 atomicAdd (a2: "(__half)((float)g * w)"); this restatement keeps that
 * rounding, sums the fp16 contributions exactly (every fp16 value is an integer multiple of 2^-24, so
 * an int64 in those units is exact and the sum order-independent) and rounds once:
 *   grad16[e] = f16( f32( (double)sum * 2^-24 ) )          (overwrite)
 *   grad16[e] = f16( f32(sum * 2^-24) + f32(grad16[e]) )    (accumulate)
 * which is the engine's destination-bucketed backward contract (csrc/grid_scatter.hip), so the two are
 * compared with array_equal. dL_dy: fp16 bits, element (i, l*F+f) at dL_dy[i * dy_stride + l*F + f].
 * abs_sum (optional, double [entries*F]) receives sum |w * dL/dy| per parameter: the conditioning of
 * each sum, used by end-to-end tests whose dL/dy differ from the engine's by fp16 rounding. */
EXPORT void orc_grid_backward_exact(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride,
                                    const uint16_t* dL_dy, uint32_t dy_stride, float max_level,
                                    const float* max_level_per_sample, int accumulate, uint16_t* grad16, double* abs_sum) {
	const uint32_t L = g->n_levels, F = g->n_features;
	const size_t np = (size_t)g->offsets[L] * F;
	int64_t* acc = (int64_t*)calloc(np, sizeof(int64_t));
	if (abs_sum) memset(abs_sum, 0, np * sizeof(double));
	#pragma omp parallel for schedule(static)
	for (size_t i = 0; i < n; ++i) {
		const float* x = pos + i * pos_stride;
		float ml = (max_level_per_sample ? max_level_per_sample[i] : max_level) * (float)L;
		for (uint32_t l = 0; l < L; ++l) {
			if ((float)l > ml + 1e-3f) continue; /* tcnn backward: '>' (the forward zeroes at '>=') */
			float frac[4]; uint32_t base[4], p[4];
			grid_corner_setup(g, l, x, frac, base);
			for (uint32_t c = 0; c < (1u << g->n_dims); ++c) {
				float w = corner_weight(g, c, frac, base, p);
				size_t e = (size_t)g->offsets[l] + grid_index(g, l, p);
				for (uint32_t f = 0; f < F; ++f) {
					float gy = hf(dL_dy[i * dy_stride + l * F + f]);
					float contrib = hf(fh(w * gy));
					int64_t q = (int64_t)(contrib * 16777216.0f);
					if (q) {
						#pragma omp atomic
						acc[e * F + f] += q;
					}
					if (abs_sum) {
						double a = fabs((double)w * (double)gy);
						#pragma omp atomic
						abs_sum[e * F + f] += a;
					}
				}
			}
		}
	}
	#pragma omp parallel for schedule(static)
	for (size_t k = 0; k < np; ++k) {
		float s = (float)((double)acc[k] * (1.0 / 16777216.0));
		if (accumulate) s += hf(grad16[k]);
		grad16[k] = fh(s);
	}
	free(acc);
}

/* Entry index per (sample, level, corner): for bit-exact integer parity of the hashing. */
EXPORT void orc_grid_indices(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride, uint32_t* idx) {
	const uint32_t L = g->n_levels, C = 1u << g->n_dims;
	for (size_t i = 0; i < n; ++i) {
		for (uint32_t l = 0; l < L; ++l) {
			float frac[4]; uint32_t base[4], p[4];
			grid_corner_setup(g, l, pos + i * pos_stride, frac, base);
			for (uint32_t c = 0; c < C; ++c) {
				corner_weight(g, c, frac, base, p);
				idx[(i * L + l) * C + c] = g->offsets[l] + grid_index(g, l, p);
			}
		}
	}
}

/* ------------------------------------------------------------------------------------------------
 * Spherical harmonics, degree 4 (tcnn SphericalHarmonicsEncoding, restated).
 * Input in [0,1]^3 (warp_direction, src/testbed_nerf.cu:407-409) mapped to 2x-1.
 * ---------------------------------------------------------------------------------------------- */
EXPORT void orc_sh4(float dx, float dy, float dz, float* o) {
	float x = dx * 2.f - 1.f, y = dy * 2.f - 1.f, z = dz * 2.f - 1.f;
	float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
	o[0] = 0.28209479177387814f;
	o[1] = -0.48860251190291987f * y;
	o[2] = 0.48860251190291987f * z;
	o[3] = -0.48860251190291987f * x;
	o[4] = 1.0925484305920792f * xy;
	o[5] = -1.0925484305920792f * yz;
	o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
	o[7] = -1.0925484305920792f * xz;
	o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
	o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
	o[10] = 2.8906114426405538f * xy * z;
	o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
	o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
	o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
	o[14] = 1.4453057213202769f * z * (x2 - y2);
	o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

/* ------------------------------------------------------------------------------------------------
 * Input gradients (tcnn Encoding::backward's dL_dinput, as NerfNetwork::backward_impl slices them:
 * include/neural-graphics-primitives/nerf_network.h:282-299 direction, :317-333 position), restated
 * analytically in double:
 *   grid: dL/dx_d = sum_l scale_l * sum_c sign_d(c) * prod_{e != d} w_e(c) * sum_f dL/dy_{l,f} T[c, f]
 *         (w_e(c) = frac_e or 1 - frac_e; levels zeroed by set_max_level contribute nothing);
 *   SH:   dL/ddir_j = 2 * sum_k dL/dSH_k * dSH_k/dd_j, d = 2 dir - 1 (the degree-4 basis of orc_sh4).
 * ---------------------------------------------------------------------------------------------- */
EXPORT void orc_grid_input_grad(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride, const uint16_t* table,
                                const float* dL_dy, uint32_t dy_stride, float max_level, double* out) {
	const uint32_t L = g->n_levels, F = g->n_features, D = g->n_dims;
	#pragma omp parallel for schedule(static)
	for (size_t i = 0; i < n; ++i) {
		const float* x = pos + i * pos_stride;
		const float ml = max_level * (float)L;
		double acc[4] = {0, 0, 0, 0};
		for (uint32_t l = 0; l < L; ++l) {
			if ((float)l >= ml + 1e-3f) continue;
			float frac[4]; uint32_t base[4], p[4];
			grid_corner_setup(g, l, x, frac, base);
			for (uint32_t c = 0; c < (1u << D); ++c) {
				corner_weight(g, c, frac, base, p);
				size_t e = (size_t)g->offsets[l] + grid_index(g, l, p);
				double gs = 0.0;
				for (uint32_t f = 0; f < F; ++f) gs += (double)dL_dy[i * dy_stride + l * F + f] * (double)hf(table[e * F + f]);
				for (uint32_t d = 0; d < D; ++d) {
					double wo = 1.0;
					for (uint32_t k = 0; k < D; ++k)
						if (k != d) wo *= (c >> k) & 1u ? (double)frac[k] : 1.0 - (double)frac[k];
					acc[d] += (double)g->scale[l] * ((c >> d) & 1u ? wo : -wo) * gs;
				}
			}
		}
		for (uint32_t d = 0; d < D; ++d) out[i * D + d] = acc[d];
	}
}

/* gradient of each SH basis function wrt d = (x, y, z), basis order of orc_sh4 */
static void sh4_basis_grad(double x, double y, double z, double gr[16][3]) {
	const double A = 0.48860251190291987, B = 1.0925484305920792, C = 0.94617469575755997, E = 0.54627421529603959,
	             G = 0.59004358992664352, H = 2.8906114426405538, I = 0.45704579946446572, J = 0.3731763325901154,
	             K = 1.4453057213202769;
	memset(gr, 0, sizeof(double) * 48);
	gr[1][1] = -A;
	gr[2][2] = A;
	gr[3][0] = -A;
	gr[4][0] = B * y; gr[4][1] = B * x;
	gr[5][1] = -B * z; gr[5][2] = -B * y;
	gr[6][2] = 2 * C * z;
	gr[7][0] = -B * z; gr[7][2] = -B * x;
	gr[8][0] = 2 * E * x; gr[8][1] = -2 * E * y;
	gr[9][0] = G * y * (-6 * x); gr[9][1] = G * (-3 * x * x + 3 * y * y);
	gr[10][0] = H * y * z; gr[10][1] = H * x * z; gr[10][2] = H * x * y;
	gr[11][1] = I * (1 - 5 * z * z); gr[11][2] = I * y * (-10 * z);
	gr[12][2] = J * (15 * z * z - 3);
	gr[13][0] = I * (1 - 5 * z * z); gr[13][2] = I * x * (-10 * z);
	gr[14][0] = K * z * 2 * x; gr[14][1] = -K * z * 2 * y; gr[14][2] = K * (x * x - y * y);
	gr[15][0] = G * (-3 * x * x + 3 * y * y); gr[15][1] = G * x * 6 * y;
}

EXPORT void orc_sh4_input_grad(const float* dir, const float* dL_dsh, double* out) {
	double gr[16][3];
	sh4_basis_grad(2.0 * dir[0] - 1.0, 2.0 * dir[1] - 1.0, 2.0 * dir[2] - 1.0, gr);
	for (int j = 0; j < 3; ++j) {
		double s = 0.0;
		for (int k = 0; k < 16; ++k) s += (double)dL_dsh[k] * gr[k][j];
		out[j] = 2.0 * s;
	}
}

/* ------------------------------------------------------------------------------------------------
 * Fully-fused MLP (tcnn FullyFusedMLP<half, W>, restated).
 * Layers: in_pad -> W (ReLU) -> [W -> W (ReLU)] x (n_hidden-1) -> out_pad (no activation).
 * Weights fp16 row-major [out x in] per layer, consecutive. Every layer: fp16 operands, fp32 sum,
 * result rounded to fp16 (our MFMA kernel's contract; tcnn's WMMA accumulates in fp16).
 * ---------------------------------------------------------------------------------------------- */
typedef struct { uint32_t in_pad, width, n_hidden, out_pad; } orc_mlp;

EXPORT uint32_t orc_mlp_n_params(const orc_mlp* m) {
	return m->width * m->in_pad + (m->n_hidden - 1) * m->width * m->width + m->out_pad * m->width;
}

static void layer_dims(const orc_mlp* m, uint32_t l, uint32_t* in, uint32_t* out, size_t* woff) {
	uint32_t nl = m->n_hidden + 1;
	size_t off = 0;
	for (uint32_t k = 0; k < l; ++k) {
		uint32_t ki = k == 0 ? m->in_pad : m->width, ko = k == nl - 1 ? m->out_pad : m->width;
		off += (size_t)ki * ko;
	}
	*in = l == 0 ? m->in_pad : m->width;
	*out = l == nl - 1 ? m->out_pad : m->width;
	*woff = off;
}

/* One sample's forward; acts receives every layer's fp16-rounded output (post-activation for hidden
 * layers), acts must hold (n_hidden)*width + out_pad floats. */
/* margin (optional): min over the hidden neurons of |pre-activation| / sum_k |W_ok a_k| — how close a
 * ReLU is to switching under accumulation-order noise (tests use it to explain outliers). */
static void mlp_forward_one_abs(const orc_mlp* m, const uint16_t* w, const float* x, float* acts, float* out_abs,
                                float* margin) {
	uint32_t nl = m->n_hidden + 1;
	float buf_in[256];
	memcpy(buf_in, x, m->in_pad * sizeof(float));
	float* dst = acts;
	for (uint32_t l = 0; l < nl; ++l) {
		uint32_t in, out; size_t off; layer_dims(m, l, &in, &out, &off);
		for (uint32_t o = 0; o < out; ++o) {
			double s = 0.0, sa = 0.0;
			const uint16_t* wr = w + off + (size_t)o * in;
			for (uint32_t k = 0; k < in; ++k) s += (double)hf(wr[k]) * (double)buf_in[k];
			if ((out_abs && l == nl - 1) || (margin && l < nl - 1))
				for (uint32_t k = 0; k < in; ++k) sa += fabs((double)hf(wr[k]) * (double)buf_in[k]);
			if (out_abs && l == nl - 1) out_abs[o] = (float)sa;
			if (margin && l < nl - 1 && sa > 0.0) {
				float r = (float)(fabs(s) / sa);
				if (r < *margin) *margin = r;
			}
			float v = rh((float)s);
			if (l < nl - 1 && v < 0.f) v = 0.f;
			dst[o] = v;
		}
		memcpy(buf_in, dst, out * sizeof(float));
		dst += out;
	}
}

static void mlp_forward_one(const orc_mlp* m, const uint16_t* w, const float* x, float* acts) {
	mlp_forward_one_abs(m, w, x, acts, NULL, NULL);
}

EXPORT void orc_set_num_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }

EXPORT void orc_mlp_forward(const orc_mlp* m, const uint16_t* w, size_t n, const float* x, float* y) {
	uint32_t nact = m->n_hidden * m->width + m->out_pad;
	#pragma omp parallel
	{
		float* acts = (float*)malloc(nact * sizeof(float));
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			mlp_forward_one(m, w, x + i * m->in_pad, acts);
			memcpy(y + i * m->out_pad, acts + m->n_hidden * m->width, m->out_pad * sizeof(float));
		}
		free(acts);
	}
}

/* Backward of one sample given dL/dy (float, representable in fp16). Accumulates dW (double) and
 * writes dL/dx (fp16-rounded) if dx != NULL. Hidden-layer gradients are rounded to fp16 after the
 * ReLU mask, as the kernel feeds them to the next MFMA in fp16. */
static void mlp_backward_one_abs(const orc_mlp* m, const uint16_t* w, const float* x, const float* acts,
                                 const float* dy, double* dW, double* dWabs, float* dx, float* dxabs) {
	uint32_t nl = m->n_hidden + 1;
	float g[256], gn[256];
	memcpy(g, dy, m->out_pad * sizeof(float));
	for (int l = (int)nl - 1; l >= 0; --l) {
		uint32_t in, out; size_t off; layer_dims(m, (uint32_t)l, &in, &out, &off);
		const float* a_in = l == 0 ? x : acts + (size_t)(l - 1) * m->width;
		/* dW[o][k] += g[o] * a_in[k] */
		for (uint32_t o = 0; o < out; ++o)
			for (uint32_t k = 0; k < in; ++k) dW[off + (size_t)o * in + k] += (double)g[o] * (double)a_in[k];
		if (dWabs)
			for (uint32_t o = 0; o < out; ++o)
				for (uint32_t k = 0; k < in; ++k) dWabs[off + (size_t)o * in + k] += fabs((double)g[o] * (double)a_in[k]);
		if (l == 0 && !dx) break;
		for (uint32_t k = 0; k < in; ++k) {
			double s = 0.0;
			for (uint32_t o = 0; o < out; ++o) s += (double)hf(w[off + (size_t)o * in + k]) * (double)g[o];
			float v = rh((float)s);
			if (l > 0 && a_in[k] <= 0.f) v = 0.f; /* ReLU' from the forward activation */
			gn[k] = v;
			if (l == 0 && dxabs) {
				double sa = 0.0;
				for (uint32_t o = 0; o < out; ++o) sa += fabs((double)hf(w[off + (size_t)o * in + k]) * (double)g[o]);
				dxabs[k] = (float)sa;
			}
		}
		if (l == 0) { memcpy(dx, gn, in * sizeof(float)); break; }
		memcpy(g, gn, in * sizeof(float));
	}
}

static void mlp_backward_one(const orc_mlp* m, const uint16_t* w, const float* x, const float* acts,
                             const float* dy, double* dW, float* dx) {
	mlp_backward_one_abs(m, w, x, acts, dy, dW, NULL, dx, NULL);
}

EXPORT void orc_mlp_backward(const orc_mlp* m, const uint16_t* w, size_t n, const float* x, const float* dy,
                             double* dW, float* dx) {
	uint32_t nact = m->n_hidden * m->width + m->out_pad;
	float* acts = (float*)malloc(nact * sizeof(float));
	for (size_t i = 0; i < n; ++i) {
		mlp_forward_one(m, w, x + i * m->in_pad, acts);
		mlp_backward_one(m, w, x + i * m->in_pad, acts, dy + i * m->out_pad, dW, dx ? dx + i * m->in_pad : NULL);
	}
	free(acts);
}

/* ------------------------------------------------------------------------------------------------
 * NerfNetwork composition (include/neural-graphics-primitives/nerf_network.h:116-335).
 * input: AoS float [n x in_stride] NerfCoordinate {pos(3), dt, dir(3)} (nerf.h:85-128),
 * dir at dir_offset (4). Output AoS fp16 [n x 16]: rows 0..2 rgb raw, row 3 density raw
 * (extract_density, nerf_network.h:32-43); rows 4..15 = rgb network padding outputs.
 * Param layout [density MLP | rgb MLP | grid | dir enc (0)] (nerf_network.h:430-443).
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
	orc_grid grid;
	orc_mlp density;   /* in_pad = L*F padded to 16, out 16 */
	orc_mlp rgb;       /* in 32 = 16 density out + 16 SH, out_pad 16 */
	uint32_t dir_offset;
	uint32_t in_stride;
} orc_nerf;

EXPORT uint32_t orc_nerf_n_params(const orc_nerf* m) {
	return orc_mlp_n_params(&m->density) + orc_mlp_n_params(&m->rgb) + m->grid.offsets[m->grid.n_levels] * m->grid.n_features;
}

static void nerf_forward_one(const orc_nerf* m, const uint16_t* params, const float* in,
                             float* enc, float* dacts, float* racts, float* rin, float* out16) {
	const orc_grid* g = &m->grid;
	uint32_t LF = g->n_levels * g->n_features;
	const uint16_t* wd = params;
	const uint16_t* wr = params + orc_mlp_n_params(&m->density);
	const uint16_t* table = wr + orc_mlp_n_params(&m->rgb);
	orc_grid_forward(g, 1, in, m->in_stride, table, 1.0f, NULL, enc);
	for (uint32_t k = 0; k < m->density.in_pad; ++k) enc[k] = k < LF ? rh(enc[k]) : 0.f;
	mlp_forward_one(&m->density, wd, enc, dacts);
	const float* dout = dacts + m->density.n_hidden * m->density.width; /* 16 */
	for (uint32_t k = 0; k < 16; ++k) rin[k] = dout[k];
	float sh[16];
	orc_sh4(in[m->dir_offset], in[m->dir_offset + 1], in[m->dir_offset + 2], sh);
	for (uint32_t k = 0; k < 16; ++k) rin[16 + k] = rh(sh[k]);
	mlp_forward_one(&m->rgb, wr, rin, racts);
	const float* rout = racts + m->rgb.n_hidden * m->rgb.width;
	for (uint32_t k = 0; k < 16; ++k) out16[k] = rout[k];
	out16[3] = dout[0];
}

EXPORT void orc_nerf_forward(const orc_nerf* m, const uint16_t* params, size_t n, const float* in, float* out) {
	#pragma omp parallel
	{
		float enc[256], dacts[1024], racts[1024], rin[32];
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i)
			nerf_forward_one(m, params, in + i * m->in_stride, enc, dacts, racts, rin, out + i * 16);
	}
}

/* Density-only inference (NerfNetwork::density, nerf_network.h:337-353): density MLP outputs [n x 16]. */
EXPORT void orc_nerf_density(const orc_nerf* m, const uint16_t* params, size_t n, const float* in, uint32_t in_stride, float* out) {
	const orc_grid* g = &m->grid;
	uint32_t LF = g->n_levels * g->n_features;
	const uint16_t* table = params + orc_mlp_n_params(&m->density) + orc_mlp_n_params(&m->rgb);
	#pragma omp parallel
	{
		float enc[256], dacts[1024];
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			orc_grid_forward(g, 1, in + i * in_stride, in_stride, table, 1.0f, NULL, enc);
			for (uint32_t k = 0; k < m->density.in_pad; ++k) enc[k] = k < LF ? rh(enc[k]) : 0.f;
			mlp_forward_one(&m->density, params, enc, dacts);
			memcpy(out + i * 16, dacts + m->density.n_hidden * m->density.width, 16 * sizeof(float));
		}
	}
}

/* Backward (nerf_network.h:256-335): dL_dout AoS float [n x 16] (rows 0..2 rgb, row 3 density).
 * grads: double [n_params] accumulated (Overwrite semantics: caller zeroes). Optionally dumps the
 * fp16-rounded dL/d(encoding) [n x density.in_pad] for layer-by-layer debugging. */
EXPORT void orc_nerf_backward(const orc_nerf* m, const uint16_t* params, size_t n, const float* in,
                              const float* dL_dout, double* grads, float* dL_denc) {
	const orc_grid* g = &m->grid;
	uint32_t LF = g->n_levels * g->n_features;
	size_t nd = orc_mlp_n_params(&m->density), nr = orc_mlp_n_params(&m->rgb);
	const uint16_t* wd = params;
	const uint16_t* wr = params + nd;
	float enc[256], dacts[1024], racts[1024], rin[32], out16[16];
	float drgb[16], drin[32], denc[256];
	for (size_t i = 0; i < n; ++i) {
		const float* x = in + i * m->in_stride;
		nerf_forward_one(m, params, x, enc, dacts, racts, rin, out16);
		for (uint32_t k = 0; k < 16; ++k) drgb[k] = k < 3 ? dL_dout[i * 16 + k] : 0.f;
		mlp_backward_one(&m->rgb, wr, rin, racts, drgb, grads + nd, drin);
		/* add_density_gradient (nerf_network.h:63-74): fp16 add into row 0 */
		float dd[16];
		for (uint32_t k = 0; k < 16; ++k) dd[k] = drin[k];
		dd[0] = rh(dd[0] + dL_dout[i * 16 + 3]);
		mlp_backward_one(&m->density, wd, enc, dacts, dd, grads, denc);
		if (dL_denc) memcpy(dL_denc + i * m->density.in_pad, denc, m->density.in_pad * sizeof(float));
		/* grid backward */
		float gy[256];
		for (uint32_t k = 0; k < LF; ++k) gy[k] = denc[k];
		orc_grid_backward(g, 1, x, m->in_stride, gy, 1.0f, NULL, grads + nd + nr);
	}
}

/* NerfNetwork backward with input gradients (nerf_network.h:256-335 with dL_dinput): per sample the
 * fp16-rounded dL/d(SH) (rows 16..31 of the rgb network's dL/dinput) and dL/d(encoding) as the engine
 * rounds them, then the analytic position and direction gradients (orc_grid_input_grad,
 * orc_sh4_input_grad) of those. dinput: float [n x in_stride], rows 0..2 and dir_offset..+2 written,
 * scaled by `scale`. dsh / denc (optional): [n x 16] / [n x density.in_pad]. */
EXPORT void orc_nerf_input_grad(const orc_nerf* m, const uint16_t* params, size_t n, const float* in, const float* dL_dout,
                                float scale, float* dinput, float* dsh_out, float* denc_out) {
	const orc_grid* g = &m->grid;
	size_t nd = orc_mlp_n_params(&m->density), nr = orc_mlp_n_params(&m->rgb);
	const uint16_t* wd = params;
	const uint16_t* wr = params + nd;
	const uint16_t* table = wr + nr;
	#pragma omp parallel
	{
		float enc[256], dacts[1024], racts[1024], rin[32], out16[16], drgb[16], drin[32], denc[256], dd[16];
		double* dW = (double*)calloc(nd + nr, sizeof(double));
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			const float* x = in + i * m->in_stride;
			nerf_forward_one(m, params, x, enc, dacts, racts, rin, out16);
			for (uint32_t k = 0; k < 16; ++k) drgb[k] = k < 3 ? dL_dout[i * 16 + k] : 0.f;
			mlp_backward_one(&m->rgb, wr, rin, racts, drgb, dW + nd, drin);
			for (uint32_t k = 0; k < 16; ++k) dd[k] = drin[k];
			dd[0] = rh(dd[0] + dL_dout[i * 16 + 3]);
			mlp_backward_one(&m->density, wd, enc, dacts, dd, dW, denc);
			double gp[4], gd[3];
			orc_grid_input_grad(g, 1, x, m->in_stride, table, denc, m->density.in_pad, 1.0f, gp);
			orc_sh4_input_grad(x + m->dir_offset, drin + 16, gd);
			float* o = dinput + i * m->in_stride;
			for (int d = 0; d < 3; ++d) o[d] = (float)(gp[d] * scale);
			for (int d = 0; d < 3; ++d) o[m->dir_offset + d] = (float)(gd[d] * scale);
			if (dsh_out) memcpy(dsh_out + i * 16, drin + 16, 16 * sizeof(float));
			if (denc_out) memcpy(denc_out + i * m->density.in_pad, denc, m->density.in_pad * sizeof(float));
		}
		free(dW);
	}
}

/* NerfNetwork::density_backward (nerf_network.h:384-428): dL_ddens float [n x 16] = dL/d(density network
 * output). grads (double [n_params], accumulated; caller zeroes): density MLP and grid sections only.
 * dinput (optional, float [n x in_stride]): rows 0..2. */
EXPORT void orc_nerf_density_backward(const orc_nerf* m, const uint16_t* params, size_t n, const float* in,
                                      const float* dL_ddens, double* grads, float* dinput) {
	const orc_grid* g = &m->grid;
	uint32_t LF = g->n_levels * g->n_features;
	size_t nd = orc_mlp_n_params(&m->density), nr = orc_mlp_n_params(&m->rgb);
	const uint16_t* table = params + nd + nr;
	float enc[256], dacts[1024], denc[256], gy[256];
	for (size_t i = 0; i < n; ++i) {
		const float* x = in + i * m->in_stride;
		orc_grid_forward(g, 1, x, m->in_stride, table, 1.0f, NULL, enc);
		for (uint32_t k = 0; k < m->density.in_pad; ++k) enc[k] = k < LF ? rh(enc[k]) : 0.f;
		mlp_forward_one(&m->density, params, enc, dacts);
		mlp_backward_one(&m->density, params, enc, dacts, dL_ddens + i * 16, grads, denc);
		for (uint32_t k = 0; k < LF; ++k) gy[k] = denc[k];
		orc_grid_backward(g, 1, x, m->in_stride, gy, 1.0f, NULL, grads + nd + nr);
		if (dinput) {
			double gp[4];
			orc_grid_input_grad(g, 1, x, m->in_stride, table, denc, m->density.in_pad, 1.0f, gp);
			for (int d = 0; d < 3; ++d) dinput[i * m->in_stride + d] = (float)gp[d];
		}
	}
}

/* Full-batch training pass (forward_impl + backward_impl, nerf_network.h:179-335), parallel over samples:
 *   out      float [n x 16]  network output (fp16-rounded values), out_abs (optional) the sum |w a| of
 *                            the contraction that produced each output (its conditioning);
 *   grads    double [nd+nr]  MLP weight gradients, abs (optional) sum |g a| per weight;
 *   denc16   fp16 bits [n x density.in_pad]  dL/d(encoding), the input of the grid backward
 *            (orc_grid_backward_exact finishes the gradient with the engine's exact-sum contract),
 *            denc_abs (optional) the sum |W g| of each dL/d(encoding) contraction;
 *   margin   (optional) float [n]: min over the sample's hidden neurons of |pre-activation| / sum |W a|.
 * Per-thread accumulators are added in thread order after the loop (double: order effects ~1e-16). */
EXPORT void orc_nerf_train_ex(const orc_nerf* m, const uint16_t* params, size_t n, const float* in, const float* dL_dout,
                              float* out, float* out_abs, double* grads, double* grads_abs, uint16_t* denc16,
                              float* denc_abs, float* margin) {
	size_t nd = orc_mlp_n_params(&m->density), nr = orc_mlp_n_params(&m->rgb);
	const uint16_t* wd = params;
	const uint16_t* wr = params + nd;
	const orc_grid* g = &m->grid;
	uint32_t LF = g->n_levels * g->n_features;
	const uint16_t* table = wr + nr;
	memset(grads, 0, (nd + nr) * sizeof(double));
	if (grads_abs) memset(grads_abs, 0, (nd + nr) * sizeof(double));
	#pragma omp parallel
	{
		double* lg = (double*)calloc(nd + nr, sizeof(double));
		double* la = grads_abs ? (double*)calloc(nd + nr, sizeof(double)) : NULL;
		float enc[256], dacts[1024], racts[1024], rin[32], drgb[16], drin[32], denc[256], dd[16], oa_r[16], oa_d[16];
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			const float* x = in + i * m->in_stride;
			orc_grid_forward(g, 1, x, m->in_stride, table, 1.0f, NULL, enc);
			for (uint32_t k = 0; k < m->density.in_pad; ++k) enc[k] = k < LF ? rh(enc[k]) : 0.f;
			float mg = 1.0f;
			mlp_forward_one_abs(&m->density, wd, enc, dacts, oa_d, &mg);
			const float* dout = dacts + m->density.n_hidden * m->density.width;
			for (uint32_t k = 0; k < 16; ++k) rin[k] = dout[k];
			float sh[16];
			orc_sh4(x[m->dir_offset], x[m->dir_offset + 1], x[m->dir_offset + 2], sh);
			for (uint32_t k = 0; k < 16; ++k) rin[16 + k] = rh(sh[k]);
			mlp_forward_one_abs(&m->rgb, wr, rin, racts, oa_r, &mg);
			if (margin) margin[i] = mg;
			const float* rout = racts + m->rgb.n_hidden * m->rgb.width;
			for (uint32_t k = 0; k < 16; ++k) {
				out[i * 16 + k] = k == 3 ? dout[0] : rout[k];
				if (out_abs) out_abs[i * 16 + k] = k == 3 ? oa_d[0] : oa_r[k];
			}
			for (uint32_t k = 0; k < 16; ++k) drgb[k] = k < 3 ? dL_dout[i * 16 + k] : 0.f;
			mlp_backward_one_abs(&m->rgb, wr, rin, racts, drgb, lg + nd, la ? la + nd : NULL, drin, NULL);
			for (uint32_t k = 0; k < 16; ++k) dd[k] = drin[k];
			dd[0] = rh(dd[0] + dL_dout[i * 16 + 3]); /* add_density_gradient, nerf_network.h:63-74 */
			mlp_backward_one_abs(&m->density, wd, enc, dacts, dd, lg, la, denc,
			                     denc_abs ? denc_abs + i * m->density.in_pad : NULL);
			for (uint32_t k = 0; k < m->density.in_pad; ++k) denc16[i * m->density.in_pad + k] = fh(denc[k]);
		}
		#pragma omp for ordered schedule(static, 1)
		for (int t = 0; t < omp_get_num_threads(); ++t) {
			#pragma omp ordered
			{
				for (size_t k = 0; k < nd + nr; ++k) grads[k] += lg[k];
				if (la) for (size_t k = 0; k < nd + nr; ++k) grads_abs[k] += la[k];
			}
		}
		free(lg);
		free(la);
	}
}

/* The same full-batch pass for tcnn::NetworkWithInputEncoding (grid -> FullyFusedMLP; the image and
 * SDF primitives, src/testbed.cu:4101-4110): param layout [MLP | grid], pos element (i, d) at
 * pos[i * pos_stride + d], dL_dout float [n x mlp.out_pad]. Outputs as orc_nerf_train_ex. */
EXPORT void orc_net_train_ex(const orc_grid* g, const orc_mlp* mlp, const uint16_t* params, size_t n, const float* pos,
                             uint32_t pos_stride, const float* dL_dout, float* out, float* out_abs, double* grads,
                             double* grads_abs, uint16_t* denc16, float* denc_abs, float* margin) {
	const size_t nm = orc_mlp_n_params(mlp);
	const uint16_t* table = params + nm;
	const uint32_t LF = g->n_levels * g->n_features, OP = mlp->out_pad, IP = mlp->in_pad;
	const uint32_t nact = mlp->n_hidden * mlp->width + OP;
	memset(grads, 0, nm * sizeof(double));
	if (grads_abs) memset(grads_abs, 0, nm * sizeof(double));
	#pragma omp parallel
	{
		double* lg = (double*)calloc(nm, sizeof(double));
		double* la = grads_abs ? (double*)calloc(nm, sizeof(double)) : NULL;
		float* acts = (float*)malloc(nact * sizeof(float));
		float enc[512], denc[512], oa[256];
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			orc_grid_forward(g, 1, pos + i * pos_stride, pos_stride, table, 1.0f, NULL, enc);
			for (uint32_t k = 0; k < IP; ++k) enc[k] = k < LF ? rh(enc[k]) : 0.f;
			float mg = 1.0f;
			mlp_forward_one_abs(mlp, params, enc, acts, oa, &mg);
			if (margin) margin[i] = mg;
			const float* o = acts + mlp->n_hidden * mlp->width;
			for (uint32_t k = 0; k < OP; ++k) {
				out[i * OP + k] = o[k];
				if (out_abs) out_abs[i * OP + k] = oa[k];
			}
			mlp_backward_one_abs(mlp, params, enc, acts, dL_dout + i * OP, lg, la, denc, denc_abs ? denc_abs + i * IP : NULL);
			for (uint32_t k = 0; k < IP; ++k) denc16[i * IP + k] = fh(denc[k]);
		}
		#pragma omp for ordered schedule(static, 1)
		for (int t = 0; t < omp_get_num_threads(); ++t) {
			#pragma omp ordered
			{
				for (size_t k = 0; k < nm; ++k) grads[k] += lg[k];
				if (la) for (size_t k = 0; k < nm; ++k) grads_abs[k] += la[k];
			}
		}
		free(lg);
		free(la);
		free(acts);
	}
}

/* ------------------------------------------------------------------------------------------------
 * Parameter initialisation (tcnn restated, unpinned): MLP matrices Xavier-uniform
 * U(+-sqrt(6/(fan_in+fan_out))), grid U(+-1e-4); draws from one pcg32 stream in param order
 * [density MLP | rgb MLP | grid] (nerf_network.h:445-457; seed 1337: src/testbed.cu:3906,4129).
 * ---------------------------------------------------------------------------------------------- */
EXPORT void orc_mlp_init(const orc_mlp* m, orc_pcg32* rng, float* p) {
	uint32_t nl = m->n_hidden + 1;
	for (uint32_t l = 0; l < nl; ++l) {
		uint32_t in, out; size_t off; layer_dims(m, l, &in, &out, &off);
		float s = sqrtf(6.0f / (float)(in + out));
		orc_generate_random_uniform(rng, (size_t)in * out, p + off, -s, s);
	}
}

EXPORT void orc_nerf_init(const orc_nerf* m, uint64_t seed, float* p) {
	orc_pcg32 rng; orc_pcg32_seed(&rng, seed, 1u);
	orc_mlp_init(&m->density, &rng, p);
	p += orc_mlp_n_params(&m->density);
	orc_mlp_init(&m->rgb, &rng, p);
	p += orc_mlp_n_params(&m->rgb);
	size_t ng = (size_t)m->grid.offsets[m->grid.n_levels] * m->grid.n_features;
	orc_generate_random_uniform(&rng, ng, p, -1e-4f, 1e-4f);
}

/* ------------------------------------------------------------------------------------------------
 * Optimizer: Ema(decay) o ExponentialDecay o Adam (tcnn, restated; configs/nerf/base.json:5-22).
 * grads fp16 (scaled by loss_scale). Adam skips non-matrix params whose gradient is exactly 0
 * (per-param step counter); l2 only on the first n_matrix params.
 * ---------------------------------------------------------------------------------------------- */
typedef struct {
	float lr, beta1, beta2, eps, l2;
	float ema_decay;      /* 0 => no EMA */
	uint32_t decay_start, decay_interval; float decay_base;
} orc_adam_cfg;

EXPORT float orc_lr_at_step(const orc_adam_cfg* c, uint32_t step) {
	/* learning rate used by optimizer step number `step` (0-based) */
	float lr = c->lr;
	if (c->decay_interval == 0) return lr;
	if (step < c->decay_start) return lr;
	uint32_t k = (step - c->decay_start) / c->decay_interval + 1;
	for (uint32_t i = 0; i < k; ++i) lr *= c->decay_base;
	return lr;
}

/* tcnn Ema: after the nested optimizer's step `step` (0-based), every parameter's EMA takes the new weight,
 * skipped parameters included: e = d e + (1 - d) w, and the inference parameter is e debiased by 1 - d^(step+1).
 * The lazy-EMA layout of the engine must equal this per-step recurrence (tests/test_gpu_ema_gaps.py). */
static inline void ema_one(float d, float debias, float w, float* e32, uint16_t* e16) {
	float v = *e32 = d * *e32 + (1.f - d) * w;
	*e16 = fh(v / debias);
}
EXPORT void orc_ema_step(float d, uint32_t step, size_t n, const float* w32, float* ema32, uint16_t* ema16) {
	float debias = 1.f - powf(d, (float)(step + 1));
	for (size_t i = 0; i < n; ++i) ema_one(d, debias, w32[i], ema32 + i, ema16 + i);
}

EXPORT void orc_adam_step(const orc_adam_cfg* c, uint32_t step, size_t n, size_t n_matrix, float loss_scale,
                          float* w32, uint16_t* w16, const uint16_t* g16, float* m1, float* m2, uint32_t* steps,
                          float* ema32, uint16_t* ema16) {
	float lr0 = orc_lr_at_step(c, step);
	for (size_t i = 0; i < n; ++i) {
		float gr = hf(g16[i]) / loss_scale;
		if (i >= n_matrix && gr == 0.f) goto ema;
		{
			float w = w32[i];
			if (i < n_matrix) gr += c->l2 * w;
			float mm = m1[i] = c->beta1 * m1[i] + (1.f - c->beta1) * gr;
			float vv = m2[i] = c->beta2 * m2[i] + (1.f - c->beta2) * (gr * gr);
			uint32_t s = ++steps[i];
			float lr = lr0 * sqrtf(1.f - powf(c->beta2, (float)s)) / (1.f - powf(c->beta1, (float)s));
			float elr = lr / (sqrtf(vv) + c->eps);
			float nw = w - elr * mm;
			w32[i] = nw;
			w16[i] = fh(nw);
		}
	ema:
		if (c->ema_decay > 0.f && ema32) ema_one(c->ema_decay, 1.f - powf(c->ema_decay, (float)(step + 1)), w32[i], ema32 + i, ema16 + i);
	}
}

/* ------------------------------------------------------------------------------------------------
 * NeRF helpers restated from the reference (src/testbed_nerf.cu, common_device.cuh).
 * ---------------------------------------------------------------------------------------------- */
/* morton3D lives in ngp_nerf_oracle.c with the occupancy-grid restatement. */

/* common_device.cuh:75-121 */
EXPORT float orc_srgb_to_linear(float srgb) {
	if (srgb <= 0.04045f) return srgb / 12.92f;
	return powf((srgb + 0.055f) / 1.055f, 2.4f);
}
EXPORT float orc_linear_to_srgb(float linear) {
	if (linear < 0.0031308f) return 12.92f * linear;
	return 1.055f * powf(linear, 0.41666f) - 0.055f;
}

EXPORT int orc_num_threads(void) {
#ifdef _OPENMP
	return omp_get_max_threads();
#else
	return 1;
#endif
}
