/*
 * ngp_tcnn_mode.c — the oracle's "tcnn mode": the reference's own fp16 arithmetic for the hash grid and the
 * fully fused MLP, beside the engine's contract (ngp_oracle.c), so a test can bound how far the engine sits from
 * what tiny-cuda-nn would compute on the same inputs.
 *
 * TEST INFRASTRUCTURE ONLY (see ngp_oracle.c). tiny-cuda-nn is ABSENT from /root/reference (pinned
 * version unrecoverable, API era ~2023): what follows restates its published algorithm, so it is "parity
 * unpinned" like the rest of the tcnn restatements. The call sites it stands behind are in the reference:
 * NerfNetwork::inference_mixed_precision / forward / backward (include/neural-graphics-primitives/
 * nerf_network.h:143-153, 201-216, 236-241, 324-333), and the in-tree analogue of the grid's fp16 atomics is
 * include/neural-graphics-primitives/takikawa_encoding.cuh:184-264.
 *
 * The engine's contract differs on purpose: fp32 blends and MLP accumulation rounded once to fp16,
 * and an exact, order-independent grid gradient sum. tcnn's arithmetic, restated:
 *   - grid forward (GridEncodingTemplated kernel_grid): per level, result = 0 (fp16 vector); for corner
 *     idx = 0 .. 2^D - 1 (bit d set: the upper corner of dimension d, weight pos_d, else 1 - pos_d),
 *     weight = the float product over the dimensions, result = fma((half)weight, value, result) as fp16 FMAs:
 *     one rounding of the weight to fp16, one rounding per FMA;
 *   - FullyFusedMLP<half, 64> layers (WMMA m16n16k16 with __half accumulator fragments): the output of a
 *     neuron accumulates 16-wide k-steps of products into an fp16 accumulator; modelled here as the k-step's 16
 *     products summed exactly and added to the accumulator with one fp16 rounding per k-step; ReLU on the fp16
 *     value; the backward's dX chain (transposed weights, same fragments) likewise, masked by ReLU' of the
 *     forward activation; the input gradient's final matmul (dL/dencoding) in the same form;
 *   - grid backward (kernel_grid_backward): every contribution (half)((float)dL_dy * weight) added to the
 *     fp16 gradient by a half2 atomicAdd: one fp16 rounding per add, in arrival order. The oracle adds in
 *     sample order (sample, level, corner): one of the orders the GPU may take.
 * Every function also returns the rounding-error bound of its own arithmetic where the test needs one.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* shared with ngp_oracle.c (same library) */
uint16_t orc_f32_to_f16(float f);
float orc_f16_to_f32(uint16_t h);
typedef struct {
	uint32_t n_dims, n_levels, n_features, log2_hashmap, base_resolution;
	float per_level_scale;
	uint32_t offsets[33];
	float scale[32];
	uint32_t resolution[32];
} orc_grid;
typedef struct { uint32_t in_pad, width, n_hidden, out_pad; } orc_mlp;
typedef struct {
	orc_grid grid;
	orc_mlp density, rgb;
	uint32_t dir_offset, in_stride;
} orc_nerf;
uint32_t orc_mlp_n_params(const orc_mlp* m);
void orc_sh4(float dx, float dy, float dz, float* o);

static inline float hf(uint16_t h) { return orc_f16_to_f32(h); }

/* Round a double to the nearest fp16 value (ties to even), returned as float. |x| >= 65520 -> inf. */
static float rn16d(double x) {
	if (x != x) return (float)x;
	const double ax = fabs(x);
	if (ax >= 65520.0) return x > 0 ? INFINITY : -INFINITY;
	int e;
	frexp(ax, &e);                       /* ax = m 2^e, m in [0.5, 1) */
	int q = e - 11;                      /* 11 significant bits: unit 2^(e - 11) */
	if (q < -24) q = -24;                /* subnormal spacing 2^-24 */
	const double unit = ldexp(1.0, q);
	const double r = nearbyint(x / unit) * unit;  /* x / unit is exact (power of two); nearbyint ties to even */
	return (float)r;
}
/* spacing of fp16 values at |x| (2^-24 in the subnormal range) */
static double ulp16(double x) {
	const double ax = fabs(x);
	if (ax < ldexp(1.0, -14)) return ldexp(1.0, -24);
	int e;
	frexp(ax, &e);
	return ldexp(1.0, e - 11);
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
static inline void corner_setup(const orc_grid* g, uint32_t l, const float* x, float* frac, uint32_t* base) {
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

/* Grid forward in tcnn's arithmetic. out: float [n x L*F] (fp16 values); bound (optional, float [n x L*F]):
 * the chain's own rounding-error bound, sum over the corners of the weight's rounding (|w - (half)w| |v|) and
 * half a spacing of each FMA's result, so |out - exact blend| <= bound. All levels active (max_level 1). */
EXPORT void orc_grid_forward_tcnn(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride, const uint16_t* table,
                                  float* out, float* bound) {
	const uint32_t L = g->n_levels, F = g->n_features;
	#pragma omp parallel for schedule(static)
	for (size_t i = 0; i < n; ++i) {
		const float* x = pos + i * pos_stride;
		for (uint32_t l = 0; l < L; ++l) {
			float frac[4]; uint32_t base[4], p[4];
			corner_setup(g, l, x, frac, base);
			float acc[8] = {0};
			double eb[8] = {0};
			for (uint32_t c = 0; c < (1u << g->n_dims); ++c) {
				const float w = corner_weight(g, c, frac, base, p);
				const float wh = hf(orc_f32_to_f16(w));  /* (T)weight */
				const size_t e = (size_t)g->offsets[l] + grid_index(g, l, p);
				for (uint32_t f = 0; f < F; ++f) {
					const double v = hf(table[e * F + f]);
					const double exact = (double)wh * v + (double)acc[f];  /* fp16 FMA: one rounding */
					acc[f] = rn16d(exact);
					eb[f] += fabs((double)wh - (double)w) * fabs(v) + 0.5 * ulp16(exact);
				}
			}
			for (uint32_t f = 0; f < F; ++f) {
				out[i * (size_t)(L * F) + l * F + f] = acc[f];
				if (bound) bound[i * (size_t)(L * F) + l * F + f] = (float)eb[f];
			}
		}
	}
}

/* One layer y = W x in the WMMA fp16-accumulator form: 16-wide k-steps, each summed exactly and added to the
 * fp16 accumulator with one rounding. W fp16 row-major [out x in] at w. */
static void layer_tcnn(const uint16_t* w, uint32_t in, uint32_t out, const float* x, float* y) {
	for (uint32_t o = 0; o < out; ++o) {
		float acc = 0.f;
		for (uint32_t k0 = 0; k0 < in; k0 += 16) {
			double s = 0.0;
			for (uint32_t k = k0; k < k0 + 16 && k < in; ++k) s += (double)hf(w[(size_t)o * in + k]) * (double)x[k];
			acc = rn16d((double)acc + s);
		}
		y[o] = acc;
	}
}
/* Transposed: y[k] = sum_o W[o][k] g[o] (the backward's dX), same k-step form over o. */
static void layer_tcnn_t(const uint16_t* w, uint32_t in, uint32_t out, const float* g, float* y) {
	for (uint32_t k = 0; k < in; ++k) {
		float acc = 0.f;
		for (uint32_t o0 = 0; o0 < out; o0 += 16) {
			double s = 0.0;
			for (uint32_t o = o0; o < o0 + 16 && o < out; ++o) s += (double)hf(w[(size_t)o * in + k]) * (double)g[o];
			acc = rn16d((double)acc + s);
		}
		y[k] = acc;
	}
}

static size_t layer_off(const orc_mlp* m, uint32_t l, uint32_t* in, uint32_t* out) {
	const uint32_t nl = m->n_hidden + 1;
	size_t off = 0;
	for (uint32_t k = 0; k < l; ++k) {
		const uint32_t ki = k == 0 ? m->in_pad : m->width, ko = k == nl - 1 ? m->out_pad : m->width;
		off += (size_t)ki * ko;
	}
	*in = l == 0 ? m->in_pad : m->width;
	*out = l == nl - 1 ? m->out_pad : m->width;
	return off;
}

/* forward of one sample: acts = every layer's fp16 output (ReLU on hidden layers), n_hidden * width + out_pad */
static void mlp_fwd_tcnn(const orc_mlp* m, const uint16_t* w, const float* x, float* acts) {
	const uint32_t nl = m->n_hidden + 1;
	const float* src = x;
	float* dst = acts;
	for (uint32_t l = 0; l < nl; ++l) {
		uint32_t in, out;
		const size_t off = layer_off(m, l, &in, &out);
		layer_tcnn(w + off, in, out, src, dst);
		if (l < nl - 1)
			for (uint32_t o = 0; o < out; ++o) dst[o] = dst[o] > 0.f ? dst[o] : 0.f;
		src = dst;
		dst += out;
	}
}
/* dX chain of one sample from dL/dy (fp16 values): dx = dL/dinput of the first layer */
static void mlp_bwd_tcnn(const orc_mlp* m, const uint16_t* w, const float* acts, const float* dy, float* dx) {
	const uint32_t nl = m->n_hidden + 1;
	float g[256], gn[256];
	memcpy(g, dy, m->out_pad * sizeof(float));
	for (int l = (int)nl - 1; l >= 0; --l) {
		uint32_t in, out;
		const size_t off = layer_off(m, (uint32_t)l, &in, &out);
		layer_tcnn_t(w + off, in, out, g, gn);
		if (l == 0) { memcpy(dx, gn, in * sizeof(float)); break; }
		const float* a_in = acts + (size_t)(l - 1) * m->width;
		for (uint32_t k = 0; k < in; ++k) g[k] = a_in[k] > 0.f ? gn[k] : 0.f;  /* ReLU' of the forward activation */
	}
}

/* NerfNetwork in tcnn's arithmetic (nerf_network.h:116-335): out float [n x 16] (rgb raw rows 0-2, density row 3,
 * the rgb network's padding rows 4-15); denc (optional) float [n x density.in_pad]: dL/d(encoding) for dL_dout
 * float [n x 16] (rows 0-2 rgb, 3 density); enc (optional) float [n x density.in_pad]: the fp16 encoding. */
EXPORT void orc_nerf_tcnn(const orc_nerf* m, const uint16_t* params, size_t n, const float* in, const float* dL_dout, float* out,
                          float* denc, float* enc_out) {
	const orc_grid* gr = &m->grid;
	const uint32_t LF = gr->n_levels * gr->n_features;
	const size_t nd = orc_mlp_n_params(&m->density), nr = orc_mlp_n_params(&m->rgb);
	const uint16_t *wd = params, *wr = params + nd, *table = params + nd + nr;
	#pragma omp parallel
	{
		float enc[256], dacts[1024], racts[1024], rin[32], sh[16], drgb[16], drin[32], dd[16], de[256];
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			const float* x = in + i * m->in_stride;
			float e16[128];
			orc_grid_forward_tcnn(gr, 1, x, m->in_stride, table, e16, NULL);
			for (uint32_t k = 0; k < m->density.in_pad; ++k) enc[k] = k < LF ? e16[k] : 0.f;
			if (enc_out) memcpy(enc_out + i * m->density.in_pad, enc, m->density.in_pad * sizeof(float));
			mlp_fwd_tcnn(&m->density, wd, enc, dacts);
			const float* dout = dacts + m->density.n_hidden * m->density.width;
			for (uint32_t k = 0; k < 16; ++k) rin[k] = dout[k];
			orc_sh4(x[m->dir_offset], x[m->dir_offset + 1], x[m->dir_offset + 2], sh);
			for (uint32_t k = 0; k < 16; ++k) rin[16 + k] = hf(orc_f32_to_f16(sh[k]));
			mlp_fwd_tcnn(&m->rgb, wr, rin, racts);
			const float* rout = racts + m->rgb.n_hidden * m->rgb.width;
			float* o = out + i * 16;
			for (uint32_t k = 0; k < 16; ++k) o[k] = rout[k];
			o[3] = dout[0];  /* extract_density (nerf_network.h:32-43) */
			if (!denc) continue;
			for (uint32_t k = 0; k < 16; ++k) drgb[k] = k < 3 ? dL_dout[i * 16 + k] : 0.f;  /* extract_rgb (:46-60) */
			mlp_bwd_tcnn(&m->rgb, wr, racts, drgb, drin);
			for (uint32_t k = 0; k < 16; ++k) dd[k] = drin[k];
			dd[0] = rn16d((double)dd[0] + (double)dL_dout[i * 16 + 3]);  /* add_density_gradient (:63-74), fp16 add */
			mlp_bwd_tcnn(&m->density, wd, dacts, dd, de);
			memcpy(denc + i * m->density.in_pad, de, m->density.in_pad * sizeof(float));
		}
	}
}

/* Single MLP behind a grid (NetworkWithInputEncoding: SDF / image), tcnn arithmetic: out float [n x out_pad];
 * denc (optional) float [n x in_pad] for dL_dout float [n x out_pad]. */
EXPORT void orc_net_tcnn(const orc_grid* gr, const orc_mlp* mm, const uint16_t* params, size_t n, const float* pos, uint32_t stride,
                         const float* dL_dout, float* out, float* denc) {
	const uint32_t LF = gr->n_levels * gr->n_features;
	const size_t nm = orc_mlp_n_params(mm);
	const uint16_t* table = params + nm;
	#pragma omp parallel
	{
		float enc[256], acts[1024], de[256];
		#pragma omp for schedule(static)
		for (size_t i = 0; i < n; ++i) {
			float e16[128];
			orc_grid_forward_tcnn(gr, 1, pos + i * stride, stride, table, e16, NULL);
			for (uint32_t k = 0; k < mm->in_pad; ++k) enc[k] = k < LF ? e16[k] : 0.f;
			mlp_fwd_tcnn(mm, params, enc, acts);
			memcpy(out + i * mm->out_pad, acts + mm->n_hidden * mm->width, mm->out_pad * sizeof(float));
			if (!denc) continue;
			mlp_bwd_tcnn(mm, params, acts, dL_dout + i * mm->out_pad, de);
			memcpy(denc + i * mm->in_pad, de, mm->in_pad * sizeof(float));
		}
	}
}

/* Grid backward in tcnn's arithmetic: every contribution (half)(dL/dy * w) added to the fp16 gradient with one
 * rounding per add, in sample order (overwrite: the gradient starts at 0). dL_dy fp16 bits [n x dy_stride].
 * grad16 out: fp16 bits [entries x F]; bound (optional, double [entries x F]): the sum of half a spacing of every
 * add's result, so |grad16 - exact sum of the rounded contributions| <= bound. Sequential (the order is the
 * point); all levels active. */
EXPORT void orc_grid_backward_tcnn(const orc_grid* g, size_t n, const float* pos, uint32_t pos_stride, const uint16_t* dL_dy,
                                   uint32_t dy_stride, uint16_t* grad16, double* bound) {
	const uint32_t L = g->n_levels, F = g->n_features;
	const size_t np = (size_t)g->offsets[L] * F;
	float* acc = (float*)calloc(np, sizeof(float));
	if (bound) memset(bound, 0, np * sizeof(double));
	for (size_t i = 0; i < n; ++i) {
		const float* x = pos + i * pos_stride;
		for (uint32_t l = 0; l < L; ++l) {
			float frac[4]; uint32_t base[4], p[4];
			corner_setup(g, l, x, frac, base);
			for (uint32_t c = 0; c < (1u << g->n_dims); ++c) {
				const float w = corner_weight(g, c, frac, base, p);
				const size_t e = (size_t)g->offsets[l] + grid_index(g, l, p);
				for (uint32_t f = 0; f < F; ++f) {
					const float contrib = hf(orc_f32_to_f16(hf(dL_dy[i * dy_stride + l * F + f]) * w));
					if (contrib == 0.f) continue;
					const double exact = (double)acc[e * F + f] + (double)contrib;
					acc[e * F + f] = rn16d(exact);
					if (bound) bound[e * F + f] += 0.5 * ulp16(exact);
				}
			}
		}
	}
	for (size_t k = 0; k < np; ++k) grad16[k] = orc_f32_to_f16(acc[k]);
	free(acc);
}
