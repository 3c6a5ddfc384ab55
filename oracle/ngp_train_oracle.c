/*
 * ngp_train_oracle.c — CPU restatement of the image (BASELINE C1) and SDF (BASELINE C5) training
 * data paths and of tcnn's losses.
 *
 * TEST INFRASTRUCTURE ONLY (see ngp_oracle.c): loaded by tests/ as the checker, never by the product.
 *
 * Follows: src/testbed_image.cu:62-76 (stratify2_kernel), :167-212 (eval_image_kernel_and_snap),
 * :214-285 (train_image); src/testbed_sdf.cu:222-231 (perturb_sdf_samples), :467-472
 * (scale_to_aabb_kernel), :615-627 (sample_discrete, sample_uniform_on_triangle_kernel), :1187-1275
 * (generate_training_samples_sdf); include/neural-graphics-primitives/triangle.cuh:26-85
 * (sample_uniform_position, ray_intersect, distance_sq); random_val.cuh:45-54,84-99
 * (cylindrical_to_dir, fibonacci_dir); common.h:268-292 (binary_search); common_device.cuh:99-105
 * (linear_to_srgb); src/triangle_bvh.cu:415-433 (signed_distance_raystab).
 * tcnn† (absent, restated; parity unpinned): generate_random_uniform element k = draw k;
 * generate_random_logistic = logit(clamp(u)) * stddev * sqrt(3)/pi + mean; L2/L1/MAPE/SMAPE/
 * RelativeL2 losses normalised by n * dims.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

typedef struct { uint64_t state, inc; } orc_pcg32;
void orc_pcg32_advance(orc_pcg32* r, int64_t delta);
float orc_pcg32_next_float(orc_pcg32* r);
uint16_t orc_f32_to_f16(float f);
float orc_f16_to_f32(uint16_t h);

/* ---- losses ------------------------------------------------------------------------------- */
static void loss_one(int type, float pred, float target, float inv_n, float* value, float* grad) {
	const float d = pred - target;
	if (type == 0) { *value = d * d * inv_n; *grad = 2.0f * d * inv_n; }
	else if (type == 1) { *value = fabsf(d) * inv_n; *grad = copysignf(1.0f, d) * inv_n; }
	else if (type == 2) { const float sc = 1.0f / (fabsf(target) + 1e-2f); *value = fabsf(d) * sc * inv_n; *grad = copysignf(1.0f, d) * sc * inv_n; }
	else if (type == 3) { const float sc = 2.0f / (fabsf(pred) + fabsf(target) + 1e-2f); *value = fabsf(d) * sc * inv_n; *grad = copysignf(1.0f, d) * sc * inv_n; }
	else { const float den = pred * pred + 1e-2f; *value = d * d / den * inv_n; *grad = 2.0f * d / den * inv_n; }
}

/* out16: [n x out_stride] half bits; target [n x target_stride]; dL16 [n x dL_stride] half bits */
EXPORT double orc_loss(int type, uint32_t n, uint32_t dims, const uint16_t* out16, uint32_t out_stride, const float* target,
                       uint32_t target_stride, float loss_scale, uint16_t* dL16, uint32_t dL_stride, float* values) {
	const float inv_n = 1.0f / ((float)n * (float)dims);
	double total = 0.0;
	for (uint32_t i = 0; i < n; ++i) {
		float sum = 0.f;
		for (uint32_t j = 0; j < dL_stride; ++j) {
			if (j < dims) {
				float v, g;
				loss_one(type, orc_f16_to_f32(out16[(size_t)i * out_stride + j]), target[(size_t)i * target_stride + j], inv_n, &v, &g);
				sum += v;
				dL16[(size_t)i * dL_stride + j] = orc_f32_to_f16(loss_scale * g);
			} else {
				dL16[(size_t)i * dL_stride + j] = 0;
			}
		}
		if (values) values[i] = sum;
		total += sum;
	}
	return total;
}

/* ---- image ---------------------------------------------------------------------------------- */
static float linear_to_srgb(float x) { return x < 0.0031308f ? 12.92f * x : 1.055f * powf(x, 0.41666f) - 0.055f; }

EXPORT void orc_image_samples(uint32_t n, orc_pcg32* rng, int random_mode, int snap, int linear_colors, uint32_t W, uint32_t H,
                              const float* tex, float* positions, float* targets) {
	uint32_t log2_n = ~0u;
	if (n && (n & (n - 1)) == 0) {
		uint32_t l = 0;
		while ((1u << l) < n) ++l;
		if (l % 2 == 0) log2_n = l;
	}
	orc_pcg32 r = *rng;
	for (uint32_t i = 0; i < n; ++i) {
		float px = orc_pcg32_next_float(&r), py = orc_pcg32_next_float(&r);
		if (random_mode == 3 && log2_n != ~0u) {
			const uint32_t log2s = log2_n / 2, size = 1u << log2s;
			const uint32_t idx = i & ((1u << log2_n) - 1u);
			const uint32_t x = idx & (size - 1u), y = idx >> log2s;
			px = px / (float)size + ((float)x / (float)size);
			py = py / (float)size + ((float)y / (float)size);
		}
		float val[3];
#define RD(X, Y, O) do { const float* t_ = tex + ((size_t)(Y) * W + (X)) * 4; for (int c_ = 0; c_ < 3; ++c_) (O)[c_] = linear_colors ? t_[c_] : linear_to_srgb(t_[c_]); } while (0)
		if (snap) {
			int ix = (int)floorf(px * (float)W), iy = (int)floorf(py * (float)H);
			px = ((float)ix + 0.5f) / (float)W;
			py = ((float)iy + 0.5f) / (float)H;
			if (ix < 0) ix = 0;
			if (ix > (int)W - 1) ix = (int)W - 1;
			if (iy < 0) iy = 0;
			if (iy > (int)H - 1) iy = (int)H - 1;
			RD(ix, iy, val);
		} else {
			const float fx = fminf(fmaxf(px * (float)W - 0.5f, 0.0f), (float)W - (1.0f + 1e-4f));
			const float fy = fminf(fmaxf(py * (float)H - 0.5f, 0.0f), (float)H - (1.0f + 1e-4f));
			const int x0 = (int)fx, y0 = (int)fy;
			const float wx = fx - (float)x0, wy = fy - (float)y0;
			int ix = x0, iy = y0;
			if (ix < 0) ix = 0;
			if (ix > (int)W - 2) ix = (int)W - 2;
			if (iy < 0) iy = 0;
			if (iy > (int)H - 2) iy = (int)H - 2;
			float v00[3], v10[3], v01[3], v11[3];
			RD(ix, iy, v00); RD(ix + 1, iy, v10); RD(ix, iy + 1, v01); RD(ix + 1, iy + 1, v11);
			for (int c = 0; c < 3; ++c)
				val[c] = (1 - wx) * (1 - wy) * v00[c] + wx * (1 - wy) * v10[c] + (1 - wx) * wy * v01[c] + wx * wy * v11[c];
		}
#undef RD
		positions[2 * (size_t)i] = px;
		positions[2 * (size_t)i + 1] = py;
		for (int c = 0; c < 3; ++c) targets[3 * (size_t)i + c] = val[c];
	}
	orc_pcg32_advance(rng, 2 * (int64_t)n);
}

/* ---- SDF ------------------------------------------------------------------------------------ */
typedef struct { float x, y, z; } F3;
static F3 ld3(const float* p) { F3 r = {p[0], p[1], p[2]}; return r; }
static F3 sub(F3 a, F3 b) { F3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static F3 add(F3 a, F3 b) { F3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static F3 mul(F3 a, float s) { F3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static F3 cross(F3 a, F3 b) { F3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; return r; }
static float len2(F3 a) { return dot(a, a); }
static float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
static float clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

static uint32_t binary_search(float val, const float* data, uint32_t length) {
	if (length == 0) return 0;
	uint32_t first = 0, count = length;
	while (count > 0) {
		uint32_t it = first;
		const uint32_t step = count / 2;
		it += step;
		if (data[it] < val) { first = ++it; count -= step + 1; }
		else count = step;
	}
	return first;
}

static float logistic_sample(float u, float mean, float stddev) {
	const float x = fminf(fmaxf(u, 1e-9f), 1.0f - 1e-9f);
	return -logf(1.0f / x - 1.0f) * stddev * 0.551328895f + mean;
}

/* triangle_distribution.build (discrete_distribution.h:20-36) */
EXPORT void orc_triangle_cdf(uint32_t n_tris, const float* tris, float* cdf) {
	float total = 0.f;
	for (uint32_t i = 0; i < n_tris; ++i) {
		const float* t = tris + 9 * (size_t)i;
		F3 c = cross(sub(ld3(t + 3), ld3(t)), sub(ld3(t + 6), ld3(t)));
		total += 0.5f * sqrtf(len2(c));
	}
	const float inv = 1.0f / total;
	float acc = 0.f;
	for (uint32_t i = 0; i < n_tris; ++i) {
		const float* t = tris + 9 * (size_t)i;
		F3 c = cross(sub(ld3(t + 3), ld3(t)), sub(ld3(t + 6), ld3(t)));
		acc += 0.5f * sqrtf(len2(c)) * inv;
		cdf[i] = acc;
	}
	if (n_tris) cdf[n_tris - 1] = 1.0f;
}

/* positions / upper-bound distances of generate_training_samples_sdf, before the signed distance */
EXPORT void orc_sdf_samples(uint32_t n, orc_pcg32* rng, uint32_t n_tris, const float* tris, const float* cdf,
                            const float* aabb_min, const float* aabb_max, float stddev, float* positions, float* distances) {
	const uint32_t base = n / 8, n_exact = 4 * base, n_offset = 3 * base, n_uniform = base, n_surface = n_exact + n_offset;
	orc_pcg32 r = *rng;
	for (uint32_t i = 0; i < n; ++i) {
		F3 p;
		p.x = orc_pcg32_next_float(&r); p.y = orc_pcg32_next_float(&r); p.z = orc_pcg32_next_float(&r);
		float dist = 0.f;
		if (i < n_surface) {
			uint32_t t = binary_search(p.x, cdf, n_tris);
			if (t > n_tris - 1) t = n_tris - 1;
			const float* tri = tris + 9 * (size_t)t;
			const float sx = sqrtf(p.y);
			const float f0 = 1.0f - sx, f1 = sx * (1.0f - p.z), f2 = sx * p.z;
			p = add(add(mul(ld3(tri), f0), mul(ld3(tri + 3), f1)), mul(ld3(tri + 6), f2));
		} else if (i < n_surface + n_uniform) {
			const F3 mn = {aabb_min[0], aabb_min[1], aabb_min[2]};
			const F3 diag = {aabb_max[0] - mn.x, aabb_max[1] - mn.y, aabb_max[2] - mn.z};
			F3 q = {mn.x + p.x * diag.x, mn.y + p.y * diag.y, mn.z + p.z * diag.z};
			p = q;
			dist = sqrtf(len2(diag)) * 1.001f;
		}
		positions[3 * (size_t)i] = p.x; positions[3 * (size_t)i + 1] = p.y; positions[3 * (size_t)i + 2] = p.z;
		distances[i] = dist;
	}
	/* perturbations: draws 3n .. 3n + 3 n_offset of the same stream */
	for (uint32_t j = 0; j < n_offset; ++j) {
		F3 q;
		q.x = logistic_sample(orc_pcg32_next_float(&r), 0.f, stddev);
		q.y = logistic_sample(orc_pcg32_next_float(&r), 0.f, stddev);
		q.z = logistic_sample(orc_pcg32_next_float(&r), 0.f, stddev);
		float* pp = positions + 3 * (size_t)(n_exact + j);
		pp[0] += q.x; pp[1] += q.y; pp[2] += q.z;
		distances[n_exact + j] = sqrtf(len2(q)) * 1.001f;
	}
	orc_pcg32_advance(rng, 3 * (int64_t)n + 3 * (int64_t)n_offset);
}

static float tri_distance_sq(const float* t, F3 pos) {
	const F3 A = ld3(t), B = ld3(t + 3), Cc = ld3(t + 6);
	const F3 v21 = sub(B, A), p1 = sub(pos, A);
	const F3 v32 = sub(Cc, B), p2 = sub(pos, B);
	const F3 v13 = sub(A, Cc), p3 = sub(pos, Cc);
	const F3 nor = cross(v21, v13);
	if (sgn(dot(cross(v21, nor), p1)) + sgn(dot(cross(v32, nor), p2)) + sgn(dot(cross(v13, nor), p3)) < 2.0f) {
		const float e1 = len2(sub(mul(v21, clamp01(dot(v21, p1) / len2(v21))), p1));
		const float e2 = len2(sub(mul(v32, clamp01(dot(v32, p2) / len2(v32))), p2));
		const float e3 = len2(sub(mul(v13, clamp01(dot(v13, p3) / len2(v13))), p3));
		return fminf(fminf(e1, e2), e3);
	}
	const float d = dot(nor, p1);
	return d * d / len2(nor);
}

static float tri_ray(const float* t, F3 ro, F3 rd) {
	const F3 A = ld3(t);
	const F3 v1v0 = sub(ld3(t + 3), A), v2v0 = sub(ld3(t + 6), A), rov0 = sub(ro, A);
	const F3 nn = cross(v1v0, v2v0);
	const F3 q = cross(rov0, rd);
	const float d = 1.0f / dot(rd, nn);
	const float u = d * -dot(q, v2v0);
	const float v = d * dot(q, v1v0);
	float tt = d * -dot(nn, rov0);
	if (u < 0.0f || u > 1.0f || v < 0.0f || (u + v) > 1.0f || tt < 0.0f) tt = 3.402823466e38f;
	return tt;
}

static F3 fib_dir32(uint32_t i, float ox, float oy) {
	const float eps = 1.33f;
	const float golden = 1.6180339887498948482045868343656f;
	float a = (i + eps) / (32 - 1 + 2 * eps) + ox;
	float b = i / golden + oy;
	a = a - floorf(a);
	b = b - floorf(b);
	const float cos_theta = -2.0f * a + 1.0f;
	const float phi = 2.0f * 3.14159265358979323846f * (b - 0.5f);
	const float sin_theta = sqrtf(fmaxf(1.0f - cos_theta * cos_theta, 0.0f));
	F3 r = {sin_theta * cosf(phi), sin_theta * sinf(phi), cos_theta};
	return r;
}

/* signed_distance_raystab_kernel (src/triangle_bvh.cu:688-703) over every triangle (the BVH only
 * prunes): per element i a default pcg32 advanced by 2 i gives the stab-ray offset random_val_2d. */
EXPORT void orc_sdf_signed_distance(uint32_t n, const float* positions, uint32_t n_tris, const float* tris, float* distances) {
#pragma omp parallel for schedule(dynamic, 1)
	for (uint32_t i = 0; i < n; ++i) {
		orc_pcg32 r0 = {0x853c49e6748fea9bULL, 0xda3e39cb94b95bdbULL};
		orc_pcg32_advance(&r0, 2 * (int64_t)i);
		const float ox = orc_pcg32_next_float(&r0), oy = orc_pcg32_next_float(&r0);
		const F3 p = ld3(positions + 3 * (size_t)i);
		float best = 3.402823466e38f;
		for (uint32_t t = 0; t < n_tris; ++t) best = fminf(best, tri_distance_sq(tris + 9 * (size_t)t, p));
		const float d = sqrtf(best);
		int escaped = 0;
		for (uint32_t k = 0; k < 32 && !escaped; ++k) {
			const F3 dir = fib_dir32(k, ox, oy);
			float mint = 10.0f;
			for (uint32_t t = 0; t < n_tris; ++t) mint = fminf(mint, tri_ray(tris + 9 * (size_t)t, p, dir));
			escaped = !(mint < 10.0f);
		}
		distances[i] = escaped ? d : -d;
	}
}
