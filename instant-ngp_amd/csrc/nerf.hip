// nerf.hip — NeRF training kernels for gfx950 (see nerf.h). Each kernel cites the reference kernel
// it re-implements; float formulas follow the reference line by line (glm vector ops written out
// per component, -ffp-contract=off). Every exp/log whose result decides an integer (cone-angle
// stepping, compositing termination and compaction) is ngp_expf/ngp_logf from ngp_math.h, the same
// instruction sequence the oracle runs, so sample indices, coordinates and compacted counts match the
// oracle bit for bit at every cone angle (the reference's libdevice logf/expf/__expf are <= 2-ulp
// approximations of the same functions).

#include <cmath>
#include <functional>
#include <cstring>

#include "nerf.h"
#include "ngp_math.h"
#include "profiler.h"
#include "rng.h"

namespace ngp {
namespace nerf {

// ------------------------------------------------------------------------------------------------
// device math
// ------------------------------------------------------------------------------------------------
struct V3 { float x, y, z; };
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }

// t / MIN_CONE_STEPSIZE, correctly rounded, in three instructions: q = t * RN(1/c) and one residual
// correction. Checked exhaustively against the IEEE quotient for every float t >= 0
// (tools/microbench/div_check.c): equal for 1.5e-31 <= t <= 5.7e35; outside that the IEEE divide runs.
// Both the quotient and the residual step are odd in t, so the same holds for -t (the linear segment
// below `at` divides t - at <= 0).
__device__ __forceinline__ float div_min_stepsize(float t) {
	constexpr float c = MIN_CONE_STEPSIZE;
	const float r = 1.0f / c;  // folded to RN(1/c) at compile time
	const float at = fabsf(t);
	if (__builtin_expect(at >= 1e-30f && at <= 1e35f, 1)) {
		const float q = t * r;
		return __builtin_fmaf(__builtin_fmaf(-q, c, t), r, q);
	}
	return t / c;
}
// x / MAX_CONE_STEPSIZE: MAX = MIN * 2^10 exactly, so (barring subnormals, excluded by the range test)
// RN(x / MAX) = RN(x / MIN) * 2^-10.
static_assert(MAX_CONE_STEPSIZE == MIN_CONE_STEPSIZE * 1024.0f, "MAX_CONE_STEPSIZE = MIN * 2^10");
__device__ __forceinline__ float div_max_stepsize(float t) {
	const float at = fabsf(t);
	if (__builtin_expect(at >= 1e-30f && at <= 1e35f, 1)) return div_min_stepsize(t) * (1.0f / 1024.0f);
	return t / MAX_CONE_STEPSIZE;
}

// testbed_nerf.cu:114-184. The constants of a cone angle (log(1 + cone), the two linear segments'
// bounds) are computed once per ray or thread (make_cone), not at every step: with the shared
// software logf/expf (ngp_math.h) they are ~10 transcendental evaluations per call. Same operations
// and values as evaluating them inline.
struct Cone {
	float c, log1p_c, a, b, at, bt, rl;  // rl = RN(1 / log1p_c)
};
// host and device: the sampler computes it once per launch on the host (same ngp_math.h operations)
__host__ __device__ inline Cone make_cone(float c) {
	Cone k{c, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
	if (c <= 1e-5f) return k;
	k.log1p_c = ngp_logf(1.0f + c);
	k.rl = 1.0f / k.log1p_c;
	k.a = (ngp_logf(MIN_CONE_STEPSIZE) - ngp_logf(k.log1p_c)) / k.log1p_c;
	k.b = (ngp_logf(MAX_CONE_STEPSIZE) - ngp_logf(k.log1p_c)) / k.log1p_c;
	k.at = ngp_expf(k.a * k.log1p_c);
	k.bt = ngp_expf(k.b * k.log1p_c);
	return k;
}
__device__ float to_stepping_space(float t, const Cone& k) {
	if (k.c <= 1e-5f) return div_min_stepsize(t);
	if (t <= k.at) return div_min_stepsize(t - k.at) + k.a;
	if (t <= k.bt) return ngp_div_rc(ngp_logf_pos(t), k.log1p_c, k.rl);  // at < t <= bt: positive, normal
	return div_max_stepsize(t - k.bt) + k.b;
}
__device__ float from_stepping_space(float n, const Cone& k) {
	if (k.c <= 1e-5f) return n * MIN_CONE_STEPSIZE;
	if (n <= k.a) return (n - k.a) * MIN_CONE_STEPSIZE + k.at;
	if (n <= k.b) return ngp_expf_mid(n * k.log1p_c);  // a l < n l <= b l, i.e. log(at) .. log(bt): |.| << 80
	return (n - k.b) * MAX_CONE_STEPSIZE + k.bt;
}
__device__ __forceinline__ float advance_n_steps(float t, const Cone& k, float n) { return from_stepping_space(to_stepping_space(t, k) + n, k); }
__device__ __forceinline__ float calc_dt(float t, const Cone& k) { return advance_n_steps(t, k, 1.0f) - t; }

__device__ __forceinline__ float signf_(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }  // glm::sign

// testbed_nerf.cu:272-315
__device__ float distance_to_next_voxel(V3 pos, V3 dir, V3 idir, float res) {
	const V3 p = v3(res * (pos.x - 0.5f), res * (pos.y - 0.5f), res * (pos.z - 0.5f));
	const float tx = (floorf(p.x + 0.5f + 0.5f * signf_(dir.x)) - p.x) * idir.x;
	const float ty = (floorf(p.y + 0.5f + 0.5f * signf_(dir.y)) - p.y) * idir.y;
	const float tz = (floorf(p.z + 0.5f + 0.5f * signf_(dir.z)) - p.z) * idir.z;
	const float t = fminf(fminf(tx, ty), tz);
	return fmaxf(t * (1.0f / res), 0.0f);  // res is a power of two: same rounding as t / res, no IEEE divide
}
// n_t = to_stepping_space(t): callers that already hold it (the sampler's empty-space march, which
// also needs it for calc_dt) pass it in.
__device__ __forceinline__ float advance_to_next_voxel_n(float t, float n_t, const Cone& cone, V3 pos, V3 dir, V3 idir, uint32_t mip) {
	const float res = scalbnf((float)GRIDSIZE, -(int)mip);
	const float t_target = to_stepping_space(t + distance_to_next_voxel(pos, dir, idir, res), cone);
	return from_stepping_space(n_t + ceilf(fmaxf(t_target - n_t, 0.5f)), cone);
}
__device__ float advance_to_next_voxel(float t, const Cone& cone, V3 pos, V3 dir, V3 idir, uint32_t mip) {
	return advance_to_next_voxel_n(t, to_stepping_space(t, cone), cone, pos, dir, idir, mip);
}

// testbed_nerf.cu:614-633
__device__ uint32_t mip_from_pos(V3 pos, uint32_t max_cascade) {
	int exponent;
	const float maxval = fmaxf(fmaxf(fabsf(pos.x - 0.5f), fabsf(pos.y - 0.5f)), fabsf(pos.z - 0.5f));
	frexpf(maxval, &exponent);
	const int e = exponent + 1;
	return (uint32_t)(e < 0 ? 0 : (e > (int)max_cascade ? (int)max_cascade : e));
}
__device__ uint32_t mip_from_dt(float dt, V3 pos, uint32_t max_cascade) {
	const uint32_t mip = mip_from_pos(pos, max_cascade);
	dt *= 2 * GRIDSIZE;
	if (dt < 1.0f) return mip;
	int exponent;
	frexpf(dt, &exponent);
	int v = (int)mip > exponent ? (int)mip : exponent;  // tcnn::clamp(mip, exponent, max_cascade)
	return (uint32_t)(v < (int)max_cascade ? v : (int)max_cascade);
}

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
	v = (v * 0x00010001u) & 0xFF0000FFu;
	v = (v * 0x00000101u) & 0x0F00F00Fu;
	v = (v * 0x00000011u) & 0xC30C30C3u;
	v = (v * 0x00000005u) & 0x49249249u;
	return v;
}
// tcnn morton3D: x in bit 0 (consistent with morton3D_invert(idx >> 0) = x, testbed_nerf.cu:518-520)
__device__ __forceinline__ uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) {
	return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
__device__ __forceinline__ uint32_t morton3D_invert(uint32_t x) {
	x = x & 0x49249249u;
	x = (x | (x >> 2)) & 0xc30c30c3u;
	x = (x | (x >> 4)) & 0x0f00f00fu;
	x = (x | (x >> 8)) & 0xff0000ffu;
	x = (x | (x >> 16)) & 0x0000ffffu;
	return x;
}

// testbed_nerf.cu:433-457
__device__ uint32_t cascaded_grid_idx_at(V3 pos, uint32_t mip) {
	const float mip_scale = scalbnf(1.0f, -(int)mip);
	pos = v3((pos.x - 0.5f) * mip_scale + 0.5f, (pos.y - 0.5f) * mip_scale + 0.5f, (pos.z - 0.5f) * mip_scale + 0.5f);
	const int ix = (int)(pos.x * (float)GRIDSIZE), iy = (int)(pos.y * (float)GRIDSIZE), iz = (int)(pos.z * (float)GRIDSIZE);
	if (ix < 0 || ix >= (int)GRIDSIZE || iy < 0 || iy >= (int)GRIDSIZE || iz < 0 || iz >= (int)GRIDSIZE) return 0xFFFFFFFFu;
	return morton3D((uint32_t)ix, (uint32_t)iy, (uint32_t)iz);
}
__device__ bool density_grid_occupied_at(V3 pos, const uint8_t* bitfield, uint32_t mip) {
	const uint32_t idx = cascaded_grid_idx_at(pos, mip);
	if (idx == 0xFFFFFFFFu) return false;
	return bitfield[idx / 8 + GRID_N_CELLS * mip / 8] & (1 << (idx % 8));
}

struct Aabb { V3 mn, mx; };
__device__ __forceinline__ bool aabb_contains(const Aabb& b, V3 p) {
	return p.x >= b.mn.x && p.x <= b.mx.x && p.y >= b.mn.y && p.y <= b.mx.y && p.z >= b.mn.z && p.z <= b.mx.z;
}
// bounding_box.cuh:163-216
__device__ void aabb_ray_intersect(const Aabb& b, V3 pos, V3 dir, float* out_min, float* out_max) {
	const float FMAX = 3.402823466e+38f;
	float tmin = (b.mn.x - pos.x) / dir.x, tmax = (b.mx.x - pos.x) / dir.x;
	if (tmin > tmax) { float t = tmin; tmin = tmax; tmax = t; }
	float tymin = (b.mn.y - pos.y) / dir.y, tymax = (b.mx.y - pos.y) / dir.y;
	if (tymin > tymax) { float t = tymin; tymin = tymax; tymax = t; }
	if (tmin > tymax || tymin > tmax) { *out_min = FMAX; *out_max = FMAX; return; }
	if (tymin > tmin) tmin = tymin;
	if (tymax < tmax) tmax = tymax;
	float tzmin = (b.mn.z - pos.z) / dir.z, tzmax = (b.mx.z - pos.z) / dir.z;
	if (tzmin > tzmax) { float t = tzmin; tzmin = tzmax; tzmax = t; }
	if (tmin > tzmax || tzmin > tmax) { *out_min = FMAX; *out_max = FMAX; return; }
	if (tzmin > tmin) tmin = tzmin;
	if (tzmax < tmax) tmax = tzmax;
	*out_min = tmin; *out_max = tmax;
}

__device__ __forceinline__ float warp_dt(float dt) {  // :413-416
	const float max_stepsize = MIN_CONE_STEPSIZE * (1 << (CASCADES - 1));
	return (dt - MIN_CONE_STEPSIZE) / (max_stepsize - MIN_CONE_STEPSIZE);
}
__device__ __forceinline__ float unwarp_dt(float dt) {  // :418-421
	const float max_stepsize = MIN_CONE_STEPSIZE * (1 << (CASCADES - 1));
	return dt * (max_stepsize - MIN_CONE_STEPSIZE) + MIN_CONE_STEPSIZE;
}

// common_device.cuh:75-121
__device__ __forceinline__ float srgb_to_linear(float s) { return s <= 0.04045f ? s / 12.92f : powf((s + 0.055f) / 1.055f, 2.4f); }
__device__ __forceinline__ float linear_to_srgb(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * powf(l, 0.41666f) - 0.055f; }

__device__ __forceinline__ float logistic(float x) { return 1.0f / (1.0f + ngp_expf_fast(-x)); }  // tcnn::logistic
// testbed_nerf.cu:317-378 (the reference's __expf; ngp_expf here and in the oracle)
__device__ float network_to_rgb(float v, uint32_t act) {
	switch (act) {
		case ACT_NONE: return v;
		case ACT_RELU: return v > 0.0f ? v : 0.0f;
		case ACT_LOGISTIC: return logistic(v);
		case ACT_EXP: return ngp_expf_mid(fminf(fmaxf(v, -10.0f), 10.0f));
	}
	return 0.0f;
}
__device__ float network_to_rgb_derivative(float v, uint32_t act) {
	switch (act) {
		case ACT_NONE: return 1.0f;
		case ACT_RELU: return v > 0.0f ? 1.0f : 0.0f;
		case ACT_LOGISTIC: { const float d = logistic(v); return d * (1 - d); }
		case ACT_EXP: return ngp_expf_mid(fminf(fmaxf(v, -10.0f), 10.0f));
	}
	return 0.0f;
}
__device__ float network_to_density(float v, uint32_t act) {
	switch (act) {
		case ACT_NONE: return v;
		case ACT_RELU: return v > 0.0f ? v : 0.0f;
		case ACT_LOGISTIC: return logistic(v);
		case ACT_EXP: return ngp_expf_fast(v);
	}
	return 0.0f;
}
__device__ float network_to_density_derivative(float v, uint32_t act) {
	switch (act) {
		case ACT_NONE: return 1.0f;
		case ACT_RELU: return v > 0.0f ? 1.0f : 0.0f;
		case ACT_LOGISTIC: { const float d = logistic(v); return d * (1 - d); }
		case ACT_EXP: return ngp_expf_mid(fminf(fmaxf(v, -15.0f), 15.0f));
	}
	return 0.0f;
}

// loss_and_gradient (testbed_nerf.cu:1340-1355) per channel
__device__ void loss_channel(float target, float pred, uint32_t type, float* loss, float* grad) {
	const float d = pred - target;
	switch (type) {
		case LOSS_RELL2: { const float den = pred * pred + 1e-2f; *loss = d * d / den; *grad = 2.0f * d / den; return; }
		case LOSS_L1: *loss = fabsf(d); *grad = copysignf(1.0f, d); return;
		case LOSS_MAPE: { const float den = fabsf(pred) + 1e-2f; *loss = fabsf(d) / den; *grad = copysignf(1.0f / den, d); return; }
		case LOSS_SMAPE: { const float den = 0.5f * (fabsf(pred) + fabsf(target)) + 1e-2f; *loss = fabsf(d) / den; *grad = copysignf(1.0f / den, d); return; }
		case LOSS_HUBER: {
			const float alpha = 0.1f, ad = fabsf(d), sq = 0.5f / alpha * d * d;
			*loss = (ad > alpha ? (ad - 0.5f * alpha) : sq) / 5.0f;
			*grad = (ad > alpha ? (d > 0 ? 1.0f : -1.0f) : (d / alpha)) / 5.0f;
			return;
		}
		case LOSS_LOGL1: { const float div = fabsf(d) + 1.0f; *loss = ngp_logf(div); *grad = copysignf(1.0f / div, d); return; }
		default: *loss = d * d; *grad = 2.0f * d; return;
	}
}

__device__ __forceinline__ Aabb cfg_aabb(const ngp_nerf_config& c) {
	return Aabb{v3(c.aabb_min[0], c.aabb_min[1], c.aabb_min[2]), v3(c.aabb_max[0], c.aabb_max[1], c.aabb_max[2])};
}

// image_idx (testbed_nerf.cu:1317-1338), uniform branch
__device__ __forceinline__ uint32_t image_idx(uint32_t base_idx, uint32_t n_rays, uint32_t n_images) {
	return ((base_idx * n_images) / n_rays) % n_images;
}

// nerf_random_image_pos_training (:1292-1315) without error-map CDFs
__device__ void random_image_pos(Rng& rng, uint32_t w, uint32_t h, bool snap, float* u, float* v) {
	*u = pcg_float(rng);
	*v = pcg_float(rng);
	if (snap) {
		int px = (int)(*u * (float)w), py = (int)(*v * (float)h);
		px = px < 0 ? 0 : (px > (int)w - 1 ? (int)w - 1 : px);
		py = py < 0 ? 0 : (py > (int)h - 1 ? (int)h - 1 : py);
		*u = ((float)px + 0.5f) / (float)w;
		*v = ((float)py + 0.5f) / (float)h;
	}
}

__device__ __forceinline__ uint64_t pixel_index(float u, float v, uint32_t w, uint32_t h) {  // image_pos + pixel_idx
	int px = (int)(u * (float)w), py = (int)(v * (float)h);
	px = px < 0 ? 0 : (px > (int)w - 1 ? (int)w - 1 : px);
	py = py < 0 ? 0 : (py > (int)h - 1 ? (int)h - 1 : py);
	return (uint64_t)px + (uint64_t)py * w;
}

// Ray setup shared by the sampler's two passes (testbed_nerf.cu:1415-1493).
struct RaySetup {
	bool valid;
	V3 o, d, dn, idir;
	float startt, cone;
};

__device__ RaySetup setup_ray(const Camera* cams, const uint32_t* pixels, uint32_t n_images, const ngp_nerf_config& cfg,
                              uint32_t ig, uint32_t n_rays_div, Rng rng, const Cone& cone) {
	RaySetup r;
	r.valid = false;
	const uint32_t img = image_idx(ig, n_rays_div, n_images);
	const Camera& cam = cams[img];
	pcg_advance(rng, (uint64_t)ig * N_MAX_RANDOM_SAMPLES_PER_RAY);
	float u, v;
	random_image_pos(rng, cam.width, cam.height, cfg.snap_to_pixel_centers != 0, &u, &v);
	const uint32_t raw = pixels[cam.pixel_offset + pixel_index(u, v, cam.width, cam.height)];
	if (raw == 0x00FF00FFu) return r;  // masked (read_rgba returns -1)
	(void)pcg_float(rng);              // motionblur_time
	// uv_to_ray (common_device.cuh:443-510): pinhole, then the lens undistortion
	float dx = (u - cam.principal[0]) * (float)cam.width / cam.focal[0];
	float dy = (v - cam.principal[1]) * (float)cam.height / cam.focal[1];
	lens_undistort(cam.lens_mode, cam.lens, &dx, &dy);
	const float dz = 1.0f;
	const float* m = cam.m;
	r.d = v3(m[0] * dx + m[3] * dy + m[6] * dz, m[1] * dx + m[4] * dy + m[7] * dz, m[2] * dx + m[5] * dy + m[8] * dz);
	r.o = v3(m[9], m[10], m[11]);
	const float inv = 1.0f / sqrtf(r.d.x * r.d.x + r.d.y * r.d.y + r.d.z * r.d.z);
	r.dn = v3(r.d.x * inv, r.d.y * inv, r.d.z * inv);
	float tmin, tmax;
	aabb_ray_intersect(cfg_aabb(cfg), r.o, r.dn, &tmin, &tmax);
	r.cone = cfg.cone_angle_constant;
	tmin = fmaxf(tmin, 0.0f);
	r.startt = advance_n_steps(tmin, cone, pcg_float(rng));
	r.idir = v3(1.0f / r.dn.x, 1.0f / r.dn.y, 1.0f / r.dn.z);
	r.valid = true;
	return r;
}

// Conservative end of sampling along a ray: for t > sampling_end no occupancy test of the sampler can
// succeed, so the count pass stops there with the same result (no exact skip positions are needed
// after the last occupied cell). Found by marching BACKWARD from the aabb exit through the pooled
// bitfield mips: a cell empty at mip m >= the mip the sampler would use there (mip_from_dt) is empty
// at every finer mip (bitfield_max_pool ORs children into parents, testbed_nerf.cu:788-809), and that
// mip never grows as t decreases. The forward march through the trailing empty space (one skip per
// mip-0 voxel, ~70 % of the pass at Lego scale) is replaced by a handful of coarse backward jumps.
// Occupancy of the mip-m cell containing p in the DDA frame (cell boundaries where res*(p - 0.5) is
// an integer, the frame advance_to_next_voxel / the backward jump use), OR-ed with the sampler's own
// classification of p (cascaded_grid_idx_at rounds (p - 0.5) * 2^-m + 0.5, which can land in the
// neighbouring cell within a few ulps of a face): the scan only jumps over cells empty in both.
// Row-cooperative: lane L probes mip mu + L, so the climb to the coarsest empty mip is one parallel
// load round trip instead of up to 7 dependent ones; both classifications are loaded unconditionally.
__device__ __forceinline__ bool scan_occupied_2load(V3 p, const uint8_t* bitfield, uint32_t m) {
	const uint32_t i0 = cascaded_grid_idx_at(p, m);
	const float res = scalbnf((float)GRIDSIZE, -(int)m);
	const int ix = (int)floorf(res * (p.x - 0.5f)) + (int)GRIDSIZE / 2;
	const int iy = (int)floorf(res * (p.y - 0.5f)) + (int)GRIDSIZE / 2;
	const int iz = (int)floorf(res * (p.z - 0.5f)) + (int)GRIDSIZE / 2;
	const bool in1 = !(ix < 0 || ix >= (int)GRIDSIZE || iy < 0 || iy >= (int)GRIDSIZE || iz < 0 || iz >= (int)GRIDSIZE);
	const uint32_t i1 = in1 ? morton3D((uint32_t)ix, (uint32_t)iy, (uint32_t)iz) : 0u;
	const uint32_t j0 = i0 == 0xFFFFFFFFu ? 0u : i0;
	const uint8_t b0 = bitfield[j0 / 8 + GRID_N_CELLS * m / 8], b1 = bitfield[i1 / 8 + GRID_N_CELLS * m / 8];
	return (i0 != 0xFFFFFFFFu && (b0 & (1 << (j0 % 8)))) || (in1 && (b1 & (1 << (i1 % 8))));
}

template <uint32_t G>
__device__ float sampling_end_row(V3 o, V3 d, V3 idir, float t_start, const Cone& cone, const Aabb& box, const uint8_t* bitfield,
                                  uint32_t max_cascade, uint32_t L) {
	static_assert(G >= CASCADES || 2 * G == CASCADES, "one lane per mip, or two");
	float tmin, tmax;
	aabb_ray_intersect(box, o, d, &tmin, &tmax);
	if (!(tmax < 3.0e38f)) return t_start;
	const V3 nd = v3(-d.x, -d.y, -d.z), nidir = v3(-idir.x, -idir.y, -idir.z);
	const uint32_t shift = __lane_id() & (64u - G);
	float t = tmax;
	for (int it = 0; it < 8192; ++it) {
		if (t <= t_start) return t_start;
		const V3 p = v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);
		const uint32_t mu = mip_from_dt(calc_dt(t, cone), p, max_cascade);
		const uint32_t mL = mu + L;
		const bool probe = mL < CASCADES;
		const bool occ = probe && scan_occupied_2load(p, bitfield, probe ? mL : 0u);
		uint32_t bits = (uint32_t)(__ballot(occ) >> shift) & ((1u << G) - 1u);
		if (G < CASCADES) {  // lanes probe mips mu + L and mu + L + G
			const bool probe2 = mL + G < CASCADES;
			const bool occ2 = probe2 && scan_occupied_2load(p, bitfield, probe2 ? mL + G : 0u);
			bits |= ((uint32_t)(__ballot(occ2) >> shift) & ((1u << G) - 1u)) << G;
		}
		if (bits & 1u) return t + 2.0f * SQRT3 / scalbnf((float)GRIDSIZE, -(int)mu);
		const uint32_t m = bits ? mu + __builtin_ctz(bits) - 1u : CASCADES - 1u;
		const float res = scalbnf((float)GRIDSIZE, -(int)m);
		t -= distance_to_next_voxel(p, nd, nidir, res);
		t -= fmaxf(fabsf(t), 1.0f) * 2.5e-7f;
	}
	return 3.402823466e38f;
}

// ------------------------------------------------------------------------------------------------
// Ray-parallel marching. The reference marches one ray per thread (testbed_nerf.cu:1432-1480); at
// ~23 K rays per step that is ~1.4 waves per CU and every step of a long ray waits on one dependent
// bitfield load. Here a ray owns a lane group (RG = 8 lanes, half a DPP row): the group speculates the next RG states
// of the reference's sequential march (all occupied: t += calc_dt(t); or all empty:
// advance_to_next_voxel), tests their occupancy in parallel (one load latency per RG states) and
// keeps the prefix that the sequential march would take, switching speculation mode at the first
// lane that disagrees. The t chain itself is evaluated with the reference's float ops in order (every
// lane of the row evaluates it redundantly), so sample positions stay bit-exact with the sequential
// algorithm. The count pass stores the t of every occupied step (tbuf, STEPS floats per ray) and the
// ray geometry, so the write pass is a flat copy instead of a second march.
// ------------------------------------------------------------------------------------------------
#ifndef NGP_SAMPLER_RG
#define NGP_SAMPLER_RG 8
#endif
constexpr uint32_t RG = NGP_SAMPLER_RG;  // lanes per ray (16 = one DPP row)
#ifndef NGP_SAMPLER_EMPTY_SPEC
#define NGP_SAMPLER_EMPTY_SPEC 1  // cone stepping: one guess-and-verify loop for both modes (0: occupied guess-and-verify, empty chain in every lane)
#endif
#ifndef NGP_SAMPLER_ROUND_CAP
#define NGP_SAMPLER_ROUND_CAP 1  // verify rounds per march iteration (0: until every lane is verified)
#endif
#ifndef NGP_SAMPLER_PRIO
#define NGP_SAMPLER_PRIO 3  // s_setprio of the cone-stepping count pass (it shares the SIMDs with the training pass and
                            // is the fox step's critical path): neutral in round 4, fox -1 % since the early counter
                            // publish starts it under the training pass (gpurun_out/r06bl, r06bm)
#endif
#ifndef NGP_SAMPLER_END_CONE
#define NGP_SAMPLER_END_CONE 0  // sampling_end under cone stepping (off: measured slower with the speculative march)
#endif
#ifndef NGP_SAMPLER_UNIFIED0
#define NGP_SAMPLER_UNIFIED0 1  // the same for cone 0 (0: occupied guess-and-verify, empty chain)
#endif

constexpr uint32_t LG = 16;  // lanes per ray in the loss passes: one DPP row
#ifndef NGP_LOSS_PF
#define NGP_LOSS_PF 2  // loss pass 1: chunks of 16 samples whose loads are in flight ahead of the compositing
#endif
#ifndef NGP_LOSS_XCD
#define NGP_LOSS_XCD 1  // loss pass 1 reads its rays on the XCD that wrote their samples (k_loss_pass1)
#endif
#ifndef NGP_LOSS2_LANES
#define NGP_LOSS2_LANES 64  // loss pass 2 with pass 1's kept state: lanes per ray (k_loss_pass2)
#endif
// a ray's lanes must be one wave: lane 0 overwrites numsteps[2i + 1] after every lane has read it in the same
// wave instruction (128 or 256 lanes per ray let a second wave read the overwritten value: wrong samples)
static_assert(NGP_LOSS2_LANES >= 16 && NGP_LOSS2_LANES <= 64, "loss pass 2: at most one wave per ray");
#ifndef NGP_LOSS_SELECT
#define NGP_LOSS_SELECT 1  // loss pass 1: compositing steps committed with selects instead of branches (pass 2
                           // measured slower that way: its steps already run under a per-lane mask)
#endif
#ifndef NGP_LOSS2_PF
#define NGP_LOSS2_PF 1  // loss pass 2: depth 2 takes 86 VGPRs (5 waves/SIMD) and measured 41 -> 45 us (Lego stand-in)
#endif
static_assert(RG >= 4 && RG <= 16 && (RG & (RG - 1)) == 0, "sampler group: 4, 8 or 16 lanes");
#ifndef NGP_SAMPLER_RG0
#define NGP_SAMPLER_RG0 4  // lanes per ray at cone 0 (k_sample_count<true>, the Lego stand-in): 8 -> 4 measured
                           // Lego 0.451-0.453 -> 0.443-0.446 ms per step; the cone-stepping march (fox) stays at
                           // RG (4 there: 0.546 -> 0.605 ms, gpurun_out/r05zzg)
#endif
static_assert(NGP_SAMPLER_RG0 >= 4 && NGP_SAMPLER_RG0 <= 16 && (NGP_SAMPLER_RG0 & (NGP_SAMPLER_RG0 - 1)) == 0,
              "sampler group: 4, 8 or 16 lanes");
template <bool CONE0> constexpr uint32_t sampler_rg() { return CONE0 ? NGP_SAMPLER_RG0 : RG; }
#ifndef NGP_SAMPLER_BLOCK
#define NGP_SAMPLER_BLOCK 256
#endif

template <uint32_t G>
__device__ __forceinline__ uint32_t row_ballot(bool p) {  // this ray's G lanes of a wave ballot
	const unsigned long long b = __ballot(p);
	return (uint32_t)(b >> (__lane_id() & (64u - G))) & ((1u << G) - 1u);
}
__device__ __forceinline__ float dpp_shr1(float v) {  // lane l - 1 of the same DPP row (lane 0 of a row: 0)
	return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));
}
template <int K> __device__ __forceinline__ float row_bcast(float v) {  // v of lane K of this row (row_newbcast)
	return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + K, 0xF, 0xF, false));
}

struct RayGeo {  // per ray, count pass -> write pass
	float o[3], d[3], dn[3];
	float pad[3];
};

// The march's state transitions. CONE0: cone_angle <= 1e-5 (every aabb_scale 1 scene), where
// to/from_stepping_space are t / MIN_CONE_STEPSIZE and back, calc_dt(t) stays within a few ulps of
// MIN_CONE_STEPSIZE (dt * 2 * GRIDSIZE ~ 0.43 < 1), so mip_from_dt(dt, pos) == mip_from_pos(pos);
// with max_cascade 0 that is mip 0. Same values as the generic path, fewer instructions per state.
template <bool CONE0>
struct Marcher {
	V3 o, dn, idir;
	Cone cone;
	uint32_t max_cascade;
	__device__ __forceinline__ V3 pos(float t) const { return v3(o.x + t * dn.x, o.y + t * dn.y, o.z + t * dn.z); }
	__device__ __forceinline__ Cone k() const { return CONE0 ? Cone{} : cone; }
	__device__ __forceinline__ float dt_at(float t) const { return calc_dt(t, k()); }
	__device__ __forceinline__ uint32_t mip_at(float dt, V3 p) const {
		if (CONE0) return max_cascade == 0 ? 0u : mip_from_pos(p, max_cascade);
		return mip_from_dt(dt, p, max_cascade);
	}
	__device__ __forceinline__ float step_occupied(float t) const { return t + dt_at(t); }
	// advance_to_next_voxel from t, sharing to_stepping_space(t) with calc_dt(t) (same values as
	// evaluating both separately); *mip_out: the mip the sampler tests t's occupancy at.
	// In the exponential segment of the stepping space two of the step's four transcendentals only
	// decide integers: the mip (the binary exponent of calc_dt(t) * 2 GRIDSIZE) and the number of
	// stepping-space steps to the next voxel (a ceil). Both are first taken from hardware exp/log
	// (relative error ~1e-6, bound below) and recomputed exactly only when the approximate value lies
	// within a margin (>= 10x that error) of a decision boundary: same integers as the exact evaluation.
	// Both errors grow like 1 / log(1 + cone) (= cone.rl): the margins scale with it, so a small cone
	// (cone_angle_constant down to 1e-5) simply takes the exact path more often, never a wrong integer.
	__device__ __forceinline__ float step_empty(float t, uint32_t* mip_out = nullptr) const {
		return step_empty_n(t, to_stepping_space(t, k()), mip_out);
	}
	// step_empty given n = to(t) (the verify step has it for every candidate)
	__device__ __forceinline__ float step_empty_n(float t, float n, uint32_t* mip_out = nullptr) const {
		const V3 p = pos(t);
		uint32_t mip;
		if (CONE0) {
			mip = mip_at(0.0f, p);
			if (mip_out) *mip_out = mip;
			return advance_to_next_voxel_n(t, n, k(), p, dn, idir, mip);
		}
		const float c = empty_steps(t, n, p, &mip);
		if (mip_out) *mip_out = mip;
		return from_stepping_space(n + c, cone);
	}
	// Cone stepping: the number of stepping-space steps advance_to_next_voxel takes from t (n = to(t),
	// p = pos(t)), ceil(max(to(target) - n, 0.5)), and t's mip.
	__device__ __forceinline__ float empty_steps(float t, float n, V3 p, uint32_t* mip_out) const {
		const float n1 = n + 1.0f;
		float dt;
		if (n1 > cone.a && n1 <= cone.b) {
			// from_stepping_space(n1) = ngp_expf(n1 * log1p_c); __expf: v_exp_f32 (~2 ulp) of
			// the same argument, so dt * 2 GRIDSIZE is off by <= ~3e-7 * t / dt ~ 3e-7 * rl relative
			// (~8e-5 at cone 1/256). Margin: 13x that, relative to the boundary (mantissa 0.5 = powers of two)
			dt = __expf(n1 * cone.log1p_c) - t;
			int e;
			const float mant = frexpf(dt * (2 * GRIDSIZE), &e);
			const float mm = 3.9e-6f * cone.rl;  // 1e-3 at cone 1/256
			if (mant < 0.5f + 0.5f * mm || mant > 1.0f - mm) dt = from_stepping_space(n1, cone) - t;
		} else {
			dt = from_stepping_space(n1, cone) - t;
		}
		const uint32_t mip = mip_at(dt, p);
		*mip_out = mip;
		const float res = scalbnf((float)GRIDSIZE, -(int)mip);
		const float target = t + distance_to_next_voxel(p, dn, idir, res);
		float x;
		if (target > cone.at && target <= cone.bt) {
			// to_stepping_space(target) = ngp_logf(target) / log1p_c; __logf (v_log_f32) is within
			// ~1e-6 absolute for target in (at, bt], i.e. ~1e-6 * rl stepping-space units (~3e-4 at cone
			// 1/256); margin 15x that (4e-3 at cone 1/256; >= 0.5 below cone ~3e-5: always exact)
			x = __logf(target) * cone.rl - n;
			if (fabsf(x - rintf(x)) < 1.5625e-5f * cone.rl) x = to_stepping_space(target, cone) - n;
		} else {
			x = to_stepping_space(target, cone) - n;
		}
		return ceilf(fmaxf(x, 0.5f));
	}
	// Either mode: the state after t and t's mip. occ: t + calc_dt(t) (calc_dt = from(n + 1)
	// - t); empty: advance_to_next_voxel = from(n + empty_steps). One to() and one from() either way, so
	// a wave whose rays are in different modes evaluates the two software transcendentals once.
	__device__ __forceinline__ float step_any(float t, bool occ, uint32_t* mip_out, float* n_out = nullptr) const {
		const V3 p = pos(t);
		const float n = to_stepping_space(t, k());
		if (n_out) *n_out = n;
		uint32_t mip = CONE0 ? mip_at(0.0f, p) : 0u;
		float c = 1.0f;
		if (!occ) c = CONE0 ? empty_steps0(t, n, p, mip) : empty_steps(t, n, p, &mip);
		const float e = from_stepping_space(n + c, k());
		if (!occ) {
			*mip_out = mip;
			return e;
		}
		const float dt = e - t;
		*mip_out = CONE0 ? mip : mip_at(dt, p);
		return t + dt;
	}
	// cone 0: the steps of advance_to_next_voxel_n (mip: mip_at(0, p))
	__device__ __forceinline__ float empty_steps0(float t, float n, V3 p, uint32_t mip) const {
		const float target = t + distance_to_next_voxel(p, dn, idir, scalbnf((float)GRIDSIZE, -(int)mip));
		return ceilf(fmaxf(to_stepping_space(target, Cone{}) - n, 0.5f));
	}
	// Guesses only (the speculative empty-space march verifies every state they lead to): the
	// stepping-space conversions with hardware exp/log in the exponential segment.
	__device__ __forceinline__ float to_fast(float t) const {
		if (t <= cone.at) return div_min_stepsize(t - cone.at) + cone.a;
		if (t <= cone.bt) return __logf(t) * cone.rl;
		return div_max_stepsize(t - cone.bt) + cone.b;
	}
	__device__ __forceinline__ float from_fast(float n) const {
		if (n <= cone.a) return (n - cone.a) * MIN_CONE_STEPSIZE + cone.at;
		if (n <= cone.b) return __expf(n * cone.log1p_c);
		return (n - cone.b) * MAX_CONE_STEPSIZE + cone.bt;
	}
	// Guess of the state j >= 1 empty-space steps after the exact state (tb, nb = to(tb)), assuming each
	// step crosses one voxel boundary at tb's mip: b_j, the j-th boundary crossing of the ray's DDA from
	// pos(tb), then state j = from(nb + ceil(to(b_j) - nb)); returns that ceil (advance_to_next_voxel from inside the cell
	// before b_j lands on the first lattice point past it; nb plus an integer is exact). No dependency
	// between the lanes' guesses; wrong ones (a mip change, two crossings in one step, a tie at a cell
	// corner) only cost a verify round.
	__device__ __forceinline__ float guess_empty_steps(float tb, float nb, uint32_t j) const {
		const V3 p = pos(tb);
		const float res = scalbnf((float)GRIDSIZE, -(int)mip_at(CONE0 ? 0.0f : from_fast(nb + 1.0f) - tb, p));
		const float qx = res * (p.x - 0.5f), qy = res * (p.y - 0.5f), qz = res * (p.z - 0.5f);
		float sx = (floorf(qx + 0.5f + 0.5f * signf_(dn.x)) - qx) * idir.x;
		float sy = (floorf(qy + 0.5f + 0.5f * signf_(dn.y)) - qy) * idir.y;
		float sz = (floorf(qz + 0.5f + 0.5f * signf_(dn.z)) - qz) * idir.z;
		const float ax = fabsf(idir.x), ay = fabsf(idir.y), az = fabsf(idir.z);
		float s = 0.0f;
#pragma unroll
		for (uint32_t k = 0; k + 1 < sampler_rg<CONE0>(); ++k) {
			if (k < j) {
				s = fminf(fminf(sx, sy), sz);
				if (sx == s) sx += ax;
				else if (sy == s) sy += ay;
				else sz += az;
			}
		}
		const float b = tb + fmaxf(s, 0.0f) * (1.0f / res);
		return ceilf(fmaxf((CONE0 ? to_stepping_space(b, Cone{}) : to_fast(b)) - nb, 0.5f));
	}
};

#if NGP_SAMPLER_DIAG == 4  // instrumentation aid: per-ray march statistics (tools/nerf_step_profile.py --sampler-stats)
// [0] empty iterations [1] occupied iterations [2] occupied verify rounds [3] rays [4] occupied states
// [5] max iterations of one ray [6] empty-mode exits (mode switches) [7] empty verify rounds
// [8 + b] rays with 2^b <= iterations < 2^(b+1); wall_clock64 ticks summed over rays: [40] setup_ray
// [41] sampling_end [42] guess + verify [43] occupancy test [44] whole march loop; [45] max ticks of one ray;
// [46] the initial guesses of the unified loop (part of [42])
__device__ unsigned long long g_sampler_stats[48];
extern "C" __attribute__((visibility("default"))) int ngp_debug_sampler_stats(unsigned long long* out, int n) {
	if (!out) {
		static const unsigned long long z[48] = {};
		return hipMemcpyToSymbol(HIP_SYMBOL(g_sampler_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
	}
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sampler_stats), sizeof(unsigned long long) * (n < 48 ? n : 48)) == hipSuccess ? 0 : -1;
}
#define SAMPLER_STAT(...) __VA_ARGS__
// a timestamp the scheduler keeps in program order
__device__ __forceinline__ unsigned long long sampler_clock() {
	__builtin_amdgcn_sched_barrier(0);
	const unsigned long long t = wall_clock64();
	__builtin_amdgcn_sched_barrier(0);
	return t;
}
#else
#define SAMPLER_STAT(...)
#endif

// ngp_debug_math_check: the device forms of the shared math against their reference operations, over whole
// input ranges. which 0: ngp_div_2pf(f) vs the IEEE f / (2 + f) for all 2^23 reduced logf arguments f.
__global__ void k_check_div_2pf(unsigned long long* bad) {
	const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
	if (m >= (1u << 23)) return;
	const float f = __uint_as_float(m + 0x3f3504f3u) - 1.0f;
	const float want = f / (2.0f + f);
	if (__float_as_uint(ngp_div_2pf(f)) != __float_as_uint(want)) atomicAdd(bad, 1ull);
}
extern "C" __attribute__((visibility("default"))) int ngp_debug_math_check(int which, void* stream, uint64_t* mismatches) {
	if (!mismatches || which != 0) return NGP_INVALID;
	hipStream_t s = (hipStream_t)stream;
	unsigned long long* d = nullptr;
	if (hipMallocAsync((void**)&d, 8, s) != hipSuccess) return NGP_ERROR;
	int rc = NGP_OK;
	if (hipMemsetAsync(d, 0, 8, s) != hipSuccess) rc = NGP_ERROR;
	if (rc == NGP_OK) {
		k_check_div_2pf<<<(1u << 23) / 256, 256, 0, s>>>(d);
		if (hipGetLastError() != hipSuccess) rc = NGP_ERROR;
	}
	unsigned long long h = 0;
	if (rc == NGP_OK && hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, s) != hipSuccess) rc = NGP_ERROR;
	if (hipStreamSynchronize(s) != hipSuccess) rc = NGP_ERROR;
	(void)hipFreeAsync(d, s);
	(void)hipStreamSynchronize(s);
	*mismatches = h;
	return rc;
}

// generate_training_samples_nerf pass 1: count the occupied steps of ray i (lane L of its group), keep their t;
// returns the count (uniform over the group).
template <bool CONE0>
__device__ __forceinline__ uint32_t count_ray(const Camera* __restrict__ cams, const uint32_t* __restrict__ pixels, uint32_t n_images,
                                              const ngp_nerf_config& cfg, const SampleArgs& a, uint32_t* __restrict__ nsteps,
                                              float* __restrict__ tbuf, RayGeo* __restrict__ geo, const Cone& cone, uint32_t i,
                                              uint32_t L) {
	constexpr uint32_t RGk = sampler_rg<CONE0>();
	if (!CONE0 && NGP_SAMPLER_PRIO) __builtin_amdgcn_s_setprio(NGP_SAMPLER_PRIO);
	SAMPLER_STAT(const unsigned long long ck0 = sampler_clock();)
	const RaySetup r = setup_ray(cams, pixels, n_images, cfg, i + a.ray_offset, a.n_rays_total_for_image_idx, a.rng, cone);
	SAMPLER_STAT(const unsigned long long ck1 = sampler_clock(); unsigned long long ck2 = ck1, ck_g = 0, ck_o = 0, ck_q = 0;)
	uint32_t j = 0;
	if (r.valid) {
		const Aabb box = cfg_aabb(cfg);
		const Marcher<CONE0> m{r.o, r.dn, r.idir, cone, cfg.max_cascade};
		float t = r.startt;
#if NGP_SAMPLER_DIAG == 2
		const float t_end = 3.0e38f;
#else
		// Under cone stepping the speculative march crosses trailing empty space faster than the backward
		// scan finds its start (fox: 0.356 ms with it, 0.334 without, profiles/r03ak); at cone 0 it pays.
		const float t_end = (CONE0 || NGP_SAMPLER_END_CONE)
		                        ? sampling_end_row<RGk>(r.o, r.dn, r.idir, t, m.cone, box, a.bitfield, cfg.max_cascade, L)
		                        : 3.0e38f;
#endif
#if NGP_SAMPLER_DIAG == 1  // timing aid: sampling_end twice (cost of one = difference to the default build)
		const float t_end2 = sampling_end_row<RGk>(r.o, r.dn, r.idir, t + 0.0f * t_end, m.cone, box, a.bitfield, cfg.max_cascade, L);
		if (t_end2 != t_end) t = t_end2;
#endif
		float* tout = tbuf + (size_t)i * STEPS;
		bool occ_mode = false;  // rays enter the aabb in empty space far more often than not
		bool have_n0 = false;   // unified loop: n0_next = to(t) is known (the verify step computed it for the new state)
		float n0_next = 0.f;
		SAMPLER_STAT(ck2 = sampler_clock();)
		SAMPLER_STAT(uint32_t st_e = 0; uint32_t st_o = 0; uint32_t st_r = 0; uint32_t st_x = 0; uint32_t st_q = 0;)
		for (;;) {
			SAMPLER_STAT(if (occ_mode) ++st_o; else ++st_e; const unsigned long long cka = sampler_clock();)
			// lanes [0, nvalid) take the next nvalid states of the sequential march, assuming it stays in
			// the current mode (all occupied / all empty)
			float tl, last;  // last: the state after lane nvalid-1's (the march continues there if every lane stays in the mode)
			uint32_t mipl;   // the mip lane L's state is tested at
			float nk = 0.f;  // unified loop: to(tl), from its verify step (reused when the ray leaves an occupied run at this lane)
			uint32_t nvalid = RGk;  // lanes holding verified states
			if (CONE0 ? NGP_SAMPLER_UNIFIED0 : NGP_SAMPLER_EMPTY_SPEC) {
				// Both modes in one guess-and-verify loop. Every state is from(n + c) with n =
				// to(previous state): c = 1 in an occupied run (t + calc_dt(t)), c = the ceil of
				// advance_to_next_voxel in an empty one. Lane L guesses state L as from(to(t) + C_L): C_L = L
				// when occupied (to(from(n)) == n nearly always), the voxel DDA's estimate when empty
				// (guess_empty_steps). All lanes verify at once: lane L redoes the exact step from lane L-1's
				// guess. The verified prefix is exact; the first lane that fails takes the exact state from its
				// predecessor and the lanes after it are re-guessed from there. The rays of a wave sit in
				// different modes most of the time; sharing the loop (and its exact to()/from() per lane and
				// round) means the wave no longer runs one mode's loop after the other's.
				const float n0 = have_n0 ? n0_next : to_stepping_space(t, m.k());
				have_n0 = false;
				const float c0 = occ_mode ? (float)L : m.guess_empty_steps(t, n0, L);
				float cand = L == 0 ? t : from_stepping_space(n0 + c0, m.k());
				SAMPLER_STAT(ck_q += sampler_clock() - cka;)
				uint32_t v0 = 1, mk = 0, rounds = 0;
				float nxt, tcap = 0.0f;
				for (;;) {
					SAMPLER_STAT(if (occ_mode) ++st_r; else ++st_q;)
					nxt = m.step_any(cand, occ_mode, &mk, &nk);
					const float expct = dpp_shr1(nxt);
					const uint32_t v = __builtin_ctz(row_ballot<RGk>(L >= v0 && __float_as_uint(expct) != __float_as_uint(cand)) | (1u << RGk));
					if (v >= RGk) break;
					const float tv = __shfl(expct, (int)v, (int)RGk);
					// The wave runs the loop until its slowest ray is verified. After NGP_SAMPLER_ROUND_CAP rounds a
					// ray keeps its verified prefix (lanes < v) and continues from tv (the exact state after it)
					// in the next iteration.
					if (NGP_SAMPLER_ROUND_CAP && ++rounds >= NGP_SAMPLER_ROUND_CAP) {
						nvalid = v;
						tcap = tv;
						break;
					}
					const float nv = to_stepping_space(tv, m.k());
					const float cv = occ_mode ? (float)(L - v) : m.guess_empty_steps(tv, nv, L - v);
					cand = L < v ? cand : (L == v ? tv : from_stepping_space(nv + cv, m.k()));
					v0 = v + 1;
				}
				tl = cand;
				mipl = mk;
				last = __shfl(nxt, (int)(RGk - 1), (int)RGk);
				if (nvalid < RGk) last = tcap;
			} else if (occ_mode) {
				// Occupied run: t_{k+1} = t_k + calc_dt(t_k) = from(to(t_k) + 1) in stepping space, and
				// to(from(n)) == n nearly always. Guess state L as from(to(t) + L) and verify every guess at
				// once (lane L redoes the exact step from lane L-1's state): the verified prefix is exact; the
				// first lane that fails takes the exact state from its verified predecessor and the lanes
				// after it are re-guessed from there. Each round verifies at least one more lane, most runs
				// take one round instead of a chain of RGk dependent steps.
				const float n0 = to_stepping_space(t, m.k());
				float cand = L == 0 ? t : from_stepping_space(n0 + (float)L, m.k());
				uint32_t v0 = 1;
				float dt, nxt;
				for (;;) {
					SAMPLER_STAT(++st_r;)
					dt = m.dt_at(cand);
					nxt = cand + dt;  // step_occupied(cand)
					const float expct = dpp_shr1(nxt);
					const uint32_t v = __builtin_ctz(row_ballot<RGk>(L >= v0 && __float_as_uint(expct) != __float_as_uint(cand)) | (1u << RGk));
					if (v >= RGk) break;
					const float tv = __shfl(expct, (int)v, (int)RGk);
					cand = L < v ? cand : (L == v ? tv : from_stepping_space(to_stepping_space(tv, m.k()) + (float)(L - v), m.k()));
					v0 = v + 1;
				}
				tl = cand;
				mipl = m.mip_at(CONE0 ? 0.0f : dt, m.pos(tl));
				last = __shfl(nxt, (int)(RGk - 1), (int)RGk);
			} else {
				// empty space: the chain evaluated in order by every lane of the group; lane L keeps state L
				float tk = t;
				tl = t;
				mipl = 0;
#pragma unroll 1  // rolled: the unrolled chain (8 inlined steps) overflowed the instruction cache
				for (uint32_t kk = 0; kk < RGk; ++kk) {
					uint32_t mk;
					const float tn = m.step_empty(tk, &mk);
					if (L == kk) { tl = tk; mipl = mk; }
					tk = tn;
				}
				last = tk;
			}
			SAMPLER_STAT(const unsigned long long ckb = sampler_clock(); ck_g += ckb - cka;)
			const V3 pos = m.pos(tl);
			const uint32_t mip = mipl;
			const bool inside = L < nvalid && tl <= t_end && aabb_contains(box, pos) && (occ_mode ? j + L : j) < STEPS;
			const bool occ = inside && density_grid_occupied_at(pos, a.bitfield, mip);
			const uint32_t cont = row_ballot<RGk>(inside && occ == occ_mode);
			const uint32_t f = __builtin_ctz(~cont | (1u << RGk));  // first lane the sequential march leaves the mode at
			SAMPLER_STAT(ck_o += sampler_clock() - ckb;)
			if (occ_mode) {
#if NGP_SAMPLER_DIAG == 5  // timing aid: every occupied state stored twice (mirrored copy; cost of the stores)
				if (L < f) { tout[j + L] = tl; tout[STEPS - 1 - (j + L)] = tl; }
#else
				if (L < f) tout[j + L] = tl;
#endif
				j += f;
			}
			if (f >= nvalid) {  // every state taken stayed in the mode: continue after the last one
				t = last;
				continue;
			}
			if (!((row_ballot<RGk>(inside) >> f) & 1u)) break;  // left the aabb / sampling range / step budget
			const float tf = __shfl(tl, (int)f, (int)RGk);
			if (occ_mode) {  // empty cell at lane f: advance_to_next_voxel
				// cone stepping: lane f's to() from its verify step (at cone 0 to() is a multiply, cheaper than the shuffle)
				if (!CONE0 && NGP_SAMPLER_EMPTY_SPEC) t = m.step_empty_n(tf, __shfl(nk, (int)f, (int)RGk));
				else t = m.step_empty(tf);
			}
			else {  // occupied cell at lane f: sample it next
				t = tf;
				if (!CONE0 && NGP_SAMPLER_EMPTY_SPEC) {
					n0_next = __shfl(nk, (int)f, (int)RGk);
					have_n0 = true;
				}
			}
			SAMPLER_STAT(st_x += occ_mode ? 0u : 1u;)
			occ_mode = !occ_mode;
		}
		SAMPLER_STAT(if (L == 0) {
			atomicAdd(&g_sampler_stats[0], (unsigned long long)st_e);
			atomicAdd(&g_sampler_stats[1], (unsigned long long)st_o);
			atomicAdd(&g_sampler_stats[2], (unsigned long long)st_r);
			atomicAdd(&g_sampler_stats[3], 1ull);
			atomicAdd(&g_sampler_stats[4], (unsigned long long)j);
			atomicMax(&g_sampler_stats[5], (unsigned long long)(st_e + st_o));
			atomicAdd(&g_sampler_stats[6], (unsigned long long)st_x);
			atomicAdd(&g_sampler_stats[7], (unsigned long long)st_q);
			atomicAdd(&g_sampler_stats[8 + (31 - __builtin_clz(st_e + st_o))], 1ull);
			const unsigned long long ck3 = sampler_clock();
			atomicAdd(&g_sampler_stats[40], ck1 - ck0);
			atomicAdd(&g_sampler_stats[41], ck2 - ck1);
			atomicAdd(&g_sampler_stats[42], ck_g);
			atomicAdd(&g_sampler_stats[43], ck_o);
			atomicAdd(&g_sampler_stats[44], ck3 - ck2);
			atomicMax(&g_sampler_stats[45], ck3 - ck0);
			atomicAdd(&g_sampler_stats[46], ck_q);
		})
	}
	if (L == 0) {
		nsteps[i] = j;
		RayGeo g;
		g.o[0] = r.o.x; g.o[1] = r.o.y; g.o[2] = r.o.z;
		g.d[0] = r.d.x; g.d[1] = r.d.y; g.d[2] = r.d.z;
		g.dn[0] = r.dn.x; g.dn[1] = r.dn.y; g.dn[2] = r.dn.z;
		g.pad[0] = r.cone; g.pad[1] = g.pad[2] = 0.f;
		geo[i] = g;
	}
	return j;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
	return v;
}

// The count pass, and per wave the sum of its rays' counts and the number of its rays with samples (wsum[2 w],
// wsum[2 w + 1]): the sampler's prefix sums over rays become a scan over waves (k_sample_bscan, ~2 K values at
// the Lego stand-in's ~32 K rays) plus an in-wave prefix in k_sample_write, instead of a scan over the rays.
template <bool CONE0>
__global__ void __launch_bounds__(256) k_sample_count(const Camera* __restrict__ cams, const uint32_t* __restrict__ pixels,
                                                      uint32_t n_images, const ngp_nerf_config cfg, SampleArgs a,
                                                      uint32_t* __restrict__ nsteps, float* __restrict__ tbuf,
                                                      RayGeo* __restrict__ geo, const Cone cone, uint32_t* __restrict__ wsum) {
	constexpr uint32_t RGk = sampler_rg<CONE0>();
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t i = gid / RGk, L = gid % RGk;
	const bool live = i < a.n_rays;  // whole rows
	uint32_t j = 0;
	if (live) j = count_ray<CONE0>(cams, pixels, n_images, cfg, a, nsteps, tbuf, geo, cone, i, L);
	const bool head = live && L == 0;
	const uint32_t sum = wave_sum(head ? j : 0u);
	const uint32_t nz = (uint32_t)__popcll(__ballot(head && j > 0));
	if ((threadIdx.x & 63) == 0) {
		const uint32_t w = gid / 64;
		wsum[2 * w] = sum;
		wsum[2 * w + 1] = nz;
	}
}

// pass 2: write the ray records and the NerfCoordinates of kept rays from the stored t values; one
// wave per ray (most rays take one or two iterations, consecutive lanes write consecutive samples).
constexpr uint32_t WG = 64;
#ifndef NGP_SW_STAGE
#define NGP_SW_STAGE 1  // records staged in LDS, written as contiguous wave stores
#endif
// pass 2: write the ray records and the NerfCoordinates of kept rays from the stored t values.
// The ray's sample base (exclusive prefix of the counts, the reference's atomicAdd on numsteps_counter in ray order)
// and its slot among the kept rays: bpre (the count wave's prefixes, k_sample_bscan) plus the prefix over the
// rays of its count wave before it (rpw rays per count wave). A ray is kept when it has samples and they fit
// under max_samples (testbed_nerf.cu:1616-1619); the inclusive prefix grows with the ray index, so the kept
// rays are the rays with samples before the first that does not fit, and a kept ray's slot counts every ray
// with samples before it.
__global__ void __launch_bounds__(256) k_sample_write(const ngp_nerf_config cfg, SampleArgs a, const uint32_t* __restrict__ nsteps,
                                                      const uint32_t* __restrict__ bpre, uint32_t rpw, const float* __restrict__ tbuf,
                                                      const RayGeo* __restrict__ geo, const Cone cone) {
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t i = gid / WG, L = gid % WG;
	if (i >= a.n_rays) return;  // whole waves
	const uint32_t w = i / rpw, r0 = w * rpw;
	const uint32_t nl = (r0 + L < i) ? nsteps[r0 + L] : 0u;  // the count wave's rays before ray i
	const uint32_t before = wave_sum(nl);
	const uint32_t nz_before = (uint32_t)__popcll(__ballot(nl > 0));
	const uint32_t numsteps = nsteps[i], b = bpre[2 * w] + before;
	if (numsteps == 0 || b + numsteps > a.max_samples) return;
	const uint32_t s = bpre[2 * w + 1] + nz_before;
	const RayGeo g = geo[i];
	if (L == 0) {
		a.ray_indices[s] = i + a.ray_offset;
		float* ro = a.rays + (size_t)s * 6;
		ro[0] = g.o[0]; ro[1] = g.o[1]; ro[2] = g.o[2]; ro[3] = g.d[0]; ro[4] = g.d[1]; ro[5] = g.d[2];
		a.numsteps[2 * s] = numsteps;
		a.numsteps[2 * s + 1] = b;
	}
	const Aabb box = cfg_aabb(cfg);
	const V3 diag = v3(box.mx.x - box.mn.x, box.mx.y - box.mn.y, box.mx.z - box.mn.z);
	const V3 wdir = v3((g.dn[0] + 1.0f) * 0.5f, (g.dn[1] + 1.0f) * 0.5f, (g.dn[2] + 1.0f) * 0.5f);
	const float* tin = tbuf + (size_t)i * STEPS;
#if NGP_SW_STAGE
	// a wave's 64 records (7 floats each, 28-B stride) are staged in LDS and written back as 7 contiguous
	// 256-B wave stores instead of 7 stores that each touch 14 lines
	__shared__ float stage[256 / WG][WG * 7];
	float* st = stage[threadIdx.x / WG];
	for (uint32_t j0 = 0; j0 < numsteps; j0 += WG) {
		const uint32_t jj = j0 + L;
		if (jj < numsteps) {
			const float t = tin[jj];
			const V3 pos = v3(g.o[0] + t * g.dn[0], g.o[1] + t * g.dn[1], g.o[2] + t * g.dn[2]);
			const float dt = calc_dt(t, cone);
			float* c = st + L * 7;  // stride 7 words: conflict-free
			c[0] = (pos.x - box.mn.x) / diag.x; c[1] = (pos.y - box.mn.y) / diag.y; c[2] = (pos.z - box.mn.z) / diag.z;
			c[3] = warp_dt(dt);
			c[4] = wdir.x; c[5] = wdir.y; c[6] = wdir.z;
		}
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		const uint32_t nf = min(WG, numsteps - j0) * 7;
		float* dst = a.coords + (size_t)(b + j0) * 7;
#pragma unroll
		for (uint32_t k = 0; k < 7; ++k)
			if (L + k * WG < nf) dst[L + k * WG] = st[L + k * WG];
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	}
#else
	for (uint32_t jj = L; jj < numsteps; jj += WG) {
		const float t = tin[jj];
		const V3 pos = v3(g.o[0] + t * g.dn[0], g.o[1] + t * g.dn[1], g.o[2] + t * g.dn[2]);
		const float dt = calc_dt(t, cone);
		float* c = a.coords + (size_t)(b + jj) * 7;
		c[0] = (pos.x - box.mn.x) / diag.x; c[1] = (pos.y - box.mn.y) / diag.y; c[2] = (pos.z - box.mn.z) / diag.z;
		c[3] = warp_dt(dt);
		c[4] = wdir.x; c[5] = wdir.y; c[6] = wdir.z;
	}
#endif
}

// Single-workgroup scans of one step's per-wave / per-group sums (the sampler's count waves, the loss's groups of
// 4 rays: ~2-8 K values at ~32 K rays): one launch of 1024 threads, tiles of 4096 values, 4 consecutive ones per
// thread (16-B coalesced loads and stores), one block scan per tile. Round 6: they replaced scans over every
// ray (one single-block scan of up to 8 tiles, or above 32 K rays a device-wide hipcub scan: 2 launches per
// scan, and 3 scans per step).
constexpr uint32_t SCAN1_THREADS = 1024, SCAN1_TILE = 4 * SCAN1_THREADS;
// exclusive sum of one value per thread over the block, and the block total; lds: 32 words
__device__ __forceinline__ uint32_t block_exclusive_sum(uint32_t v, uint32_t* lds, uint32_t* total) {
	constexpr uint32_t NW = SCAN1_THREADS / 64;
	const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	uint32_t x = v;
#pragma unroll
	for (uint32_t d = 1; d < 64; d <<= 1) {
		const uint32_t y = __shfl_up(x, d, 64);
		if (lane >= d) x += y;
	}
	if (lane == 63) lds[w] = x;
	__syncthreads();
	if (w == 0) {
		uint32_t y = lane < NW ? lds[lane] : 0u;
#pragma unroll
		for (uint32_t d = 1; d < NW; d <<= 1) {
			const uint32_t z = __shfl_up(y, d, 64);
			if (lane >= d) y += z;
		}
		if (lane < NW) lds[NW + lane] = y;  // inclusive
	}
	__syncthreads();
	const uint32_t r = (w ? lds[NW + w - 1] : 0u) + x - v;
	*total = lds[2 * NW - 1];
	__syncthreads();
	return r;
}
__device__ __forceinline__ void scan1_load(const uint32_t* in, uint32_t n, uint32_t i, uint32_t v[4]) {
	if (i + 3 < n && ((uintptr_t)in & 15) == 0) {
		const uint4 q = *(const uint4*)(in + i);
		v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
	} else {
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) v[k] = i + k < n ? in[i + k] : 0u;
	}
}
__device__ __forceinline__ void scan1_store(uint32_t* out, uint32_t n, uint32_t i, const uint32_t v[4]) {
	if (i + 3 < n && ((uintptr_t)out & 15) == 0) {
		*(uint4*)(out + i) = uint4{v[0], v[1], v[2], v[3]};
	} else {
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k)
			if (i + k < n) out[i + k] = v[k];
	}
}
// Exclusive prefix sums of the sums of groups of 4 consecutive values (gpre[g] = in[0] + .. + in[4 g - 1]) and the
// total, one block: a quarter of the block scans of a per-element scan (the loss's compaction: ~32 K rays, two
// tiles instead of eight); a consumer adds the at most 3 values of its group before it.
__global__ void __launch_bounds__(SCAN1_THREADS) k_scan4(uint32_t n, const uint32_t* __restrict__ in, uint32_t* __restrict__ gpre,
                                                         uint32_t* __restrict__ total, const uint32_t* __restrict__ ray_counter,
                                                         volatile uint32_t* pub_host, uint32_t pub_seq) {
	__shared__ uint32_t lds[32];
	const uint32_t ng = (n + 3) / 4;
	uint32_t run = 0;
	for (uint32_t g0 = 0; g0 < ng; g0 += SCAN1_TILE) {
		uint32_t gs[4];
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			uint32_t v[4];
			scan1_load(in, n, 4 * (g0 + 4 * threadIdx.x + k), v);
			gs[k] = v[0] + v[1] + v[2] + v[3];
		}
		uint32_t tot;
		uint32_t b = run + block_exclusive_sum(gs[0] + gs[1] + gs[2] + gs[3], lds, &tot);
		uint32_t o[4];
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			o[k] = b;
			b += gs[k];
		}
		scan1_store(gpre, ng, g0 + 4 * threadIdx.x, o);
		run += tot;
	}
	if (threadIdx.x == 0) {
		*total = run;
		if (pub_host) {  // LossArgs::pub_host: the step's counters are final here
			pub_host[0] = ray_counter[0]; pub_host[1] = ray_counter[1]; pub_host[2] = run; pub_host[3] = 0u;
			__threadfence_system();
			pub_host[4] = pub_seq;
		}
	}
}
// The count waves' exclusive prefixes (bpre[2 w]: samples before wave w, bpre[2 w + 1]: rays with samples
// before it) from their sums, one block; and the counters: rays kept, and the total count of every ray (the
// reference's numsteps_counter, dropped rays included). The one wave whose rays cross max_samples is found
// here and its rays counted in order.
__global__ void __launch_bounds__(SCAN1_THREADS) k_sample_bscan(uint32_t nw, const uint32_t* __restrict__ wsum, uint32_t* __restrict__ bpre,
                                                                const uint32_t* __restrict__ nsteps, uint32_t n_rays, uint32_t rpw,
                                                                uint32_t max_samples, uint32_t* __restrict__ counters) {
	__shared__ uint32_t lds[32];
	__shared__ uint32_t cross[3];  // the crossing wave, its prefixes
	if (threadIdx.x == 0) cross[0] = nw;
	uint32_t run_s = 0, run_z = 0;
	for (uint32_t t0 = 0; t0 < nw; t0 += SCAN1_TILE) {
		uint32_t sv[4], zv[4];
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			const uint32_t w = t0 + 4 * threadIdx.x + k;
			sv[k] = w < nw ? wsum[2 * w] : 0u;
			zv[k] = w < nw ? wsum[2 * w + 1] : 0u;
		}
		uint32_t ts, tz;
		uint32_t bs = run_s + block_exclusive_sum(sv[0] + sv[1] + sv[2] + sv[3], lds, &ts);
		uint32_t bz = run_z + block_exclusive_sum(zv[0] + zv[1] + zv[2] + zv[3], lds, &tz);
#pragma unroll
		for (uint32_t k = 0; k < 4; ++k) {
			const uint32_t w = t0 + 4 * threadIdx.x + k;
			if (w < nw) {
				bpre[2 * w] = bs;
				bpre[2 * w + 1] = bz;
				if (bs <= max_samples && bs + sv[k] > max_samples) {  // at most one wave
					cross[0] = w; cross[1] = bs; cross[2] = bz;
				}
			}
			bs += sv[k];
			bz += zv[k];
		}
		run_s += ts;
		run_z += tz;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t kept = run_z;
		if (cross[0] < nw) {
			uint32_t b = cross[1];
			kept = cross[2];
			for (uint32_t r = cross[0] * rpw; r < min(n_rays, (cross[0] + 1) * rpw); ++r) {
				const uint32_t n = nsteps[r];
				if (b + n > max_samples) break;
				kept += n > 0 ? 1u : 0u;
				b += n;
			}
		}
		counters[0] = kept;
		counters[1] = run_s;
	}
}

size_t sample_tmp_f32(uint32_t n_rays) { return (size_t)n_rays * (STEPS + sizeof(RayGeo) / 4); }

// count waves of the sampler's count pass: whole blocks of NGP_SAMPLER_BLOCK threads, RGk lanes per ray
static uint32_t sample_count_waves(uint32_t n_rays, uint32_t rgk) {
	return (uint32_t)(div_round_up((size_t)n_rays * rgk, NGP_SAMPLER_BLOCK) * (NGP_SAMPLER_BLOCK / 64));
}
size_t sample_tmp_u32(uint32_t n_rays) { return n_rays + 4 * (size_t)sample_count_waves(n_rays, std::max(RG, sampler_rg<true>())); }

void sample_rays(const Dataset& ds, const ngp_nerf_config& cfg, const SampleArgs& a, uint32_t* tmp, float* tmpf, hipStream_t s) {
	if (a.n_rays == 0) return;
	NGP_CHECK(tmpf != nullptr, "sample_rays: float scratch of sample_tmp_f32(n_rays) floats required");
	const bool cone0 = cfg.cone_angle_constant <= 1e-5f;
	const uint32_t rgk = cone0 ? sampler_rg<true>() : RG;
	const uint32_t nw = sample_count_waves(a.n_rays, rgk);
	uint32_t* nsteps = tmp;
	uint32_t* wsum = tmp + a.n_rays;    // 2 per count wave
	uint32_t* bpre = wsum + 2 * (size_t)nw;
	float* tbuf = tmpf;
	RayGeo* geo = (RayGeo*)(tmpf + (size_t)a.n_rays * STEPS);
	const uint32_t blocks = div_round_up((size_t)a.n_rays * RG, NGP_SAMPLER_BLOCK);
	const uint32_t blocks0 = div_round_up((size_t)a.n_rays * sampler_rg<true>(), NGP_SAMPLER_BLOCK);
	const Cone cone = make_cone(cfg.cone_angle_constant);  // every ray's cone (setup_ray: r.cone)
	{
		ProfScope ps("sample_count", s);
		if (cone0)
			k_sample_count<true><<<blocks0, NGP_SAMPLER_BLOCK, 0, s>>>(ds.d_cams, ds.d_pixels, ds.n_images, cfg, a, nsteps, tbuf, geo, cone,
			                                                          wsum);
		else
			k_sample_count<false><<<blocks, NGP_SAMPLER_BLOCK, 0, s>>>(ds.d_cams, ds.d_pixels, ds.n_images, cfg, a, nsteps, tbuf, geo, cone,
			                                                           wsum);
		NGP_HIP(hipGetLastError());
	}
	NGP_CHECK(nw == (cone0 ? blocks0 : blocks) * (NGP_SAMPLER_BLOCK / 64) && 64 % rgk == 0, "sampler: count waves");
	{
		ProfScope ps("sample_scans", s);
		k_sample_bscan<<<1, SCAN1_THREADS, 0, s>>>(nw, wsum, bpre, nsteps, a.n_rays, 64 / rgk, a.max_samples, a.counters);
		NGP_HIP(hipGetLastError());
	}
	ProfScope ps("sample_write", s);
	k_sample_write<<<div_round_up((size_t)a.n_rays * WG, 256), 256, 0, s>>>(cfg, a, nsteps, bpre, 64 / rgk, tbuf, geo, cone);
	NGP_HIP(hipGetLastError());
}


// ------------------------------------------------------------------------------------------------
// compute_loss_kernel_train_nerf (testbed_nerf.cu:1660-2012), split at its atomicAdd into two passes
// around a prefix scan. The error map deposit (:1869-1899, always on in the reference's training) is
// done in pass 2 after the compaction early-out, as there; sharpness / envmap / exposure / depth
// supervision are off in the reference's default training and not implemented.
// A ray owns one DPP row: lanes load and activate 16 samples at once (network output, dt, exp), and
// the compositing recurrence (T *= 1 - alpha, rgb += alpha T c) runs over the row in sample order
// with row_newbcast broadcasts, i.e. with the reference's float ops in the reference's order.
// ------------------------------------------------------------------------------------------------
struct LossRay {  // pass-1 results kept for pass 2
	float grad[3];
	float rgb_ray[3];
	float mean_loss;
	float u, v;    // the ray's image position and image (the error map deposit)
	uint32_t img;
	float pad[2];
};

__device__ __forceinline__ V3 unwarp_pos(const float* c, const Aabb& b) {
	return v3(b.mn.x + c[0] * (b.mx.x - b.mn.x), b.mn.y + c[1] * (b.mx.y - b.mn.y), b.mn.z + c[2] * (b.mx.z - b.mn.z));
}

#define NGP_ROW_UNROLL16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

__global__ void __launch_bounds__(256) k_loss_pass1(const Camera* __restrict__ cams, const uint32_t* __restrict__ pixels,
                                                    uint32_t n_images, const ngp_nerf_config cfg, LossArgs a,
                                                    uint32_t* __restrict__ craw, LossRay* __restrict__ lr) {
	// XCD-aware ray order (NGP_LOSS_XCD): the block on XCD x = blockIdx % 8 takes the rays whose samples
	// k_sample_write wrote from XCD x (a wave per ray there: ray i on XCD (i / 4) % 8), so their coordinates
	// can still be in that XCD's L2: rays 128 m + 32 q + 4 x + j (q, j in 0..3) for block 8 m + x
	uint32_t i;
	const uint32_t L = threadIdx.x % LG;
	if (NGP_LOSS_XCD) {
		const uint32_t m = blockIdx.x / 8, x = blockIdx.x % 8, r = threadIdx.x / LG;
		i = 128 * m + 32 * (r / 4) + 4 * x + (r % 4);
	} else {
		i = (blockIdx.x * blockDim.x + threadIdx.x) / LG;
	}
	if (i >= a.n_rays) return;
	if (L == 0 && a.zero_loss && a.loss) a.loss[i] = 0.0f;  // pass 2 writes the compacted rays' loss after it
	if (i >= *a.ray_counter) { if (L == 0) craw[i] = 0; return; }
	const uint32_t numsteps = a.numsteps[2 * i], base = a.numsteps[2 * i + 1];
	const f16* out = a.network_output + (size_t)base * a.out_stride;
	const float* ci = a.coords_in + (size_t)base * 7;
	// target texel first (same random stream as the sampler for the same ray): its dependent chain of
	// loads (ray index -> camera -> pixel) overlaps the compositing loop instead of following it
	const uint32_t ray_idx = a.ray_indices[i];
	Rng rng = a.rng;
	pcg_advance(rng, (uint64_t)ray_idx * N_MAX_RANDOM_SAMPLES_PER_RAY);
	const uint32_t img = image_idx(ray_idx, a.n_rays_total_for_image_idx, n_images);
	const Camera& cam = cams[img];
	float u, v;
	random_image_pos(rng, cam.width, cam.height, cfg.snap_to_pixel_centers != 0, &u, &v);
	pcg_advance(rng, 1);  // motionblur_time
	// The per-ray colour work (12 powf in the default configuration) is split over the row: lane ch < 3
	// finishes colour channel ch with the reference's per-channel operations, and lane 0 gathers the
	// three results (the other lanes repeat channel 2).
	const uint32_t ch = L < 3 ? L : 2;
	float bg[3] = {cfg.background_color[0], cfg.background_color[1], cfg.background_color[2]};
	if (cfg.random_bg_color) { bg[0] = pcg_float(rng); bg[1] = pcg_float(rng); bg[2] = pcg_float(rng); }
	float bgc = srgb_to_linear(ch == 0 ? bg[0] : ch == 1 ? bg[1] : bg[2]);
	// read_rgba, Byte images (common_device.cuh:885-904)
	const uint32_t raw = pixels[cam.pixel_offset + pixel_index(u, v, cam.width, cam.height)];
	float t = 1.f;
	const float eps = 1e-4f;
	float rr = 0.f, rg = 0.f, rb = 0.f;
	uint32_t cn = 0;
	bool stop = false;
	const bool keep_state = NGP_LOSS_SELECT && a.state != nullptr;
	// software pipelining: the loads of the next NGP_LOSS_PF chunks are in flight while a chunk's
	// compositing chain runs (the chunk loop is unrolled by the depth, so every buffer keeps its registers)
	f16x4 ob[NGP_LOSS_PF];
	float db[NGP_LOSS_PF];
#pragma unroll
	for (uint32_t d = 0; d < NGP_LOSS_PF; ++d) {
		ob[d] = f16x4{(f16)0.f, (f16)0.f, (f16)0.f, (f16)0.f};
		db[d] = 0.f;
		if (L + d * LG < numsteps) {
			ob[d] = *(const f16x4*)(out + (size_t)(L + d * LG) * a.out_stride);
			db[d] = ci[(size_t)(L + d * LG) * 7 + 3];
		}
	}
	for (uint32_t c0 = 0; c0 < numsteps && !stop; c0 += NGP_LOSS_PF * LG)
#pragma unroll
	for (uint32_t d = 0; d < NGP_LOSS_PF; ++d) {
		const uint32_t c = c0 + d * LG;
		if (c >= numsteps || stop) break;
		const uint32_t jj = c + L;
		const f16x4 o = ob[d];
		const float dtw = db[d];
		if (jj + NGP_LOSS_PF * LG < numsteps) {
			ob[d] = *(const f16x4*)(out + (size_t)(jj + NGP_LOSS_PF * LG) * a.out_stride);
			db[d] = ci[(size_t)(jj + NGP_LOSS_PF * LG) * 7 + 3];
		}
		float alpha = 0.f, cr = 0.f, cg = 0.f, cb = 0.f;
		if (jj < numsteps) {
			const float dt = unwarp_dt(dtw);
			const float density = network_to_density((float)o[3], cfg.density_activation);
			alpha = 1.f - ngp_expf_fast(-density * dt);
			cr = network_to_rgb((float)o[0], cfg.rgb_activation);
			cg = network_to_rgb((float)o[1], cfg.rgb_activation);
			cb = network_to_rgb((float)o[2], cfg.rgb_activation);
		}
#if NGP_LOSS_SELECT
		// branch-free step: the same operations, committed with selects (no exec-mask branch per sample)
#define NGP_LOSS1_STEP(K)                                                                              \
		{                                                                                              \
			const float ak = row_bcast<K>(alpha), rk = row_bcast<K>(cr), gk = row_bcast<K>(cg), bk = row_bcast<K>(cb); \
			const bool act = !stop && c + K < numsteps;                                                \
			const bool low = t < eps;                                                                  \
			stop = stop || (act && low);                                                               \
			const bool upd = act && !low;                                                              \
			const float weight = ak * t;                                                               \
			const float nr = rr + weight * rk, ng = rg + weight * gk, nb = rb + weight * bk;           \
			const float nt = t * (1.f - ak);                                                           \
			rr = upd ? nr : rr; rg = upd ? ng : rg; rb = upd ? nb : rb; t = upd ? nt : t;              \
			cn += upd ? 1u : 0u;                                                                       \
			if (keep_state && L == K) { sw = weight; sT = nt; sr = nr; sg = ng; sb = nb; su = upd; }   \
		}
#else
#define NGP_LOSS1_STEP(K)                                                                              \
		{                                                                                              \
			const float ak = row_bcast<K>(alpha), rk = row_bcast<K>(cr), gk = row_bcast<K>(cg), bk = row_bcast<K>(cb); \
			if (!stop && c + K < numsteps) {                                                           \
				if (t < eps) stop = true;                                                              \
				else {                                                                                 \
					const float weight = ak * t;                                                       \
					rr += weight * rk; rg += weight * gk; rb += weight * bk;                           \
					t *= (1.f - ak);                                                                   \
					++cn;                                                                              \
				}                                                                                      \
			}                                                                                          \
		}
#endif
		float sw = 0.f, sT = 0.f, sr = 0.f, sg = 0.f, sb = 0.f;
		bool su = false;
		NGP_ROW_UNROLL16(NGP_LOSS1_STEP)
#undef NGP_LOSS1_STEP
		if (keep_state && su && (size_t)base + jj < a.state_cap) {  // composited: pass 2 reads its state instead of compositing again
			const size_t si = (size_t)base + jj;
			a.state[si] = sw; a.state[a.state_cap + si] = sT;
			a.state[2 * a.state_cap + si] = sr; a.state[3 * a.state_cap + si] = sg; a.state[4 * a.state_cap + si] = sb;
		}
	}
	// channel ch of the target, the background and the loss (every lane of the row holds rr, rg, rb, t, cn)
	float texc, tex3;
	if (raw == 0x00FF00FFu) { texc = tex3 = -1.0f; }
	else {
		const float alpha = (float)(raw >> 24) * (1.0f / 255.0f);
		texc = srgb_to_linear((float)((raw >> (8 * ch)) & 0xff) * (1.0f / 255.0f)) * alpha;
		tex3 = alpha;
	}
	const float exposure_scale = expf(0.6931471805599453f * 0.0f);
	float target;
	if (cfg.linear_colors || cfg.color_space_linear) {
		target = exposure_scale * texc + (1.0f - tex3) * bgc;
		if (!cfg.linear_colors) { target = linear_to_srgb(target); bgc = linear_to_srgb(bgc); }
	} else {
		bgc = linear_to_srgb(bgc);
		target = tex3 > 0 ? linear_to_srgb(exposure_scale * texc / tex3) * tex3 + (1.0f - tex3) * bgc : bgc;
	}
	float pred = ch == 0 ? rr : ch == 1 ? rg : rb;
	if (cn == numsteps) pred += t * bgc;
	float lc, gc;
	loss_channel(target, pred, cfg.loss_type, &lc, &gc);
	const float l1 = row_bcast<1>(lc), l2 = row_bcast<2>(lc), g1 = row_bcast<1>(gc), g2 = row_bcast<2>(gc);
	const float p1 = row_bcast<1>(pred), p2 = row_bcast<2>(pred);
	if (L != 0) return;
	craw[i] = cn;
	LossRay q;
	q.mean_loss = (lc + l1 + l2) / 3.0f;
	q.grad[0] = gc; q.grad[1] = g1; q.grad[2] = g2;
	q.rgb_ray[0] = pred; q.rgb_ray[1] = p1; q.rgb_ray[2] = p2;
	q.u = u; q.v = v; q.img = img;
	q.pad[0] = q.pad[1] = 0.f;
	lr[i] = q;
}

// error map deposit of one compacted ray (testbed_nerf.cu:1869-1899 without the sharpness factor,
// include_sharpness_in_error is off by default): mean loss split bilinearly over the 4 texels around
// uv * res - 0.5, float atomics as in the reference (the map only steers importance sampling)
__device__ __forceinline__ void deposit_error(const LossArgs& a, const Camera* __restrict__ cams, const LossRay& q) {
	const float rx = (float)a.em_w, ry = (float)a.em_h;
	const float px = fminf(fmaxf(q.u * rx - 0.5f, 0.0f), rx - (1.0f + 1e-4f));
	const float py = fminf(fmaxf(q.v * ry - 0.5f, 0.0f), ry - (1.0f + 1e-4f));
	const int ix0 = (int)px, iy0 = (int)py;
	const float wx = px - (float)ix0, wy = py - (float)iy0;
	// clamp(pos_int, 0, resolution - 2) with the image's resolution, as the reference writes it
	const int ix = min(max(ix0, 0), (int)cams[q.img].width - 2), iy = min(max(iy0, 0), (int)cams[q.img].height - 2);
	float* em = a.error_map + (size_t)q.img * a.em_w * a.em_h;
	const float ml = q.mean_loss;
	atomicAdd(em + (size_t)iy * a.em_w + ix, (1 - wx) * (1 - wy) * ml);
	atomicAdd(em + (size_t)iy * a.em_w + ix + 1, wx * (1 - wy) * ml);
	atomicAdd(em + (size_t)(iy + 1) * a.em_w + ix, (1 - wx) * wy * ml);
	atomicAdd(em + (size_t)(iy + 1) * a.em_w + ix + 1, wx * wy * ml);
}

// LANES per ray: LG (one DPP row) when pass 2 composites again; a whole wave when it reads pass 1's kept state,
// where the samples are independent: a ray's samples then take ceil(cn / 64) rounds of loads instead of
// ceil(cn / 16), and the long rays, each round a memory latency, set the kernel's time (fox: up to ~26 rounds)
template <uint32_t LANES>
__global__ void __launch_bounds__(256) k_loss_pass2(const Camera* __restrict__ cams, const ngp_nerf_config cfg, LossArgs a,
                                                    const uint32_t* __restrict__ craw, const uint32_t* __restrict__ gpre,
                                                    const LossRay* __restrict__ lr) {
	const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t i = gid / LANES, L = gid % LANES;
	if (i >= a.n_rays || i >= *a.ray_counter) return;
	const uint32_t base = a.numsteps[2 * i + 1];
	// the exclusive prefix of the compacted counts: the ray's group of 4 (k_scan4) plus the rays of the group before it
	uint32_t compacted_base = gpre[i / 4];
	for (uint32_t r = i & ~3u; r < i; ++r) compacted_base += craw[r];
	const uint32_t mx = a.max_samples_compacted;
	const uint32_t cn = min(mx - min(mx, compacted_base), craw[i]);
	if (L == 0) {  // every lane of the row has read numsteps[2i + 1] above (one wave instruction)
		a.numsteps[2 * i] = cn;
		a.numsteps[2 * i + 1] = compacted_base;
	}
	if (cn == 0) return;
	const LossRay q = lr[i];
	if (L == 0 && a.loss) a.loss[i] = q.mean_loss / (float)a.n_rays;  // written after the compaction early-out (:1836-1866)
	if (L == 0 && a.error_map) deposit_error(a, cams, q);
	const float loss_scale = a.loss_scale / (float)a.n_rays;
	const float output_l2_reg = cfg.rgb_activation == ACT_EXP ? 1e-4f : 0.0f;
	const float output_l1_reg_density = *a.mean_density < MIN_OPTICAL_THICKNESS ? 1e-4f : 0.0f;
	const Aabb box = cfg_aabb(cfg);
	const float* ray = a.rays + (size_t)i * 6;
	const float ro0 = ray[0], ro1 = ray[1], ro2 = ray[2];
	const f16* out = a.network_output + (size_t)base * a.out_stride;
	const float* ci = a.coords_in + (size_t)base * 7;
	float* co = a.coords_out + (size_t)compacted_base * 7;
	f16* dl = a.dloss_doutput + (size_t)compacted_base * 16;
	// the gradient of compacted sample jj (cc its coordinates, o its network output, its weight my_w, the
	// transmittance after it my_t and the rgb prefix through it my_r2), written with its coordinates
	auto emit = [&](uint32_t jj, const float (&cc)[7], const f16x4& o, const float (&rgb)[3], float dt, float my_w, float my_t,
	                const float (&my_r2)[3]) __attribute__((always_inline)) {
#pragma unroll
		for (int k = 0; k < 7; ++k) co[(size_t)jj * 7 + k] = cc[k];
		const V3 pos = unwarp_pos(cc, box);
		const float ddx = pos.x - ro0, ddy = pos.y - ro1, ddz = pos.z - ro2;
		const float depth = sqrtf(ddx * ddx + ddy * ddy + ddz * ddz);
		float suffix[3];
		for (int k = 0; k < 3; ++k) suffix[k] = q.rgb_ray[k] - my_r2[k];
		f16x4 g;
		for (int k = 0; k < 3; ++k) {
			const float dloss_by_drgb = my_w * q.grad[k];
			g[k] = (f16)(loss_scale * (dloss_by_drgb * network_to_rgb_derivative((float)o[k], cfg.rgb_activation) +
			                           fmaxf(0.0f, output_l2_reg * (float)o[k])));
		}
		const float density_derivative = network_to_density_derivative((float)o[3], cfg.density_activation);
		const float dotv = q.grad[0] * (my_t * rgb[0] - suffix[0]) + q.grad[1] * (my_t * rgb[1] - suffix[1]) +
		                   q.grad[2] * (my_t * rgb[2] - suffix[2]);
		const float dloss_by_dmlp = density_derivative * (dt * (dotv + 0.0f));
		const float o3 = (float)o[3];
		g[3] = (f16)(loss_scale * dloss_by_dmlp + (o3 < 0.0f ? -output_l1_reg_density : 0.0f) +
		             (o3 > -10.0f && depth < cfg.near_distance ? 1e-4f : 0.0f));
		*(f16x4*)(dl + (size_t)jj * 16) = g;
	};
	if (LANES != LG || a.state) {  // pass 1 kept every composited sample's state: no sequential compositing here
		if ((size_t)base + cn <= a.state_cap) {
			for (uint32_t jj = L; jj < cn; jj += LANES) {
				float cc[7];
#pragma unroll
				for (int k = 0; k < 7; ++k) cc[k] = ci[(size_t)jj * 7 + k];
				const f16x4 o = *(const f16x4*)(out + (size_t)jj * a.out_stride);
				const size_t si = (size_t)base + jj;
				const float my_w = a.state[si], my_t = a.state[a.state_cap + si];
				const float my_r2[3] = {a.state[2 * a.state_cap + si], a.state[3 * a.state_cap + si], a.state[4 * a.state_cap + si]};
				float rgb[3];
				for (int k = 0; k < 3; ++k) rgb[k] = network_to_rgb((float)o[k], cfg.rgb_activation);
				emit(jj, cc, o, rgb, unwarp_dt(cc[3]), my_w, my_t, my_r2);
			}
			return;
		}
		// the ray's samples reach past the caller's state capacity (pass 1 kept no state there): every lane
		// composites the ray in sample order itself, with pass 1's operations, and emits its own samples
		float t = 1.f, r2[3] = {0.f, 0.f, 0.f};
		for (uint32_t jj = 0; jj < cn; ++jj) {
			float cc[7];
#pragma unroll
			for (int k = 0; k < 7; ++k) cc[k] = ci[(size_t)jj * 7 + k];
			const f16x4 o = *(const f16x4*)(out + (size_t)jj * a.out_stride);
			float rgb[3];
			for (int k = 0; k < 3; ++k) rgb[k] = network_to_rgb((float)o[k], cfg.rgb_activation);
			const float dt = unwarp_dt(cc[3]);
			const float alpha = 1.f - ngp_expf_fast(-network_to_density((float)o[3], cfg.density_activation) * dt);
			const float weight = alpha * t;
			r2[0] = r2[0] + weight * rgb[0]; r2[1] = r2[1] + weight * rgb[1]; r2[2] = r2[2] + weight * rgb[2];
			t = t * (1.f - alpha);
			if (jj % LANES == L) emit(jj, cc, o, rgb, dt, weight, t, r2);
		}
		return;
	}
	if constexpr (LANES == LG) {
	float r2[3] = {0.f, 0.f, 0.f};
	float t = 1.0f;
	// software pipelining as in pass 1: NGP_LOSS2_PF chunks' loads in flight ahead of the compositing
	float cb[NGP_LOSS2_PF][7];
	f16x4 ob[NGP_LOSS2_PF];
#pragma unroll
	for (uint32_t d = 0; d < NGP_LOSS2_PF; ++d) {
		ob[d] = f16x4{(f16)0.f, (f16)0.f, (f16)0.f, (f16)0.f};
#pragma unroll
		for (int k = 0; k < 7; ++k) cb[d][k] = 0.f;
		if (L + d * LG < cn) {
#pragma unroll
			for (int k = 0; k < 7; ++k) cb[d][k] = ci[(size_t)(L + d * LG) * 7 + k];
			ob[d] = *(const f16x4*)(out + (size_t)(L + d * LG) * a.out_stride);
		}
	}
	for (uint32_t cq = 0; cq < cn; cq += NGP_LOSS2_PF * LG)
#pragma unroll
	for (uint32_t d = 0; d < NGP_LOSS2_PF; ++d) {
		const uint32_t c0 = cq + d * LG;
		if (c0 >= cn) break;
		const uint32_t jj = c0 + L;
		const bool valid = jj < cn;
		float cc[7];
#pragma unroll
		for (int k = 0; k < 7; ++k) cc[k] = cb[d][k];
		const f16x4 o = ob[d];
		if (jj + NGP_LOSS2_PF * LG < cn) {
#pragma unroll
			for (int k = 0; k < 7; ++k) cb[d][k] = ci[(size_t)(jj + NGP_LOSS2_PF * LG) * 7 + k];
			ob[d] = *(const f16x4*)(out + (size_t)(jj + NGP_LOSS2_PF * LG) * a.out_stride);
		}
		float rgb[3] = {0.f, 0.f, 0.f}, alpha = 0.f, dt = 0.f;
		if (valid) {
			for (int k = 0; k < 3; ++k) rgb[k] = network_to_rgb((float)o[k], cfg.rgb_activation);
			dt = unwarp_dt(cc[3]);
			const float density = network_to_density((float)o[3], cfg.density_activation);
			alpha = 1.f - ngp_expf_fast(-density * dt);
		}
		// compositing in sample order; lane L stops after its own sample, so it ends with its weight, the
		// transmittance after it and the rgb prefix through it; the chunk's totals come from lane 15
		float my_w = 0.f;
#define NGP_LOSS2_STEP(K)                                                                              \
		{                                                                                              \
			const float ak = row_bcast<K>(alpha), rk = row_bcast<K>(rgb[0]), gk = row_bcast<K>(rgb[1]), bk = row_bcast<K>(rgb[2]); \
			if (c0 + K < cn && K <= L) {                                                               \
				const float weight = ak * t;                                                           \
				r2[0] += weight * rk; r2[1] += weight * gk; r2[2] += weight * bk;                      \
				t *= (1.0f - ak);                                                                      \
				my_w = weight;                                                                         \
			}                                                                                          \
		}
		NGP_ROW_UNROLL16(NGP_LOSS2_STEP)
#undef NGP_LOSS2_STEP
		const float my_t = t, my_r2[3] = {r2[0], r2[1], r2[2]};
		t = row_bcast<15>(t);  // a next chunk exists only if this one is full: lane 15 then took all 16 samples
		r2[0] = row_bcast<15>(r2[0]); r2[1] = row_bcast<15>(r2[1]); r2[2] = row_bcast<15>(r2[2]);
		if (!valid) continue;
		emit(jj, cc, o, rgb, dt, my_w, my_t, my_r2);
	}
	}
}

size_t loss_tmp_f32(uint32_t n_rays) { return (size_t)n_rays * (sizeof(LossRay) / 4); }

void compute_loss(const Dataset& ds, const ngp_nerf_config& cfg, const LossArgs& a, uint32_t* tmp, float* tmpf, hipStream_t s) {
	if (a.n_rays == 0) return;
	uint32_t* craw = tmp;
	uint32_t* gpre = tmp + a.n_rays;  // per group of 4 rays
	LossRay* lr = (LossRay*)tmpf;
	const uint32_t blocks = div_round_up((size_t)a.n_rays * LG, 256);
	{
		ProfScope ps("loss_pass1", s);
		static_assert(256 / LG == 16, "k_loss_pass1's XCD-aware order assumes 16 rays per block");
		const uint32_t b1 = NGP_LOSS_XCD ? 8 * div_round_up(a.n_rays, 128) : blocks;
		k_loss_pass1<<<b1, 256, 0, s>>>(ds.d_cams, ds.d_pixels, ds.n_images, cfg, a, craw, lr);
		NGP_HIP(hipGetLastError());
	}
	{
		ProfScope ps("loss_scan", s);
		k_scan4<<<1, SCAN1_THREADS, 0, s>>>(a.n_rays, craw, gpre, a.compacted_counter, a.ray_counter, a.pub_host, a.pub_seq);
		NGP_HIP(hipGetLastError());
	}
	ProfScope ps("loss_pass2", s);
	static_assert(NGP_LOSS_SELECT, "pass 1 keeps the compositing state pass 2 reads only in its select form");
	if (a.state) {
		constexpr uint32_t W = NGP_LOSS2_LANES;  // a wave per ray: see k_loss_pass2
		k_loss_pass2<W><<<div_round_up((size_t)a.n_rays * W, 256), 256, 0, s>>>(ds.d_cams, cfg, a, craw, gpre, lr);
	} else {
		k_loss_pass2<LG><<<blocks, 256, 0, s>>>(ds.d_cams, cfg, a, craw, gpre, lr);
	}
	NGP_HIP(hipGetLastError());
}

// construct_cdf_2d (testbed_nerf.cu:2356-2382): one thread per (image, row), running sums along x
constexpr float ERROR_MAP_MIN_PDF = 0.01f;
__global__ void k_cdf_2d(uint32_t n_images, uint32_t h, uint32_t w, const float* __restrict__ data, float* __restrict__ cdf_x_cond_y,
                         float* __restrict__ cdf_y) {
	const uint32_t y = blockIdx.x * blockDim.x + threadIdx.x, img = blockIdx.y;
	if (y >= h || img >= n_images) return;
	const size_t off = ((size_t)img * h + y) * w;
	float cum = 0.f;
	for (uint32_t x = 0; x < w; ++x) {
		cum += data[off + x] + 1e-10f;
		cdf_x_cond_y[off + x] = cum;
	}
	cdf_y[(size_t)img * h + y] = cum;
	const float norm = 1.0f / cum;  // __frcp_rn: the correctly rounded reciprocal
	for (uint32_t x = 0; x < w; ++x)
		cdf_x_cond_y[off + x] = (1.0f - ERROR_MAP_MIN_PDF) * cdf_x_cond_y[off + x] * norm + ERROR_MAP_MIN_PDF * (float)(x + 1) / (float)w;
}
// construct_cdf_1d (:2384-2410): one thread per image, running sums over the rows' totals
__global__ void k_cdf_1d(uint32_t n_images, uint32_t h, float* __restrict__ cdf_y, float* __restrict__ cdf_img) {
	const uint32_t img = blockIdx.x * blockDim.x + threadIdx.x;
	if (img >= n_images) return;
	float* c = cdf_y + (size_t)img * h;
	float cum = 0.f;
	for (uint32_t y = 0; y < h; ++y) {
		cum += c[y];
		c[y] = cum;
	}
	cdf_img[img] = cum;
	const float norm = 1.0f / cum;
	for (uint32_t y = 0; y < h; ++y) c[y] = (1.0f - ERROR_MAP_MIN_PDF) * c[y] * norm + ERROR_MAP_MIN_PDF * (float)(y + 1) / (float)h;
}

void error_map_cdfs(uint32_t n_images, uint32_t w, uint32_t h, const float* data, float* cdf_x_cond_y, float* cdf_y,
                    float* cdf_img, hipStream_t s) {
	if (!n_images || !w || !h) return;
	ProfScope ps("nerf_error_map_cdf", s);
	k_cdf_2d<<<dim3(div_round_up(h, 64u), n_images), 64, 0, s>>>(n_images, h, w, data, cdf_x_cond_y, cdf_y);
	NGP_HIP(hipGetLastError());
	k_cdf_1d<<<div_round_up(n_images, 64u), 64, 0, s>>>(n_images, h, cdf_y, cdf_img);
	NGP_HIP(hipGetLastError());
}


// ------------------------------------------------------------------------------------------------
// tcnn fill_rollover / fill_rollover_and_rescale
// ------------------------------------------------------------------------------------------------
__global__ void k_rollover_f16(uint32_t n_elements, uint32_t stride, const uint32_t* n_input_ptr, f16* data, bool rescale) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t n_in = *n_input_ptr;
	if (i < n_in * stride || i >= n_elements * stride || n_in == 0) return;
	f16 r = data[i % (n_in * stride)];
	if (rescale) r = (f16)((float)r * n_in / n_elements);
	data[i] = r;
}
__global__ void k_rollover_f32(uint32_t n_elements, uint32_t stride, const uint32_t* n_input_ptr, float* data) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t n_in = *n_input_ptr;
	if (i < n_in * stride || i >= n_elements * stride || n_in == 0) return;
	data[i] = data[i % (n_in * stride)];
}
// both rollovers of the training batch in one launch (dL/doutput rescaled, coordinates copied)
// Grid-stride over the rollover range only (a full batch leaves nothing to fill; launching one thread per
// element cost ~16 K empty blocks per step).
__global__ void k_rollover_pair(uint32_t n_elements, uint32_t stride16, uint32_t stride32, const uint32_t* n_input_ptr, f16* d16,
                                float* d32) {
	const uint32_t n_in = *n_input_ptr;
	if (n_in == 0 || n_in >= n_elements) return;
	const uint32_t lo = n_in * (stride16 < stride32 ? stride16 : stride32);
	const uint32_t hi = n_elements * (stride16 > stride32 ? stride16 : stride32);
	for (uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += gridDim.x * blockDim.x) {
		if (i >= n_in * stride16 && i < n_elements * stride16) {
			f16 r = d16[i % (n_in * stride16)];
			r = (f16)((float)r * n_in / n_elements);
			d16[i] = r;
		}
		if (i >= n_in * stride32 && i < n_elements * stride32) d32[i] = d32[i % (n_in * stride32)];
	}
}
// k_rollover_pair plus the step's publish and control-block writes (StepPublish): two launches less per NeRF step
__global__ void k_rollover_pair_publish(uint32_t n_elements, uint32_t stride16, uint32_t stride32, const uint32_t* n_input_ptr, f16* d16,
                                        float* d32, const StepPublish pub) {
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		volatile uint32_t* host = pub.host;
		if (host) {
			host[0] = pub.ctr[0]; host[1] = pub.ctr[1]; host[2] = pub.ctr[2]; host[3] = pub.ctr[3];
			__threadfence_system();
			host[4] = pub.seq;
		}
		pub.ctl[0] = pub.step;
		for (uint32_t k = 0; k < pub.cfg_words; ++k) pub.ctl[pub.cfg_off + k] = pub.cfg[k];
	}
	const uint32_t n_in = *n_input_ptr;
	if (n_in == 0 || n_in >= n_elements) return;
	const uint32_t lo = n_in * (stride16 < stride32 ? stride16 : stride32);
	const uint32_t hi = n_elements * (stride16 > stride32 ? stride16 : stride32);
	for (uint32_t i = lo + blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += gridDim.x * blockDim.x) {
		if (i >= n_in * stride16 && i < n_elements * stride16) {
			f16 r = d16[i % (n_in * stride16)];
			r = (f16)((float)r * n_in / n_elements);
			d16[i] = r;
		}
		if (i >= n_in * stride32 && i < n_elements * stride32) d32[i] = d32[i % (n_in * stride32)];
	}
}
void fill_rollover_pair_publish(uint32_t n_elements, const uint32_t* n_input, f16* dloss, uint32_t stride16, float* coords,
                                uint32_t stride32, const StepPublish& pub, hipStream_t s) {
	NGP_CHECK(pub.ctl && pub.cfg_words <= 32, "rollover publish: control block and config required");
	const uint64_t n = (uint64_t)n_elements * (stride16 > stride32 ? stride16 : stride32);
	const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(div_round_up(n, 256), 1024));
	k_rollover_pair_publish<<<blocks, 256, 0, s>>>(n_elements, stride16, stride32, n_input, dloss, coords, pub);
	NGP_HIP(hipGetLastError());
}
void fill_rollover_pair(uint32_t n_elements, const uint32_t* n_input, f16* dloss, uint32_t stride16, float* coords,
                        uint32_t stride32, hipStream_t s) {
	const uint64_t n = (uint64_t)n_elements * (stride16 > stride32 ? stride16 : stride32);
	const uint32_t blocks = (uint32_t)std::min<uint64_t>(div_round_up(n, 256), 1024);
	k_rollover_pair<<<blocks, 256, 0, s>>>(n_elements, stride16, stride32, n_input, dloss, coords);
	NGP_HIP(hipGetLastError());
}
void fill_rollover_f16(uint32_t n_elements, uint32_t stride, const uint32_t* n_input, f16* data, bool rescale, hipStream_t s) {
	k_rollover_f16<<<div_round_up((uint64_t)n_elements * stride, 256), 256, 0, s>>>(n_elements, stride, n_input, data, rescale);
	NGP_HIP(hipGetLastError());
}
void fill_rollover_f32(uint32_t n_elements, uint32_t stride, const uint32_t* n_input, float* data, hipStream_t s) {
	k_rollover_f32<<<div_round_up((uint64_t)n_elements * stride, 256), 256, 0, s>>>(n_elements, stride, n_input, data);
	NGP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// occupancy grid
// ------------------------------------------------------------------------------------------------
// generate_grid_samples_nerf_nonuniform (testbed_nerf.cu:635-676)
// The candidate test of generate_grid_samples_nerf_nonuniform (grid_in[idx] > thresh) for every cell of the
// sampled cascades as one bit per cell: a linear pass over the grid (32 cells -> one word, 128-B coalesced reads),
// so the samples' up-to-10 candidates are tested against a 256-KB-per-cascade mask that stays in L2 instead of
// one scattered 4-B grid read (a 64-B transaction) per candidate, in a chain.
__global__ void k_grid_mask(uint32_t n_words, const float* __restrict__ grid, float thresh, uint32_t* __restrict__ mask) {
	const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
	if (w >= n_words) return;
	const float4* g = (const float4*)(grid + (size_t)w * 32);
	uint32_t bits = 0;
#pragma unroll
	for (uint32_t q = 0; q < 8; ++q) {
		const float4 v = g[q];
		bits |= (v.x > thresh ? 1u : 0u) << (4 * q) | (v.y > thresh ? 1u : 0u) << (4 * q + 1) |
		        (v.z > thresh ? 1u : 0u) << (4 * q + 2) | (v.w > thresh ? 1u : 0u) << (4 * q + 3);
	}
	mask[w] = bits;
}

#ifndef NGP_GRID_CAND_FIRST
#define NGP_GRID_CAND_FIRST 2  // k_grid_samples: candidates whose mask words every lane loads (10: all at once)
#endif
static_assert(NGP_GRID_CAND_FIRST >= 1 && NGP_GRID_CAND_FIRST <= 10, "grid sample candidates");
__global__ void k_grid_samples(uint32_t n, Rng rng, uint32_t step, const ngp_nerf_config cfg, const uint32_t* __restrict__ mask,
                               uint32_t n_cascades, float* __restrict__ out, uint32_t* __restrict__ indices) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	pcg_advance(rng, (uint64_t)i * 4);
	const uint32_t level = (uint32_t)(pcg_float(rng) * n_cascades) % n_cascades;
	// the candidates' mask words (L2 hits) in batches of GRID_CAND_FIRST and the rest, the second batch only for the
	// lanes whose first batch has no passing cell: the first candidate that passes, as the reference's loop takes it
	// (its last candidate when none passes). The kernel is bound by the L2 request rate, and in the uniform pass nearly
	// every first candidate passes.
	constexpr uint32_t NA = NGP_GRID_CAND_FIRST;
	uint32_t cand[10], word[10];
	const uint32_t base = (i + step * n) * 56924617u + 96925573u;
#pragma unroll
	for (uint32_t j = 0; j < 10; ++j) cand[j] = (base + j * 19349663u) % GRID_N_CELLS + level * GRID_N_CELLS;
#pragma unroll
	for (uint32_t j = 0; j < NA; ++j) word[j] = mask[cand[j] >> 5];
	uint32_t idx = ~0u;
#pragma unroll
	for (int j = (int)NA - 1; j >= 0; --j)
		if ((word[j] >> (cand[j] & 31u)) & 1u) idx = cand[j];
	if (idx == ~0u) {
#pragma unroll
		for (uint32_t j = NA; j < 10; ++j) word[j] = mask[cand[j] >> 5];
		idx = cand[9];
#pragma unroll
		for (int j = 9; j >= (int)NA; --j)
			if ((word[j] >> (cand[j] & 31u)) & 1u) idx = cand[j];
	}
	const uint32_t pos_idx = idx % GRID_N_CELLS;
	const uint32_t x = morton3D_invert(pos_idx >> 0), y = morton3D_invert(pos_idx >> 1), z = morton3D_invert(pos_idx >> 2);
	const float r0 = pcg_float(rng), r1 = pcg_float(rng), r2 = pcg_float(rng);
	const float sc = scalbnf(1.0f, (int)level);
	const float px = (((float)x + r0) / (float)GRIDSIZE - 0.5f) * sc + 0.5f;
	const float py = (((float)y + r1) / (float)GRIDSIZE - 0.5f) * sc + 0.5f;
	const float pz = (((float)z + r2) / (float)GRIDSIZE - 0.5f) * sc + 0.5f;
	out[(size_t)i * 3 + 0] = (px - cfg.aabb_min[0]) / (cfg.aabb_max[0] - cfg.aabb_min[0]);
	out[(size_t)i * 3 + 1] = (py - cfg.aabb_min[1]) / (cfg.aabb_max[1] - cfg.aabb_min[1]);
	out[(size_t)i * 3 + 2] = (pz - cfg.aabb_min[2]) / (cfg.aabb_max[2] - cfg.aabb_min[2]);
	indices[i] = idx;
}

// splat_grid_samples_nerf_max_nearest_neighbor (:678-702); density_rm = density MLP output row 0 (RM)
__global__ void k_grid_splat(uint32_t n, const uint32_t* __restrict__ indices, const f16* __restrict__ density, uint32_t act,
                             float* __restrict__ grid_out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float mlp = network_to_density((float)density[i], act);
	const float thickness = mlp * scalbnf(MIN_CONE_STEPSIZE, 0);
	atomicMax((uint32_t*)&grid_out[indices[i]], __float_as_uint(thickness));
}

// ema_grid_samples_nerf (:731-754): max-filter
__global__ void k_grid_ema(uint32_t n, float decay, float* __restrict__ grid, const float* __restrict__ tmp) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float prev = grid[i];
	grid[i] = prev < 0.f ? prev : fmaxf(prev * decay, tmp[i]);
}

// reduce_sum(max(v,0)/N) over cascade 0 (:3544-3551), fixed order: 512 blocks x 256 threads, then one block.
__global__ void __launch_bounds__(256) k_grid_mean_partial(const float* __restrict__ grid, float* __restrict__ partial) {
	__shared__ float s[256];
	const uint32_t per_block = GRID_N_CELLS / 512;
	const uint32_t base = blockIdx.x * per_block;
	float acc = 0.f;
	for (uint32_t k = threadIdx.x; k < per_block; k += 256) acc += fmaxf(grid[base + k], 0.f) / (float)GRID_N_CELLS;
	s[threadIdx.x] = acc;
	__syncthreads();
	for (uint32_t off = 128; off > 0; off >>= 1) {
		if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off];
		__syncthreads();
	}
	if (threadIdx.x == 0) partial[blockIdx.x] = s[0];
}
__global__ void __launch_bounds__(512) k_grid_mean_final(const float* __restrict__ partial, float* __restrict__ mean) {
	__shared__ float s[512];
	s[threadIdx.x] = partial[threadIdx.x];
	__syncthreads();
	for (uint32_t off = 256; off > 0; off >>= 1) {
		if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off];
		__syncthreads();
	}
	if (threadIdx.x == 0) *mean = s[0];
}

// grid_to_bitfield (:762-786)
__global__ void k_grid_to_bitfield(uint32_t n_elements, uint32_t n_nonzero, const float* __restrict__ grid,
                                   uint8_t* __restrict__ bitfield, const float* __restrict__ mean) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_elements) return;
	if (i >= n_nonzero) { bitfield[i] = 0; return; }
	const float thresh = fminf(MIN_OPTICAL_THICKNESS, *mean);
	uint8_t bits = 0;
#pragma unroll
	for (uint8_t j = 0; j < 8; ++j) bits |= grid[i * 8 + j] > thresh ? ((uint8_t)1 << j) : 0;
	bitfield[i] = bits;
}

// bitfield_max_pool (:788-809)
__global__ void k_bitfield_max_pool(uint32_t n, const uint8_t* __restrict__ prev, uint8_t* __restrict__ next) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	uint8_t bits = 0;
#pragma unroll
	for (uint8_t j = 0; j < 8; ++j) bits |= prev[i * 8 + j] > 0 ? ((uint8_t)1 << j) : 0;
	const uint32_t x = morton3D_invert(i >> 0) + GRIDSIZE / 8;
	const uint32_t y = morton3D_invert(i >> 1) + GRIDSIZE / 8;
	const uint32_t z = morton3D_invert(i >> 2) + GRIDSIZE / 8;
	next[morton3D(x, y, z)] |= bits;
}

size_t grid_mask_words(uint32_t n_cascades) { return (size_t)n_cascades * GRID_N_CELLS / 32; }
void grid_generate_samples(uint32_t n, Rng rng, uint32_t step, const ngp_nerf_config& cfg, const float* grid_in,
                           uint32_t n_cascades, float thresh, float* positions, uint32_t* indices, uint32_t* mask, hipStream_t s) {
	if (n == 0) return;
	const uint32_t nw = (uint32_t)grid_mask_words(n_cascades);
	k_grid_mask<<<div_round_up(nw, 256), 256, 0, s>>>(nw, grid_in, thresh, mask);
	k_grid_samples<<<div_round_up(n, 128), 128, 0, s>>>(n, rng, step, cfg, mask, n_cascades, positions, indices);
	NGP_HIP(hipGetLastError());
}
// The splat as a counting sort by cell bin (fox: 5.2 M samples into 10.5 M cells). The direct splat's atomics are
// scattered over the whole grid and run at ~32 G/s whatever their locality (an XCD-sliced variant that kept each
// XCD's cells L2-resident measured no faster): here each sample costs two LDS atomics and 8 B of
// coalesced-ish traffic instead. Bins of 8192 cells (32 KB of LDS):
//   k_splat_hist: per-block LDS histogram of the samples' bins, added to the global counts (one atomic per bin and
//     block);
//   k_splat_scan: the bins' offsets (one block);
//   k_splat_scatter: each block reserves its range in every bin (cursor atomics), ranks its samples in LDS and writes
//     (cell in bin << 16 | density bits) there;
//   k_splat_bins: a block per bin takes the max of its samples in LDS with the same uint compare as the atomics, then
//     writes all 8192 cells (so no memset of grid_tmp).
// Max does not depend on the order, so grid_tmp is bit-identical to memset(0) + k_grid_splat.
#ifndef NGP_SPLAT_THREADS
#define NGP_SPLAT_THREADS 1024
#endif
constexpr uint32_t SPLAT_THREADS = NGP_SPLAT_THREADS;  // k_splat_hist / k_splat_scatter block size
constexpr uint32_t SPLAT_BIN_SHIFT = 13, SPLAT_BIN = 1u << SPLAT_BIN_SHIFT, SPLAT_MAX_BINS = 8 * GRID_N_CELLS / SPLAT_BIN;
#ifndef NGP_SPLAT_MAX_BLOCKS
#define NGP_SPLAT_MAX_BLOCKS 256  // 128 -> 256: fox scatter 88.5 -> 63.5 us (gpurun_out/r06as_256)
#endif
#ifndef NGP_SPLAT_CHUNK
#define NGP_SPLAT_CHUNK 4096  // samples per k_splat_hist / k_splat_scatter block at least (Lego: 256 blocks, not 64)
#endif
static uint32_t splat_blocks(uint32_t n) {
	return std::max(1u, std::min((uint32_t)NGP_SPLAT_MAX_BLOCKS, div_round_up(n, NGP_SPLAT_CHUNK)));
}
__device__ __forceinline__ void splat_chunk(uint32_t n, uint32_t nb, uint32_t* s0, uint32_t* s1) {
	*s0 = (uint32_t)((uint64_t)n * blockIdx.x / nb);
	*s1 = (uint32_t)((uint64_t)n * (blockIdx.x + 1) / nb);
}
__global__ void __launch_bounds__(SPLAT_THREADS) k_splat_hist(uint32_t n, const uint32_t* __restrict__ indices, uint32_t n_bins,
                                                   uint32_t* __restrict__ counts) {
	__shared__ uint32_t h[SPLAT_MAX_BINS];
	for (uint32_t b = threadIdx.x; b < n_bins; b += SPLAT_THREADS) h[b] = 0;
	__syncthreads();
	uint32_t s0, s1;
	splat_chunk(n, gridDim.x, &s0, &s1);
	for (uint32_t i = s0 + threadIdx.x; i < s1; i += 4 * SPLAT_THREADS) {
		uint32_t k[4];
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u) k[u] = i + u * SPLAT_THREADS < s1 ? indices[i + u * SPLAT_THREADS] : ~0u;
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u)
			if (k[u] != ~0u) atomicAdd(&h[k[u] >> SPLAT_BIN_SHIFT], 1u);
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < n_bins; b += SPLAT_THREADS)
		if (h[b]) atomicAdd(&counts[b], h[b]);
}
__global__ void __launch_bounds__(1024) k_splat_scan(uint32_t n_bins, const uint32_t* __restrict__ counts,
                                                    uint32_t* __restrict__ offsets, uint32_t* __restrict__ cursor) {
	__shared__ uint32_t sh[1024];
	const uint32_t b0 = 2 * threadIdx.x;  // two bins per thread (n_bins <= 2048)
	const uint32_t c0 = b0 < n_bins ? counts[b0] : 0u, c1 = b0 + 1 < n_bins ? counts[b0 + 1] : 0u;
	sh[threadIdx.x] = c0 + c1;
	__syncthreads();
	for (uint32_t off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
		const uint32_t v = threadIdx.x >= off ? sh[threadIdx.x - off] : 0u;
		__syncthreads();
		sh[threadIdx.x] += v;
		__syncthreads();
	}
	const uint32_t ex = sh[threadIdx.x] - c0 - c1;
	if (b0 < n_bins) { offsets[b0] = ex; cursor[b0] = ex; }
	if (b0 + 1 < n_bins) { offsets[b0 + 1] = ex + c0; cursor[b0 + 1] = ex + c0; }
	if (threadIdx.x == 1023) offsets[n_bins] = sh[1023];
}
// SORT: the samples themselves into bin order before the density evaluation, one 16-B record per sample (x, y, z and
// the cell within the bin as the 4th word: one store request per sample); else the (cell in bin, density bits) pairs
// after it.
template <bool SORT>
__global__ void __launch_bounds__(SPLAT_THREADS) k_splat_scatter(uint32_t n, const uint32_t* __restrict__ indices,
                                                                const f16* __restrict__ density,
                                                                const float* __restrict__ positions, uint32_t n_bins,
                                                                uint32_t* __restrict__ cursor, uint32_t* __restrict__ packed,
                                                                float4* __restrict__ pos_out) {
	__shared__ uint32_t h[SPLAT_MAX_BINS], base[SPLAT_MAX_BINS];
	for (uint32_t b = threadIdx.x; b < n_bins; b += SPLAT_THREADS) h[b] = 0;
	__syncthreads();
	uint32_t s0, s1;
	splat_chunk(n, gridDim.x, &s0, &s1);
	for (uint32_t i = s0 + threadIdx.x; i < s1; i += 4 * SPLAT_THREADS) {
		uint32_t k[4];
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u) k[u] = i + u * SPLAT_THREADS < s1 ? indices[i + u * SPLAT_THREADS] : ~0u;
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u)
			if (k[u] != ~0u) atomicAdd(&h[k[u] >> SPLAT_BIN_SHIFT], 1u);
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < n_bins; b += SPLAT_THREADS) {
		if (h[b]) base[b] = atomicAdd(&cursor[b], h[b]);
		h[b] = 0;
	}
	__syncthreads();
	for (uint32_t i = s0 + threadIdx.x; i < s1; i += 4 * SPLAT_THREADS) {
		uint32_t k[4];
		uint16_t d[4];
		float px[4], py[4], pz[4];
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u) {
			const bool ok = i + u * SPLAT_THREADS < s1;
			const uint32_t j = i + u * SPLAT_THREADS;
			k[u] = ok ? indices[j] : ~0u;
			if (SORT) {
				px[u] = ok ? positions[(size_t)j * 3 + 0] : 0.f;
				py[u] = ok ? positions[(size_t)j * 3 + 1] : 0.f;
				pz[u] = ok ? positions[(size_t)j * 3 + 2] : 0.f;
			} else {
				d[u] = ok ? __builtin_bit_cast(uint16_t, density[j]) : (uint16_t)0;
			}
		}
#pragma unroll
		for (uint32_t u = 0; u < 4; ++u) {
			if (k[u] == ~0u) continue;
			const uint32_t b = k[u] >> SPLAT_BIN_SHIFT;
			const uint32_t slot = base[b] + atomicAdd(&h[b], 1u);
			if (SORT) {
				pos_out[slot] = make_float4(px[u], py[u], pz[u], __uint_as_float(k[u] & (SPLAT_BIN - 1)));
			} else {
				packed[slot] = (k[u] & (SPLAT_BIN - 1)) << 16 | d[u];
			}
		}
	}
}
// SORT: bin b's samples are [offsets[b], offsets[b + 1]) of the sorted records (cell in the 4th word), their densities
// density[k - lo] for the shard [lo, hi) this rank evaluated
template <bool SORT>
__global__ void __launch_bounds__(1024) k_splat_bins(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ packed,
                                                    const float4* __restrict__ recs, const f16* __restrict__ density,
                                                    uint32_t lo, uint32_t hi, uint32_t act, float* __restrict__ grid_out) {
	__shared__ uint32_t m[SPLAT_BIN];
	for (uint32_t c = threadIdx.x; c < SPLAT_BIN; c += 1024) m[c] = 0;
	__syncthreads();
	const uint32_t b = blockIdx.x;
	const uint32_t k0 = SORT ? std::max(offsets[b], lo) : offsets[b], e = SORT ? std::min(offsets[b + 1], hi) : offsets[b + 1];
	for (uint32_t k = k0 + threadIdx.x; k < e; k += 1024) {
		uint32_t c;
		f16 d;
		if (SORT) {
			c = __float_as_uint(recs[k].w);
			d = density[k - lo];
		} else {
			const uint32_t v = packed[k];
			c = v >> 16;
			d = __builtin_bit_cast(f16, (uint16_t)(v & 0xffffu));
		}
		const float mlp = network_to_density((float)d, act);
		const float thickness = mlp * scalbnf(MIN_CONE_STEPSIZE, 0);
		atomicMax(&m[c], __float_as_uint(thickness));
	}
	__syncthreads();
	uint4* out = (uint4*)(grid_out + (size_t)b * SPLAT_BIN);
	for (uint32_t q = threadIdx.x; q < SPLAT_BIN / 4; q += 1024) out[q] = make_uint4(m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]);
}

size_t grid_splat_scratch_u32(uint32_t n, uint32_t n_cells) { return 3 * ((size_t)(n_cells >> SPLAT_BIN_SHIFT) + 1) + n; }

void grid_splat_max(uint32_t n, const uint32_t* indices, const f16* density_rm, uint32_t act, float* grid_tmp, hipStream_t s) {
	if (n == 0) return;
	k_grid_splat<<<div_round_up(n, 128), 128, 0, s>>>(n, indices, density_rm, act, grid_tmp);
	NGP_HIP(hipGetLastError());
}
// the histogram, offsets and cursors of n samples' bins (scratch: counts, offsets, cursor of n_bins + 1 words each)
static uint32_t splat_bin_offsets(uint32_t n, const uint32_t* indices, uint32_t n_cells, uint32_t* scratch, hipStream_t s) {
	const uint32_t n_bins = n_cells >> SPLAT_BIN_SHIFT;
	NGP_CHECK(n_cells % SPLAT_BIN == 0 && n_bins <= SPLAT_MAX_BINS, "grid splat: bad cell count");
	uint32_t* counts = scratch;
	NGP_HIP(hipMemsetAsync(counts, 0, (size_t)n_bins * 4, s));
	if (n) k_splat_hist<<<splat_blocks(n), SPLAT_THREADS, 0, s>>>(n, indices, n_bins, counts);
	k_splat_scan<<<1, 1024, 0, s>>>(n_bins, counts, counts + n_bins + 1, counts + 2 * (n_bins + 1));
	return n_bins;
}
void grid_splat_max_binned(uint32_t n, const uint32_t* indices, const f16* density_rm, uint32_t act, float* grid_tmp,
                           uint32_t n_cells, uint32_t* scratch, hipStream_t s) {
	const uint32_t n_bins = splat_bin_offsets(n, indices, n_cells, scratch, s);
	const uint32_t* offsets = scratch + n_bins + 1;
	uint32_t* cursor = scratch + 2 * (n_bins + 1);
	uint32_t* packed = cursor + n_bins + 1;
	if (n) k_splat_scatter<false><<<splat_blocks(n), SPLAT_THREADS, 0, s>>>(n, indices, density_rm, nullptr, n_bins, cursor, packed,
	                                                                       nullptr);
	k_splat_bins<false><<<n_bins, 1024, 0, s>>>(offsets, packed, nullptr, nullptr, 0, 0, act, grid_tmp);
	NGP_HIP(hipGetLastError());
}
size_t grid_sort_scratch_u32(uint32_t n, uint32_t n_cells) { return 3 * ((size_t)(n_cells >> SPLAT_BIN_SHIFT) + 1); }
void grid_sort_samples(uint32_t n, const float* positions, const uint32_t* indices, uint32_t n_cells, uint32_t* scratch,
                       float* recs, hipStream_t s) {
	const uint32_t n_bins = splat_bin_offsets(n, indices, n_cells, scratch, s);
	uint32_t* cursor = scratch + 2 * (n_bins + 1);
	if (n) k_splat_scatter<true><<<splat_blocks(n), SPLAT_THREADS, 0, s>>>(n, indices, nullptr, positions, n_bins, cursor, nullptr,
	                                                                      (float4*)recs);
	NGP_HIP(hipGetLastError());
}
void grid_splat_sorted(uint32_t n_cells, const uint32_t* scratch, const float* recs, const f16* density_rm, uint32_t lo,
                       uint32_t hi, uint32_t act, float* grid_tmp, hipStream_t s) {
	const uint32_t n_bins = n_cells >> SPLAT_BIN_SHIFT;
	const uint32_t* offsets = scratch + n_bins + 1;
	k_splat_bins<true><<<n_bins, 1024, 0, s>>>(offsets, nullptr, (const float4*)recs, density_rm, lo, hi, act, grid_tmp);
	NGP_HIP(hipGetLastError());
}
// The update step's finalization in three launches instead of ten (the reference's ema_grid_samples_nerf,
// update_density_grid_mean_and_bitfield and 7 bitfield_max_pool launches), the same float operations in the same
// order, so the same bits:
//   k_grid_ema_mean: the EMA of every cell; blocks [0, 512) take cascade 0 in k_grid_mean_partial's mapping and
//     accumulate its mean partials from the values they just wrote;
//   k_grid_bitfield: every block reduces the 512 partials in k_grid_mean_final's tree (block 0 stores the mean),
//     then writes 8 bitfield bytes per thread;
//   the pools into mips 1 .. max_cascade + 1 (full grids), then k_bitfield_pool_tail: one block for the mips above,
//     whose sources are zero outside a central region that halves per mip (max_cascade + 1: 64^3 cells, ...).
__global__ void __launch_bounds__(256) k_grid_ema_mean(uint32_t n, float decay, float* __restrict__ grid, const float* __restrict__ tmp,
                                                       float* __restrict__ partial) {
	__shared__ float sh[256];
	if (blockIdx.x >= 512) {
		const uint32_t i = GRID_N_CELLS + (blockIdx.x - 512) * 256 + threadIdx.x;
		if (i >= n) return;
		const float prev = grid[i];
		grid[i] = prev < 0.f ? prev : fmaxf(prev * decay, tmp[i]);
		return;
	}
	const uint32_t per_block = GRID_N_CELLS / 512;
	const uint32_t base = blockIdx.x * per_block;
	float acc = 0.f;
	for (uint32_t k = threadIdx.x; k < per_block; k += 256) {
		const float prev = grid[base + k];
		const float v = prev < 0.f ? prev : fmaxf(prev * decay, tmp[base + k]);
		grid[base + k] = v;
		acc += fmaxf(v, 0.f) / (float)GRID_N_CELLS;
	}
	sh[threadIdx.x] = acc;
	__syncthreads();
	for (uint32_t off = 128; off > 0; off >>= 1) {
		if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
		__syncthreads();
	}
	if (threadIdx.x == 0) partial[blockIdx.x] = sh[0];
}
__global__ void __launch_bounds__(512) k_grid_bitfield(uint32_t n_bytes, uint32_t n_nonzero, const float* __restrict__ grid,
                                                       uint8_t* __restrict__ bitfield, const float* __restrict__ partial,
                                                       float* __restrict__ mean_out) {
	__shared__ float sh[512];
	sh[threadIdx.x] = partial[threadIdx.x];
	__syncthreads();
	for (uint32_t off = 256; off > 0; off >>= 1) {
		if (threadIdx.x < off) sh[threadIdx.x] += sh[threadIdx.x + off];
		__syncthreads();
	}
	const float mean = sh[0];
	if (blockIdx.x == 0 && threadIdx.x == 0) *mean_out = mean;
	const float thresh = fminf(MIN_OPTICAL_THICKNESS, mean);
#pragma unroll
	for (uint32_t q = 0; q < 8; ++q) {
		const uint32_t i = (blockIdx.x * 8 + q) * 512 + threadIdx.x;
		if (i >= n_bytes) return;
		if (i >= n_nonzero) { bitfield[i] = 0; continue; }
		uint8_t bits = 0;
#pragma unroll
		for (uint8_t j = 0; j < 8; ++j) bits |= grid[i * 8 + j] > thresh ? ((uint8_t)1 << j) : 0;
		bitfield[i] = bits;
	}
}
__global__ void __launch_bounds__(1024) k_bitfield_pool_tail(uint32_t first, uint8_t* __restrict__ bitfield) {
	for (uint32_t m = first; m + 1 < CASCADES; ++m) {
		// mip m is zero outside cells [64 - h, 64 + h): h = 32 at m = first, halving per mip; in 4-cell blocks [lo, hi)
		const uint32_t h = 32u >> (m - first);
		const uint32_t lo = (64 - h) / 4, hi = (64 + h + 3) / 4, w = hi - lo;
		const uint8_t* prev = bitfield + (size_t)m * GRID_N_CELLS / 8;
		uint8_t* next = bitfield + (size_t)(m + 1) * GRID_N_CELLS / 8;
		for (uint32_t t = threadIdx.x; t < w * w * w; t += blockDim.x) {
			const uint32_t x = lo + t % w, y = lo + (t / w) % w, z = lo + t / (w * w);
			const uint32_t i = morton3D(x, y, z);
			uint8_t bits = 0;
#pragma unroll
			for (uint8_t j = 0; j < 8; ++j) bits |= prev[i * 8 + j] > 0 ? ((uint8_t)1 << j) : 0;
			next[morton3D(x + GRIDSIZE / 8, y + GRIDSIZE / 8, z + GRIDSIZE / 8)] |= bits;
		}
		__syncthreads();
	}
}
void grid_ema_mean_bitfield(uint32_t n_el, float decay, float* grid, const float* tmp, uint32_t max_cascade, float* mean_out,
                            uint8_t* bitfield, hipStream_t s) {
	float* partial = mean_out + 1;  // [1 + 512] floats
	k_grid_ema_mean<<<512 + div_round_up(n_el - GRID_N_CELLS, 256), 256, 0, s>>>(n_el, decay, grid, tmp, partial);
	const uint32_t n_bytes = GRID_N_CELLS / 8 * CASCADES;
	k_grid_bitfield<<<div_round_up(n_bytes, 8 * 512), 512, 0, s>>>(n_bytes, GRID_N_CELLS / 8 * (max_cascade + 1), grid, bitfield, partial,
	                                                              mean_out);
	const uint32_t full = std::min(max_cascade + 1, CASCADES - 1);  // mips 1 .. full from whole grids
	for (uint32_t level = 1; level <= full; ++level) {
		const uint32_t n = GRID_N_CELLS / 64;
		k_bitfield_max_pool<<<div_round_up(n, 256), 256, 0, s>>>(n, bitfield + (size_t)(level - 1) * GRID_N_CELLS / 8,
		                                                          bitfield + (size_t)level * GRID_N_CELLS / 8);
	}
	if (full + 1 < CASCADES) k_bitfield_pool_tail<<<1, 1024, 0, s>>>(full, bitfield);
	NGP_HIP(hipGetLastError());
}
void grid_ema(uint32_t n, float decay, float* grid, const float* tmp, hipStream_t s) {
	k_grid_ema<<<div_round_up(n, 256), 256, 0, s>>>(n, decay, grid, tmp);
	NGP_HIP(hipGetLastError());
}
void grid_mean_bitfield(const float* grid, uint32_t max_cascade, float* mean_out, uint8_t* bitfield, hipStream_t s) {
	float* partial = mean_out + 1;  // caller provides [1 + 512] floats
	k_grid_mean_partial<<<512, 256, 0, s>>>(grid, partial);
	k_grid_mean_final<<<1, 512, 0, s>>>(partial, mean_out);
	const uint32_t n_bytes = GRID_N_CELLS / 8 * CASCADES;
	k_grid_to_bitfield<<<div_round_up(n_bytes, 256), 256, 0, s>>>(n_bytes, GRID_N_CELLS / 8 * (max_cascade + 1), grid, bitfield, mean_out);
	for (uint32_t level = 1; level < CASCADES; ++level) {
		const uint32_t n = GRID_N_CELLS / 64;
		k_bitfield_max_pool<<<div_round_up(n, 256), 256, 0, s>>>(n, bitfield + (size_t)(level - 1) * GRID_N_CELLS / 8,
		                                                          bitfield + (size_t)level * GRID_N_CELLS / 8);
	}
	NGP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// host: effective camera matrix (glm quat_cast -> slerp(t=0, start == end) -> normalize -> mat3_cast)
// ------------------------------------------------------------------------------------------------

// ------------------------------------------------------------------------------------------------
// Rendering: NerfTracer (testbed_nerf.cu:2229-2503 init/advance, 2504-2659 trace, 948-1196
// generate_next_nerf_network_inputs / composite_kernel_nerf, 2164-2226 shade / compact), pinhole
// cameras, ERenderMode::Shade. Compaction uses atomic slots like the reference: rays are independent,
// so the image does not depend on their order.
// ------------------------------------------------------------------------------------------------
// random_val.cuh:162-291 (Burley 2019 scrambled Sobol)
__device__ uint32_t sobol_dim(uint32_t index, uint32_t dim) {
	// direction numbers of dims 0 and 1 (random_val.cuh:163-181)
	uint32_t X = 0;
	if (dim == 0) {
		X = 0;
#pragma unroll
		for (uint32_t bit = 0; bit < 32; ++bit) X ^= ((index >> bit) & 1u) * (0x80000000u >> bit);
	} else {
		uint32_t v = 0x80000000u;  // dim 1: v_k = v_{k-1} ^ (v_{k-1} >> 1)
#pragma unroll
		for (uint32_t bit = 0; bit < 32; ++bit) {
			X ^= ((index >> bit) & 1u) * v;
			v ^= v >> 1;
		}
	}
	return X;
}
__device__ __forceinline__ uint32_t hash_combine(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
__device__ __forceinline__ uint32_t reverse_bits32(uint32_t x) { return __builtin_bitreverse32(x); }
__device__ __forceinline__ uint32_t laine_karras(uint32_t x, uint32_t seed) {
	x += seed;
	x ^= x * 0x6c50b47cu;
	x ^= x * 0xb82f1e52u;
	x ^= x * 0xc7afe638u;
	x ^= x * 0x8d22f6e6u;
	return x;
}
__device__ __forceinline__ uint32_t nus_base2(uint32_t x, uint32_t seed) { return reverse_bits32(laine_karras(reverse_bits32(x), seed)); }
__device__ float ld_random_val(uint32_t index, uint32_t seed, uint32_t dim = 0) {
	const float S = (float)(1.0 / 4294967296.0);
	index = nus_base2(index, seed);
	return (float)nus_base2(sobol_dim(index, dim), hash_combine(seed, dim)) * S;
}
__device__ void ld_random_val_2d(uint32_t index, uint32_t seed, float* x, float* y) {
	const float S = (float)(1.0 / 4294967296.0);
	index = nus_base2(index, seed);
	*x = (float)nus_base2(sobol_dim(index, 0), hash_combine(seed, 0)) * S;
	*y = (float)nus_base2(sobol_dim(index, 1), hash_combine(seed, 1)) * S;
}
__device__ __forceinline__ float fractf_(float x) { return x - floorf(x); }
__device__ void ld_random_pixel_offset(uint32_t spp, float* ox, float* oy) {  // random_val.cuh:320-326
	float ax, ay, bx, by;
	ld_random_val_2d(0, 0xdeadbeefu, &ax, &ay);
	ld_random_val_2d(spp, 0xdeadbeefu, &bx, &by);
	*ox = fractf_(0.5f - ax + bx);
	*oy = fractf_(0.5f - ay + by);
}

// if_unoccupied_advance_to_next_occupied_voxel<MIP_FROM_DT = false> (testbed_nerf.cu:811-842)
__device__ float advance_to_occupied(float t, const Cone& cone, V3 o, V3 d, V3 idir, const uint8_t* bitfield, uint32_t min_mip,
                                     uint32_t max_mip, const Aabb& box) {
	while (true) {
		const V3 pos = v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);
		if (t >= 16384.0f || !aabb_contains(box, pos)) return 16384.0f;
		uint32_t mip = min(max(mip_from_pos(pos, CASCADES - 1), min_mip), max_mip);
		if (!bitfield || density_grid_occupied_at(pos, bitfield, mip)) return t;
		while (mip < max_mip && !density_grid_occupied_at(pos, bitfield, mip + 1)) ++mip;
		t = advance_to_next_voxel(t, cone, pos, d, idir, mip);
	}
}

struct Payload {  // NerfPayload (nerf.h:32-40)
	float o[3], d[3];
	float t, max_weight;
	uint32_t idx, n_steps, alive;
};

__global__ void k_render_init(RenderArgs a, Payload* __restrict__ pay, float* __restrict__ rgba) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t W = a.width, H = a.height;
	if (i >= W * H) return;
	const uint32_t x = i % W, y = i / W;
	float ox, oy;
	ld_random_pixel_offset(a.snap_to_pixel_centers ? 0u : a.sample_index, &ox, &oy);
	const float u = ((float)x + ox) / (float)W, v = ((float)y + oy) / (float)H;
	// uv_to_ray (common_device.cuh:443-510), screen_center = render_screen_center(1 - principal point)
	// (testbed.cu:852, 4376-4379, 4541) = the principal point, with
	// the training view's lens (render_with_lens_distortion, testbed.cu:845-846)
	float dx = (u - a.screen_center[0]) * (float)W / a.focal[0];
	float dy = (v - a.screen_center[1]) * (float)H / a.focal[1];
	lens_undistort(a.lens_mode, a.lens, &dx, &dy);
	const float* m = a.cam;
	V3 d = v3(m[0] * dx + m[3] * dy + m[6], m[1] * dx + m[4] * dy + m[7], m[2] * dx + m[5] * dy + m[8]);
	V3 o = v3(m[9] + d.x * a.near_distance, m[10] + d.y * a.near_distance, m[11] + d.z * a.near_distance);
	Payload p;
	p.max_weight = 0.f;
	p.idx = i;
	p.n_steps = 0;
	p.alive = 0;
	rgba[4 * (size_t)i] = rgba[4 * (size_t)i + 1] = rgba[4 * (size_t)i + 2] = rgba[4 * (size_t)i + 3] = 0.f;
	const float inv = 1.0f / sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
	d = v3(d.x * inv, d.y * inv, d.z * inv);
	p.o[0] = o.x; p.o[1] = o.y; p.o[2] = o.z;
	p.d[0] = d.x; p.d[1] = d.y; p.d[2] = d.z;
	const Aabb box{v3(a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]), v3(a.aabb_max[0], a.aabb_max[1], a.aabb_max[2])};
	float tmin, tmax;
	aabb_ray_intersect(box, o, d, &tmin, &tmax);
	float t = fmaxf(tmin, 0.0f) + 1e-6f;
	if (aabb_contains(box, v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z))) {
		// advance_pos_nerf (:844-900): jitter the start by a scrambled-Sobol fraction of a step
		const V3 idir = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
		const Cone cone = make_cone(a.cone_angle_constant);
		t = advance_n_steps(t, cone, ld_random_val(a.sample_index, i * 786433u));
		// min_mip = show_accel >= 0 ? show_accel : 0 (testbed_nerf.cu:2497)
		t = advance_to_occupied(t, cone, o, d, idir, a.bitfield, a.show_accel >= 0 ? (uint32_t)a.show_accel : 0u, a.max_mip, box);
		if (t < 16384.0f) p.alive = 1;
	}
	p.t = t;
	pay[i] = p;
}

// compact_kernel_nerf (:2198-2226)
__global__ void k_render_compact(uint32_t n, const Payload* __restrict__ src, const float* __restrict__ src_rgba,
                                 Payload* __restrict__ dst, float* __restrict__ dst_rgba, Payload* __restrict__ hit,
                                 float* __restrict__ hit_rgba, uint32_t* __restrict__ counters) {
	// One atomic per wave and list (the reference takes one per ray: ~2 M same-address atomics per
	// compaction at 1080p serialise in L2, ~10 ms). Slot order differs run to run, as with per-ray
	// atomics; every later pass is per ray (the frame is written through the payload's pixel index).
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const bool in = i < n;
	Payload p{};
	f32x4 c{0.f, 0.f, 0.f, 0.f};
	if (in) {
		p = src[i];
		c = *(const f32x4*)(src_rgba + 4 * (size_t)i);
	}
	const bool alive = in && p.alive, hitp = in && !p.alive && c[3] > 0.001f;
	const uint64_t ma = __ballot(alive), mh = __ballot(hitp);
	const uint32_t lane = __lane_id();
	const uint64_t below = (1ull << lane) - 1ull;
	uint32_t ba = 0, bh = 0;
	if (lane == 0) {
		if (ma) ba = atomicAdd(&counters[0], (uint32_t)__popcll(ma));
		if (mh) bh = atomicAdd(&counters[1], (uint32_t)__popcll(mh));
	}
	ba = (uint32_t)__shfl((int)ba, 0);
	bh = (uint32_t)__shfl((int)bh, 0);
	if (alive) {
		const uint32_t k = ba + (uint32_t)__popcll(ma & below);
		dst[k] = p;
		*(f32x4*)(dst_rgba + 4 * (size_t)k) = c;
	} else if (hitp) {
		const uint32_t k = bh + (uint32_t)__popcll(mh & below);
		hit[k] = p;
		*(f32x4*)(hit_rgba + 4 * (size_t)k) = c;
	}
}

// generate_next_nerf_network_inputs (:948-1014): coordinate (i, j) at row i + j * n
__global__ void k_render_inputs(RenderArgs a, uint32_t n, uint32_t n_steps, Payload* __restrict__ pay, float* __restrict__ coords) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	Payload& p = pay[i];
	if (!p.alive) return;
	const V3 o = v3(p.o[0], p.o[1], p.o[2]), d = v3(p.d[0], p.d[1], p.d[2]);
	const V3 idir = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
	const Aabb box{v3(a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]), v3(a.aabb_max[0], a.aabb_max[1], a.aabb_max[2])};
	const V3 diag = v3(box.mx.x - box.mn.x, box.mx.y - box.mn.y, box.mx.z - box.mn.z);
	const Cone cone = make_cone(a.cone_angle_constant);
	float t = p.t;
	for (uint32_t j = 0; j < n_steps; ++j) {
		t = advance_to_occupied(t, cone, o, d, idir, a.bitfield, a.show_accel >= 0 ? (uint32_t)a.show_accel : 0u, a.max_mip, box);
		if (t >= 16384.0f) {
			p.n_steps = j;
			return;
		}
		const float dt = calc_dt(t, cone);
		const V3 pos = v3(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
		float* c = coords + (size_t)(i + j * n) * 7;
		c[0] = (pos.x - box.mn.x) / diag.x; c[1] = (pos.y - box.mn.y) / diag.y; c[2] = (pos.z - box.mn.z) / diag.z;
		c[3] = warp_dt(dt);
		c[4] = (d.x + 1.0f) * 0.5f; c[5] = (d.y + 1.0f) * 0.5f; c[6] = (d.z + 1.0f) * 0.5f;
		t += dt;
	}
	p.t = t;
	p.n_steps = n_steps;
}

// composite_kernel_nerf (:1016-1196); network output RM [16 x stride]. The colour of a step by ERenderMode
// (:1183-1208): Shade the network's rgb; Normals normalize(-density'(raw) * d(raw density)/d(position)), the
// gradient in the coordinates' position rows (render_frame's grad); Positions (pos - 0.5) / 2 + 0.5, or with
// show_accel >= 0 the step's occupancy cell (mip = max(show_accel, mip_from_pos), red 1 - mip / 7, green and blue
// two pcg32 draws seeded by the cell); EncodingVis the warped position (the network's input); Depth dot(camera
// forward, pos - ray origin) * depth_scale; AO the step's alpha. pos = unwarp_position of the step's coordinate over
// the aabb the inputs were warped with. show_accel >= 0 also makes every step opaque (alpha 1, :1078-1080).
__global__ void k_render_composite(RenderArgs a, uint32_t n, uint32_t stride, uint32_t current_step, uint32_t n_steps,
                                   Payload* __restrict__ pay, float* __restrict__ rgba, const float* __restrict__ coords,
                                   const f16* __restrict__ out) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	Payload& p = pay[i];
	if (!p.alive) return;
	f32x4 c = *(const f32x4*)(rgba + 4 * (size_t)i);
	const uint32_t actual = p.n_steps;
	uint32_t j = 0;
	for (; j < actual; ++j) {
		const size_t r = i + (size_t)j * n;
		const float o0 = (float)out[r], o1 = (float)out[r + stride], o2 = (float)out[r + 2 * (size_t)stride];
		const float o3 = (float)out[r + 3 * (size_t)stride];
		const float T = 1.f - c[3];
		const float dt = unwarp_dt(coords[r * 7 + 3]);
		const float alpha = a.show_accel >= 0 ? 1.f : 1.f - ngp_expf_fast(-network_to_density(o3, a.density_activation) * dt);
		const float weight = alpha * T;
		float rgb[3];
		if (a.render_mode == RENDER_NORMALS) {
			const float dd = -network_to_density_derivative(o3, a.density_activation);
			const float nx = dd * coords[r * 7 + 0], ny = dd * coords[r * 7 + 1], nz = dd * coords[r * 7 + 2];
			const float inv = 1.0f / sqrtf(nx * nx + ny * ny + nz * nz);  // glm normalize (0 -> NaN, as the reference)
			rgb[0] = nx * inv; rgb[1] = ny * inv; rgb[2] = nz * inv;
		} else if (a.render_mode == RENDER_POSITIONS || a.render_mode == RENDER_DEPTH) {
			float pos[3];
#pragma unroll
			for (int k = 0; k < 3; ++k) pos[k] = coords[r * 7 + k] * (a.aabb_max[k] - a.aabb_min[k]) + a.aabb_min[k];
			if (a.render_mode == RENDER_POSITIONS && a.show_accel >= 0) {
				// :1190-1199: the cell of the cascade the march tested, coloured by its mip and a seeded pcg32
				const uint32_t mip = max((uint32_t)a.show_accel, mip_from_pos(v3(pos[0], pos[1], pos[2]), CASCADES - 1));
				const uint32_t res = GRIDSIZE >> mip;
				const int ix = (int)(pos[0] * (float)res), iy = (int)(pos[1] * (float)res), iz = (int)(pos[2] * (float)res);
				Pcg32Dev rng{0u, (1ull << 1u) | 1u};  // pcg32(initstate, initseq = 1)
				pcg_next(rng);
				rng.state += (uint64_t)(int64_t)(ix + iy * 232323 + iz * 727272);
				pcg_next(rng);
				rgb[0] = 1.f - (float)mip * (1.f / (float)(CASCADES - 1));
				rgb[1] = pcg_float(rng);
				rgb[2] = pcg_float(rng);
			} else if (a.render_mode == RENDER_POSITIONS) {
#pragma unroll
				for (int k = 0; k < 3; ++k) rgb[k] = (pos[k] - 0.5f) / 2.0f + 0.5f;
			} else {
				const float z = (a.cam[6] * (pos[0] - p.o[0]) + a.cam[7] * (pos[1] - p.o[1]) + a.cam[8] * (pos[2] - p.o[2])) * a.depth_scale;
				rgb[0] = rgb[1] = rgb[2] = z;
			}
		} else if (a.render_mode == RENDER_AO) {
			rgb[0] = rgb[1] = rgb[2] = alpha;
		} else if (a.render_mode == RENDER_ENCODING_VIS) {
#pragma unroll
			for (int k = 0; k < 3; ++k) rgb[k] = coords[r * 7 + k];  // warped_pos
		} else {
			rgb[0] = network_to_rgb(o0, a.rgb_activation);
			rgb[1] = network_to_rgb(o1, a.rgb_activation);
			rgb[2] = network_to_rgb(o2, a.rgb_activation);
		}
		c[0] += rgb[0] * weight;
		c[1] += rgb[1] * weight;
		c[2] += rgb[2] * weight;
		c[3] += weight;
		if (weight > p.max_weight) p.max_weight = weight;
		if (c[3] > (1.0f - a.min_transmittance)) {
			const float inv = 1.0f / c[3];
			c[0] *= inv; c[1] *= inv; c[2] *= inv; c[3] *= inv;
			break;
		}
	}
	if (j < n_steps) {
		p.alive = 0;
		p.n_steps = j + current_step;
	}
	*(f32x4*)(rgba + 4 * (size_t)i) = c;
}

// shade_kernel_nerf (:2164-2196) into the frame (pre-filled with the linear background), then the
// spp average (the render buffer's accumulation)
__global__ void k_render_shade(uint32_t n_hit, uint32_t linear_colors, uint32_t mode, const Payload* __restrict__ hit,
                               const float* __restrict__ hit_rgba, float* __restrict__ frame) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_hit) return;
	f32x4 c = *(const f32x4*)(hit_rgba + 4 * (size_t)i);
	if (mode == RENDER_NORMALS) {  // (0.5 n + 0.5) * a with n = normalize(rgb)
		const float inv = 1.0f / sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
		for (int k = 0; k < 3; ++k) c[k] = (0.5f * (c[k] * inv) + 0.5f) * c[3];
	} else if (!linear_colors && mode == RENDER_SHADE) {  // only Shade (and Slice) accumulate in linear colours
		c[0] = srgb_to_linear(c[0]); c[1] = srgb_to_linear(c[1]); c[2] = srgb_to_linear(c[2]);
	}
	float* f = frame + 4 * (size_t)hit[i].idx;
	for (int k = 0; k < 4; ++k) f[k] = c[k] + f[k] * (1.0f - c[3]);
}
__global__ void k_render_fill(uint32_t n, f32x4 bg, float* __restrict__ frame) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) *(f32x4*)(frame + 4 * (size_t)i) = bg;
}
__global__ void k_render_accumulate(uint32_t n4, float w, const float* __restrict__ frame, float* __restrict__ acc, bool first) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n4) acc[i] = (first ? 0.f : acc[i]) + frame[i] * w;
}

void render_frame(const RenderArgs& a, uint32_t spp, RenderWorkspace& ws, const std::function<void(uint32_t, const float*, f16*)>& infer,
                  float* out, hipStream_t s, const std::function<void(uint32_t, float*)>& grad) {
	NGP_CHECK((a.render_mode <= RENDER_DEPTH || a.render_mode == RENDER_ENCODING_VIS) && (a.render_mode != RENDER_NORMALS || grad),
	          "render: AO, Shade, Normals, Positions, Depth and EncodingVis are implemented");
	const uint32_t n_px = a.width * a.height;
	if (n_px == 0) return;
	const uint32_t MARCH_ITER = 10000, MIN_STEPS = 1, MAX_STEPS = 8, TARGET_QUERIES = 2 * 1024 * 1024;
	Payload* pay[2] = {(Payload*)ws.payload[0], (Payload*)ws.payload[1]};
	float* rgba[2] = {ws.rgba[0], ws.rgba[1]};
	Payload* hit = (Payload*)ws.payload_hit;
	for (uint32_t sidx = 0; sidx < spp; ++sidx) {
		RenderArgs r = a;
		r.sample_index = a.sample_index + sidx;
		k_render_fill<<<div_round_up(n_px, 256), 256, 0, s>>>(n_px, f32x4{a.background[0], a.background[1], a.background[2],
		                                                                    a.background[3]}, ws.frame);
		k_render_init<<<div_round_up(n_px, 128), 128, 0, s>>>(r, pay[0], rgba[0]);
		NGP_HIP(hipGetLastError());
		NGP_HIP(hipMemsetAsync(ws.counters, 0, 8, s));  // counters[1]: hits (whole trace)
		uint32_t n_alive = n_px, it = 1, db = 0;
		while (it < MARCH_ITER) {
			Payload* src = pay[db % 2];
			float* src_c = rgba[db % 2];
			Payload* dst = pay[(db + 1) % 2];
			float* dst_c = rgba[(db + 1) % 2];
			++db;
			NGP_HIP(hipMemsetAsync(ws.counters, 0, 4, s));
			k_render_compact<<<div_round_up(n_alive, 256), 256, 0, s>>>(n_alive, src, src_c, dst, dst_c, hit, ws.rgba_hit, ws.counters);
			NGP_HIP(hipGetLastError());
			NGP_HIP(hipMemcpyAsync(ws.host_counters, ws.counters, 8, hipMemcpyDeviceToHost, s));
			NGP_HIP(hipStreamSynchronize(s));
			n_alive = ws.host_counters[0];
			if (n_alive == 0) break;
			const uint32_t n_steps = std::min(std::max(TARGET_QUERIES / n_alive, MIN_STEPS), MAX_STEPS);
			k_render_inputs<<<div_round_up(n_alive, 128), 128, 0, s>>>(r, n_alive, n_steps, dst, ws.coords);
			NGP_HIP(hipGetLastError());
			const uint32_t n_el = next_multiple(n_alive * n_steps, 256);
			infer(n_el, ws.coords, ws.out);
			if (a.render_mode == RENDER_NORMALS) grad(n_el, ws.coords);
			k_render_composite<<<div_round_up(n_alive, 128), 128, 0, s>>>(r, n_alive, n_el, it, n_steps, dst, dst_c, ws.coords, ws.out);
			NGP_HIP(hipGetLastError());
			it += n_steps;
		}
		const uint32_t n_hit = ws.host_counters[1];
		if (n_hit) k_render_shade<<<div_round_up(n_hit, 256), 256, 0, s>>>(n_hit, a.linear_colors, a.render_mode, hit, ws.rgba_hit, ws.frame);
		k_render_accumulate<<<div_round_up(4 * n_px, 256), 256, 0, s>>>(4 * n_px, 1.0f / (float)spp, ws.frame, out, sidx == 0);
		NGP_HIP(hipGetLastError());
	}
}

size_t render_payload_bytes() { return sizeof(Payload); }

void effective_camera_matrix(const float xf[12], float out[12]) {
	// glm column-major m[c][r] = xf[3c + r]
	auto M = [&](int c, int r) { return xf[3 * c + r]; };
	const float fx = M(0, 0) - M(1, 1) - M(2, 2), fy = M(1, 1) - M(0, 0) - M(2, 2), fz = M(2, 2) - M(0, 0) - M(1, 1);
	const float fw = M(0, 0) + M(1, 1) + M(2, 2);
	int bi = 0;
	float big = fw;
	if (fx > big) { big = fx; bi = 1; }
	if (fy > big) { big = fy; bi = 2; }
	if (fz > big) { big = fz; bi = 3; }
	const float bv = sqrtf(big + 1.0f) * 0.5f, mult = 0.25f / bv;
	float w, x, y, z;
	switch (bi) {
		case 0: w = bv; x = (M(1, 2) - M(2, 1)) * mult; y = (M(2, 0) - M(0, 2)) * mult; z = (M(0, 1) - M(1, 0)) * mult; break;
		case 1: w = (M(1, 2) - M(2, 1)) * mult; x = bv; y = (M(0, 1) + M(1, 0)) * mult; z = (M(2, 0) + M(0, 2)) * mult; break;
		case 2: w = (M(2, 0) - M(0, 2)) * mult; x = (M(0, 1) + M(1, 0)) * mult; y = bv; z = (M(1, 2) + M(2, 1)) * mult; break;
		default: w = (M(0, 1) - M(1, 0)) * mult; x = (M(2, 0) + M(0, 2)) * mult; y = (M(1, 2) + M(2, 1)) * mult; z = bv; break;
	}
	// slerp(q, q, 0) takes the linear branch: q * 1 + q * 0 = q; then normalize
	const float len = sqrtf(w * w + x * x + y * y + z * z);
	if (len <= 0.f) { w = 1.f; x = y = z = 0.f; }
	else { const float inv = 1.0f / len; w *= inv; x *= inv; y *= inv; z *= inv; }
	const float qxx = x * x, qyy = y * y, qzz = z * z, qxz = x * z, qxy = x * y, qyz = y * z, qwx = w * x, qwy = w * y, qwz = w * z;
	out[0] = 1.f - 2.f * (qyy + qzz); out[1] = 2.f * (qxy + qwz); out[2] = 2.f * (qxz - qwy);
	out[3] = 2.f * (qxy - qwz); out[4] = 1.f - 2.f * (qxx + qzz); out[5] = 2.f * (qyz + qwx);
	out[6] = 2.f * (qxz + qwy); out[7] = 2.f * (qyz - qwx); out[8] = 1.f - 2.f * (qxx + qyy);
	out[9] = xf[9]; out[10] = xf[10]; out[11] = xf[11];
}

Dataset::~Dataset() {
	if (d_cams) (void)hipFree(d_cams);
	if (d_pixels) (void)hipFree(d_pixels);
}

}  // namespace nerf
}  // namespace ngp
