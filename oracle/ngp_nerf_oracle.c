/*
 * ngp_nerf_oracle.c — CPU restatement of the NeRF training kernels of src/testbed_nerf.cu.
 * TEST INFRASTRUCTURE ONLY (see ngp_oracle.c header). Sequential, deterministic: slots are assigned in
 * ray order, which is the multiset-equivalent of the reference's atomicAdd ordering.
 * Parity status: restated from code present in the reference (file:line per function); no golden
 * vectors exist in the reference for these kernels, and the reference cannot run here.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ngp_math.h" /* the engine's expf/logf: see the header */

#define EXPORT __attribute__((visibility("default")))

typedef struct { uint64_t state, inc; } orc_pcg32;
uint32_t orc_pcg32_next_uint(orc_pcg32* r);
float orc_pcg32_next_float(orc_pcg32* r);
void orc_pcg32_advance(orc_pcg32* r, int64_t delta);
void orc_pcg32_seed(orc_pcg32* r, uint64_t initstate, uint64_t initseq);
float orc_f16_to_f32(uint16_t h);
uint16_t orc_f32_to_f16(float f);

#define GRIDSIZE 128u
#define N_CELLS (GRIDSIZE * GRIDSIZE * GRIDSIZE)
#define CASCADES 8u
#define NSTEPS 1024u
#define SQRT3 1.73205080757f
#define MIN_STEP (SQRT3 / NSTEPS)
#define MAX_STEP (MIN_STEP * (1 << (CASCADES - 1)) * NSTEPS / GRIDSIZE)
#define MIN_OPT 0.01f

/* mirrors ngp_nerf_config / ngp_nerf_image of include/ngp_engine.h (same field order) */
typedef struct {
	float aabb_min[3], aabb_max[3];
	float cone_angle_constant;
	uint32_t max_cascade, snap_to_pixel_centers, random_bg_color, linear_colors, color_space_linear;
	float background_color[3];
	uint32_t rgb_activation, density_activation, loss_type;
	float near_distance;
	uint32_t target_batch_size;
} ocfg;

typedef struct {
	uint32_t width, height;
	float focal_length[2], principal_point[2];
	float xform[12];
	uint32_t lens_mode;
	float lens_params[4];
} oimg;

/* ---- lens models (common_device.cuh:288-378): 1 OpenCV {k1,k2,p1,p2}, 2 OpenCV fisheye {k1..k4} ---- */
static void lens_delta(uint32_t mode, const float* k, float u, float v, float* du, float* dv) {
	if (mode == 1) { /* opencv_lens_distortion_delta :289-303 */
		const float u2 = u * u, uv = u * v, v2 = v * v;
		const float r2 = u2 + v2;
		const float radial = k[0] * r2 + k[1] * r2 * r2;
		*du = u * radial + 2.0f * k[2] * uv + k[3] * (r2 + 2.0f * u2);
		*dv = v * radial + 2.0f * k[3] * uv + k[2] * (r2 + 2.0f * v2);
	} else if (mode == 2) { /* opencv_fisheye_lens_distortion_delta :305-327 */
		const float r = sqrtf(u * u + v * v);
		if (r > 2.220446049250313e-16f) {
			const float th = atanf(r), th2 = th * th, th4 = th2 * th2, th6 = th4 * th2, th8 = th4 * th4;
			const float thd = th * (1.0f + k[0] * th2 + k[1] * th4 + k[2] * th6 + k[3] * th8);
			*du = u * thd / r - u;
			*dv = v * thd / r - v;
		} else {
			*du = 0.0f; *dv = 0.0f;
		}
	} else {
		*du = 0.0f; *dv = 0.0f;
	}
}

/* iterative_lens_undistortion :330-369 (Newton, central differences, glm mat2 inverse) */
static void lens_undistort(uint32_t mode, const float* k, float* u, float* v) {
	if (mode != 1 && mode != 2) return;
	const float x0u = *u, x0v = *v;
	float xu = *u, xv = *v;
	for (uint32_t i = 0; i < 100; ++i) {
		const float s0 = fmaxf(1.1920928955078125e-07f, fabsf(1e-6f * xu));
		const float s1 = fmaxf(1.1920928955078125e-07f, fabsf(1e-6f * xv));
		float d0, d1, b00, b01, f00, f01, b10, b11, f10, f11;
		lens_delta(mode, k, xu, xv, &d0, &d1);
		lens_delta(mode, k, xu - s0, xv, &b00, &b01);
		lens_delta(mode, k, xu + s0, xv, &f00, &f01);
		lens_delta(mode, k, xu, xv - s1, &b10, &b11);
		lens_delta(mode, k, xu, xv + s1, &f10, &f11);
		const float j00 = 1.0f + (f00 - b00) / (2.0f * s0), j10 = (f10 - b10) / (2.0f * s1);
		const float j01 = (f01 - b01) / (2.0f * s0), j11 = 1.0f + (f11 - b11) / (2.0f * s1);
		const float od = 1.0f / (j00 * j11 - j10 * j01);
		const float i00 = j11 * od, i01 = -j01 * od, i10 = -j10 * od, i11 = j00 * od;
		const float ru = xu + d0 - x0u, rv = xv + d1 - x0v;
		const float su = i00 * ru + i10 * rv, sv = i01 * ru + i11 * rv;
		xu -= su; xv -= sv;
		if (su * su + sv * sv < 1e-10f) break;
	}
	*u = xu; *v = xv;
}

EXPORT void orc_lens_undistort(uint32_t mode, const float* k, float* u, float* v) { lens_undistort(mode, k, u, v); }

/* ---- stepping (testbed_nerf.cu:114-184) ---- */
static float to_step(float t, float c) {
	if (c <= 1e-5f) return t / MIN_STEP;
	float l = ngp_logf(1.0f + c);
	float a = (ngp_logf(MIN_STEP) - ngp_logf(l)) / l, b = (ngp_logf(MAX_STEP) - ngp_logf(l)) / l;
	float at = ngp_expf(a * l), bt = ngp_expf(b * l);
	if (t <= at) return (t - at) / MIN_STEP + a;
	else if (t <= bt) return ngp_div_rc(ngp_logf(t), l, 1.0f / l);
	else return (t - bt) / MAX_STEP + b;
}
static float from_step(float n, float c) {
	if (c <= 1e-5f) return n * MIN_STEP;
	float l = ngp_logf(1.0f + c);
	float a = (ngp_logf(MIN_STEP) - ngp_logf(l)) / l, b = (ngp_logf(MAX_STEP) - ngp_logf(l)) / l;
	float at = ngp_expf(a * l), bt = ngp_expf(b * l);
	if (n <= a) return (n - a) * MIN_STEP + at;
	else if (n <= b) return ngp_expf(n * l);
	else return (n - b) * MAX_STEP + bt;
}
static float calc_dt(float t, float c) { return from_step(to_step(t, c) + 1.0f, c) - t; }
static float sgn(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

static float dist_next_voxel(const float* pos, const float* dir, const float* idir, float res) {
	float p[3], t[3];
	for (int k = 0; k < 3; ++k) p[k] = res * (pos[k] - 0.5f);
	for (int k = 0; k < 3; ++k) t[k] = (floorf(p[k] + 0.5f + 0.5f * sgn(dir[k])) - p[k]) * idir[k];
	float m = fminf(fminf(t[0], t[1]), t[2]);
	return fmaxf(m / res, 0.0f);
}
static float advance_voxel(float t, float c, const float* pos, const float* dir, const float* idir, uint32_t mip) {
	float res = scalbnf((float)GRIDSIZE, -(int)mip);
	float tt = t + dist_next_voxel(pos, dir, idir, res);
	t = to_step(t, c);
	tt = to_step(tt, c);
	return from_step(t + ceilf(fmaxf(tt - t, 0.5f)), c);
}

/* testbed_nerf.cu:614-633 */
static uint32_t mip_pos(const float* p, uint32_t mc) {
	int e;
	float m = fmaxf(fmaxf(fabsf(p[0] - 0.5f), fabsf(p[1] - 0.5f)), fabsf(p[2] - 0.5f));
	frexpf(m, &e);
	int v = e + 1;
	if (v < 0) v = 0;
	if (v > (int)mc) v = (int)mc;
	return (uint32_t)v;
}
static uint32_t mip_dt(float dt, const float* p, uint32_t mc) {
	uint32_t m = mip_pos(p, mc);
	dt *= 2 * GRIDSIZE;
	if (dt < 1.0f) return m;
	int e;
	frexpf(dt, &e);
	int v = (int)m < e ? e : (int)m;
	if (v > (int)mc) v = (int)mc;
	return (uint32_t)v;
}

static uint32_t ebits(uint32_t v) {
	v = (v * 0x00010001u) & 0xFF0000FFu;
	v = (v * 0x00000101u) & 0x0F00F00Fu;
	v = (v * 0x00000011u) & 0xC30C30C3u;
	v = (v * 0x00000005u) & 0x49249249u;
	return v;
}
/* tcnn morton3D with x in bit 0 (round trip of morton3D_invert(idx>>0) = x, testbed_nerf.cu:518-520) */
EXPORT uint32_t orc_morton3D(uint32_t x, uint32_t y, uint32_t z) { return ebits(x) | (ebits(y) << 1) | (ebits(z) << 2); }
EXPORT uint32_t orc_morton3D_invert(uint32_t x) {
	x = x & 0x49249249u;
	x = (x | (x >> 2)) & 0xc30c30c3u;
	x = (x | (x >> 4)) & 0x0f00f00fu;
	x = (x | (x >> 8)) & 0xff0000ffu;
	x = (x | (x >> 16)) & 0x0000ffffu;
	return x;
}

/* testbed_nerf.cu:433-457 */
static uint32_t grid_idx_at(const float* p, uint32_t mip) {
	float s = scalbnf(1.0f, -(int)mip), q[3];
	for (int k = 0; k < 3; ++k) q[k] = (p[k] - 0.5f) * s + 0.5f;
	int i[3];
	for (int k = 0; k < 3; ++k) i[k] = (int)(q[k] * (float)GRIDSIZE);
	for (int k = 0; k < 3; ++k)
		if (i[k] < 0 || i[k] >= (int)GRIDSIZE) return 0xFFFFFFFFu;
	return orc_morton3D((uint32_t)i[0], (uint32_t)i[1], (uint32_t)i[2]);
}
static int occupied(const float* p, const uint8_t* bf, uint32_t mip) {
	uint32_t idx = grid_idx_at(p, mip);
	if (idx == 0xFFFFFFFFu) return 0;
	return (bf[idx / 8 + N_CELLS * mip / 8] >> (idx % 8)) & 1;
}

static int contains(const ocfg* c, const float* p) {
	for (int k = 0; k < 3; ++k)
		if (!(p[k] >= c->aabb_min[k] && p[k] <= c->aabb_max[k])) return 0;
	return 1;
}
/* bounding_box.cuh:163-216 */
static void ray_box(const ocfg* c, const float* o, const float* d, float* tmin_o, float* tmax_o) {
	float tmin = (c->aabb_min[0] - o[0]) / d[0], tmax = (c->aabb_max[0] - o[0]) / d[0], tt;
	if (tmin > tmax) { tt = tmin; tmin = tmax; tmax = tt; }
	float tymin = (c->aabb_min[1] - o[1]) / d[1], tymax = (c->aabb_max[1] - o[1]) / d[1];
	if (tymin > tymax) { tt = tymin; tymin = tymax; tymax = tt; }
	if (tmin > tymax || tymin > tmax) { *tmin_o = *tmax_o = 3.402823466e+38f; return; }
	if (tymin > tmin) tmin = tymin;
	if (tymax < tmax) tmax = tymax;
	float tzmin = (c->aabb_min[2] - o[2]) / d[2], tzmax = (c->aabb_max[2] - o[2]) / d[2];
	if (tzmin > tzmax) { tt = tzmin; tzmin = tzmax; tzmax = tt; }
	if (tmin > tzmax || tzmin > tmax) { *tmin_o = *tmax_o = 3.402823466e+38f; return; }
	if (tzmin > tmin) tmin = tzmin;
	if (tzmax < tmax) tmax = tzmax;
	*tmin_o = tmin; *tmax_o = tmax;
}

/* get_xform_given_rolling_shutter with start == end, t = 0 (common_device.cuh:401-408): glm quat_cast,
 * slerp (linear branch returns the input), normalize, mat3_cast. xf column-major m[c][r] = xf[3c+r]. */
EXPORT void orc_camera_matrix(const float* xf, float* out) {
#define MM(c, r) xf[3 * (c) + (r)]
	float fx = MM(0, 0) - MM(1, 1) - MM(2, 2), fy = MM(1, 1) - MM(0, 0) - MM(2, 2), fz = MM(2, 2) - MM(0, 0) - MM(1, 1);
	float fw = MM(0, 0) + MM(1, 1) + MM(2, 2);
	int bi = 0;
	float big = fw;
	if (fx > big) { big = fx; bi = 1; }
	if (fy > big) { big = fy; bi = 2; }
	if (fz > big) { big = fz; bi = 3; }
	float bv = sqrtf(big + 1.0f) * 0.5f, mu = 0.25f / bv, q[4]; /* w x y z */
	if (bi == 0) { q[0] = bv; q[1] = (MM(1, 2) - MM(2, 1)) * mu; q[2] = (MM(2, 0) - MM(0, 2)) * mu; q[3] = (MM(0, 1) - MM(1, 0)) * mu; }
	else if (bi == 1) { q[0] = (MM(1, 2) - MM(2, 1)) * mu; q[1] = bv; q[2] = (MM(0, 1) + MM(1, 0)) * mu; q[3] = (MM(2, 0) + MM(0, 2)) * mu; }
	else if (bi == 2) { q[0] = (MM(2, 0) - MM(0, 2)) * mu; q[1] = (MM(0, 1) + MM(1, 0)) * mu; q[2] = bv; q[3] = (MM(1, 2) + MM(2, 1)) * mu; }
	else { q[0] = (MM(0, 1) - MM(1, 0)) * mu; q[1] = (MM(2, 0) + MM(0, 2)) * mu; q[2] = (MM(1, 2) + MM(2, 1)) * mu; q[3] = bv; }
#undef MM
	float len = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
	if (len <= 0.f) { q[0] = 1.f; q[1] = q[2] = q[3] = 0.f; }
	else { float inv = 1.0f / len; for (int k = 0; k < 4; ++k) q[k] *= inv; }
	float w = q[0], x = q[1], y = q[2], z = q[3];
	float xx = x * x, yy = y * y, zz = z * z, xz = x * z, xy = x * y, yz = y * z, wx = w * x, wy = w * y, wz = w * z;
	out[0] = 1.f - 2.f * (yy + zz); out[1] = 2.f * (xy + wz); out[2] = 2.f * (xz - wy);
	out[3] = 2.f * (xy - wz); out[4] = 1.f - 2.f * (xx + zz); out[5] = 2.f * (yz + wx);
	out[6] = 2.f * (xz + wy); out[7] = 2.f * (yz - wx); out[8] = 1.f - 2.f * (xx + yy);
	out[9] = xf[9]; out[10] = xf[10]; out[11] = xf[11];
}

static void rand_uv(orc_pcg32* r, const oimg* im, int snap, float* u, float* v) {
	*u = orc_pcg32_next_float(r);
	*v = orc_pcg32_next_float(r);
	if (snap) {
		int px = (int)(*u * (float)im->width), py = (int)(*v * (float)im->height);
		if (px < 0) px = 0;
		if (px > (int)im->width - 1) px = (int)im->width - 1;
		if (py < 0) py = 0;
		if (py > (int)im->height - 1) py = (int)im->height - 1;
		*u = ((float)px + 0.5f) / (float)im->width;
		*v = ((float)py + 0.5f) / (float)im->height;
	}
}
static uint64_t pix(float u, float v, const oimg* im) {
	int px = (int)(u * (float)im->width), py = (int)(v * (float)im->height);
	if (px < 0) px = 0;
	if (px > (int)im->width - 1) px = (int)im->width - 1;
	if (py < 0) py = 0;
	if (py > (int)im->height - 1) py = (int)im->height - 1;
	return (uint64_t)px + (uint64_t)py * im->width;
}

typedef struct { int valid; float o[3], d[3], dn[3], idir[3], startt, cone; } oray;

static oray setup(const ocfg* c, const oimg* ims, const float* cams, const uint32_t* const* px, uint32_t n_img, uint32_t ig,
                  uint32_t n_div, orc_pcg32 rng) {
	oray r;
	memset(&r, 0, sizeof(r));
	uint32_t img = ((ig * n_img) / n_div) % n_img; /* image_idx, testbed_nerf.cu:1317-1338 */
	const oimg* im = &ims[img];
	orc_pcg32_advance(&rng, (int64_t)ig * 16);
	float u, v;
	rand_uv(&rng, im, c->snap_to_pixel_centers != 0, &u, &v);
	if (px[img][pix(u, v, im)] == 0x00FF00FFu) return r;
	(void)orc_pcg32_next_float(&rng); /* motionblur_time */
	const float* m = cams + 12 * img;
	float dx = (u - im->principal_point[0]) * (float)im->width / im->focal_length[0];
	float dy = (v - im->principal_point[1]) * (float)im->height / im->focal_length[1];
	lens_undistort(im->lens_mode, im->lens_params, &dx, &dy);
	float dz = 1.0f;
	r.d[0] = m[0] * dx + m[3] * dy + m[6] * dz;
	r.d[1] = m[1] * dx + m[4] * dy + m[7] * dz;
	r.d[2] = m[2] * dx + m[5] * dy + m[8] * dz;
	r.o[0] = m[9]; r.o[1] = m[10]; r.o[2] = m[11];
	float inv = 1.0f / sqrtf(r.d[0] * r.d[0] + r.d[1] * r.d[1] + r.d[2] * r.d[2]);
	for (int k = 0; k < 3; ++k) r.dn[k] = r.d[k] * inv;
	float tmin, tmax;
	ray_box(c, r.o, r.dn, &tmin, &tmax);
	r.cone = c->cone_angle_constant;
	tmin = fmaxf(tmin, 0.0f);
	r.startt = from_step(to_step(tmin, r.cone) + orc_pcg32_next_float(&rng), r.cone);
	for (int k = 0; k < 3; ++k) r.idir[k] = 1.0f / r.dn[k];
	r.valid = 1;
	return r;
}

/* generate_training_samples_nerf (testbed_nerf.cu:1382-1658) */
EXPORT void orc_nerf_generate_samples(const ocfg* c, const oimg* ims, const uint32_t* const* px, uint32_t n_img, uint32_t n_rays,
                                      uint32_t ray_offset, uint32_t n_div, orc_pcg32 rng, uint32_t max_samples, const uint8_t* bf,
                                      uint32_t* ray_indices, float* rays, uint32_t* numsteps, float* coords, uint32_t* counters) {
	float* cams = (float*)malloc(sizeof(float) * 12 * n_img);
	for (uint32_t i = 0; i < n_img; ++i) orc_camera_matrix(ims[i].xform, cams + 12 * i);
	uint32_t total = 0, kept = 0;
	float diag[3];
	for (int k = 0; k < 3; ++k) diag[k] = c->aabb_max[k] - c->aabb_min[k];
	/* The reference marches each ray twice (count, then write) and takes its base from an atomic
	 * counter; here the slots follow ray order (a prefix over the counts). Pass 1 counts
	 * every ray's occupied steps (rays are independent: parallel), the prefix runs in ray order, pass 2
	 * re-marches the kept rays and writes their samples. */
	uint32_t* cnt = (uint32_t*)calloc(n_rays ? n_rays : 1, sizeof(uint32_t));
	uint32_t* slot = (uint32_t*)malloc(sizeof(uint32_t) * (n_rays ? n_rays : 1));
	uint32_t* basev = (uint32_t*)malloc(sizeof(uint32_t) * (n_rays ? n_rays : 1));
	#pragma omp parallel for schedule(dynamic, 64)
	for (uint32_t i = 0; i < n_rays; ++i) {
		uint32_t ig = i + ray_offset;
		oray r = setup(c, ims, cams, px, n_img, ig, n_div ? n_div : n_rays, rng);
		if (!r.valid) continue;
		uint32_t j = 0;
		float t = r.startt, pos[3];
		for (;;) {
			for (int k = 0; k < 3; ++k) pos[k] = r.o[k] + t * r.dn[k];
			if (!(contains(c, pos) && j < NSTEPS)) break;
			float dt = calc_dt(t, r.cone);
			uint32_t mip = mip_dt(dt, pos, c->max_cascade);
			if (occupied(pos, bf, mip)) { ++j; t += dt; }
			else t = advance_voxel(t, r.cone, pos, r.dn, r.idir, mip);
		}
		cnt[i] = j;
	}
	for (uint32_t i = 0; i < n_rays; ++i) {
		slot[i] = 0xffffffffu;
		const uint32_t j = cnt[i];
		if (j == 0) continue;
		uint32_t base = total;
		total += j;
		if (base + j > max_samples) continue;
		slot[i] = kept++;
		basev[i] = base;
	}
	#pragma omp parallel for schedule(dynamic, 64)
	for (uint32_t i = 0; i < n_rays; ++i) {
		if (slot[i] == 0xffffffffu) continue;
		uint32_t ig = i + ray_offset;
		oray r = setup(c, ims, cams, px, n_img, ig, n_div ? n_div : n_rays, rng);
		const uint32_t s = slot[i], j = cnt[i], base = basev[i];
		ray_indices[s] = ig;
		for (int k = 0; k < 3; ++k) { rays[6 * s + k] = r.o[k]; rays[6 * s + 3 + k] = r.d[k]; }
		numsteps[2 * s] = j;
		numsteps[2 * s + 1] = base;
		uint32_t jj = 0;
		float t = r.startt, pos[3];
		for (;;) {
			for (int k = 0; k < 3; ++k) pos[k] = r.o[k] + t * r.dn[k];
			if (!(contains(c, pos) && jj < j)) break;
			float dt = calc_dt(t, r.cone);
			uint32_t mip = mip_dt(dt, pos, c->max_cascade);
			if (occupied(pos, bf, mip)) {
				float* co = coords + (size_t)(base + jj) * 7;
				for (int k = 0; k < 3; ++k) co[k] = (pos[k] - c->aabb_min[k]) / diag[k];
				float maxs = MIN_STEP * (1 << (CASCADES - 1));
				co[3] = (dt - MIN_STEP) / (maxs - MIN_STEP);
				for (int k = 0; k < 3; ++k) co[4 + k] = (r.dn[k] + 1.0f) * 0.5f;
				++jj;
				t += dt;
			} else {
				t = advance_voxel(t, r.cone, pos, r.dn, r.idir, mip);
			}
		}
	}
	free(cnt); free(slot); free(basev);
	counters[0] = kept;
	counters[1] = total;
	free(cams);
}

static float s2l(float s) { return s <= 0.04045f ? s / 12.92f : powf((s + 0.055f) / 1.055f, 2.4f); }
static float l2s(float l) { return l < 0.0031308f ? 12.92f * l : 1.055f * powf(l, 0.41666f) - 0.055f; }
static float logistic(float x) { return 1.0f / (1.0f + ngp_expf(-x)); }
static float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }
/* testbed_nerf.cu:317-378 (ngp_expf for the reference's __expf) */
static float to_rgb(float v, uint32_t a) {
	switch (a) { case 0: return v; case 1: return v > 0 ? v : 0; case 2: return logistic(v); default: return ngp_expf(clampf(v, -10.f, 10.f)); }
}
static float to_rgb_d(float v, uint32_t a) {
	switch (a) { case 0: return 1; case 1: return v > 0 ? 1.f : 0.f; case 2: { float d = logistic(v); return d * (1 - d); } default: return ngp_expf(clampf(v, -10.f, 10.f)); }
}
static float to_dens(float v, uint32_t a) {
	switch (a) { case 0: return v; case 1: return v > 0 ? v : 0; case 2: return logistic(v); default: return ngp_expf(v); }
}
static float to_dens_d(float v, uint32_t a) {
	switch (a) { case 0: return 1; case 1: return v > 0 ? 1.f : 0.f; case 2: { float d = logistic(v); return d * (1 - d); } default: return ngp_expf(clampf(v, -15.f, 15.f)); }
}
/* testbed_nerf.cu:186-276, 1340-1355 */
static void lossg(float tgt, float p, uint32_t type, float* l, float* g) {
	float d = p - tgt;
	switch (type) {
		case 6: { float den = p * p + 1e-2f; *l = d * d / den; *g = 2.0f * d / den; return; }
		case 1: *l = fabsf(d); *g = copysignf(1.0f, d); return;
		case 2: { float den = fabsf(p) + 1e-2f; *l = fabsf(d) / den; *g = copysignf(1.0f / den, d); return; }
		case 3: { float den = 0.5f * (fabsf(p) + fabsf(tgt)) + 1e-2f; *l = fabsf(d) / den; *g = copysignf(1.0f / den, d); return; }
		case 4: {
			float al = 0.1f, ad = fabsf(d), sq = 0.5f / al * d * d;
			*l = (ad > al ? (ad - 0.5f * al) : sq) / 5.0f;
			*g = (ad > al ? (d > 0 ? 1.0f : -1.0f) : (d / al)) / 5.0f;
			return;
		}
		case 5: { float dv = fabsf(d) + 1.0f; *l = ngp_logf(dv); *g = copysignf(1.0f / dv, d); return; }
		default: *l = d * d; *g = 2.0f * d; return;
	}
}

/* The error map deposit of one compacted ray (testbed_nerf.cu:1869-1899, no sharpness factor): the mean
 * loss split bilinearly over the texels around uv * res - 0.5; idx clamped with the image's resolution. */
static void deposit_error(float* em, uint32_t w, uint32_t h, const oimg* im, uint32_t img, float u, float v, float ml) {
	const float rx = (float)w, ry = (float)h;
	const float px = fminf(fmaxf(u * rx - 0.5f, 0.0f), rx - (1.0f + 1e-4f));
	const float py = fminf(fmaxf(v * ry - 0.5f, 0.0f), ry - (1.0f + 1e-4f));
	const int ix0 = (int)px, iy0 = (int)py;
	const float wx = px - (float)ix0, wy = py - (float)iy0;
	int ix = ix0 < 0 ? 0 : ix0, iy = iy0 < 0 ? 0 : iy0;
	if (ix > (int)im->width - 2) ix = (int)im->width - 2;
	if (iy > (int)im->height - 2) iy = (int)im->height - 2;
	float* e = em + (size_t)img * w * h;
	e[(size_t)iy * w + ix] += (1 - wx) * (1 - wy) * ml;
	e[(size_t)iy * w + ix + 1] += wx * (1 - wy) * ml;
	e[(size_t)(iy + 1) * w + ix] += (1 - wx) * wy * ml;
	e[(size_t)(iy + 1) * w + ix + 1] += wx * wy * ml;
}

/* compute_loss_kernel_train_nerf (testbed_nerf.cu:1660-2012); network_output fp16 bits [n x 16];
 * dloss fp16 bits [max_c x 16] (rows 0..3 written); error_map [n_img][em_h][em_w] or NULL. */
EXPORT void orc_nerf_compute_loss_em(const ocfg* c, const oimg* ims, const uint32_t* const* px, uint32_t n_img, uint32_t n_rays,
                                     uint32_t n_div, orc_pcg32 rng0, uint32_t max_c, uint32_t ray_counter, const uint16_t* out16,
                                     const uint32_t* ray_indices, const float* rays, uint32_t* numsteps, const float* coords_in,
                                     float* coords_out, uint16_t* dloss, float* loss, uint32_t* compacted_counter, float mean_density,
                                     float loss_scale, float* error_map, uint32_t em_w, uint32_t em_h) {
	uint32_t ctotal = 0;
	float diag[3];
	for (int k = 0; k < 3; ++k) diag[k] = c->aabb_max[k] - c->aabb_min[k];
	const float maxs = MIN_STEP * (1 << (CASCADES - 1));
	for (uint32_t i = 0; i < ray_counter && i < n_rays; ++i) {
		uint32_t ns = numsteps[2 * i], base = numsteps[2 * i + 1];
		const uint16_t* o = out16 + (size_t)base * 16;
		const float* ci = coords_in + (size_t)base * 7;
		float t = 1.f, rgb_ray[3] = {0, 0, 0};
		uint32_t cn = 0;
		for (; cn < ns; ++cn) {
			if (t < 1e-4f) break;
			float dt = ci[(size_t)cn * 7 + 3] * (maxs - MIN_STEP) + MIN_STEP;
			float dens = to_dens(orc_f16_to_f32(o[cn * 16 + 3]), c->density_activation);
			float alpha = 1.f - ngp_expf(-dens * dt), w = alpha * t;
			for (int k = 0; k < 3; ++k) rgb_ray[k] += w * to_rgb(orc_f16_to_f32(o[cn * 16 + k]), c->rgb_activation);
			t *= (1.f - alpha);
		}
		uint32_t ray_idx = ray_indices[i];
		orc_pcg32 rng = rng0;
		orc_pcg32_advance(&rng, (int64_t)ray_idx * 16);
		uint32_t img = ((ray_idx * n_img) / (n_div ? n_div : n_rays)) % n_img;
		const oimg* im = &ims[img];
		float u, v;
		rand_uv(&rng, im, c->snap_to_pixel_centers != 0, &u, &v);
		orc_pcg32_advance(&rng, 1);
		float bg[3] = {c->background_color[0], c->background_color[1], c->background_color[2]};
		if (c->random_bg_color) for (int k = 0; k < 3; ++k) bg[k] = orc_pcg32_next_float(&rng);
		for (int k = 0; k < 3; ++k) bg[k] = s2l(bg[k]);
		uint32_t raw = px[img][pix(u, v, im)];
		float tex[4];
		if (raw == 0x00FF00FFu) tex[0] = tex[1] = tex[2] = tex[3] = -1.0f;
		else {
			float a = (float)(raw >> 24) * (1.0f / 255.0f);
			for (int k = 0; k < 3; ++k) tex[k] = s2l((float)((raw >> (8 * k)) & 0xff) * (1.0f / 255.0f)) * a;
			tex[3] = a;
		}
		float es = expf(0.6931471805599453f * 0.0f), tgt[3];
		if (c->linear_colors || c->color_space_linear) {
			for (int k = 0; k < 3; ++k) tgt[k] = es * tex[k] + (1.0f - tex[3]) * bg[k];
			if (!c->linear_colors) for (int k = 0; k < 3; ++k) { tgt[k] = l2s(tgt[k]); bg[k] = l2s(bg[k]); }
		} else {
			for (int k = 0; k < 3; ++k) bg[k] = l2s(bg[k]);
			if (tex[3] > 0) for (int k = 0; k < 3; ++k) tgt[k] = l2s(es * tex[k] / tex[3]) * tex[3] + (1.0f - tex[3]) * bg[k];
			else for (int k = 0; k < 3; ++k) tgt[k] = bg[k];
		}
		if (cn == ns) for (int k = 0; k < 3; ++k) rgb_ray[k] += t * bg[k];
		uint32_t cbase = ctotal;
		ctotal += cn;
		uint32_t mn = max_c < cbase ? max_c : cbase;
		uint32_t cnum = (max_c - mn) < cn ? (max_c - mn) : cn;
		numsteps[2 * i] = cnum;
		numsteps[2 * i + 1] = cbase;
		if (cnum == 0) continue;
		float l[3], g[3];
		for (int k = 0; k < 3; ++k) lossg(tgt[k], rgb_ray[k], c->loss_type, &l[k], &g[k]);
		if (loss) loss[i] = ((l[0] + l[1] + l[2]) / 3.0f) / (float)n_rays;
		if (error_map) deposit_error(error_map, em_w, em_h, im, img, u, v, (l[0] + l[1] + l[2]) / 3.0f);
		float ls = loss_scale / (float)n_rays;
		float l2reg = c->rgb_activation == 3 ? 1e-4f : 0.0f, l1d = mean_density < MIN_OPT ? 1e-4f : 0.0f;
		const float* ray = rays + (size_t)i * 6;
		float r2[3] = {0, 0, 0};
		t = 1.0f;
		for (uint32_t j = 0; j < cnum; ++j) {
			const float* cc = ci + (size_t)j * 7;
			memcpy(coords_out + (size_t)(cbase + j) * 7, cc, 7 * sizeof(float));
			float pos[3], dd[3];
			for (int k = 0; k < 3; ++k) { pos[k] = c->aabb_min[k] + cc[k] * diag[k]; dd[k] = pos[k] - ray[k]; }
			float depth = sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
			float dt = cc[3] * (maxs - MIN_STEP) + MIN_STEP;
			float ov[4], rgb[3];
			for (int k = 0; k < 4; ++k) ov[k] = orc_f16_to_f32(o[j * 16 + k]);
			for (int k = 0; k < 3; ++k) rgb[k] = to_rgb(ov[k], c->rgb_activation);
			float dens = to_dens(ov[3], c->density_activation);
			float alpha = 1.f - ngp_expf(-dens * dt), w = alpha * t;
			for (int k = 0; k < 3; ++k) r2[k] += w * rgb[k];
			t *= (1.0f - alpha);
			float suf[3];
			for (int k = 0; k < 3; ++k) suf[k] = rgb_ray[k] - r2[k];
			uint16_t* dl = dloss + (size_t)(cbase + j) * 16;
			for (int k = 0; k < 3; ++k)
				dl[k] = orc_f32_to_f16(ls * (w * g[k] * to_rgb_d(ov[k], c->rgb_activation) + fmaxf(0.0f, l2reg * ov[k])));
			float dotv = g[0] * (t * rgb[0] - suf[0]) + g[1] * (t * rgb[1] - suf[1]) + g[2] * (t * rgb[2] - suf[2]);
			float dmlp = to_dens_d(ov[3], c->density_activation) * (dt * (dotv + 0.0f));
			dl[3] = orc_f32_to_f16(ls * dmlp + (ov[3] < 0.0f ? -l1d : 0.0f) + (ov[3] > -10.0f && depth < c->near_distance ? 1e-4f : 0.0f));
		}
	}
	*compacted_counter = ctotal;
}
EXPORT void orc_nerf_compute_loss(const ocfg* c, const oimg* ims, const uint32_t* const* px, uint32_t n_img, uint32_t n_rays,
                                  uint32_t n_div, orc_pcg32 rng0, uint32_t max_c, uint32_t ray_counter, const uint16_t* out16,
                                  const uint32_t* ray_indices, const float* rays, uint32_t* numsteps, const float* coords_in,
                                  float* coords_out, uint16_t* dloss, float* loss, uint32_t* compacted_counter, float mean_density,
                                  float loss_scale) {
	orc_nerf_compute_loss_em(c, ims, px, n_img, n_rays, n_div, rng0, max_c, ray_counter, out16, ray_indices, rays, numsteps,
	                         coords_in, coords_out, dloss, loss, compacted_counter, mean_density, loss_scale, NULL, 0, 0);
}

/* generate_grid_samples_nerf_nonuniform (testbed_nerf.cu:635-676) */
EXPORT void orc_nerf_grid_samples(const ocfg* c, uint32_t n, orc_pcg32 rng0, uint32_t step, const float* grid, uint32_t n_casc,
                                  float thresh, float* out, uint32_t* indices) {
	for (uint32_t i = 0; i < n; ++i) {
		orc_pcg32 rng = rng0;
		orc_pcg32_advance(&rng, (int64_t)i * 4);
		uint32_t level = (uint32_t)(orc_pcg32_next_float(&rng) * n_casc) % n_casc, idx = 0;
		for (uint32_t j = 0; j < 10; ++j) {
			idx = ((i + step * n) * 56924617u + j * 19349663u + 96925573u) % N_CELLS;
			idx += level * N_CELLS;
			if (grid[idx] > thresh) break;
		}
		uint32_t p = idx % N_CELLS;
		uint32_t x = orc_morton3D_invert(p), y = orc_morton3D_invert(p >> 1), z = orc_morton3D_invert(p >> 2);
		float r[3];
		for (int k = 0; k < 3; ++k) r[k] = orc_pcg32_next_float(&rng);
		float s = scalbnf(1.0f, (int)level), xyz[3] = {(float)x, (float)y, (float)z};
		for (int k = 0; k < 3; ++k) {
			float pp = ((xyz[k] + r[k]) / (float)GRIDSIZE - 0.5f) * s + 0.5f;
			out[(size_t)i * 3 + k] = (pp - c->aabb_min[k]) / (c->aabb_max[k] - c->aabb_min[k]);
		}
		indices[i] = idx;
	}
}

/* splat (:678-702), ema (:731-754) */
EXPORT void orc_nerf_grid_splat_ema(uint32_t n, const uint32_t* indices, const uint16_t* density16, uint32_t act, uint32_t n_el,
                                    float decay, float* grid) {
	float* tmp = (float*)calloc(n_el, sizeof(float));
	for (uint32_t i = 0; i < n; ++i) {
		float th = to_dens(orc_f16_to_f32(density16[i]), act) * scalbnf(MIN_STEP, 0);
		if (th > tmp[indices[i]] || (tmp[indices[i]] == 0.f)) {
			/* atomicMax on the uint bits: the same as a float max for non-negative values */
			uint32_t a, b;
			memcpy(&a, &th, 4);
			memcpy(&b, &tmp[indices[i]], 4);
			if (a > b) tmp[indices[i]] = th;
		}
	}
	for (uint32_t i = 0; i < n_el; ++i) {
		float prev = grid[i];
		grid[i] = prev < 0.f ? prev : fmaxf(prev * decay, tmp[i]);
	}
	free(tmp);
}

/* update_density_grid_mean_and_bitfield (:3538-3567), grid_to_bitfield (:762-786), bitfield_max_pool
 * (:788-809). The reference's mean is reduce_sum(max(v,0)/N) over cascade 0 (:3544-3551), a device
 * reduction whose float order is unspecified. The contract fixes one order, and this restatement
 * follows it step for step so the mean (and every bitfield bit that depends on it) is bit-exact:
 * 512 partials, partial b = a 256-wide pairwise tree over lanes t of the running sums
 * acc_t = sum_{k = t, t+256, ..} max(v[b*4096+k], 0)/N (in k order); then a 512-wide pairwise tree of
 * the partials. Both trees add s[t] += s[t+off] for off = width/2 .. 1. */
EXPORT float orc_nerf_grid_mean(const float* grid) {
	const uint32_t blocks = 512, threads = 256, per_block = N_CELLS / 512;
	float partial[512], s[512];
	for (uint32_t b = 0; b < blocks; ++b) {
		for (uint32_t t = 0; t < threads; ++t) {
			float acc = 0.f;
			for (uint32_t k = t; k < per_block; k += threads) acc += fmaxf(grid[b * per_block + k], 0.f) / (float)N_CELLS;
			s[t] = acc;
		}
		for (uint32_t off = threads / 2; off > 0; off >>= 1)
			for (uint32_t t = 0; t < off; ++t) s[t] += s[t + off];
		partial[b] = s[0];
	}
	for (uint32_t off = blocks / 2; off > 0; off >>= 1)
		for (uint32_t t = 0; t < off; ++t) partial[t] += partial[t + off];
	return partial[0];
}
EXPORT void orc_nerf_grid_bitfield(const float* grid, uint32_t max_cascade, float mean, uint8_t* bf) {
	uint32_t n_bytes = N_CELLS / 8 * CASCADES, n_nz = N_CELLS / 8 * (max_cascade + 1);
	float th = fminf(MIN_OPT, mean);
	for (uint32_t i = 0; i < n_bytes; ++i) {
		if (i >= n_nz) { bf[i] = 0; continue; }
		uint8_t b = 0;
		for (uint32_t j = 0; j < 8; ++j) b |= grid[i * 8 + j] > th ? (uint8_t)(1u << j) : 0;
		bf[i] = b;
	}
	for (uint32_t level = 1; level < CASCADES; ++level) {
		const uint8_t* prev = bf + (size_t)(level - 1) * N_CELLS / 8;
		uint8_t* next = bf + (size_t)level * N_CELLS / 8;
		for (uint32_t i = 0; i < N_CELLS / 64; ++i) {
			uint8_t b = 0;
			for (uint32_t j = 0; j < 8; ++j) b |= prev[i * 8 + j] > 0 ? (uint8_t)(1u << j) : 0;
			uint32_t x = orc_morton3D_invert(i) + GRIDSIZE / 8, y = orc_morton3D_invert(i >> 1) + GRIDSIZE / 8,
			         z = orc_morton3D_invert(i >> 2) + GRIDSIZE / 8;
			next[orc_morton3D(x, y, z)] |= b;
		}
	}
}

/* tcnn fill_rollover(_and_rescale) */
EXPORT void orc_fill_rollover_f32(uint32_t n_el, uint32_t stride, uint32_t n_in, float* d) {
	if (n_in == 0) return;
	for (uint32_t i = n_in * stride; i < n_el * stride; ++i) d[i] = d[i % (n_in * stride)];
}
EXPORT void orc_fill_rollover_f16(uint32_t n_el, uint32_t stride, uint32_t n_in, uint16_t* d, int rescale) {
	if (n_in == 0) return;
	for (uint32_t i = n_in * stride; i < n_el * stride; ++i) {
		uint16_t r = d[i % (n_in * stride)];
		if (rescale) r = orc_f32_to_f16(orc_f16_to_f32(r) * n_in / n_el);
		d[i] = r;
	}
}

/* ------------------------------------------------------------------------------------------------
 * Rendering (NerfTracer, testbed_nerf.cu:2229-2503, 2504-2659, 948-1196, 2164-2226), restated per
 * ray: every ray is marched on its own (the GPU marches in compaction rounds of up to 8 steps; the
 * per-ray sample sequence is the same). Two passes so the network can be evaluated in between:
 * orc_nerf_render_march writes each pixel's sample coordinates (at most max_per_ray), then
 * orc_nerf_render_composite composites the network outputs and shades over the background.
 * random_val.cuh:162-326: scrambled Sobol (Burley 2019) for the pixel offset and the start jitter.
 * ---------------------------------------------------------------------------------------------- */
static uint32_t sobol_d(uint32_t index, uint32_t dim) {
	uint32_t X = 0, v = 0x80000000u;
	for (uint32_t bit = 0; bit < 32; ++bit) {
		if ((index >> bit) & 1u) X ^= dim == 0 ? (0x80000000u >> bit) : v;
		v ^= v >> 1;
	}
	return X;
}
static uint32_t hcomb(uint32_t seed, uint32_t v) { return seed ^ (v + (seed << 6) + (seed >> 2)); }
static uint32_t rbits(uint32_t x) {
	x = (((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1));
	x = (((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2));
	x = (((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4));
	x = (((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8));
	return (x >> 16) | (x << 16);
}
static uint32_t lkp(uint32_t x, uint32_t seed) {
	x += seed; x ^= x * 0x6c50b47cu; x ^= x * 0xb82f1e52u; x ^= x * 0xc7afe638u; x ^= x * 0x8d22f6e6u;
	return x;
}
static uint32_t nus(uint32_t x, uint32_t seed) { return rbits(lkp(rbits(x), seed)); }
EXPORT float orc_ld_random_val(uint32_t index, uint32_t seed, uint32_t dim) {
	const float S = (float)(1.0 / 4294967296.0);
	index = nus(index, seed);
	return (float)nus(sobol_d(index, dim), hcomb(seed, dim)) * S;
}
static float fractf_(float x) { return x - floorf(x); }
static void pixel_offset(uint32_t spp, float* ox, float* oy) {
	const float ax = orc_ld_random_val(0, 0xdeadbeefu, 0), ay = orc_ld_random_val(0, 0xdeadbeefu, 1);
	const float bx = orc_ld_random_val(spp, 0xdeadbeefu, 0), by = orc_ld_random_val(spp, 0xdeadbeefu, 1);
	*ox = fractf_(0.5f - ax + bx);
	*oy = fractf_(0.5f - ay + by);
}

/* if_unoccupied_advance_to_next_occupied_voxel (testbed_nerf.cu:811-842): mip = clamp(mip_from_pos, min_mip, max_mip) */
static float adv_occupied(float t, float cone, const float* o, const float* d, const float* idir, const uint8_t* bf,
                          uint32_t min_mip, uint32_t max_mip, const ocfg* c) {
	for (;;) {
		float pos[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
		if (t >= 16384.0f || !contains(c, pos)) return 16384.0f;
		uint32_t mip = mip_pos(pos, CASCADES - 1);
		if (mip < min_mip) mip = min_mip;
		if (mip > max_mip) mip = max_mip;
		if (!bf || occupied(pos, bf, mip)) return t;
		while (mip < max_mip && !occupied(pos, bf, mip + 1)) ++mip;
		t = advance_voxel(t, cone, pos, d, idir, mip);
	}
}

/* coords: [W*H x max_per_ray x 7]; counts: [W*H] (-1 when the ray misses the aabb) */
EXPORT void orc_nerf_render_march(const ocfg* c, const oimg* cam, const uint8_t* bf, uint32_t sample_index, uint32_t max_per_ray,
                                  float* coords, int32_t* counts, int show_accel) {
	const uint32_t min_mip = show_accel >= 0 ? (uint32_t)show_accel : 0u;  /* testbed_nerf.cu:2497, 2594 */
	float m[12];
	orc_camera_matrix(cam->xform, m);
	const uint32_t W = cam->width, H = cam->height;
	float ox, oy;
	pixel_offset(c->snap_to_pixel_centers ? 0u : sample_index, &ox, &oy);
	const float diag[3] = {c->aabb_max[0] - c->aabb_min[0], c->aabb_max[1] - c->aabb_min[1], c->aabb_max[2] - c->aabb_min[2]};
	for (uint32_t i = 0; i < W * H; ++i) {
		const uint32_t x = i % W, y = i / W;
		const float u = ((float)x + ox) / (float)W, v = ((float)y + oy) / (float)H;
		/* screen centre = render_screen_center(m_screen_center = 1 - principal point), testbed.cu:852,
		 * 4376-4379 (zoom 1) = (0.5 - (1 - pp)) + 0.5 */
		const float scx = (0.5f - (1.0f - cam->principal_point[0])) + 0.5f, scy = (0.5f - (1.0f - cam->principal_point[1])) + 0.5f;
		float dx = (u - scx) * (float)W / cam->focal_length[0];
		float dy = (v - scy) * (float)H / cam->focal_length[1];
		lens_undistort(cam->lens_mode, cam->lens_params, &dx, &dy);
		float d[3] = {m[0] * dx + m[3] * dy + m[6], m[1] * dx + m[4] * dy + m[7], m[2] * dx + m[5] * dy + m[8]};
		const float o[3] = {m[9], m[10], m[11]};
		const float inv = 1.0f / sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
		d[0] *= inv; d[1] *= inv; d[2] *= inv;
		float tmin, tmax;
		ray_box(c, o, d, &tmin, &tmax);
		float t = fmaxf(tmin, 0.0f) + 1e-6f;
		const float p0[3] = {o[0] + t * d[0], o[1] + t * d[1], o[2] + t * d[2]};
		counts[i] = -1;
		if (!contains(c, p0)) continue;
		const float idir[3] = {1.0f / d[0], 1.0f / d[1], 1.0f / d[2]};
		const float cone = c->cone_angle_constant;
		t = from_step(to_step(t, cone) + orc_ld_random_val(sample_index, i * 786433u, 0), cone);
		uint32_t k = 0;
		for (; k < max_per_ray; ++k) {
			t = adv_occupied(t, cone, o, d, idir, bf, min_mip, c->max_cascade, c);
			if (t >= 16384.0f) break;
			const float dt = calc_dt(t, cone);
			const float pos[3] = {o[0] + d[0] * t, o[1] + d[1] * t, o[2] + d[2] * t};
			float* q = coords + ((size_t)i * max_per_ray + k) * 7;
			q[0] = (pos[0] - c->aabb_min[0]) / diag[0]; q[1] = (pos[1] - c->aabb_min[1]) / diag[1]; q[2] = (pos[2] - c->aabb_min[2]) / diag[2];
			q[3] = (dt - MIN_STEP) / (MIN_STEP * (1 << (CASCADES - 1)) - MIN_STEP);
			q[4] = (d[0] + 1.0f) * 0.5f; q[5] = (d[1] + 1.0f) * 0.5f; q[6] = (d[2] + 1.0f) * 0.5f;
			t += dt;
		}
		counts[i] = (int32_t)k;
	}
}

/* out16: network outputs [W*H x max_per_ray x 16] (AoS, half bits); frame: [W*H x 4] linear rgba.
 * mode: ERenderMode (common.h:110-119) 0 AO, 1 Shade, 3 Positions, 4 Depth: the step colour of composite_kernel_nerf
 * (testbed_nerf.cu:1189-1208; pos = unwarp_position over the aabb; Depth: dot(camera forward, pos - ray origin) *
 * depth_scale with the origin the render's camera position, m_render_near_distance 0); shade_kernel_nerf
 * (:2164-2196) decodes sRGB for Shade only. cam: the view (its camera matrix, for Depth). */
EXPORT void orc_nerf_render_composite_mode(const ocfg* c, const oimg* cam, uint32_t n_px, uint32_t max_per_ray, const float* coords,
                                           const int32_t* counts, const uint16_t* out16, float min_transmittance, const float* bg,
                                           int mode, float depth_scale, int show_accel, float* frame) {
	float m[12];
	orc_camera_matrix(cam->xform, m);
	const float diag[3] = {c->aabb_max[0] - c->aabb_min[0], c->aabb_max[1] - c->aabb_min[1], c->aabb_max[2] - c->aabb_min[2]};
	for (uint32_t i = 0; i < n_px; ++i) {
		float r = 0, g = 0, b = 0, a = 0;
		for (int32_t k = 0; k < counts[i]; ++k) {
			const uint16_t* o = out16 + ((size_t)i * max_per_ray + k) * 16;
			const float T = 1.f - a;
			const float dt = coords[((size_t)i * max_per_ray + k) * 7 + 3] * (MIN_STEP * (1 << (CASCADES - 1)) - MIN_STEP) + MIN_STEP;
			/* show_accel >= 0: every step opaque (testbed_nerf.cu:1078-1080) */
			const float alpha = show_accel >= 0 ? 1.f : 1.f - ngp_expf(-to_dens(orc_f16_to_f32(o[3]), c->density_activation) * dt);
			const float w = alpha * T;
			float rgb[3];
			if (mode == 1) {
				for (int q = 0; q < 3; ++q) rgb[q] = to_rgb(orc_f16_to_f32(o[q]), c->rgb_activation);
			} else if (mode == 0) {
				rgb[0] = rgb[1] = rgb[2] = alpha;
			} else if (mode == 9) {  /* EncodingVis: the warped position (:1202-1203) */
				const float* wp = coords + ((size_t)i * max_per_ray + k) * 7;
				for (int q = 0; q < 3; ++q) rgb[q] = wp[q];
			} else {
				const float* wp = coords + ((size_t)i * max_per_ray + k) * 7;
				float pos[3];
				for (int q = 0; q < 3; ++q) pos[q] = wp[q] * diag[q] + c->aabb_min[q];
				if (mode == 3 && show_accel >= 0) {  /* :1190-1199 */
					uint32_t mip = mip_pos(pos, CASCADES - 1);
					if (mip < (uint32_t)show_accel) mip = (uint32_t)show_accel;
					const uint32_t res = GRIDSIZE >> mip;
					const int ix = (int)(pos[0] * (float)res), iy = (int)(pos[1] * (float)res), iz = (int)(pos[2] * (float)res);
					orc_pcg32 rng;
					orc_pcg32_seed(&rng, (uint64_t)(int64_t)(ix + iy * 232323 + iz * 727272), 1u);
					rgb[0] = 1.f - (float)mip * (1.f / (float)(CASCADES - 1));
					rgb[1] = orc_pcg32_next_float(&rng);
					rgb[2] = orc_pcg32_next_float(&rng);
				} else if (mode == 3) {
					for (int q = 0; q < 3; ++q) rgb[q] = (pos[q] - 0.5f) / 2.0f + 0.5f;
				} else {
					const float z = (m[6] * (pos[0] - m[9]) + m[7] * (pos[1] - m[10]) + m[8] * (pos[2] - m[11])) * depth_scale;
					rgb[0] = rgb[1] = rgb[2] = z;
				}
			}
			r += rgb[0] * w;
			g += rgb[1] * w;
			b += rgb[2] * w;
			a += w;
			if (a > 1.0f - min_transmittance) { const float inv = 1.0f / a; r *= inv; g *= inv; b *= inv; a *= inv; break; }
		}
		float* f = frame + 4 * (size_t)i;
		f[0] = bg[0]; f[1] = bg[1]; f[2] = bg[2]; f[3] = bg[3];
		if (counts[i] < 0 || !(a > 0.001f)) continue;
		if (!c->linear_colors && mode == 1) { r = s2l(r); g = s2l(g); b = s2l(b); }
		const float cc[4] = {r, g, b, a};
		for (int k = 0; k < 4; ++k) f[k] = cc[k] + f[k] * (1.0f - a);
	}
}
EXPORT void orc_nerf_render_composite(const ocfg* c, const oimg* cam, uint32_t n_px, uint32_t max_per_ray, const float* coords,
                                      const int32_t* counts, const uint16_t* out16, float min_transmittance, const float* bg, float* frame) {
	orc_nerf_render_composite_mode(c, cam, n_px, max_per_ray, coords, counts, out16, min_transmittance, bg, 1, 1.0f, -1, frame);
}

/* The shared transcendental (instant-ngp_amd/csrc/ngp_math.h), exported for its accuracy test:
 * fn 0 ngp_expf, 1 ngp_logf, and the variants the kernels call where the argument is bounded (each
 * must equal the full function there): 2 ngp_expf_mid, 3 ngp_logf_pos, 4 ngp_expf_fast, 5 the
 * stepping-space division ngp_div_rc(x, log(1 + 1/256)). */
EXPORT void orc_math_eval(int fn, size_t n, const float* x, float* y) {
	const float l = ngp_logf(1.0f + 1.0f / 256.0f), rl = 1.0f / l;
	for (size_t i = 0; i < n; ++i) {
		switch (fn) {
			case 0: y[i] = ngp_expf(x[i]); break;
			case 1: y[i] = ngp_logf(x[i]); break;
			case 2: y[i] = ngp_expf_mid(x[i]); break;
			case 3: y[i] = ngp_logf_pos(x[i]); break;
			case 4: y[i] = ngp_expf_fast(x[i]); break;
			default: y[i] = ngp_div_rc(x[i], l, rl); break;
		}
	}
}

/* ---- NerfCounters (testbed_nerf.cu:3568-3609) and the step's inference size (:3923-3930) ---------
 * tcnn::batch_size_granularity = 256 (tcnn absent: SURVEY §8a row a11 "granularity†"). */
static uint32_t next_mult(uint32_t v, uint32_t m) { return (v + m - 1) / m * m; }

/* NerfCounters::update_after_training: from the sampler's step counter (all steps, dropped rays
 * included) and the compacted counter, the measured sizes, the loss scalar (reduce_sum(loss[R]) *
 * measured / target) and the next rays_per_batch = min(next_multiple((u32)(R * target / measured), 256),
 * 2^18), in the reference's float arithmetic. Returns the new rays_per_batch; both counters 0 -> the
 * reference returns early with R unchanged and the measured sizes zeroed. */
EXPORT uint32_t orc_nerf_counters_update(uint32_t rays_per_batch, uint32_t target_batch_size, uint32_t numsteps_counter,
                                         uint32_t compacted_counter, float loss_sum, float* loss_scalar,
                                         uint32_t* measured_batch_size, uint32_t* measured_before_compaction) {
	*measured_batch_size = 0;
	*measured_before_compaction = 0;
	*loss_scalar = 0.f;
	if (numsteps_counter == 0 || compacted_counter == 0) return rays_per_batch;
	*measured_before_compaction = numsteps_counter;
	*measured_batch_size = compacted_counter;
	*loss_scalar = loss_sum * (float)compacted_counter / (float)target_batch_size;
	uint32_t r = (uint32_t)((float)rays_per_batch * (float)target_batch_size / (float)compacted_counter);
	r = next_mult(r, 256);
	return r < (1u << 18) ? r : (1u << 18);
}

/* train_nerf_step's inference size: max_samples while nothing has been measured, else
 * next_multiple(min(measured_before_compaction, max_samples), 256) (testbed_nerf.cu:3923-3930). */
EXPORT uint32_t orc_nerf_max_inference(uint32_t measured_before_compaction, uint32_t max_samples) {
	if (measured_before_compaction == 0) return max_samples;
	return next_mult(measured_before_compaction < max_samples ? measured_before_compaction : max_samples, 256);
}
