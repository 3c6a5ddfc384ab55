// lens.h — camera lens models of the NeRF training/render rays (reference Lens, ELensMode:
// include/neural-graphics-primitives/common_device.cuh:288-378 and its use in uv_to_ray :443-510 /
// pos_to_uv :547-585). Perspective, OpenCV (k1, k2, p1, p2) and OpenCV fisheye (k1..k4); FTheta,
// LatLong and Equirectangular are out of scope (no dataset here uses them). Float arithmetic in the
// reference's operation order; the oracle restates it in C (oracle/ngp_nerf_oracle.c orc_lens_*).
#pragma once
#include <cmath>
#include <cstdint>

namespace ngp {

enum LensMode : uint32_t { LENS_PERSPECTIVE = 0, LENS_OPENCV = 1, LENS_OPENCV_FISHEYE = 2 };

// opencv_lens_distortion_delta (:289-303)
__host__ __device__ inline void opencv_delta(const float* k, float u, float v, float* du, float* dv) {
	const float k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
	const float u2 = u * u, uv = u * v, v2 = v * v;
	const float r2 = u2 + v2;
	const float radial = k1 * r2 + k2 * r2 * r2;
	*du = u * radial + 2.0f * p1 * uv + p2 * (r2 + 2.0f * u2);
	*dv = v * radial + 2.0f * p2 * uv + p1 * (r2 + 2.0f * v2);
}

// opencv_fisheye_lens_distortion_delta (:305-327)
__host__ __device__ inline void fisheye_delta(const float* k, float u, float v, float* du, float* dv) {
	const float r = sqrtf(u * u + v * v);
	if (r > 2.220446049250313e-16f) {
		const float theta = atanf(r);
		const float theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2, theta8 = theta4 * theta4;
		const float thetad = theta * (1.0f + k[0] * theta2 + k[1] * theta4 + k[2] * theta6 + k[3] * theta8);
		*du = u * thetad / r - u;
		*dv = v * thetad / r - v;
	} else {
		*du = 0.0f;
		*dv = 0.0f;
	}
}

__host__ __device__ inline void lens_delta(uint32_t mode, const float* k, float u, float v, float* du, float* dv) {
	if (mode == LENS_OPENCV) opencv_delta(k, u, v, du, dv);
	else if (mode == LENS_OPENCV_FISHEYE) fisheye_delta(k, u, v, du, dv);
	else { *du = 0.0f; *dv = 0.0f; }
}

// iterative_lens_undistortion (:330-369): Newton with central-difference Jacobian, <= 100 steps
__host__ __device__ inline void lens_undistort(uint32_t mode, const float* k, float* u, float* v) {
	if (mode != LENS_OPENCV && mode != LENS_OPENCV_FISHEYE) return;
	const float x0u = *u, x0v = *v;
	float xu = *u, xv = *v;
	for (uint32_t i = 0; i < 100; ++i) {
		const float step0 = fmaxf(1.1920928955078125e-07f, fabsf(1e-6f * xu));
		const float step1 = fmaxf(1.1920928955078125e-07f, fabsf(1e-6f * xv));
		float d0, d1, b00, b01, f00, f01, b10, b11, f10, f11;
		lens_delta(mode, k, xu, xv, &d0, &d1);
		lens_delta(mode, k, xu - step0, xv, &b00, &b01);
		lens_delta(mode, k, xu + step0, xv, &f00, &f01);
		lens_delta(mode, k, xu, xv - step1, &b10, &b11);
		lens_delta(mode, k, xu, xv + step1, &f10, &f11);
		// J columns (glm mat2): J[0] = (1 + d(du)/du, d(dv)/du), J[1] = (d(du)/dv, 1 + d(dv)/dv)
		const float j00 = 1.0f + (f00 - b00) / (2.0f * step0);
		const float j10 = (f10 - b10) / (2.0f * step1);
		const float j01 = (f01 - b01) / (2.0f * step0);
		const float j11 = 1.0f + (f11 - b11) / (2.0f * step1);
		// glm::inverse (mat2) then mat2 * vec2
		const float od = 1.0f / (j00 * j11 - j10 * j01);
		const float i00 = j11 * od, i01 = -j01 * od, i10 = -j10 * od, i11 = j00 * od;
		const float ru = xu + d0 - x0u, rv = xv + d1 - x0v;
		const float su = i00 * ru + i10 * rv, sv = i01 * ru + i11 * rv;
		xu -= su;
		xv -= sv;
		if (su * su + sv * sv < 1e-10f) break;
	}
	*u = xu;
	*v = xv;
}

}  // namespace ngp
