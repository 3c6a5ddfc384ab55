// training.hip — tcnn losses, image sampling (BASELINE C1) and SDF sampling (BASELINE C5) on gfx950.
// See training.h for the reference call sites; every kernel cites the code it restates.
#include "training.h"
#include "profiler.h"

#include <cmath>
#include <cstring>

namespace ngp {

// ------------------------------------------------------------------------------------------------
// Losses (tcnn Loss classes, restated: values / gradients normalised by n_total = n * dims, the
// gradient scaled by loss_scale and rounded to the network precision; padding columns get 0).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void loss_one(uint32_t type, float pred, float target, float inv_n, float& value, float& grad) {
	const float d = pred - target;
	switch (type) {
		case TL_L2: value = d * d * inv_n; grad = 2.0f * d * inv_n; break;
		case TL_L1: value = fabsf(d) * inv_n; grad = copysignf(1.0f, d) * inv_n; break;
		case TL_MAPE: {
			const float sc = 1.0f / (fabsf(target) + 1e-2f);
			value = fabsf(d) * sc * inv_n; grad = copysignf(1.0f, d) * sc * inv_n; break;
		}
		case TL_SMAPE: {
			const float sc = 2.0f / (fabsf(pred) + fabsf(target) + 1e-2f);
			value = fabsf(d) * sc * inv_n; grad = copysignf(1.0f, d) * sc * inv_n; break;
		}
		default: {  // TL_RELATIVE_L2
			const float den = pred * pred + 1e-2f;
			value = d * d / den * inv_n; grad = 2.0f * d / den * inv_n; break;
		}
	}
}

__global__ void __launch_bounds__(256) k_loss(uint32_t type, const LossEvalArgs a) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	float sum = 0.f;
	if (i < a.n) {
		const float inv_n = 1.0f / ((float)a.n * (float)a.dims);
		f16* g = a.dL_dout + (size_t)i * a.dL_stride;
		for (uint32_t j = 0; j < a.dL_stride; ++j) {
			if (j < a.dims) {
				float v, gr;
				loss_one(type, (float)a.out[(size_t)i * a.out_stride + j], a.target[(size_t)i * a.target_stride + j], inv_n, v, gr);
				sum += v;
				g[j] = to_f16(a.loss_scale * gr);
			} else {
				g[j] = (f16)0.f;
			}
		}
		if (a.values) a.values[i] = sum;
	}
	if (a.loss_sum) {
		// wave sum, one atomic per wave (the loss scalar is a reporting value, order-dependent in fp32)
		for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
		if ((threadIdx.x & 63) == 0 && sum != 0.f) atomicAdd(a.loss_sum, sum);
	}
}

void loss_evaluate(uint32_t type, const LossEvalArgs& a, hipStream_t s) {
	NGP_CHECK(type <= TL_RELATIVE_L2, "loss: unsupported type");
	NGP_CHECK(a.dims >= 1 && a.dims <= a.dL_stride && a.dims <= a.out_stride && a.dims <= a.target_stride, "loss: bad dims");
	if (a.n == 0) return;
	k_loss<<<div_round_up(a.n, 256), 256, 0, s>>>(type, a);
	NGP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Image training data (src/testbed_image.cu:214-285)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float linear_to_srgb(float x) {  // common_device.cuh:99-105
	return x < 0.0031308f ? 12.92f * x : 1.055f * powf(x, 0.41666f) - 0.055f;
}

// generate_random_uniform (element k = draw k of m_rng; tcnn†) + stratify2_kernel (:62-76)
// + eval_image_kernel_and_snap<float, 3> (:167-212), one thread per sample.
__global__ void __launch_bounds__(256) k_image_samples(const ImageSampleArgs a, uint32_t log2_n) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= a.n) return;
	HostPcg32 r = a.rng;
	Pcg32Dev rng{r.state, r.inc};
	pcg_advance(rng, 2ull * i);
	float px = pcg_float(rng), py = pcg_float(rng);
	if (a.random_mode == IMG_STRATIFIED && log2_n != ~0u) {
		const uint32_t log2s = log2_n / 2, size = 1u << log2s;
		const uint32_t idx = i & ((1u << log2_n) - 1u);
		const uint32_t x = idx & (size - 1u), y = idx >> log2s;
		px = px / (float)size + ((float)x / (float)size);
		py = py / (float)size + ((float)y / (float)size);
	}
	const int W = (int)a.width, H = (int)a.height;
	auto read = [&](int x, int y, float* o) {
		const float* t = a.texture + ((size_t)y * W + x) * 4;
#pragma unroll
		for (int c = 0; c < 3; ++c) o[c] = a.linear_colors ? t[c] : linear_to_srgb(t[c]);
	};
	float val[3];
	if (a.snap_to_pixel_centers) {
		int ix = (int)floorf(px * (float)W), iy = (int)floorf(py * (float)H);
		px = ((float)ix + 0.5f) / (float)W;
		py = ((float)iy + 0.5f) / (float)H;
		ix = min(max(ix, 0), W - 1);
		iy = min(max(iy, 0), H - 1);
		read(ix, iy, val);
	} else {
		const float fx = fminf(fmaxf(px * (float)W - 0.5f, 0.0f), (float)W - (1.0f + 1e-4f));
		const float fy = fminf(fmaxf(py * (float)H - 0.5f, 0.0f), (float)H - (1.0f + 1e-4f));
		const int x0 = (int)fx, y0 = (int)fy;
		const float wx = fx - (float)x0, wy = fy - (float)y0;
		const int ix = min(max(x0, 0), W - 2), iy = min(max(y0, 0), H - 2);
		float v00[3], v10[3], v01[3], v11[3];
		read(ix, iy, v00); read(ix + 1, iy, v10); read(ix, iy + 1, v01); read(ix + 1, iy + 1, v11);
#pragma unroll
		for (int c = 0; c < 3; ++c)
			val[c] = (1 - wx) * (1 - wy) * v00[c] + wx * (1 - wy) * v10[c] + (1 - wx) * wy * v01[c] + wx * wy * v11[c];
	}
	a.positions[2 * (size_t)i] = px;
	a.positions[2 * (size_t)i + 1] = py;
#pragma unroll
	for (int c = 0; c < 3; ++c) a.targets[3 * (size_t)i + c] = val[c];
}

void image_generate_samples(const ImageSampleArgs& a, hipStream_t s) {
	NGP_CHECK(a.width >= 2 && a.height >= 2, "image: needs at least 2x2 pixels");
	if (a.n == 0) return;
	uint32_t log2_n = ~0u;
	if ((a.n & (a.n - 1)) == 0) {
		uint32_t l = 0;
		while ((1u << l) < a.n) ++l;
		if (l % 2 == 0) log2_n = l;  // "Can't stratify a non-square batch size" otherwise (a warning there)
	}
	k_image_samples<<<div_round_up(a.n, 256), 256, 0, s>>>(a, log2_n);
	NGP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// SDF training data (src/testbed_sdf.cu:1187-1275)
// ------------------------------------------------------------------------------------------------
struct F3 { float x, y, z; };
__device__ __forceinline__ F3 ld3(const float* p) { return F3{p[0], p[1], p[2]}; }
__device__ __forceinline__ F3 sub(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 add(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 mul(F3 a, float s) { return F3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ F3 cross(F3 a, F3 b) { return F3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
__device__ __forceinline__ float len2(F3 a) { return dot(a, a); }
__device__ __forceinline__ float sgn(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

// binary_search (common.h:268-292): first index with data[it] >= val
__device__ uint32_t binary_search(float val, const float* data, uint32_t length) {
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

// logit with tcnn's clamp (tcnn† generate_random_logistic: mean + stddev * logit(u) * sqrt(3)/pi)
__device__ __forceinline__ float logistic_sample(float u, float mean, float stddev) {
	const float x = fminf(fmaxf(u, 1e-9f), 1.0f - 1e-9f);
	return -logf(1.0f / x - 1.0f) * stddev * 0.551328895f + mean;
}

__global__ void __launch_bounds__(256) k_sdf_samples(const SdfMeshDev m, const SdfSampleArgs a, uint32_t n_exact, uint32_t n_offset,
                                                     uint32_t n_uniform) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= a.n) return;
	const uint32_t n_surface = n_exact + n_offset;
	Pcg32Dev rng{a.rng.state, a.rng.inc};
	pcg_advance(rng, 3ull * i);  // generate_random_uniform(n*3): element k = draw k
	F3 p{pcg_float(rng), pcg_float(rng), pcg_float(rng)};
	float dist = 0.f;
	if (i < n_surface) {
		// sample_uniform_on_triangle_kernel (:619-627) + Triangle::sample_uniform_position (triangle.cuh:26-33)
		const uint32_t t = min(binary_search(p.x, m.cdf, m.n_triangles), m.n_triangles - 1);
		const float* tri = m.tris + 9 * (size_t)t;
		const float sx = sqrtf(p.y);
		const float f0 = 1.0f - sx, f1 = sx * (1.0f - p.z), f2 = sx * p.z;
		p = add(add(mul(ld3(tri), f0), mul(ld3(tri + 3), f1)), mul(ld3(tri + 6), f2));
	} else if (i < n_surface + n_uniform) {
		// scale_to_aabb_kernel (:467-472) + assign_float(length(diag) * 1.001) (:1239-1251)
		const F3 mn{a.aabb_min[0], a.aabb_min[1], a.aabb_min[2]};
		const F3 diag{a.aabb_max[0] - mn.x, a.aabb_max[1] - mn.y, a.aabb_max[2] - mn.z};
		p = F3{mn.x + p.x * diag.x, mn.y + p.y * diag.y, mn.z + p.z * diag.z};
		dist = sqrtf(len2(diag)) * 1.001f;
	}
	if (i >= n_exact && i < n_surface) {
		// generate_random_logistic(n_offset * 3) drawn after the uniform positions (m_rng advanced by 3n),
		// then perturb_sdf_samples (:222-231)
		const uint32_t j = i - n_exact;
		Pcg32Dev r2{a.rng.state, a.rng.inc};
		pcg_advance(r2, 3ull * a.n + 3ull * j);
		F3 q{logistic_sample(pcg_float(r2), 0.f, a.stddev), logistic_sample(pcg_float(r2), 0.f, a.stddev),
		     logistic_sample(pcg_float(r2), 0.f, a.stddev)};
		a.perturbations[3 * (size_t)j] = q.x;
		a.perturbations[3 * (size_t)j + 1] = q.y;
		a.perturbations[3 * (size_t)j + 2] = q.z;
		p = add(p, q);
		dist = sqrtf(len2(q)) * 1.001f;
	}
	a.positions[3 * (size_t)i] = p.x;
	a.positions[3 * (size_t)i + 1] = p.y;
	a.positions[3 * (size_t)i + 2] = p.z;
	a.distances[i] = dist;
}

void sdf_generate_samples(const SdfMeshDev& m, const SdfSampleArgs& a, hipStream_t s) {
	NGP_CHECK(m.n_triangles > 0, "sdf: empty mesh");
	NGP_CHECK(a.n % 8 == 0, "sdf: the number of samples must be a multiple of 8");
	if (a.n == 0) return;
	const uint32_t base = a.n / 8;
	{
		ProfScope ps("sdf_samples", s);
		k_sdf_samples<<<div_round_up(a.n, 256), 256, 0, s>>>(m, a, 4 * base, 3 * base, base);
		NGP_HIP(hipGetLastError());
	}
	// the distances written above are upper bounds of the true ones (perturbation length / aabb
	// diagonal x 1.001): signed_distance_gpu(..., use_existing_distances_as_upper_bounds = true)
	sdf_signed_distance(m, 4 * base, a.positions + 3 * (size_t)(4 * base), a.distances + 4 * base, true, s);
}

// ---- shuffle --------------------------------------------------------------------------------
// tcnn's shuffle permutation is not recoverable; any bijection keeps train_sdf's
// semantics (de-correlate the freshly generated batch). perm(i) = (A * i + seed * B) mod n with A
// coprime to n, computed in 64-bit.
static uint64_t gcd64(uint64_t a, uint64_t b) { while (b) { const uint64_t t = a % b; a = b; b = t; } return a; }
static uint32_t shuffle_multiplier(uint32_t n) {
	uint64_t a = 2654435761ull % n;
	if (a == 0) a = 1;
	while (gcd64(a, n) != 1) ++a;
	return (uint32_t)a;
}
uint32_t sdf_shuffle_index(uint32_t i, uint32_t n, uint32_t seed) {
	const uint64_t A = shuffle_multiplier(n);
	return (uint32_t)((A * i + (uint64_t)seed * 40503ull) % n);
}

__global__ void k_sdf_shuffle(uint32_t n, uint64_t A, uint64_t off, const float* __restrict__ pin, const float* __restrict__ din,
                              float* __restrict__ pout, float* __restrict__ dout) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const uint32_t j = (uint32_t)((A * i + off) % n);
	pout[3 * (size_t)j] = pin[3 * (size_t)i];
	pout[3 * (size_t)j + 1] = pin[3 * (size_t)i + 1];
	pout[3 * (size_t)j + 2] = pin[3 * (size_t)i + 2];
	dout[j] = din[i];
}

void sdf_shuffle(uint32_t n, uint32_t seed, const float* pos_in, const float* dist_in, float* pos_out, float* dist_out, hipStream_t s) {
	if (n == 0) return;
	k_sdf_shuffle<<<div_round_up(n, 256), 256, 0, s>>>(n, shuffle_multiplier(n), ((uint64_t)seed * 40503ull) % n, pos_in, dist_in,
	                                                    pos_out, dist_out);
	NGP_HIP(hipGetLastError());
}

}  // namespace ngp
