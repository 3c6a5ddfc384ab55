// grid.h — multiresolution hash-grid encoding for gfx950.
//
// Replaces tcnn::GridEncodingTemplated (tiny-cuda-nn, absent from the reference: SURVEY F1), as
// created by NerfNetwork (include/neural-graphics-primitives/nerf_network.h:93-95) and by
// Testbed::reset_network (src/testbed.cu:4101). Semantics: SURVEY §8a rows a1 (forward) and a2
// (backward); the oracle restatement is oracle/ngp_oracle.c (orc_grid_*).
#pragma once
#include "common.h"

namespace ngp {

struct GridDesc {
	uint32_t n_dims = 3, n_levels = 16, n_features = 2, log2_hashmap = 19, base_resolution = 16;
	float per_level_scale = 2.0f;
	uint32_t offsets[33] = {};  // entry offset of each level; offsets[L] = total entries
	float scale[32] = {};       // exp2f(l*log2 b)*N_min - 1
	uint32_t resolution[32] = {};
	uint32_t n_entries() const { return offsets[n_levels]; }
	uint64_t n_params() const { return (uint64_t)offsets[n_levels] * n_features; }
};

// Host: offset table identical to tcnn's (dense level rounded up to 8 entries, clamped to 2^log2T).
void grid_desc_init(GridDesc& g, uint32_t D, uint32_t L, uint32_t F, uint32_t log2T, uint32_t Nmin, float b);

enum Layout : uint32_t { AoS = 0, SoA = 1 };

struct GridFwdArgs {
	uint32_t n;
	const float* pos;          // element (i, d) at pos[i * pos_stride + d]
	uint32_t pos_stride;
	const f16* table;          // [entries x F]
	f16* out;                  // AoS: out[i * out_stride + l*F + f]; SoA: out[(l*F + f) * out_stride + i]
	uint32_t out_stride;
	uint32_t out_layout;
	float max_level;           // levels >= max_level*L + 1e-3 are zeroed (tcnn set_max_level)
	const float* max_level_per_sample;  // optional (set_max_level_gpu)
};

struct GridBwdArgs {
	uint32_t n;
	const float* pos;
	uint32_t pos_stride;
	const f16* dL_dy;          // same layout convention as GridFwdArgs::out
	uint32_t dy_stride;
	uint32_t dy_layout;
	f16* grad;                 // [entries x F], accumulated with packed fp16 atomics
	float max_level;
	const float* max_level_per_sample;
	uint32_t level_begin = 0;  // levels below were handled elsewhere (windowed backward)
};

// Optional by-product of the training forward: the bucket histogram of the sorted backward
// (grid_scatter.hip k_sc_hist), counted from the corner indices the forward computes anyway.
// hist[(vb_base[l] + bucket) * n_chunks + chunk]; one forward block = one chunk of `chunk` samples.
struct GridHist {
	uint32_t* hist;
	uint32_t B, n_chunks, chunk;
	uint32_t vb_base[33];
};

void grid_forward(const GridDesc& g, const GridFwdArgs& a, hipStream_t stream, const GridHist* hist = nullptr);
// true when grid_forward writes whole AoS rows (padding columns included: no memset needed)
bool grid_forward_rows_ok(const GridDesc& g, const GridFwdArgs& a);
void grid_backward(const GridDesc& g, const GridBwdArgs& a, hipStream_t stream);

// ---- device-side building blocks (shared with fused kernels) ---------------------------------
struct GridConst {
	uint32_t n_levels, n_features;
	uint32_t offsets[33];
	float scale[32];
	uint32_t resolution[32];
};

__device__ __forceinline__ uint32_t grid_index3(uint32_t T, uint32_t res, uint32_t x, uint32_t y, uint32_t z) {
	// tcnn grid_index: dense while the stride fits in T, else coherent prime hash (1, 2654435761, 805459861)
	uint32_t stride = 1, index = 0;
	index += x * stride; stride *= res;
	if (stride <= T) { index += y * stride; stride *= res; }
	if (stride <= T) { index += z * stride; stride *= res; }
	if (T < stride) index = x ^ (y * 2654435761u) ^ (z * 805459861u);
	return index % T;
}

__device__ __forceinline__ uint32_t grid_index2(uint32_t T, uint32_t res, uint32_t x, uint32_t y) {
	uint32_t stride = 1, index = 0;
	index += x * stride; stride *= res;
	if (stride <= T) { index += y * stride; stride *= res; }
	if (T < stride) index = x ^ (y * 2654435761u);
	return index % T;
}

template <uint32_t D>
__device__ __forceinline__ uint32_t corner_index(const GridConst& c, uint32_t l, const uint32_t* base, uint32_t corner) {
	const uint32_t T = c.offsets[l + 1] - c.offsets[l];
	const uint32_t res = c.resolution[l];
	const uint32_t x = base[0] + (corner & 1u);
	const uint32_t y = base[1] + ((corner >> 1) & 1u);
	if constexpr (D == 3) {
		const uint32_t z = base[2] + ((corner >> 2) & 1u);
		return c.offsets[l] + grid_index3(T, res, x, y, z);
	} else {
		return c.offsets[l] + grid_index2(T, res, x, y);
	}
}

template <uint32_t D>
__device__ __forceinline__ float corner_weight(const float* frac, uint32_t corner) {
	float w = 1.0f;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) w *= ((corner >> d) & 1u) ? frac[d] : 1.0f - frac[d];
	return w;
}

template <uint32_t D>
__device__ __forceinline__ void level_setup(const GridConst& c, uint32_t l, const float* x, float* frac, uint32_t* base) {
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		float p = __builtin_fmaf(c.scale[l], x[d], 0.5f);
		float t = floorf(p);
		base[d] = (uint32_t)(int)t;
		frac[d] = p - t;
	}
}

GridConst make_grid_const(const GridDesc& g);
int device_cu_count();

}  // namespace ngp
