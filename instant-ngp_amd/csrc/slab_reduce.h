// slab_reduce.h — the MLP weight-gradient slab reduction as a block body, shared by k_reduce_slabs
// (mlp.hip) and the grid backward's last kernel (grid_scatter.hip k_sc_split_reduce), which runs it in
// extra blocks beside its own so the reduction needs no launch of its own.
#pragma once
#include "common.h"

namespace ngp {

// One launch's worth of slab reduction: grad[p] (+)= sum over n_slabs slabs of slabs[slab * n + p].
struct SlabJob {
	const float* slabs = nullptr;
	uint32_t n_slabs = 0, n = 0;
	f16* grad = nullptr;
	float* grad32 = nullptr;  // set: the fp16-rounded sums widened into it instead (the sharded optimizer's input)
	bool accumulate = false;
	uint32_t stride = 0;  // elements between consecutive slabs (0: n); > n reduces a leading range only
};
constexpr uint32_t SLAB_THREADS = 256;
__host__ __device__ constexpr uint32_t slab_blocks(uint32_t n) { return (n + 31) / 32; }

// Block `blk` (256 threads) = 32 parameters x 8 slab groups; each thread sums every 8th slab of one
// parameter, then the 8 partial sums are added in a fixed order (deterministic).
// gsh (optional, 32 entries of LDS): also receives the block's fp16 gradients (the fused MLP update).
__device__ __forceinline__ void reduce_slabs_block(const SlabJob& j, uint32_t blk, f16* gsh = nullptr) {
	__shared__ float part[8][33];
	const uint32_t p = blk * 32 + (threadIdx.x & 31), g = threadIdx.x >> 5;
	const size_t st = j.stride ? j.stride : j.n;
	float s = 0.f;
	if (p < j.n) {
		// 8 independent loads in flight per step (the adds stay in slab order: deterministic)
		uint32_t b = g;
		for (; b + 56 < j.n_slabs; b += 64) {
			float v[8];
#pragma unroll
			for (int k = 0; k < 8; ++k) v[k] = j.slabs[(size_t)(b + 8 * k) * st + p];
#pragma unroll
			for (int k = 0; k < 8; ++k) s += v[k];
		}
		for (; b < j.n_slabs; b += 8) s += j.slabs[(size_t)b * st + p];
	}
	part[g][threadIdx.x & 31] = s;
	__syncthreads();
	if (g == 0 && p < j.n) {
		float t = j.accumulate ? (float)j.grad[p] : 0.f;
#pragma unroll
		for (int k = 0; k < 8; ++k) t += part[k][threadIdx.x];
		if (j.grad32) j.grad32[p] = (float)(f16)t;
		else j.grad[p] = (f16)t;
		if (gsh) gsh[threadIdx.x] = (f16)t;
	}
}

}  // namespace ngp
