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
// log2T = GRID_LOG2_DENSE: a dense grid (tcnn DenseGrid), every level res^D entries with no hashmap cap
constexpr uint32_t GRID_LOG2_DENSE = 31;
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
// hist[chunk * vb_base[L] + vb_base[l] + bucket]; one forward block = one chunk of `chunk` samples.
// With bricks (grid_scatter.h ScatterPlan::LD > 0) the leading LD dense levels are not counted per corner:
// each sample counts once in its brick's bucket (vbs [0, n_bricks), brick_of).
struct GridHist {
	uint32_t* hist;
	uint32_t B, n_chunks, chunk;
	uint32_t vb_base[33];
	uint32_t brick_first = 0, brick_levels = 0, n_bricks = 0, brick_cells = 8, bricks_per_dim = 0, brick_vb0 = 0;  // levels [first, levels)
};

// mode: 0/1 per-sample kernels, 2 XCD-partitioned (level, chunk) kernel (L2-local tables; measured
// slower than the per-sample row kernel on C2 and C2p, kept as an option)
void grid_forward(const GridDesc& g, const GridFwdArgs& a, hipStream_t stream, const GridHist* hist = nullptr);
// true when grid_forward writes whole AoS rows (padding columns included: no memset needed)
bool grid_forward_rows_ok(const GridDesc& g, const GridFwdArgs& a);
void grid_backward(const GridDesc& g, const GridBwdArgs& a, hipStream_t stream);

// Input gradients (tcnn Encoding::backward's dL_dinput; NerfNetwork::backward_impl slices them into
// the pos rows and the direction rows, nerf_network.h:282-299, 317-333). Per sample, fp32:
//   dL/dx_d = sum_l scale_l * sum_c (dw_c/dx_d / scale_l) * sum_f dL/dy_{l,f} * T[c, f]
// where w_c is the trilinear weight of corner c (levels the forward zeroes, l >= max_level L + 1e-3,
// contribute nothing); and, when dL_dsh is given, the direction gradient through the degree-4 SH
// encoding of d = 2 dir - 1:  dL/ddir_j = 2 * sum_k dL/dSH_k * dSH_k/dd_j.  Both are multiplied by
// out_scale (tcnn input_gradient divides out its backprop scale).
struct InputGradArgs {
	uint32_t n;
	const float* pos; uint32_t pos_stride;   // encoding input: element (i, d) at pos[i * pos_stride + d]
	const f16* table;                        // [entries x F]
	const f16* dL_dy; uint32_t dy_stride;    // dL/d(encoding) AoS: dL_dy[i * dy_stride + l*F + f]
	float max_level; const float* max_level_per_sample;
	const f16* dL_dsh;                       // optional: dL/d(SH encoding) [n x 16]
	uint32_t dir_offset;                     // direction rows of the input (pos + dir_offset) and output
	float* out; uint32_t out_stride;         // dL/dinput: rows 0..D-1 (and dir_offset..+2) of each sample's row
	float out_scale;
};
void grid_input_gradient(const GridDesc& g, const InputGradArgs& a, hipStream_t stream);

// ---- device-side building blocks (shared with fused kernels) ---------------------------------
struct GridConst {
	uint32_t n_levels, n_features;
	uint32_t offsets[33];
	float scale[32];
	uint32_t resolution[32];
	uint32_t hashed;  // bit l: level l is hashed (grid_index3's 32-bit stride > T; T is then a power of two)
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

// Entry index of a corner. Same function as grid_index3/2 (tcnn grid_index) given the level kind
// from GridConst::hashed: dense levels need the modulo only for out-of-range coordinates, hashed
// levels have power-of-two T. Corner bit d offsets dimension d by one.
template <uint32_t D>
__device__ __forceinline__ uint32_t corner_index(const GridConst& c, uint32_t l, const uint32_t* base, uint32_t corner) {
	const uint32_t x = base[0] + (corner & 1u);
	const uint32_t y = base[1] + ((corner >> 1) & 1u);
	if ((c.hashed >> l) & 1u) {
		const uint32_t mask = c.offsets[l + 1] - c.offsets[l] - 1u;
		if constexpr (D == 3) {
			const uint32_t z = base[2] + ((corner >> 2) & 1u);
			return c.offsets[l] + ((x ^ (y * 2654435761u) ^ (z * 805459861u)) & mask);
		} else {
			return c.offsets[l] + ((x ^ (y * 2654435761u)) & mask);
		}
	}
	const uint32_t res = c.resolution[l];
	uint32_t idx;
	if constexpr (D == 3) {
		const uint32_t z = base[2] + ((corner >> 2) & 1u);
		idx = x + res * (y + res * z);
	} else {
		idx = x + res * y;
	}
	// in-range coordinates give idx < res^D <= T; out-of-range ones wrap like tcnn's index % T
	const uint32_t T = c.offsets[l + 1] - c.offsets[l];
	if (__builtin_expect(idx >= T, 0)) idx %= T;
	return c.offsets[l] + idx;
}

// All 2^D corner indices of one level. A dense level with res^D <= T whose cell is in range (base < res:
// positions in [0, 1]) has every corner index below 2 T, so index % T is min(id, id - T), and the corners
// are corner 0's index plus constants: one branch per level instead of a modulo test per corner. Other
// cells and levels take corner_index (the same integers).
template <uint32_t D>
__device__ __forceinline__ void corner_indices(const GridConst& c, uint32_t l, const uint32_t* base, uint32_t* idx) {
	const uint32_t res = c.resolution[l], T = c.offsets[l + 1] - c.offsets[l];
	uint64_t vol = res;
#pragma unroll
	for (uint32_t d = 1; d < D; ++d) vol *= res;
	bool fast = !((c.hashed >> l) & 1u) && vol <= T;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) fast = fast && base[d] < res;
	if (__builtin_expect(fast, 1)) {
		const uint32_t r2 = res * res;
		const uint32_t i0 = D == 3 ? base[0] + res * (base[1] + res * base[2]) : base[0] + res * base[1];
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) {
			const uint32_t id = i0 + (k & 1u) + (((k >> 1) & 1u) ? res : 0u) + ((D == 3 && ((k >> 2) & 1u)) ? r2 : 0u);
			idx[k] = c.offsets[l] + min(id, id - T);
		}
	} else {
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) idx[k] = corner_index<D>(c, l, base, k);
	}
}

// Gather the 2^D corner entries of one level. The two corners of an x-edge are adjacent entries on
// dense levels, and on hashed levels when base x is even (the hash's x prime is 1, so x+1 flips bit
// 0 only): then both come from one 2F-wide load — half the gather requests of a dense level.
template <uint32_t F> struct GridVec;
template <> struct GridVec<1> { typedef f16 T; typedef f16 __attribute__((ext_vector_type(2), aligned(2))) P; };
template <> struct GridVec<2> { typedef f16x2 T; typedef f16 __attribute__((ext_vector_type(4), aligned(4))) P; };
template <> struct GridVec<4> { typedef f16x4 T; typedef f16 __attribute__((ext_vector_type(8), aligned(8))) P; };
template <> struct GridVec<8> { typedef f16x8 T; typedef f16x8 P; };

#ifndef NGP_GATHER16
#define NGP_GATHER16 0  // 1: F = 2 gathers by aligned 16-B groups (gather_pairs_f2; measured slower at C2')
#endif
template <uint32_t D>
__device__ __forceinline__ void gather_pairs_f2(const uint32_t* idx, const f16* __restrict__ table, f16x2* v);
template <uint32_t D, uint32_t F>
__device__ __forceinline__ void gather_corners(const GridConst& c, uint32_t l, const uint32_t* base, const f16* __restrict__ table,
                                               typename GridVec<F>::T* v) {
	typedef typename GridVec<F>::T V;
	typedef typename GridVec<F>::P P;
	if constexpr (F == 2 && NGP_GATHER16) {
		uint32_t idx[1u << D];
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) idx[k] = corner_index<D>(c, l, base, k);
		gather_pairs_f2<D>(idx, table, v);
	} else if constexpr (F == 2 || F == 4) {
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); k += 2) {
			const uint32_t i0 = corner_index<D>(c, l, base, k), i1 = corner_index<D>(c, l, base, k + 1);
			// dense: i1 == i0 + 1 (unless wrapped); hashed with even base x: i1 == i0 ^ 1
			const uint32_t lo_i = min(i0, i1);
			if (max(i0, i1) == lo_i + 1u) {
				const P p = *(const P*)(table + (size_t)lo_i * F);
				V lo, hi;
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) { lo[f] = p[f]; hi[f] = p[F + f]; }
				const bool swap = i1 < i0;
				v[k] = swap ? hi : lo;
				v[k + 1] = swap ? lo : hi;
			} else {
				v[k] = *(const V*)(table + (size_t)i0 * F);
				v[k + 1] = *(const V*)(table + (size_t)i1 * F);
			}
		}
	} else {
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) v[k] = *(const V*)(table + (size_t)corner_index<D>(c, l, base, k) * F);
	}
}
// F = 2: an x-edge pair whose entries share an aligned group of 4 (16 B) is one 16-B load even when the
// two are not adjacent: on a hashed level with base x = 1 mod 4 the pair is (4m, 4m + 3) or (4m + 3, 4m)
// half of the time, two requests with 8-B loads. The gathers are bound by the L2's request rate (§5), so
// a hashed level's expected requests per pair fall from ~1.31 to ~1.19.
__device__ __forceinline__ f16x2 pick4(const uint32_t (&g)[4], uint32_t i) {
	const uint32_t lo = (i & 1u) ? g[1] : g[0], hi = (i & 1u) ? g[3] : g[2];
	return __builtin_bit_cast(f16x2, (i & 2u) ? hi : lo);
}
template <uint32_t D>
__device__ __forceinline__ void gather_pairs_f2(const uint32_t* idx, const f16* __restrict__ table, f16x2* v) {
	typedef GridVec<2>::P P;
#pragma unroll
	for (uint32_t k = 0; k < (1u << D); k += 2) {
		const uint32_t i0 = idx[k], i1 = idx[k + 1];
		const uint32_t lo_i = min(i0, i1);
		if ((i0 >> 2) == (i1 >> 2)) {
			const uint32_t* gp = (const uint32_t*)(table + (size_t)(i0 & ~3u) * 2);
			typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
			const u32x4g q = *(const u32x4g*)gp;
			const uint32_t g[4] = {q[0], q[1], q[2], q[3]};
			v[k] = pick4(g, i0 & 3u);
			v[k + 1] = pick4(g, i1 & 3u);
		} else if (max(i0, i1) == lo_i + 1u) {
			const P p = *(const P*)(table + (size_t)lo_i * 2);
			const f16x2 a{p[0], p[1]}, b{p[2], p[3]};
			const bool swap = i1 < i0;
			v[k] = swap ? b : a;
			v[k + 1] = swap ? a : b;
		} else {
			v[k] = *(const f16x2*)(table + (size_t)i0 * 2);
			v[k + 1] = *(const f16x2*)(table + (size_t)i1 * 2);
		}
	}
}

// the same gather from precomputed corner indices (corner_indices)
template <uint32_t D, uint32_t F>
__device__ __forceinline__ void gather_corners_at(const uint32_t* idx, const f16* __restrict__ table, typename GridVec<F>::T* v) {
	typedef typename GridVec<F>::T V;
	typedef typename GridVec<F>::P P;
	if constexpr (F == 2 && NGP_GATHER16) {
		gather_pairs_f2<D>(idx, table, v);
	} else if constexpr (F == 2 || F == 4) {
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); k += 2) {
			const uint32_t i0 = idx[k], i1 = idx[k + 1];
			// dense: i1 == i0 + 1 (unless wrapped); hashed with even base x: i1 == i0 ^ 1
			const uint32_t lo_i = min(i0, i1);
			if (max(i0, i1) == lo_i + 1u) {
				const P p = *(const P*)(table + (size_t)lo_i * F);
				V lo, hi;
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) { lo[f] = p[f]; hi[f] = p[F + f]; }
				const bool swap = i1 < i0;
				v[k] = swap ? hi : lo;
				v[k + 1] = swap ? lo : hi;
			} else {
				v[k] = *(const V*)(table + (size_t)i0 * F);
				v[k + 1] = *(const V*)(table + (size_t)i1 * F);
			}
		}
	} else {
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) v[k] = *(const V*)(table + (size_t)idx[k] * F);
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

// The brick of a 3D sample for the brick-summed dense levels 0..LD-1 (grid_scatter.hip): its cell at the
// finest of them, f = LD - 1 (level_setup's arithmetic), divided by the brick edge in cells, clamped to the
// brick grid (positions outside [0, 1] land in an edge brick; their corners outside its region take the
// exact global fallback).
__device__ __forceinline__ uint32_t brick_of(const GridConst& c, uint32_t f, uint32_t K, uint32_t NB, const float* x) {
	uint32_t id = 0, mul = 1;
#pragma unroll
	for (uint32_t d = 0; d < 3; ++d) {
		const int cell = (int)floorf(__builtin_fmaf(c.scale[f], x[d], 0.5f));
		const int b = cell < 0 ? 0 : min(cell / (int)K, (int)NB - 1);
		id += (uint32_t)b * mul;
		mul *= NB;
	}
	return id;
}

// Histogram add of one corner's bucket j (< 2^few_bits buckets in the level, few_bits <= 4): the lanes with
// the same bucket are found with ballots and their leader adds their count once (k_sc_hist; the forward's
// fused histogram keeps per-lane atomics, where the ballots measured no faster).
__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t j, uint32_t few_bits) {
	if (few_bits > 4) { atomicAdd(&h[j], 1u); return; }
	uint64_t peers = __ballot(1);
	for (uint32_t b = 0; b < few_bits; ++b) {
		const uint64_t m = __ballot((j >> b) & 1u);
		peers &= ((j >> b) & 1u) ? m : ~m;
	}
	if (__lane_id() == (uint32_t)(__ffsll((unsigned long long)peers) - 1)) atomicAdd(&h[j], (uint32_t)__popcll(peers));
}

GridConst make_grid_const(const GridDesc& g);
int device_cu_count();

}  // namespace ngp
