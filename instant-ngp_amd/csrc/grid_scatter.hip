// grid_scatter.hip — hash-grid backward as a destination-bucketed exact reduction.
//
// The tcnn backward (tcnn::kernel_grid_backward, half2 atomicAdd per (sample, level, corner)) is bound
// on MI355X by the memory-side atomic rate: ~21 G requests/s, one request per 64-B segment and
// wave-instruction, repeated addresses not merged (profiles/r01_atomics2.txt). Here the same
// contributions — weight * dL/dy rounded to fp16 exactly as tcnn rounds them before its atomic — are
// counting-sorted by destination bucket (2^B consecutive entries of one level), and one workgroup per
// bucket sums them in LDS with 64-bit integer atomics in units of 2^-24 (the fp16 quantum, so every
// fp16 contribution is exact and the sum is order-independent; LDS integer atomics run ~12x faster
// than LDS float atomics on gfx950, profiles/r01_lds_atomics.txt). The sum is rounded once to fp16
// and stored; buckets too large for one workgroup (coarse levels) are summed in parts whose exact
// int64 partial sums are added by a reduce kernel (no fp16 atomics: bitwise reproducible).
//
// Work is cut into (chunk of samples, level) blocks so no block walks the levels serially:
//   prepare (positions only)
//     k_sc_hist       per (chunk, level): LDS histogram over the level's buckets -> hist[chunk][bucket]
//                     (one contiguous row segment per block)
//     k_sc_scan       per bucket: exclusive scan over its chunks -> cursor within the bucket
//                     cur[chunk][bucket] and the bucket total tot[bucket] (lanes = consecutive buckets,
//                     so every hist read and cur write is a coalesced row segment). Every sample emits 2^D
//                     items per level, so level l starts at item n * 2^D * l.
//     k_sc_plan       bucket starts, and the parts list of oversized buckets
//   backward
//     k_sc_scatter    per (chunk, level): items ranked per bucket in LDS, staged in bucket order, written
//                     out as runs: (entry & (2^B-1)) u16 + F fp16 values
//     k_sc_accumulate per part of an oversized bucket (int64 partial sums to scratch), then per bucket:
//                     zero LDS, accumulate, store every entry once (no memset, no atomics)
//     k_sc_split_reduce  per oversized bucket: sum its parts (exact), write every entry once
//
// Bricks (ScatterPlan::bk, 3D grids): the leading dense levels (C2: 0-2 of 4) do not go through items. The
// histogram counts each sample once in its brick (K^3 cells of the finest of those levels), the scatter's
// brick slot writes the sample's index as its one item, every non-empty brick is a "split" bucket whose
// parts (brick_part samples each) sum levels 0..LD-1 of their samples in LDS over the brick's region and
// store the exact int64 sums (a slab, in the split scratch), and extra blocks of k_sc_split_reduce add, per
// dense entry, the slabs of the bricks whose regions hold it. The contributions and their fixed-point sums
// are those of the item path, so the gradient is the same to the bit. C2: 3 of 4 levels' items (63 MB
// written and read) become 4 B per sample plus ~24 MB of slabs.
#include "grid_scatter.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace ngp {

namespace {

#ifndef NGP_SC_FASTIDX
#define NGP_SC_FASTIDX 1  // scatter: corner indices of an in-range dense cell without a modulo test per corner
#endif
#ifndef NGP_SC_PAIR_RANK
#define NGP_SC_PAIR_RANK 1  // scatter: one rank add per x-edge pair of corners in one bucket (bucket_rank_cnt; C2 backward -2.2 us)
#endif
#ifndef NGP_ACC_TAIL_BATCH
#define NGP_ACC_TAIL_BATCH 1  // accumulate, F = 2: the last partial round's item loads issued together (accumulate_items)
#endif
#ifndef NGP_ACC_SKIP0
#define NGP_ACC_SKIP0 1   // accumulate: skip the LDS atomic of a zero contribution (a branch per feature)
#endif
constexpr uint32_t SC_THREADS = 256;
constexpr uint32_t SC_BT = 1024;             // bucket/split blocks: 2 per CU by LDS, 32 waves to hide latency
// (chunk, level) blocks: 512 samples with 512 threads where a chunk fills each bucket with long runs
// (C2: ~40 items per bucket and chunk); sparse tables (C5: T=2^22, ~3.6 items per bucket in a
// 512-sample chunk) take 1024-sample chunks with 1024 threads, whose runs are twice as long and whose
// per-(chunk, bucket) histogram and cursor arrays are half the size (C5 backward 385 -> 355 us;
// 2048-sample chunks measured slower, 372 us).
constexpr size_t SC_LDS_BYTES = 64 * 1024;   // one bucket's int64 accumulators (+ one pad entry per feature plane)
constexpr size_t SC_LDS_PAD_BYTES = 8 * 8;  // up to F = 8 planes
constexpr size_t SC_LIST_BYTES = 4096 * 2;  // fused update: u16 list of a bucket's updated pairs (NE * F / 2 <= 4096)
constexpr float FIX_SCALE = 16777216.0f;     // 2^24: fp16 values are integer multiples of 2^-24

template <uint32_t F> struct ValVec;
template <> struct ValVec<1> { typedef f16 T; };
template <> struct ValVec<2> { typedef f16x2 T; };
template <> struct ValVec<4> { typedef f16x4 T; };
template <> struct ValVec<8> { typedef f16x8 T; };

// Inclusive prefix sum over the 64 lanes of a wave with DPP (VALU latency, no LDS round trips).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
	uint32_t s = x;
	s += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, true);   // row_shr:1
	s += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, true);   // row_shr:2
	s += __builtin_amdgcn_update_dpp(0u, x, 0x113, 0xf, 0xf, true);   // row_shr:3
	s += __builtin_amdgcn_update_dpp(0u, s, 0x114, 0xf, 0xe, false);  // row_shr:4, lanes 4..15 of each row
	s += __builtin_amdgcn_update_dpp(0u, s, 0x118, 0xf, 0xc, false);  // row_shr:8, lanes 8..15
	s += __builtin_amdgcn_update_dpp(0u, s, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
	s += __builtin_amdgcn_update_dpp(0u, s, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
	return s;
}

// Exclusive scan of cnt[0..n) into off[0..n] (off[n] = total) by one NT-thread block.
template <uint32_t NT>
__device__ __forceinline__ void block_exclusive_scan(const uint32_t* cnt, uint32_t* off, uint32_t n, uint32_t* wsum) {
	uint32_t carry = 0;
	for (uint32_t b0 = 0; b0 < n; b0 += NT) {
		const uint32_t b = b0 + threadIdx.x;
		const uint32_t v = b < n ? cnt[b] : 0u;
		const uint32_t incl = wave_inclusive_scan(v);
		if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
		__syncthreads();
		uint32_t pre = carry;
		for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) pre += wsum[w];
		if (b < n) off[b] = pre + incl - v;
#pragma unroll
		for (uint32_t w = 0; w < NT / 64; ++w) carry += wsum[w];
		__syncthreads();
	}
	if (threadIdx.x == 0) off[n] = carry;
}

// Rank of this lane's item within bucket j of the block histogram lh. Levels with few buckets (the
// coarse dense ones: 2 and 16 buckets at C2) would send most of a wave's LDS atomics to one address, so
// there the lanes with the same bucket are found with ballots and their leader adds their count once.
__device__ __forceinline__ uint32_t bucket_rank(uint32_t* lh, uint32_t j, uint32_t few_bits) {
	if (few_bits > 4) return atomicAdd(&lh[j], 1u);
	uint64_t peers = __ballot(1);
	for (uint32_t b = 0; b < few_bits; ++b) {
		const uint64_t m = __ballot((j >> b) & 1u);
		peers &= ((j >> b) & 1u) ? m : ~m;
	}
	const uint32_t lane = __lane_id();
	const uint32_t leader = __ffsll((unsigned long long)peers) - 1;
	uint32_t base = 0;
	if (lane == leader) base = atomicAdd(&lh[j], (uint32_t)__popcll(peers));
	base = __shfl(base, leader);
	return base + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
}

// The same for cnt (0, 1 or 2) consecutive items of bucket j: the first of their ranks. The two corners of an
// x-edge usually share a bucket (adjacent entries on a dense level; entries i and i ^ 1 on a hashed level
// with even base x), so the scatter ranks them with one add of 2 instead of two adds of 1.
__device__ __forceinline__ uint32_t bucket_rank_cnt(uint32_t* lh, uint32_t j, uint32_t cnt, uint32_t few_bits) {
	if (few_bits > 4) return cnt ? atomicAdd(&lh[j], cnt) : 0u;
	uint64_t peers = __ballot(cnt != 0);
	if (peers == 0ull) return 0u;  // wave-uniform
	for (uint32_t b = 0; b < few_bits; ++b) {
		const uint64_t m = __ballot((j >> b) & 1u);
		peers &= ((j >> b) & 1u) ? m : ~m;
	}
	const uint64_t two = __ballot(cnt == 2);
	const uint32_t lane = __lane_id();
	const uint32_t leader = peers ? (uint32_t)(__ffsll((unsigned long long)peers) - 1) : lane;
	uint32_t base = 0;
	if (cnt && lane == leader) base = atomicAdd(&lh[j], (uint32_t)(__popcll(peers) + __popcll(peers & two)));
	base = __shfl(base, leader);
	const uint64_t below = peers & ((1ull << lane) - 1ull);
	return base + (uint32_t)(__popcll(below) + __popcll(below & two));
}

template <uint32_t D>
__device__ __forceinline__ void load_pos(const GridBwdArgs& a, uint32_t i, float* x) {
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * a.pos_stride + d];
}

struct Levels {
	uint32_t vb_base[33];  // first bucket of each level; vb_base[L] = number of buckets (bricks first: vbs [0, NBK))
};

// sample index as a brick item: low 16 bits in the idx slot, high 16 in the first value element
template <uint32_t F>
__device__ __forceinline__ typename ValVec<F>::T brick_item_hi(uint32_t i) {
	typename ValVec<F>::T v{};
	const f16 h = __builtin_bit_cast(f16, (uint16_t)(i >> 16));
	if constexpr (F == 1) v = h; else v[0] = h;
	return v;
}
template <uint32_t F>
__device__ __forceinline__ uint32_t brick_item(const uint16_t* item_idx, const f16* item_val, uint32_t t) {
	return (uint32_t)item_idx[t] | ((uint32_t)__builtin_bit_cast(uint16_t, item_val[(size_t)t * F]) << 16);
}
// global fallback table of the brick levels: int64 [offsets[LD] * F], then the "used" flag
struct BrickFallback {
	unsigned long long* fix;
	uint32_t* flag;
};

template <uint32_t D, uint32_t CHUNK>
__global__ void __launch_bounds__(SC_THREADS) k_sc_hist(const GridConst c, const Levels lv, const BrickConst bk, const GridBwdArgs a,
                                                        uint32_t B, uint32_t n_chunks, uint32_t* __restrict__ hist) {
	extern __shared__ uint32_t h[];
	const uint32_t chunk = blockIdx.x, l = blockIdx.y;
	if (l >= bk.LB && l < bk.LD) {  // brick levels: the finest one's block counts each sample's brick
		if constexpr (D == 3) {
			if (l + 1 != bk.LD) return;
			for (uint32_t j = threadIdx.x; j < bk.NBK; j += blockDim.x) h[j] = 0;
			__syncthreads();
			for (uint32_t q = 0; q < CHUNK / SC_THREADS; ++q) {
				const uint32_t i = chunk * CHUNK + q * SC_THREADS + threadIdx.x;
				if (i >= a.n) continue;
				float x[3];
				load_pos<3>(a, i, x);
				atomicAdd(&h[brick_of(c, l, bk.K, bk.NB, x)], 1u);
			}
			__syncthreads();
			for (uint32_t j = threadIdx.x; j < bk.NBK; j += blockDim.x) hist[(size_t)chunk * lv.vb_base[c.n_levels] + bk.vb0 + j] = h[j];
		}
		return;
	}
	const uint32_t nvb = lv.vb_base[l + 1] - lv.vb_base[l];
	const uint32_t few_bits = nvb <= 1 ? 0u : nvb <= 2 ? 1u : nvb <= 4 ? 2u : nvb <= 8 ? 3u : nvb <= 16 ? 4u : 32u;
	for (uint32_t j = threadIdx.x; j < nvb; j += blockDim.x) h[j] = 0;
	__syncthreads();
	const uint32_t off_l = c.offsets[l];
#pragma unroll
	for (uint32_t q = 0; q < CHUNK / SC_THREADS; ++q) {
		const uint32_t i = chunk * CHUNK + q * SC_THREADS + threadIdx.x;
		if (i >= a.n) continue;
		float x[D];
		load_pos<D>(a, i, x);
		float frac[D]; uint32_t base[D];
		level_setup<D>(c, l, x, frac, base);
		uint32_t cidx[1u << D];
		corner_indices<D>(c, l, base, cidx);
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) hist_add(h, (cidx[k] - off_l) >> B, few_bits);
	}
	__syncthreads();
	for (uint32_t j = threadIdx.x; j < nvb; j += blockDim.x) hist[(size_t)chunk * lv.vb_base[c.n_levels] + lv.vb_base[l] + j] = h[j];
}

// per bucket: exclusive scan of hist[0..n_chunks)[bucket] -> cur[chunk][bucket]; tot[bucket] = total.
// Block = 64 consecutive buckets (lanes) x SCAN_SEG chunk segments (waves): each wave sums its segment's
// counts, the segment offsets come through LDS, then the wave re-reads its segment (L2) and writes the
// cursors. Reads and writes are 256-B row segments.
constexpr uint32_t SCAN_SEG = 16, SCAN_REG = 32;
__global__ void __launch_bounds__(64 * SCAN_SEG) k_sc_scan(const uint32_t* __restrict__ hist, uint32_t n_chunks, uint32_t n_vb,
                                                         uint32_t* __restrict__ cur, uint32_t* __restrict__ tot) {
	__shared__ uint32_t seg_sum[SCAN_SEG][64];
	const uint32_t lane = threadIdx.x & 63, seg = threadIdx.x >> 6;
	const uint32_t vb = blockIdx.x * 64 + lane;
	const uint32_t per = (n_chunks + SCAN_SEG - 1) / SCAN_SEG;
	const uint32_t c0 = min(seg * per, n_chunks), c1 = min(c0 + per, n_chunks);
	if (per <= SCAN_REG) {
		// the whole segment in registers: one load latency, no second read (C2: 32 chunks per segment)
		uint32_t v[SCAN_REG], sum = 0;
#pragma unroll
		for (uint32_t u = 0; u < SCAN_REG; ++u) v[u] = (vb < n_vb && c0 + u < c1) ? hist[(size_t)(c0 + u) * n_vb + vb] : 0u;
#pragma unroll
		for (uint32_t u = 0; u < SCAN_REG; ++u) sum += v[u];
		seg_sum[seg][lane] = sum;
		__syncthreads();
		uint32_t run = 0, total = 0;
		for (uint32_t q = 0; q < SCAN_SEG; ++q) {
			const uint32_t x = seg_sum[q][lane];
			if (q < seg) run += x;
			total += x;
		}
		if (vb >= n_vb) return;
#pragma unroll
		for (uint32_t u = 0; u < SCAN_REG; ++u) {
			if (c0 + u < c1) cur[(size_t)(c0 + u) * n_vb + vb] = run;
			run += v[u];
		}
		if (seg == 0) tot[vb] = total;
		return;
	}
	constexpr uint32_t U = 8;
	uint32_t sum = 0;
	if (vb < n_vb) {
		uint32_t c = c0;
		for (; c + U <= c1; c += U) {
			uint32_t v[U];
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) v[u] = hist[(size_t)(c + u) * n_vb + vb];
#pragma unroll
			for (uint32_t u = 0; u < U; ++u) sum += v[u];
		}
		for (; c < c1; ++c) sum += hist[(size_t)c * n_vb + vb];
	}
	seg_sum[seg][lane] = sum;
	__syncthreads();
	uint32_t run = 0, total = 0;
	for (uint32_t q = 0; q < SCAN_SEG; ++q) {
		const uint32_t v = seg_sum[q][lane];
		if (q < seg) run += v;
		total += v;
	}
	if (vb >= n_vb) return;
	uint32_t c = c0;
	for (; c + U <= c1; c += U) {
		uint32_t v[U];
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) v[u] = hist[(size_t)(c + u) * n_vb + vb];
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			cur[(size_t)(c + u) * n_vb + vb] = run;
			run += v[u];
		}
	}
	for (; c < c1; ++c) {
		const uint32_t v = hist[(size_t)c * n_vb + vb];
		cur[(size_t)c * n_vb + vb] = run;
		run += v;
	}
	if (seg == 0) tot[vb] = total;
}

// One block: bucket starts lo[vb] (exclusive scan of tot over all buckets — levels are consecutive
// and each holds n * 2^D items), and the split list for buckets above split_limit: parts of `part`
// items at split[2 + 3p ..] = {bucket, lo, hi} (split[0] = parts), split buckets at splitb[3b ..] =
// {bucket, first part, parts} (split[1] = buckets). Everything downstream is then a static grid.
// Thread t owns SC_PLAN_K consecutive buckets per round, all loaded up front (1 for C2's 402 buckets;
// 32 for C5's ~18k, one round: one load latency instead of one per 1024 buckets).
constexpr uint32_t SC_PLAN_THREADS = 1024;
template <uint32_t SC_PLAN_K>
__global__ void __launch_bounds__(SC_PLAN_THREADS) k_sc_plan(const uint32_t* __restrict__ tot, uint32_t n_vb, uint32_t split_limit,
                                                             uint32_t part, uint32_t* __restrict__ lo_out,
                                                             uint32_t* __restrict__ split, uint32_t* __restrict__ splitb,
                                                             uint32_t brick_vb0, uint32_t n_bricks, uint32_t brick_part, uint32_t* __restrict__ bp,
                                                             uint32_t* __restrict__ fb_flag) {
	// bricks (vbs [brick_vb0, + n_bricks)): every non-empty one is summed in parts of brick_part samples, each storing a
	// slab; bp[2 b] = first part, bp[2 b + 1] = parts. They are not split buckets of k_sc_split_reduce.
	if (fb_flag && threadIdx.x == 0) *fb_flag = 0u;  // the previous step's finalize has read and cleared the fallback
	__shared__ uint32_t wsum[3][SC_PLAN_THREADS / 64];
	const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
	// buckets per thread; a multiple of 4 when SC_PLAN_K is, so totals and starts move as 16-B vectors
	// (the workspace arrays are 256-B aligned, every thread's first bucket a multiple of 4)
	constexpr bool VEC = SC_PLAN_K % 4 == 0;
	uint32_t K = min(SC_PLAN_K, (n_vb + SC_PLAN_THREADS - 1) / SC_PLAN_THREADS);
	if (VEC) K = (K + 3) & ~3u;
	uint32_t c_lo = 0, c_parts = 0, c_sb = 0;
	for (uint32_t b0 = 0; b0 < n_vb; b0 += SC_PLAN_THREADS * K) {
		const uint32_t v0 = b0 + threadIdx.x * K;
		uint32_t t[SC_PLAN_K];
		if (VEC) {
#pragma unroll
			for (uint32_t k = 0; k < SC_PLAN_K; k += 4) {
				if (k < K && v0 + k + 3 < n_vb) {
					const uint4 q = *(const uint4*)(tot + v0 + k);
					t[k] = q.x; t[k + 1] = q.y; t[k + 2] = q.z; t[k + 3] = q.w;
				} else {
#pragma unroll
					for (uint32_t j = 0; j < 4; ++j) t[k + j] = (k + j < K && v0 + k + j < n_vb) ? tot[v0 + k + j] : 0u;
				}
			}
		} else {
#pragma unroll
			for (uint32_t k = 0; k < SC_PLAN_K; ++k) t[k] = (k < K && v0 + k < n_vb) ? tot[v0 + k] : 0u;
		}
		uint32_t s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
		for (uint32_t k = 0; k < SC_PLAN_K; ++k) {
			const bool brick = v0 + k - brick_vb0 < n_bricks;
			const uint32_t sp = (brick ? t[k] > 0 : t[k] > split_limit) ? 1u : 0u;
			const uint32_t pk = brick ? brick_part : part;
			s0 += t[k]; s1 += sp ? (t[k] + pk - 1) / pk : 0u; s2 += brick ? 0u : sp;
		}
		const uint32_t i0 = wave_inclusive_scan(s0), i1 = wave_inclusive_scan(s1), i2 = wave_inclusive_scan(s2);
		if (lane == 63) { wsum[0][wave] = i0; wsum[1][wave] = i1; wsum[2][wave] = i2; }
		__syncthreads();
		uint32_t p0 = c_lo, p1 = c_parts, p2 = c_sb;
		for (uint32_t w = 0; w < SC_PLAN_THREADS / 64; ++w) {
			if (w < wave) { p0 += wsum[0][w]; p1 += wsum[1][w]; p2 += wsum[2][w]; }
			c_lo += wsum[0][w]; c_parts += wsum[1][w]; c_sb += wsum[2][w];
		}
		__syncthreads();
		uint32_t lo = p0 + i0 - s0, first = p1 + i1 - s1, b = p2 + i2 - s2;
		if (VEC) {  // the bucket starts as 16-B stores; the split / brick lists below as before
			uint32_t l = lo;
#pragma unroll
			for (uint32_t k = 0; k < SC_PLAN_K; k += 4) {
				const uint32_t l0 = l, l1 = l0 + t[k], l2 = l1 + t[k + 1], l3 = l2 + t[k + 2];
				l = l3 + t[k + 3];
				if (k < K && v0 + k + 3 < n_vb) {
					*(uint4*)(lo_out + v0 + k) = uint4{l0, l1, l2, l3};
				} else {
					const uint32_t lv[4] = {l0, l1, l2, l3};
#pragma unroll
					for (uint32_t j = 0; j < 4; ++j)
						if (k + j < K && v0 + k + j < n_vb) lo_out[v0 + k + j] = lv[j];
				}
			}
		}
#pragma unroll
		for (uint32_t k = 0; k < SC_PLAN_K; ++k) {
			if (k >= K || v0 + k >= n_vb) break;
			const uint32_t vb = v0 + k, tk = t[k];
			if (!VEC) lo_out[vb] = lo;
			if (vb - brick_vb0 < n_bricks) {
				const uint32_t parts = (tk + brick_part - 1) / brick_part;
				bp[2 * (vb - brick_vb0)] = first; bp[2 * (vb - brick_vb0) + 1] = parts;
				for (uint32_t q = 0; q < parts; ++q) {
					uint32_t* d = split + 2 + 3 * (size_t)(first + q);
					d[0] = vb; d[1] = lo + q * brick_part; d[2] = min(lo + (q + 1) * brick_part, lo + tk);
				}
				first += parts;
			} else if (tk > split_limit) {
				const uint32_t parts = (tk + part - 1) / part;
				splitb[3 * b] = vb; splitb[3 * b + 1] = first; splitb[3 * b + 2] = parts;
				for (uint32_t q = 0; q < parts; ++q) {
					uint32_t* d = split + 2 + 3 * (size_t)(first + q);
					d[0] = vb; d[1] = lo + q * part; d[2] = min(lo + (q + 1) * part, lo + tk);
				}
				first += parts;
				++b;
			}
			lo += tk;
		}
	}
	if (threadIdx.x == 0) { split[0] = c_parts; split[1] = c_sb; }
}

// The brick slot of a chunk: one item per sample (its index) in its brick's bucket, ranked, staged and
// written out like the level items.
template <uint32_t F, uint32_t SC_CHUNK, uint32_t SC_ST>
__device__ void scatter_bricks(const GridConst& c, const BrickConst& bk, const GridBwdArgs& a, uint32_t n_vb, uint32_t chunk,
                               const uint32_t* __restrict__ cur_t, const uint32_t* __restrict__ lo_vb,
                               uint16_t* __restrict__ item_idx, f16* __restrict__ item_val, uint32_t* lds, uint32_t* wsum) {
	typedef typename ValVec<F>::T V;
	constexpr uint32_t SC_SSPT = SC_CHUNK / SC_ST;
	const uint32_t nvb = bk.NBK;
	uint32_t* cur = lds;
	uint32_t* lh = cur + nvb;
	uint32_t* loff = lh + nvb;
	uint16_t* st_b = (uint16_t*)(loff + nvb + 1);
	uint32_t* st_i = (uint32_t*)(((uintptr_t)(st_b + SC_CHUNK) + 15) & ~(uintptr_t)15);
	for (uint32_t j = threadIdx.x; j < nvb; j += blockDim.x) {
		cur[j] = lo_vb[bk.vb0 + j] + cur_t[(size_t)chunk * n_vb + bk.vb0 + j];
		lh[j] = 0;
	}
	__syncthreads();
	uint32_t e[SC_SSPT], r[SC_SSPT];
#pragma unroll
	for (uint32_t q = 0; q < SC_SSPT; ++q) {
		const uint32_t i = chunk * SC_CHUNK + q * SC_ST + threadIdx.x;
		if (i >= a.n) continue;
		float x[3];
		load_pos<3>(a, i, x);
		e[q] = brick_of(c, bk.LD - 1, bk.K, bk.NB, x);
		r[q] = atomicAdd(&lh[e[q]], 1u);
	}
	__syncthreads();
	block_exclusive_scan<SC_ST>(lh, loff, nvb, wsum);
	__syncthreads();
#pragma unroll
	for (uint32_t q = 0; q < SC_SSPT; ++q) {
		const uint32_t i = chunk * SC_CHUNK + q * SC_ST + threadIdx.x;
		if (i >= a.n) continue;
		const uint32_t slot = loff[e[q]] + r[q];
		st_b[slot] = (uint16_t)e[q];
		st_i[slot] = i;
	}
	__syncthreads();
	const uint32_t n_it = loff[nvb];
	for (uint32_t t = threadIdx.x; t < n_it; t += blockDim.x) {
		const uint32_t j = st_b[t], i = st_i[t];
		const uint32_t gpos = cur[j] + (t - loff[j]);
		item_idx[gpos] = (uint16_t)(i & 0xffffu);
		*(V*)(item_val + (size_t)gpos * F) = brick_item_hi<F>(i);
	}
}

template <uint32_t D, uint32_t F, uint32_t SC_CHUNK, uint32_t SC_ST>
__global__ void __launch_bounds__(SC_ST) k_sc_scatter(const GridConst c, const Levels lv, const BrickConst bk, const GridBwdArgs a, uint32_t B,
                                                      uint32_t n_vb, uint32_t n_chunks, uint32_t xcd_map, const uint32_t* __restrict__ cur_t,
                                                      const uint32_t* __restrict__ lo_vb, uint16_t* __restrict__ item_idx,
                                                      f16* __restrict__ item_val, uint32_t debug) {
	typedef typename ValVec<F>::T V;
	constexpr uint32_t NC = 1u << D;
	constexpr uint32_t NIT = SC_CHUNK * NC;  // items per block
	constexpr uint32_t SC_SSPT = SC_CHUNK / SC_ST;  // samples per thread
	extern __shared__ uint32_t lds[];
	__shared__ uint32_t wsum[SC_ST / 64];
	// slots per chunk: one per item level, the brick slot in place of the brick levels (slot LB)
	const uint32_t n_slots = c.n_levels - (bk.LD - bk.LB) + (bk.LD ? 1u : 0u);
	// XCD-aware order: blocks b and b + 8 share an XCD (round-robin dispatch), so the L level blocks of a
	// chunk run back to back on one XCD and its positions and dL/dy rows leave HBM once, not L times
	uint32_t chunk, l;
	if (xcd_map == 1) {
		const uint32_t slot = blockIdx.x >> 3;
		l = slot % n_slots;
		chunk = (slot / n_slots) * 8 + (blockIdx.x & 7);
	} else if (xcd_map == 2) {
		// and each XCD owns a contiguous range of chunks: neighbouring runs of a bucket meet in one L2
		const uint32_t slot = blockIdx.x >> 3, cpx = (n_chunks + 7) >> 3;
		l = slot % n_slots;
		chunk = (blockIdx.x & 7) * cpx + slot / n_slots;
		if (slot / n_slots >= cpx) return;
	} else {
		chunk = blockIdx.x % n_chunks;
		l = blockIdx.x / n_chunks;
	}
	if (chunk >= n_chunks) return;
	if (bk.LD && l >= bk.LB) {
		if constexpr (D == 3) {
			if (l == bk.LB) {
				scatter_bricks<F, SC_CHUNK, SC_ST>(c, bk, a, n_vb, chunk, cur_t, lo_vb, item_idx, item_val, lds, wsum);
				return;
			}
		}
		l = l - bk.LB - 1 + bk.LD;
	}
	const uint32_t nvb = lv.vb_base[l + 1] - lv.vb_base[l];
	uint32_t* cur = lds;                                   // [nvb] this block's global cursor per bucket
	uint32_t* lh = cur + nvb;                              // [nvb] counts
	uint32_t* loff = lh + nvb;                             // [nvb + 1] block-local exclusive offsets
	uint16_t* st_b = (uint16_t*)(loff + nvb + 1);          // [NIT] bucket of the item in slot order
	uint16_t* st_idx = st_b + NIT;                         // [NIT]
	V* st_val = (V*)(((uintptr_t)(st_idx + NIT) + 15) & ~(uintptr_t)15);  // [NIT]
	// global start of (bucket, this chunk): bucket start (k_sc_plan) + the chunk's cursor (k_sc_scan)
	for (uint32_t j = threadIdx.x; j < nvb; j += blockDim.x) {
		const uint32_t vb = lv.vb_base[l] + j;
		cur[j] = lo_vb[vb] + cur_t[(size_t)chunk * n_vb + vb];
		lh[j] = 0;
	}
	__syncthreads();
	const uint32_t off_l = c.offsets[l];
	const uint32_t mask = (1u << B) - 1u;
	const uint32_t few_bits = nvb <= 1 ? 0u : nvb <= 2 ? 1u : nvb <= 4 ? 2u : nvb <= 8 ? 3u : nvb <= 16 ? 4u : 32u;
	uint32_t e[SC_SSPT][NC], r[SC_SSPT][NC];
	V val[SC_SSPT][NC];
	uint32_t n_have = 0;
#pragma unroll
	for (uint32_t q = 0; q < SC_SSPT; ++q) {
		const uint32_t i = chunk * SC_CHUNK + q * SC_ST + threadIdx.x;
		if (i >= a.n) continue;
		n_have = q + 1;
		float x[D];
		load_pos<D>(a, i, x);
		const float ml = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
		const bool active = !((float)l > ml + 1e-3f);  // tcnn backward: levels beyond max_level get nothing
		float g[F];
		if (a.dy_layout == AoS) {
			V gv;
			if (active) gv = *(const V*)(a.dL_dy + (size_t)i * a.dy_stride + l * F);
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				if constexpr (F == 1) g[f] = active ? (float)gv : 0.f;
				else g[f] = active ? (float)gv[f] : 0.f;
			}
		} else {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) g[f] = active ? (float)a.dL_dy[(size_t)(l * F + f) * a.dy_stride + i] : 0.f;
		}
		float frac[D]; uint32_t base[D];
		level_setup<D>(c, l, x, frac, base);
#if NGP_SC_FASTIDX
		uint32_t cidx[NC];
		corner_indices<D>(c, l, base, cidx);
#endif
#pragma unroll
		for (uint32_t k = 0; k < NC; ++k) {
#if NGP_SC_FASTIDX
			e[q][k] = cidx[k] - off_l;
#else
			e[q][k] = corner_index<D>(c, l, base, k) - off_l;
#endif
#if NGP_SC_PAIR_RANK
			if (k & 1u) {  // ranks of the x-edge pair (k - 1, k)
				const uint32_t j0 = e[q][k - 1] >> B, j1 = e[q][k] >> B;
				const bool same = j0 == j1;
				const uint32_t r0 = bucket_rank_cnt(lh, j0, same ? 2u : 1u, few_bits);
				const uint32_t r1 = bucket_rank_cnt(lh, j1, same ? 0u : 1u, few_bits);
				r[q][k - 1] = r0;
				r[q][k] = same ? r0 + 1u : r1;
			}
#else
			r[q][k] = bucket_rank(lh, e[q][k] >> B, few_bits);
#endif
			const float w = corner_weight<D>(frac, k);
			if constexpr (F == 1) val[q][k] = to_f16(w * g[0]);
			else {
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) val[q][k][f] = to_f16(w * g[f]);
			}
		}
	}
	__syncthreads();
	block_exclusive_scan<SC_ST>(lh, loff, nvb, wsum);
	__syncthreads();
#pragma unroll
	for (uint32_t q = 0; q < SC_SSPT; ++q) {
		if (q >= n_have) break;
#pragma unroll
		for (uint32_t k = 0; k < NC; ++k) {
			const uint32_t j = e[q][k] >> B;
			const uint32_t slot = loff[j] + r[q][k];
			st_b[slot] = (uint16_t)j;
			st_idx[slot] = (uint16_t)(e[q][k] & mask);
			st_val[slot] = val[q][k];
		}
	}
	__syncthreads();
	const uint32_t n_it = loff[nvb];
	if (!(debug & 8))
		for (uint32_t t = threadIdx.x; t < n_it; t += blockDim.x) {
			const uint32_t j = st_b[t];
			const uint32_t gpos = cur[j] + (t - loff[j]);
			item_idx[gpos] = st_idx[t];
			*(V*)(item_val + (size_t)gpos * F) = st_val[t];
		}
}

// LDS accumulators are feature-major, acc[f * NEP + entry] with NEP = NE + 1: a wave's lanes hit 2 *
// (random entry) banks instead of 8 * entry (entry-major int64 x F=4), ~4x fewer bank conflicts; the
// one-entry pad puts the F planes of one entry in different banks. Lane l adds feature (k + l) % F at
// step k, so lanes that share a hot entry (NeRF batches concentrate on the object: C2's coarse
// levels) spread their same-address adds over F addresses in F banks instead of serialising on one.
template <uint32_t F>
__device__ __forceinline__ void accumulate_items(unsigned long long* acc, uint32_t NE, uint32_t lo, uint32_t hi,
                                                 const uint16_t* __restrict__ item_idx, const f16* __restrict__ item_val,
                                                 uint32_t debug = 0) {
	typedef typename ValVec<F>::T V;
	if (debug & 32) {  // timing experiment: the loads without the LDS atomics
		float sum = 0.f;
		for (uint32_t t = lo + threadIdx.x; t < hi; t += blockDim.x) {
			const V vv = *(const V*)(item_val + (size_t)t * F);
			if constexpr (F == 1) sum += (float)vv; else sum += (float)vv[0];
			sum += (float)item_idx[t];
		}
		acc[threadIdx.x] = (unsigned long long)sum;
		return;
	}
	// U items per thread in flight: the loop is bound by memory-level parallelism, not LDS
	constexpr uint32_t U = 8;
	const uint32_t NEP = NE + 1;
	const uint32_t rot = (debug & 64) ? 0u : threadIdx.x % F;
	auto add_item = [&](uint32_t j, const V& vv) {
#pragma unroll
		for (uint32_t k = 0; k < F; ++k) {
			const uint32_t f = (k + rot) & (F - 1);
			float x;
			if constexpr (F == 1) x = (float)vv;
			else {
				x = (float)vv[0];
#pragma unroll
				for (uint32_t q = 1; q < F; ++q) x = f == q ? (float)vv[q] : x;
			}
#if NGP_ACC_SKIP0
			if (x != 0.f) atomicAdd(&acc[f * NEP + j], (unsigned long long)(long long)(x * FIX_SCALE));
#else
			atomicAdd(&acc[f * NEP + j], (unsigned long long)(long long)(x * FIX_SCALE));  // adding 0 is exact
#endif
		}
	};
	const uint32_t step = blockDim.x * U;
	uint32_t t0 = lo;
	for (; t0 + step <= hi; t0 += step) {
		uint32_t j[U];
		V v[U];
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			const uint32_t t = t0 + u * blockDim.x + threadIdx.x;
			j[u] = item_idx[t];
			v[u] = *(const V*)(item_val + (size_t)t * F);
		}
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) add_item(j[u], v[u]);
	}
	// the tail batch measured: C5 1.218 -> 1.199 ms, C2' 0.3057 -> 0.3005 ms (F = 2, 512-thread blocks), C2 0.1340 ->
	// 0.1355 ms (F = 4, 1024 threads: most lanes' clamped loads are wasted), so F = 2 only (gpurun_out/r06m, r06n)
	if (!NGP_ACC_TAIL_BATCH || F != 2) {
		for (uint32_t t = t0 + threadIdx.x; t < hi; t += blockDim.x) add_item(item_idx[t], *(const V*)(item_val + (size_t)t * F));
		return;
	}
	if (t0 >= hi) return;
	// the last partial round (the whole bucket when it holds fewer than blockDim * U items, C5's sparse buckets:
	// ~2.6 k items, 5 per thread): its loads issued together, clamped to the last item, instead of one load
	// round trip per item
	{
		uint32_t j[U];
		V v[U];
#pragma unroll
		for (uint32_t u = 0; u < U; ++u) {
			const uint32_t t = min(t0 + u * blockDim.x + threadIdx.x, hi - 1);
			j[u] = item_idx[t];
			v[u] = *(const V*)(item_val + (size_t)t * F);
		}
#pragma unroll
		for (uint32_t u = 0; u < U; ++u)
			if (t0 + u * blockDim.x + threadIdx.x < hi) add_item(j[u], v[u]);
	}
}

__device__ __forceinline__ float fix_to_f32(unsigned long long q) { return (float)((double)(long long)q * (1.0 / FIX_SCALE)); }

// One part of brick vb (items [lo, hi) = sample indices): the contributions of its samples to levels
// 0..LD-1, to_f16(w * dL/dy) as the scatter forms them, summed exactly in LDS over the brick's region
// (acc[f * (R + 1) + local]), then stored as the part's slab dst[f * NE + local]. Work item = (level,
// sample), level-major, so a wave's lanes share the level. Lane l starts at feature l % F (as
// accumulate_items: spreads a hot entry's same-address adds). Corners outside the region (positions
// outside [0, 1]) are added to the global fallback table instead.
template <uint32_t F>
__device__ void accumulate_brick(const GridConst& c, const BrickConst& bk, const GridBwdArgs& a, uint32_t vb, uint32_t lo, uint32_t hi,
                                 const uint16_t* __restrict__ item_idx, const f16* __restrict__ item_val, unsigned long long* acc,
                                 unsigned long long* __restrict__ dst, uint32_t NE, const BrickFallback& fb) {
	typedef typename ValVec<F>::T V;
	const uint32_t RP = bk.R + 1;
	for (uint32_t k = threadIdx.x; k < RP * F; k += blockDim.x) acc[k] = 0ull;
	__syncthreads();
	const uint32_t b3[3] = {vb % bk.NB, (vb / bk.NB) % bk.NB, vb / (bk.NB * bk.NB)};
	const uint32_t ns = hi - lo, rot = threadIdx.x % F;
	for (uint32_t w = threadIdx.x; w < ns * (bk.LD - bk.LB); w += blockDim.x) {
		const uint32_t l = bk.LB + w / ns, i = brick_item<F>(item_idx, item_val, lo + w % ns);
		float x[3];
		load_pos<3>(a, i, x);
		const float ml = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
		if ((float)l > ml + 1e-3f) continue;  // tcnn backward: masked levels contribute zeros
		float g[F];
		if (a.dy_layout == AoS) {
			const V gv = *(const V*)(a.dL_dy + (size_t)i * a.dy_stride + l * F);
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				if constexpr (F == 1) g[f] = (float)gv; else g[f] = (float)gv[f];
			}
		} else {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) g[f] = (float)a.dL_dy[(size_t)(l * F + f) * a.dy_stride + i];
		}
		float frac[3]; uint32_t base[3];
		level_setup<3>(c, l, x, frac, base);
		const uint32_t W = bk.W[l], res = c.resolution[l];
		uint32_t r0[3];
		bool lo_in[3], hi_in[3];  // corner coordinate base + bit in 0..res (what the finalize's preimages cover)
#pragma unroll
		for (uint32_t d = 0; d < 3; ++d) {
			r0[d] = base[d] - bk.lo[l][b3[d]];
			lo_in[d] = base[d] <= res;
			hi_in[d] = base[d] + 1u <= res;
		}
#pragma unroll
		for (uint32_t k = 0; k < 8; ++k) {
			const uint32_t rx = r0[0] + (k & 1u), ry = r0[1] + ((k >> 1) & 1u), rz = r0[2] + ((k >> 2) & 1u);
			const float wk = corner_weight<3>(frac, k);
			const bool in = rx < W && ry < W && rz < W && ((k & 1u) ? hi_in[0] : lo_in[0]) && ((k & 2u) ? hi_in[1] : lo_in[1]) &&
			                ((k & 4u) ? hi_in[2] : lo_in[2]);
			const uint32_t local = bk.regoff[l] + rx + W * (ry + W * rz);
#pragma unroll
			for (uint32_t q = 0; q < F; ++q) {
				const uint32_t f = (q + rot) & (F - 1);
				float gf = g[0];
#pragma unroll
				for (uint32_t u = 1; u < F; ++u) gf = f == u ? g[u] : gf;
				const float v = (float)to_f16(wk * gf);
				if (v == 0.f) continue;
				const unsigned long long fx = (unsigned long long)(long long)(v * FIX_SCALE);
				if (__builtin_expect(in, 1)) atomicAdd(&acc[f * RP + local], fx);
				else {
					atomicAdd(&fb.fix[(size_t)corner_index<3>(c, l, base, k) * F + f], fx);
					*fb.flag = 1u;
				}
			}
		}
	}
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < bk.R * F; k += blockDim.x) dst[(k / bk.R) * NE + k % bk.R] = acc[(k / bk.R) * RP + k % bk.R];
}

// Sums of one brick-level entry's F features: the slabs of every part of every brick whose region holds a
// corner that indexes it, plus the fallback table (then cleared; read only when the flag is set). A dense
// level's corner coordinates run 0..res (a cell's upper corner at coordinate res is tcnn's index
// x + res (y + res z) unclamped, modulo T = res^3), so entry (x, y, z) is also the corner (x + res, y - 1, z)
// when x = 0, and so on with the borrow through y and z: at most 2 candidates per coordinate.
template <uint32_t F>
__device__ __forceinline__ void brick_entry_sums(const GridConst& c, const BrickConst& bk, uint32_t e, uint32_t NE,
                                                 const uint32_t* __restrict__ bp, const unsigned long long* __restrict__ scratch,
                                                 const BrickFallback& fb, bool fb_used, unsigned long long (&q)[F]) {
#pragma unroll
	for (uint32_t f = 0; f < F; ++f) q[f] = 0ull;
	uint32_t l = 0;
	while (c.offsets[l + 1] <= e) ++l;
	const int res = (int)c.resolution[l], idx = (int)(e - c.offsets[l]);
	const int cc[3] = {idx % res, (idx / res) % res, idx / (res * res)};
	const uint32_t W = bk.W[l];
	// bricks whose region holds coordinate v along one dimension: lo <= v < lo + W, a contiguous range
	auto range = [&](int v, uint32_t& b0, uint32_t& b1) {
		b0 = bk.NB; b1 = 0;
		for (uint32_t b = 0; b < bk.NB; ++b) {
			const int lb = bk.lo[l][b];
			if (lb <= v && v < lb + (int)W) { b0 = min(b0, b); b1 = b + 1; }
		}
	};
	// corner coordinate candidates of a coordinate t - borrow: (value, borrow out)
	auto cands = [&](int t, int* v, int* bo) {
		int n = 0;
		if (t >= 0) { v[n] = t; bo[n] = 0; ++n; }
		if (t == 0) { v[n] = res; bo[n] = 1; ++n; }
		if (t == -1) { v[n] = res - 1; bo[n] = 1; ++n; }
		return n;
	};
	int va[2], ba[2];
	const int na = cands(cc[0], va, ba);
	for (int ia = 0; ia < na; ++ia) {
		int vb_[2], bb[2];
		const int nb = cands(cc[1] - ba[ia], vb_, bb);
		for (int ib = 0; ib < nb; ++ib) {
			int vc[2], bc[2];
			const int nc = cands(cc[2] - bb[ib], vc, bc);  // a borrow out of z wraps modulo T = res^3
			for (int ic = 0; ic < nc; ++ic) {
				const int v3[3] = {va[ia], vb_[ib], vc[ic]};
				uint32_t b0[3], b1[3];
#pragma unroll
				for (int d = 0; d < 3; ++d) range(v3[d], b0[d], b1[d]);
				for (uint32_t bz = b0[2]; bz < b1[2]; ++bz)
					for (uint32_t by = b0[1]; by < b1[1]; ++by)
						for (uint32_t bx = b0[0]; bx < b1[0]; ++bx) {
							const uint32_t b = bx + bk.NB * (by + bk.NB * bz);
							const uint32_t first = bp[2 * b], parts = bp[2 * b + 1];
							const uint32_t local = bk.regoff[l] + (uint32_t)(v3[0] - bk.lo[l][bx]) +
							                       W * ((uint32_t)(v3[1] - bk.lo[l][by]) + W * (uint32_t)(v3[2] - bk.lo[l][bz]));
							for (uint32_t p = 0; p < parts; ++p) {
								const unsigned long long* src = scratch + (size_t)(first + p) * NE * F + local;
#pragma unroll
								for (uint32_t f = 0; f < F; ++f) q[f] += src[(size_t)f * NE];
							}
						}
			}
		}
	}
	if (fb_used) {
		unsigned long long* src = fb.fix + (size_t)e * F;
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) {
			const unsigned long long v = src[f];
			if (v) { q[f] += v; src[f] = 0ull; }
		}
	}
}

// bucket vb -> (first entry, entries)
__device__ __forceinline__ void bucket_entries(const GridConst& c, const Levels& lv, uint32_t B, uint32_t vb, uint32_t& e0, uint32_t& n_e) {
	uint32_t l = 0;
	while (lv.vb_base[l + 1] <= vb) ++l;
	const uint32_t j = vb - lv.vb_base[l];
	e0 = c.offsets[l] + (j << B);
	n_e = min(1u << B, c.offsets[l + 1] - e0);
}

// (entry pair k of a bucket) -> the two accumulator slots (feature-major layout)
template <uint32_t F>
__device__ __forceinline__ void pair_slots(uint32_t k, uint32_t NE, uint32_t& a, uint32_t& b) {  // NE: plane stride
	if constexpr (F == 1) { a = 2 * k; b = 2 * k + 1; }
	else {
		const uint32_t j = k / (F / 2), fp = k % (F / 2);
		a = (2 * fp) * NE + j; b = (2 * fp + 1) * NE + j;
	}
}

// The gradient store of parameter pair k (of the grid) in the non-fused modes: fp16 into `grad`, or (G32) the
// same fp16-rounded values widened into g32.
template <bool G32>
__device__ __forceinline__ void store_pair(f16* grad, float* g32, size_t k, float s0, float s1) {
	if constexpr (G32) {
		typedef float f32x2 __attribute__((ext_vector_type(2)));
		((f32x2*)g32)[k] = f32x2{(float)(f16)s0, (float)(f16)s1};
	} else {
		((f16x2*)grad)[k] = f16x2{(f16)s0, (f16)s1};
	}
}

// One workgroup per work unit, heaviest first: blocks [0, max_parts) are the parts of oversized
// buckets (coarse levels, where thousands of samples share a handful of entries; exact int64 partial
// sums to their scratch slot, added by k_sc_split_reduce), blocks max_parts + vb the other buckets:
// exact sum, written once per entry with plain stores (overwrite: every entry, untouched ones get 0
// — no separate memset; accumulate: old + sum).
// MODE (a template parameter, so that the plain instantiation keeps its register allocation: a runtime
// branch for the fused update cost C2' 25 %): SC_STORE_F16 the fp16 gradient store; SC_FUSED_ADAM the grid's
// optimizer update (FusedAdam) instead of the store; SC_STORE_F32 the fp16-rounded gradient widened to fp32
// into fa.g32 (the sharded optimizer's reduce-scatter input: no separate widening pass).
template <uint32_t F, uint32_t MODE>
__global__ void __launch_bounds__(SC_BT) k_sc_accumulate(const GridConst c, const Levels lv, const BrickConst bk, const GridBwdArgs a,
                                                         const uint32_t* __restrict__ tot,
                                                         const uint32_t* __restrict__ lo_arr, uint32_t B, uint32_t split_limit,
                                                         uint32_t max_parts, const uint16_t* __restrict__ item_idx,
                                                         const f16* __restrict__ item_val, f16* __restrict__ grad, bool overwrite,
                                                         const uint32_t* __restrict__ split, unsigned long long* __restrict__ scratch,
                                                         uint32_t debug, const FusedAdam fa, const BrickFallback fb, uint32_t vb_off,
                                                         uint32_t part_lo, uint32_t part_hi) {
	constexpr bool FUSED = MODE == SC_FUSED_ADAM, G32 = MODE == SC_STORE_F32;
	extern __shared__ unsigned long long acc[];
	const uint32_t NE = 1u << B, NEP = NE + 1;  // feature planes padded by one entry (accumulate_items)
	if (blockIdx.x < max_parts) {
		if (blockIdx.x >= split[0]) return;
		const uint32_t* d = split + 2 + 3 * (size_t)blockIdx.x;
		if (d[0] < part_lo || d[0] >= part_hi) return;  // BwdParts: a split part of a bucket of another range
		const uint32_t lo = d[1], hi = d[2];
		if (d[0] - bk.vb0 < bk.NBK) {
			accumulate_brick<F>(c, bk, a, d[0] - bk.vb0, lo, hi, item_idx, item_val, acc, scratch + (size_t)blockIdx.x * NE * F, NE, fb);
			return;
		}
		for (uint32_t k = threadIdx.x; k < NEP * F; k += blockDim.x) acc[k] = 0ull;
		__syncthreads();
		if (!(debug & 1)) accumulate_items<F>(acc, NE, lo, hi, item_idx, item_val, debug);
		__syncthreads();
		// scratch keeps the unpadded layout [f * NE + entry] (k_sc_split_reduce)
		unsigned long long* dst = scratch + (size_t)blockIdx.x * NE * F;
		for (uint32_t k = threadIdx.x; k < NE * F; k += blockDim.x) dst[k] = acc[(k / NE) * NEP + k % NE];
		return;
	}
	const uint32_t vb = blockIdx.x - max_parts + vb_off;  // vb_off: a launch over buckets [vb_off, ..) (BwdParts)
	if (vb - bk.vb0 < bk.NBK) return;  // bricks: parts only
	const uint32_t t = tot[vb];
	if (t > split_limit) return;
	uint32_t e0, n_e;
	bucket_entries(c, lv, B, vb, e0, n_e);
	f16* g = grad + (size_t)e0 * F;
	if (t == 0) {  // no contribution: gradient 0 (fused update: every entry of the bucket is skipped)
		if (overwrite && !FUSED)
			for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) store_pair<G32>(grad, fa.g32, (size_t)e0 * F / 2 + k, 0.f, 0.f);
		return;
	}
	const uint32_t lo = lo_arr[vb];
	for (uint32_t k = threadIdx.x; k < NEP * F; k += blockDim.x) acc[k] = 0ull;
	__syncthreads();
	if (!(debug & 1)) accumulate_items<F>(acc, NE, lo, lo + t, item_idx, item_val, debug);
	__syncthreads();
	// two fp16 per thread-step (n_e * F is even: levels hold multiples of 8 entries); pair k of the
	// bucket is parameter pair (e0 F) / 2 + k of the grid
	if constexpr (FUSED) {
		// the pairs with a gradient (about a quarter at C5) are listed first (wave ballots, one LDS atomic per
		// wave), then updated densely: a block runs ~1 round of record load -> update -> store instead of one
		// per 1024 pairs with most lanes idle. Pairs are independent, so the list order does not matter.
		// Only for sparse buckets (fewer than 2 items per entry: C5's hashed levels); dense ones (C2', ~4 per
		// entry) update in place, where the list pass measured slower (r03bz: C2' 329 -> 335 us; r03ca/cb:
		// threshold 1 vs 2 items per entry, C5 1.262 vs 1.20 ms on a faster box, C2' unchanged).
		if (t >= 2 * n_e) {
			for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) {
				uint32_t ia, ib;
				pair_slots<F>(k, NEP, ia, ib);
				fused_adam_pair(fa, e0 * F / 2 + k, (f16)fix_to_f32(acc[ia]), (f16)fix_to_f32(acc[ib]));
			}
			return;
		}
		__shared__ uint32_t n_list;
		uint16_t* list = (uint16_t*)(acc + NEP * F);
		if (threadIdx.x == 0) n_list = 0;
		__syncthreads();
		const uint32_t lane = threadIdx.x & 63;
		for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) {
			uint32_t ia, ib;
			pair_slots<F>(k, NEP, ia, ib);
			const f16 h0 = (f16)fix_to_f32(acc[ia]), h1 = (f16)fix_to_f32(acc[ib]);
			const bool act = (float)h0 / fa.loss_scale != 0.f || (float)h1 / fa.loss_scale != 0.f;  // fused_adam_load's test
			const unsigned long long m = __ballot(act);
			if (m == 0ull) continue;
			const uint32_t leader = __ffsll((long long)m) - 1;
			uint32_t base = 0;
			if (lane == leader) base = atomicAdd(&n_list, (uint32_t)__popcll(m));
			base = __shfl(base, leader);
			if (act) list[base + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)k;
		}
		__syncthreads();
		const uint32_t na = n_list;
		for (uint32_t i = threadIdx.x; i < na; i += blockDim.x) {
			const uint32_t k = list[i];
			uint32_t ia, ib;
			pair_slots<F>(k, NEP, ia, ib);
			fused_adam_pair(fa, e0 * F / 2 + k, (f16)fix_to_f32(acc[ia]), (f16)fix_to_f32(acc[ib]));
		}
		return;
	}
	for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) {
		uint32_t ia, ib;
		pair_slots<F>(k, NEP, ia, ib);
		float s0 = fix_to_f32(acc[ia]), s1 = fix_to_f32(acc[ib]);
		if (!G32 && !overwrite) {
			const f16x2 o = ((const f16x2*)g)[k];
			s0 += (float)o[0];
			s1 += (float)o[1];
		}
		store_pair<G32>(grad, fa.g32, (size_t)e0 * F / 2 + k, s0, s1);
	}
}

// One workgroup per split bucket: sum its parts' int64 partials (exact, so the order is immaterial)
// and write every entry once — no fp16 atomics, bitwise reproducible. Columns x >= slab_x0 of the grid
// run the MLP's dW slab reduction (SlabJob) instead: this kernel leaves most of the chip idle, so the
// reduction fits beside it.
// Columns [fin_x0, gridDim.x) finalize the brick levels: one entry per thread (two for F = 1), every feature
// summed over the bricks' slabs in one pass over the geometry (brick_entry_sums), written as parameter pairs
// (pair k = features 2k, 2k + 1 of the grid's leading entries).
template <uint32_t F, uint32_t MODE>
__global__ void __launch_bounds__(SC_THREADS) k_sc_split_reduce(const GridConst c, const Levels lv, uint32_t B,
                                                                const uint32_t* __restrict__ split, const uint32_t* __restrict__ splitb,
                                                                const unsigned long long* __restrict__ scratch, f16* __restrict__ grad,
                                                                bool overwrite, const SlabJob sj, uint32_t slab_x0, const FusedAdam fa,
                                                                const BrickConst bk, const uint32_t* __restrict__ bp, const BrickFallback fb,
                                                                uint32_t fin_x0, uint32_t part_lo, uint32_t part_hi) {
	static_assert(SC_THREADS == SLAB_THREADS, "slab blocks share the split-reduce block shape");
	constexpr bool FUSED = MODE == SC_FUSED_ADAM, G32 = MODE == SC_STORE_F32;
	if (blockIdx.x >= fin_x0) {
		constexpr uint32_t EPT = F == 1 ? 2 : 1;  // entries per thread: whole parameter pairs
		const uint32_t blk = blockIdx.y * (gridDim.x - fin_x0) + (blockIdx.x - fin_x0);
		const uint32_t e0 = c.offsets[bk.LB] + (blk * blockDim.x + threadIdx.x) * EPT;
		if (e0 >= c.offsets[bk.LD]) return;
		const uint32_t NE = 1u << B;
		const bool used = *fb.flag != 0u;
		float s[EPT * F];
#pragma unroll
		for (uint32_t u = 0; u < EPT; ++u) {
			unsigned long long q[F];
			brick_entry_sums<F>(c, bk, e0 + u, NE, bp, scratch, fb, used, q);
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) s[u * F + f] = fix_to_f32(q[f]);
		}
		// pairs (e0 F) / 2 .. of the grid
#pragma unroll
		for (uint32_t h = 0; h < EPT * F / 2; ++h) {
			const uint32_t k = e0 * F / 2 + h;
			float s0 = s[2 * h], s1 = s[2 * h + 1];
			if (FUSED) {
				fused_adam_pair(fa, k, (f16)s0, (f16)s1);
				continue;
			}
			if (!G32 && !overwrite) {
				const f16x2 o = ((const f16x2*)grad)[k];
				s0 += (float)o[0];
				s1 += (float)o[1];
			}
			store_pair<G32>(grad, fa.g32, k, s0, s1);
		}
		return;
	}
	if (blockIdx.x >= slab_x0) {
		const uint32_t blk = blockIdx.y * (fin_x0 - slab_x0) + (blockIdx.x - slab_x0);
		if (blk >= slab_blocks(sj.n)) return;
		if (!FUSED || fa.mlp_n == 0) {
			reduce_slabs_block(sj, blk);
			return;
		}
		// the MLP's optimizer update for this block's 32 parameters (8 groups of 4), from the gradients
		// just reduced: k_adam_lazy4's lazy_update on [0, mlp_n) without a launch of its own
		__shared__ f16 gsh[32];
		reduce_slabs_block(sj, blk, gsh);
		__syncthreads();
		const uint32_t i0 = blk * 32 + 4 * threadIdx.x;
		if (threadIdx.x >= 8 || i0 >= fa.mlp_n) return;
		AdamState st{};
		st.w16 = fa.mlp_w16; st.rec = fa.mlp_rec; st.frags = fa.frags; st.fragmap = fa.fragmap; st.bias_tab = fa.bias_tab;
		const AdamConfig cfg = fa.cfg_dev ? *fa.cfg_dev : fa.cfg;
		const uint32_t step = (fa.step_base ? *fa.step_base : 0u) + fa.step_add;
		LazyGroup G;
		G.i0 = i0;
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			G.g[k] = (float)gsh[4 * threadIdx.x + k] / fa.loss_scale;
			G.act[k] = true;  // matrix parameters: updated every step
		}
		G.any[0] = G.any[1] = true;
#pragma unroll
		for (int r = 0; r < 2; ++r) {
			const f32x4* rp = (const f32x4*)(fa.mlp_rec + (i0 >> 1) + r);
			G.q[r][0] = rp[0]; G.q[r][1] = rp[1]; G.q[r][2] = rp[2];
		}
		lazy_update(st, cfg, step, fa.mlp_n, G);
		return;
	}
	// grid (split bucket, 256-pair chunk): one pair per thread, the parts' loads 8 at a time
	if (blockIdx.x >= split[1]) return;
	const uint32_t vb = splitb[3 * blockIdx.x], first = splitb[3 * blockIdx.x + 1], parts = splitb[3 * blockIdx.x + 2];
	if (vb < part_lo || vb >= part_hi) return;  // BwdParts: a split bucket of another range
	const uint32_t NE = 1u << B;
	uint32_t e0, n_e;
	bucket_entries(c, lv, B, vb, e0, n_e);
	f16* g = grad + (size_t)e0 * F;
	const uint32_t k = blockIdx.y * blockDim.x + threadIdx.x;
	if (k < n_e * F / 2) {
		uint32_t ia, ib;
		pair_slots<F>(k, NE, ia, ib);
		const size_t pstride = (size_t)NE * F;
		const unsigned long long* src = scratch + (size_t)first * pstride;
		unsigned long long q0 = 0, q1 = 0;
		uint32_t p = 0;
		for (; p + 8 <= parts; p += 8) {
			unsigned long long x0[8], x1[8];
#pragma unroll
			for (int u = 0; u < 8; ++u) { x0[u] = src[(p + u) * pstride + ia]; x1[u] = src[(p + u) * pstride + ib]; }
#pragma unroll
			for (int u = 0; u < 8; ++u) { q0 += x0[u]; q1 += x1[u]; }
		}
		for (; p < parts; ++p) { q0 += src[p * pstride + ia]; q1 += src[p * pstride + ib]; }
		float s0 = fix_to_f32(q0), s1 = fix_to_f32(q1);
		if (FUSED) {
			fused_adam_pair(fa, e0 * F / 2 + k, (f16)s0, (f16)s1);
			return;
		}
		if (!G32 && !overwrite) {
			const f16x2 o = ((const f16x2*)g)[k];
			s0 += (float)o[0];
			s1 += (float)o[1];
		}
		store_pair<G32>(grad, fa.g32, (size_t)e0 * F / 2 + k, s0, s1);
	}
}

// scatter block LDS: cursors, counts and offsets per bucket, then the staged items (bucket u16,
// entry u16, F fp16 values)
size_t scatter_lds_bytes(uint32_t max_lb, uint32_t chunk, uint32_t D, uint32_t F) {
	const size_t nit = (size_t)chunk << D;
	return (size_t)(3 * max_lb + 1) * 4 + nit * 4 + 16 + nit * F * 2;
}

Levels make_levels(const GridDesc& g, uint32_t B, const BrickConst& bk) {
	Levels lv{};
	uint32_t vb = 0;  // level LB's range holds the bricks [bk.vb0, + NBK); levels LB+1..LD-1 own no buckets
	for (uint32_t l = 0; l < g.n_levels; ++l) {
		lv.vb_base[l] = vb;
		if (bk.LD && l == bk.LB) vb += bk.NBK;
		else if (!(l >= bk.LB && l < bk.LD)) vb += (g.offsets[l + 1] - g.offsets[l] + (1u << B) - 1) >> B;
	}
	for (uint32_t l = g.n_levels; l <= 32; ++l) lv.vb_base[l] = vb;
	return lv;
}

template <uint32_t D>
void launch_backward(uint32_t F, const GridConst& c, const Levels& lv, const GridBwdArgs& a, const ScatterPlan& p, char* ws,
                     hipStream_t s, bool overwrite, uint32_t debug, const SlabJob* slab, const FusedAdam& fa, const BwdParts* parts) {
	const uint32_t* tot = (const uint32_t*)(ws + p.off_tot);
	const uint32_t* cur_t = (const uint32_t*)(ws + p.off_cur);
	const uint32_t* split = (const uint32_t*)(ws + p.off_split);
	const uint32_t* lo = (const uint32_t*)(ws + p.off_lo);
	const uint32_t* splitb = (const uint32_t*)(ws + p.off_splitb);
	unsigned long long* scratch = (unsigned long long*)(ws + p.off_scratch);
	uint16_t* idx = (uint16_t*)(ws + p.off_idx);
	f16* val = (f16*)(ws + p.off_val);
	const uint32_t* bp = (const uint32_t*)(ws + p.off_bp);
	const BrickFallback fb{(unsigned long long*)(ws + p.off_fb), (uint32_t*)(ws + p.off_fb + (size_t)c.offsets[p.bk.LD] * c.n_features * 8)};
	const size_t lds_s = scatter_lds_bytes(p.max_lb, p.spb, D, F);
	const uint32_t xcd_map = p.xcd_map;
	const uint32_t n_slots = c.n_levels - (p.bk.LD - p.bk.LB) + (p.bk.LD ? 1u : 0u);
	const dim3 grid_s(xcd_map ? (uint32_t)div_round_up(p.n_chunks, 8) * 8 * n_slots : p.n_chunks * n_slots);
	auto go = [&](auto scatter, auto accum, auto splitr) {
		ensure_dynamic_lds((const void*)scatter, lds_s);
		if (!(debug & 4))
			scatter<<<grid_s, p.spb == 512 ? 512 : 1024, lds_s, s>>>(c, lv, p.bk, a, p.B, p.n_buckets, p.n_chunks, xcd_map, cur_t, lo, idx, val,
			                                                          debug);
		NGP_HIP(hipGetLastError());
		const size_t lds_a = ((size_t)8 << p.B) * c.n_features + SC_LDS_PAD_BYTES + (fa.rec ? SC_LIST_BYTES : 0);
		ensure_dynamic_lds((const void*)accum, lds_a);
		const bool parted = parts && parts->k > 0;
		const uint32_t gy = (uint32_t)div_round_up(((size_t)1 << p.B) * c.n_features / 2, SC_THREADS);
		const SlabJob sj = slab ? *slab : SlabJob{};
		const uint32_t slab_x = slab ? (uint32_t)div_round_up(slab_blocks(sj.n), gy) : 0u;
		const size_t fin_entries = (size_t)c.offsets[p.bk.LD] - c.offsets[p.bk.LB];
		const size_t fin_threads = c.n_features == 1 ? div_round_up(fin_entries, 2) : fin_entries;
		const uint32_t fin_x = (uint32_t)div_round_up(div_round_up(fin_threads, SC_THREADS), gy);
		if (!parted) {
			accum<<<p.max_split_blocks + p.n_buckets, p.bt, lds_a, s>>>(c, lv, p.bk, a, tot, lo, p.B, p.split_limit, p.max_split_blocks,
			                                                             idx, val, a.grad, overwrite, split, scratch, debug, fa, fb, 0u,
			                                                             0u, ~0u);
			NGP_HIP(hipGetLastError());
			const dim3 grid_r(p.max_split_buckets + slab_x + fin_x, gy);
			splitr<<<grid_r, SC_THREADS, 0, s>>>(c, lv, p.B, split, splitb, scratch, a.grad, overwrite, sj, p.max_split_buckets, fa, p.bk, bp,
			                                     fb, p.max_split_buckets + slab_x, 0u, ~0u);
			NGP_HIP(hipGetLastError());
			return;
		}
		// parted (no bricks): the bucket ranges from the last to the first, each with its own split parts and split
		// buckets, so a range's gradient is final when its two launches are; the MLP's slabs with range 0, which
		// holds the MLP's parameters. The highest ranges (the hashed levels) rarely hold a split bucket: their
		// exchange starts while the heavy coarse levels are still summed.
		NGP_CHECK(!p.bk.LD, "grid backward parts: not with bricks");
		for (uint32_t jj = 0; jj < parts->k; ++jj) {
			const uint32_t j = parts->k - 1 - jj;
			const uint32_t v0 = j ? std::min(parts->vb_end[j - 1], p.n_buckets) : 0u;
			const uint32_t v1 = j + 1 == parts->k ? p.n_buckets : std::min(parts->vb_end[j], p.n_buckets);
			NGP_CHECK(v0 <= v1, "grid backward parts: bucket ranges out of order");
			accum<<<p.max_split_blocks + (v1 - v0), p.bt, lds_a, s>>>(c, lv, p.bk, a, tot, lo, p.B, p.split_limit, p.max_split_blocks,
			                                                           idx, val, a.grad, overwrite, split, scratch, debug, fa, fb, v0,
			                                                           v0, v1);
			NGP_HIP(hipGetLastError());
			const uint32_t sx = j == 0 ? slab_x : 0u;
			const dim3 grid_r(p.max_split_buckets + sx, gy);
			splitr<<<grid_r, SC_THREADS, 0, s>>>(c, lv, p.B, split, splitb, scratch, a.grad, overwrite, sj, p.max_split_buckets, fa, p.bk, bp,
			                                     fb, p.max_split_buckets + sx, v0, v1);
			NGP_HIP(hipGetLastError());
			if (parts->after) parts->after(parts->user, j, s);
		}
	};
	auto by_chunk = [&](auto sc512, auto sc1024, auto accum, auto splitr) {
		if (p.spb == 512) go(sc512, accum, splitr);
		else go(sc1024, accum, splitr);
	};
#define NGP_SC_F(FF)                                                                                                 \
	if (fa.rec) by_chunk(k_sc_scatter<D, FF, 512, 512>, k_sc_scatter<D, FF, 1024, 1024>, k_sc_accumulate<FF, SC_FUSED_ADAM>, \
	                     k_sc_split_reduce<FF, SC_FUSED_ADAM>);                                                      \
	else if (fa.g32) by_chunk(k_sc_scatter<D, FF, 512, 512>, k_sc_scatter<D, FF, 1024, 1024>,                       \
	                          k_sc_accumulate<FF, SC_STORE_F32>, k_sc_split_reduce<FF, SC_STORE_F32>);              \
	else by_chunk(k_sc_scatter<D, FF, 512, 512>, k_sc_scatter<D, FF, 1024, 1024>, k_sc_accumulate<FF, SC_STORE_F16>,  \
	              k_sc_split_reduce<FF, SC_STORE_F16>)
	switch (F) {
		case 1: NGP_SC_F(1); break;
		case 2: NGP_SC_F(2); break;
		case 4: NGP_SC_F(4); break;
		case 8: NGP_SC_F(8); break;
		default: throw Error("grid backward: unsupported F");
	}
#undef NGP_SC_F
}

// Brick geometry for dense levels LB..LD-1 (3D). Finest level f = LD - 1: brick b covers cells
// [K b, K b + K) and so corners [K b, K b + K]. A coarser level l gets, per brick coordinate, the corners of
// every cell a position of that range can fall in (computed in double, one cell of margin each side for the
// float rounding of the samples' own level_setup), W[l] = the widest such range. A level joins only if a
// brick spans at least MIN_CELLS of its cells per dimension: coarser ones put a brick's thousands of
// contributions on a few dozen LDS counters (C2's level 0: ~2 cells, ~170 adds per counter and brick),
// which serialised the first version (r04j: backward 72 -> 164 us with levels 0-2). Returns LD = 0 when no
// range fits the bucket's LDS tile (R <= NE) or saves bytes: the slabs (one per non-empty brick and part, R * F
// int64, written and read once) must cost under 3/4 of the items they replace (2^D per sample and level, also
// written and read once).
static BrickConst make_bricks(const GridDesc& g, uint32_t n, uint32_t B, uint32_t brick_part) {
	BrickConst best;
	if (g.n_dims != 3) return best;
	if (const char* e = getenv("NGP_SC_BRICKS")) { if (atoi(e) == 0) return best; }
	double min_cells = 3.0;
	if (const char* e = getenv("NGP_SC_BRICK_MIN_CELLS")) min_cells = atof(e);
	const uint32_t F = g.n_features, NE = 1u << B;
	// dense levels with T = res^3 exactly (even res: the unclamped upper corners alias modulo res^3 only,
	// brick_entry_sums), at most 4
	uint32_t dense = 0;
	while (dense < g.n_levels && dense < 4) {
		const uint64_t r = g.resolution[dense];
		if (r * r * r != g.offsets[dense + 1] - g.offsets[dense]) break;
		++dense;
	}
	double best_save = 0.0;
	for (uint32_t LD = 1; LD <= dense; ++LD)
		for (uint32_t LB = 0; LB < LD; ++LB) {
			BrickConst bk;
			bk.LB = LB; bk.LD = LD; bk.K = 8;
			const uint32_t f = LD - 1, cells = g.resolution[f];  // positions in [0, 1]: cells 0..res-1
			bk.NB = (cells + bk.K - 1) / bk.K;
			if (bk.NB < 2 || bk.NB > 32) continue;
			if ((double)bk.K * g.scale[LB] / g.scale[f] < min_cells) continue;
			bk.NBK = bk.NB * bk.NB * bk.NB;
			bool ok = true;
			for (uint32_t l = LB; l < LD && ok; ++l) {
				uint32_t W = 0;
				for (uint32_t b = 0; b < bk.NB; ++b) {
					int64_t c_lo, c_hi;
					if (l == f) { c_lo = (int64_t)bk.K * b; c_hi = c_lo + bk.K; }
					else {
						const double sl = g.scale[l], sf = g.scale[f];
						const double lower = sl * ((double)bk.K * b - 0.5) / sf + 0.5, upper = sl * ((double)bk.K * b + bk.K - 0.5) / sf + 0.5;
						c_lo = (int64_t)std::floor(lower) - 1;
						c_hi = (int64_t)std::floor(upper) + 2;  // last cell (+ margin) + its upper corner
					}
					c_lo = std::max<int64_t>(c_lo, 0);
					c_hi = std::min<int64_t>(c_hi, (int64_t)g.resolution[l]);  // the last cell's upper corner is coordinate res
					bk.lo[l][b] = (uint16_t)c_lo;
					W = std::max<uint32_t>(W, (uint32_t)(c_hi - c_lo + 1));
				}
				bk.W[l] = W;
				bk.regoff[l] = bk.R;
				bk.R += W * W * W;
				ok = bk.R <= NE;
			}
			if (!ok) continue;
			// parts: one per non-empty brick, more where bricks hold over brick_part samples
			const double parts = std::max((double)std::min<uint64_t>(bk.NBK, n), (double)n / brick_part);
			const double slabs = parts * bk.R * F * 8;
			const double items = (double)n * (LD - LB) * 8 * (2 + 2 * F);
			const double save = 0.75 * items - slabs;
			if (save > best_save) { best_save = save; best = bk; }
		}
	// the bricks sit in level LB's bucket range: after the buckets of levels 0..LB-1
	if (best.LD)
		for (uint32_t l = 0; l < best.LB; ++l) best.vb0 += (g.offsets[l + 1] - g.offsets[l] + NE - 1) >> B;
	return best;
}

}  // namespace

ScatterPlan make_scatter_plan(const GridDesc& g, uint32_t n, bool bricks) {
	ScatterPlan p;
	const uint32_t F = g.n_features;
	// bucket = 2^B entries of one level whose F int64 accumulators fill SC_LDS_BYTES
	p.B = 0;
	size_t lds_budget = SC_LDS_BYTES;  // experiment knob NGP_SC_LDS_KB (<= 64)
	if (const char* e = getenv("NGP_SC_LDS_KB")) lds_budget = std::min<size_t>(SC_LDS_BYTES, (size_t)atoi(e) * 1024);
	while (((size_t)2 << p.B) * F * 8 <= lds_budget && p.B < 16) ++p.B;
	if (const char* e = getenv("NGP_SC_BRICK_PART")) p.brick_part = std::max(1, atoi(e));
	if (bricks) p.bk = make_bricks(g, n, p.B, p.brick_part);
	const Levels lv = make_levels(g, p.B, p.bk);
	p.n_buckets = lv.vb_base[g.n_levels];
	p.max_lb = p.bk.NBK;
	for (uint32_t l = 0; l < g.n_levels; ++l) p.max_lb = std::max(p.max_lb, lv.vb_base[l + 1] - lv.vb_base[l]);
	NGP_CHECK((size_t)p.max_lb * 4 <= 32 * 1024, "grid backward: level too large for the bucket histogram");
	// samples per chunk: 1024 when 512-sample chunks would average fewer than 16 items per (chunk,
	// bucket) and the scatter block's LDS allows it
	const uint64_t items_per_sample = ((uint64_t)(g.n_levels - (p.bk.LD - p.bk.LB)) << g.n_dims) + (p.bk.LD ? 1u : 0u);
	p.spb = 512;
	if (512ull * items_per_sample < 16ull * p.n_buckets && scatter_lds_bytes(p.max_lb, 1024, g.n_dims, F) <= 160 * 1024) p.spb = 1024;
	if (const char* e = getenv("NGP_SC_CHUNK")) p.spb = (uint32_t)atoi(e);
	NGP_CHECK(p.spb == 512 || p.spb == 1024, "grid backward: chunk must be 512 or 1024 samples");
	NGP_CHECK(scatter_lds_bytes(p.max_lb, p.spb, g.n_dims, F) <= 160 * 1024, "grid backward: scatter chunk exceeds LDS");
	p.n_chunks = (uint32_t)div_round_up(n, p.spb);
	p.n_items = (uint64_t)n * items_per_sample;
	NGP_CHECK(p.n_items < (1ull << 32), "grid backward: too many contributions for 32-bit offsets");
	p.split_limit = 49152;
	p.part = 49152;
	if (const char* e = getenv("NGP_SC_PART")) p.part = (uint32_t)atoi(e);
	if (const char* e = getenv("NGP_SC_LIMIT")) p.split_limit = (uint32_t)atoi(e);
	p.max_split_blocks = (uint32_t)(div_round_up(p.n_items, (uint64_t)p.part) + div_round_up(p.n_items, (uint64_t)p.split_limit) + 1);
	if (p.bk.LD) p.max_split_blocks += (uint32_t)(std::min<uint64_t>(p.bk.NBK, n) + div_round_up((uint64_t)n, (uint64_t)p.brick_part));
	p.max_split_buckets = (uint32_t)(div_round_up(p.n_items, (uint64_t)p.split_limit) + 1);
	p.xcd_map = 2;
	if (const char* e = getenv("NGP_SC_XCD")) p.xcd_map = (uint32_t)atoi(e);
	// accumulation block: 512 threads for F = 2 (4 blocks per CU by waves; C2' 328 -> 315 us, C5 1.250 ->
	// 1.235 ms), 1024 for F = 4 (C2: 144 -> 151 us at 512) (profiles/r03ce)
	p.bt = F == 2 ? 512 : 1024;
	if (const char* e = getenv("NGP_SC_BT")) p.bt = (uint32_t)atoi(e);
	NGP_CHECK(p.bt >= 64 && p.bt <= SC_BT && p.bt % 64 == 0, "grid backward: NGP_SC_BT must be a multiple of 64 up to 1024");
	const uint64_t len = (uint64_t)p.n_buckets * p.n_chunks;
	NGP_CHECK(len < (1ull << 31), "grid backward: bucket histogram too large");
	auto align = [](size_t v) { return (v + 255) / 256 * 256; };
	p.off_hist = 0;
	p.off_cur = align(p.off_hist + len * 4);
	p.off_tot = align(p.off_cur + len * 4);
	p.off_split = align(p.off_tot + (size_t)p.n_buckets * 4);
	p.off_lo = align(p.off_split + (2 + 3 * (size_t)p.max_split_blocks) * 4);
	p.off_splitb = align(p.off_lo + (size_t)p.n_buckets * 4);
	p.off_scratch = align(p.off_splitb + 3 * (size_t)p.max_split_buckets * 4);
	p.off_idx = align(p.off_scratch + (size_t)p.max_split_blocks * ((size_t)1 << p.B) * g.n_features * 8);
	p.off_val = align(p.off_idx + p.n_items * 2);
	p.off_bp = align(p.off_val + p.n_items * F * 2);
	p.off_fb = align(p.off_bp + (size_t)p.bk.NBK * 8);
	p.total = align(p.off_fb + (size_t)g.offsets[p.bk.LD] * F * 8 + 4);
	return p;
}

bool scatter_hist(const GridDesc& g, const ScatterPlan& p, void* workspace, GridHist& h) {
	if ((size_t)p.n_buckets * 4 > 48 * 1024 || p.spb != 512) return false;
	const Levels lv = make_levels(g, p.B, p.bk);
	h.hist = (uint32_t*)((char*)workspace + p.off_hist);
	h.B = p.B; h.n_chunks = p.n_chunks; h.chunk = p.spb;
	for (int l = 0; l <= 32; ++l) h.vb_base[l] = lv.vb_base[l];
	h.brick_first = p.bk.LB; h.brick_levels = p.bk.LD; h.n_bricks = p.bk.NBK; h.brick_cells = p.bk.K; h.bricks_per_dim = p.bk.NB;
	h.brick_vb0 = p.bk.vb0;
	return true;
}

void grid_scatter_prepare(const GridDesc& g, const GridBwdArgs& a, const ScatterPlan& p, void* workspace, hipStream_t s, bool hist_done) {
	if (a.n == 0) return;
	char* ws = (char*)workspace;
	uint32_t* hist = (uint32_t*)(ws + p.off_hist);
	if (!hist_done) {
		const GridConst c = make_grid_const(g);
		const Levels lv = make_levels(g, p.B, p.bk);
		const dim3 grid_h(p.n_chunks, g.n_levels);
		const size_t lds_h = (size_t)p.max_lb * 4;
		auto go = [&](auto k3, auto k2) {
			if (g.n_dims == 3) k3<<<grid_h, SC_THREADS, lds_h, s>>>(c, lv, p.bk, a, p.B, p.n_chunks, hist);
			else k2<<<grid_h, SC_THREADS, lds_h, s>>>(c, lv, p.bk, a, p.B, p.n_chunks, hist);
		};
		if (p.spb == 512) go(k_sc_hist<3, 512>, k_sc_hist<2, 512>);
		else go(k_sc_hist<3, 1024>, k_sc_hist<2, 1024>);
		NGP_HIP(hipGetLastError());
	}
	k_sc_scan<<<div_round_up(p.n_buckets, 64), 64 * SCAN_SEG, 0, s>>>(hist, p.n_chunks, p.n_buckets, (uint32_t*)(ws + p.off_cur), (uint32_t*)(ws + p.off_tot));
	NGP_HIP(hipGetLastError());
	const auto plan = p.n_buckets <= SC_PLAN_THREADS ? k_sc_plan<1> : p.n_buckets <= 8 * SC_PLAN_THREADS ? k_sc_plan<8> : k_sc_plan<32>;
	plan<<<1, SC_PLAN_THREADS, 0, s>>>((const uint32_t*)(ws + p.off_tot), p.n_buckets, p.split_limit, p.part,
	                                        (uint32_t*)(ws + p.off_lo), (uint32_t*)(ws + p.off_split), (uint32_t*)(ws + p.off_splitb),
	                                        p.bk.vb0, p.bk.NBK, p.brick_part, (uint32_t*)(ws + p.off_bp),
	                                        p.bk.LD ? (uint32_t*)(ws + p.off_fb + (size_t)g.offsets[p.bk.LD] * g.n_features * 8) : nullptr);
	NGP_HIP(hipGetLastError());
}

uint32_t scatter_bucket_at_param(const GridDesc& g, const ScatterPlan& p, uint64_t param) {
	const Levels lv = make_levels(g, p.B, p.bk);
	for (uint32_t vb = 0; vb < p.n_buckets; ++vb) {
		uint32_t l = 0;
		while (lv.vb_base[l + 1] <= vb) ++l;
		const uint64_t e1 = std::min<uint64_t>((uint64_t)g.offsets[l] + ((uint64_t)(vb - lv.vb_base[l] + 1) << p.B), g.offsets[l + 1]);
		if (e1 * g.n_features > param) return vb;
	}
	return p.n_buckets;
}

void grid_backward_sorted(const GridDesc& g, const GridBwdArgs& b, const ScatterPlan& p, void* workspace, hipStream_t s,
                          bool overwrite, uint32_t debug, const SlabJob* slab, const FusedAdam* fused, const BwdParts* parts) {
	if (b.n == 0) return;
	NGP_CHECK(b.level_begin == 0, "grid_backward_sorted handles all levels");
	NGP_CHECK(!fused || (overwrite && g.n_features >= 2), "fused optimizer: overwrite mode, F >= 2");
	NGP_CHECK(!parts || !parts->k || (!p.bk.LD && !(fused && fused->rec) && parts->k <= BwdParts::MAX),
	          "grid backward parts: not with bricks or the fused update");
	const GridConst c = make_grid_const(g);
	const Levels lv = make_levels(g, p.B, p.bk);
	const FusedAdam fa = fused ? *fused : FusedAdam{};
	if (g.n_dims == 3) launch_backward<3>(g.n_features, c, lv, b, p, (char*)workspace, s, overwrite, debug, slab, fa, parts);
	else launch_backward<2>(g.n_features, c, lv, b, p, (char*)workspace, s, overwrite, debug, slab, fa, parts);
}

}  // namespace ngp
