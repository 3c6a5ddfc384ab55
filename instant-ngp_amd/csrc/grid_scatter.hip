// grid_scatter.hip — hash-grid backward as a destination-bucketed exact reduction.
//
// The tcnn backward (tcnn::kernel_grid_backward, half2 atomicAdd per (sample, level, corner)) is bound
// on MI355X by the memory-side atomic rate: ~21 G requests/s, one request per 64-B segment and
// wave-instruction, repeated addresses not merged (profiles/r01_atomics2.txt). Here the same
// contributions — weight * dL/dy rounded to fp16 exactly as tcnn rounds them before its atomic — are
// counting-sorted by destination bucket (2^B consecutive table entries), and one workgroup per
// bucket chunk sums them in LDS with 64-bit integer atomics in units of 2^-24 (the fp16 quantum, so
// every fp16 contribution is exact and the sum is order-independent; LDS integer atomics run ~12x
// faster than LDS float atomics on gfx950, profiles/r01_lds_atomics.txt). Each touched entry then
// takes one packed fp16 atomic per bucket chunk, coalesced along the table.
//
//   k_sc_hist    per block of samples: LDS histogram of item buckets -> hist[bucket][block]
//   (hipCUB)     exclusive scan of hist -> item offsets (bucket-major, so buckets are contiguous)
//   k_sc_scatter per block and level: LDS counting sort by bucket, then (entry & (2^B-1)) as u16 and
//                the F fp16 values written out as runs (coalesced)
//   k_sc_bucket  per bucket: zero LDS, accumulate, store every entry once (no memset, no atomics)
//   k_sc_split   parts of oversized buckets (coarse levels): accumulate, packed fp16 atomics
#include <hipcub/hipcub.hpp>

#include "grid_scatter.h"

#include <algorithm>

namespace ngp {

namespace {

constexpr uint32_t SC_THREADS = 256;
constexpr uint32_t SC_SPT = 1;                // samples per thread in the scatter (2 measured slower: LDS-bound occupancy)
constexpr size_t SC_LDS_BYTES = 64 * 1024;  // one bucket's int64 accumulators
constexpr float FIX_SCALE = 16777216.0f;    // 2^24: fp16 values are integer multiples of 2^-24

template <uint32_t D>
__device__ __forceinline__ void load_pos(const GridBwdArgs& a, uint32_t i, float* x) {
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * a.pos_stride + d];
}

template <uint32_t D>
__global__ void __launch_bounds__(SC_THREADS) k_sc_hist(const GridConst c, const GridBwdArgs a, uint32_t spb, uint32_t B,
                                                        uint32_t n_buckets, uint32_t* __restrict__ hist) {
	extern __shared__ uint32_t h[];
	for (uint32_t b = threadIdx.x; b < n_buckets; b += blockDim.x) h[b] = 0;
	__syncthreads();
	const uint32_t lo = blockIdx.x * spb, hi = min(lo + spb, a.n);
	for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
		float x[D];
		load_pos<D>(a, i, x);
		for (uint32_t l = 0; l < c.n_levels; ++l) {
			float frac[D]; uint32_t base[D];
			level_setup<D>(c, l, x, frac, base);
#pragma unroll
			for (uint32_t k = 0; k < (1u << D); ++k) atomicAdd(&h[corner_index<D>(c, l, base, k) >> B], 1u);
		}
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < n_buckets; b += blockDim.x) hist[(size_t)b * gridDim.x + blockIdx.x] = h[b];
}

template <uint32_t F> struct ValVec;
template <> struct ValVec<1> { typedef f16 T; };
template <> struct ValVec<2> { typedef f16x2 T; };
template <> struct ValVec<4> { typedef f16x4 T; };
template <> struct ValVec<8> { typedef f16x8 T; };

// Scatter, one level at a time: the block's items of the level are counting-sorted by bucket in LDS
// first, then written out as runs, so consecutive lanes store consecutive addresses (a scattered
// per-item store costs a memory request each, like an atomic).
template <uint32_t D, uint32_t F, uint32_t SPT>
__global__ void __launch_bounds__(SC_THREADS) k_sc_scatter(const GridConst c, const GridBwdArgs a, uint32_t spb, uint32_t B,
                                                           uint32_t n_buckets, uint32_t max_lb, const uint32_t* __restrict__ offs,
                                                           uint16_t* __restrict__ item_idx, f16* __restrict__ item_val, uint32_t debug) {
	typedef typename ValVec<F>::T V;
	constexpr uint32_t NC = 1u << D;
	extern __shared__ uint32_t lds[];
	uint32_t* cur = lds;                            // [n_buckets] global cursors of this block
	uint32_t* lh = cur + n_buckets;                 // [max_lb] level-local bucket counts
	uint32_t* loff = lh + max_lb;                   // [max_lb + 1] level-local exclusive offsets
	uint32_t* st_pos = loff + max_lb + 1;                 // [spb * NC] global item position
	uint16_t* st_idx = (uint16_t*)(st_pos + spb * NC);    // [spb * NC]
	V* st_val = (V*)(((uintptr_t)(st_idx + spb * NC) + 15) & ~(uintptr_t)15);  // [spb * NC]
	const uint32_t LF = c.n_levels * F;
	f16* st_dl = (f16*)(((uintptr_t)(st_val + spb * NC) + 15) & ~(uintptr_t)15);  // [spb * LF] (AoS dL/dy rows)
	__shared__ uint32_t wsum[SC_THREADS / 64];
	if (!(debug & 64))
	for (uint32_t b = threadIdx.x; b < n_buckets; b += blockDim.x) cur[b] = offs[(size_t)b * gridDim.x + blockIdx.x];
	const uint32_t mask = (1u << B) - 1u;
	const uint32_t lo = blockIdx.x * spb, hi = min(lo + spb, a.n);
	const uint32_t n_it = (hi - lo) * NC;
	// everything the level loop reads from memory is loaded once up front (the loop is a chain of
	// barriers; a global-load latency per level would serialise it)
	const bool aos = a.dy_layout == AoS;
	if (aos && !(debug & 128)) {
		const bool vec = (LF % 8) == 0 && (a.dy_stride % 8) == 0 && (((uintptr_t)a.dL_dy) & 15) == 0;
		if (vec) {
			const uint32_t per = LF / 8;
			for (uint32_t t = threadIdx.x; t < (hi - lo) * per; t += blockDim.x) {
				const uint32_t sI = t / per, j = t % per;
				((f16x8*)st_dl)[sI * per + j] = *(const f16x8*)(a.dL_dy + (size_t)(lo + sI) * a.dy_stride + 8 * j);
			}
		} else {
			for (uint32_t t = threadIdx.x; t < (hi - lo) * LF; t += blockDim.x) {
				const uint32_t sI = t / LF, j = t % LF;
				st_dl[sI * LF + j] = a.dL_dy[(size_t)(lo + sI) * a.dy_stride + j];
			}
		}
	}
	float xs[SPT][D], mls[SPT];
#pragma unroll
	for (uint32_t q = 0; q < SPT; ++q) {
		const uint32_t i = lo + q * blockDim.x + threadIdx.x;
		if (i < hi) {
			load_pos<D>(a, i, xs[q]);
			mls[q] = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
		}
	}
	for (uint32_t l = 0; l < c.n_levels; ++l) {
		const uint32_t b_first = c.offsets[l] >> B;
		const uint32_t nlb = ((c.offsets[l + 1] - 1) >> B) - b_first + 1;
		for (uint32_t b = threadIdx.x; b < nlb; b += blockDim.x) lh[b] = 0;
		__syncthreads();
		// 1. this thread's SPT samples: items of the level, rank within (block, bucket)
		uint32_t e[SPT][NC], r[SPT][NC];
		V val[SPT][NC];
#pragma unroll
		for (uint32_t q = 0; q < SPT; ++q) {
			const uint32_t sI = q * blockDim.x + threadIdx.x;
			const uint32_t i = lo + sI;
			if (i >= hi) continue;
			const float* x = xs[q];
			const bool active = !((float)l > mls[q] + 1e-3f);  // tcnn backward: levels beyond max_level get nothing
			float g[F];
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				float v = 0.f;
				if (active)
					v = aos ? (float)st_dl[sI * LF + l * F + f] : (float)a.dL_dy[(size_t)(l * F + f) * a.dy_stride + i];
				g[f] = v;
			}
			float frac[D]; uint32_t base[D];
			level_setup<D>(c, l, x, frac, base);
#pragma unroll
			for (uint32_t k = 0; k < NC; ++k) {
				e[q][k] = corner_index<D>(c, l, base, k);
				r[q][k] = (debug & 32) ? k : atomicAdd(&lh[(e[q][k] >> B) - b_first], 1u);
				const float w = corner_weight<D>(frac, k);
				if constexpr (F == 1) val[q][k] = (f16)(w * g[0]);
				else {
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) val[q][k][f] = (f16)(w * g[f]);
				}
			}
		}
		__syncthreads();
		// 2. block-local exclusive scan of lh: wave scans, carried across passes of blockDim buckets
		for (uint32_t b0 = 0; b0 < nlb; b0 += blockDim.x) {
			const uint32_t b = b0 + threadIdx.x;
			const uint32_t v = b < nlb ? lh[b] : 0u;
			uint32_t incl = v;
#pragma unroll
			for (uint32_t o = 1; o < 64; o <<= 1) {
				const uint32_t t = __shfl_up(incl, o, 64);
				if ((threadIdx.x & 63) >= o) incl += t;
			}
			if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
			__syncthreads();
			uint32_t carry = b0 ? loff[b0] : 0u;
			for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) carry += wsum[w];
			__syncthreads();  // loff[b0] read by all before it is overwritten below
			if (b < nlb) loff[b] = carry + incl - v;
			if (threadIdx.x == blockDim.x - 1) loff[min(b0 + blockDim.x, nlb)] = carry + incl;
			__syncthreads();
		}
		// 3. stage items at their block-local sorted slot, with their final global position
#pragma unroll
		for (uint32_t q = 0; q < SPT; ++q) {
			if (debug & 16) break;
			if (lo + q * blockDim.x + threadIdx.x >= hi) continue;
#pragma unroll
			for (uint32_t k = 0; k < NC; ++k) {
				const uint32_t lb = (e[q][k] >> B) - b_first;
				const uint32_t slot = loff[lb] + r[q][k];
				st_pos[slot] = cur[b_first + lb] + r[q][k];
				st_idx[slot] = (uint16_t)(e[q][k] & mask);
				st_val[slot] = val[q][k];
			}
		}
		__syncthreads();
		// 4. write out: consecutive slots of a bucket are consecutive global positions (coalesced runs)
		if (!(debug & 8))
		for (uint32_t t = threadIdx.x; t < n_it; t += blockDim.x) {
			const uint32_t gpos = st_pos[t];
			item_idx[gpos] = st_idx[t];
			*(V*)(item_val + (size_t)gpos * F) = st_val[t];
		}
		for (uint32_t b = threadIdx.x; b < nlb; b += blockDim.x) cur[b_first + b] += lh[b];
		__syncthreads();
	}
}

// bucket start = offs[b * n_blocks] (bucket-major scan); end of the last bucket = n_items
__device__ __forceinline__ uint32_t bucket_start(const uint32_t* offs, uint32_t n_blocks, uint32_t n_buckets, uint32_t n_items,
                                                 uint32_t b) {
	return b >= n_buckets ? n_items : offs[(size_t)b * n_blocks];
}

template <uint32_t F>
__device__ __forceinline__ void accumulate_items(unsigned long long* acc, uint32_t lo, uint32_t hi, const uint16_t* __restrict__ item_idx,
                                                 const f16* __restrict__ item_val) {
	typedef typename ValVec<F>::T V;
	// U items per thread in flight: the loop is bound by memory-level parallelism, not LDS
	constexpr uint32_t U = 8;
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
		for (uint32_t u = 0; u < U; ++u) {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				float x;
				if constexpr (F == 1) x = (float)v[u]; else x = (float)v[u][f];
				if (x != 0.f) atomicAdd(&acc[j[u] * F + f], (unsigned long long)(long long)(x * FIX_SCALE));
			}
		}
	}
	for (uint32_t t = t0 + threadIdx.x; t < hi; t += blockDim.x) {
		const uint32_t jj = item_idx[t];
		const V vv = *(const V*)(item_val + (size_t)t * F);
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) {
			float x;
			if constexpr (F == 1) x = (float)vv; else x = (float)vv[f];
			if (x != 0.f) atomicAdd(&acc[jj * F + f], (unsigned long long)(long long)(x * FIX_SCALE));
		}
	}
}

__device__ __forceinline__ f16 fix_to_f16(unsigned long long q) { return (f16)(float)((double)(long long)q * (1.0 / FIX_SCALE)); }

// One workgroup per bucket: exact sum of the bucket's items, written once per entry with plain
// stores (overwrite: every entry, untouched ones get 0 — no separate memset; accumulate: old + sum).
// Buckets above `split_limit` items are zeroed here (overwrite) and queued for k_sc_split.
template <uint32_t F>
__global__ void __launch_bounds__(SC_THREADS) k_sc_bucket(const uint32_t* __restrict__ offs, uint32_t n_blocks, uint32_t n_buckets,
                                                          uint32_t n_items, uint32_t B, uint32_t n_entries, uint32_t split_limit,
                                                          uint32_t part, const uint16_t* __restrict__ item_idx,
                                                          const f16* __restrict__ item_val, f16* __restrict__ grad, bool overwrite,
                                                          uint32_t* __restrict__ split,
                                                          uint32_t debug) {
	extern __shared__ unsigned long long acc[];
	const uint32_t b = blockIdx.x;
	const uint32_t lo = bucket_start(offs, n_blocks, n_buckets, n_items, b);
	const uint32_t hi = bucket_start(offs, n_blocks, n_buckets, n_items, b + 1);
	const uint32_t e0 = b << B;
	const uint32_t n_e = min(1u << B, n_entries - e0);
	f16* g = grad + (size_t)e0 * F;
	if (hi - lo > split_limit || lo == hi) {
		if (overwrite)
			for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) ((uint32_t*)g)[k] = 0u;
		if (lo != hi) {  // queue the parts: split[0] counts parts, split[1 + 3p ..] = {bucket, lo, hi}
			__shared__ uint32_t base;
			const uint32_t parts = (hi - lo + part - 1) / part;
			if (threadIdx.x == 0) base = atomicAdd(&split[0], parts);
			__syncthreads();
			for (uint32_t q = threadIdx.x; q < parts; q += blockDim.x) {
				uint32_t* d = split + 1 + 3 * (size_t)(base + q);
				d[0] = b; d[1] = lo + q * part; d[2] = min(lo + (q + 1) * part, hi);
			}
		}
		return;
	}
	for (uint32_t k = threadIdx.x; k < n_e * F; k += blockDim.x) acc[k] = 0ull;
	__syncthreads();
	if (!(debug & 1)) accumulate_items<F>(acc, lo, hi, item_idx, item_val);
	__syncthreads();
	// flush: two fp16 per thread-step (n_e * F is even: entries come in multiples of 8)
	for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) {
		f16x2 v{fix_to_f16(acc[2 * k]), fix_to_f16(acc[2 * k + 1])};
		if (!overwrite) {
			const f16x2 o = ((const f16x2*)g)[k];
			v = f16x2{(f16)((float)o[0] + (float)((double)(long long)acc[2 * k] * (1.0 / FIX_SCALE))),
			          (f16)((float)o[1] + (float)((double)(long long)acc[2 * k + 1] * (1.0 / FIX_SCALE)))};
		}
		((f16x2*)g)[k] = v;
	}
}

// Oversized buckets (coarse levels, where thousands of samples share a handful of entries): parts of
// `part` items, each summed exactly in LDS and added with one packed fp16 atomic per touched pair.
template <uint32_t F>
__global__ void __launch_bounds__(SC_THREADS) k_sc_split(const uint32_t* __restrict__ offs, uint32_t n_blocks, uint32_t n_buckets,
                                                         uint32_t n_items, uint32_t B, uint32_t n_entries, uint32_t part,
                                                         const uint16_t* __restrict__ item_idx, const f16* __restrict__ item_val,
                                                         f16* __restrict__ grad, const uint32_t* __restrict__ split, uint32_t debug) {
	extern __shared__ unsigned long long acc[];
	if (blockIdx.x >= split[0]) return;
	const uint32_t* d = split + 1 + 3 * (size_t)blockIdx.x;
	const uint32_t b = d[0], lo = d[1], hi = d[2];
	const uint32_t e0 = b << B;
	const uint32_t n_e = min(1u << B, n_entries - e0);
	for (uint32_t k = threadIdx.x; k < n_e * F; k += blockDim.x) acc[k] = 0ull;
	__syncthreads();
	if (!(debug & 1)) accumulate_items<F>(acc, lo, hi, item_idx, item_val);
	__syncthreads();
	for (uint32_t k = threadIdx.x; k < n_e * F / 2; k += blockDim.x) {
		const unsigned long long q0 = acc[2 * k], q1 = acc[2 * k + 1];
		if (q0 == 0ull && q1 == 0ull) continue;
		atomic_add_f16x2(grad + (size_t)e0 * F + 2 * k, f16x2{fix_to_f16(q0), fix_to_f16(q1)});
	}
}

}  // namespace

ScatterPlan make_scatter_plan(const GridDesc& g, uint32_t n) {
	ScatterPlan p;
	const uint32_t F = g.n_features;
	// bucket = 2^B entries whose F int64 accumulators fill SC_LDS_BYTES
	p.B = 0;
	while (((size_t)2 << p.B) * F * 8 <= SC_LDS_BYTES && p.B < 16) ++p.B;
	const uint32_t n_entries = g.offsets[g.n_levels];
	p.n_buckets = (uint32_t)div_round_up(n_entries, 1u << p.B);
	NGP_CHECK((size_t)p.n_buckets * 4 <= 64 * 1024, "grid backward: table too large for the bucket histogram");
	// SC_SPT samples per thread per block (the scatter stages a block's items of a level in LDS)
	p.spb = SC_THREADS * SC_SPT;
	p.n_blocks = (uint32_t)div_round_up(n, p.spb);
	p.max_lb = 0;
	for (uint32_t l = 0; l < g.n_levels; ++l)
		p.max_lb = std::max(p.max_lb, ((g.offsets[l + 1] - 1) >> p.B) - (g.offsets[l] >> p.B) + 1);
	p.n_items = (uint64_t)n * g.n_levels * (1u << g.n_dims);
	NGP_CHECK(p.n_items < (1ull << 32), "grid backward: too many contributions for 32-bit offsets");
	p.split_limit = 65536;
	p.part = 16384;
	p.max_split_blocks = (uint32_t)(div_round_up(p.n_items, (uint64_t)p.part) + div_round_up(p.n_items, (uint64_t)p.split_limit) + 1);
	const uint32_t len = p.n_buckets * p.n_blocks;
	NGP_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, p.cub_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)len));
	auto align = [](size_t v) { return (v + 255) / 256 * 256; };
	p.off_hist = 0;
	p.off_scan = align(p.off_hist + (size_t)len * 4);
	p.off_cub = align(p.off_scan + (size_t)len * 4);
	p.off_split = align(p.off_cub + p.cub_bytes);
	p.off_idx = align(p.off_split + (1 + 3 * (size_t)p.max_split_blocks) * 4);
	p.off_val = align(p.off_idx + p.n_items * 2);
	p.total = align(p.off_val + p.n_items * F * 2);
	return p;
}

void grid_scatter_prepare(const GridDesc& g, const GridBwdArgs& a, const ScatterPlan& p, void* workspace, hipStream_t s) {
	if (a.n == 0) return;
	char* ws = (char*)workspace;
	GridConst c = make_grid_const(g);
	uint32_t* hist = (uint32_t*)(ws + p.off_hist);
	uint32_t* scan = (uint32_t*)(ws + p.off_scan);
	const size_t lds_h = (size_t)p.n_buckets * 4;
	if (g.n_dims == 3) k_sc_hist<3><<<p.n_blocks, SC_THREADS, lds_h, s>>>(c, a, p.spb, p.B, p.n_buckets, hist);
	else k_sc_hist<2><<<p.n_blocks, SC_THREADS, lds_h, s>>>(c, a, p.spb, p.B, p.n_buckets, hist);
	NGP_HIP(hipGetLastError());
	size_t bytes = p.cub_bytes;
	NGP_HIP(hipcub::DeviceScan::ExclusiveSum((void*)(ws + p.off_cub), bytes, hist, scan, (int)(p.n_buckets * p.n_blocks), s));
	NGP_HIP(hipMemsetAsync(ws + p.off_split, 0, 4, s));
}

namespace {
template <uint32_t D>
void launch_sorted(uint32_t F, const GridConst& c, const GridBwdArgs& a, const ScatterPlan& p, char* ws, hipStream_t s,
                   bool overwrite, uint32_t debug) {
	const uint32_t* scan = (const uint32_t*)(ws + p.off_scan);
	uint32_t* split = (uint32_t*)(ws + p.off_split);
	uint16_t* idx = (uint16_t*)(ws + p.off_idx);
	f16* val = (f16*)(ws + p.off_val);
	const uint32_t NC = 1u << D;
	const size_t lds_s = (size_t)(p.n_buckets + 2 * p.max_lb + 1) * 4 + (size_t)p.spb * NC * 6 + 16 + (size_t)p.spb * NC * F * 2 +
	                     16 + (size_t)p.spb * c.n_levels * F * 2;
	const uint32_t n_entries = c.offsets[c.n_levels];
	const uint32_t n_items = (uint32_t)p.n_items;
	auto go = [&](auto scatter, auto bucket, auto splitk) {
		NGP_HIP(hipFuncSetAttribute((const void*)scatter, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_s));
		if (!(debug & 4)) scatter<<<p.n_blocks, SC_THREADS, lds_s, s>>>(c, a, p.spb, p.B, p.n_buckets, p.max_lb, scan, idx, val, debug);
		NGP_HIP(hipGetLastError());
		NGP_HIP(hipFuncSetAttribute((const void*)bucket, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SC_LDS_BYTES));
		NGP_HIP(hipFuncSetAttribute((const void*)splitk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)SC_LDS_BYTES));
		bucket<<<p.n_buckets, SC_THREADS, SC_LDS_BYTES, s>>>(scan, p.n_blocks, p.n_buckets, n_items, p.B, n_entries, p.split_limit,
		                                                     p.part, idx, val, a.grad, overwrite, split, debug);
		NGP_HIP(hipGetLastError());
		splitk<<<p.max_split_blocks, SC_THREADS, SC_LDS_BYTES, s>>>(scan, p.n_blocks, p.n_buckets, n_items, p.B, n_entries, p.part,
		                                                            idx, val, a.grad, split, debug);
		NGP_HIP(hipGetLastError());
	};
	switch (F) {
		case 1: go(k_sc_scatter<D, 1, SC_SPT>, k_sc_bucket<1>, k_sc_split<1>); break;
		case 2: go(k_sc_scatter<D, 2, SC_SPT>, k_sc_bucket<2>, k_sc_split<2>); break;
		case 4: go(k_sc_scatter<D, 4, SC_SPT>, k_sc_bucket<4>, k_sc_split<4>); break;
		case 8: go(k_sc_scatter<D, 8, SC_SPT>, k_sc_bucket<8>, k_sc_split<8>); break;
		default: throw Error("grid backward: unsupported F");
	}
}
}  // namespace

void grid_backward_sorted(const GridDesc& g, const GridBwdArgs& b, const ScatterPlan& p, void* workspace, hipStream_t s,
                          bool overwrite, uint32_t debug) {
	if (b.n == 0) return;
	NGP_CHECK(b.level_begin == 0, "grid_backward_sorted handles all levels");
	GridConst c = make_grid_const(g);
	if (g.n_dims == 3) launch_sorted<3>(g.n_features, c, b, p, (char*)workspace, s, overwrite, debug);
	else launch_sorted<2>(g.n_features, c, b, p, (char*)workspace, s, overwrite, debug);
}

}  // namespace ngp
