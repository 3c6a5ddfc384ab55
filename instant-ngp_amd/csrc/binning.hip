// binning.hip — spatial binning of samples and the LDS-windowed hash-grid backward.
//
// Why: MI355X executes global float atomics at the memory side at ~21 G requests/s (one request per
// 64-B segment touched by a wave-instruction; distinct dwords of a segment merge, repeated addresses
// do not; profiles/r01_atomics*.txt). The tcnn-style backward issues one request per (sample, level,
// x-pair of corners) — 5.2 M for C2 — so it is request-bound (~240 us). Here samples are
// counting-sorted into R^D spatial bins; a workgroup owns one bin, accumulates the bin's vertex window
// of each level in LDS as integer fixed point (LDS float atomics are 12x slower than integer ones,
// profiles/r01_lds_atomics.txt) and flushes the window row by row as whole aligned 8-entry groups.
// Requests drop to about bins x window surface instead of samples x corners. Levels whose window
// does not fit LDS fall back to the direct kernel (grid.hip). Same weights and entries as tcnn; the
// per-vertex partial sums are exact fixed-point sums rounded once to fp16 at the flush.
#include <hipcub/hipcub.hpp>

#include "binning.h"

#include <cmath>

namespace ngp {

template <uint32_t D>
__device__ __forceinline__ uint32_t bin_of(const float* x, uint32_t R) {
	uint32_t b = 0, mul = 1;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) {
		int c = (int)(x[d] * (float)R);
		c = c < 0 ? 0 : (c >= (int)R ? (int)R - 1 : c);
		b += (uint32_t)c * mul;
		mul *= R;
	}
	return b;
}

// Histogram per block of BIN_BLOCK samples, written bin-major: hist[bin * n_blocks + block].
template <uint32_t D>
__global__ void __launch_bounds__(256) k_bin_hist(uint32_t n, const float* __restrict__ pos, uint32_t stride, uint32_t R,
                                                  uint32_t n_bins, uint32_t* __restrict__ hist) {
	extern __shared__ uint32_t h[];
	for (uint32_t b = threadIdx.x; b < n_bins; b += blockDim.x) h[b] = 0;
	__syncthreads();
#pragma unroll
	for (uint32_t k = 0; k < BIN_BLOCK / 256; ++k) {
		const uint32_t i = blockIdx.x * BIN_BLOCK + k * 256 + threadIdx.x;
		if (i < n) {
			float x[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) x[d] = pos[(size_t)i * stride + d];
			atomicAdd(&h[bin_of<D>(x, R)], 1u);
		}
	}
	__syncthreads();
	for (uint32_t b = threadIdx.x; b < n_bins; b += blockDim.x) hist[(size_t)b * gridDim.x + blockIdx.x] = h[b];
}

// In-place exclusive scan of `len` u32 with one 1024-thread workgroup.
__global__ void __launch_bounds__(1024) k_scan_exclusive(uint32_t* __restrict__ a, uint32_t len) {
	__shared__ uint32_t part[1024];
	const uint32_t chunk = (len + 1023) / 1024;
	const uint32_t lo = threadIdx.x * chunk, hi = min(lo + chunk, len);
	uint32_t s = 0;
	for (uint32_t i = lo; i < hi; ++i) s += a[i];
	part[threadIdx.x] = s;
	__syncthreads();
	for (uint32_t off = 1; off < 1024; off <<= 1) {
		const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
		__syncthreads();
		part[threadIdx.x] += v;
		__syncthreads();
	}
	uint32_t run = part[threadIdx.x] - s;
	for (uint32_t i = lo; i < hi; ++i) {
		const uint32_t v = a[i];
		a[i] = run;
		run += v;
	}
}

template <uint32_t D>
__global__ void __launch_bounds__(256) k_bin_scatter(uint32_t n, const float* __restrict__ pos, uint32_t stride, uint32_t R,
                                                     uint32_t n_bins, const uint32_t* __restrict__ offs,
                                                     uint32_t* __restrict__ sorted) {
	extern __shared__ uint32_t cur[];
	for (uint32_t b = threadIdx.x; b < n_bins; b += blockDim.x) cur[b] = offs[(size_t)b * gridDim.x + blockIdx.x];
	__syncthreads();
#pragma unroll
	for (uint32_t k = 0; k < BIN_BLOCK / 256; ++k) {
		const uint32_t i = blockIdx.x * BIN_BLOCK + k * 256 + threadIdx.x;
		if (i < n) {
			float x[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) x[d] = pos[(size_t)i * stride + d];
			const uint32_t p = atomicAdd(&cur[bin_of<D>(x, R)], 1u);
			sorted[p] = i;
		}
	}
}

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t entry_of(const GridConst& c, uint32_t D, uint32_t l, uint32_t x, uint32_t y, uint32_t z) {
	const uint32_t T = c.offsets[l + 1] - c.offsets[l];
	return c.offsets[l] + (D == 3 ? grid_index3(T, c.resolution[l], x, y, z) : grid_index2(T, c.resolution[l], x, y));
}

// Sum over the 64 lanes of a wave with DPP (VALU rate, no LDS traffic); the total lands in lane 63.
// Integer adds: the result does not depend on the reduction order.
__device__ __forceinline__ int32_t wave_sum_lane63(int32_t x) {
	x += __builtin_amdgcn_update_dpp(0, x, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
	x += __builtin_amdgcn_update_dpp(0, x, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
	x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
	x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
	x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
	x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
	return x;
}

// Hash-grid backward over spatial bins (one workgroup per bin at a time). Per windowed level the
// bin's vertex window lives in LDS as 32-bit fixed point (integer LDS atomics run ~12x faster than
// float ones on gfx950, profiles/r01_lds_atomics.txt; integer sums are order-independent). The
// fixed-point step 2^-S is chosen per (bin, level) from max|dL/dy| x count so no sum can overflow.
// Lanes of a wave whose samples share a cell (coarse levels) are pre-reduced with DPP and added by
// 2^D*F lanes at once; the rest add per lane. The window is flushed as aligned 8-vertex x-groups
// (one 64-B segment for F=4 fp16; the x prime of the coherent hash is 1, so the group stays aligned
// in hashed levels too) with packed fp16 atomics, skipping untouched vertices.
template <uint32_t D, uint32_t F>
__global__ void __launch_bounds__(256) k_grid_backward_win(const GridConst c, const WinArgs a) {
	static_assert(F >= 2, "windowed backward needs F >= 2");
	constexpr uint32_t NC = 1u << D;
	constexpr uint32_t P = F / 2;
	extern __shared__ int32_t win[];
	__shared__ uint32_t s_max[16];
	const uint32_t nb = a.n_hist_blocks;
	const uint32_t nwin = a.n_win;
	const uint32_t lane = threadIdx.x & 63;
	const float invR = 1.0f / (float)a.R;

	for (uint32_t bin = blockIdx.x; bin < a.n_bins; bin += gridDim.x) {
		const uint32_t start = a.offs[(size_t)bin * nb];
		const uint32_t end = bin + 1 < a.n_bins ? a.offs[(size_t)(bin + 1) * nb] : a.n;
		if (start == end) continue;
		const uint32_t count = end - start;
		uint32_t bc[3] = {0, 0, 0};
		{
			uint32_t t = bin;
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) { bc[d] = t % a.R; t /= a.R; }
		}
		// pass 0: per-level max |dL/dy| over the bin (non-negative floats order like their bits)
		if (threadIdx.x < 16) s_max[threadIdx.x] = 0u;
		__syncthreads();
		for (uint32_t l = 0; l < nwin; ++l) {
			float m = 0.f;
			for (uint32_t s = start + threadIdx.x; s < end; s += blockDim.x) {
				const f16* gp = a.dL_dy + (size_t)a.sorted[s] * a.dy_stride + l * F;
#pragma unroll
				for (uint32_t f = 0; f < F; f += 2) {
					const f16x2 v = *(const f16x2*)(gp + f);
					m = fmaxf(m, fmaxf(fabsf((float)v[0]), fabsf((float)v[1])));
				}
			}
			if (m > 0.f) atomicMax(&s_max[l], __float_as_uint(m));
		}
		__syncthreads();

		for (uint32_t l = 0; l < nwin; ++l) {
			const float mx = __uint_as_float(s_max[l]);
			if (!(mx > 0.f)) continue;  // block-uniform
			int e2;
			frexpf(mx * (float)count, &e2);  // mx * count < 2^e2
			const int S = 30 - e2;           // every |sum| <= mx * count < 2^30 in units of 2^-S
			const float to_fix = ldexpf(1.0f, S), from_fix = ldexpf(1.0f, -S);
			const float sc = c.scale[l];
			const uint32_t W = a.W[l];
			int org[3] = {0, 0, 0};
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) org[d] = (int)floorf(__builtin_fmaf(sc, (float)bc[d] * invR, 0.5f));
			const uint32_t nv = D == 3 ? W * W * W : W * W;
			for (uint32_t k = threadIdx.x; k < nv * F; k += blockDim.x) win[k] = 0;
			__syncthreads();

			// accumulate; every lane of a wave runs the same trip count (DPP needs the full wave)
			if (!(a.debug & 1))
			for (uint32_t s0 = start; s0 < end; s0 += blockDim.x) {
				const uint32_t s = s0 + threadIdx.x;
				const bool valid = s < end;
				float g[F];
				float frac[D];
				int base[D];
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) g[f] = 0.f;
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) { frac[d] = 0.f; base[d] = 0; }
				uint32_t key = 0xffffffffu;
				bool inside = false;
				if (valid) {
					const uint32_t i = a.sorted[s];
					const f16* gp = a.dL_dy + (size_t)i * a.dy_stride + l * F;
#pragma unroll
					for (uint32_t f = 0; f < F; f += 2) {
						const f16x2 v = *(const f16x2*)(gp + f);
						g[f] = (float)v[0]; g[f + 1] = (float)v[1];
					}
					inside = true;
					uint32_t lk = 0, mul = 1;
#pragma unroll
					for (uint32_t d = 0; d < D; ++d) {
						const float p = __builtin_fmaf(sc, a.pos[(size_t)i * a.pos_stride + d], 0.5f);
						const float t = floorf(p);
						base[d] = (int)t;
						frac[d] = p - t;
						const int lc = base[d] - org[d];
						inside &= lc >= 0 && lc + 1 < (int)W;
						lk += (uint32_t)lc * mul;
						mul *= W;
					}
					key = inside ? lk : 0xfffffffeu;
				}
				uint64_t rem = __ballot(valid && inside);
				// cells shared by >= 8 lanes: DPP pre-reduction, then NC*F lanes add the sums
				for (int iter = 0; rem && iter < 4; ++iter) {
					const uint32_t leader = (uint32_t)__builtin_ctzll(rem);
					const uint32_t key0 = __builtin_amdgcn_readlane(key, leader);
					const bool member = ((rem >> lane) & 1ull) && key == key0;
					const uint64_t mm = __ballot(member);
					if (__popcll(mm) < 8) break;
					int32_t mine = 0;
#pragma unroll
					for (uint32_t k = 0; k < NC; ++k) {
						float wk = 1.f;
#pragma unroll
						for (uint32_t d = 0; d < D; ++d) wk *= ((k >> d) & 1u) ? frac[d] : 1.0f - frac[d];
#pragma unroll
						for (uint32_t f = 0; f < F; ++f) {
							const int32_t v = member ? __float2int_rn(wk * g[f] * to_fix) : 0;
							const int32_t tot = __builtin_amdgcn_readlane(wave_sum_lane63(v), 63);
							if (lane == k * F + f) mine = tot;
						}
					}
					if (lane < NC * F) {
						const uint32_t k = lane / F, f = lane % F;
						uint32_t lidx = key0, mul = 1;
#pragma unroll
						for (uint32_t d = 0; d < D; ++d) { lidx += ((k >> d) & 1u) * mul; mul *= W; }
						if (mine != 0) atomicAdd(&win[lidx * F + f], mine);
					}
					rem &= ~mm;
				}
				if ((rem >> lane) & 1ull) {
#pragma unroll
					for (uint32_t k = 0; k < NC; ++k) {
						float wk = 1.f;
						uint32_t lidx = key, mul = 1;
#pragma unroll
						for (uint32_t d = 0; d < D; ++d) {
							const uint32_t bit = (k >> d) & 1u;
							wk *= bit ? frac[d] : 1.0f - frac[d];
							lidx += bit * mul;
							mul *= W;
						}
#pragma unroll
						for (uint32_t f = 0; f < F; ++f) {
							const int32_t v = __float2int_rn(wk * g[f] * to_fix);
							if (v != 0) atomicAdd(&win[lidx * F + f], v);
						}
					}
				} else if (valid && !inside) {  // outside the window (positions beyond [0,1]): global atomics
#pragma unroll
					for (uint32_t k = 0; k < NC; ++k) {
						float wk = 1.f;
						uint32_t v3[3] = {0, 0, 0};
#pragma unroll
						for (uint32_t d = 0; d < D; ++d) {
							const uint32_t bit = (k >> d) & 1u;
							wk *= bit ? frac[d] : 1.0f - frac[d];
							v3[d] = (uint32_t)(base[d] + (int)bit);
						}
						const uint32_t e = entry_of(c, D, l, v3[0], v3[1], v3[2]);
#pragma unroll
						for (uint32_t f = 0; f < F; f += 2)
							atomic_add_f16x2(a.grad + (size_t)e * F + f, f16x2{(f16)(wk * g[f]), (f16)(wk * g[f + 1])});
					}
				}
			}
			__syncthreads();

			// flush: rows of the window, aligned 8-vertex x-groups, P feature pairs per vertex
			const int gx0 = org[0] & ~7;
			const uint32_t groups = (uint32_t)(((org[0] + (int)W - 1) >> 3) - (org[0] >> 3) + 1);
			const uint32_t rows = D == 3 ? W * W : W;
			const uint32_t items = (a.debug & 2) ? 0 : rows * groups * 8 * P;
			for (uint32_t w = threadIdx.x; w < items; w += blockDim.x) {
				const uint32_t pair = w % P;
				const uint32_t vtx = (w / P) % 8;
				const uint32_t grp = (w / (P * 8)) % groups;
				const uint32_t row = w / (P * 8 * groups);
				const int gx = gx0 + 8 * (int)grp + (int)vtx;
				const int lx = gx - org[0];
				if (lx < 0 || lx >= (int)W) continue;
				const uint32_t ly = row % W, lz = D == 3 ? row / W : 0;
				const int32_t* src = win + (size_t)(lx + W * (ly + W * lz)) * F + 2 * pair;
				const int32_t v0 = src[0], v1 = src[1];
				if (v0 == 0 && v1 == 0) continue;
				const uint32_t e = entry_of(c, D, l, (uint32_t)gx, (uint32_t)(org[1] + (int)ly),
				                            D == 3 ? (uint32_t)(org[2] + (int)lz) : 0u);
				atomic_add_f16x2(a.grad + (size_t)e * F + 2 * pair, f16x2{(f16)((float)v0 * from_fix), (f16)((float)v1 * from_fix)});
			}
			__syncthreads();
		}
	}
}

// ------------------------------------------------------------------------------------------------
// Host
// ------------------------------------------------------------------------------------------------
WinPlan make_win_plan(const GridDesc& g, uint32_t n, size_t lds_budget_bytes) {
	// Cost model in units of global atomic requests (~21 G/s on MI355X, profiles/r01_atomics2.txt):
	// a windowed level costs its flushed segments per bin plus LDS work; a direct level costs one
	// request per (sample, x-pair of corners). Levels are windowed as a prefix (windows grow with level).
	WinPlan best{};
	if (g.n_features < 2) return best;
	const double seg_per_group = std::max(1.0, g.n_features * 16.0 / 64.0);  // 8 vertices x F fp16
	const double direct_per_level = (double)n * (1u << (g.n_dims - 1)) * 1.125 * seg_per_group;
	double best_cost = 1e300;
	for (uint32_t R : {4u, 6u, 8u, 10u, 12u, 16u, 20u, 24u, 32u}) {
		const uint64_t n_bins = g.n_dims == 3 ? (uint64_t)R * R * R : (uint64_t)R * R;
		if (n_bins > 32768) continue;
		WinPlan p{};
		p.R = R;
		p.n_bins = (uint32_t)n_bins;
		double cost = 0;
		uint32_t l = 0;
		for (; l < g.n_levels && l < 16; ++l) {
			const float sc = g.scale[l];
			int wmax = 0;
			for (uint32_t b = 0; b < R; ++b) {
				const int lo = (int)floorf(fmaf(sc, (float)b / (float)R, 0.5f));
				const int hi = (int)floorf(fmaf(sc, (float)(b + 1) / (float)R, 0.5f));
				wmax = std::max(wmax, hi - lo);
			}
			const uint32_t W = (uint32_t)wmax + 2;
			const uint64_t v = g.n_dims == 3 ? (uint64_t)W * W * W : (uint64_t)W * W;
			if (v * g.n_features * sizeof(int32_t) > lds_budget_bytes) break;
			const double rows = g.n_dims == 3 ? (double)W * W : (double)W;
			const double flush = std::min((double)n_bins, (double)n) * rows * (W / 8.0 + 1.0) * seg_per_group;
			// LDS integer atomics: ~2 lane-ops/clk/CU with conflicts -> ~1.2 T/s, i.e. ~60 per request-time
			const double lds = (double)n * (1u << g.n_dims) * g.n_features / 60.0;
			const double win_cost = flush + lds + (double)std::min<uint64_t>(n_bins, n) * 64.0;
			if (win_cost > direct_per_level) break;
			p.W[l] = W;
			p.max_verts = std::max<uint32_t>(p.max_verts, (uint32_t)v);
			cost += win_cost;
		}
		p.n_win = l;
		cost += direct_per_level * (g.n_levels - l);
		cost += (double)n * 0.05;  // binning
		if (p.n_win > 0 && cost < best_cost) { best_cost = cost; best = p; }
	}
	return best;
}

size_t bin_workspace_u32(const WinPlan& p, uint32_t n) {
	const uint32_t len = bin_hist_len(p, n);
	size_t bytes = 0;
	NGP_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)len));
	return 2 * (size_t)len + (bytes + 3) / 4 + 64;
}

const uint32_t* bin_offsets(const WinPlan& p, uint32_t n, const uint32_t* ws) { return ws + bin_hist_len(p, n); }

void bin_samples(uint32_t D, uint32_t n, const float* pos, uint32_t stride, const WinPlan& p, uint32_t* hist,
                 uint32_t* sorted, hipStream_t s) {
	const uint32_t nb = div_round_up(n, BIN_BLOCK);
	const size_t lds = p.n_bins * sizeof(uint32_t);
	if (D == 3) k_bin_hist<3><<<nb, 256, lds, s>>>(n, pos, stride, p.R, p.n_bins, hist);
	else k_bin_hist<2><<<nb, 256, lds, s>>>(n, pos, stride, p.R, p.n_bins, hist);
	NGP_HIP(hipGetLastError());
	// exclusive scan of the bin-major histogram (hipCUB device scan, in place via the tail buffer)
	const uint32_t len = p.n_bins * nb;
	uint32_t* scanned = hist + len;
	size_t bytes = 0;
	NGP_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, hist, scanned, (int)len, s));
	NGP_HIP(hipcub::DeviceScan::ExclusiveSum((void*)(scanned + len), bytes, hist, scanned, (int)len, s));
	hist = scanned;
	if (D == 3) k_bin_scatter<3><<<nb, 256, lds, s>>>(n, pos, stride, p.R, p.n_bins, hist, sorted);
	else k_bin_scatter<2><<<nb, 256, lds, s>>>(n, pos, stride, p.R, p.n_bins, hist, sorted);
	NGP_HIP(hipGetLastError());
}

void grid_backward_windowed(const GridDesc& g, const WinPlan& p, const GridBwdArgs& b, const uint32_t* hist,
                            const uint32_t* sorted, hipStream_t s) {
	WinArgs a{};
	a.n = b.n; a.pos = b.pos; a.pos_stride = b.pos_stride; a.dL_dy = b.dL_dy; a.dy_stride = b.dy_stride; a.grad = b.grad;
	a.sorted = sorted; a.offs = bin_offsets(p, b.n, hist); a.n_hist_blocks = div_round_up(b.n, BIN_BLOCK);
	a.debug = p.debug;
	a.R = p.R; a.n_bins = p.n_bins; a.n_win = p.n_win;
	for (uint32_t l = 0; l < 16; ++l) a.W[l] = p.W[l];
	GridConst c = make_grid_const(g);
	const size_t lds = (size_t)p.max_verts * g.n_features * sizeof(int32_t);
	const uint32_t blocks = std::min<uint32_t>(p.n_bins, 8 * device_cu_count());
	auto launch = [&](auto kern) {
		ensure_dynamic_lds((const void*)kern, lds);
		kern<<<blocks, 256, lds, s>>>(c, a);
	};
	const uint32_t key = g.n_dims * 10 + g.n_features;
	switch (key) {
		case 32: launch(k_grid_backward_win<3, 2>); break;
		case 34: launch(k_grid_backward_win<3, 4>); break;
		case 38: launch(k_grid_backward_win<3, 8>); break;
		case 22: launch(k_grid_backward_win<2, 2>); break;
		case 24: launch(k_grid_backward_win<2, 4>); break;
		case 28: launch(k_grid_backward_win<2, 8>); break;
		default: throw Error("windowed grid backward: unsupported (D, F)");
	}
	NGP_HIP(hipGetLastError());
}

}  // namespace ngp
