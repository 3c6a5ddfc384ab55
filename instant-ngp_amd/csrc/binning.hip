// binning.hip — spatial binning of samples and the LDS-windowed hash-grid backward.
//
// Why: MI355X executes global float atomics at the memory side at ~21 G requests/s (one request per
// 64-B segment touched by a wave-instruction; profiles/r01_atomics.txt). The tcnn-style backward
// issues one request per (sample, level, corner) — 8.4 M for C2 — so it is request-bound at ~400 us.
// Here samples are counting-sorted into R^D spatial bins; a workgroup owns one bin, accumulates the
// bin's vertex window of each coarse level in LDS (fp32, ds_add_f32), and flushes the window row by
// row as whole aligned 8-entry groups (one 64-B segment for F=4 fp16; the coherent hash keeps an
// aligned x-group inside one aligned 8-entry group since the x prime is 1). Requests drop to about
// bins x window surface instead of samples x corners. Levels whose window does not fit LDS fall back
// to the direct kernel (grid.hip). Semantics are unchanged (same weights, same entries, fp16 sums).
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

template <uint32_t D, uint32_t F>
__global__ void __launch_bounds__(512) k_grid_backward_win(const GridConst c, const WinArgs a) {
	static_assert(F >= 2, "windowed backward needs F >= 2");
	constexpr uint32_t P = F / 2;
	extern __shared__ float win[];
	const uint32_t nb = a.n_hist_blocks;
	const uint32_t nwin = a.n_win;
	const uint32_t total_f = a.voff[nwin] * F;
	const float invR = 1.0f / (float)a.R;

	for (uint32_t bin = blockIdx.x; bin < a.n_bins; bin += gridDim.x) {
		const uint32_t start = a.offs[(size_t)bin * nb];
		const uint32_t end = bin + 1 < a.n_bins ? a.offs[(size_t)(bin + 1) * nb] : a.n;
		if (start == end) continue;
		uint32_t bc[3] = {0, 0, 0};
		{
			uint32_t t = bin;
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) { bc[d] = t % a.R; t /= a.R; }
		}
		for (uint32_t k = threadIdx.x; k < total_f; k += blockDim.x) win[k] = 0.f;
		__syncthreads();

		// accumulate: one work item per (sample, windowed level)
		const uint32_t items = (a.debug & 1) ? 0 : (end - start) * nwin;
		for (uint32_t w = threadIdx.x; w < items; w += blockDim.x) {
			const uint32_t l = w % nwin;
			const uint32_t i = a.sorted[start + w / nwin];
			float x[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * a.pos_stride + d];
			float g[F];
			{
				const f16* gp = a.dL_dy + (size_t)i * a.dy_stride + l * F;
#pragma unroll
				for (uint32_t f = 0; f < F; f += 2) {
					const f16x2 v = *(const f16x2*)(gp + f);
					g[f] = (float)v[0]; g[f + 1] = (float)v[1];
				}
			}
			const float sc = c.scale[l];
			const uint32_t W = a.W[l];
			int org[D];
			float frac[D];
			uint32_t base[D];
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) {
				org[d] = (int)floorf(__builtin_fmaf(sc, (float)bc[d] * invR, 0.5f));
				const float p = __builtin_fmaf(sc, x[d], 0.5f);
				const float t = floorf(p);
				base[d] = (uint32_t)(int)t;
				frac[d] = p - t;
			}
#pragma unroll
			for (uint32_t k = 0; k < (1u << D); ++k) {
				float wk = 1.f;
				uint32_t v[3] = {0, 0, 0};
				bool inside = true;
				uint32_t lidx = 0, mul = 1;
#pragma unroll
				for (uint32_t d = 0; d < D; ++d) {
					const uint32_t bit = (k >> d) & 1u;
					wk *= bit ? frac[d] : 1.0f - frac[d];
					v[d] = base[d] + bit;
					const int lc = (int)v[d] - org[d];
					inside &= lc >= 0 && lc < (int)W;
					lidx += (uint32_t)lc * mul;
					mul *= W;
				}
				if (inside) {
					float* dst = win + (size_t)(a.voff[l] + lidx) * F;
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) atomicAdd(dst + f, wk * g[f]);
				} else {  // outside the window (positions beyond [0,1]): direct global atomic
					const uint32_t e = entry_of(c, D, l, v[0], v[1], v[2]);
#pragma unroll
					for (uint32_t f = 0; f < F; f += 2)
						atomic_add_f16x2(a.grad + (size_t)e * F + f, f16x2{(f16)(wk * g[f]), (f16)(wk * g[f + 1])});
				}
			}
		}
		__syncthreads();

		// flush: rows of the window, aligned 8-vertex x-groups, P feature pairs per vertex
		for (uint32_t l = 0; l < nwin; ++l) {
			const float sc = c.scale[l];
			const uint32_t W = a.W[l];
			int org[3] = {0, 0, 0};
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) org[d] = (int)floorf(__builtin_fmaf(sc, (float)bc[d] * invR, 0.5f));
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
				const float* src = win + (size_t)(a.voff[l] + lx + W * (ly + W * lz)) * F + 2 * pair;
				const float v0 = src[0], v1 = src[1];
				if (v0 == 0.f && v1 == 0.f) continue;
				const uint32_t e = entry_of(c, D, l, (uint32_t)gx, (uint32_t)(org[1] + (int)ly),
				                            D == 3 ? (uint32_t)(org[2] + (int)lz) : 0u);
				atomic_add_f16x2(a.grad + (size_t)e * F + 2 * pair, f16x2{(f16)v0, (f16)v1});
			}
		}
		__syncthreads();
	}
}

// ------------------------------------------------------------------------------------------------
// Host
// ------------------------------------------------------------------------------------------------
WinPlan make_win_plan(const GridDesc& g, uint32_t n, size_t lds_budget_bytes) {
	WinPlan best{};
	best.n_win = 0;
	if (g.n_features < 2) return best;
	double best_cost = 1e300;
	for (uint32_t R : {4u, 8u, 16u, 32u, 64u}) {
		const uint64_t n_bins = g.n_dims == 3 ? (uint64_t)R * R * R : (uint64_t)R * R;
		if (n_bins > 8192 || n_bins < 64) continue;
		WinPlan p{};
		p.R = R;
		p.n_bins = (uint32_t)n_bins;
		uint64_t verts = 0;
		double flush_req = 0;
		for (uint32_t l = 0; l < g.n_levels && l < 16; ++l) {
			const float sc = g.scale[l];
			int wmax = 0;
			for (uint32_t b = 0; b < R; ++b) {
				const int lo = (int)floorf(fmaf(sc, (float)b / (float)R, 0.5f));
				const int hi = (int)floorf(fmaf(sc, (float)(b + 1) / (float)R, 0.5f));
				wmax = std::max(wmax, hi - lo);
			}
			const uint32_t W = (uint32_t)wmax + 2;
			const uint64_t v = g.n_dims == 3 ? (uint64_t)W * W * W : (uint64_t)W * W;
			if ((verts + v) * g.n_features * sizeof(float) > lds_budget_bytes) break;
			// only window a level when the flush issues fewer segment requests than direct atomics
			const double rows = g.n_dims == 3 ? (double)W * W : (double)W;
			const double req_win = (double)n_bins * rows * (W / 8.0 + 1.0) * std::max(1.0, g.n_features * 16.0 / 64.0);
			const double req_direct = (double)n * (1u << (g.n_dims - 1)) * 1.125;
			if (req_win > req_direct) break;
			p.W[l] = W;
			p.voff[l] = (uint32_t)verts;
			verts += v;
			p.n_win = l + 1;
			flush_req += req_win;
		}
		p.voff[p.n_win] = (uint32_t)verts;
		const double direct = (double)n * (g.n_levels - p.n_win) * (1u << (g.n_dims - 1)) * 1.125;
		const double cost = flush_req + direct + (double)n * p.n_win * 0.02;  // + LDS work (small)
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
	for (uint32_t l = 0; l <= 16; ++l) a.voff[l] = p.voff[l];
	GridConst c = make_grid_const(g);
	const size_t lds = (size_t)p.voff[p.n_win] * g.n_features * sizeof(float);
	const uint32_t blocks = std::min<uint32_t>(p.n_bins, 2 * device_cu_count());
	auto launch = [&](auto kern) {
		NGP_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
		kern<<<blocks, 512, lds, s>>>(c, a);
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
