// grid.hip — hash-grid encoding kernels (forward gather, backward packed-fp16 scatter).
//
// Forward: one thread per sample walks all levels; per level the 2^D corner entries are gathered as
// one F*2-byte vector each (8 B for F=4) from the L2/Infinity-Cache-resident table and trilinearly
// blended in fp32 (tcnn blends in the table precision; see DESIGN.md §Grid for the tolerance).
// Backward: F/2 lanes per sample so that the lanes updating one entry hit one 64-B atomic segment —
// MI355X executes global float atomics at the memory side at ~21 G requests/s (measured,
// profiles/r01_atomics.txt), so requests, not bytes, are the cost.
#include "grid.h"

#include <algorithm>

#include <cmath>
#include <cstring>

namespace ngp {

void grid_desc_init(GridDesc& g, uint32_t D, uint32_t L, uint32_t F, uint32_t log2T, uint32_t Nmin, float b) {
	NGP_CHECK(D == 2 || D == 3, "GridEncoding: n_dims must be 2 or 3");
	NGP_CHECK(L >= 1 && L <= 32, "GridEncoding: n_levels must be in [1, 32]");
	NGP_CHECK(F == 1 || F == 2 || F == 4 || F == 8, "GridEncoding: n_features_per_level must be 1, 2, 4 or 8");
	NGP_CHECK((log2T >= 4 && log2T <= 28) || log2T == GRID_LOG2_DENSE, "GridEncoding: log2_hashmap_size out of range");
	g = GridDesc{};
	g.n_dims = D; g.n_levels = L; g.n_features = F; g.log2_hashmap = log2T; g.base_resolution = Nmin;
	g.per_level_scale = b;
	const float log2b = log2f(b);
	uint32_t off = 0;
	for (uint32_t l = 0; l < L; ++l) {
		float s = exp2f((float)l * log2b) * (float)Nmin - 1.0f;
		uint32_t res = (uint32_t)ceilf(s) + 1u;
		g.scale[l] = s;
		g.resolution[l] = res;
		const uint32_t max_params = 0xffffffffu / 2;
		uint32_t n;
		if (powf((float)res, (float)D) > (float)max_params) n = max_params;
		else { n = 1; for (uint32_t d = 0; d < D; ++d) n *= res; }
		n = (n + 7u) / 8u * 8u;
		if (n > (1u << log2T)) n = 1u << log2T;
		g.offsets[l] = off;
		off += n;
	}
	g.offsets[L] = off;
}

GridConst make_grid_const(const GridDesc& g) {
	GridConst c;
	c.n_levels = g.n_levels;
	c.n_features = g.n_features;
	memcpy(c.offsets, g.offsets, sizeof(c.offsets));
	memcpy(c.scale, g.scale, sizeof(c.scale));
	memcpy(c.resolution, g.resolution, sizeof(c.resolution));
	c.hashed = 0;
	for (uint32_t l = 0; l < g.n_levels; ++l) {
		// the kind exactly as grid_index3/2 decide it: 32-bit stride, multiplied while it fits in T
		// (fine levels of large-scale grids wrap the stride and stay "dense", with index % T)
		const uint32_t T = g.offsets[l + 1] - g.offsets[l];
		uint32_t stride = g.resolution[l];
		for (uint32_t d = 1; d < g.n_dims; ++d)
			if (stride <= T) stride *= g.resolution[l];
		if (T < stride) {
			NGP_CHECK((T & (T - 1)) == 0, "GridEncoding: hashed level size must be a power of two");
			c.hashed |= 1u << l;
		}
	}
	return c;
}

template <uint32_t F> struct FeatVec;
template <> struct FeatVec<1> { typedef f16 T; };
template <> struct FeatVec<2> { typedef f16x2 T; };
template <> struct FeatVec<4> { typedef f16x4 T; };
template <> struct FeatVec<8> { typedef f16x8 T; };

template <uint32_t D, uint32_t F>
__global__ void __launch_bounds__(256) k_grid_forward(const GridConst c, const GridFwdArgs a) {
	typedef typename FeatVec<F>::T V;
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= a.n) return;
	float x[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * a.pos_stride + d];
	const float ml = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
	for (uint32_t l = 0; l < c.n_levels; ++l) {
		float acc[F];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) acc[f] = 0.f;
		if (!((float)l >= ml + 1e-3f)) {
			float frac[D]; uint32_t base[D];
			level_setup<D>(c, l, x, frac, base);
			V v[1u << D];
			gather_corners<D, F>(c, l, base, a.table, v);
#pragma unroll
			for (uint32_t k = 0; k < (1u << D); ++k) {
				const float w = corner_weight<D>(frac, k);
				if constexpr (F == 1) acc[0] = __builtin_fmaf(w, (float)v[k], acc[0]);
				else {
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) acc[f] = __builtin_fmaf(w, (float)v[k][f], acc[f]);
				}
			}
		}
		// keep the fp32 sum opaque so the last FMA is not fused with the f16 conversion (v_fma_mix*):
		// the contract is round-to-fp32 then RNE to fp16, as the oracle does
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) asm volatile("" : "+v"(acc[f]));
		if (a.out_layout == AoS) {
			V o;
			if constexpr (F == 1) o = (f16)acc[0];
			else {
#pragma unroll
				for (uint32_t f = 0; f < F; ++f) o[f] = (f16)acc[f];
			}
			*(V*)(a.out + (size_t)i * a.out_stride + l * F) = o;
		} else {
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) a.out[(size_t)(l * F + f) * a.out_stride + i] = (f16)acc[f];
		}
	}
}

// AoS fast path: every level's result stays in registers and the whole row (out_stride halves,
// zero-padded past L*F) is written with back-to-back 16-B stores, so each 64-B segment is filled by
// one wave within a few cycles. Per-level 8-B stores spaced a level's gathers apart reach HBM as
// partial segments (rocprof WRITE_SIZE 3.6x the 8.4 MB of a C2 batch, profiles/r01b_pmc_c2.json).
#ifndef NGP_FWD_FASTIDX
#define NGP_FWD_FASTIDX 1  // corner indices once per level (corner_indices), shared by the histogram and the gather;
                           // F >= 4 only (C2 forward 28.9 -> 27.3 us; with 16 levels of F = 2 the index arrays cost
                           // registers: C2' step 350 -> 393 us, profiles/r03bp)
#endif
template <uint32_t D, uint32_t F, bool HIST>
__global__ void __launch_bounds__(HIST ? 512 : 256) k_grid_forward_rows(const GridConst c, const GridFwdArgs a, const GridHist h) {
	typedef typename FeatVec<F>::T V;
	constexpr uint32_t MAXL = 32 / F;
	extern __shared__ __attribute__((aligned(16))) uint32_t hl[];  // HIST: [vb_base[L]] bucket counts of this chunk
	if constexpr (HIST) {
		for (uint32_t j = threadIdx.x; j < h.vb_base[c.n_levels]; j += blockDim.x) hl[j] = 0;
		__syncthreads();
	}
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < a.n) {
	float x[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * a.pos_stride + d];
	const float ml = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
	if constexpr (HIST && D == 3) {
		if (h.brick_levels) atomicAdd(&hl[h.brick_vb0 + brick_of(c, h.brick_levels - 1, h.brick_cells, h.bricks_per_dim, x)], 1u);
	}
	f16 row[32];
#pragma unroll
	for (uint32_t l = 0; l < MAXL; ++l) {
		float acc[F];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) acc[f] = 0.f;
		const bool active = l < c.n_levels && !((float)l >= ml + 1e-3f);
		const bool count = HIST && !(l >= h.brick_first && l < h.brick_levels);  // brick levels: counted once per sample above
		if (count && l < c.n_levels && !active) {
			// the backward stages items for masked levels too (with zero values): count them
			float frac[D]; uint32_t base[D];
			level_setup<D>(c, l, x, frac, base);
#pragma unroll
			for (uint32_t k = 0; k < (1u << D); ++k)
				atomicAdd(&hl[h.vb_base[l] + ((corner_index<D>(c, l, base, k) - c.offsets[l]) >> h.B)], 1u);
		}
		if (active) {
			float frac[D]; uint32_t base[D];
			level_setup<D>(c, l, x, frac, base);
			V v[1u << D];
			if constexpr (NGP_FWD_FASTIDX && F >= 4) {
				uint32_t cidx[1u << D];
				corner_indices<D>(c, l, base, cidx);
				if (count) {
#pragma unroll
					for (uint32_t k = 0; k < (1u << D); ++k) atomicAdd(&hl[h.vb_base[l] + ((cidx[k] - c.offsets[l]) >> h.B)], 1u);
				}
				gather_corners_at<D, F>(cidx, a.table, v);
			} else {
				if (count) {
#pragma unroll
					for (uint32_t k = 0; k < (1u << D); ++k)
						atomicAdd(&hl[h.vb_base[l] + ((corner_index<D>(c, l, base, k) - c.offsets[l]) >> h.B)], 1u);
				}
				gather_corners<D, F>(c, l, base, a.table, v);
			}
#pragma unroll
			for (uint32_t k = 0; k < (1u << D); ++k) {
				const float w = corner_weight<D>(frac, k);
				if constexpr (F == 1) acc[0] = __builtin_fmaf(w, (float)v[k], acc[0]);
				else {
#pragma unroll
					for (uint32_t f = 0; f < F; ++f) acc[f] = __builtin_fmaf(w, (float)v[k][f], acc[f]);
				}
			}
		}
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) {
			asm volatile("" : "+v"(acc[f]));  // round to fp32, then RNE to fp16 (no v_fma_mix fusion)
			row[l * F + f] = (f16)acc[f];
		}
	}
	f16x8* dst = (f16x8*)(a.out + (size_t)i * a.out_stride);
#pragma unroll
	for (uint32_t q = 0; q < 4; ++q) {
		if (8 * q >= a.out_stride) break;
		dst[q] = f16x8{row[8 * q], row[8 * q + 1], row[8 * q + 2], row[8 * q + 3],
		               row[8 * q + 4], row[8 * q + 5], row[8 * q + 6], row[8 * q + 7]};
	}
	}
	if constexpr (HIST) {
		__syncthreads();
		for (uint32_t j = threadIdx.x; j < h.vb_base[c.n_levels]; j += blockDim.x) h.hist[(size_t)blockIdx.x * h.vb_base[c.n_levels] + j] = hl[j];
	}
}

// Backward: 2P lanes per sample (P = feature pairs per entry), ordered [x0: pair 0..P-1 | x1: pair
// 0..P-1]. One wave-instruction then updates a corner and its +x neighbour, which are adjacent
// entries (dense levels) or in one aligned 8-entry group 7/8 of the time (the hash keeps x coherent:
// prime 1), so both land in one 64-B atomic segment = one memory-side request instead of two.
template <uint32_t D, uint32_t F>
__global__ void __launch_bounds__(256) k_grid_backward(const GridConst c, const GridBwdArgs a) {
	constexpr uint32_t P = F >= 2 ? F / 2 : 1;
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t i = t / (2 * P);
	const uint32_t sub = t % (2 * P);
	const uint32_t xbit = sub / P, pair = sub % P;
	if (i >= a.n) return;
	float x[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) x[d] = a.pos[(size_t)i * a.pos_stride + d];
	const float ml = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
	for (uint32_t l = a.level_begin; l < c.n_levels; ++l) {
		if ((float)l > ml + 1e-3f) break;
		float g0, g1;
		const uint32_t f0 = l * F + (F >= 2 ? 2 * pair : 0);
		if (a.dy_layout == AoS) {
			if constexpr (F >= 2) {
				f16x2 g = *(const f16x2*)(a.dL_dy + (size_t)i * a.dy_stride + f0);
				g0 = (float)g[0]; g1 = (float)g[1];
			} else {
				g0 = (float)a.dL_dy[(size_t)i * a.dy_stride + f0]; g1 = 0.f;
			}
		} else {
			g0 = (float)a.dL_dy[(size_t)f0 * a.dy_stride + i];
			g1 = F >= 2 ? (float)a.dL_dy[(size_t)(f0 + 1) * a.dy_stride + i] : 0.f;
		}
		float frac[D]; uint32_t base[D];
		level_setup<D>(c, l, x, frac, base);
#pragma unroll
		for (uint32_t q = 0; q < (1u << (D - 1)); ++q) {
			const uint32_t k = xbit | (q << 1);
			const float w = corner_weight<D>(frac, k);
			const uint32_t e = corner_index<D>(c, l, base, k);
			if constexpr (F >= 2) {
				atomic_add_f16x2(a.grad + (size_t)e * F + 2 * pair, f16x2{to_f16(w * g0), to_f16(w * g1)});
			} else {
				// F == 1: pack with a +0 partner so the 4-byte aligned packed add touches only entry e
				const size_t idx = e;
				f16x2 v = (idx & 1) ? f16x2{(f16)0.f, to_f16(w * g0)} : f16x2{to_f16(w * g0), (f16)0.f};
				atomic_add_f16x2(a.grad + (idx & ~(size_t)1), v);
			}
		}
	}
}

bool grid_forward_rows_ok(const GridDesc& g, const GridFwdArgs& a) {
	return a.out_layout == AoS && a.out_stride % 8 == 0 && a.out_stride <= 32 && g.n_levels * g.n_features <= a.out_stride &&
	       ((uintptr_t)a.out & 15) == 0;
}

template <uint32_t D>
static void launch_fwd(uint32_t F, const GridConst& c, const GridFwdArgs& a, hipStream_t s, bool rows, const GridHist* h) {
	const dim3 grid(div_round_up(a.n, 256)), block(256);
	if (h) {
		NGP_CHECK(rows && h->chunk == 512, "grid forward histogram: needs the row kernel and 512-sample chunks");
		const dim3 grid_h(div_round_up(a.n, 512));
		NGP_CHECK(grid_h.x == h->n_chunks, "grid forward histogram: chunk count mismatch");
		const size_t lds = (size_t)h->vb_base[c.n_levels] * 4;
		auto go = [&](auto kern) {
			ensure_dynamic_lds((const void*)kern, lds);
			kern<<<grid_h, 512, lds, s>>>(c, a, *h);
		};
		switch (F) {
			case 1: go(k_grid_forward_rows<D, 1, true>); return;
			case 2: go(k_grid_forward_rows<D, 2, true>); return;
			case 4: go(k_grid_forward_rows<D, 4, true>); return;
			case 8: go(k_grid_forward_rows<D, 8, true>); return;
			default: throw Error("GridEncoding: unsupported F");
		}
	}
	const GridHist none{};
	if (rows) {
		switch (F) {
			case 1: k_grid_forward_rows<D, 1, false><<<grid, block, 0, s>>>(c, a, none); return;
			case 2: k_grid_forward_rows<D, 2, false><<<grid, block, 0, s>>>(c, a, none); return;
			case 4: k_grid_forward_rows<D, 4, false><<<grid, block, 0, s>>>(c, a, none); return;
			case 8: k_grid_forward_rows<D, 8, false><<<grid, block, 0, s>>>(c, a, none); return;
			default: throw Error("GridEncoding: unsupported F");
		}
	}
	switch (F) {
		case 1: k_grid_forward<D, 1><<<grid, block, 0, s>>>(c, a); break;
		case 2: k_grid_forward<D, 2><<<grid, block, 0, s>>>(c, a); break;
		case 4: k_grid_forward<D, 4><<<grid, block, 0, s>>>(c, a); break;
		case 8: k_grid_forward<D, 8><<<grid, block, 0, s>>>(c, a); break;
		default: throw Error("GridEncoding: unsupported F");
	}
}

template <uint32_t D>
static void launch_bwd(uint32_t F, const GridConst& c, const GridBwdArgs& a, hipStream_t s) {
	const uint32_t P = F >= 2 ? F / 2 : 1;
	const dim3 grid(div_round_up((uint64_t)a.n * 2 * P, 256)), block(256);
	switch (F) {
		case 1: k_grid_backward<D, 1><<<grid, block, 0, s>>>(c, a); break;
		case 2: k_grid_backward<D, 2><<<grid, block, 0, s>>>(c, a); break;
		case 4: k_grid_backward<D, 4><<<grid, block, 0, s>>>(c, a); break;
		case 8: k_grid_backward<D, 8><<<grid, block, 0, s>>>(c, a); break;
		default: throw Error("GridEncoding: unsupported F");
	}
}

// ---- input gradients ------------------------------------------------------------------------------
// One thread per sample (the NeRF normals / SDF normals path: a render-time query, not the training hot
// path). Corner order c = 0..2^D-1, feature order f = 0..F-1, fp32 without contraction (the oracle's
// orc_grid_input_grad restates it in double).
template <uint32_t D, uint32_t F>
__global__ void __launch_bounds__(256) k_input_grad(const GridConst c, const InputGradArgs a) {
	typedef typename FeatVec<F>::T V;
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= a.n) return;
	const float* xp = a.pos + (size_t)i * a.pos_stride;
	float x[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) x[d] = xp[d];
	const float ml = (a.max_level_per_sample ? a.max_level_per_sample[i] : a.max_level) * (float)c.n_levels;
	const f16* gy = a.dL_dy + (size_t)i * a.dy_stride;
	float acc[D];
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) acc[d] = 0.f;
	for (uint32_t l = 0; l < c.n_levels; ++l) {
		if ((float)l >= ml + 1e-3f) continue;  // zeroed in the forward: the output does not depend on x
		float frac[D];
		uint32_t base[D];
		level_setup<D>(c, l, x, frac, base);
		float g[F];
#pragma unroll
		for (uint32_t f = 0; f < F; ++f) g[f] = (float)gy[l * F + f];
		float la[D];
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) la[d] = 0.f;
#pragma unroll
		for (uint32_t k = 0; k < (1u << D); ++k) {
			const V v = *(const V*)(a.table + (size_t)corner_index<D>(c, l, base, k) * F);
			float gs = 0.f;
#pragma unroll
			for (uint32_t f = 0; f < F; ++f) {
				if constexpr (F == 1) gs = gs + g[0] * (float)v;
				else gs = gs + g[f] * (float)v[f];
			}
#pragma unroll
			for (uint32_t d = 0; d < D; ++d) {
				float wo = 1.f;  // product of the other dimensions' weights, in dimension order
#pragma unroll
				for (uint32_t e = 0; e < D; ++e)
					if (e != d) wo = wo * (((k >> e) & 1u) ? frac[e] : 1.f - frac[e]);
				const float t = wo * gs;
				la[d] = ((k >> d) & 1u) ? la[d] + t : la[d] - t;
			}
		}
#pragma unroll
		for (uint32_t d = 0; d < D; ++d) acc[d] = acc[d] + c.scale[l] * la[d];
	}
	float* o = a.out + (size_t)i * a.out_stride;
#pragma unroll
	for (uint32_t d = 0; d < D; ++d) o[d] = acc[d] * a.out_scale;
	if (a.dL_dsh) {
		// d/dd of the 16 degree-4 real SH basis functions (the forward: mlp.hip sh4_frag), d = 2 dir - 1
		const float* dp = a.pos + (size_t)i * a.pos_stride + a.dir_offset;
		const float X = dp[0] * 2.f - 1.f, Y = dp[1] * 2.f - 1.f, Z = dp[2] * 2.f - 1.f;
		float s[16];
#pragma unroll
		for (int k = 0; k < 16; ++k) s[k] = (float)a.dL_dsh[(size_t)i * 16 + k];
		const float A = 0.48860251190291987f, B = 1.0925484305920792f, C = 0.94617469575755997f, E = 0.54627421529603959f,
		            G = 0.59004358992664352f, H = 2.8906114426405538f, I = 0.45704579946446572f, J = 0.3731763325901154f,
		            K = 1.4453057213202769f;
		const float X2 = X * X, Y2 = Y * Y, Z2 = Z * Z;
		float gx = 0.f, gy2 = 0.f, gz = 0.f;
		// k: 1 -A y | 2 A z | 3 -A x | 4 B xy | 5 -B yz | 6 C z^2 - c | 7 -B xz | 8 E (x^2 - y^2)
		//    9 G y (y^2 - 3x^2) | 10 H xyz | 11 I y (1 - 5z^2) | 12 J z (5z^2 - 3) | 13 I x (1 - 5z^2)
		//    14 K z (x^2 - y^2) | 15 G x (3y^2 - x^2)
		gx = gx + s[3] * (-A);
		gx = gx + s[4] * (B * Y);
		gx = gx + s[7] * (-B * Z);
		gx = gx + s[8] * (2.f * E * X);
		gx = gx + s[9] * (-6.f * G * X * Y);
		gx = gx + s[10] * (H * Y * Z);
		gx = gx + s[13] * (I * (1.f - 5.f * Z2));
		gx = gx + s[14] * (2.f * K * X * Z);
		gx = gx + s[15] * (3.f * G * (Y2 - X2));
		gy2 = gy2 + s[1] * (-A);
		gy2 = gy2 + s[4] * (B * X);
		gy2 = gy2 + s[5] * (-B * Z);
		gy2 = gy2 + s[8] * (-2.f * E * Y);
		gy2 = gy2 + s[9] * (3.f * G * (Y2 - X2));
		gy2 = gy2 + s[10] * (H * X * Z);
		gy2 = gy2 + s[11] * (I * (1.f - 5.f * Z2));
		gy2 = gy2 + s[14] * (-2.f * K * Y * Z);
		gy2 = gy2 + s[15] * (6.f * G * X * Y);
		gz = gz + s[2] * A;
		gz = gz + s[5] * (-B * Y);
		gz = gz + s[6] * (2.f * C * Z);
		gz = gz + s[7] * (-B * X);
		gz = gz + s[10] * (H * X * Y);
		gz = gz + s[11] * (-10.f * I * Y * Z);
		gz = gz + s[12] * (J * (15.f * Z2 - 3.f));
		gz = gz + s[13] * (-10.f * I * X * Z);
		gz = gz + s[14] * (K * (X2 - Y2));
		float* od = o + a.dir_offset;
		od[0] = 2.f * gx * a.out_scale;
		od[1] = 2.f * gy2 * a.out_scale;
		od[2] = 2.f * gz * a.out_scale;
	}
}

template <uint32_t D>
static void launch_input_grad(uint32_t F, const GridConst& c, const InputGradArgs& a, hipStream_t s) {
	const dim3 grid(div_round_up(a.n, 256)), block(256);
	switch (F) {
		case 1: k_input_grad<D, 1><<<grid, block, 0, s>>>(c, a); break;
		case 2: k_input_grad<D, 2><<<grid, block, 0, s>>>(c, a); break;
		case 4: k_input_grad<D, 4><<<grid, block, 0, s>>>(c, a); break;
		case 8: k_input_grad<D, 8><<<grid, block, 0, s>>>(c, a); break;
		default: throw Error("GridEncoding: unsupported F");
	}
}

void grid_input_gradient(const GridDesc& g, const InputGradArgs& a, hipStream_t stream) {
	if (a.n == 0) return;
	NGP_CHECK(!a.dL_dsh || g.n_dims == 3, "input gradient: the SH direction encoding needs a 3D grid");
	GridConst c = make_grid_const(g);
	if (g.n_dims == 3) launch_input_grad<3>(g.n_features, c, a, stream);
	else launch_input_grad<2>(g.n_features, c, a, stream);
	NGP_HIP(hipGetLastError());
}

void grid_forward(const GridDesc& g, const GridFwdArgs& a, hipStream_t stream, const GridHist* hist) {
	if (a.n == 0) return;
	GridConst c = make_grid_const(g);
	const bool rows = grid_forward_rows_ok(g, a);
	if (g.n_dims == 3) launch_fwd<3>(g.n_features, c, a, stream, rows, hist);
	else launch_fwd<2>(g.n_features, c, a, stream, rows, hist);
	NGP_HIP(hipGetLastError());
}

void grid_backward(const GridDesc& g, const GridBwdArgs& a, hipStream_t stream) {
	if (a.n == 0) return;
	GridConst c = make_grid_const(g);
	if (g.n_dims == 3) launch_bwd<3>(g.n_features, c, a, stream);
	else launch_bwd<2>(g.n_features, c, a, stream);
	NGP_HIP(hipGetLastError());
}

}  // namespace ngp
