// mlp_train16.hip — the NerfNetwork training pass (tcnn FullyFusedMLP<half, 64> forward + backward as composed
// by ngp::NerfNetwork, nerf_network.h:179-335) at TWO waves per SIMD.
//
// Why a second training kernel (mlp.hip k_nerf_mlp_train keeps its 32x32 layout for the other configs): that
// kernel holds all 42 weight fragments in registers (168 AGPRs + 228 VGPRs) and four 34-KB LDS images per
// block, so each SIMD runs one wave and the forward chain's MFMA -> pack -> MFMA dependencies, the image
// stores and the LDS reads of the dW phase all stall the SIMD (PMC MfmaUtil 0.17). Here:
//   * a wave owns 16 samples: v_mfma_f32_16x16x32_f16 (and 16x16x16 where K is 16) with the samples as the
//     MFMA N dimension, so a 64-wide layer output is 4 tiles x 4 registers instead of 2 x 16;
//   * the forward weights stay in registers, the backward (transposed) weights live once per block in LDS;
//   * a block of 8 waves (2 per SIMD) covers 4 tiles of 32 samples per iteration: waves 2p and 2p+1 write
//     samples 0-15 and 16-31 of pair image p, which is laid out exactly as k_nerf_mlp_train's 32-sample image
//     of the same tile, so the dW phase (16x16x32 MFMAs, K = 32 samples of one image, images in a fixed order)
//     is the same computation, split over 8 waves instead of 4.
//
// Layouts (16x16 tiles, g = lane >> 4, n = lane & 15 = the wave's sample):
//   accumulator  D[m][n]: lane (n, g) reg r holds row m = 4g + r
//   K=32 operand B[k][n]: lane (n, g) holds 8 k; a 64-row activation packs as step s = {tile 2s regs 0..3,
//                tile 2s+1 regs 0..3}: k = 32s + {4g + 0..3, 16 + 4g + 0..3} ("permuted"); the forward
//                weights are built with the same k order, so a layer's output IS the next layer's operand
//   K=16 operand lane (n, g) holds k = 4g + 0..3: a 16-row tile's own order
// Numerics: fp16 operands, fp32 accumulation, each layer output rounded to fp16 once (RNE), ReLU on the
// rounded value: the contract of the oracle (oracle/ngp_oracle.c orc_mlp_*) and of k_nerf_mlp_train.
#include "mlp.h"

namespace ngp {
namespace {

__device__ __forceinline__ f32x4 mma32(f16x8 a, f16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f32x4 mma16(f16x4 a, f16x4 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0); }

typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f16x2 cvt2(float a, float b) { return __builtin_convertvector(f32x2v{a, b}, f16x2); }
__device__ __forceinline__ f16x2 relu2(f16x2 x) { return __builtin_elementwise_max(x, f16x2{(f16)0.f, (f16)0.f}); }
// g where the (ReLU'd, >= 0) activation a is nonzero, else 0, on packed fp16 bits (see mlp.hip relu_mask_bits)
__device__ __forceinline__ uint32_t relu_mask_bits(uint32_t a, uint32_t g) {
	uint32_t t, r;
	asm("v_and_b32 %0, 0x7fff7fff, %2\n\t"
	    "v_pk_min_u16 %0, %0, %3\n\t"
	    "v_pk_mul_lo_u16 %1, %4, %0"
	    : "=&v"(t), "=v"(r)
	    : "v"(a), "v"(0x00010001u), "v"(g));
	return r;
}

// accumulator tile -> fp16 x4 (optionally ReLU)
__device__ __forceinline__ f16x4 pack4(const f32x4& a, bool relu) {
	f16x2 lo = cvt2(a[0], a[1]), hi = cvt2(a[2], a[3]);
	if (relu) { lo = relu2(lo); hi = relu2(hi); }
	return f16x4{lo[0], lo[1], hi[0], hi[1]};
}
__device__ __forceinline__ f16x8 cat(f16x4 a, f16x4 b) { return f16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }
// 64-row output (4 tiles) -> the two K=32 operand steps, ReLU'd
__device__ __forceinline__ void pack64(const f32x4 (&acc)[4], f16x8 (&out)[2]) {
	out[0] = cat(pack4(acc[0], true), pack4(acc[1], true));
	out[1] = cat(pack4(acc[2], true), pack4(acc[3], true));
}
// ReLU backward of a 64-row dX (4 tiles) against the packed forward activation, rounded to fp16
__device__ __forceinline__ void mask64(const f32x4 (&acc)[4], const f16x8 (&act)[2], f16x8 (&out)[2]) {
#pragma unroll
	for (int s = 0; s < 2; ++s) {
		const u32x4v a = __builtin_bit_cast(u32x4v, act[s]);
		u32x4v r;
		r[0] = relu_mask_bits(a[0], __builtin_bit_cast(uint32_t, cvt2(acc[2 * s][0], acc[2 * s][1])));
		r[1] = relu_mask_bits(a[1], __builtin_bit_cast(uint32_t, cvt2(acc[2 * s][2], acc[2 * s][3])));
		r[2] = relu_mask_bits(a[2], __builtin_bit_cast(uint32_t, cvt2(acc[2 * s + 1][0], acc[2 * s + 1][1])));
		r[3] = relu_mask_bits(a[3], __builtin_bit_cast(uint32_t, cvt2(acc[2 * s + 1][2], acc[2 * s + 1][3])));
		out[s] = __builtin_bit_cast(f16x8, r);
	}
}

// k of element j in K=32 step s of lane group g: permuted (a packed 64-row activation) or standard
__device__ __forceinline__ uint32_t kperm(uint32_t s, uint32_t j, uint32_t g) { return 32 * s + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4)); }
// A layer's weights W[out x in] staged in LDS with a padded row stride (in + 2 halves: the 16 rows a
// fragment reads at one column fall into 16 different banks)
struct LW {
	const f16* w;
	uint32_t out, in, stride;
};
// One weight fragment element: transposed = false: A = W (m = output unit, k = input unit); true: A = W^T
// (m = input unit, k = output unit)
__device__ __forceinline__ f16 wval(const LW& L, bool tr, uint32_t m, uint32_t k) {
	const uint32_t o = tr ? k : m, i = tr ? m : k;
	return o < L.out && i < L.in ? L.w[o * L.stride + i] : (f16)0.f;
}
// Non-transposed fragments read whole dwords (k runs of 4 or 8 along a padded row, 4-B aligned: the rows are
// (in + 2) halves apart, in even), in range at every call site (m < out, k < in); transposed ones gather
// 2-B elements down a column.
__device__ __forceinline__ uint32_t wpair(const LW& L, uint32_t m, uint32_t k) { return *(const uint32_t*)(L.w + m * L.stride + k); }
__device__ __forceinline__ f16x8 wfrag32(const LW& L, bool tr, uint32_t t, uint32_t s, bool perm, uint32_t lane) {
	const uint32_t m = 16 * t + (lane & 15), g = lane >> 4;
	if (!tr) {
		const uint32_t k0 = perm ? 32 * s + 4 * g : 32 * s + 8 * g, k1 = perm ? k0 + 16 : k0 + 4;
		return __builtin_bit_cast(f16x8, u32x4v{wpair(L, m, k0), wpair(L, m, k0 + 2), wpair(L, m, k1), wpair(L, m, k1 + 2)});
	}
	f16x8 v;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) v[j] = wval(L, tr, m, perm ? kperm(s, j, g) : 32 * s + 8 * g + j);
	return v;
}
__device__ __forceinline__ f16x4 wfrag16(const LW& L, bool tr, uint32_t t, uint32_t lane) {
	const uint32_t m = 16 * t + (lane & 15), g = lane >> 4;
	if (!tr) return __builtin_bit_cast(f16x4, u32x2{wpair(L, m, 4 * g), wpair(L, m, 4 * g + 2)});
	f16x4 v;
#pragma unroll
	for (uint32_t j = 0; j < 4; ++j) v[j] = wval(L, tr, m, 4 * g + j);
	return v;
}

// Operand for 16x16x32 with K = the 32 samples of a pair image (see mlp.hip img_frag)
__device__ __forceinline__ f16x8 img_frag(const f16* img, int stride, int feat0, int lane) {
	const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
	const f16* a0 = img + (8 * g + q) * stride + feat0 + 4 * p;
	const f16x4 lo = lds_read_tr16(a0);
	const f16x4 hi = lds_read_tr16(a0 + 4 * stride);
	return f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// a 16-row tile (acc layout: rows 4g + 0..3) of this lane's sample into its image row at feat0
__device__ __forceinline__ void img_put4(f16* row, int feat0, int g, f16x4 v) { *(f16x4*)(row + feat0 + 4 * g) = v; }
// a packed 64-row activation (two K=32 steps) into its image row: step s covers 32s + 4g + 0..3, 32s + 16 + 4g + 0..3
__device__ __forceinline__ void img_put64(f16* row, int g, const f16x8 (&f)[2]) {
#pragma unroll
	for (int s = 0; s < 2; ++s) {
		*(f16x4*)(row + 32 * s + 4 * g) = f16x4{f[s][0], f[s][1], f[s][2], f[s][3]};
		*(f16x4*)(row + 32 * s + 16 + 4 * g) = f16x4{f[s][4], f[s][5], f[s][6], f[s][7]};
	}
}

// SH degree 4 of the warped direction (tcnn SphericalHarmonics; oracle orc_sh4): features 4g..4g+3
__device__ __forceinline__ f16x4 sh4_quad(float dx, float dy, float dz, int g) {
	const float x = dx * 2.f - 1.f, y = dy * 2.f - 1.f, z = dz * 2.f - 1.f;
	const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
	float o[4];
	if (g == 0) {
		o[0] = 0.28209479177387814f;
		o[1] = -0.48860251190291987f * y;
		o[2] = 0.48860251190291987f * z;
		o[3] = -0.48860251190291987f * x;
	} else if (g == 1) {
		o[0] = 1.0925484305920792f * xy;
		o[1] = -1.0925484305920792f * yz;
		o[2] = 0.94617469575755997f * z2 - 0.31539156525251999f;
		o[3] = -1.0925484305920792f * xz;
	} else if (g == 2) {
		o[0] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
		o[1] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
		o[2] = 2.8906114426405538f * xy * z;
		o[3] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
	} else {
		o[0] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
		o[1] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
		o[2] = 1.4453057213202769f * z * (x2 - y2);
		o[3] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
	}
	return f16x4{(f16)o[0], (f16)o[1], (f16)o[2], (f16)o[3]};
}

}  // namespace

// Pair-image layout (halves; 32 samples per image, the same strides as mlp.hip's NerfTrainLayout) and the
// LDS copy of the backward weights.
template <int ES, int DH, int RH>
struct Train16Layout {
	static constexpr int S_XE = 16 * ES + 4, S_64 = 64 + 4, S_RIN = 32 + 4, S_16 = 16 + 4;
	static constexpr int I_XE = 0;
	static constexpr int I_HD = I_XE + 32 * S_XE;                // DH x [32][64]
	static constexpr int I_RIN = I_HD + DH * 32 * S_64;          // [32][32] density out | SH
	static constexpr int I_HR = I_RIN + 32 * S_RIN;              // RH x [32][64]
	static constexpr int I_ZRO = I_HR + RH * 32 * S_64;          // dZ rgb output [32][16]
	static constexpr int I_ZRH = I_ZRO + 32 * S_16;              // (RH-1) x [32][64], j-th = layer RH-1-j
	static constexpr int I_ZR0 = I_ZRH + (RH - 1) * 32 * S_64;   // dZ rgb layer 0
	static constexpr int I_ZDO = I_ZR0 + 32 * S_64;              // dZ density output [32][16]
	static constexpr int I_ZDH = I_ZDO + 32 * S_16;              // (DH-1) x [32][64]
	static constexpr int I_ZD0 = I_ZDH + (DH - 1) * 32 * S_64;   // dZ density layer 0
	static constexpr int IMG_HALVES = I_ZD0 + 32 * S_64;
	// backward weight fragments in LDS (f16x8 = 16 B per lane for K=32 steps, f16x4 = 8 B for K=16)
	static constexpr int B_RO = 0;                               // W_ro^T: 4 tiles, K = 16        (f16x4)
	static constexpr int B_RH = B_RO + 4 * 64 * 4;               // W_rh^T: (RH-1) x 4 tiles x 2 steps (f16x8), layers RH-1..1
	static constexpr int B_R0 = B_RH + (RH - 1) * 8 * 64 * 8;    // W_r0^T: 2 tiles x 2 steps    (f16x8)
	static constexpr int B_DO = B_R0 + 4 * 64 * 8;               // W_do^T: 4 tiles, K = 16        (f16x4)
	static constexpr int B_DH = B_DO + 4 * 64 * 4;               // W_dh^T: (DH-1) x 4 x 2       (f16x8), layers DH-1..1
	static constexpr int B_D0 = B_DH + (DH - 1) * 8 * 64 * 8;    // W_d0^T: ES tiles x 2 steps   (f16x8)
	static constexpr int W_HALVES = B_D0 + ES * 2 * 64 * 8;
	static constexpr size_t LDS_BYTES = (4 * (size_t)IMG_HALVES + W_HALVES) * sizeof(f16);
	// staged parameters (kernel start, in the image region): each layer [out x (in + 2)]
	__host__ __device__ static constexpr uint32_t stage_d(int l) {
		return l == 0 ? 0u : 64u * (16 * ES + 2) + (uint32_t)(l - 1) * 64u * 66u;
	}
	static constexpr uint32_t STAGE_D = 64u * (16 * ES + 2) + (DH - 1) * 64u * 66u + 16u * 66u;
	__host__ __device__ static constexpr uint32_t stage_r(int l) {
		return STAGE_D + (l == 0 ? 0u : 64u * 34u + (uint32_t)(l - 1) * 64u * 66u);
	}
	static constexpr uint32_t STAGE_HALVES = STAGE_D + 64u * 34u + (RH - 1) * 64u * 66u + 16u * 66u;
	// the same layers transposed ([in x (out + 2)]), for the backward fragments: their A = W^T rows are then
	// dword runs too instead of 2-B gathers down a column
	__host__ __device__ static constexpr uint32_t stage_dt(int l) {
		return STAGE_HALVES + (l == 0 ? 0u : 16u * ES * 66u + (uint32_t)(l - 1) * 64u * 66u);
	}
	static constexpr uint32_t STAGE_DT = STAGE_HALVES + 16u * ES * 66u + (DH - 1) * 64u * 66u + 64u * 18u;
	__host__ __device__ static constexpr uint32_t stage_rt(int l) {
		return STAGE_DT + (l == 0 ? 0u : 32u * 66u + (uint32_t)(l - 1) * 64u * 66u);
	}
	static constexpr uint32_t STAGE_ALL = STAGE_DT + 32u * 66u + (RH - 1) * 64u * 66u + 64u * 18u;
	static_assert(STAGE_ALL <= 4 * IMG_HALVES, "parameter staging must fit the image region");
};

// Timing experiments only (-DNGP_T16_CLOCK, DESIGN §6 phase costs): block 0..1023's thread 0 stamps the
// 100-MHz wall clock at the phase boundaries (slots: 0 entry, 1 staged, 2 loop entry, then per iteration i
// 3 + 12 i + k for k = 0 inputs read, 1 density layer 0, 2 density output + SH, 3 rgb layer 0, 4 rgb hidden,
// 5 images written, 6 rgb backward chain, 7 density backward chain, 8 dL/denc stored, 9 barrier, 10 dW,
// 11 barrier; 127 exit); ngp_debug_t16_clock copies them out. Scheduling barriers around each stamp keep
// the phases apart (the stamped kernel is slower than the plain one).
#ifdef NGP_T16_CLOCK
constexpr int T16_SLOTS = 128;
__device__ uint64_t g_t16_clock[1024 * T16_SLOTS];
#define T16_MARK(i)                                                                                     \
	do {                                                                                                \
		__builtin_amdgcn_sched_barrier(0);                                                              \
		if (threadIdx.x == 0 && blockIdx.x < 1024 && (i) < T16_SLOTS) g_t16_clock[blockIdx.x * T16_SLOTS + (i)] = wall_clock64(); \
		__builtin_amdgcn_sched_barrier(0);                                                              \
	} while (0)
#define T16_IT(k) T16_MARK(3 + 12 * it + (k))
#else
#define T16_MARK(i) do {} while (0)
#define T16_IT(k) do {} while (0)
#endif

template <int ES, int DH, int RH>
__global__ void __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) k_nerf_mlp_train16(const NerfMlpArgs a) {
	using T = Train16Layout<ES, DH, RH>;
	extern __shared__ __attribute__((aligned(16))) char smem[];
	f16* imgs = (f16*)smem;
	f16* wl = imgs + 4 * T::IMG_HALVES;
	const int lane = threadIdx.x & 63, g = lane >> 4, sn = lane & 15;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int pair = wave >> 1, half = wave & 1;
	f16* img = imgs + pair * T::IMG_HALVES;
	// the MLP parameters staged in the image region, layer by layer with padded rows (T::stage_*); the
	// fragments are gathered from there (from global they cost ~150 scattered 2-B loads per lane, and from an
	// unpadded copy 16-way bank conflicts)
	f16* stage = imgs;
	T16_MARK(0);
	auto wd = [&](int l) {  // density MLP: [64 x 16ES], (DH-1) x [64 x 64], [16 x 64]
		return LW{stage + T::stage_d(l), l == DH ? 16u : 64u, l == 0 ? 16u * ES : 64u, (l == 0 ? 16u * ES : 64u) + 2u};
	};
	auto wr = [&](int l) {  // rgb MLP: [64 x 32], (RH-1) x [64 x 64], [16 x 64]
		return LW{stage + T::stage_r(l), l == RH ? 16u : 64u, l == 0 ? 32u : 64u, (l == 0 ? 32u : 64u) + 2u};
	};
	auto wdt = [&](int l) {  // transposed copies: [in x out]
		return LW{stage + T::stage_dt(l), l == 0 ? 16u * ES : 64u, l == DH ? 16u : 64u, (l == DH ? 16u : 64u) + 2u};
	};
	auto wrt = [&](int l) {
		return LW{stage + T::stage_rt(l), l == 0 ? 32u : 64u, l == RH ? 16u : 64u, (l == RH ? 16u : 64u) + 2u};
	};
	{
		// 16-B chunks (8 halves of one row: every row length is a multiple of 8), all loads issued before the
		// first store; a scalar copy loop waited on one L2 round trip per iteration (~20 of them)
		constexpr uint32_t ND = 64 * 16 * ES + (DH - 1) * 64 * 64 + 16 * 64, NR = 64 * 32 + (RH - 1) * 64 * 64 + 16 * 64;
		constexpr uint32_t NCH = (ND + NR) / 8, PER = (NCH + 511) / 512;
		const f16* pd = a.params + a.density_woff;
		const f16* pr = a.params + a.rgb_woff;
		f16x8 v[PER];
#pragma unroll
		for (uint32_t k = 0; k < PER; ++k) {
			const uint32_t c = threadIdx.x + 512 * k;
			if (c < NCH) v[k] = *(const f16x8*)(c < ND / 8 ? pd + 8 * c : pr + 8 * (c - ND / 8));
		}
		auto put8 = [&](const LW& L, const LW& Lt, uint32_t h, f16x8 x) {  // h = the chunk's first element in [out x in]
			const uint32_t o = h / L.in, i = h % L.in;
			uint32_t* d = (uint32_t*)(L.w + o * L.stride + i);
			const u32x4v u = __builtin_bit_cast(u32x4v, x);
			d[0] = u[0]; d[1] = u[1]; d[2] = u[2]; d[3] = u[3];
			f16* t = (f16*)Lt.w + i * Lt.stride + o;
#pragma unroll
			for (int j = 0; j < 8; ++j) t[j * Lt.stride] = x[j];
		};
#pragma unroll
		for (uint32_t k = 0; k < PER; ++k) {
			const uint32_t c = threadIdx.x + 512 * k;
			if (c >= NCH) continue;
			if (c < ND / 8) {
				uint32_t h = 8 * c;
#pragma unroll
				for (int l = 0; l <= DH; ++l) {
					const LW L = wd(l);
					if (h < L.out * L.in) { put8(L, wdt(l), h, v[k]); break; }
					h -= L.out * L.in;
				}
			} else {
				uint32_t h = 8 * c - ND;
#pragma unroll
				for (int l = 0; l <= RH; ++l) {
					const LW L = wr(l);
					if (h < L.out * L.in) { put8(L, wrt(l), h, v[k]); break; }
					h -= L.out * L.in;
				}
			}
		}
	}
	__syncthreads();
	T16_MARK(1);

	// backward (transposed) weights -> LDS, one copy per block: A = W^T, read as rows of the transposed copies
	for (int t = threadIdx.x; t < 4 * 64; t += blockDim.x) {  // K=16 fragments: W_ro^T and W_do^T, 4 tiles each
		const int tile = t >> 6, l = t & 63;
		*(f16x4*)(wl + T::B_RO + t * 4) = wfrag16(wrt(RH), false, tile, l);
		*(f16x4*)(wl + T::B_DO + t * 4) = wfrag16(wdt(DH), false, tile, l);
	}
	for (int t = threadIdx.x; t < (RH - 1) * 8 * 64; t += blockDim.x) {
		const int j = t / 512, f = (t >> 6) & 7, l = t & 63;  // j-th = layer RH-1-j; f = tile * 2 + step
		*(f16x8*)(wl + T::B_RH + t * 8) = wfrag32(wrt(RH - 1 - j), false, f >> 1, f & 1, true, l);
	}
	for (int t = threadIdx.x; t < 4 * 64; t += blockDim.x) {
		const int f = t >> 6, l = t & 63;
		*(f16x8*)(wl + T::B_R0 + t * 8) = wfrag32(wrt(0), false, f >> 1, f & 1, true, l);
	}
	for (int t = threadIdx.x; t < (DH - 1) * 8 * 64; t += blockDim.x) {
		const int j = t / 512, f = (t >> 6) & 7, l = t & 63;
		*(f16x8*)(wl + T::B_DH + t * 8) = wfrag32(wdt(DH - 1 - j), false, f >> 1, f & 1, true, l);
	}
	for (int t = threadIdx.x; t < ES * 2 * 64; t += blockDim.x) {
		const int f = t >> 6, l = t & 63;
		*(f16x8*)(wl + T::B_D0 + t * 8) = wfrag32(wdt(0), false, f >> 1, f & 1, true, l);
	}
	// forward weights in registers
	f16x4 wd0_16[ES == 1 ? 4 : 1];
	f16x8 wd0_32[ES == 2 ? 4 : 1];
	if constexpr (ES == 1) {
#pragma unroll
		for (int t = 0; t < 4; ++t) wd0_16[t] = wfrag16(wd(0), false, t, lane);
	} else {
#pragma unroll
		for (int t = 0; t < 4; ++t) wd0_32[t] = wfrag32(wd(0), false, t, 0, false, lane);
	}
	f16x8 wdh[DH > 1 ? DH - 1 : 1][8];
#pragma unroll
	for (int l = 1; l < DH; ++l)
#pragma unroll
		for (int f = 0; f < 8; ++f) wdh[l - 1][f] = wfrag32(wd(l), false, f >> 1, f & 1, true, lane);
	f16x8 wdo[2], wr0[4], wro[2];
	f16x8 wrh[RH > 1 ? RH - 1 : 1][8];
#pragma unroll
	for (int s = 0; s < 2; ++s) wdo[s] = wfrag32(wd(DH), false, 0, s, true, lane);
	// rgb layer 0: k = [density output rows 0..15 (the dout tile's own order) | SH 0..15]
#pragma unroll
	for (int t = 0; t < 4; ++t) wr0[t] = wfrag32(wr(0), false, t, 0, true, lane);
#pragma unroll
	for (int l = 1; l < RH; ++l)
#pragma unroll
		for (int f = 0; f < 8; ++f) wrh[l - 1][f] = wfrag32(wr(l), false, f >> 1, f & 1, true, lane);
#pragma unroll
	for (int s = 0; s < 2; ++s) wro[s] = wfrag32(wr(RH), false, 0, s, true, lane);

	// this wave's dW tiles (16x16 fp32): waves 0-3 row block m = wave of the hidden layers (n 0..3 per layer)
	// and of density layer 0 (n 0..ES-1); waves 4-7 (v = wave - 4) the output layers' column v and rgb layer
	// 0's row block v (n 0, 1): 4 + ES and 4 tiles at C2, 7 operand fragments per image either way
	constexpr int NH = (RH - 1) + (DH - 1);      // 64x64 hidden layers
	constexpr int NT_A = 4 * NH + ES;            // tiles of waves 0-3
	constexpr int NT_B = 4;                      // tiles of waves 4-7
	constexpr int NT = NT_A > NT_B ? NT_A : NT_B;
	f32x4 dw[NT];
#pragma unroll
	for (int q = 0; q < NT; ++q) dw[q] = f32x4{0.f, 0.f, 0.f, 0.f};

	// phase B operands of one pair image: waves 0-3 per hidden layer {dZ rows 16 wave, inputs n = 0..3} (rgb
	// layers RH-1..1, then density DH-1..1), then {dZ density layer 0, encoding n = 0..ES-1}; waves 4-7 {dZ rgb
	// output, rgb last hidden v, dZ rgb layer 0 rows 16 v, [density out | SH] 0, 16, dZ density output,
	// density last hidden v}
	constexpr int NOPS_A = 5 * ((RH - 1) + (DH - 1)) + 1 + ES;
	constexpr int NOPS = NOPS_A > 7 ? NOPS_A : 7;
	auto load_ops = [&](int p, f16x8 (&o)[NOPS]) {
		const f16* im = imgs + p * T::IMG_HALVES;
		if (wave < 4) {
			int k = 0;
#pragma unroll
			for (int j = 0; j < RH - 1; ++j, k += 5) {
				o[k] = img_frag(im + T::I_ZRH + j * 32 * T::S_64, T::S_64, 16 * wave, lane);
#pragma unroll
				for (int n = 0; n < 4; ++n) o[k + 1 + n] = img_frag(im + T::I_HR + (RH - 2 - j) * 32 * T::S_64, T::S_64, 16 * n, lane);
			}
#pragma unroll
			for (int j = 0; j < DH - 1; ++j, k += 5) {
				o[k] = img_frag(im + T::I_ZDH + j * 32 * T::S_64, T::S_64, 16 * wave, lane);
#pragma unroll
				for (int n = 0; n < 4; ++n) o[k + 1 + n] = img_frag(im + T::I_HD + (DH - 2 - j) * 32 * T::S_64, T::S_64, 16 * n, lane);
			}
			o[k] = img_frag(im + T::I_ZD0, T::S_64, 16 * wave, lane);
#pragma unroll
			for (int n = 0; n < ES; ++n) o[k + 1 + n] = img_frag(im + T::I_XE, T::S_XE, 16 * n, lane);
		} else {
			const int v = wave - 4;
			o[0] = img_frag(im + T::I_ZRO, T::S_16, 0, lane);
			o[1] = img_frag(im + T::I_HR + (RH - 1) * 32 * T::S_64, T::S_64, 16 * v, lane);
			o[2] = img_frag(im + T::I_ZR0, T::S_64, 16 * v, lane);
			o[3] = img_frag(im + T::I_RIN, T::S_RIN, 0, lane);
			o[4] = img_frag(im + T::I_RIN, T::S_RIN, 16, lane);
			o[5] = img_frag(im + T::I_ZDO, T::S_16, 0, lane);
			o[6] = img_frag(im + T::I_HD + (DH - 1) * 32 * T::S_64, T::S_64, 16 * v, lane);
		}
	};

	const uint32_t n_tiles = (a.n + 31) / 32;
	// inputs of this lane's sample, prefetched PF iterations ahead (one: a deeper ring measured no faster and
	// its registers are needed by phase B's double buffer)
#ifndef NGP_T16_PF
#define NGP_T16_PF 1
#endif
	constexpr int PF = NGP_T16_PF;
	struct In {
		f16x4 xe16;
		f16x8 xe32;
		float cd[3];
		f16x4 dl;
	};
	In pf[PF];
	auto load_inputs = [&](In& d, uint32_t tile) {
		const uint32_t smp = tile * 32 + 16 * half + sn;
		const uint32_t ls = smp < a.n ? smp : 0;  // past-the-end tiles read sample 0 (unconditional loads)
		if constexpr (ES == 1) d.xe16 = *(const f16x4*)(a.enc + (size_t)ls * a.enc_stride + 4 * g);
		else d.xe32 = *(const f16x8*)(a.enc + (size_t)ls * a.enc_stride + 8 * g);
		const float* cd = a.coords + (size_t)ls * a.coord_stride + a.dir_offset;
		d.cd[0] = cd[0]; d.cd[1] = cd[1]; d.cd[2] = cd[2];
		d.dl = *(const f16x4*)(a.dL_dout + (size_t)ls * a.dL_stride);
	};
#pragma unroll
	for (int k = 0; k < PF; ++k) load_inputs(pf[k], blockIdx.x * 4 + pair + k * gridDim.x * 4);
	__syncthreads();  // backward weights in LDS; the staged parameters are no longer read (images overwrite them)
	T16_MARK(2);
	[[maybe_unused]] uint32_t it = 0;

#ifndef NGP_T16_SH_AHEAD
#define NGP_T16_SH_AHEAD 0  // 1: the next tile's SH computed in the dW phase (VALU idle there, LDS-bound)
#endif
	f16x4 sh_next{};  // NGP_T16_SH_AHEAD: SH of this lane's sample in the next tile
	if constexpr (NGP_T16_SH_AHEAD) {
		const uint32_t s0 = (blockIdx.x * 4 + pair) * 32 + 16 * half + sn;
		if (s0 < a.n) sh_next = sh4_quad(pf[0].cd[0], pf[0].cd[1], pf[0].cd[2], g);
	}
	for (uint32_t base = blockIdx.x * 4; base < n_tiles; base += gridDim.x * 4) {
		const uint32_t tile = base + pair;
		const uint32_t sample = tile * 32 + 16 * half + sn;
		const bool valid = sample < a.n;
		const f16x4 xe16 = valid ? pf[0].xe16 : f16x4{};
		const f16x8 xe32 = valid ? pf[0].xe32 : f16x8{};
		const float cdx = pf[0].cd[0], cdy = pf[0].cd[1], cdz = pf[0].cd[2];
		const f16x4 dl_cur = valid ? pf[0].dl : f16x4{};
#pragma unroll
		for (int k = 0; k + 1 < PF; ++k) pf[k] = pf[k + 1];
		load_inputs(pf[PF - 1], tile + PF * gridDim.x * 4);
		const int r = 16 * half + sn;       // this lane's row in the pair images
		T16_IT(0);

		// ---- forward -----------------------------------------------------------------------------
		if constexpr (ES == 1) img_put4(img + T::I_XE + r * T::S_XE, 0, g, xe16);
		else {
			*(f16x8*)(img + T::I_XE + r * T::S_XE + 8 * g) = xe32;
		}
		f32x4 acc[4];
		f16x8 hd[DH][2];
#pragma unroll
		for (int t = 0; t < 4; ++t) {
			if constexpr (ES == 1) acc[t] = mma16(wd0_16[t], xe16, f32x4{0.f, 0.f, 0.f, 0.f});
			else acc[t] = mma32(wd0_32[t], xe32, f32x4{0.f, 0.f, 0.f, 0.f});
		}
		pack64(acc, hd[0]);
		T16_IT(1);
#pragma unroll
		for (int l = 1; l < DH; ++l) {
#pragma unroll
			for (int t = 0; t < 4; ++t) {
				f32x4 c = mma32(wdh[l - 1][2 * t], hd[l - 1][0], f32x4{0.f, 0.f, 0.f, 0.f});
				acc[t] = mma32(wdh[l - 1][2 * t + 1], hd[l - 1][1], c);
			}
			pack64(acc, hd[l]);
		}
		f32x4 dacc = mma32(wdo[1], hd[DH - 1][1], mma32(wdo[0], hd[DH - 1][0], f32x4{0.f, 0.f, 0.f, 0.f}));
		const f16x4 dout = pack4(dacc, false);                                          // density network output rows 4g..4g+3
		const f16x4 sh = NGP_T16_SH_AHEAD ? sh_next : (valid ? sh4_quad(cdx, cdy, cdz, g) : f16x4{});
		const f16x8 rin = cat(dout, sh);                                                // [density out | SH], permuted k
		T16_IT(2);
#pragma unroll
		for (int t = 0; t < 4; ++t) acc[t] = mma32(wr0[t], rin, f32x4{0.f, 0.f, 0.f, 0.f});
		f16x8 hr[RH][2];
		pack64(acc, hr[0]);
		T16_IT(3);
#pragma unroll
		for (int l = 1; l < RH; ++l) {
#pragma unroll
			for (int t = 0; t < 4; ++t) {
				f32x4 c = mma32(wrh[l - 1][2 * t], hr[l - 1][0], f32x4{0.f, 0.f, 0.f, 0.f});
				acc[t] = mma32(wrh[l - 1][2 * t + 1], hr[l - 1][1], c);
			}
			pack64(acc, hr[l]);
		}
		T16_IT(4);
		if (a.out) {
			const f32x4 racc = mma32(wro[1], hr[RH - 1][1], mma32(wro[0], hr[RH - 1][0], f32x4{0.f, 0.f, 0.f, 0.f}));
			f16x4 ro = pack4(racc, false);
			if (g == 0) ro[3] = dout[0];  // extract_density (nerf_network.h:32-43)
			if (!valid) {
			} else if (a.out_layout == 2) {
				if (g == 0) *(f16x4*)(a.out + (size_t)sample * a.out_stride) = ro;
			} else if (a.out_layout == 0) {
				*(f16x4*)(a.out + (size_t)sample * a.out_stride + 4 * g) = ro;
			} else {
#pragma unroll
				for (int j = 0; j < 4; ++j) a.out[(size_t)(4 * g + j) * a.out_stride + sample] = ro[j];
			}
		}
		// the backward chain's weight fragments, requested before the image writes (a wave's LDS requests are
		// served in order: reads queued behind the writes wait for them) and a layer or more ahead of their
		// MFMAs; the scheduling barrier keeps the compiler from sinking them next to their uses, where each
		// MFMA waited out an LDS round trip (phase clock)
		f16x4 b_ro[4], b_do[4];
		f16x8 b_rh[RH > 1 ? 8 : 1], b_r0[2];
#pragma unroll
		for (int t = 0; t < 4; ++t) b_ro[t] = *(const f16x4*)(wl + T::B_RO + (t * 64 + lane) * 4);
		if constexpr (RH > 1) {
#pragma unroll
			for (int f = 0; f < 8; ++f) b_rh[f] = *(const f16x8*)(wl + T::B_RH + (f * 64 + lane) * 8);
		}
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int l = 0; l < DH; ++l) img_put64(img + T::I_HD + l * 32 * T::S_64 + r * T::S_64, g, hd[l]);
		img_put4(img + T::I_RIN + r * T::S_RIN, 0, g, dout);
		img_put4(img + T::I_RIN + r * T::S_RIN, 16, g, sh);
#pragma unroll
		for (int l = 0; l < RH; ++l) img_put64(img + T::I_HR + l * 32 * T::S_64 + r * T::S_64, g, hr[l]);

		T16_IT(5);
		// ---- backward dX chain, every dZ kept in the pair image ------------------------------------
#ifndef NGP_T16_SKIP_BWD  // timing experiments only (phase costs)
		const float dsig = (float)dl_cur[3];
		const f16x4 dz1 = g == 0 ? f16x4{dl_cur[0], dl_cur[1], dl_cur[2], (f16)0.f} : f16x4{};  // extract_rgb (:46-60)
		img_put4(img + T::I_ZRO + r * T::S_16, 0, g, dz1);
#pragma unroll
		for (int t = 0; t < 4; ++t) acc[t] = mma16(b_ro[t], dz1, f32x4{0.f, 0.f, 0.f, 0.f});
		f16x8 dz[2];
		mask64(acc, hr[RH - 1], dz);
		// the density layer 0 fragments of dL/denc, a chain ahead
		f16x8 b_d0[2 * ES];
#pragma unroll
		for (int f = 0; f < 2; ++f) b_r0[f] = *(const f16x8*)(wl + T::B_R0 + (f * 64 + lane) * 8);
#pragma unroll
		for (int t = 0; t < 4; ++t) b_do[t] = *(const f16x4*)(wl + T::B_DO + (t * 64 + lane) * 4);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int l = RH - 1; l >= 1; --l) {
			const int j = RH - 1 - l;
			img_put64(img + T::I_ZRH + j * 32 * T::S_64 + r * T::S_64, g, dz);
			const f16* wb = wl + T::B_RH + j * 8 * 64 * 8;
#pragma unroll
			for (int t = 0; t < 4; ++t) {
				// layer RH-1's fragments were requested with the forward's image writes
				const f16x8 w0 = j == 0 ? b_rh[2 * t] : *(const f16x8*)(wb + ((2 * t) * 64 + lane) * 8);
				const f16x8 w1 = j == 0 ? b_rh[2 * t + 1] : *(const f16x8*)(wb + ((2 * t + 1) * 64 + lane) * 8);
				f32x4 c = mma32(w0, dz[0], f32x4{0.f, 0.f, 0.f, 0.f});
				acc[t] = mma32(w1, dz[1], c);
			}
			mask64(acc, hr[l - 1], dz);
		}
		img_put64(img + T::I_ZR0 + r * T::S_64, g, dz);
		T16_IT(6);
		// dL/d(rgb input): tile 0 = the density output rows, tile 1 = the SH rows (input gradients only)
		f32x4 dd_acc = mma32(b_r0[1], dz[1], mma32(b_r0[0], dz[0], f32x4{0.f, 0.f, 0.f, 0.f}));
		f16x4 dd = pack4(dd_acc, false);
		if (g == 0) dd[0] = (f16)((float)dd[0] + dsig);  // add_density_gradient (:63-74)
		// MFMAs take operands from every lane whatever EXEC says: only wave-uniform branches around them, the
		// per-lane `valid` guards only the stores
		if (a.dL_dsh) {
			const f32x4 sacc = mma32(*(const f16x8*)(wl + T::B_R0 + (3 * 64 + lane) * 8), dz[1],
			                         mma32(*(const f16x8*)(wl + T::B_R0 + (2 * 64 + lane) * 8), dz[0], f32x4{0.f, 0.f, 0.f, 0.f}));
			if (valid) *(f16x4*)(a.dL_dsh + (size_t)sample * 16 + 4 * g) = pack4(sacc, false);
		}
#pragma unroll
		for (int f = 0; f < 2 * ES; ++f) b_d0[f] = *(const f16x8*)(wl + T::B_D0 + (f * 64 + lane) * 8);
		__builtin_amdgcn_sched_barrier(0);
		img_put4(img + T::I_ZDO + r * T::S_16, 0, g, dd);
#pragma unroll
		for (int t = 0; t < 4; ++t) acc[t] = mma16(b_do[t], dd, f32x4{0.f, 0.f, 0.f, 0.f});
		mask64(acc, hd[DH - 1], dz);
#pragma unroll
		for (int l = DH - 1; l >= 1; --l) {
			const int j = DH - 1 - l;
			img_put64(img + T::I_ZDH + j * 32 * T::S_64 + r * T::S_64, g, dz);
			const f16* wb = wl + T::B_DH + j * 8 * 64 * 8;
#pragma unroll
			for (int t = 0; t < 4; ++t) {
				f32x4 c = mma32(*(const f16x8*)(wb + ((2 * t) * 64 + lane) * 8), dz[0], f32x4{0.f, 0.f, 0.f, 0.f});
				acc[t] = mma32(*(const f16x8*)(wb + ((2 * t + 1) * 64 + lane) * 8), dz[1], c);
			}
			mask64(acc, hd[l - 1], dz);
		}
		img_put64(img + T::I_ZD0 + r * T::S_64, g, dz);
		T16_IT(7);
		if (a.dL_denc) {
#pragma unroll
			for (int t = 0; t < ES; ++t) {
				const f32x4 e = mma32(b_d0[2 * t + 1], dz[1], mma32(b_d0[2 * t], dz[0], f32x4{0.f, 0.f, 0.f, 0.f}));
				if (valid) *(f16x4*)(a.dL_denc + (size_t)sample * a.denc_stride + 16 * t + 4 * g) = pack4(e, false);
			}
		}
#endif
		T16_IT(8);
		__syncthreads();
		T16_IT(9);
		if constexpr (NGP_T16_SH_AHEAD) {  // pf[0] holds the next tile's inputs (requested at this iteration's start)
			const uint32_t s1 = (tile + gridDim.x * 4) * 32 + 16 * half + sn;
			sh_next = s1 < a.n ? sh4_quad(pf[0].cd[0], pf[0].cd[1], pf[0].cd[2], g) : f16x4{};
		}

		// ---- dW over the four pair images (K = 32 samples per MFMA), images in a fixed order ---------
#ifndef NGP_T16_SKIP_B
		// operands of image p + 1 requested before image p's MFMAs (two register buffers)
		f16x8 ops[2][NOPS];
		load_ops(0, ops[0]);
#pragma unroll
		for (int p = 0; p < 4; ++p) {
			if (p < 3) load_ops(p + 1, ops[(p + 1) & 1]);
			const f16x8(&o)[NOPS] = ops[p & 1];
			if (wave < 4) {
				int q = 0, k = 0;
#pragma unroll
				for (int j = 0; j < (RH - 1) + (DH - 1); ++j, k += 5)
#pragma unroll
					for (int n = 0; n < 4; ++n, ++q) dw[q] = mma32(o[k], o[k + 1 + n], dw[q]);
#pragma unroll
				for (int n = 0; n < ES; ++n, ++q) dw[q] = mma32(o[k], o[k + 1 + n], dw[q]);
			} else {
				dw[0] = mma32(o[0], o[1], dw[0]);
				dw[1] = mma32(o[2], o[3], dw[1]);
				dw[2] = mma32(o[2], o[4], dw[2]);
				dw[3] = mma32(o[5], o[6], dw[3]);
			}
		}
#endif
		T16_IT(10);
		__syncthreads();
		T16_IT(11);
		++it;
	}

	// this wave's dW tiles -> the block's slab at their parameter-slice positions [out x in]
	float* slab = a.dw_slab + (size_t)blockIdx.x * a.n_matrix;
	auto put = [&](const f32x4& v, uint32_t woff, uint32_t in_dim, int m, int n) {
#pragma unroll
		for (int rr = 0; rr < 4; ++rr) slab[woff + (uint32_t)(16 * m + 4 * g + rr) * in_dim + 16 * n + sn] = v[rr];
	};
	const uint32_t dw0 = a.density_woff, rw0 = a.rgb_woff;
	if (wave < 4) {
		int q = 0;
#pragma unroll
		for (int j = 0; j < RH - 1; ++j)
#pragma unroll
			for (int n = 0; n < 4; ++n, ++q) put(dw[q], rw0 + 64 * 32 + 64 * 64 * (RH - 2 - j), 64, wave, n);
#pragma unroll
		for (int j = 0; j < DH - 1; ++j)
#pragma unroll
			for (int n = 0; n < 4; ++n, ++q) put(dw[q], dw0 + 64 * 16 * ES + 64 * 64 * (DH - 2 - j), 64, wave, n);
#pragma unroll
		for (int n = 0; n < ES; ++n, ++q) put(dw[q], dw0, 16 * ES, wave, n);
	} else {
		const int v = wave - 4;
		put(dw[0], rw0 + 64 * 32 + 64 * 64 * (RH - 1), 64, 0, v);
		put(dw[1], rw0, 32, v, 0);
		put(dw[2], rw0, 32, v, 1);
		put(dw[3], dw0 + 64 * 16 * ES + 64 * 64 * (DH - 1), 64, 0, v);
	}
	T16_MARK(127);
}

template <int ES, int DH, int RH>
static bool launch_train16(const NerfMlpArgs& a, hipStream_t s) {
	using T = Train16Layout<ES, DH, RH>;
	if constexpr (T::LDS_BYTES > 160 * 1024) {
		return false;
	} else {
		const uint32_t blocks = nerf_mlp_train_blocks(a.n);
		if (blocks == 0) return true;
		auto k = k_nerf_mlp_train16<ES, DH, RH>;
		ensure_dynamic_lds((const void*)k, T::LDS_BYTES);
		k<<<blocks, 512, T::LDS_BYTES, s>>>(a);
		NGP_HIP(hipGetLastError());
		return true;
	}
}

bool nerf_mlp_train16_run(const NerfMlpPlan& p, const NerfMlpArgs& a, hipStream_t s) {
	if (!a.params || a.n == 0) return false;
	// the parameter staging reads 16-B chunks
	if (((uintptr_t)(a.params + a.density_woff) | (uintptr_t)(a.params + a.rgb_woff)) % 16) return false;
	const uint32_t key = p.enc_steps * 100 + p.d_hidden * 10 + p.r_hidden;
	switch (key) {
		case 112: return launch_train16<1, 1, 2>(a, s);
		case 111: return launch_train16<1, 1, 1>(a, s);
		case 212: return launch_train16<2, 1, 2>(a, s);
		case 211: return launch_train16<2, 1, 1>(a, s);
		default: return false;
	}
}

}  // namespace ngp

#ifdef NGP_T16_CLOCK
extern "C" __attribute__((visibility("default"))) int ngp_debug_t16_clock(uint64_t* out, uint32_t n) {
	return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ngp::g_t16_clock), (size_t)(n < 1024 * ngp::T16_SLOTS ? n : 1024 * ngp::T16_SLOTS) * 8, 0,
	                                hipMemcpyDeviceToHost);
}
#endif
