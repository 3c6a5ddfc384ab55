// mlp.hip — MFMA kernels for the NerfNetwork MLP pair and for a single MLP (see mlp.h for the
// register/LDS layout contract).
#include "mlp.h"
#include "slab_reduce.h"

#include <type_traits>

namespace ngp {

// ------------------------------------------------------------------------------------------------
// Fragment plans
// ------------------------------------------------------------------------------------------------
static void add_frags(std::vector<FragDesc>& v, uint32_t woff, uint32_t in, uint32_t out, uint32_t tiles, uint32_t steps,
                      bool transposed, int perm_steps_mask) {
	for (uint32_t t = 0; t < tiles; ++t)
		for (uint32_t s = 0; s < steps; ++s) {
			FragDesc d;
			d.woff = woff; d.in_dim = (uint16_t)in; d.out_dim = (uint16_t)out;
			d.tile = (uint8_t)t; d.step = (uint8_t)s; d.transposed = transposed ? 1 : 0;
			d.perm = (perm_steps_mask >> s) & 1;
			v.push_back(d);
		}
}

NerfMlpPlan make_nerf_mlp_plan(uint32_t enc_width, uint32_t width, uint32_t d_hidden, uint32_t r_hidden) {
	NGP_CHECK(width == 64, "FullyFusedMLP: this engine implements n_neurons == 64");
	NGP_CHECK(enc_width == 16 || enc_width == 32, "NerfNetwork: position encoding width must pad to 16 or 32");
	NGP_CHECK(d_hidden >= 1 && d_hidden <= 3 && r_hidden >= 1 && r_hidden <= 3, "NerfNetwork: 1..3 hidden layers supported");
	NerfMlpPlan p;
	p.enc_steps = enc_width / 16; p.d_hidden = d_hidden; p.r_hidden = r_hidden;
	p.density = MlpDims{enc_width, width, d_hidden, 16};
	p.rgb = MlpDims{32, width, r_hidden, 16};
	const uint32_t rw = p.density.n_params();  // rgb MLP follows the density MLP (nerf_network.h:430-443)
	auto& v = p.descs;
	// forward fragments
	add_frags(v, p.density.layer_off(0), enc_width, 64, 2, p.enc_steps, false, 0);
	for (uint32_t h = 1; h < d_hidden; ++h) add_frags(v, p.density.layer_off(h), 64, 64, 2, 4, false, 0xF);
	add_frags(v, p.density.layer_off(d_hidden), 64, 16, 1, 4, false, 0xF);
	add_frags(v, rw + p.rgb.layer_off(0), 32, 64, 2, 2, false, 0x1);  // step 0 = packed density output, step 1 = SH
	for (uint32_t h = 1; h < r_hidden; ++h) add_frags(v, rw + p.rgb.layer_off(h), 64, 64, 2, 4, false, 0xF);
	add_frags(v, rw + p.rgb.layer_off(r_hidden), 64, 16, 1, 4, false, 0xF);
	p.n_fwd_frags = (uint32_t)v.size();
	// backward (transposed) fragments, in the order the backward chain consumes them
	add_frags(v, rw + p.rgb.layer_off(r_hidden), 64, 16, 2, 1, true, 0xF);
	for (uint32_t h = r_hidden - 1; h >= 1; --h) add_frags(v, rw + p.rgb.layer_off(h), 64, 64, 2, 4, true, 0xF);
	add_frags(v, rw + p.rgb.layer_off(0), 32, 64, 1, 4, true, 0xF);
	add_frags(v, p.density.layer_off(d_hidden), 64, 16, 2, 1, true, 0xF);
	for (uint32_t h = d_hidden - 1; h >= 1; --h) add_frags(v, p.density.layer_off(h), 64, 64, 2, 4, true, 0xF);
	add_frags(v, p.density.layer_off(0), enc_width, 64, (enc_width + 31) / 32, 4, true, 0xF);
	p.n_bwd_frags = (uint32_t)v.size() - p.n_fwd_frags;
	return p;
}

MlpPlan make_mlp_plan(uint32_t enc_width, uint32_t width, uint32_t hidden, uint32_t out_pad) {
	NGP_CHECK(width == 16 || width == 32 || width == 64, "FullyFusedMLP: this engine implements n_neurons 16, 32 and 64");
	NGP_CHECK(enc_width == 16 || enc_width == 32, "NetworkWithInputEncoding: encoding width must pad to 16 or 32");
	NGP_CHECK(out_pad == 16, "FullyFusedMLP: output width must pad to 16");
	NGP_CHECK(hidden >= 1 && hidden <= 4, "FullyFusedMLP: 1..4 hidden layers supported");
	MlpPlan p;
	p.enc_steps = enc_width / 16; p.hidden = hidden;
	p.mlp = MlpDims{enc_width, width, hidden, out_pad};
	auto& v = p.descs;
	// hidden outputs: HT tiles of 32 rows; hidden inputs: HS k-steps of 16 (MlpLayout)
	const uint32_t W = width, HT = (W + 31) / 32, HS = W / 16, pm = (1u << HS) - 1u;
	add_frags(v, p.mlp.layer_off(0), enc_width, W, HT, p.enc_steps, false, 0);
	for (uint32_t h = 1; h < hidden; ++h) add_frags(v, p.mlp.layer_off(h), W, W, HT, HS, false, pm);
	add_frags(v, p.mlp.layer_off(hidden), W, 16, 1, HS, false, pm);
	p.n_fwd_frags = (uint32_t)v.size();
	add_frags(v, p.mlp.layer_off(hidden), W, 16, HT, 1, true, 0xF);
	for (uint32_t h = hidden - 1; h >= 1; --h) add_frags(v, p.mlp.layer_off(h), W, W, HT, HS, true, pm);
	add_frags(v, p.mlp.layer_off(0), enc_width, W, (enc_width + 31) / 32, HS, true, pm);
	p.n_bwd_frags = (uint32_t)v.size() - p.n_fwd_frags;
	return p;
}

// k index held by element j of lane half h in k-step s.
__device__ __forceinline__ uint32_t frag_k(uint32_t s, uint32_t j, uint32_t h, bool perm) {
	return perm ? 16 * s + 8 * (j >> 2) + 4 * h + (j & 3) : 16 * s + 8 * h + j;
}

__global__ void k_prepare_frags(const FragDesc* __restrict__ descs, uint32_t n_frags, const f16* __restrict__ params,
                                f16x8* __restrict__ frags) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n_frags * 64) return;
	const FragDesc d = descs[t / 64];
	const uint32_t lane = t % 64, h = lane >> 5, r = 32 * d.tile + (lane & 31);
	f16x8 v;
#pragma unroll
	for (uint32_t j = 0; j < 8; ++j) {
		const uint32_t k = frag_k(d.step, j, h, d.perm);
		f16 x = (f16)0.f;
		if (!d.transposed) {  // A = W: row r = output unit, k = input unit
			if (r < d.out_dim && k < d.in_dim) x = params[d.woff + r * d.in_dim + k];
		} else {              // A = W^T: row r = input unit, k = output unit
			if (r < d.in_dim && k < d.out_dim) x = params[d.woff + k * d.in_dim + r];
		}
		v[j] = x;
	}
	frags[t] = v;
}

void prepare_frags(const FragDesc* descs_dev, uint32_t n_frags, const f16* params, f16x8* frags, hipStream_t s) {
	k_prepare_frags<<<div_round_up(n_frags * 64, 256), 256, 0, s>>>(descs_dev, n_frags, params, frags);
	NGP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Device building blocks
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
	return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
	return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// acc[t] = sum_s A(frag base + t*STEPS + s) * in[s]
template <int TILES, int STEPS>
__device__ __forceinline__ void layer_fwd(f32x16 (&acc)[TILES], const f16x8* in, const f16x8* frags, int lane) {
#pragma unroll
	for (int t = 0; t < TILES; ++t) {
		f32x16 c = {};
#pragma unroll
		for (int s = 0; s < STEPS; ++s) c = mfma32(frags[(t * STEPS + s) * 64 + lane], in[s], c);
		acc[t] = c;
	}
}

// Same layer with the weight fragments held in registers (w[off + t * STEPS + s]); off is a
// compile-time constant after unrolling, so the array never leaves registers.
template <int TILES, int STEPS, int NR>
__device__ __forceinline__ void layer_fwd_reg(f32x16 (&acc)[TILES], const f16x8 (&in)[STEPS], const f16x8 (&w)[NR], int off) {
#pragma unroll
	for (int t = 0; t < TILES; ++t) {
		f32x16 c = {};
#pragma unroll
		for (int s = 0; s < STEPS; ++s) c = mfma32(w[off + t * STEPS + s], in[s], c);
		acc[t] = c;
	}
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// two fp32 -> packed fp16, round to nearest even (v_cvt_pk_f16_f32 on gfx950)
__device__ __forceinline__ f16x2 cvt2(float a, float b) { return __builtin_convertvector(f32x2{a, b}, f16x2); }
#ifndef NGP_RELU_INT
#define NGP_RELU_INT 1
#endif
typedef short s16x2 __attribute__((ext_vector_type(2)));
// ReLU on a packed pair. NGP_RELU_INT: as a signed 16-bit max (v_pk_max_i16): a negative half, -0
// included, has its sign bit set and becomes +0; a non-negative one orders like its integer bits.
// Equal to max(x, 0) for every non-NaN x, and never yields -0, so the backward mask needs no sign
// clear. (A NaN with the sign bit clear passes through instead of becoming 0.)
__device__ __forceinline__ f16x2 relu2(f16x2 x) {
#if NGP_RELU_INT
	return __builtin_bit_cast(f16x2, __builtin_elementwise_max(__builtin_bit_cast(s16x2, x), s16x2{0, 0}));
#else
	return __builtin_elementwise_max(x, f16x2{(f16)0.f, (f16)0.f});
#endif
}
// backward ReLU: g where the (already ReLU'd, so >= 0) activation is nonzero, else 0, on packed bits:
// a min 1 is 1 or 0 per half, times g's bits (v_pk_min_u16 + v_pk_mul_lo_u16). Keeps no per-element
// lane masks alive between the forward and the backward pass.
__device__ __forceinline__ uint32_t relu_mask_bits(uint32_t a, uint32_t g) {
	// written out: the compiler otherwise turns the idiom back into per-half compares and selects
	uint32_t t, r;
#if NGP_RELU_INT
	asm("v_pk_min_u16 %0, %2, %3\n\t"
	    "v_pk_mul_lo_u16 %1, %4, %0"
	    : "=&v"(t), "=v"(r)
	    : "v"(a), "v"(0x00010001u), "v"(g));
#else
	// v_pk_max_f16 may return -0 for a -0 input: clear the sign first
	asm("v_and_b32 %0, 0x7fff7fff, %2\n\t"
	    "v_pk_min_u16 %0, %0, %3\n\t"
	    "v_pk_mul_lo_u16 %1, %4, %0"
	    : "=&v"(t), "=v"(r)
	    : "v"(a), "v"(0x00010001u), "v"(g));
#endif
	return r;
}
__device__ __forceinline__ f16x8 cat4(f16x2 a, f16x2 b, f16x2 c, f16x2 d) {
	return f16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// Round an accumulator tile to fp16 (optionally ReLU) and split into the two k-step fragments.
__device__ __forceinline__ void pack_tile(const f32x16& a, f16x8& lo, f16x8& hi, bool relu) {
	f16x2 l[4], h[4];
#pragma unroll
	for (int q = 0; q < 4; ++q) {
		l[q] = cvt2(a[2 * q], a[2 * q + 1]);
		h[q] = cvt2(a[8 + 2 * q], a[8 + 2 * q + 1]);
		if (relu) { l[q] = relu2(l[q]); h[q] = relu2(h[q]); }
	}
	lo = cat4(l[0], l[1], l[2], l[3]);
	hi = cat4(h[0], h[1], h[2], h[3]);
}

template <int TILES>
__device__ __forceinline__ void pack_tiles(const f32x16 (&acc)[TILES], f16x8 (&out)[2 * TILES], bool relu) {
#pragma unroll
	for (int t = 0; t < TILES; ++t) pack_tile(acc[t], out[2 * t], out[2 * t + 1], relu);
}

// ReLU backward against the saved (packed) forward activation, then round to fp16.
template <int TILES>
__device__ __forceinline__ void mask_pack(const f32x16 (&acc)[TILES], const f16x8 (&act)[2 * TILES], f16x8 (&out)[2 * TILES]) {
#pragma unroll
	for (int t = 0; t < TILES; ++t)
#pragma unroll
		for (int h = 0; h < 2; ++h) {
			typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
			const u32x4 a = __builtin_bit_cast(u32x4, act[2 * t + h]);
			u32x4 r;
#pragma unroll
			for (int q = 0; q < 4; ++q)
				r[q] = relu_mask_bits(a[q], __builtin_bit_cast(uint32_t, cvt2(acc[t][8 * h + 2 * q], acc[t][8 * h + 2 * q + 1])));
			out[2 * t + h] = __builtin_bit_cast(f16x8, r);
		}
}

// Write packed accumulator-layout fragments (frags[2t+s] = tile t regs 8s..8s+7) of one sample
// column into the wave's [sample][feature] image: features 32t + 16s + 8k + 4h + (0..3).
template <int NFRAG>
__device__ __forceinline__ void img_store_acc(f16* img, int stride, const f16x8* f, int lane, int feat0 = 0) {
	const int smp = lane & 31, h = lane >> 5;
	f16* row = img + smp * stride + feat0 + 4 * h;
#pragma unroll
	for (int q = 0; q < NFRAG; ++q) {
		// frag q covers tile q>>1, regs 8(q&1)..: features 32(q>>1) + 16(q&1) + 8k + 4h, k = 0,1
		const int base = 32 * (q >> 1) + 16 * (q & 1);
		*(f16x4*)(row + base) = f16x4{f[q][0], f[q][1], f[q][2], f[q][3]};
		*(f16x4*)(row + base + 8) = f16x4{f[q][4], f[q][5], f[q][6], f[q][7]};
	}
}

// Standard-order fragment (lane half h holds features 16s + 8h + 0..7) into the image.
__device__ __forceinline__ void img_store_std(f16* img, int stride, const f16x8& f, int s, int lane) {
	const int smp = lane & 31, h = lane >> 5;
	*(f16x8*)(img + smp * stride + 16 * s + 8 * h) = f;
}

// Operand for v_mfma_f32_16x16x32_f16 with K = the 32 samples: lane gets feature feat0 + (lane&15),
// samples 8(lane>>4) + 0..7, via two ds_read_b64_tr_b16 (4 samples x 16 features per 16-lane group).
__device__ __forceinline__ f16x8 img_frag(const f16* img, int stride, int feat0, int lane) {
	const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
	const f16* a0 = img + (8 * g + q) * stride + feat0 + 4 * p;
	const f16x4 lo = lds_read_tr16(a0);
	const f16x4 hi = lds_read_tr16(a0 + 4 * stride);
	return f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// dW[out x in] += dZ * X^T over the wave's 32 samples, 16x16 tiles (mt over out, nt over in).
template <int MT, int NT>
__device__ __forceinline__ void dw_accum(f32x4* dw, const f16* dz_img, int dz_stride, const f16* x_img, int x_stride, int lane) {
	f16x8 a[MT], b[NT];
#pragma unroll
	for (int m = 0; m < MT; ++m) a[m] = img_frag(dz_img, dz_stride, 16 * m, lane);
#pragma unroll
	for (int n = 0; n < NT; ++n) b[n] = img_frag(x_img, x_stride, 16 * n, lane);
#pragma unroll
	for (int m = 0; m < MT; ++m)
#pragma unroll
		for (int n = 0; n < NT; ++n) dw[m * NT + n] = mfma16(a[m], b[n], dw[m * NT + n]);
}

// Flush one layer's dW tiles (16x16, 4 regs: out = 16m + 4(lane>>4) + r, in = 16n + (lane&15)) into
// the block's fp32 LDS reduction buffer laid out as the parameter slice [out x in]. Waves flush one
// after another (FIRST: store, else add) so the sum order is fixed: bitwise-reproducible gradients.
template <int MT, int NT, bool FIRST>
__device__ __forceinline__ void dw_flush(const f32x4* dw, float* red, uint32_t woff, uint32_t in_dim, int lane,
                                         std::integral_constant<bool, FIRST>) {
	constexpr bool first = FIRST;
#pragma unroll
	for (int m = 0; m < MT; ++m)
#pragma unroll
		for (int n = 0; n < NT; ++n)
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const uint32_t o = 16 * m + 4 * (lane >> 4) + r, i = 16 * n + (lane & 15);
				float* p = red + woff + o * in_dim + i;
				*p = first ? dw[m * NT + n][r] : *p + dw[m * NT + n][r];
			}
}

// Block reduction of the per-wave dW registers into one fp32 slab, in a fixed order. n_reg LDS regions
// of n_matrix floats (4 when they fit): waves w < n_reg store into region w, later waves add into
// region w % n_reg in turn, then all threads sum the regions (0 + 1 + ...) and write the slab with
// 16-B stores. FLUSH(red, first) stores/adds one wave's tiles at their parameter-slice offsets.
template <typename Flush>
__device__ __forceinline__ void dw_block_reduce(float* lds, uint32_t n_matrix, uint32_t n_reg, int wave, float* slab, Flush flush) {
	for (int round = 0; round * (int)n_reg < 4; ++round) {
		__syncthreads();
		if (wave / (int)n_reg == round) {
			float* red = lds + (size_t)(wave % n_reg) * n_matrix;
			if (round == 0) flush(red, std::true_type{});
			else flush(red, std::false_type{});
		}
	}
	__syncthreads();
	for (uint32_t i = 4 * threadIdx.x; i < n_matrix; i += 4 * blockDim.x) {
		f32x4 v = *(const f32x4*)(lds + i);
		for (uint32_t r = 1; r < n_reg; ++r) v += *(const f32x4*)(lds + (size_t)r * n_matrix + i);
		*(f32x4*)(slab + i) = v;
	}
}

// SH degree 4 of the warped direction (tcnn SphericalHarmonics; oracle orc_sh4), features 8h..8h+7.
__device__ __forceinline__ f16x8 sh4_frag(float dx, float dy, float dz, int h) {
	const float x = dx * 2.f - 1.f, y = dy * 2.f - 1.f, z = dz * 2.f - 1.f;
	const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
	float o[8];
	if (h == 0) {
		o[0] = 0.28209479177387814f;
		o[1] = -0.48860251190291987f * y;
		o[2] = 0.48860251190291987f * z;
		o[3] = -0.48860251190291987f * x;
		o[4] = 1.0925484305920792f * xy;
		o[5] = -1.0925484305920792f * yz;
		o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
		o[7] = -1.0925484305920792f * xz;
	} else {
		o[0] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
		o[1] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
		o[2] = 2.8906114426405538f * xy * z;
		o[3] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
		o[4] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
		o[5] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
		o[6] = 1.4453057213202769f * z * (x2 - y2);
		o[7] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
	}
	f16x8 r;
#pragma unroll
	for (int j = 0; j < 8; ++j) r[j] = (f16)o[j];
	return r;
}

// Store rows 0..15 of an accumulator-layout output (regs 0..7) for one sample: lane half h holds
// rows 4h..4h+3 (regs 0..3) and 8+4h..8+4h+3 (regs 4..7).
__device__ __forceinline__ void store_out16(f16* out, uint32_t stride, uint32_t layout, uint32_t n, uint32_t sample, int h,
                                            const f16x8& v) {
	if (layout == MLP_LAYOUT_ROW0) {  // row 0 only (lane half 0, register 0)
		if (h == 0) out[sample] = v[0];
	} else if (layout == 2) {  // NGP_LAYOUT_AOS_RGBD: rows 0..3 only (lane half 0 holds them)
		if (h == 0) *(f16x4*)(out + (size_t)sample * stride) = f16x4{v[0], v[1], v[2], v[3]};
	} else if (layout == 0) {
		f16* row = out + (size_t)sample * stride;
		*(f16x4*)(row + 4 * h) = f16x4{v[0], v[1], v[2], v[3]};
		*(f16x4*)(row + 8 + 4 * h) = f16x4{v[4], v[5], v[6], v[7]};
	} else {
#pragma unroll
		for (int j = 0; j < 8; ++j) out[(size_t)(8 * (j >> 2) + 4 * h + (j & 3)) * stride + sample] = v[j];
	}
}

// dL/d(SH encoding) of one sample, fp16 [16]: the upper half (rows 16..31) of the rgb network's
// dL/dinput tile, lane half h holding SH rows 4h..4h+3 (regs 0..3) and 8+4h..8+4h+3 (regs 4..7)
__device__ __forceinline__ void store_dsh(f16* dsh_out, uint32_t sample, int h, const f16x8& v) {
	f16* row = dsh_out + (size_t)sample * 16 + 4 * h;
	*(f16x4*)(row + 0) = f16x4{v[0], v[1], v[2], v[3]};
	*(f16x4*)(row + 8) = f16x4{v[4], v[5], v[6], v[7]};
}

// The fused-encoding paths' gather of one level's 8 corners (F = 4) given the cell's base corner: the
// integers of corner_index (grid.h; tcnn grid_index), dense and hashed indices both formed and selected so
// the two lane halves (different levels) do not diverge. A dense index is reduced with min(id, id - T),
// which is id % T for id < 2 T (every in-range cell); a lane with a larger one (a position far outside
// [0, 1]) takes the modulo in a branch that is almost never entered. The loads are unconditional (the
// index is in the level's table either way) and an inactive level's values are zeroed afterwards, so
// the 8 loads issue back to back.
__device__ __forceinline__ void fuse_gather_level(const f16* tab, const uint32_t (&base)[3], uint32_t res, uint32_t T, bool hashed,
                                                  bool active, f16x4 (&g)[8]) {
	uint32_t idx[8];
	bool wrap = false;
#pragma unroll
	for (uint32_t k = 0; k < 8; ++k) {
		const uint32_t cx = base[0] + (k & 1u), cy = base[1] + ((k >> 1) & 1u), cz = base[2] + ((k >> 2) & 1u);
		const uint32_t ih = (cx ^ (cy * 2654435761u) ^ (cz * 805459861u)) & (T - 1u);
		const uint32_t id = cx + res * (cy + res * cz);
		const uint32_t im = min(id, id - T);
		wrap |= !hashed && im >= T;
		idx[k] = hashed ? ih : im;
	}
	if (__builtin_expect(wrap, 0)) {
#pragma unroll
		for (uint32_t k = 0; k < 8; ++k) {
			const uint32_t cx = base[0] + (k & 1u), cy = base[1] + ((k >> 1) & 1u), cz = base[2] + ((k >> 2) & 1u);
			idx[k] = (cx + res * (cy + res * cz)) % T;
		}
	}
	f16x4 v[8];
#pragma unroll
	for (uint32_t k = 0; k < 8; ++k) v[k] = *(const f16x4*)(tab + (size_t)idx[k] * 4);
#pragma unroll
	for (uint32_t k = 0; k < 8; ++k) g[k] = active ? v[k] : f16x4{};
}

// ------------------------------------------------------------------------------------------------
// NerfNetwork MLP pair: density (enc -> 64 x DH -> 16) and rgb ([density out | SH] -> 64 x RH -> 16)
// ------------------------------------------------------------------------------------------------
template <int ES, int DH, int RH>
struct NerfLayout {
	// forward fragment offsets
	static constexpr int F_D0 = 0;
	static constexpr int F_DH = F_D0 + 2 * ES;
	static constexpr int F_DO = F_DH + 8 * (DH - 1);
	static constexpr int F_R0 = F_DO + 4;
	static constexpr int F_RH = F_R0 + 4;
	static constexpr int F_RO = F_RH + 8 * (RH - 1);
	static constexpr int N_FWD = F_RO + 4;
	// backward fragment offsets
	static constexpr int B_RO = N_FWD;
	static constexpr int B_RH = B_RO + 2;                 // layers RH-1 .. 1
	static constexpr int B_R0 = B_RH + 8 * (RH - 1);
	static constexpr int B_DO = B_R0 + 4;
	static constexpr int B_DH = B_DO + 2;                 // layers DH-1 .. 1
	static constexpr int B_D0 = B_DH + 8 * (DH - 1);
	static constexpr int ET = (ES + 1) / 2;               // 32-row tiles of the encoding gradient
	static constexpr int N_ALL = B_D0 + 4 * ET;
	// per-wave LDS images (halves); strides padded by 4 halves (8 B) against bank conflicts
	static constexpr int S_XE = 16 * ES + 4;
	static constexpr int S_64 = 64 + 4;
	static constexpr int S_RIN = 32 + 4;
	static constexpr int I_XE = 0;
	static constexpr int I_HD = I_XE + 32 * S_XE;         // DH images
	static constexpr int I_RIN = I_HD + DH * 32 * S_64;
	static constexpr int I_HR = I_RIN + 32 * S_RIN;       // RH images
	static constexpr int I_DZ = I_HR + RH * 32 * S_64;
	static constexpr int IMG_HALVES = I_DZ + 32 * S_64;
	// dW accumulator tiles (16x16)
	static constexpr int W_RO = 0;                        // 1 x 4
	static constexpr int W_RH = W_RO + 4;                 // (RH-1) x 16
	static constexpr int W_R0 = W_RH + 16 * (RH - 1);     // 4 x 2
	static constexpr int W_DO = W_R0 + 8;                 // 1 x 4
	static constexpr int W_DH = W_DO + 4;                 // (DH-1) x 16
	static constexpr int W_D0 = W_DH + 16 * (DH - 1);     // 4 x ES
	static constexpr int N_DW = W_D0 + 4 * ES;
};

template <int ES, int DH, int RH, int MODE>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) k_nerf_mlp(const NerfMlpArgs a) {
	using Lay = NerfLayout<ES, DH, RH>;
	constexpr bool DTRAIN = MODE == MLP_DENSITY_TRAIN;  // density network forward + backward only
	constexpr bool TRAIN = MODE == MLP_TRAIN || DTRAIN;
	constexpr bool DENSITY = MODE == MLP_DENSITY;
	constexpr bool FUSE = MODE == MLP_INFER_ENC;
	static_assert(!FUSE || ES == 1, "fused encoding: one 16-wide encoding step");
	constexpr int NFRAG = TRAIN ? Lay::N_ALL : (DENSITY ? Lay::F_R0 : Lay::N_FWD);
	extern __shared__ __attribute__((aligned(16))) char smem[];
	f16x8* lfrag = (f16x8*)smem;
	const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;

	for (int i = threadIdx.x; i < NFRAG * 64; i += blockDim.x) lfrag[i] = a.frags[i];
	__syncthreads();
	// training: the forward weight fragments stay in registers for every tile the wave processes (the
	// kernel runs one wave per SIMD, so LDS latency is otherwise exposed at each layer)
	constexpr bool WREG = TRAIN && Lay::N_FWD <= 24;  // larger networks would spill
	f16x8 wreg[WREG ? Lay::N_FWD : 1];
	if constexpr (WREG) {
#pragma unroll
		for (int q = 0; q < Lay::N_FWD; ++q) wreg[q] = lfrag[q * 64 + lane];
	}
#define NGP_FWD(T, S, ACC, IN, OFF)                                             \
	do {                                                                        \
		if constexpr (WREG) layer_fwd_reg<T, S>(ACC, IN, wreg, OFF);           \
		else layer_fwd<T, S>(ACC, IN, lfrag + (OFF) * 64, lane);                \
	} while (0)

	f16* img = (f16*)(smem + NFRAG * 1024) + wave * Lay::IMG_HALVES;
	f32x4 dw[TRAIN ? Lay::N_DW : 1];
	if constexpr (TRAIN) {
#pragma unroll
		for (int q = 0; q < Lay::N_DW; ++q) dw[q] = f32x4{0.f, 0.f, 0.f, 0.f};
	}

	const uint32_t n_tiles = (a.n + 31) / 32;
	// One wave per SIMD: the next tile's global inputs (encoding, direction, dL/dout) are loaded while
	// this tile computes, so their latency is not exposed once per tile.
	f16x8 xe_n[ES];
	float cd_n[3] = {0.f, 0.f, 0.f};
	f16x4 dl_n{};
	f16x8 dd_n{};  // DTRAIN: dL/d(density output) rows (j&3) + 8(j>>2) + 4h, the B-operand order of a packed tile
	// FUSE (MLP_INFER_ENC, ES == 1, F == 4): lane half h encodes levels 2h and 2h+1 of its sample (the 8
	// features of its B operand). The next tile's corner gathers are issued with the other prefetches
	// and blended at the top of the next iteration, so the gather latency hides under this tile's MFMAs.
	// The positions are loaded one tile further ahead still, so the gather addresses never wait on a load.
	f16x4 graw[FUSE ? 2 : 1][8];
	float gfrac[FUSE ? 2 : 1][3];
	float px_n[3];
	// this lane's two levels, held in registers: GridConst indexed by a per-lane level would become
	// kernarg loads with a full vmcnt wait inside the gather sequence
	uint32_t lv_off[2], lv_T[2], lv_res[2];
	float lv_scale[2];
	bool lv_hashed[2], lv_active[2];
	if constexpr (FUSE) {
		const float ml = a.max_level * (float)a.gc.n_levels;
#pragma unroll
		for (int j = 0; j < 2; ++j) {
			const uint32_t l0 = j, l1 = 2 + j;  // levels of lane half 0 and 1 (compile-time kernarg reads)
			lv_off[j] = h ? a.gc.offsets[l1] : a.gc.offsets[l0];
			lv_T[j] = h ? a.gc.offsets[l1 + 1] - a.gc.offsets[l1] : a.gc.offsets[l0 + 1] - a.gc.offsets[l0];
			lv_res[j] = h ? a.gc.resolution[l1] : a.gc.resolution[l0];
			lv_scale[j] = h ? a.gc.scale[l1] : a.gc.scale[l0];
			lv_hashed[j] = (a.gc.hashed >> (h ? l1 : l0)) & 1u;
			lv_active[j] = !((float)(h ? l1 : l0) >= ml + 1e-3f);
		}
	}
	auto load_pos = [&](uint32_t tile) {
		const uint32_t smp = tile * 32 + (lane & 31);
		const float* cp = a.coords + (size_t)(smp < a.n ? smp : 0) * a.coord_stride;
		px_n[0] = cp[0]; px_n[1] = cp[1]; px_n[2] = cp[2];
	};
	auto load_inputs = [&](uint32_t tile) {
		const uint32_t smp = tile * 32 + (lane & 31);
		const uint32_t ls = smp < a.n ? smp : 0;
		if constexpr (FUSE) {
			const float x[3] = {px_n[0], px_n[1], px_n[2]};
			load_pos(tile + gridDim.x * 4);
#pragma unroll
			for (int j = 0; j < 2; ++j) {
				// level_setup + corner_index (grid.h) with the level's constants in registers; dense and
				// hashed indices are both formed and selected, so the two lane halves do not diverge
				uint32_t base[3];
#pragma unroll
				for (int d = 0; d < 3; ++d) {
					const float p = __builtin_fmaf(lv_scale[j], x[d], 0.5f);
					const float t = floorf(p);
					base[d] = (uint32_t)(int)t;
					gfrac[j][d] = p - t;
				}
				fuse_gather_level(a.table + (size_t)lv_off[j] * 4, base, lv_res[j], lv_T[j], lv_hashed[j], lv_active[j], graw[j]);
			}
		} else {
#pragma unroll
			for (int s = 0; s < ES; ++s) xe_n[s] = *(const f16x8*)(a.enc + (size_t)ls * a.enc_stride + 16 * s + 8 * h);
		}
		if constexpr (!DENSITY && !DTRAIN) {
			const float* cd = a.coords + (size_t)ls * a.coord_stride + a.dir_offset;
			cd_n[0] = cd[0]; cd_n[1] = cd[1]; cd_n[2] = cd[2];
		}
		if constexpr (DTRAIN) {
			const f16* r = a.dL_ddens + (size_t)ls * a.ddens_stride + 4 * h;
			const f16x4 lo = *(const f16x4*)r, hi = *(const f16x4*)(r + 8);
			dd_n = f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
		} else if constexpr (TRAIN) {
			dl_n = *(const f16x4*)(a.dL_dout + (size_t)ls * a.dL_stride);
		}
	};
	if (blockIdx.x * 4 + wave < n_tiles) {
		if constexpr (FUSE) load_pos(blockIdx.x * 4 + wave);
		load_inputs(blockIdx.x * 4 + wave);
	}
	for (uint32_t tile = blockIdx.x * 4 + wave; tile < n_tiles; tile += gridDim.x * 4) {
		const uint32_t sample = tile * 32 + (lane & 31);
		const bool valid = sample < a.n;
		f16x8 xe[ES];
		if constexpr (FUSE) {
			// trilinear blend in k_grid_forward_rows' order (fp32 FMAs, one RNE rounding per feature)
			f16x8 r;
#pragma unroll
			for (int j = 0; j < 2; ++j) {
				float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
				for (uint32_t k = 0; k < 8; ++k) {
					const float w = corner_weight<3>(gfrac[j], k);
#pragma unroll
					for (int f = 0; f < 4; ++f) acc[f] = __builtin_fmaf(w, (float)graw[j][k][f], acc[f]);
				}
#pragma unroll
				for (int f = 0; f < 4; ++f) {
					asm volatile("" : "+v"(acc[f]));
					r[4 * j + f] = (f16)acc[f];
				}
			}
			xe[0] = valid ? r : f16x8{};
		} else {
#pragma unroll
			for (int s = 0; s < ES; ++s) xe[s] = valid ? xe_n[s] : f16x8{};
		}
		const float cdx = cd_n[0], cdy = cd_n[1], cdz = cd_n[2];
		const f16x4 dl_cur = dl_n;
		const f16x8 dd_cur = dd_n;
		load_inputs(tile + gridDim.x * 4);  // unconditional (past-the-end tiles read sample 0): no phi copies

		// ---- density forward -------------------------------------------------------------------
		if constexpr (TRAIN) {
#pragma unroll
			for (int s = 0; s < ES; ++s) img_store_std(img + Lay::I_XE, Lay::S_XE, xe[s], s, lane);
		}
		f32x16 acc[2];
		f16x8 hd[DH][4];
		NGP_FWD(2, ES, acc, xe, Lay::F_D0);
		pack_tiles<2>(acc, hd[0], true);
#pragma unroll
		for (int l = 1; l < DH; ++l) {
			NGP_FWD(2, 4, acc, hd[l - 1], Lay::F_DH + 8 * (l - 1));
			pack_tiles<2>(acc, hd[l], true);
		}
		f32x16 dacc[1];
		NGP_FWD(1, 4, dacc, hd[DH - 1], Lay::F_DO);
		f16x8 dout[2];
		pack_tile(dacc[0], dout[0], dout[1], false);  // dout[0] = rows 0..15 (density network output)
		if constexpr (DENSITY) {
			if (valid) store_out16(a.out, a.out_stride, a.out_layout, a.n, sample, h, dout[0]);
			continue;
		}
		// density network backward from dL/d(density output) `dd` (the NeRF training pass after
		// add_density_gradient, or density_backward's own dL/doutput): dW of the density layers, dL/d(encoding)
		auto density_backward = [&](f16x8 (&dd)[1], f16* dz_img) {
			f16x8 dz[4];
			img_store_acc<1>(dz_img, Lay::S_64, dd, lane);
			dw_accum<1, 4>(dw + Lay::W_DO, dz_img, Lay::S_64, img + Lay::I_HD + (DH - 1) * 32 * Lay::S_64, Lay::S_64, lane);
			layer_fwd<2, 1>(acc, dd, lfrag + Lay::B_DO * 64, lane);
			mask_pack<2>(acc, hd[DH - 1], dz);
#pragma unroll
			for (int l = DH - 1; l >= 1; --l) {
				img_store_acc<4>(dz_img, Lay::S_64, dz, lane);
				dw_accum<4, 4>(dw + Lay::W_DH + 16 * (DH - 1 - l), dz_img, Lay::S_64, img + Lay::I_HD + (l - 1) * 32 * Lay::S_64,
				               Lay::S_64, lane);
				layer_fwd<2, 4>(acc, dz, lfrag + (Lay::B_DH + 8 * (DH - 1 - l)) * 64, lane);
				mask_pack<2>(acc, hd[l - 1], dz);
			}
			img_store_acc<4>(dz_img, Lay::S_64, dz, lane);
			dw_accum<4, ES>(dw + Lay::W_D0, dz_img, Lay::S_64, img + Lay::I_XE, Lay::S_XE, lane);
			if (a.dL_denc) {
				// the MFMAs run with the full wave (every lane supplies A rows); only the stores are masked
				f32x16 ae[Lay::ET];
				layer_fwd<Lay::ET, 4>(ae, dz, lfrag + Lay::B_D0 * 64, lane);
#pragma unroll
				for (int t = 0; t < Lay::ET; ++t) {
					f16x8 lo, hi;
					pack_tile(ae[t], lo, hi, false);
					if (!valid) continue;
					// rows 32t + 8k + 4h + (0..3): lo holds k = 0,1; hi holds k = 2,3
					f16* row = a.dL_denc + (size_t)sample * a.denc_stride + 32 * t + 4 * h;
					*(f16x4*)(row + 0) = f16x4{lo[0], lo[1], lo[2], lo[3]};
					*(f16x4*)(row + 8) = f16x4{lo[4], lo[5], lo[6], lo[7]};
					if (32 * t + 16 < 16 * ES) {
						*(f16x4*)(row + 16) = f16x4{hi[0], hi[1], hi[2], hi[3]};
						*(f16x4*)(row + 24) = f16x4{hi[4], hi[5], hi[6], hi[7]};
					}
				}
			}
		};
		if constexpr (DTRAIN) {
			// NerfNetwork::density_forward / density_backward (nerf_network.h:355-428)
			if (a.out && valid) store_out16(a.out, a.out_stride, a.out_layout, a.n, sample, h, dout[0]);
#pragma unroll
			for (int l = 0; l < DH; ++l) img_store_acc<4>(img + Lay::I_HD + l * 32 * Lay::S_64, Lay::S_64, hd[l], lane);
			f16x8 dd[1] = {valid ? dd_cur : f16x8{}};
			density_backward(dd, img + Lay::I_DZ);
			continue;
		}

		// ---- rgb forward -----------------------------------------------------------------------
		f16x8 rin[2] = {dout[0], sh4_frag(cdx, cdy, cdz, h)};
		if (!valid) rin[1] = f16x8{};
		f16x8 hr[RH][4];
		NGP_FWD(2, 2, acc, rin, Lay::F_R0);
		pack_tiles<2>(acc, hr[0], true);
#pragma unroll
		for (int l = 1; l < RH; ++l) {
			NGP_FWD(2, 4, acc, hr[l - 1], Lay::F_RH + 8 * (l - 1));
			pack_tiles<2>(acc, hr[l], true);
		}
		f32x16 racc[1];
		NGP_FWD(1, 4, racc, hr[RH - 1], Lay::F_RO);
		if (a.out && valid) {
			f16x8 ro, ro_hi;
			pack_tile(racc[0], ro, ro_hi, false);
			if (h == 0) ro[3] = dout[0][0];  // extract_density: row 3 <- density row 0 (nerf_network.h:32-43)
			store_out16(a.out, a.out_stride, a.out_layout, a.n, sample, h, ro);
		}
		if constexpr (!TRAIN) continue;
		else {
			// ---- images of the forward activations (dW operands) ------------------------------
#pragma unroll
			for (int l = 0; l < DH; ++l) img_store_acc<4>(img + Lay::I_HD + l * 32 * Lay::S_64, Lay::S_64, hd[l], lane);
			{
				f16x8 d1[1] = {dout[0]};
				img_store_acc<1>(img + Lay::I_RIN, Lay::S_RIN, d1, lane);
				img_store_std(img + Lay::I_RIN, Lay::S_RIN, rin[1], 1, lane);
			}
#pragma unroll
			for (int l = 0; l < RH; ++l) img_store_acc<4>(img + Lay::I_HR + l * 32 * Lay::S_64, Lay::S_64, hr[l], lane);

			// ---- rgb backward ---------------------------------------------------------------
			f16* dz_img = img + Lay::I_DZ;
			float dsig = 0.f;
			f16x8 dz1[1];
			{
				f16x4 d = valid ? dl_cur : f16x4{};
				dsig = (float)d[3];
				// extract_rgb (nerf_network.h:46-60): rows 0..2 of dL/drgb, the rest zero
				dz1[0] = h == 0 ? f16x8{d[0], d[1], d[2], (f16)0.f, 0, 0, 0, 0} : f16x8{};
			}
			img_store_acc<1>(dz_img, Lay::S_64, dz1, lane);
			dw_accum<1, 4>(dw + Lay::W_RO, dz_img, Lay::S_64, img + Lay::I_HR + (RH - 1) * 32 * Lay::S_64, Lay::S_64, lane);
			f16x8 dz[4];
			layer_fwd<2, 1>(acc, dz1, lfrag + Lay::B_RO * 64, lane);
			mask_pack<2>(acc, hr[RH - 1], dz);
#pragma unroll
			for (int l = RH - 1; l >= 1; --l) {
				img_store_acc<4>(dz_img, Lay::S_64, dz, lane);
				dw_accum<4, 4>(dw + Lay::W_RH + 16 * (RH - 1 - l), dz_img, Lay::S_64, img + Lay::I_HR + (l - 1) * 32 * Lay::S_64,
				               Lay::S_64, lane);
				layer_fwd<2, 4>(acc, dz, lfrag + (Lay::B_RH + 8 * (RH - 1 - l)) * 64, lane);
				mask_pack<2>(acc, hr[l - 1], dz);
			}
			img_store_acc<4>(dz_img, Lay::S_64, dz, lane);
			dw_accum<4, 2>(dw + Lay::W_R0, dz_img, Lay::S_64, img + Lay::I_RIN, Lay::S_RIN, lane);
			f32x16 a1[1];
			layer_fwd<1, 4>(a1, dz, lfrag + Lay::B_R0 * 64, lane);
			// dL/d(rgb input): rows 0..15 = dL/d(density output), rows 16..31 = dL/d(SH encoding);
			// add_density_gradient (nerf_network.h:63-74) in fp16
			f16x8 dd[1], dsh;
			pack_tile(a1[0], dd[0], dsh, false);
			if (h == 0) dd[0][0] = (f16)((float)dd[0][0] + dsig);
			if (a.dL_dsh && valid) store_dsh(a.dL_dsh, sample, h, dsh);

			// ---- density backward ------------------------------------------------------------
			density_backward(dd, dz_img);
		}
	}

	if constexpr (TRAIN) {
		// block reduction of dW (parameter-slice layout) into one slab per block
		const uint32_t dw0 = a.density_woff, rw0 = a.rgb_woff;
		const uint32_t d_out_off = dw0 + 64 * 16 * ES + 64 * 64 * (DH - 1);
		const uint32_t r_out_off = rw0 + 64 * 32 + 64 * 64 * (RH - 1);
		dw_block_reduce((float*)smem, a.n_matrix, a.n_reg, wave, a.dw_slab + (size_t)blockIdx.x * a.n_matrix,
		                [&](float* red, auto first) {
			dw_flush<1, 4>(dw + Lay::W_RO, red, r_out_off, 64, lane, first);
#pragma unroll
			for (int l = RH - 1; l >= 1; --l)
				dw_flush<4, 4>(dw + Lay::W_RH + 16 * (RH - 1 - l), red, rw0 + 64 * 32 + 64 * 64 * (l - 1), 64, lane, first);
			dw_flush<4, 2>(dw + Lay::W_R0, red, rw0, 32, lane, first);
			dw_flush<1, 4>(dw + Lay::W_DO, red, d_out_off, 64, lane, first);
#pragma unroll
			for (int l = DH - 1; l >= 1; --l)
				dw_flush<4, 4>(dw + Lay::W_DH + 16 * (DH - 1 - l), red, dw0 + 64 * 16 * ES + 64 * 64 * (l - 1), 64, lane, first);
			dw_flush<4, ES>(dw + Lay::W_D0, red, dw0, 16 * ES, lane, first);
		});
	}
}

// ------------------------------------------------------------------------------------------------
// NerfNetwork training pass, weight gradients split across the block's four waves
// ------------------------------------------------------------------------------------------------
// k_nerf_mlp<TRAIN> keeps every layer's dW in each wave's registers (36 16x16 fp32 tiles at C2 =
// 144 registers), which leaves no room for the weight fragments: the backward reads them from LDS
// with a wait per layer, one wave per SIMD. Here a block of 4 waves processes 4 tiles of 32 samples
// per iteration in two phases:
//   A  each wave runs its tile's forward and backward dX chains with ALL weight fragments in
//      registers (no LDS reads), and writes the activations and every layer's output gradient dZ
//      to its LDS image [sample][feature];
//   B  after a barrier, wave w accumulates its quarter of dW over the 4 images (K = 128 samples):
//      row block m = w of the 64-row layers, column block n = w of the 16-row output layers
//      (9 tiles = 36 registers at C2), then a second barrier frees the images.
// Each wave ends up with disjoint dW tiles and stores them straight into the block's slab (no
// cross-wave reduction). Sum order is fixed (block iterations, then waves 0..3): bitwise
// reproducible like the one-wave-per-tile kernel.
template <int ES, int DH, int RH>
struct NerfTrainLayout {
	using L = NerfLayout<ES, DH, RH>;
	static constexpr int N_BWD = L::N_ALL - L::N_FWD;
	static constexpr int S_16 = 16 + 4;
	// per-wave images (halves)
	static constexpr int I_XE = 0;                                  // [32][16 ES]
	static constexpr int I_HD = I_XE + 32 * L::S_XE;                // DH x [32][64]
	static constexpr int I_RIN = I_HD + DH * 32 * L::S_64;          // [32][32] density out | SH
	static constexpr int I_HR = I_RIN + 32 * L::S_RIN;              // RH x [32][64]
	static constexpr int I_ZRO = I_HR + RH * 32 * L::S_64;          // dZ rgb output [32][16]
	static constexpr int I_ZRH = I_ZRO + 32 * S_16;                 // (RH-1) x [32][64], j-th = layer RH-1-j
	static constexpr int I_ZR0 = I_ZRH + (RH - 1) * 32 * L::S_64;   // dZ rgb layer 0
	static constexpr int I_ZDO = I_ZR0 + 32 * L::S_64;              // dZ density output [32][16]
	static constexpr int I_ZDH = I_ZDO + 32 * S_16;                 // (DH-1) x [32][64]
	static constexpr int I_ZD0 = I_ZDH + (DH - 1) * 32 * L::S_64;   // dZ density layer 0
	static constexpr int IMG_HALVES = I_ZD0 + 32 * L::S_64;
	static constexpr size_t LDS_BYTES = 4 * (size_t)IMG_HALVES * sizeof(f16);
	// this wave's dW tiles
	static constexpr int W_RO = 0;                    // rgb output:  m 0,    n = wave
	static constexpr int W_RH = 1;                    // rgb hidden:  m = wave, n 0..3 (RH-1 layers)
	static constexpr int W_R0 = W_RH + 4 * (RH - 1);  // rgb layer 0: m = wave, n 0..1
	static constexpr int W_DO = W_R0 + 2;             // density out: m 0,    n = wave
	static constexpr int W_DH = W_DO + 1;             // density hidden: m = wave, n 0..3
	static constexpr int W_D0 = W_DH + 4 * (DH - 1);  // density layer 0: m = wave, n 0..ES-1
	static constexpr int N_DW = W_D0 + ES;
};

// dW[m0+m][n0+n] += dZ^T X over one image's 32 samples (16x16x32 MFMAs, K = samples)
template <int MC, int NC>
__device__ __forceinline__ void dw_part(f32x4* dw, const f16* dz_img, int dz_stride, int m0, const f16* x_img, int x_stride, int n0,
                                        int lane) {
	f16x8 a[MC], b[NC];
#pragma unroll
	for (int m = 0; m < MC; ++m) a[m] = img_frag(dz_img, dz_stride, 16 * (m0 + m), lane);
#pragma unroll
	for (int n = 0; n < NC; ++n) b[n] = img_frag(x_img, x_stride, 16 * (n0 + n), lane);
#pragma unroll
	for (int m = 0; m < MC; ++m)
#pragma unroll
		for (int n = 0; n < NC; ++n) dw[m * NC + n] = mfma16(a[m], b[n], dw[m * NC + n]);
}

// Store dW tiles (16x16, 4 regs: out = 16m + 4(lane>>4) + r, in = 16n + (lane&15)) into the slab at
// their parameter-slice positions [out x in].
template <int MC, int NC>
__device__ __forceinline__ void dw_store(const f32x4* dw, float* slab, uint32_t woff, uint32_t in_dim, int m0, int n0, int lane) {
#pragma unroll
	for (int m = 0; m < MC; ++m)
#pragma unroll
		for (int n = 0; n < NC; ++n)
#pragma unroll
			for (int r = 0; r < 4; ++r) {
				const uint32_t o = 16 * (m0 + m) + 4 * (lane >> 4) + r, i = 16 * (n0 + n) + (lane & 15);
				slab[woff + o * in_dim + i] = dw[m * NC + n][r];
			}
}

// One image's phase-B operands (16x16x32 A/B fragments) for this wave's dW tiles (NerfTrainLayout W_*)
template <int ES, int DH, int RH>
struct PhaseBOps {
	f16x8 ro_a, ro_b;
	f16x8 rh_a[RH > 1 ? RH - 1 : 1], rh_b[RH > 1 ? RH - 1 : 1][4];
	f16x8 r0_a, r0_b[2];
	f16x8 do_a, do_b;
	f16x8 dh_a[DH > 1 ? DH - 1 : 1], dh_b[DH > 1 ? DH - 1 : 1][4];
	f16x8 d0_a, d0_b[ES];
};

// Phase B: this wave's quarter of dW over the block's four images (NerfTrainLayout W_*), between the
// two barriers of an iteration.
// DB: the next image's operands are requested before this image's MFMAs (two operand sets live)
template <int ES, int DH, int RH, bool DB = true>
__device__ __forceinline__ void train_phase_b(f32x4* dw, const f16* img_all, int wave, int lane) {
	using Lay = NerfLayout<ES, DH, RH>;
	using T = NerfTrainLayout<ES, DH, RH>;
	// The operands of image w + 1 (28 ds_read_b64_tr_b16) are requested before image w's 9 MFMA tiles,
	// which lets the scheduler keep more reads in flight (30.9 -> 30.5 us at C2; pinning that order
	// with sched_barrier measured 31.4 us: at most 15 LDS reads can be outstanding per wave). Same
	// products in the same order as dw_part: the gradients are unchanged bit for bit.
	PhaseBOps<ES, DH, RH> ops[DB ? 2 : 1];
	auto load_ops = [&](int w, PhaseBOps<ES, DH, RH>& o) {
		const f16* im = img_all + w * T::IMG_HALVES;
		o.ro_a = img_frag(im + T::I_ZRO, T::S_16, 0, lane);
		o.ro_b = img_frag(im + T::I_HR + (RH - 1) * 32 * Lay::S_64, Lay::S_64, 16 * wave, lane);
#pragma unroll
		for (int j = 0; j < RH - 1; ++j) {
			o.rh_a[j] = img_frag(im + T::I_ZRH + j * 32 * Lay::S_64, Lay::S_64, 16 * wave, lane);
#pragma unroll
			for (int n = 0; n < 4; ++n) o.rh_b[j][n] = img_frag(im + T::I_HR + (RH - 2 - j) * 32 * Lay::S_64, Lay::S_64, 16 * n, lane);
		}
		o.r0_a = img_frag(im + T::I_ZR0, Lay::S_64, 16 * wave, lane);
#pragma unroll
		for (int n = 0; n < 2; ++n) o.r0_b[n] = img_frag(im + T::I_RIN, Lay::S_RIN, 16 * n, lane);
		o.do_a = img_frag(im + T::I_ZDO, T::S_16, 0, lane);
		o.do_b = img_frag(im + T::I_HD + (DH - 1) * 32 * Lay::S_64, Lay::S_64, 16 * wave, lane);
#pragma unroll
		for (int j = 0; j < DH - 1; ++j) {
			o.dh_a[j] = img_frag(im + T::I_ZDH + j * 32 * Lay::S_64, Lay::S_64, 16 * wave, lane);
#pragma unroll
			for (int n = 0; n < 4; ++n) o.dh_b[j][n] = img_frag(im + T::I_HD + (DH - 2 - j) * 32 * Lay::S_64, Lay::S_64, 16 * n, lane);
		}
		o.d0_a = img_frag(im + T::I_ZD0, Lay::S_64, 16 * wave, lane);
#pragma unroll
		for (int n = 0; n < ES; ++n) o.d0_b[n] = img_frag(im + T::I_XE, Lay::S_XE, 16 * n, lane);
	};
	if (DB) load_ops(0, ops[0]);
#pragma unroll
	for (int w = 0; w < 4; ++w) {
		if (!DB) load_ops(w, ops[0]);
		else if (w < 3) load_ops(w + 1, ops[(w + 1) & (DB ? 1 : 0)]);
		const PhaseBOps<ES, DH, RH>& o = ops[w & (DB ? 1 : 0)];
		dw[T::W_RO] = mfma16(o.ro_a, o.ro_b, dw[T::W_RO]);
#pragma unroll
		for (int j = 0; j < RH - 1; ++j)
#pragma unroll
			for (int n = 0; n < 4; ++n) dw[T::W_RH + 4 * j + n] = mfma16(o.rh_a[j], o.rh_b[j][n], dw[T::W_RH + 4 * j + n]);
#pragma unroll
		for (int n = 0; n < 2; ++n) dw[T::W_R0 + n] = mfma16(o.r0_a, o.r0_b[n], dw[T::W_R0 + n]);
		dw[T::W_DO] = mfma16(o.do_a, o.do_b, dw[T::W_DO]);
#pragma unroll
		for (int j = 0; j < DH - 1; ++j)
#pragma unroll
			for (int n = 0; n < 4; ++n) dw[T::W_DH + 4 * j + n] = mfma16(o.dh_a[j], o.dh_b[j][n], dw[T::W_DH + 4 * j + n]);
#pragma unroll
		for (int n = 0; n < ES; ++n) dw[T::W_D0 + n] = mfma16(o.d0_a, o.d0_b[n], dw[T::W_D0 + n]);
	}
}

// this wave's dW tiles -> the block's slab (parameter-slice layout; the waves' tiles are disjoint)
template <int ES, int DH, int RH>
__device__ __forceinline__ void train_store_dw(const f32x4* dw, const NerfMlpArgs& a, int wave, int lane) {
	using T = NerfTrainLayout<ES, DH, RH>;
	float* slab = a.dw_slab + (size_t)blockIdx.x * a.n_matrix;
	const uint32_t dw0 = a.density_woff, rw0 = a.rgb_woff;
	dw_store<1, 1>(dw + T::W_RO, slab, rw0 + 64 * 32 + 64 * 64 * (RH - 1), 64, 0, wave, lane);
#pragma unroll
	for (int j = 0; j < RH - 1; ++j) dw_store<1, 4>(dw + T::W_RH + 4 * j, slab, rw0 + 64 * 32 + 64 * 64 * (RH - 2 - j), 64, wave, 0, lane);
	dw_store<1, 2>(dw + T::W_R0, slab, rw0, 32, wave, 0, lane);
	dw_store<1, 1>(dw + T::W_DO, slab, dw0 + 64 * 16 * ES + 64 * 64 * (DH - 1), 64, 0, wave, lane);
#pragma unroll
	for (int j = 0; j < DH - 1; ++j) dw_store<1, 4>(dw + T::W_DH + 4 * j, slab, dw0 + 64 * 16 * ES + 64 * 64 * (DH - 2 - j), 64, wave, 0, lane);
	dw_store<1, ES>(dw + T::W_D0, slab, dw0, 16 * ES, wave, 0, lane);
}

// Timing experiments only (-DNGP_TRAIN_CLOCK, DESIGN §6 phase costs; tools/train_clock.py): thread 0 of blocks
// 0..1023 (wave 0) stamps the 100-MHz wall clock at the phase boundaries: slot 0 entry, 1 weights loaded, then per
// iteration i slots 2 + 10 i + k for k = 0 inputs taken, 1 density forward, 2 rgb forward (+ output store),
// 3 images written, 4 rgb backward chain, 5 density backward chain, 6 dL/denc stored, 7 barrier, 8 dW, 9 barrier;
// slot 127 exit. Scheduling barriers keep the phases apart, so the stamped kernel is slower than the plain one.
#ifdef NGP_TRAIN_CLOCK
constexpr int TRC_SLOTS = 128;
__device__ uint64_t g_train_clock[1024 * TRC_SLOTS];
#define TRC_MARK(i)                                                                                               \
	do {                                                                                                          \
		__builtin_amdgcn_sched_barrier(0);                                                                        \
		if (threadIdx.x == 0 && blockIdx.x < 1024 && (i) < TRC_SLOTS) g_train_clock[blockIdx.x * TRC_SLOTS + (i)] = wall_clock64(); \
		__builtin_amdgcn_sched_barrier(0);                                                                        \
	} while (0)
#define TRC_IT(k) TRC_MARK(2 + 10 * (int)trc_it + (k))
#else
#define TRC_MARK(i) do {} while (0)
#define TRC_IT(k) do {} while (0)
#endif

template <int ES, int DH, int RH>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) k_nerf_mlp_train(const NerfMlpArgs a) {
	TRC_MARK(0);
	using Lay = NerfLayout<ES, DH, RH>;
	using T = NerfTrainLayout<ES, DH, RH>;
	extern __shared__ __attribute__((aligned(16))) char smem[];
	const int lane = threadIdx.x & 63, h = lane >> 5;
	const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	f16* img_all = (f16*)smem;
	f16* img = img_all + wave * T::IMG_HALVES;

	// every weight fragment in registers for the whole kernel (loaded once from global)
	f16x8 wreg[Lay::N_FWD], breg[T::N_BWD];
#pragma unroll
	for (int q = 0; q < Lay::N_FWD; ++q) wreg[q] = a.frags[q * 64 + lane];
#pragma unroll
	for (int q = 0; q < T::N_BWD; ++q) breg[q] = a.frags[(Lay::N_FWD + q) * 64 + lane];
	// The fragments live in the accumulator file (AGPRs can be an MFMA's A operand): left to itself the
	// register allocator parks them there anyway under VGPR pressure and copies them back with one
	// v_accvgpr_read per register before each use (~100 VALU per tile); pinned, the MFMAs read them in place.
#pragma unroll
	for (int q = 0; q < Lay::N_FWD; ++q) asm volatile("" : "+a"(wreg[q]));
#pragma unroll
	for (int q = 0; q < T::N_BWD; ++q) asm volatile("" : "+a"(breg[q]));
	f32x4 dw[T::N_DW];
#pragma unroll
	for (int q = 0; q < T::N_DW; ++q) dw[q] = f32x4{0.f, 0.f, 0.f, 0.f};
	TRC_MARK(1);

	const uint32_t n_tiles = (a.n + 31) / 32;
	f16x8 xe_n[ES];
	float cd_n[3];
	f16x4 dl_n;
	auto load_inputs = [&](uint32_t tile) {
		const uint32_t smp = tile * 32 + (lane & 31);
		const uint32_t ls = smp < a.n ? smp : 0;
#pragma unroll
		for (int s = 0; s < ES; ++s) xe_n[s] = *(const f16x8*)(a.enc + (size_t)ls * a.enc_stride + 16 * s + 8 * h);
		const float* cd = a.coords + (size_t)ls * a.coord_stride + a.dir_offset;
		cd_n[0] = cd[0]; cd_n[1] = cd[1]; cd_n[2] = cd[2];
		dl_n = *(const f16x4*)(a.dL_dout + (size_t)ls * a.dL_stride);
	};
	load_inputs(blockIdx.x * 4 + wave);
	// every wave runs the same number of iterations (the barriers need all four); tiles past the end
	// run on zero inputs and zero output gradients, so their dW contribution is exactly zero
#ifdef NGP_TRAIN_CLOCK
	uint32_t trc_it = 0;
#endif
	for (uint32_t base = blockIdx.x * 4; base < n_tiles; base += gridDim.x * 4) {
		const uint32_t tile = base + wave;
		const uint32_t sample = tile * 32 + (lane & 31);
		const bool valid = sample < a.n;
		f16x8 xe[ES];
#pragma unroll
		for (int s = 0; s < ES; ++s) xe[s] = valid ? xe_n[s] : f16x8{};
		const float cdx = cd_n[0], cdy = cd_n[1], cdz = cd_n[2];
		const f16x4 dl_cur = dl_n;
		load_inputs(tile + gridDim.x * 4);  // unconditional (past-the-end tiles read sample 0)
		TRC_IT(0);

		// ---- phase A: forward ----------------------------------------------------------------
#pragma unroll
		for (int s = 0; s < ES; ++s) img_store_std(img + T::I_XE, Lay::S_XE, xe[s], s, lane);
		f32x16 acc[2];
		f16x8 hd[DH][4];
		layer_fwd_reg<2, ES>(acc, xe, wreg, Lay::F_D0);
		pack_tiles<2>(acc, hd[0], true);
#pragma unroll
		for (int l = 1; l < DH; ++l) {
			layer_fwd_reg<2, 4>(acc, hd[l - 1], wreg, Lay::F_DH + 8 * (l - 1));
			pack_tiles<2>(acc, hd[l], true);
		}
		f32x16 dacc[1];
		layer_fwd_reg<1, 4>(dacc, hd[DH - 1], wreg, Lay::F_DO);
		f16x8 dout[2];
		pack_tile(dacc[0], dout[0], dout[1], false);
		TRC_IT(1);
		f16x8 rin[2] = {dout[0], sh4_frag(cdx, cdy, cdz, h)};
		if (!valid) rin[1] = f16x8{};
		f16x8 hr[RH][4];
		layer_fwd_reg<2, 2>(acc, rin, wreg, Lay::F_R0);
		pack_tiles<2>(acc, hr[0], true);
#pragma unroll
		for (int l = 1; l < RH; ++l) {
			layer_fwd_reg<2, 4>(acc, hr[l - 1], wreg, Lay::F_RH + 8 * (l - 1));
			pack_tiles<2>(acc, hr[l], true);
		}
		f32x16 racc[1];
		layer_fwd_reg<1, 4>(racc, hr[RH - 1], wreg, Lay::F_RO);
		if (a.out && valid) {
			f16x8 ro, ro_hi;
			pack_tile(racc[0], ro, ro_hi, false);
			if (h == 0) ro[3] = dout[0][0];  // extract_density (nerf_network.h:32-43)
			store_out16(a.out, a.out_stride, a.out_layout, a.n, sample, h, ro);
		}
		TRC_IT(2);
#pragma unroll
		for (int l = 0; l < DH; ++l) img_store_acc<4>(img + T::I_HD + l * 32 * Lay::S_64, Lay::S_64, hd[l], lane);
		{
			f16x8 d1[1] = {dout[0]};
			img_store_acc<1>(img + T::I_RIN, Lay::S_RIN, d1, lane);
			img_store_std(img + T::I_RIN, Lay::S_RIN, rin[1], 1, lane);
		}
#pragma unroll
		for (int l = 0; l < RH; ++l) img_store_acc<4>(img + T::I_HR + l * 32 * Lay::S_64, Lay::S_64, hr[l], lane);
		TRC_IT(3);

		// ---- phase A: backward dX chain, every dZ kept in LDS ---------------------------------
		float dsig;
		f16x8 dz1[1];
		{
			const f16x4 d = valid ? dl_cur : f16x4{};
			dsig = (float)d[3];
			dz1[0] = h == 0 ? f16x8{d[0], d[1], d[2], (f16)0.f, 0, 0, 0, 0} : f16x8{};  // extract_rgb (:46-60)
		}
		img_store_acc<1>(img + T::I_ZRO, T::S_16, dz1, lane);
		f16x8 dz[4];
		layer_fwd_reg<2, 1>(acc, dz1, breg, Lay::B_RO - Lay::N_FWD);
		mask_pack<2>(acc, hr[RH - 1], dz);
#pragma unroll
		for (int l = RH - 1; l >= 1; --l) {
			img_store_acc<4>(img + T::I_ZRH + (RH - 1 - l) * 32 * Lay::S_64, Lay::S_64, dz, lane);
			layer_fwd_reg<2, 4>(acc, dz, breg, Lay::B_RH - Lay::N_FWD + 8 * (RH - 1 - l));
			mask_pack<2>(acc, hr[l - 1], dz);
		}
		img_store_acc<4>(img + T::I_ZR0, Lay::S_64, dz, lane);
		f32x16 a1[1];
		layer_fwd_reg<1, 4>(a1, dz, breg, Lay::B_R0 - Lay::N_FWD);
		f16x8 dd[1], dsh;
		pack_tile(a1[0], dd[0], dsh, false);  // dsh: rows 16..31 of dL/d(rgb input) = dL/d(SH encoding)
		if (h == 0) dd[0][0] = (f16)((float)dd[0][0] + dsig);  // add_density_gradient (:63-74)
		if (a.dL_dsh && valid) store_dsh(a.dL_dsh, sample, h, dsh);
		TRC_IT(4);
		img_store_acc<1>(img + T::I_ZDO, T::S_16, dd, lane);
		layer_fwd_reg<2, 1>(acc, dd, breg, Lay::B_DO - Lay::N_FWD);
		mask_pack<2>(acc, hd[DH - 1], dz);
#pragma unroll
		for (int l = DH - 1; l >= 1; --l) {
			img_store_acc<4>(img + T::I_ZDH + (DH - 1 - l) * 32 * Lay::S_64, Lay::S_64, dz, lane);
			layer_fwd_reg<2, 4>(acc, dz, breg, Lay::B_DH - Lay::N_FWD + 8 * (DH - 1 - l));
			mask_pack<2>(acc, hd[l - 1], dz);
		}
		img_store_acc<4>(img + T::I_ZD0, Lay::S_64, dz, lane);
		TRC_IT(5);
		if (a.dL_denc) {
			f32x16 ae[Lay::ET];
			layer_fwd_reg<Lay::ET, 4>(ae, dz, breg, Lay::B_D0 - Lay::N_FWD);
#pragma unroll
			for (int t = 0; t < Lay::ET; ++t) {
				f16x8 lo, hi;
				pack_tile(ae[t], lo, hi, false);
				if (!valid) continue;
				f16* row = a.dL_denc + (size_t)sample * a.denc_stride + 32 * t + 4 * h;
				*(f16x4*)(row + 0) = f16x4{lo[0], lo[1], lo[2], lo[3]};
				*(f16x4*)(row + 8) = f16x4{lo[4], lo[5], lo[6], lo[7]};
				if (32 * t + 16 < 16 * ES) {
					*(f16x4*)(row + 16) = f16x4{hi[0], hi[1], hi[2], hi[3]};
					*(f16x4*)(row + 24) = f16x4{hi[4], hi[5], hi[6], hi[7]};
				}
			}
		}
		TRC_IT(6);
		__syncthreads();
		TRC_IT(7);

		// ---- phase B: this wave's quarter of dW over the four images ---------------------------
		train_phase_b<ES, DH, RH>(dw, img_all, wave, lane);
		TRC_IT(8);
		__syncthreads();
		TRC_IT(9);
#ifdef NGP_TRAIN_CLOCK
		++trc_it;
#endif
	}
	train_store_dw<ES, DH, RH>(dw, a, wave, lane);
	TRC_MARK(127);
}

template <int ES, int DH, int RH, int MODE>
static void launch_nerf(const NerfMlpArgs& a, hipStream_t s) {
	using Lay = NerfLayout<ES, DH, RH>;
	constexpr bool TRAIN = MODE == MLP_TRAIN || MODE == MLP_DENSITY_TRAIN;
	constexpr int NFRAG = TRAIN ? Lay::N_ALL : (MODE == MLP_DENSITY ? Lay::F_R0 : Lay::N_FWD);
	size_t lds = (size_t)NFRAG * 1024 + (TRAIN ? 4 * Lay::IMG_HALVES * sizeof(f16) : 0);
	uint32_t n_reg = 4;
	while (n_reg > 1 && (size_t)n_reg * a.n_matrix * sizeof(float) > 160 * 1024) n_reg /= 2;
	if (TRAIN) lds = std::max(lds, (size_t)n_reg * a.n_matrix * sizeof(float));
	NGP_CHECK(lds <= 160 * 1024, "NerfNetwork MLP: LDS budget exceeded");
	const uint32_t tiles = (a.n + 31) / 32;
	uint32_t blocks = TRAIN ? nerf_mlp_train_blocks(a.n) : std::min<uint32_t>(div_round_up(tiles, 4), 8 * device_cu_count());
	if (blocks == 0) return;
	if constexpr (TRAIN && MODE != MLP_DENSITY_TRAIN && NerfTrainLayout<ES, DH, RH>::LDS_BYTES <= 160 * 1024 && Lay::N_ALL <= 44) {
		// weight gradients split across the waves, all fragments in registers (k_nerf_mlp_train)
		void (*kt)(const NerfMlpArgs) = k_nerf_mlp_train<ES, DH, RH>;
		const size_t lt = NerfTrainLayout<ES, DH, RH>::LDS_BYTES;
		ensure_dynamic_lds((const void*)kt, lt);
		kt<<<blocks, 256, lt, s>>>(a);
		NGP_HIP(hipGetLastError());
		return;
	}
	auto kern = k_nerf_mlp<ES, DH, RH, MODE>;
	ensure_dynamic_lds((const void*)kern, lds);
	auto ak = a;
	ak.n_reg = n_reg;
	kern<<<blocks, 256, lds, s>>>(ak);
	NGP_HIP(hipGetLastError());
}

uint32_t nerf_mlp_train_blocks(uint32_t n) {
	// NGP_MLP_TRAIN_BLOCKS: blocks per CU x 100 (experiment knob; default 100 = one block per CU)
	static const uint32_t per_cu100 = [] {
		const char* v = getenv("NGP_MLP_TRAIN_BLOCKS");
		const int x = v ? atoi(v) : 100;
		return (uint32_t)(x >= 25 && x <= 1600 ? x : 100);
	}();
	const uint32_t tiles = (n + 31) / 32;
	return std::max<uint32_t>(1, std::min<uint32_t>(div_round_up(tiles, 4), device_cu_count() * per_cu100 / 100));
}

template <int MODE>
static void dispatch_nerf(const NerfMlpPlan& p, const NerfMlpArgs& a, hipStream_t s) {
	const uint32_t key = p.enc_steps * 100 + p.d_hidden * 10 + p.r_hidden;
	switch (key) {
		case 112: launch_nerf<1, 1, 2, MODE>(a, s); break;
		case 212: launch_nerf<2, 1, 2, MODE>(a, s); break;
		case 111: launch_nerf<1, 1, 1, MODE>(a, s); break;
		case 122: launch_nerf<1, 2, 2, MODE>(a, s); break;
		case 113: launch_nerf<1, 1, 3, MODE>(a, s); break;
		case 213: launch_nerf<2, 1, 3, MODE>(a, s); break;
		case 222: launch_nerf<2, 2, 2, MODE>(a, s); break;
		default: throw Error("NerfNetwork: unsupported (encoding width, density/rgb hidden layers) combination");
	}
}

template <int MODE>
static void dispatch_nerf_fused(const NerfMlpPlan& p, const NerfMlpArgs& a, hipStream_t s) {
	const uint32_t key = p.enc_steps * 100 + p.d_hidden * 10 + p.r_hidden;
	if (key == 112) launch_nerf<1, 1, 2, MODE>(a, s);
	else if (key == 111) launch_nerf<1, 1, 1, MODE>(a, s);
	else if (key == 113) launch_nerf<1, 1, 3, MODE>(a, s);
	else throw Error("NerfNetwork: the fused encoding needs one encoding step and one density hidden layer");
}

void nerf_mlp_run(const NerfMlpPlan& p, MlpMode mode, const NerfMlpArgs& a, hipStream_t s) {
	if (a.n == 0) return;
	switch (mode) {
		case MLP_INFER: dispatch_nerf<MLP_INFER>(p, a, s); break;
		case MLP_TRAIN: dispatch_nerf<MLP_TRAIN>(p, a, s); break;
		case MLP_DENSITY: dispatch_nerf<MLP_DENSITY>(p, a, s); break;
		case MLP_INFER_ENC: dispatch_nerf_fused<MLP_INFER_ENC>(p, a, s); break;
		case MLP_DENSITY_TRAIN: dispatch_nerf<MLP_DENSITY_TRAIN>(p, a, s); break;
	}
}

bool nerf_mlp_fused_encoding_ok(const GridDesc& g, uint32_t enc_width) {
	return g.n_dims == 3 && g.n_levels == 4 && g.n_features == 4 && enc_width == 16;
}

// ------------------------------------------------------------------------------------------------
// Single MLP (NetworkWithInputEncoding): enc -> 64 x NH -> 16
// ------------------------------------------------------------------------------------------------
// WD = n_neurons (16, 32 or 64): hidden layers are HT = ceil(WD / 32) accumulator tiles of 32 rows (a
// 16-wide layer uses rows 0..15 of one tile; the padded rows have zero weights, so they hold zero and
// never reach the next layer, which reads HS = WD / 16 k-steps).
template <int ES, int NH, int WD>
struct MlpLayout {
	static constexpr int HT = (WD + 31) / 32;
	static constexpr int HS = WD / 16;
	static constexpr int F_0 = 0;
	static constexpr int F_H = F_0 + HT * ES;
	static constexpr int F_O = F_H + HT * HS * (NH - 1);
	static constexpr int N_FWD = F_O + HS;
	static constexpr int B_O = N_FWD;
	static constexpr int B_H = B_O + HT;
	static constexpr int B_0 = B_H + HT * HS * (NH - 1);
	static constexpr int ET = (ES + 1) / 2;
	static constexpr int N_ALL = B_0 + ET * HS;
	static constexpr int S_XE = 16 * ES + 4;
	static constexpr int S_W = WD + 4;
	static constexpr int I_XE = 0;
	static constexpr int I_H = I_XE + 32 * S_XE;
	static constexpr int I_DZ = I_H + NH * 32 * S_W;
	static constexpr int IMG_HALVES = I_DZ + 32 * S_W;
	static constexpr int W_O = 0;
	static constexpr int W_H = HS;
	static constexpr int W_0 = W_H + HS * HS * (NH - 1);
	static constexpr int N_DW = W_0 + HS * ES;
};

template <int ES, int NH, int WD, int MODE>
__global__ void __launch_bounds__(256, 1) k_mlp(const MlpArgs a) {
	using Lay = MlpLayout<ES, NH, WD>;
	constexpr int HT = Lay::HT, HS = Lay::HS;
	constexpr bool TRAIN = MODE == MLP_TRAIN;
	constexpr int NFRAG = TRAIN ? Lay::N_ALL : Lay::N_FWD;
	extern __shared__ __attribute__((aligned(16))) char smem[];
	f16x8* lfrag = (f16x8*)smem;
	const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
	for (int i = threadIdx.x; i < NFRAG * 64; i += blockDim.x) lfrag[i] = a.frags[i];
	__syncthreads();
	f16* img = (f16*)(smem + NFRAG * 1024) + wave * Lay::IMG_HALVES;
	f32x4 dw[TRAIN ? Lay::N_DW : 1];
	if constexpr (TRAIN) {
#pragma unroll
		for (int q = 0; q < Lay::N_DW; ++q) dw[q] = f32x4{0.f, 0.f, 0.f, 0.f};
	}
	const uint32_t n_tiles = (a.n + 31) / 32;
	for (uint32_t tile = blockIdx.x * 4 + wave; tile < n_tiles; tile += gridDim.x * 4) {
		const uint32_t sample = tile * 32 + (lane & 31);
		const bool valid = sample < a.n;
		const uint32_t ls = valid ? sample : 0;
		f16x8 xe[ES];
#pragma unroll
		for (int s = 0; s < ES; ++s) {
			xe[s] = *(const f16x8*)(a.enc + (size_t)ls * a.enc_stride + 16 * s + 8 * h);
			if (!valid) xe[s] = f16x8{};
			if constexpr (TRAIN) img_store_std(img + Lay::I_XE, Lay::S_XE, xe[s], s, lane);
		}
		f32x16 acc[HT];
		f16x8 hh[NH][2 * HT];
		layer_fwd<HT, ES>(acc, xe, lfrag + Lay::F_0 * 64, lane);
		pack_tiles<HT>(acc, hh[0], true);
#pragma unroll
		for (int l = 1; l < NH; ++l) {
			layer_fwd<HT, HS>(acc, hh[l - 1], lfrag + (Lay::F_H + HT * HS * (l - 1)) * 64, lane);
			pack_tiles<HT>(acc, hh[l], true);
		}
		f32x16 oacc[1];
		layer_fwd<1, HS>(oacc, hh[NH - 1], lfrag + Lay::F_O * 64, lane);
		if (a.out && valid) {
			f16x8 lo, hi;
			pack_tile(oacc[0], lo, hi, false);
			store_out16(a.out, a.out_stride, a.out_layout, a.n, sample, h, lo);
		}
		if constexpr (TRAIN) {
#pragma unroll
			for (int l = 0; l < NH; ++l) img_store_acc<HS>(img + Lay::I_H + l * 32 * Lay::S_W, Lay::S_W, hh[l], lane);
			f16* dz_img = img + Lay::I_DZ;
			f16x8 dzo[1];
			{
				// all 16 padded output rows carry gradient (tcnn loss writes the padded rows as zero)
				f16x8 d = f16x8{};
				if (valid) {
					const f16* r = a.dL_dout + (size_t)sample * a.dL_stride;
					const f16x4 p0 = *(const f16x4*)(r + 4 * h), p1 = *(const f16x4*)(r + 8 + 4 * h);
					d = f16x8{p0[0], p0[1], p0[2], p0[3], p1[0], p1[1], p1[2], p1[3]};
				}
				dzo[0] = d;
			}
			img_store_acc<1>(dz_img, Lay::S_W, dzo, lane);
			dw_accum<1, HS>(dw + Lay::W_O, dz_img, Lay::S_W, img + Lay::I_H + (NH - 1) * 32 * Lay::S_W, Lay::S_W, lane);
			f16x8 dz[2 * HT];
			layer_fwd<HT, 1>(acc, dzo, lfrag + Lay::B_O * 64, lane);
			mask_pack<HT>(acc, hh[NH - 1], dz);
#pragma unroll
			for (int l = NH - 1; l >= 1; --l) {
				img_store_acc<HS>(dz_img, Lay::S_W, dz, lane);
				dw_accum<HS, HS>(dw + Lay::W_H + HS * HS * (NH - 1 - l), dz_img, Lay::S_W, img + Lay::I_H + (l - 1) * 32 * Lay::S_W, Lay::S_W, lane);
				layer_fwd<HT, HS>(acc, dz, lfrag + (Lay::B_H + HT * HS * (NH - 1 - l)) * 64, lane);
				mask_pack<HT>(acc, hh[l - 1], dz);
			}
			img_store_acc<HS>(dz_img, Lay::S_W, dz, lane);
			dw_accum<HS, ES>(dw + Lay::W_0, dz_img, Lay::S_W, img + Lay::I_XE, Lay::S_XE, lane);
			if (a.dL_denc) {
				f32x16 ae[Lay::ET];
				layer_fwd<Lay::ET, HS>(ae, dz, lfrag + Lay::B_0 * 64, lane);
#pragma unroll
				for (int t = 0; t < Lay::ET; ++t) {
					f16x8 lo, hi;
					pack_tile(ae[t], lo, hi, false);
					if (!valid) continue;
					f16* row = a.dL_denc + (size_t)sample * a.denc_stride + 32 * t + 4 * h;
					*(f16x4*)(row + 0) = f16x4{lo[0], lo[1], lo[2], lo[3]};
					*(f16x4*)(row + 8) = f16x4{lo[4], lo[5], lo[6], lo[7]};
					if (32 * t + 16 < 16 * ES) {
						*(f16x4*)(row + 16) = f16x4{hi[0], hi[1], hi[2], hi[3]};
						*(f16x4*)(row + 24) = f16x4{hi[4], hi[5], hi[6], hi[7]};
					}
				}
			}
		}
	}
	if constexpr (TRAIN) {
		const uint32_t o_off = WD * 16 * ES + WD * WD * (NH - 1);
		dw_block_reduce((float*)smem, a.n_matrix, a.n_reg, wave, a.dw_slab + (size_t)blockIdx.x * a.n_matrix,
		                [&](float* red, auto first) {
			dw_flush<1, HS>(dw + Lay::W_O, red, o_off, WD, lane, first);
#pragma unroll
			for (int l = NH - 1; l >= 1; --l)
				dw_flush<HS, HS>(dw + Lay::W_H + HS * HS * (NH - 1 - l), red, WD * 16 * ES + WD * WD * (l - 1), WD, lane, first);
			dw_flush<HS, ES>(dw + Lay::W_0, red, 0, 16 * ES, lane, first);
		});
	}
}

uint32_t mlp_train_blocks(uint32_t n) { return nerf_mlp_train_blocks(n); }

template <int ES, int NH, int WD, int MODE>
static void launch_mlp(const MlpArgs& a, hipStream_t s) {
	using Lay = MlpLayout<ES, NH, WD>;
	constexpr bool TRAIN = MODE == MLP_TRAIN;
	constexpr int NFRAG = TRAIN ? Lay::N_ALL : Lay::N_FWD;
	size_t lds = (size_t)NFRAG * 1024 + (TRAIN ? 4 * Lay::IMG_HALVES * sizeof(f16) : 0);
	uint32_t n_reg = 4;
	while (n_reg > 1 && (size_t)n_reg * a.n_matrix * sizeof(float) > 160 * 1024) n_reg /= 2;
	if (TRAIN) lds = std::max(lds, (size_t)n_reg * a.n_matrix * sizeof(float));
	NGP_CHECK(lds <= 160 * 1024, "MLP: LDS budget exceeded");
	const uint32_t tiles = (a.n + 31) / 32;
	uint32_t blocks = TRAIN ? mlp_train_blocks(a.n) : std::min<uint32_t>(div_round_up(tiles, 4), 8 * device_cu_count());
	auto kern = k_mlp<ES, NH, WD, MODE>;
	ensure_dynamic_lds((const void*)kern, lds);
	auto ak = a;
	ak.n_reg = n_reg;
	kern<<<blocks, 256, lds, s>>>(ak);
	NGP_HIP(hipGetLastError());
}

template <int WD, int MODE>
static void dispatch_mlp_w(const MlpPlan& p, const MlpArgs& a, hipStream_t s) {
	switch (p.enc_steps * 10 + p.hidden) {
		case 11: launch_mlp<1, 1, WD, MODE>(a, s); break;
		case 12: launch_mlp<1, 2, WD, MODE>(a, s); break;
		case 13: launch_mlp<1, 3, WD, MODE>(a, s); break;
		case 21: launch_mlp<2, 1, WD, MODE>(a, s); break;
		case 22: launch_mlp<2, 2, WD, MODE>(a, s); break;
		case 23: launch_mlp<2, 3, WD, MODE>(a, s); break;
		case 24: launch_mlp<2, 4, WD, MODE>(a, s); break;
		default: throw Error("FullyFusedMLP: unsupported (encoding width, hidden layers) combination");
	}
}
template <int MODE>
static void dispatch_mlp(const MlpPlan& p, const MlpArgs& a, hipStream_t s) {
	switch (p.mlp.width) {
		case 16: dispatch_mlp_w<16, MODE>(p, a, s); break;
		case 32: dispatch_mlp_w<32, MODE>(p, a, s); break;
		case 64: dispatch_mlp_w<64, MODE>(p, a, s); break;
		default: throw Error("FullyFusedMLP: n_neurons must be 16, 32 or 64");
	}
}

void mlp_run(const MlpPlan& p, MlpMode mode, const MlpArgs& a, hipStream_t s) {
	if (a.n == 0) return;
	if (mode == MLP_TRAIN) dispatch_mlp<MLP_TRAIN>(p, a, s);
	else dispatch_mlp<MLP_INFER>(p, a, s);
}

// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(SLAB_THREADS) k_reduce_slabs(const SlabJob j) { reduce_slabs_block(j, blockIdx.x); }

void reduce_slabs(const float* slabs, uint32_t n_slabs, uint32_t n, f16* grad, bool accumulate, hipStream_t s, uint32_t stride) {
	SlabJob j;
	j.slabs = slabs; j.n_slabs = n_slabs; j.n = n; j.grad = grad; j.accumulate = accumulate; j.stride = stride;
	k_reduce_slabs<<<slab_blocks(n), SLAB_THREADS, 0, s>>>(j);
	NGP_HIP(hipGetLastError());
}

}  // namespace ngp

#ifdef NGP_TRAIN_CLOCK
extern "C" __attribute__((visibility("default"))) int ngp_debug_train_clock(uint64_t* out, uint32_t n) {
	return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ngp::g_train_clock),
	                                (size_t)(n < 1024 * ngp::TRC_SLOTS ? n : 1024 * ngp::TRC_SLOTS) * 8, 0, hipMemcpyDeviceToHost);
}
#endif
