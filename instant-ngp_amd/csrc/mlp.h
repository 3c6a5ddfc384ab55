// mlp.h — fully-fused 64-wide fp16 MLPs on CDNA4 MFMA (replaces tcnn::FullyFusedMLP<half, 64>,
// SURVEY §8a row a3, as composed by ngp::NerfNetwork, nerf_network.h:81-335).
//
// Orientation: samples are the MFMA N (lane) dimension. A layer computes Y^T = W * X^T with
// v_mfma_f32_32x32x16_f16: A = weight fragment (LDS), B = activations of 32 samples (registers).
// A 32x32 accumulator tile holds sample = lane&31 and rows (r&3) + 8(r>>2) + 4(lane>>5), so packing
// registers 8s..8s+7 to fp16 gives the B operand of the next layer's k-step s directly (the k order
// inside a step is permuted; the weight fragments are pre-permuted to match). The forward chain and
// the backward dX chain therefore never leave registers. Weight gradients need the batch as the
// contraction axis: activations and output gradients are written to per-wave LDS images
// [sample][feature] and read back with ds_read_b64_tr_b16 as v_mfma_f32_16x16x32_f16 operands
// (K = 32 samples per instruction). Numerics: fp16 operands, fp32 accumulation, every layer output
// rounded to fp16 (RNE) — the oracle's contract (oracle/ngp_oracle.c orc_mlp_*).
#pragma once
#include "common.h"
#include "grid.h"

namespace ngp {

// One 1-KiB weight fragment = 64 lanes x 8 halves. Descriptor used by the preparation kernel.
struct FragDesc {
	uint32_t woff;      // offset of W (row-major [out x in]) in the parameter buffer
	uint16_t in_dim, out_dim;
	uint8_t tile, step, transposed, perm;  // perm: k order of a packed accumulator
};

// Parameter-space layout of one MLP (tcnn FullyFusedMLP order: layer 0, hidden..., output).
struct MlpDims {
	uint32_t in_pad, width, n_hidden, out_pad;
	uint32_t n_params() const { return width * in_pad + (n_hidden - 1) * width * width + out_pad * width; }
	uint32_t layer_in(uint32_t l) const { return l == 0 ? in_pad : width; }
	uint32_t layer_out(uint32_t l) const { return l == n_hidden ? out_pad : width; }
	uint32_t layer_off(uint32_t l) const {
		uint32_t o = 0;
		for (uint32_t k = 0; k < l; ++k) o += layer_in(k) * layer_out(k);
		return o;
	}
};

struct NerfMlpArgs {
	uint32_t n;
	const f16* enc; uint32_t enc_stride;          // density network input, AoS [n x enc_stride]
	const float* coords; uint32_t coord_stride;   // NerfCoordinate AoS, for the SH direction encoding
	uint32_t dir_offset;
	const f16x8* frags;                           // prepared fragments (global), copied to LDS
	uint32_t n_frags;
	f16* out; uint32_t out_stride; uint32_t out_layout;   // [n x 16] (rgb raw 0..2, density raw 3)
	const f16* dL_dout; uint32_t dL_stride;       // training: [n x 16]
	f16* dL_denc; uint32_t denc_stride;           // training: [n x enc] (nullptr: skip)
	float* dw_slab;                               // training: [gridDim.x x n_matrix] partial sums
	uint32_t n_matrix;                            // matrix params = density MLP + rgb MLP
	uint32_t n_reg;                               // LDS regions of the dW block reduction (set at launch)
	uint32_t density_woff, rgb_woff;              // parameter offsets of the two MLPs
	// MLP_INFER_ENC: the density network's input is encoded in the kernel (hash-grid gather and
	// trilinear blend of the sample's levels, same arithmetic as k_grid_forward_rows) instead of read
	const f16* table;                             // grid parameters [entries x F]
	float max_level;                              // tcnn set_max_level (global; per-sample masks not fused)
	GridConst gc;
	// input gradients (nerf_network.h:282-299): dL/d(SH encoding) = rows 16..31 of the rgb network's dL/dinput,
	// fp16 [n x 16] (nullptr: skip)
	f16* dL_dsh;
	// MLP_DENSITY_TRAIN (NerfNetwork::density_backward, nerf_network.h:384-428): dL/d(density network output),
	// fp16 AoS [n x ddens_stride] (16 rows; stride a multiple of 4)
	const f16* dL_ddens; uint32_t ddens_stride;
};

struct MlpArgs {  // single MLP behind an encoding (tcnn::NetworkWithInputEncoding): image / SDF
	uint32_t n;
	const f16* enc; uint32_t enc_stride;
	const f16x8* frags; uint32_t n_frags;
	f16* out; uint32_t out_stride; uint32_t out_layout;
	const f16* dL_dout; uint32_t dL_stride;
	f16* dL_denc; uint32_t denc_stride;
	float* dw_slab; uint32_t n_matrix;
	uint32_t n_reg;
};

// Host API ---------------------------------------------------------------------------------------
struct NerfMlpPlan {
	uint32_t enc_steps, d_hidden, r_hidden;
	MlpDims density, rgb;
	uint32_t n_fwd_frags, n_bwd_frags;
	std::vector<FragDesc> descs;  // fwd frags then bwd frags
};
struct MlpPlan {
	uint32_t enc_steps, hidden;
	MlpDims mlp;
	uint32_t n_fwd_frags, n_bwd_frags;
	std::vector<FragDesc> descs;
};

NerfMlpPlan make_nerf_mlp_plan(uint32_t enc_width, uint32_t width, uint32_t d_hidden, uint32_t r_hidden);
MlpPlan make_mlp_plan(uint32_t enc_width, uint32_t width, uint32_t hidden, uint32_t out_pad);

void prepare_frags(const FragDesc* descs_dev, uint32_t n_frags, const f16* params, f16x8* frags, hipStream_t s);

enum MlpMode : uint32_t { MLP_INFER = 0, MLP_TRAIN = 1, MLP_DENSITY = 2, MLP_INFER_ENC = 3,
                          MLP_DENSITY_TRAIN = 5 };  // density network forward + backward only (NeRF)
// MLP_INFER_ENC is fused for 3D grids with 4 levels of 4 features (one 16-wide encoding step: C2)
// internal output layout of the density network: row 0 only, as a flat array of n (the density grid update
// reads nothing else)
constexpr uint32_t MLP_LAYOUT_ROW0 = 3;  // == DENSITY_LAYOUT_ROW0 (engine_internal.h)
bool nerf_mlp_fused_encoding_ok(const GridDesc& g, uint32_t enc_width);

// Launch sizes for the training kernel: one persistent block per CU (slab count = blocks).
uint32_t nerf_mlp_train_blocks(uint32_t n);
void nerf_mlp_run(const NerfMlpPlan& p, MlpMode mode, const NerfMlpArgs& a, hipStream_t s);
uint32_t mlp_train_blocks(uint32_t n);
void mlp_run(const MlpPlan& p, MlpMode mode, const MlpArgs& a, hipStream_t s);

// Sum [n_slabs x n] fp32 slabs into fp16 gradients: out = (accumulate ? out : 0) + sum.
// stride: elements between consecutive slabs (0: n); larger reduces only the leading n of each slab.
void reduce_slabs(const float* slabs, uint32_t n_slabs, uint32_t n, f16* grad, bool accumulate, hipStream_t s,
                  uint32_t stride = 0);

}  // namespace ngp
