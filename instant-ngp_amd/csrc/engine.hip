// engine.hip — model / trainer objects behind the C-ABI (include/ngp_engine.h).
//
// Mirrors the tcnn object graph the reference's Testbed builds in reset_network
// (src/testbed.cu:3903-4151): NerfNetwork = position GridEncoding -> density FullyFusedMLP ->
// [density out | SH(dir)] -> rgb FullyFusedMLP; NetworkWithInputEncoding = encoding -> MLP;
// Trainer = fp32 master weights + fp16 params/inference params/gradients + optimizer state.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>

#include "../../include/ngp_engine.h"
#include "common.h"
#include "engine_internal.h"
#include "grid_scatter.h"
#include "grid.h"
#include "json.h"
#include "mlp.h"
#include "optimizer.h"
#include "profiler.h"
#include "training.h"

static_assert(ngp::DENSITY_LAYOUT_ROW0 == ngp::MLP_LAYOUT_ROW0, "the row-0 density layout of mlp.h and engine_internal.h");

namespace ngp {

int device_cu_count() {
	static int cached = -1;
	if (cached < 0) {
		int dev = 0;
		NGP_HIP(hipGetDevice(&dev));
		NGP_HIP(hipDeviceGetAttribute(&cached, hipDeviceAttributeMultiprocessorCount, dev));
	}
	return cached;
}

// Growable device buffer (grows outside the hot loop; ngp_model_reserve pre-sizes it).
// Every reallocation bumps *epoch (the owning model's workspace epoch): a captured HIP graph holds raw
// workspace pointers, so graph launches check the epoch they were captured at.
struct DevBuf {
	void* p = nullptr;
	size_t bytes = 0;
	uint64_t* epoch = nullptr;
	void* get(size_t need) {
		if (need > bytes) {
			if (p) NGP_HIP(hipFree(p));
			p = nullptr;
			NGP_HIP(hipMalloc(&p, need));
			NGP_HIP(hipMemset(p, 0, need));  // workspaces that must start zeroed (the grid backward's brick fallback table)
			bytes = need;
			if (epoch) ++*epoch;
		}
		return p;
	}
	~DevBuf() { if (p) (void)hipFree(p); }
};

// ---- pcg32 (tcnn::pcg32, random_val.cuh:26-43) used for parameter initialisation -------------
struct Pcg32 {
	uint64_t state = 0x853c49e6748fea9bULL, inc = 0xda3e39cb94b95bdbULL;
	static constexpr uint64_t MULT = 0x5851f42d4c957f2dULL;
	Pcg32(uint64_t initstate, uint64_t initseq = 1u) {
		state = 0u; inc = (initseq << 1u) | 1u; next_uint(); state += initstate; next_uint();
	}
	uint32_t next_uint() {
		uint64_t old = state;
		state = old * MULT + inc;
		uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u), rot = (uint32_t)(old >> 59u);
		return (xs >> rot) | (xs << ((~rot + 1u) & 31));
	}
	float next_float() { uint32_t u = (next_uint() >> 9) | 0x3f800000u; float f; memcpy(&f, &u, 4); return f - 1.0f; }
	void advance(uint64_t delta) {
		uint64_t cm = MULT, cp = inc, am = 1u, ap = 0u;
		while (delta > 0) {
			if (delta & 1) { am *= cm; ap = ap * cm + cp; }
			cp = (cm + 1) * cp; cm *= cm; delta /= 2;
		}
		state = am * state + ap;
	}
	// tcnn generate_random_uniform: element k takes draw k of the stream; the caller advances by n
	void uniform(size_t n, float* out, float lo, float hi) {
		Pcg32 r = *this;
		for (size_t k = 0; k < n; ++k) out[k] = r.next_float() * (hi - lo) + lo;
		advance(n);
	}
};

static void init_mlp(const MlpDims& d, Pcg32& rng, float* p, float scale) {
	for (uint32_t l = 0; l <= d.n_hidden; ++l) {
		const uint32_t in = d.layer_in(l), out = d.layer_out(l);
		const float s = sqrtf(6.0f / (float)(in + out)) * scale;  // Xavier-uniform
		rng.uniform((size_t)in * out, p + d.layer_off(l), -s, s);
	}
}

// tcnn's GridEncoding otypes: HashGrid (= Grid with type Hash) and DenseGrid (= Grid with type Dense, e.g.
// configs/nerf/densegrid.json). A dense level holds res^D entries (rounded to 8) with no hashmap cap, so its
// stride never exceeds its size and grid_index never hashes: the hash-grid kernels run it unchanged with the
// cap lifted (GRID_LOG2_DENSE). TiledGrid is not implemented.
static GridDesc parse_grid(uint32_t n_dims, const Json& j) {
	const std::string ot = j.string_or("otype", "HashGrid");
	NGP_CHECK(iequals(ot, "HashGrid") || iequals(ot, "DenseGrid") || iequals(ot, "Grid"),
	          "encoding: HashGrid and DenseGrid are implemented (got " + ot + ")");
	const std::string type = j.string_or("type", iequals(ot, "DenseGrid") ? "Dense" : "Hash");
	NGP_CHECK(iequals(type, "Hash") || iequals(type, "Dense"), "encoding: grid type Hash or Dense (got " + type + ")");
	NGP_CHECK(iequals(j.string_or("interpolation", "Linear"), "Linear"), "encoding: only linear interpolation is implemented");
	GridDesc g;
	grid_desc_init(g, n_dims, (uint32_t)j.number_or("n_levels", 16), (uint32_t)j.number_or("n_features_per_level", 2),
	               iequals(type, "Dense") ? GRID_LOG2_DENSE : (uint32_t)j.number_or("log2_hashmap_size", 19),
	               (uint32_t)j.number_or("base_resolution", 16), (float)j.number_or("per_level_scale", 2.0));
	return g;
}

static uint32_t parse_mlp_hidden(const Json& j, uint32_t* width) {
	const std::string ot = j.string_or("otype", "FullyFusedMLP");
	NGP_CHECK(iequals(ot, "FullyFusedMLP") || iequals(ot, "CutlassMLP") || iequals(ot, "MegakernelMLP"),
	          "network: only FullyFusedMLP-shaped networks are implemented (got " + ot + ")");
	NGP_CHECK(iequals(j.string_or("activation", "ReLU"), "ReLU"), "network: only ReLU hidden activation is implemented");
	NGP_CHECK(iequals(j.string_or("output_activation", "None"), "None"), "network: only output_activation None is implemented");
	*width = (uint32_t)j.number_or("n_neurons", 64);
	return (uint32_t)j.number_or("n_hidden_layers", 2);
}

}  // namespace ngp

using namespace ngp;

struct ngp_ctx {
	uint32_t n;
	const float* input;
	uint32_t input_stride;
	bool use_inference_params;
	uint64_t generation;  // the model workspace generation the encoding lives in
	bool density_only = false;  // from ngp_density_forward: only ngp_density_backward may consume it
};

namespace ngp {
// Optional parts of a backward pass (ngp_model::train_pass)
struct BwdExtra {
	float* dL_dinput = nullptr;     // fp32 AoS [n x dinput_stride]: rows 0..D-1 (+ the direction rows of a NerfNetwork)
	uint32_t dinput_stride = 0;
	float dinput_scale = 1.f;
	bool density_only = false;      // NerfNetwork::density_backward: the density network alone
	const f16* ddens = nullptr;     // its dL/d(density output), fp16 AoS [n x ddens_stride]
	uint32_t ddens_stride = 0;
	bool inference = false;         // the forward context ran on the inference (EMA) parameters: so does the backward
};
}  // namespace ngp

struct ngp_model {
	bool nerf = true;
	GridDesc grid;
	uint32_t n_pos_dims = 3, n_dir_dims = 3, n_extra_dims = 0, dir_offset = 4, n_input_dims = 3, n_output_dims = 4;
	uint32_t enc_width = 16;
	NerfMlpPlan nplan;
	MlpPlan mplan;
	uint64_t mlp0_params = 0, mlp1_params = 0, grid_params = 0, n_params = 0;
	FragDesc* d_descs = nullptr;
	uint32_t* d_fragmap = nullptr;  // [n_matrix x 2] fragment slot (f16 index) of each matrix param: fwd, bwd
	bool frags_current = false;     // `frags` holds the fragments of the current `params` (kept by the optimizer)
	uint32_t n_all_frags = 0;
	DevBuf frags, frags_inf, enc, denc, slabs, scatter_ws, out_ws, dl_ws, dsh_ws, dl1_ws;
	int grid_backward_mode = 0;  // 0 auto, 1 direct (tcnn-style), 3 bucketed (grid_scatter.h)
	uint32_t win_debug = 0;      // timing experiments only (see grid_scatter.h)
	ScatterPlan sc_plan;
	uint32_t sc_plan_n = 0;
	bool sc_prepared = false;               // phase 1 of the bucketed backward already enqueued (side stream)
	bool sc_hist_done = false;              // the training forward produced the bucket histogram
	bool frags_async = false;               // training fragments already enqueued on the side stream
	// side-stream overlap (bitmask): 1 bucket histogram under forward + MLP, 2 weight fragments,
	// 4 dW slab reduction under the grid backward, 8 optimizer step advance. Each costs a cross-queue
	// dependency edge, which in a HIP graph is not free.
	uint32_t overlap = 0;
	bool fused_hist = true;                 // option "fused_hist": bucket histogram inside the training forward
	bool fuse_infer = true;                 // option "fuse_infer": NerfNetwork inference encodes inside the MLP kernel
	bool fuse_slabs = true;                 // option "fuse_slabs": dW slab reduction inside the grid backward's last kernel
	bool fuse_opt = true;                   // option "fuse_opt": lazy-layout optimizer update inside the grid backward (training_step)
	bool fuse_mlp_opt = true;               // option "fuse_mlp_opt": ... and the MLP section's update in its dW slab blocks (no optimizer launch)
	bool grid_bricks = false;               // option "grid_bricks": dense levels of the bucketed backward summed per brick (off: measured slower)
	hipStream_t side = nullptr;             // overlaps fragments + bucket histogram with forward + MLP,
	                                        // and the dW slab reduction with the grid backward
	hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_frags = nullptr, ev_mlp = nullptr, ev_red = nullptr;
	f16 *params = nullptr, *inference_params = nullptr, *gradients = nullptr;
	// lazy-EMA trainer: brings the inference (EMA) parameters up to date before they are read
	void (*inference_hook)(void*, hipStream_t) = nullptr;
	void* inference_hook_ctx = nullptr;
	void sync_inference(hipStream_t s) { if (inference_hook) inference_hook(inference_hook_ctx, s); }
	float max_level = 1.0f;
	const float* max_level_per_sample = nullptr;
	// false: the last training pass did not write the fp16 gradient buffer (the grid's update ran inside the
	// backward, or the backward stored the gradient as fp32 for the sharded exchange): ngp_trainer_gradients_valid
	bool grads_valid = true;
	// the sharded exchange's consumer of the grid backward's parts (BwdParts): set by the trainer around one
	// training pass, used when the bucketed backward runs without bricks or the fused update
	const BwdParts* bwd_parts = nullptr;
	bool parts_ok(uint32_t n) const {
		return use_sorted(n) && fuse_slabs && !(overlap & 4) && !grid_bricks && grid.n_features >= 2;
	}
	uint64_t generation = 0;
	uint64_t ws_epoch = 0;  // bumped by every workspace reallocation (DevBuf::epoch)
	std::unique_ptr<ngp_ctx> last_ctx;

	ngp_model() {
		for (DevBuf* b : {&frags, &frags_inf, &enc, &denc, &slabs, &scatter_ws, &out_ws, &dl_ws, &dsh_ws, &dl1_ws}) b->epoch = &ws_epoch;
	}

	~ngp_model() {
		if (d_descs) (void)hipFree(d_descs);
		if (d_fragmap) (void)hipFree(d_fragmap);
		for (hipEvent_t e : {ev_fork, ev_join, ev_frags, ev_mlp, ev_red})
			if (e) (void)hipEventDestroy(e);
		if (side) (void)hipStreamDestroy(side);
	}
	// allocate every buffer a training pass over n samples touches (nothing may allocate during graph capture)
	void reserve(uint32_t n) {
		enc.get((size_t)n * enc_width * sizeof(f16));
		denc.get((size_t)n * enc_width * sizeof(f16));
		const uint32_t blocks = nerf ? nerf_mlp_train_blocks(n) : mlp_train_blocks(n);
		slabs.get((size_t)blocks * n_matrix() * sizeof(float));
		frags.get((size_t)n_all_frags * 1024);
		frags_inf.get((size_t)n_all_frags * 1024);
		if (use_sorted(n)) {
			sorted_workspace(n);
			ensure_side_stream();
		}
	}
	void ensure_side_stream() {
		if (side) return;
		NGP_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
		NGP_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
		NGP_HIP(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
		NGP_HIP(hipEventCreateWithFlags(&ev_frags, hipEventDisableTiming));
		NGP_HIP(hipEventCreateWithFlags(&ev_mlp, hipEventDisableTiming));
		NGP_HIP(hipEventCreateWithFlags(&ev_red, hipEventDisableTiming));
	}
	bool use_sorted(uint32_t n) const { return grid_backward_mode == 3 || (grid_backward_mode == 0 && n >= 4096); }
	// the backward can store the whole gradient as fp32 itself (FusedAdam::g32): bucketed grid backward with the
	// dW slab reduction in its last kernel
	bool grad32_ok(uint32_t n) const { return use_sorted(n) && fuse_slabs && !(overlap & 4) && grid.n_features >= 2; }
	bool side_prepare(uint32_t n) const { return use_sorted(n) && (overlap & 1); }
	const ScatterPlan& sc_plan_for(uint32_t n) {
		if (sc_plan_n != n) {
			sc_plan = make_scatter_plan(grid, n, grid_bricks);
			sc_plan_n = n;
			fb_dirty = true;  // the brick fallback table may now lie over bytes the previous plan used (items)
		}
		return sc_plan;
	}
	// The brick levels' fallback table must be zero when a backward adds into it (each finalize clears the
	// entries it reads, so it stays zero between steps of one plan). A new plan moves it (its offset follows
	// the item regions, sized by the batch): zero it once on the stream before the plan's first backward.
	bool fb_dirty = true;
	void clear_brick_fallback(hipStream_t s, void* ws) {
		if (!fb_dirty) return;
		if (sc_plan.bk.LD) NGP_HIP(hipMemsetAsync((char*)ws + sc_plan.off_fb, 0, sc_plan.total - sc_plan.off_fb, s));
		fb_dirty = false;
	}
	void* sorted_workspace(uint32_t n) { return scatter_ws.get(sc_plan_for(n).total); }
	// Phase 1 of the bucketed grid backward on a side stream: it only needs the positions, so it runs
	// concurrently with the forward encoding and the MLP; train_pass joins before the scatter.
	void prepare_grid_backward_async(hipStream_t s, uint32_t n, const float* in, uint32_t stride) {
		if (!side_prepare(n)) return;
		ensure_side_stream();
		void* ws = sorted_workspace(n);
		clear_brick_fallback(s, ws);  // on s, before the fork: the side stream's plan kernel writes the flag after it
		GridBwdArgs b{n, in, stride, nullptr, 0, AoS, nullptr, max_level, max_level_per_sample};
		NGP_HIP(hipEventRecord(ev_fork, s));
		NGP_HIP(hipStreamWaitEvent(side, ev_fork, 0));
		// the training MLP's weight fragments depend only on the parameters: build them here, off the
		// critical path (run_mlp waits on ev_frags instead of launching k_prepare_frags itself)
		if ((overlap & 2) && !frags_current) {
			prep(side, false);
			NGP_HIP(hipEventRecord(ev_frags, side));
			frags_async = true;
		}
		{
			ProfScope ps("grid_bwd_prepare", side);
			grid_scatter_prepare(grid, b, sc_plan, ws, side);
		}
		NGP_HIP(hipEventRecord(ev_join, side));
		sc_prepared = true;
	}

	const std::vector<FragDesc>& descs() const { return nerf ? nplan.descs : mplan.descs; }
	uint64_t grid_offset() const { return mlp0_params + mlp1_params; }
	uint64_t n_matrix() const { return mlp0_params + mlp1_params; }

	void finalize() {
		grid_params = grid.n_params();
		n_params = mlp0_params + mlp1_params + grid_params;
		const auto& d = descs();
		n_all_frags = (uint32_t)d.size();
		NGP_HIP(hipMalloc(&d_descs, d.size() * sizeof(FragDesc)));
		NGP_HIP(hipMemcpy(d_descs, d.data(), d.size() * sizeof(FragDesc), hipMemcpyHostToDevice));
		// inverse of k_prepare_frags: where each matrix parameter lives in the fragment buffer
		std::vector<uint32_t> map(2 * n_matrix(), ~0u);
		for (uint32_t f = 0; f < n_all_frags; ++f)
			for (uint32_t lane = 0; lane < 64; ++lane)
				for (uint32_t j = 0; j < 8; ++j) {
					const FragDesc& q = d[f];
					const uint32_t h = lane >> 5, r = 32 * q.tile + (lane & 31);
					const uint32_t k = q.perm ? 16 * q.step + 8 * (j >> 2) + 4 * h + (j & 3) : 16 * q.step + 8 * h + j;
					uint64_t pi;
					if (!q.transposed) {
						if (!(r < q.out_dim && k < q.in_dim)) continue;
						pi = q.woff + (uint64_t)r * q.in_dim + k;
					} else {
						if (!(r < q.in_dim && k < q.out_dim)) continue;
						pi = q.woff + (uint64_t)k * q.in_dim + r;
					}
					NGP_CHECK(pi < n_matrix() && map[2 * pi + q.transposed] == ~0u, "fragment map: parameter mapped twice");
					map[2 * pi + q.transposed] = (f * 64 + lane) * 8 + j;
				}
		NGP_HIP(hipMalloc(&d_fragmap, map.size() * sizeof(uint32_t)));
		NGP_HIP(hipMemcpy(d_fragmap, map.data(), map.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
	}
	void require_params(bool inference) const {
		NGP_CHECK(inference ? inference_params != nullptr : params != nullptr,
		          "model has no parameters: call ngp_model_set_params or create a trainer first");
	}
	const f16* pick(bool inference) const { return inference ? inference_params : params; }
	bool fused_encoding_ok() const {
		return nerf && !max_level_per_sample && nerf_mlp_fused_encoding_ok(grid, enc_width) && nplan.enc_steps == 1 &&
		       nplan.d_hidden == 1 && nplan.r_hidden >= 1 && nplan.r_hidden <= 3;
	}
	bool fused_inference_ok() const { return fuse_infer && fused_encoding_ok(); }
	f16x8* prep(hipStream_t s, bool inference) {
		f16x8* f = (f16x8*)(inference ? frags_inf : frags).get((size_t)n_all_frags * 1024);
		if (inference) sync_inference(s);
		ProfScope ps("prepare_frags", s);
		prepare_frags(d_descs, n_all_frags, pick(inference), f, s);
		if (!inference) frags_current = true;
		return f;
	}
	// want_hist: a training forward whose backward follows on the same positions — count the sorted
	// backward's bucket histogram in the forward kernel (its corner indices are computed anyway).
	void encode(hipStream_t s, uint32_t n, const float* in, uint32_t stride, f16* out, uint32_t out_stride, uint32_t layout, bool inference,
	            bool want_hist = false) {
		if (inference) sync_inference(s);
		GridFwdArgs a{n, in, stride, pick(inference) + grid_offset(), out, out_stride, layout, max_level, max_level_per_sample};
		if (enc_width > grid.n_levels * grid.n_features && layout == AoS && !grid_forward_rows_ok(grid, a)) {
			// zero the padding columns (tcnn pads the encoding output with zeros); the row kernel writes them
			NGP_HIP(hipMemsetAsync(out, 0, (size_t)n * out_stride * sizeof(f16), s));
		}
		sc_hist_done = false;
		GridHist h;
		const bool fuse = want_hist && fused_hist && use_sorted(n) && !sc_prepared && grid_forward_rows_ok(grid, a) &&
		                  scatter_hist(grid, sc_plan_for(n), sorted_workspace(n), h);
		ProfScope ps("grid_forward", s);
		grid_forward(grid, a, s, fuse ? &h : nullptr);
		sc_hist_done = fuse;
	}
	void run_mlp(hipStream_t s, MlpMode mode, uint32_t n, const float* in, uint32_t stride, const f16* encbuf, f16* out,
	             uint32_t out_stride, uint32_t out_layout, const f16* dL, uint32_t dL_stride, f16* dL_denc, float* slab,
	             bool inference, const BwdExtra* ex = nullptr, f16* dL_dsh = nullptr) {
		f16x8* f;
		if (frags_async && !inference) {
			f = (f16x8*)frags.p;
			NGP_HIP(hipStreamWaitEvent(s, ev_frags, 0));
			frags_async = false;
		} else if (!inference && frags_current && frags.p) {
			f = (f16x8*)frags.p;  // kept current by the optimizer (k_adam_ema writes the fragment slots)
		} else {
			f = prep(s, inference);
		}
		if (nerf) {
			NerfMlpArgs a{};
			a.n = n; a.enc = encbuf; a.enc_stride = enc_width; a.coords = in; a.coord_stride = stride; a.dir_offset = dir_offset;
			a.frags = f; a.n_frags = n_all_frags; a.out = out; a.out_stride = out_stride; a.out_layout = out_layout;
			a.dL_dout = dL; a.dL_stride = dL_stride; a.dL_denc = dL_denc; a.denc_stride = enc_width; a.dw_slab = slab;
			a.n_matrix = (uint32_t)n_matrix(); a.density_woff = 0; a.rgb_woff = (uint32_t)mlp0_params;
			a.dL_dsh = dL_dsh;
			if (ex) { a.dL_ddens = ex->ddens; a.ddens_stride = ex->ddens_stride; }
			if (mode == MLP_INFER_ENC) {
				if (inference) sync_inference(s);
				a.table = pick(inference) + grid_offset(); a.max_level = max_level; a.gc = make_grid_const(grid);
			}
			ProfScope ps(mode == MLP_TRAIN ? "mlp_train" : mode == MLP_DENSITY ? "mlp_density"
			             : mode == MLP_INFER_ENC ? "mlp_infer_enc"
			             : mode == MLP_DENSITY_TRAIN ? "mlp_density_train" : "mlp_infer", s);
			nerf_mlp_run(nplan, mode, a, s);
		} else {
			MlpArgs a{};
			a.n = n; a.enc = encbuf; a.enc_stride = enc_width; a.frags = f; a.n_frags = n_all_frags;
			a.out = out; a.out_stride = out_stride; a.out_layout = out_layout; a.dL_dout = dL; a.dL_stride = dL_stride;
			a.dL_denc = dL_denc; a.denc_stride = enc_width; a.dw_slab = slab; a.n_matrix = (uint32_t)n_matrix();
			ProfScope ps(mode == MLP_TRAIN ? "mlp_train" : "mlp_infer", s);
			mlp_run(mplan, mode == MLP_DENSITY ? MLP_INFER : mode, a, s);
		}
	}
	// backward given the encoding already in `encbuf`: MLP fwd+bwd (+output), dW slabs, grid scatter.
	// ex (optional): input gradients and the density-only backward (BwdExtra); grad_mode NGP_GRAD_IGNORE
	// leaves the parameter gradients untouched (tcnn EGradientMode::Ignore, input_gradient).
	void train_pass(hipStream_t s, uint32_t n, const float* in, uint32_t stride, const f16* encbuf, f16* out, uint32_t out_stride,
	                const void* dL, uint32_t dL_stride, int grad_mode, const BwdExtra& ex = BwdExtra{}, const FusedAdam* fopt = nullptr) {
		NGP_CHECK(gradients || grad_mode == NGP_GRAD_IGNORE, "model has no gradient buffer: call ngp_model_set_params");
		NGP_CHECK(!ex.density_only || (nerf && encbuf), "density backward: a NerfNetwork with its encoding");
		f16* dL_denc = (f16*)denc.get((size_t)n * enc_width * sizeof(f16));
		const uint32_t blocks = nerf ? nerf_mlp_train_blocks(n) : mlp_train_blocks(n);
		float* slab = (float*)slabs.get((size_t)blocks * n_matrix() * sizeof(float));
		f16* dsh = ex.dL_dinput && nerf && !ex.density_only ? (f16*)dsh_ws.get((size_t)n * 16 * sizeof(f16)) : nullptr;
		NGP_CHECK(encbuf, "train_pass: the encoding buffer");
		const MlpMode mode = ex.density_only ? MLP_DENSITY_TRAIN : MLP_TRAIN;
		run_mlp(s, mode, n, in, stride, encbuf, out, out_stride, AoS, (const f16*)dL, dL_stride, dL_denc, slab, ex.inference, &ex,
		        dsh);
		// dL/dinput through the grid (position rows) and the SH encoding (direction rows, NerfNetwork). Run
		// last: dL_dinput may alias the input (the reference passes positions_matrix for both,
		// testbed_nerf.cu:2616), which the grid backward still reads
		auto input_gradient = [&]() {
			if (!ex.dL_dinput) return;
			ProfScope ps("input_gradient", s);
			if (ex.inference) sync_inference(s);
			InputGradArgs ia{n, in, stride, pick(ex.inference) + grid_offset(), dL_denc, enc_width, max_level, max_level_per_sample, dsh,
			                 dir_offset, ex.dL_dinput, ex.dinput_stride, ex.dinput_scale};
			grid_input_gradient(grid, ia, s);
		};
		if (grad_mode == NGP_GRAD_IGNORE) {
			input_gradient();
			return;
		}
		grads_valid = !(fopt && (fopt->rec || fopt->g32));
		// the dW slab reduction (MLP section of the gradient) and the grid backward (grid section) are
		// independent: for large batches the reduction runs in extra blocks of the grid backward's last
		// kernel (fuse_slabs, default), or on the side stream under it (overlap bit 4). The density-only
		// backward reduces the density MLP's leading slice of each slab (the rgb gradients stay untouched).
		const bool ovl = use_sorted(n) && (overlap & 4);
		const bool fused = use_sorted(n) && !ovl && fuse_slabs && !ex.density_only;
		const uint32_t n_red = ex.density_only ? (uint32_t)mlp0_params : (uint32_t)n_matrix();
		SlabJob sj;
		sj.slabs = slab; sj.n_slabs = blocks; sj.n = n_red; sj.grad = gradients; sj.stride = (uint32_t)n_matrix();
		sj.accumulate = grad_mode == NGP_GRAD_ACCUMULATE;
		FusedAdam f32store;
		if (fopt && fopt->g32) {
			// the sharded optimizer's input: the whole gradient stored widened to fp32 by the backward itself
			NGP_CHECK(fused && grad_mode == NGP_GRAD_OVERWRITE && !fopt->rec, "fp32 gradient store: fused slab reduction");
			sj.grad32 = fopt->g32;
			f32store.g32 = fopt->g32 + grid_offset();
			fopt = &f32store;
		}
		hipStream_t rs = s;
		if (ovl) {
			ensure_side_stream();
			NGP_HIP(hipEventRecord(ev_mlp, s));
			NGP_HIP(hipStreamWaitEvent(side, ev_mlp, 0));
			rs = side;
		}
		if (!fused) {
			ProfScope ps("reduce_slabs", rs);
			reduce_slabs(slab, blocks, n_red, gradients, grad_mode == NGP_GRAD_ACCUMULATE, rs, (uint32_t)n_matrix());
		}
		if (ovl) NGP_HIP(hipEventRecord(ev_red, side));
		GridBwdArgs b{n, in, stride, dL_denc, enc_width, AoS, gradients + grid_offset(), max_level, max_level_per_sample};
		FusedAdam fmlp;
		if (fopt && fopt->mlp_n) {
			// the MLP's update in the slab blocks (trainer: mlp_opt_in_backward): the fragment slots are written
			// in place when they hold the current parameters, as the optimizer launch would (run_step)
			NGP_CHECK(fused && grad_mode == NGP_GRAD_OVERWRITE && fopt->mlp_n == n_matrix(), "fused MLP update: slab reduction not fused");
			fmlp = *fopt;
			fmlp.frags = frags_current ? (f16*)frags.p : nullptr;
			fmlp.fragmap = d_fragmap;
			fopt = &fmlp;
		}
		scatter_grid_grad(s, b, grad_mode != NGP_GRAD_ACCUMULATE, fused ? &sj : nullptr, fopt);
		if (ovl) NGP_HIP(hipStreamWaitEvent(s, ev_red, 0));
		input_gradient();
	}
	// Hash-grid backward: destination-bucketed exact sums (n >= 4096, or mode 3), else tcnn-style direct
	// packed-f16 atomics (small batches, where the bucket plan costs more than the atomics).
	void scatter_grid_grad(hipStream_t s, GridBwdArgs b, bool overwrite, const SlabJob* slab = nullptr, const FusedAdam* fopt = nullptr) {
		if (use_sorted(b.n)) {
			void* ws = sorted_workspace(b.n);
			clear_brick_fallback(s, ws);
			if (sc_prepared) {
				NGP_HIP(hipStreamWaitEvent(s, ev_join, 0));
				sc_prepared = false;
			} else {
				ProfScope ps("grid_bwd_prepare", s);
				grid_scatter_prepare(grid, b, sc_plan, ws, s, sc_hist_done);
			}
			sc_hist_done = false;
			// _adam: with the grid's optimizer update
			ProfScope ps(fopt && fopt->rec ? "grid_backward_adam" : "grid_backward_sorted", s);
			grid_backward_sorted(grid, b, sc_plan, ws, s, overwrite, win_debug, slab, fopt,
			                     bwd_parts && !sc_plan.bk.LD && !(fopt && fopt->rec) ? bwd_parts : nullptr);
			return;
		}
		NGP_CHECK(!slab && !fopt, "fused slab reduction / optimizer need the sorted grid backward");
		if (overwrite) {
			ProfScope ps("grid_grad_zero", s);
			NGP_HIP(hipMemsetAsync(b.grad, 0, grid_params * sizeof(f16), s));
		}
		ProfScope ps("grid_backward", s);
		grid_backward(grid, b, s);
	}
};

struct ngp_trainer {
	ngp_model* model = nullptr;
	AdamConfig cfg;
	uint32_t step = 0;
	uint64_t n = 0;
	void* arena = nullptr;
	float *w32 = nullptr, *m1 = nullptr, *m2 = nullptr, *ema32 = nullptr;
	f16 *w16 = nullptr, *inf16 = nullptr, *g16 = nullptr;
	uint32_t* steps = nullptr;
	float* bias_tab = nullptr;  // adam_bias_table for cfg.beta1/beta2 (built at creation)
	// lazy-EMA layout (optimizer.h AdamRec), chosen for large tables: a step touches only the state of
	// updated parameters; the inference (EMA) parameters are brought up to date when read
	AdamRec* rec = nullptr;
	bool inf_stale = false;
	// lazy layout: the fp32 weights live in the records (AdamRec::w); w32 is their mirror, stale after a step
	bool w32_stale = false;
	void sync_w32() {
		if (!rec || !w32_stale) return;
		require_full_state("full-precision weights");
		NGP_HIP(hipDeviceSynchronize());  // the optimizer may still run on a caller's non-blocking stream
		adam_rec_weights((uint32_t)n, rec, w32, false, nullptr);
		NGP_HIP(hipDeviceSynchronize());
		w32_stale = false;
	}
	void materialize(hipStream_t s, bool force = false) {
		if (!rec || (!inf_stale && !force)) return;
		require_full_state("inference (EMA) parameters");
		AdamState st{w32, w16, g16, nullptr, nullptr, nullptr, nullptr, inf16, nullptr, nullptr, nullptr, 0, nullptr, rec};
		ema_materialize(cfg, (uint32_t)n, step, st, s);
		inf_stale = false;
	}
	static void materialize_hook(void* self, hipStream_t s) { ((ngp_trainer*)self)->materialize(s); }
	void bind_model() {
		ngp_model_set_params(model, w16, cfg.ema_decay > 0.f ? inf16 : w16, g16);
		if (rec) { model->inference_hook = materialize_hook; model->inference_hook_ctx = this; }
	}
	uint32_t* ctl = nullptr;  // device {optimizer step, block counter, .., AdamConfig at ctl + CTL_CFG}; `step` mirrors ctl[0]
	ngp_allreduce_fn allreduce = nullptr;  // gradient exchange inside captured steps (ngp_trainer_set_allreduce)
	void* allreduce_user = nullptr;
	uint32_t world = 1;
	// sharded optimizer (ngp_trainer_set_data_parallel): this rank, the fp32 gradient staging of the
	// reduce-scatter [n_pad] and the parameter count padded to a multiple of 8 world (w16 and the records
	// are allocated with SHARD_PAD spare parameters for it)
	static constexpr uint64_t SHARD_PAD = 2048;
	uint32_t dp_rank = 0;
	bool dp_rank_known = false;
	bool shard_opt = true;       // trainer option "shard_opt"
	bool shards_valid = true;    // false: a sharded step left other ranks' records stale here (gather_shards)
	float* g32 = nullptr;
	uint64_t g32_count = 0;
	uint64_t n_pad = 0;
	// The exchange in parameter parts (trainer option "dp_parts"): part j = parameters [pb[j], pb[j + 1]), multiples
	// of 8 world; rank r owns the r-th of the world equal slices of every part. Each part is reduce-scattered,
	// its slice updated and all-gathered as soon as the backward has summed it (BwdParts), on the exchange
	// stream xs, while the backward sums the next part. Default 1 part: measured at world 1 the parted
	// step costs 35-40 us more (the bucket ranges' own launches, and the step's graph runs the two streams' work in
	// sequence), more than the overlap could hide at N = 8 under DESIGN §7's bandwidth model.
	uint32_t dp_parts = 1;
	bool dp_wire16 = false;      // option "dp_wire16": reduce-scatter the fp16 gradient (half the bytes; rounded per hop)
	std::vector<uint64_t> pb;
	hipStream_t xs = nullptr;
	hipEvent_t ev_part[BwdParts::MAX] = {}, ev_xs = nullptr;
	struct PartStep {  // one sharded step's exchange state (issue_part)
		hipStream_t s = nullptr;
		ngp::Exchange e;
		float loss_scale = 1.f;
		const uint32_t* step_base = nullptr;
		uint32_t step_add = 0;
		bool wire16 = false, overlap = false;
		uint32_t issued = 0;
		int rc = NGP_OK;
	} ps_;
	BwdParts bparts;
	~ngp_trainer() {
		if (arena) (void)hipFree(arena);
		if (bias_tab) (void)hipFree(bias_tab);
		if (g32) (void)hipFree(g32);
		for (hipEvent_t ev : ev_part)
			if (ev) (void)hipEventDestroy(ev);
		if (ev_xs) (void)hipEventDestroy(ev_xs);
		if (xs) (void)hipStreamDestroy(xs);
	}
	ngp::Exchange exchange() const {
		ngp::Exchange e;
		e.fn = allreduce; e.user = allreduce_user; e.rank = dp_rank; e.world = world; e.world_factor = (float)world;
		e.rank_known = dp_rank_known;
		return e;
	}
	// the sharded optimizer applies to this exchange: the lazy layout owning the model's buffers, rank known
	bool sharded(const ngp::Exchange& e) const {
		return e.fn && e.rank_known && shard_opt && rec && g32 && e.world == world && model->params == w16 &&
		       model->gradients == g16 && !pb.empty();
	}
	void require_full_state(const char* what) const {
		if (!shards_valid)
			throw Error(std::string(what) + ": the optimizer state is sharded over the data-parallel ranks; call "
			            "ngp_trainer_gather_shards on every rank first");
	}
	// part bounds for `world` ranks: dp_parts parts of about n_pad / dp_parts, multiples of 8 world
	void make_part_bounds(uint32_t w) {
		const uint64_t q = 8ull * w;
		pb.assign(1, 0);
		for (uint32_t j = 1; j < dp_parts; ++j) {
			const uint64_t b = (n_pad * j / dp_parts) / q * q;
			if (b > pb.back() && b < n_pad) pb.push_back(b);
		}
		pb.push_back(n_pad);
	}
	void ensure_exchange_stream() {
		if (xs) return;
		// the exchange stream at the highest priority: a stream of the default priority may share a hardware queue
		// with the step's stream (GPU_MAX_HW_QUEUES), which would run its work in submission order, after the step's
		// next launches. NGP_XS_PRIORITY=0: the default priority (A/B)
		int lo = 0, hi = 0;
		NGP_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
		const char* e = getenv("NGP_XS_PRIORITY");
		NGP_HIP(hipStreamCreateWithPriority(&xs, hipStreamNonBlocking, e && atoi(e) == 0 ? 0 : hi));
		for (hipEvent_t& ev : ev_part) NGP_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
		NGP_HIP(hipEventCreateWithFlags(&ev_xs, hipEventDisableTiming));
	}
	// this rank's slice of part j, clamped to the parameters
	void part_slice(uint32_t j, uint64_t& lo, uint64_t& hi) const {
		const uint64_t c = (pb[j + 1] - pb[j]) / world;
		lo = std::min<uint64_t>(pb[j] + (uint64_t)dp_rank * c, n);
		hi = std::min<uint64_t>(lo + c, n);
	}
	// the MLP section lies in this rank's slice of part 0: the update keeps its weight fragments current
	bool mlp_owned() const {
		uint64_t lo, hi;
		part_slice(0, lo, hi);
		return lo == 0 && hi >= model->n_matrix();
	}
	// Exchange + update of part j (sharded step): reduce-scatter of the summed gradient, this rank's slice of the
	// records updated from the sums (fp32 wire: rounded to fp16 once, as the all-reduce path narrows; fp16 wire:
	// RCCL's per-hop fp16 sum), all-gather of the slice's fp16 weights. On xs behind an event when the backward
	// hands the parts over while it runs, else on the step's stream.
	void issue_part(uint32_t j) {
		PartStep& q = ps_;
		// parts go out from the last to the first (the order the parted backward finishes them), on every rank
		if (q.rc != NGP_OK || j + 1 >= pb.size() || j + 2 + q.issued != pb.size()) { q.rc = NGP_ERROR; return; }
		hipStream_t x = q.s;
		if (q.overlap) {
			NGP_HIP(hipEventRecord(ev_part[j], q.s));
			NGP_HIP(hipStreamWaitEvent(xs, ev_part[j], 0));
			x = xs;
		}
		const uint64_t a = pb[j], len = pb[j + 1] - pb[j];
		const ngp::Exchange& e = q.e;
		if (e.fn(e.user, q.wire16 ? (void*)(g16 + a) : (void*)(g32 + a), len, q.wire16 ? NGP_DTYPE_F16 : NGP_DTYPE_F32,
		         NGP_REDUCE_SCATTER_SUM, x) != NGP_OK) { q.rc = NGP_ERROR; return; }
		uint64_t lo, hi;
		part_slice(j, lo, hi);
		ngp_model* m = model;
		const bool mlp_here = lo == 0 && hi >= m->n_matrix();
		AdamState st{w32, w16, g16, nullptr, nullptr, nullptr, nullptr, inf16,
		             mlp_here && m->frags_current ? (f16*)m->frags.p : nullptr, m->d_fragmap, q.step_base, q.step_add,
		             q.step_base ? (const AdamConfig*)(ctl + CTL_CFG) : nullptr, rec, bias_tab, q.wire16 ? nullptr : g32};
		{
			ProfScope ps("optimizer", x);
			adam_lazy_range(cfg, (uint32_t)lo, (uint32_t)hi, (uint32_t)m->n_matrix(), q.loss_scale, st, x);
		}
		if (e.fn(e.user, w16 + a, len, NGP_DTYPE_F16, NGP_ALL_GATHER, x) != NGP_OK) { q.rc = NGP_ERROR; return; }
		++q.issued;
	}
	static void part_done(void* self, uint32_t j, hipStream_t) { ((ngp_trainer*)self)->issue_part(j); }
	// Before a sharded step's training pass: the exchange state, and the backward's parts when it can hand them
	// over (bucketed backward storing the fp32 gradient, or the fp16 one for the fp16 wire): returns them for
	// ngp_model::bwd_parts, or nullptr (then every part is exchanged after the backward).
	// stores_input: the backward writes the wire's input itself (fp32 wire: the fp32 store, FusedAdam::g32).
	const BwdParts* begin_shard_step(hipStream_t s, float loss_scale, const ngp::Exchange& e, const uint32_t* step_base,
	                                 uint32_t step_add, uint32_t n_batch, bool stores_input) {
		ps_ = PartStep{};
		ps_.s = s; ps_.e = e; ps_.loss_scale = loss_scale; ps_.step_base = step_base; ps_.step_add = step_add;
		ps_.wire16 = dp_wire16;
		ngp_model* m = model;
		if (pb.size() < 3 || !m->parts_ok(n_batch) || !(stores_input || dp_wire16)) return nullptr;
		ensure_exchange_stream();
		ps_.overlap = true;
		const ScatterPlan& p = m->sc_plan_for(n_batch);
		// the MLP's gradient (slab reduction with bucket range 0) must lie in part 0
		if (p.bk.LD || pb[1] < m->grid_offset()) { ps_.overlap = false; return nullptr; }
		bparts = BwdParts{};
		bparts.k = (uint32_t)pb.size() - 1;
		const uint64_t go = m->grid_offset();
		// range j ends at the bucket holding part j + 1's first parameter: that bucket is summed with range j + 1,
		// before part j + 1 goes out, so every part is final when its exchange starts
		for (uint32_t j = 0; j < bparts.k; ++j)
			bparts.vb_end[j] = j + 1 == bparts.k ? p.n_buckets : scatter_bucket_at_param(m->grid, p, pb[j + 1] > go ? pb[j + 1] - go : 0);
		bparts.after = part_done;
		bparts.user = this;
		return &bparts;
	}
	// After the training pass: the parts the backward did not hand over, the join of the exchange stream, the MLP's
	// fragments from the gathered weights where another rank updated them.
	int shard_step(bool stored) {
		PartStep& q = ps_;
		hipStream_t s = q.s;
		ngp_model* m = model;
		if (q.issued == 0) {
			q.overlap = false;  // nothing handed over (not the bucketed backward): every part here, on s
			if (!stored && !q.wire16) widen_f16(g16, g32, n, s);  // the backward did not write the fp32 input itself
		}
		while (q.rc == NGP_OK && q.issued + 1 < pb.size()) issue_part((uint32_t)pb.size() - 2 - q.issued);
		if (q.rc != NGP_OK) return NGP_ERROR;
		if (q.overlap) {
			NGP_HIP(hipEventRecord(ev_xs, xs));
			NGP_HIP(hipStreamWaitEvent(s, ev_xs, 0));
		}
		if (!mlp_owned() && m->n_matrix() > 0) m->prep(s, false);  // fragments of the gathered MLP weights
		inf_stale = w32_stale = true;
		if (q.e.world > 1) shards_valid = false;
		return NGP_OK;
	}
	void sync_device_step() { NGP_HIP(hipMemcpy(ctl, &step, sizeof(uint32_t), hipMemcpyHostToDevice)); }
	// One optimizer step on stream s. step_base/step_add: see AdamState (optimizer.h).
	// n_first: parameters [0, n_first) only (the MLP, when the grid's update ran fused in the backward)
	void run_step(hipStream_t s, float loss_scale, const uint32_t* step_base, uint32_t step_add, uint64_t n_first = 0) {
		ngp_model* m = model;
		const bool own = m->params == w16;
		// captured steps (step_base = ctl) read the hyperparameters from the ctl block, which every graph
		// launch refreshes with the step: set_learning_rate / set_option reach replayed steps too
		AdamState st{w32, w16, g16, m1, m2, steps, ema32, inf16,
		             own && m->frags_current ? (f16*)m->frags.p : nullptr, m->d_fragmap, step_base, step_add,
		             step_base ? (const AdamConfig*)(ctl + CTL_CFG) : nullptr, rec, bias_tab};
		ProfScope ps("optimizer", s);
		adam_ema_update(cfg, (uint32_t)(n_first ? n_first : n), (uint32_t)m->n_matrix(), loss_scale, st, s);
		if (rec) inf_stale = w32_stale = true;
	}
	// The grid's lazy update fused into the backward (model option fuse_opt): lazy layout, no gradient
	// exchange (the all-reduce needs the stored gradients), the sorted backward, F >= 2, and an MLP
	// section that is a whole number of 4-parameter groups (k_adam_lazy4 then runs on it alone).
	bool fused_update_ok(uint32_t n_batch) const {
		const ngp_model* m = model;
		return rec && !allreduce && m->fuse_opt && m->use_sorted(n_batch) && m->grid.n_features >= 2 && m->n_matrix() % 4 == 0 &&
		       m->grid_offset() % 2 == 0 && m->params == w16 && m->gradients == g16;
	}
	FusedAdam fused_update(float loss_scale, uint32_t n_batch) const {
		FusedAdam fa;
		const uint64_t go = model->grid_offset();
		fa.w16 = w16 + go; fa.rec = rec + go / 2;
		fa.loss_scale = loss_scale; fa.cfg = cfg; fa.step_add = step;
		fa.bias_tab = bias_tab;
		if (mlp_opt_in_backward(n_batch)) {
			fa.mlp_n = (uint32_t)model->n_matrix();
			fa.mlp_w16 = w16;
			fa.mlp_rec = rec;
		}
		return fa;
	}
	// With the grid's update fused (fused_update_ok), the MLP section's update runs in the dW slab blocks of
	// the grid backward's last kernel when the slab reduction is fused there (model options fuse_slabs,
	// fuse_mlp_opt; not under the side-stream reduction, overlap bit 4): no optimizer launch.
	bool mlp_opt_in_backward(uint32_t n_batch) const {
		const ngp_model* m = model;
		return m->fuse_mlp_opt && m->fuse_slabs && !(m->overlap & 4) && m->use_sorted(n_batch) && m->n_matrix() > 0;
	}
	void mlp_step_done() {  // run_step's bookkeeping when the update ran in the backward
		if (rec) inf_stale = w32_stale = true;
	}
};

// A captured training step (forward_backward + optimizer) replayed as one HIP graph launch.
struct ngp_graph {
	hipGraph_t graph = nullptr;
	hipGraphExec_t exec = nullptr;
	ngp_trainer* trainer = nullptr;
	uint32_t steps_per_launch = 1;
	uint64_t ws_epoch = 0;  // the model's workspace epoch at capture
	// the graph holds a sharded exchange over world > 1 ranks: every launch leaves the other ranks' optimizer
	// records stale on this rank again (ngp_trainer_gather_shards)
	bool shards_stale = false;
	// the graph's backward writes the gradient for the sharded exchange as fp32 only: g16 is not written
	bool g16_stale = false;
	void launched() {
		trainer->step += steps_per_launch;
		if (steps_per_launch && trainer->rec) trainer->inf_stale = trainer->w32_stale = true;
		if (shards_stale) trainer->shards_valid = false;
		if (g16_stale) trainer->model->grads_valid = false;
	}
	~ngp_graph() {
		if (exec) (void)hipGraphExecDestroy(exec);
		if (graph) (void)hipGraphDestroy(graph);
	}
};

// dL/doutput of tcnn's input_gradient: row `dim` of every sample = scale, every other row 0
__global__ static void k_one_hot_f16(f16* out, uint32_t n, uint32_t width, uint32_t dim, f16 v) {
	const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
	if (i < (uint64_t)n * width) out[i] = (i % width) == dim ? v : (f16)0.f;
}
static void fill_one_hot_f16(f16* out, uint32_t n, uint32_t width, uint32_t dim, float v, hipStream_t s) {
	k_one_hot_f16<<<div_round_up((uint64_t)n * width, 256), 256, 0, s>>>(out, n, width, dim, (f16)v);
	NGP_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

#define NGP_TRY(...)                        \
	try {                                   \
		__VA_ARGS__;                        \
		return NGP_OK;                      \
	} catch (const std::exception& e) {     \
		g_last_error = e.what();            \
		return NGP_ERROR;                   \
	}

#define NGP_ARG(cond)                                                          \
	do {                                                                       \
		if (!(cond)) { g_last_error = "invalid argument: " #cond; return NGP_INVALID; } \
	} while (0)

static hipStream_t S(void* s) { return (hipStream_t)s; }

namespace ngp {
void set_last_error(const char* msg) { g_last_error = msg; }
}  // namespace ngp

extern "C" {

const char* ngp_last_error(void) { return g_last_error.c_str(); }
const char* ngp_version(void) { return "ngp-mi355x 0.1 (gfx950)"; }

int ngp_device_info(int* cu_count, char* name, size_t name_len) {
	NGP_TRY({
		int dev = 0;
		NGP_HIP(hipGetDevice(&dev));
		hipDeviceProp_t p;
		NGP_HIP(hipGetDeviceProperties(&p, dev));
		if (cu_count) *cu_count = p.multiProcessorCount;
		if (name && name_len) { strncpy(name, p.gcnArchName, name_len - 1); name[name_len - 1] = 0; }
	});
}

int ngp_malloc(void** ptr, size_t bytes) { NGP_ARG(ptr); NGP_TRY(NGP_HIP(hipMalloc(ptr, bytes))); }
int ngp_free(void* ptr) { NGP_TRY(NGP_HIP(hipFree(ptr))); }
int ngp_memcpy(void* dst, const void* src, size_t bytes, int kind) { NGP_TRY(NGP_HIP(hipMemcpy(dst, src, bytes, (hipMemcpyKind)kind))); }
int ngp_stream_synchronize(void* stream) { NGP_TRY(NGP_HIP(hipStreamSynchronize(S(stream)))); }

// NGP_MODEL_OPTS="key=value,key=value": engine options applied to every model at creation (A/B runs of whole
// programs, tools/ab.sh); an unknown key or a bad value fails the creation
static void apply_env_options(ngp_model* m) {
	const char* env = getenv("NGP_MODEL_OPTS");
	if (!env || !*env) return;
	std::string all = env;
	size_t pos = 0;
	while (pos < all.size()) {
		size_t end = all.find(',', pos);
		if (end == std::string::npos) end = all.size();
		const std::string kv = all.substr(pos, end - pos);
		pos = end + 1;
		if (kv.empty()) continue;
		const size_t eq = kv.find('=');
		NGP_CHECK(eq != std::string::npos, "NGP_MODEL_OPTS: expected key=value, got " + kv);
		if (ngp_model_set_option(m, kv.substr(0, eq).c_str(), atof(kv.c_str() + eq + 1)) != NGP_OK) throw Error(g_last_error);
	}
}

int ngp_nerf_network_create(uint32_t n_pos_dims, uint32_t n_dir_dims, uint32_t n_extra_dims, uint32_t dir_offset,
                            const char* pos_encoding_json, const char* dir_encoding_json, const char* density_network_json,
                            const char* rgb_network_json, ngp_model** out) {
	NGP_ARG(out && pos_encoding_json && density_network_json && rgb_network_json);
	NGP_TRY({
		auto m = std::make_unique<ngp_model>();
		m->nerf = true;
		NGP_CHECK(n_pos_dims == 3, "NerfNetwork: n_pos_dims must be 3");
		NGP_CHECK(n_dir_dims == 3, "NerfNetwork: n_dir_dims must be 3");
		NGP_CHECK(n_extra_dims == 0, "NerfNetwork: extra dims (latent codes) are not implemented");
		m->n_pos_dims = n_pos_dims; m->n_dir_dims = n_dir_dims; m->n_extra_dims = n_extra_dims; m->dir_offset = dir_offset;
		m->grid = parse_grid(3, Json::parse(pos_encoding_json));
		if (dir_encoding_json) {
			Json d = Json::parse(dir_encoding_json);
			const Json* sh = &d;
			if (iequals(d.string_or("otype", ""), "Composite")) sh = &d["nested"].arr.at(0);
			NGP_CHECK(iequals(sh->string_or("otype", ""), "SphericalHarmonics") && (int)sh->number_or("degree", 4) == 4,
			          "NerfNetwork: dir_encoding must be SphericalHarmonics of degree 4");
		}
		uint32_t wd, wr;
		const uint32_t dh = parse_mlp_hidden(Json::parse(density_network_json), &wd);
		const uint32_t rh = parse_mlp_hidden(Json::parse(rgb_network_json), &wr);
		NGP_CHECK(wd == wr, "NerfNetwork: density and rgb networks must share n_neurons");
		m->enc_width = next_multiple(m->grid.n_levels * m->grid.n_features, 16);
		m->nplan = make_nerf_mlp_plan(m->enc_width, wd, dh, rh);
		m->mlp0_params = m->nplan.density.n_params();
		m->mlp1_params = m->nplan.rgb.n_params();
		m->n_input_dims = dir_offset + n_dir_dims + n_extra_dims;
		m->n_output_dims = 4;
		m->finalize();
		apply_env_options(m.get());
		*out = m.release();
	});
}

int ngp_network_with_input_encoding_create(uint32_t n_input_dims, uint32_t n_output_dims, const char* encoding_json,
                                           const char* network_json, ngp_model** out) {
	NGP_ARG(out && encoding_json && network_json);
	NGP_TRY({
		auto m = std::make_unique<ngp_model>();
		m->nerf = false;
		NGP_CHECK(n_input_dims == 2 || n_input_dims == 3, "NetworkWithInputEncoding: 2 or 3 input dims");
		NGP_CHECK(n_output_dims >= 1 && n_output_dims <= 16, "NetworkWithInputEncoding: 1..16 outputs");
		m->n_pos_dims = n_input_dims; m->n_input_dims = n_input_dims; m->n_output_dims = n_output_dims;
		m->grid = parse_grid(n_input_dims, Json::parse(encoding_json));
		uint32_t w;
		const uint32_t hid = parse_mlp_hidden(Json::parse(network_json), &w);
		m->enc_width = next_multiple(m->grid.n_levels * m->grid.n_features, 16);
		m->mplan = make_mlp_plan(m->enc_width, w, hid, 16);
		m->mlp0_params = m->mplan.mlp.n_params();
		m->mlp1_params = 0;
		m->finalize();
		apply_env_options(m.get());
		*out = m.release();
	});
}

void ngp_model_destroy(ngp_model* m) { delete m; }
uint64_t ngp_model_n_params(const ngp_model* m) { return m ? m->n_params : 0; }
uint64_t ngp_model_n_matrix_params(const ngp_model* m) { return m ? m->n_matrix() : 0; }
uint32_t ngp_model_input_width(const ngp_model* m) { return m ? m->n_input_dims : 0; }
uint32_t ngp_model_padded_output_width(const ngp_model* m) { return m ? 16 : 0; }
uint32_t ngp_model_output_width(const ngp_model* m) { return m ? m->n_output_dims : 0; }

int ngp_model_param_layout(const ngp_model* m, ngp_param_layout* o) {
	NGP_ARG(m && o);
	NGP_TRY({
		memset(o, 0, sizeof(*o));
		o->density_mlp_offset = 0; o->density_mlp_params = m->mlp0_params;
		o->rgb_mlp_offset = m->mlp0_params; o->rgb_mlp_params = m->mlp1_params;
		o->grid_offset = m->grid_offset(); o->grid_params = m->grid_params;
		o->grid_dims = m->grid.n_dims; o->grid_levels = m->grid.n_levels; o->grid_features = m->grid.n_features;
		o->grid_log2_hashmap = m->grid.log2_hashmap; o->grid_base_resolution = m->grid.base_resolution;
		o->grid_per_level_scale = m->grid.per_level_scale;
		memcpy(o->grid_level_offsets, m->grid.offsets, sizeof(o->grid_level_offsets));
		memcpy(o->grid_resolution, m->grid.resolution, sizeof(o->grid_resolution));
		memcpy(o->grid_scale, m->grid.scale, sizeof(o->grid_scale));
		o->encoding_width = m->enc_width;
	});
}

int ngp_model_set_params(ngp_model* m, void* params, void* inference_params, void* gradients) {
	NGP_ARG(m);
	NGP_TRY({
		m->inference_hook = nullptr;  // a trainer that binds its own buffers installs its hook afterwards
		m->inference_hook_ctx = nullptr;
		m->params = (f16*)params;
		m->frags_current = false;
		m->inference_params = (f16*)(inference_params ? inference_params : params);
		m->gradients = (f16*)gradients;
	});
}

int ngp_model_initialize_params(const ngp_model* m, uint64_t seed, float* p, float scale) {
	NGP_ARG(m && p);
	NGP_TRY({
		Pcg32 rng(seed);
		if (m->nerf) {
			init_mlp(m->nplan.density, rng, p, scale);
			init_mlp(m->nplan.rgb, rng, p + m->mlp0_params, scale);
		} else {
			init_mlp(m->mplan.mlp, rng, p, scale);
		}
		rng.uniform(m->grid_params, p + m->grid_offset(), -1e-4f * scale, 1e-4f * scale);
	});
}

int ngp_model_set_max_level(ngp_model* m, float max_level, const float* per_sample) {
	NGP_ARG(m);
	NGP_TRY({ m->max_level = max_level; m->max_level_per_sample = per_sample; });
}

int ngp_model_set_option(ngp_model* m, const char* key, double value) {
	NGP_ARG(m && key);
	NGP_TRY({
		const std::string k = key;
		if (k == "grid_backward_mode") {
			NGP_CHECK(value == 0 || value == 1 || value == 3, "grid_backward_mode must be 0 (auto), 1 (direct), 3 (bucketed)");
			m->grid_backward_mode = (int)value;
		} else if (k == "overlap") {
			NGP_CHECK(value >= 0 && value <= 15, "overlap is a bitmask in [0, 15]");
			m->overlap = (uint32_t)value;
		} else if (k == "fused_hist") {
			m->fused_hist = value != 0;
		} else if (k == "fuse_infer") {
			m->fuse_infer = value != 0;
		} else if (k == "fuse_slabs") {
			m->fuse_slabs = value != 0;
		} else if (k == "fuse_opt") {
			m->fuse_opt = value != 0;
		} else if (k == "fuse_mlp_opt") {
			m->fuse_mlp_opt = value != 0;
		} else if (k == "grid_bricks") {
			m->grid_bricks = value != 0;
			m->sc_plan_n = 0;  // re-plan at the next batch
		} else if (k == "win_debug") {
			m->win_debug = (uint32_t)value;
		} else {
			throw Error("unknown model option: " + k);
		}
		// a graph captured before the change launches the old kernels: mark it stale (the NeRF trainer re-captures,
		// ngp_graph_launch of a caller's graph fails loudly)
		++m->ws_epoch;
	});
}

int ngp_model_query(const ngp_model* m, const char* key, double* value) {
	NGP_ARG(m && key && value);
	NGP_TRY({
		const std::string k = key;
		if (k == "grid_brick_levels") *value = m->sc_plan_n ? (double)(m->sc_plan.bk.LD - m->sc_plan.bk.LB) : 0.0;
		else throw Error("unknown model query: " + k);
	});
}

int ngp_model_reserve(ngp_model* m, uint32_t n) {
	NGP_ARG(m);
	NGP_TRY({ m->reserve(n); });
}

uint64_t ngp_model_workspace_epoch(const ngp_model* m) { return m ? m->ws_epoch : 0; }

int ngp_model_workspace(ngp_model* m, const char* name, void** ptr, uint64_t* bytes) {
	NGP_ARG(m && name && ptr);
	NGP_TRY({
		const std::string k(name);
		DevBuf* b = k == "encoding" ? &m->enc : k == "dL_dencoding" ? &m->denc : k == "dw_slabs" ? &m->slabs
		          : k == "dL_dsh" ? &m->dsh_ws : nullptr;
		NGP_CHECK(b, "ngp_model_workspace: unknown workspace '" + k + "' (encoding, dL_dencoding, dL_dsh, dw_slabs)");
		*ptr = b->p;
		if (bytes) *bytes = b->bytes;
	});
}

int ngp_encoding_forward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                         uint32_t output_stride, uint32_t output_layout, int use_inference_params) {
	NGP_ARG(m && (n == 0 || (input && output)) && output_layout <= 1);
	NGP_TRY({
		m->require_params(use_inference_params);
		m->encode(S(stream), n, input, input_stride, (f16*)output, output_stride, output_layout, use_inference_params);
	});
}

int ngp_encoding_backward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                          const void* dL_doutput, uint32_t dL_stride, uint32_t dL_layout, float* dL_dinput,
                          uint32_t dL_dinput_stride, int grad_mode) {
	NGP_ARG(m && (n == 0 || (input && dL_doutput)) && dL_layout <= 1 && grad_mode >= 0 && grad_mode <= NGP_GRAD_IGNORE);
	NGP_ARG(!dL_dinput || (dL_layout == NGP_LAYOUT_AOS && dL_dinput_stride >= m->grid.n_dims));
	NGP_TRY({
		if (n == 0) return NGP_OK;
		m->require_params(false);
		if (grad_mode != NGP_GRAD_IGNORE) {
			NGP_CHECK(m->gradients, "model has no gradient buffer");
			GridBwdArgs b{n, input, input_stride, (const f16*)dL_doutput, dL_stride, dL_layout, m->gradients + m->grid_offset(),
			              m->max_level, m->max_level_per_sample};
			m->scatter_grid_grad(S(stream), b, grad_mode != NGP_GRAD_ACCUMULATE);
		}
		// last: dL_dinput may alias the input, which the parameter backward above still reads
		if (dL_dinput) {
			ProfScope ps("input_gradient", S(stream));
			InputGradArgs ia{n, input, input_stride, m->params + m->grid_offset(), (const f16*)dL_doutput, dL_stride, m->max_level,
			                 m->max_level_per_sample, nullptr, 0, dL_dinput, dL_dinput_stride, 1.f};
			grid_input_gradient(m->grid, ia, S(stream));
		}
	});
}

}  // extern "C"
// NerfNetwork::density (ngp_density's body): the density network's output rows in `output_layout` (AoS, SoA, or
// MLP_LAYOUT_ROW0 for the density grid update, which reads row 0 only).
int ngp::density_impl(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                      uint32_t output_stride, uint32_t output_layout, int use_inference_params) {
	NGP_TRY({
		NGP_CHECK(m->nerf, "density() is a NerfNetwork method");
		if (n == 0) return NGP_OK;
		m->require_params(use_inference_params);
		f16* e = (f16*)m->enc.get((size_t)n * m->enc_width * sizeof(f16));
		m->encode(S(stream), n, input, input_stride, e, m->enc_width, AoS, use_inference_params);
		m->run_mlp(S(stream), MLP_DENSITY, n, input, input_stride, e, (f16*)output, output_stride, output_layout, nullptr, 0,
		           nullptr, nullptr, use_inference_params);
		m->generation++;
	});
}
extern "C" {

int ngp_inference(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                  uint32_t output_stride, uint32_t output_layout, int use_inference_params) {
	NGP_ARG(m && (n == 0 || (input && output)) && (output_layout <= 1 || (output_layout == NGP_LAYOUT_AOS_RGBD && m->nerf &&
	                                                                        output_stride >= 4)));
	NGP_TRY({
		if (n == 0) return NGP_OK;
		m->require_params(use_inference_params);
		if (m->fused_inference_ok()) {
			// the encoding never reaches HBM: the MLP kernel gathers and blends the grid levels itself
			m->run_mlp(S(stream), MLP_INFER_ENC, n, input, input_stride, nullptr, (f16*)output, output_stride, output_layout,
			           nullptr, 0, nullptr, nullptr, use_inference_params);
		} else {
			f16* e = (f16*)m->enc.get((size_t)n * m->enc_width * sizeof(f16));
			m->encode(S(stream), n, input, input_stride, e, m->enc_width, AoS, use_inference_params);
			m->run_mlp(S(stream), MLP_INFER, n, input, input_stride, e, (f16*)output, output_stride, output_layout, nullptr, 0,
			           nullptr, nullptr, use_inference_params);
		}
		m->generation++;
	});
}

int ngp_density(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                uint32_t output_stride, uint32_t output_layout, int use_inference_params) {
	NGP_ARG(m && (n == 0 || (input && output)) && output_layout <= 1);
	return ngp::density_impl(m, stream, n, input, input_stride, output, output_stride, output_layout, use_inference_params);
}

int ngp_forward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                uint32_t output_stride, int use_inference_params, ngp_ctx** ctx) {
	NGP_ARG(m && ctx && (n == 0 || input));
	NGP_TRY({
		m->require_params(use_inference_params);
		f16* e = (f16*)m->enc.get((size_t)(n ? n : 1) * m->enc_width * sizeof(f16));
		m->generation++;
		if (n) {
			m->encode(S(stream), n, input, input_stride, e, m->enc_width, AoS, use_inference_params);
			if (output)
				m->run_mlp(S(stream), MLP_INFER, n, input, input_stride, e, (f16*)output, output_stride, AoS, nullptr, 0, nullptr,
				           nullptr, use_inference_params);
		}
		*ctx = new ngp_ctx{n, input, input_stride, (bool)use_inference_params, m->generation};
	});
}

static int check_dinput(const ngp_model* m, float* dL_dinput, uint32_t stride) {
	if (!dL_dinput) return NGP_OK;
	const uint32_t need = m->nerf ? m->dir_offset + 3 : m->n_pos_dims;
	if (stride < need) {
		g_last_error = "dL_dinput: stride smaller than the rows the input gradient writes";
		return NGP_INVALID;
	}
	return NGP_OK;
}

int ngp_backward(ngp_model* m, void* stream, ngp_ctx* ctx, const void* dL_doutput, uint32_t dL_stride, float* dL_dinput,
                 uint32_t dL_dinput_stride, int grad_mode) {
	NGP_ARG(m && ctx && (ctx->n == 0 || dL_doutput) && grad_mode >= 0 && grad_mode <= NGP_GRAD_IGNORE);
	if (check_dinput(m, dL_dinput, dL_dinput_stride) != NGP_OK) return NGP_INVALID;
	NGP_TRY({
		NGP_CHECK(ctx->generation == m->generation,
		          "backward: the forward context is stale (another forward/inference ran on this model since)");
		NGP_CHECK(!ctx->density_only, "backward: this context is from density_forward (use density_backward)");
		if (ctx->n == 0) return NGP_OK;
		BwdExtra ex;
		ex.dL_dinput = dL_dinput; ex.dinput_stride = dL_dinput_stride;
		ex.inference = ctx->use_inference_params;  // backward_impl passes use_inference_params to every sub-backward
		m->train_pass(S(stream), ctx->n, ctx->input, ctx->input_stride, (const f16*)m->enc.p, nullptr, 0, dL_doutput, dL_stride,
		              grad_mode, ex);
	});
}

int ngp_density_forward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                        uint32_t output_stride, int use_inference_params, ngp_ctx** ctx) {
	NGP_ARG(m && ctx && (n == 0 || input) && (!output || output_stride >= 16));
	NGP_TRY({
		NGP_CHECK(m->nerf, "density_forward is a NerfNetwork method");
		m->require_params(use_inference_params);
		f16* e = (f16*)m->enc.get((size_t)(n ? n : 1) * m->enc_width * sizeof(f16));
		m->generation++;
		if (n) {
			m->encode(S(stream), n, input, input_stride, e, m->enc_width, AoS, use_inference_params);
			if (output)
				m->run_mlp(S(stream), MLP_DENSITY, n, input, input_stride, e, (f16*)output, output_stride, AoS, nullptr, 0, nullptr,
				           nullptr, use_inference_params);
		}
		*ctx = new ngp_ctx{n, input, input_stride, (bool)use_inference_params, m->generation, true};
	});
}

int ngp_density_backward(ngp_model* m, void* stream, ngp_ctx* ctx, const void* dL_doutput, uint32_t dL_stride, float* dL_dinput,
                         uint32_t dL_dinput_stride, int grad_mode) {
	NGP_ARG(m && ctx && (ctx->n == 0 || dL_doutput) && dL_stride >= 16 && dL_stride % 4 == 0 && grad_mode >= 0 &&
	        grad_mode <= NGP_GRAD_IGNORE && (!dL_dinput || dL_dinput_stride >= 3));
	NGP_TRY({
		NGP_CHECK(m->nerf, "density_backward is a NerfNetwork method");
		NGP_CHECK(ctx->generation == m->generation,
		          "density_backward: the forward context is stale (another forward/inference ran on this model since)");
		NGP_CHECK(ctx->density_only, "density_backward: this context is from forward (use backward)");
		if (ctx->n == 0) return NGP_OK;
		BwdExtra ex;
		ex.dL_dinput = dL_dinput; ex.dinput_stride = dL_dinput_stride;
		ex.density_only = true; ex.ddens = (const f16*)dL_doutput; ex.ddens_stride = dL_stride;
		ex.inference = ctx->use_inference_params;
		m->train_pass(S(stream), ctx->n, ctx->input, ctx->input_stride, (const f16*)m->enc.p, nullptr, 0, nullptr, 0, grad_mode, ex);
	});
}

int ngp_input_gradient(ngp_model* m, void* stream, uint32_t dim, uint32_t n, const float* input, uint32_t input_stride,
                       float* d_dinput, uint32_t d_dinput_stride, float backprop_scale) {
	NGP_ARG(m && (n == 0 || (input && d_dinput)) && dim < 16 && backprop_scale != 0.f);
	if (check_dinput(m, d_dinput, d_dinput_stride) != NGP_OK) return NGP_INVALID;
	NGP_TRY({
		if (n == 0) return NGP_OK;
		m->require_params(false);
		hipStream_t s = S(stream);
		f16* e = (f16*)m->enc.get((size_t)n * m->enc_width * sizeof(f16));
		f16* dl = (f16*)m->dl1_ws.get((size_t)n * 16 * sizeof(f16));
		m->generation++;
		m->encode(s, n, input, input_stride, e, m->enc_width, AoS, false);
		// one-hot dL/doutput: row `dim` = backprop_scale (fp16), every other row 0
		fill_one_hot_f16(dl, n, 16, dim, backprop_scale, s);
		BwdExtra ex;
		ex.dL_dinput = d_dinput; ex.dinput_stride = d_dinput_stride; ex.dinput_scale = 1.f / backprop_scale;
		m->train_pass(s, n, input, input_stride, e, nullptr, 0, dl, 16, NGP_GRAD_IGNORE, ex);
	});
}

void ngp_ctx_destroy(ngp_ctx* ctx) { delete ctx; }

int ngp_forward_backward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                         uint32_t output_stride, const void* dL_doutput, uint32_t dL_stride, int grad_mode) {
	return ngp::forward_backward_with(m, stream, n, input, input_stride, output, output_stride, dL_doutput, dL_stride, grad_mode,
	                                  nullptr);
}
}  // extern "C"

// ngp_forward_backward, optionally with the grid's lazy optimizer update fused into the backward (fopt:
// captured training steps, ngp_trainer_fused_update)
int ngp::forward_backward_with(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                               uint32_t output_stride, const void* dL_doutput, uint32_t dL_stride, int grad_mode,
                               const FusedAdam* fopt) {
	NGP_ARG(m && (n == 0 || (input && dL_doutput)));
	NGP_TRY({
		if (n == 0) return NGP_OK;
		m->require_params(false);
		f16* e = (f16*)m->enc.get((size_t)n * m->enc_width * sizeof(f16));
		m->generation++;
		m->prepare_grid_backward_async(S(stream), n, input, input_stride);
		m->encode(S(stream), n, input, input_stride, e, m->enc_width, AoS, false, true);
		m->train_pass(S(stream), n, input, input_stride, e, (f16*)output, output_stride, dL_doutput, dL_stride, grad_mode,
		              BwdExtra{}, fopt);
	});
}
extern "C" {

// ---- trainer ------------------------------------------------------------------------------
static void parse_optimizer(const Json& j, AdamConfig& c) {
	const std::string ot = j.string_or("otype", "Adam");
	if (iequals(ot, "Ema")) {
		c.ema_decay = (float)j.number_or("decay", 0.99);
		parse_optimizer(j["nested"], c);
	} else if (iequals(ot, "ExponentialDecay")) {
		c.decay_start = (uint32_t)j.number_or("decay_start", 0);
		c.decay_interval = (uint32_t)j.number_or("decay_interval", 10000);
		c.decay_base = (float)j.number_or("decay_base", 0.1);
		parse_optimizer(j["nested"], c);
	} else if (iequals(ot, "Adam")) {
		c.lr = (float)j.number_or("learning_rate", 1e-3);
		c.beta1 = (float)j.number_or("beta1", 0.9);
		c.beta2 = (float)j.number_or("beta2", 0.999);
		c.eps = (float)j.number_or("epsilon", 1e-8);
		c.l2 = (float)j.number_or("l2_reg", 1e-8);
	} else {
		throw Error("optimizer: unsupported otype " + ot + " (Ema / ExponentialDecay / Adam implemented)");
	}
}

int ngp_trainer_create(ngp_model* m, const char* optimizer_json, uint64_t seed, ngp_trainer** out) {
	NGP_ARG(m && out);
	NGP_TRY({
		auto t = std::make_unique<ngp_trainer>();
		t->model = m;
		if (optimizer_json) parse_optimizer(Json::parse(optimizer_json), t->cfg);
		if (const char* e = getenv("NGP_EMA_CLOSED_FORM")) t->cfg.ema_closed_form = atoi(e) != 0;  // A/B runs
		// the betas are fixed for the trainer's lifetime (only the learning rate has a setter)
		NGP_HIP(hipMalloc(&t->bias_tab, (size_t)BIAS_TAB_CAP * 2 * sizeof(float)));
		adam_bias_table(t->bias_tab, t->cfg.beta1, t->cfg.beta2, nullptr);
		NGP_HIP(hipDeviceSynchronize());
		const uint64_t n = m->n_params;
		t->n = n;
		auto al = [](size_t b) { return (b + 255) / 256 * 256; };
		// w16 and the records carry SHARD_PAD spare parameters: the sharded optimizer pads to a multiple of 8 world
		const size_t b32 = al(n * 4), b16 = al((n + ngp_trainer::SHARD_PAD) * 2);
		// lazy-EMA records from 2^20 parameters (C5: 105 M parameters, ~28 % updated per step; C2' 13 M: captured
		// step 351 -> 330 us with the fused update, profiles/r03bw; C2, 3.3 M parameters, ~96 % updated: pass
		// 140.6-142.8 -> 136.0 us since the MLP's update runs in the backward, NeRF steps unchanged with the
		// EMA's closed-form catch-up, gpurun_out/r04cg); the eager arrays for small models. NGP_LAZY_EMA=0/1
		// forces the choice.
		bool lazy = n >= (1ull << 20);
		if (const char* e = getenv("NGP_LAZY_EMA")) lazy = atoi(e) != 0;
		lazy = lazy && n % 4 == 0;
		const size_t brec = al((n + ngp_trainer::SHARD_PAD) / 2 * sizeof(AdamRec));
		const size_t total = b32 + (lazy ? brec : 4 * b32) + 3 * b16 + 256 /*ctl*/;
		NGP_HIP(hipMalloc(&t->arena, total));
		char* p = (char*)t->arena;
		t->w32 = (float*)p; p += b32;
		if (lazy) {
			t->rec = (AdamRec*)p; p += brec;
		} else {
			t->m1 = (float*)p; p += b32;
			t->m2 = (float*)p; p += b32;
			t->ema32 = (float*)p; p += b32;
			t->steps = (uint32_t*)p; p += b32;
		}
		t->w16 = (f16*)p; p += b16;
		t->inf16 = (f16*)p; p += b16;
		t->g16 = (f16*)p; p += b16;
		t->ctl = (uint32_t*)p; p += 256;
		NGP_HIP(hipMemset(t->arena, 0, total));
		std::vector<float> host(n);
		if (ngp_model_initialize_params(m, seed, host.data(), 1.0f) != NGP_OK) throw Error(g_last_error);
		*out = t.release();
		if (ngp_trainer_set_params_full_precision(*out, host.data(), n) != NGP_OK) throw Error(g_last_error);
	});
}

void ngp_trainer_destroy(ngp_trainer* t) {
	if (!t) return;
	if (t->model && t->model->params == t->w16) ngp_model_set_params(t->model, nullptr, nullptr, nullptr);
	delete t;
}

int ngp_trainer_optimizer_step(ngp_trainer* t, void* stream, float loss_scale) {
	NGP_ARG(t && loss_scale > 0.f);
	NGP_TRY({
		t->run_step(S(stream), loss_scale, nullptr, t->step);
		t->step++;
	});
}

int ngp_loss_evaluate(int loss_type, void* stream, uint32_t n, uint32_t dims, const void* output, uint32_t output_stride,
                      const float* target, uint32_t target_stride, float loss_scale, void* dL_doutput, uint32_t dL_stride,
                      float* values, float* loss_sum) {
	NGP_ARG(loss_type >= 0 && (n == 0 || (output && target && dL_doutput)));
	NGP_TRY({
		LossEvalArgs a{n, dims, (const f16*)output, output_stride, target, target_stride, loss_scale, (f16*)dL_doutput, dL_stride,
		               values, loss_sum};
		loss_evaluate((uint32_t)loss_type, a, S(stream));
	});
}

// tcnn::Trainer::training_step(stream, input, target, data_pdf = nullptr, run_optimizer)
// (src/testbed_image.cu:276, src/testbed_sdf.cu:1304): forward -> loss -> backward [-> optimizer].
// The fused MLP kernel needs dL/doutput up front, so the forward runs once as inference (output for
// the loss) and once more inside the backward (recompute instead of stored activations).
int ngp_trainer_training_step(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                              const float* target, uint32_t target_stride, int loss_type, float loss_scale, int run_optimizer,
                              float* loss_sum) {
	NGP_ARG(t && (n == 0 || (input && target)) && loss_scale > 0.f && loss_type >= 0);
	NGP_TRY({
		if (n == 0) return NGP_OK;
		ngp_model* m = t->model;
		m->require_params(false);
		NGP_CHECK(m->gradients == t->g16, "training_step: the model's gradient buffer must be this trainer's");
		hipStream_t s = S(stream);
		const uint32_t W = 16;  // padded_output_width (nerf_network.h:463-465; FullyFusedMLP pads to 16)
		f16* e = (f16*)m->enc.get((size_t)n * m->enc_width * sizeof(f16));
		f16* out = (f16*)m->out_ws.get((size_t)n * W * sizeof(f16));
		f16* dl = (f16*)m->dl_ws.get((size_t)n * W * sizeof(f16));
		m->generation++;
		m->encode(s, n, input, input_stride, e, m->enc_width, AoS, false, true);
		m->run_mlp(s, MLP_INFER, n, input, input_stride, e, out, W, AoS, nullptr, 0, nullptr, nullptr, false);
		LossEvalArgs la{n, m->n_output_dims, out, W, target, target_stride, loss_scale, dl, W, nullptr, loss_sum};
		{
			ProfScope ps("loss", s);
			loss_evaluate((uint32_t)loss_type, la, s);
		}
		// the grid's optimizer update runs inside the backward where possible (fused_update_ok): its
		// gradient is then not stored, and the optimizer launch covers the MLP section alone
		const bool fuse = run_optimizer && t->fused_update_ok(n);
		const FusedAdam fa = fuse ? t->fused_update(loss_scale, n) : FusedAdam{};
		m->train_pass(s, n, input, input_stride, e, nullptr, 0, dl, W, NGP_GRAD_OVERWRITE, BwdExtra{}, fuse ? &fa : nullptr);
		if (run_optimizer) {
			if (fa.mlp_n) t->mlp_step_done();
			else t->run_step(s, loss_scale, nullptr, t->step, fuse ? m->n_matrix() : 0);
			t->step++;
		}
	});
}

int ngp_trainer_capture_training_step(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                                      const void* dL_doutput, uint32_t dL_stride, float loss_scale, uint32_t n_steps,
                                      int with_optimizer, ngp_graph** out) {
	NGP_ARG(t);
	return ngp::capture_training_step_with(t, stream, n, input, input_stride, dL_doutput, dL_stride, loss_scale, n_steps,
	                                       with_optimizer, t->exchange(), out);
}
}  // extern "C"

// One training step as the captured graph runs it: forward_backward (the grid's lazy update fused into the
// backward when `fuse`), [gradient exchange: one all-reduce, or the sharded reduce-scatter / slice update /
// all-gather], optimizer. step_base = the trainer's ctl block (captured: the step is the device base + k,
// hyperparameters read from the ctl block) or nullptr (eager: host step + k).
static int train_step_body(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                           const void* dL_doutput, uint32_t dL_stride, float loss_scale, int with_optimizer,
                           const Exchange& ex, bool fuse, const uint32_t* step_base, uint32_t k) {
	ngp_model* m = t->model;
	FusedAdam fa;
	if (fuse) {
		fa = t->fused_update(loss_scale * ex.world_factor, n);
		if (step_base) {
			fa.step_base = step_base;
			fa.step_add = k;
			fa.cfg_dev = (const AdamConfig*)(t->ctl + CTL_CFG);
		} else {
			fa.step_add = t->step + k;
		}
	}
	const bool shard = with_optimizer && t->sharded(ex);
	// sharded: the backward writes the fp32 reduce-scatter input itself where it can (no widening pass); with the
	// fp16 wire it stores the fp16 gradient as usual
	const bool direct32 = shard && !t->dp_wire16 && m->grad32_ok(n);
	if (direct32) fa.g32 = t->g32;
	int rc = NGP_OK;
	if (shard) {
		try {
			// the exchange of each part starts as soon as the backward has summed it (BwdParts)
			m->bwd_parts = t->begin_shard_step(S(stream), loss_scale * ex.world_factor, ex, step_base, step_base ? k : t->step + k,
			                                   n, direct32);
		} catch (const std::exception& e) {
			g_last_error = e.what();
			rc = NGP_ERROR;
		}
	}
	if (rc == NGP_OK)
		rc = forward_backward_with(m, stream, n, input, input_stride, nullptr, 0, dL_doutput, dL_stride, NGP_GRAD_OVERWRITE,
		                           fuse || direct32 ? &fa : nullptr);
	m->bwd_parts = nullptr;
	if (rc == NGP_OK && ex.fn) {
		try {
			// the summed gradient of the ranks: the mean (or, NeRF, the 1-GPU gradient) via the loss scale
			rc = shard ? t->shard_step(direct32) : ex.fn(ex.user, t->g16, t->n, NGP_DTYPE_F16, NGP_REDUCE_SUM, stream);
		} catch (const std::exception& e) {
			g_last_error = e.what();
			rc = NGP_ERROR;
		}
		if (rc != NGP_OK && g_last_error.empty()) g_last_error = "gradient exchange failed";
	}
	if (rc == NGP_OK && with_optimizer && !shard) {
		try {
			if (fa.mlp_n) t->mlp_step_done();
			else t->run_step(S(stream), loss_scale * ex.world_factor, step_base, step_base ? k : t->step + k,
			                 fuse ? m->n_matrix() : 0);
		} catch (const std::exception& e) {
			g_last_error = e.what();
			rc = NGP_ERROR;
		}
	}
	return rc;
}

int ngp::train_step_with(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                         const void* dL_doutput, uint32_t dL_stride, float loss_scale, const Exchange& ex) {
	NGP_ARG(t && n > 0 && input && dL_doutput && loss_scale > 0.f);
	NGP_TRY({
		ngp_model* m = t->model;
		m->require_params(false);
		NGP_CHECK(m->gradients == t->g16, "train_step: the model's gradient buffer must be this trainer's");
		const bool fuse = !ex.fn && t->fused_update_ok(n);
		if (train_step_body(t, stream, n, input, input_stride, dL_doutput, dL_stride, loss_scale, 1, ex, fuse, nullptr, 0) != NGP_OK)
			throw Error(g_last_error);
		t->step++;
	});
}

extern "C" {
int ngp_trainer_train_step(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                           const void* dL_doutput, uint32_t dL_stride, float loss_scale) {
	NGP_ARG(t);
	return ngp::train_step_with(t, stream, n, input, input_stride, dL_doutput, dL_stride, loss_scale, t->exchange());
}

int ngp_trainer_fused_update_active(const ngp_trainer* t, uint32_t n_batch) {
	return t && !t->allreduce && t->fused_update_ok(n_batch) ? 1 : 0;
}
}  // extern "C"

// The capture with an explicit gradient exchange hook and world factor (ngp_trainer_capture_training_step
// passes the trainer's own; the data-parallel NeRF trainer passes its communicator with world factor 1,
// because its shards' dL/doutput is already scaled by 128 / R_global, so the summed gradient is the
// 1-GPU gradient).
int ngp::capture_training_step_with(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                                    const void* dL_doutput, uint32_t dL_stride, float loss_scale, uint32_t n_steps,
                                    int with_optimizer, const Exchange& ex, ngp_graph** out) {
	NGP_ARG(t && out && stream && n > 0 && input && dL_doutput && loss_scale > 0.f && n_steps >= 1 && ex.world >= 1);
	NGP_TRY({
		ngp_model* m = t->model;
		m->require_params(false);
		NGP_CHECK(m->gradients == t->g16, "capture: the model's gradient buffer must be this trainer's");
		m->reserve(n);
		hipStream_t s = S(stream);
		auto g = std::make_unique<ngp_graph>();
		g->trainer = t;
		g->steps_per_launch = with_optimizer ? n_steps : 0;
		// the grid's update inside the backward where possible (lazy layout, no exchange): as training_step
		const bool fuse = with_optimizer && !ex.fn && t->fused_update_ok(n);
		NGP_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
		int rc = NGP_OK;
		for (uint32_t k = 0; k < n_steps && rc == NGP_OK; ++k)
			rc = train_step_body(t, stream, n, input, input_stride, dL_doutput, dL_stride, loss_scale, with_optimizer, ex, fuse,
			                     t->ctl, k);  // step = device base (set per launch) + k
		hipGraph_t graph = nullptr;
		const hipError_t end = hipStreamEndCapture(s, &graph);
		g->ws_epoch = m->ws_epoch;
		g->shards_stale = with_optimizer && t->sharded(ex) && ex.world > 1;
		g->g16_stale = !m->grads_valid;
		if (rc != NGP_OK) {
			if (graph) (void)hipGraphDestroy(graph);
			throw Error(g_last_error);
		}
		NGP_HIP(end);
		g->graph = graph;
		NGP_HIP(hipGraphInstantiate(&g->exec, g->graph, nullptr, nullptr, 0));
		*out = g.release();
	});
}
void ngp::trainer_ctl_values(const ngp_trainer* t, uint32_t** ctl, uint32_t* step, uint32_t* cfg_off, uint32_t* cfg_words, uint32_t* cfg) {
	static_assert(sizeof(AdamConfig) % 4 == 0 && sizeof(AdamConfig) <= 32 * 4, "AdamConfig as at most 32 words");
	*ctl = t->ctl;
	*step = t->step;
	*cfg_off = CTL_CFG;
	*cfg_words = sizeof(AdamConfig) / 4;
	memcpy(cfg, &t->cfg, sizeof(AdamConfig));
}
void ngp::graph_launch_ctl_written(ngp_graph* g, void* stream) {
	NGP_CHECK(g && g->exec, "graph launch: no graph");
	NGP_CHECK(g->ws_epoch == g->trainer->model->ws_epoch, "graph launch: the model's workspaces were reallocated (or its options changed) since capture");
	NGP_HIP(hipGraphLaunch(g->exec, S(stream)));
	g->launched();
}

extern "C" {

// The sharded optimizer's buffers for `world` ranks: the fp32 gradient staging of the reduce-scatter, sized
// outside any capture (the records and w16 carry SHARD_PAD spare parameters for the padding)
static void trainer_prepare_shards(ngp_trainer* t, uint32_t world) {
	if (!t->rec) return;
	const uint64_t q = 8ull * world, n_pad = (t->n + q - 1) / q * q;
	NGP_CHECK(n_pad - t->n <= ngp_trainer::SHARD_PAD, "sharded optimizer: too many ranks for the parameter padding");
	t->n_pad = n_pad;
	t->make_part_bounds(world);
	if (t->g32 && t->g32_count == n_pad) return;
	if (t->g32) NGP_HIP(hipFree(t->g32));
	t->g32 = nullptr;
	NGP_HIP(hipMalloc(&t->g32, n_pad * sizeof(float)));
	NGP_HIP(hipMemset(t->g32, 0, n_pad * sizeof(float)));  // the padding stays 0: it sums to 0 in the reduce-scatter
	t->g32_count = n_pad;
}

int ngp_trainer_set_data_parallel(ngp_trainer* t, uint32_t rank, uint32_t world, ngp_allreduce_fn fn, void* user) {
	NGP_ARG(t && world >= 1 && rank < world && (fn || world == 1));
	NGP_TRY({
		NGP_CHECK(t->shards_valid, "set_data_parallel: gather the sharded optimizer state first (ngp_trainer_gather_shards)");
		t->allreduce = fn;
		t->allreduce_user = user;
		t->world = fn ? world : 1;
		t->dp_rank = fn ? rank : 0;
		t->dp_rank_known = fn != nullptr;
		if (fn) trainer_prepare_shards(t, world);
		// the engine's communicator widens fp16 all-reduces to fp32 (the unsharded path): staging sized now
		if (fn == ngp_dp_comm_allreduce && user)
			NGP_CHECK(ngp_dp_comm_reserve((ngp_dp_comm*)user, t->n) == NGP_OK, "ngp_dp_comm_reserve failed");
	});
}

int ngp_trainer_gather_shards(ngp_trainer* t, void* stream) {
	NGP_ARG(t);
	NGP_TRY({
		if (t->shards_valid) return NGP_OK;
		NGP_CHECK(t->allreduce && t->rec && t->n_pad && t->pb.size() >= 2, "gather_shards: no sharded exchange attached");
		// records of each part's parameter pairs, 12 floats each: rank r's slice of the part holds the pairs of its
		// parameter slice
		static_assert(sizeof(AdamRec) == 12 * sizeof(float), "AdamRec: 12 floats");
		for (size_t j = 0; j + 1 < t->pb.size(); ++j)
			if (t->allreduce(t->allreduce_user, t->rec + t->pb[j] / 2, (t->pb[j + 1] - t->pb[j]) / 2 * 12, NGP_DTYPE_F32, NGP_ALL_GATHER,
			                 stream) != NGP_OK)
				throw Error(g_last_error.empty() ? "gather_shards: all-gather failed" : g_last_error);
		NGP_HIP(hipStreamSynchronize(S(stream)));
		t->shards_valid = true;
	});
}

int ngp_trainer_set_allreduce(ngp_trainer* t, uint32_t world, ngp_allreduce_fn allreduce, void* user) {
	NGP_ARG(t && world >= 1);
	NGP_TRY({
		NGP_CHECK(t->shards_valid, "set_allreduce: gather the sharded optimizer state first (ngp_trainer_gather_shards)");
		t->allreduce = allreduce;
		t->allreduce_user = user;
		t->world = allreduce ? world : 1;
		t->dp_rank = 0;
		t->dp_rank_known = false;
		// the engine's communicator widens the fp16 sum to fp32: size its staging now, outside any capture
		if (allreduce == ngp_dp_comm_allreduce && user)
			NGP_CHECK(ngp_dp_comm_reserve((ngp_dp_comm*)user, t->n) == NGP_OK, "ngp_dp_comm_reserve failed");
	});
}

int ngp_graph_launch(ngp_graph* g, void* stream) {
	NGP_ARG(g && g->exec);
	NGP_TRY({
		NGP_CHECK(g->ws_epoch == g->trainer->model->ws_epoch,
		          "graph launch: the model's workspaces were reallocated since capture (a larger batch or a density "
		          "pass grew them); capture again (ngp_model_workspace_epoch tells when)");
		if (g->steps_per_launch) set_device_ctl(g->trainer->ctl, g->trainer->step, g->trainer->cfg, S(stream));
		NGP_HIP(hipGraphLaunch(g->exec, S(stream)));
		g->launched();
	});
}

void ngp_graph_destroy(ngp_graph* g) { delete g; }

void* ngp_trainer_gradients(ngp_trainer* t) { return t ? t->g16 : nullptr; }
int ngp_trainer_gradients_valid(const ngp_trainer* t) {
	return t && t->model->gradients == t->g16 && t->model->grads_valid ? 1 : 0;
}
void* ngp_trainer_params(ngp_trainer* t) { return t ? t->w16 : nullptr; }
void* ngp_trainer_inference_params(ngp_trainer* t) {
	if (!t) return nullptr;
	if (t->rec && t->inf_stale) {  // lazy EMA: bring the inference parameters up to date before handing them out
		try {
			NGP_HIP(hipDeviceSynchronize());  // the optimizer may still run on a caller's non-blocking stream
			t->materialize(nullptr);
			NGP_HIP(hipDeviceSynchronize());
		} catch (const std::exception& e) {
			g_last_error = e.what();
			return nullptr;
		}
	}
	return t->cfg.ema_decay > 0.f ? t->inf16 : t->w16;
}
// Lazy layout: the mirror of the records' weights, refreshed here (a read accessor: writes into it do not reach
// the records; set_params_full_precision does, as in tcnn).
float* ngp_trainer_params_full_precision(ngp_trainer* t) {
	if (!t) return nullptr;
	try {
		t->sync_w32();
		// the caller may write into the mirror: it is not the master copy, so the next reader (serialize, this
		// accessor) refreshes it from the records again instead of trusting it
		if (t->rec) t->w32_stale = true;
	} catch (const std::exception& e) {
		g_last_error = e.what();
		return nullptr;
	}
	return t->w32;
}
uint32_t ngp_trainer_step(const ngp_trainer* t) { return t ? t->step : 0; }
uint64_t ngp_trainer_n_params(const ngp_trainer* t) { return t ? t->n : 0; }
float ngp_trainer_learning_rate(const ngp_trainer* t) { return t ? t->cfg.lr_at(t->step) : 0.f; }
int ngp_trainer_set_learning_rate(ngp_trainer* t, float lr) {
	NGP_ARG(t && lr >= 0.f);
	NGP_TRY({ t->cfg.lr = lr; });
}
// Trainer options (engine extension). "ema_closed_form": 0 (default) = the lazy layout's owed EMA steps are
// replayed exactly (optimizer.h ema_catch_up: bit for bit the eager layout), 1 = closed form for gaps of more
// than 32 steps (A/B and the tolerance test only).
int ngp_trainer_set_option(ngp_trainer* t, const char* key, double value) {
	NGP_ARG(t && key);
	NGP_TRY({
		const std::string k = key;
		if (k == "ema_closed_form") {
			t->cfg.ema_closed_form = value != 0 ? 1u : 0u;
		} else if (k == "shard_opt") {
			NGP_CHECK(t->shards_valid, "shard_opt: gather the sharded optimizer state first (ngp_trainer_gather_shards)");
			t->shard_opt = value != 0;
		} else if (k == "dp_parts") {
			NGP_CHECK(t->shards_valid, "dp_parts: gather the sharded optimizer state first (ngp_trainer_gather_shards)");
			NGP_CHECK(value >= 1 && value <= BwdParts::MAX, "dp_parts: 1 to 8");
			t->dp_parts = (uint32_t)value;
			if (t->n_pad) t->make_part_bounds(t->world);
		} else if (k == "dp_wire16") {
			t->dp_wire16 = value != 0;
		} else {
			throw Error("ngp_trainer_set_option: unknown option " + k);
		}
	});
}

__global__ static void k_f32_to_f16(const float* a, f16* b, f16* c, uint64_t n) {
	const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
	if (i < n) { b[i] = (f16)a[i]; c[i] = (f16)a[i]; }
}

int ngp_trainer_set_params_full_precision(ngp_trainer* t, const float* params_host, uint64_t n) {
	NGP_ARG(t && params_host && n == t->n);
	NGP_TRY({
		t->require_full_state("set_params_full_precision");
		if (t->rec && t->step > 0) {
			// lazy EMA: entries skipped since their last update still owe EMA steps on the OLD weight (the eager
			// layout applied them every step). Replay them before the weights change; the records are then
			// current (done = step), as every eager EMA is.
			NGP_HIP(hipDeviceSynchronize());
			t->materialize(nullptr, true);
			NGP_HIP(hipDeviceSynchronize());
		}
		NGP_HIP(hipMemcpy(t->w32, params_host, n * 4, hipMemcpyHostToDevice));
		k_f32_to_f16<<<div_round_up(n, 256), 256>>>(t->w32, t->w16, t->inf16, n);
		NGP_HIP(hipGetLastError());
		if (t->rec) adam_rec_weights((uint32_t)n, t->rec, t->w32, true, nullptr);
		NGP_HIP(hipDeviceSynchronize());
		t->inf_stale = t->w32_stale = false;  // inference parameters = the new weights, as in the eager layout
		t->bind_model();
	});
}

// Blob: magic, version, n, step, then w32, m1, m2, ema32 (f32), steps (u32)
int ngp_trainer_serialize(ngp_trainer* t, void* buf, uint64_t* size) {
	NGP_ARG(t && size);
	NGP_TRY({
		const uint64_t need = 32 + t->n * 4 * 5;
		if (!buf) { *size = need; return NGP_OK; }
		t->require_full_state("serialize");
		NGP_CHECK(*size >= need, "serialize: buffer too small");
		char* p = (char*)buf;
		const uint64_t hdr[4] = {0x4e47504d49333535ULL /* "NGPMI355" */, 1, t->n, t->step};
		memcpy(p, hdr, 32); p += 32;
		NGP_HIP(hipDeviceSynchronize());
		if (t->rec) t->w32_stale = true;  // lazy layout: the blob's weights always come from the records
		t->sync_w32();
		DevBuf soa;
		float *m1 = t->m1, *m2 = t->m2, *ema32 = t->ema32;
		uint32_t* steps = t->steps;
		if (t->rec) {  // lazy layout: every EMA brought up to date, then the eager arrays of the blob
			t->materialize(nullptr);
			char* q = (char*)soa.get(t->n * 16);
			m1 = (float*)q; m2 = (float*)(q + t->n * 4); ema32 = (float*)(q + t->n * 8); steps = (uint32_t*)(q + t->n * 12);
			adam_rec_to_soa((uint32_t)t->n, t->rec, m1, m2, ema32, steps, nullptr);
			NGP_HIP(hipDeviceSynchronize());
		}
		for (void* src : {(void*)t->w32, (void*)m1, (void*)m2, (void*)ema32, (void*)steps}) {
			NGP_HIP(hipMemcpy(p, src, t->n * 4, hipMemcpyDeviceToHost));
			p += t->n * 4;
		}
		*size = need;
	});
}

int ngp_trainer_deserialize(ngp_trainer* t, const void* buf, uint64_t size) {
	NGP_ARG(t && buf);
	NGP_TRY({
		const char* p = (const char*)buf;
		uint64_t hdr[4];
		NGP_CHECK(size >= 32, "deserialize: truncated");
		memcpy(hdr, p, 32); p += 32;
		NGP_CHECK(hdr[0] == 0x4e47504d49333535ULL && hdr[1] == 1, "deserialize: bad magic/version");
		NGP_CHECK(hdr[2] == t->n && size >= 32 + t->n * 20, "deserialize: parameter count mismatch");
		t->step = (uint32_t)hdr[3];
		t->sync_device_step();
		DevBuf soa;
		float *m1 = t->m1, *m2 = t->m2, *ema32 = t->ema32;
		uint32_t* steps = t->steps;
		if (t->rec) {
			char* q = (char*)soa.get(t->n * 16);
			m1 = (float*)q; m2 = (float*)(q + t->n * 4); ema32 = (float*)(q + t->n * 8); steps = (uint32_t*)(q + t->n * 12);
		}
		for (void* dst : {(void*)t->w32, (void*)m1, (void*)m2, (void*)ema32, (void*)steps}) {
			NGP_HIP(hipMemcpy(dst, p, t->n * 4, hipMemcpyHostToDevice));
			p += t->n * 4;
		}
		if (t->rec) {
			adam_soa_to_rec((uint32_t)t->n, m1, m2, ema32, steps, t->step, t->rec, nullptr);
			adam_rec_weights((uint32_t)t->n, t->rec, t->w32, true, nullptr);
		}
		t->inf_stale = t->w32_stale = false;  // inference parameters = the restored weights (below), as in the eager layout
		t->shards_valid = true;              // every record restored on every rank
		k_f32_to_f16<<<div_round_up(t->n, 256), 256>>>(t->w32, t->w16, t->inf16, t->n);
		NGP_HIP(hipGetLastError());
		NGP_HIP(hipDeviceSynchronize());
		t->model->frags_current = false;
	});
}

}  // extern "C"
