// optimizer.h — Ema o ExponentialDecay o Adam (tcnn optimizer chain, restated).
#pragma once
#include "common.h"

namespace ngp {

struct AdamConfig {
	float lr = 1e-2f, beta1 = 0.9f, beta2 = 0.99f, eps = 1e-15f, l2 = 1e-6f;
	float ema_decay = 0.f;  // 0 => no Ema wrapper
	uint32_t decay_start = 0, decay_interval = 0;  // 0 interval => no ExponentialDecay wrapper
	float decay_base = 1.f;
	// lazy layout: how a skipped parameter's owed EMA steps are applied (ema_catch_up). 0 = exact replay (bit
	// for bit the eager layout), 1 = closed form past EMA_CATCH_UP_LOOP steps (trainer option "ema_closed_form")
	uint32_t ema_closed_form = 0;
	float lr_at(uint32_t step) const;  // learning rate used by optimizer step `step` (0-based)
};

// One fused update. The optimizer step used for the schedule / bias correction / EMA debias is
// (step_base ? *step_base : 0) + step_add: eager steps pass the host step in step_add; a captured HIP
// graph of K steps reads the base from device memory (set once per launch) plus the step's index.
// frags/fragmap (optional): the MLP weight fragments (mlp.h) are rewritten in place from the new fp16
// matrix params, so the next MLP launch needs no k_prepare_frags (fragmap: 2 slots per matrix param).
// Lazy-EMA layout (large tables, ngp_trainer lazy_ema): the per-parameter state of a PAIR of
// parameters in one 48-B record, so a step touches only the records of updated parameters. `done` =
// number of optimizer steps whose EMA the parameter has received; a parameter that is skipped (zero
// grid gradient) keeps its weight, so its missing EMA steps are the same recurrence on the same
// weight and are applied, in order and with the same fp32 operations, when it is next updated or when
// the inference (EMA) parameters are read (ema_materialize): bit-identical to the eager update (ema_catch_up).
// The fp32 master weights of the pair live in the record too (`w`): an update then reads and writes one
// record instead of the record plus a separate line of the w32 array. The trainer's w32 array is a
// mirror in this layout, refreshed when it is read (adam_rec_weights).
struct AdamRec {
	float m1[2], m2[2];
	uint32_t steps[2];
	float ema[2];
	uint32_t done[2];
	float w[2];
};
static_assert(sizeof(AdamRec) == 48, "AdamRec is three 16-B words (64-B records measured slower: 976 -> 1019 us at C5)");

struct AdamState {
	float* w32; f16* w16; const f16* g16;
	float* m1; float* m2; uint32_t* steps;
	float* ema32; f16* ema16;
	f16* frags; const uint32_t* fragmap;
	const uint32_t* step_base; uint32_t step_add;
	const AdamConfig* cfg_dev;  // non-null (captured steps): hyperparameters read from device memory
	AdamRec* rec = nullptr;     // non-null: lazy-EMA layout (m1/m2/steps/ema32 unused)
	const float* bias_tab = nullptr;  // adam_bias_table (nullable)
	// lazy layout, sharded data parallelism: the gradient is the ranks' fp32 sum of their fp16 gradients
	// (reduce-scatter); it is rounded to fp16 once here, as the all-reduce path narrows it (dp_comm.hip)
	const float* g32 = nullptr;
};
// ---- device helpers shared by optimizer.hip and the fused update in the grid backward ----------
// Adam's bias correction depends on the parameter's own step s only: the factors sqrtf(1 - beta2^s) and
// 1 - beta1^s are tabulated once per trainer for s < BIAS_TAB_CAP by the same device powf/sqrtf
// (adam_bias_table), so the per-parameter update reads two floats instead of evaluating two powf; the
// step size lr * A / B keeps its operations and order, so the result is bit-identical. Layout: float2
// per s; entry 0 holds the betas the table was built for (a mismatch falls back to powf).
constexpr uint32_t BIAS_TAB_CAP = 1u << 20;
__device__ __forceinline__ float adam_step_size(const AdamConfig& c, float lr, uint32_t sk, const float* tab) {
	typedef float f32x2_t __attribute__((ext_vector_type(2)));
	if (tab && sk < BIAS_TAB_CAP && tab[0] == c.beta1 && tab[1] == c.beta2) {
		const f32x2_t q = ((const f32x2_t*)tab)[sk];
		return lr * q[0] / q[1];
	}
	return lr * sqrtf(1.f - powf(c.beta2, (float)sk)) / (1.f - powf(c.beta1, (float)sk));
}
void adam_bias_table(float* tab, float beta1, float beta2, hipStream_t s);
// Learning rate of optimizer step `step` (ExponentialDecay wrapper).
__device__ __forceinline__ float lr_schedule(const AdamConfig& c, uint32_t step) {
	float r = c.lr;
	if (c.decay_interval == 0 || step < c.decay_start) return r;
	const uint32_t k = (step - c.decay_start) / c.decay_interval + 1;
	for (uint32_t i = 0; i < k; ++i) r *= c.decay_base;
	return r;
}
// The eager EMA of step j: e = d * e + (1 - d) * w (w after step j's update), output e / (1 - d^(j+1)). Every
// site evaluates the recurrence as ema_step, RN(RN(d e) + RN((1 - d) w)) (the engine builds with
// -ffp-contract=off, as the oracle does), so the eager kernels, the lazy update and the catch-up below round
// identically.
__device__ __forceinline__ float ema_step(float e, float d, float dw) { return d * e + dw; }
// A parameter skipped for k steps kept its weight w, so its EMA is owed k applications of that recurrence
// with a constant addend. The map e -> RN(RN(d e) + RN((1 - d) w)) is non-decreasing in e (d > 0, RN is
// monotone), so the replayed sequence is monotone and, on the finite set of floats, reaches a fixed point
// after which every step leaves it unchanged. The exact catch-up therefore replays until the gap is
// exhausted or a step changes nothing: bit for bit the eager layout's value whatever the gap, in at most a
// few hundred steps (d = 0.95: the distance to w shrinks by 0.95 per step until one step's change rounds
// away; 200-600 steps from random float starts). Replaying the whole gap made a rarely touched entry loop
// over tens of thousands of steps (NeRF: entries at the edge of the occupied space) while the kernel waited
// for that thread. closed != 0 (AdamConfig::ema_closed_form): past EMA_CATCH_UP_LOOP steps use
// d^k e + (1 - d^k) w instead, which differs from the replay by rounding (tests/test_gpu_ema_gaps.py).
constexpr uint32_t EMA_CATCH_UP_LOOP = 32;
__device__ __forceinline__ float ema_catch_up(float e, float w, float d, uint32_t from, uint32_t to, uint32_t closed = 0) {
	if (to <= from) return e;
	uint32_t k = to - from;
	if (closed && k > EMA_CATCH_UP_LOOP) {
		const float dk = powf(d, (float)k);
		return dk * e + (1.f - dk) * w;
	}
	const float dw = (1.f - d) * w;
	for (; k >= 4; k -= 4) {
		const float e1 = ema_step(e, d, dw), e2 = ema_step(e1, d, dw), e3 = ema_step(e2, d, dw), e4 = ema_step(e3, d, dw);
		if (e4 == e3) return e4;  // fixed point: the rest of the gap leaves it unchanged
		e = e4;
	}
	for (; k; --k) e = ema_step(e, d, dw);
	return e;
}

// Four parameters (two records) per group; a record none of whose parameters is updated this step is
// neither read nor written (grid entries without gradient: the bulk of a large table). A thread owns
// two groups half the table apart and issues both groups' state loads before either computes (the
// loads depend on the gradient test: two chains in flight instead of one).
struct LazyGroup {
	uint32_t i0;
	bool act[4], any[2];
	float g[4];
	f32x4 q[2][3];
};

__device__ __forceinline__ void lazy_update(const AdamState& st, const AdamConfig& c, uint32_t step, uint32_t n_matrix, LazyGroup& G) {
	if (!G.any[0] && !G.any[1]) return;
	const uint32_t i0 = G.i0;
	const float lr = lr_schedule(c, step);
	const float d = c.ema_decay;
	float w[4];
#pragma unroll
	for (int r = 0; r < 2; ++r) {
		if (!G.any[r]) continue;
		w[2 * r] = G.q[r][2][2];  // the pair's fp32 weights (AdamRec::w)
		w[2 * r + 1] = G.q[r][2][3];
		AdamRec rc;
		rc.m1[0] = G.q[r][0][0]; rc.m1[1] = G.q[r][0][1]; rc.m2[0] = G.q[r][0][2]; rc.m2[1] = G.q[r][0][3];
		rc.steps[0] = __float_as_uint(G.q[r][1][0]); rc.steps[1] = __float_as_uint(G.q[r][1][1]);
		rc.ema[0] = G.q[r][1][2]; rc.ema[1] = G.q[r][1][3];
		rc.done[0] = __float_as_uint(G.q[r][2][0]); rc.done[1] = __float_as_uint(G.q[r][2][1]);
#pragma unroll
		for (int k = 0; k < 2; ++k) {
			const int p = 2 * r + k;
			if (!G.act[p]) continue;
			// missing EMA steps first, with the weight those steps saw (unchanged since the last update)
			if (d > 0.f) rc.ema[k] = ema_catch_up(rc.ema[k], w[p], d, rc.done[k], step, c.ema_closed_form);
			float gk = G.g[p];
			if (i0 + p < n_matrix) gk += c.l2 * w[p];
			const float mm = c.beta1 * rc.m1[k] + (1.f - c.beta1) * gk;
			const float vv = c.beta2 * rc.m2[k] + (1.f - c.beta2) * (gk * gk);
			rc.m1[k] = mm;
			rc.m2[k] = vv;
			const uint32_t sk = rc.steps[k] + 1;
			rc.steps[k] = sk;
			const float lr_s = adam_step_size(c, lr, sk, st.bias_tab);
			w[p] = w[p] - lr_s / (sqrtf(vv) + c.eps) * mm;
			if (d > 0.f) rc.ema[k] = ema_step(rc.ema[k], d, (1.f - d) * w[p]);
			rc.done[k] = step + 1;
		}
		f32x4* rp = (f32x4*)(st.rec + (i0 >> 1) + r);
		rp[0] = f32x4{rc.m1[0], rc.m1[1], rc.m2[0], rc.m2[1]};
		rp[1] = f32x4{__uint_as_float(rc.steps[0]), __uint_as_float(rc.steps[1]), rc.ema[0], rc.ema[1]};
		rp[2] = f32x4{__uint_as_float(rc.done[0]), __uint_as_float(rc.done[1]), w[2 * r], w[2 * r + 1]};
		*(f16x2*)(st.w16 + i0 + 2 * r) = f16x2{(f16)w[2 * r], (f16)w[2 * r + 1]};
	}
	if (st.frags && i0 < n_matrix) {
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			if (i0 + k >= n_matrix || !G.act[k]) continue;
			const uint32_t q0 = st.fragmap[2 * (i0 + k)], q1 = st.fragmap[2 * (i0 + k) + 1];
			const f16 wh = (f16)w[k];
			if (q0 != ~0u) st.frags[q0] = wh;
			if (q1 != ~0u) st.frags[q1] = wh;
		}
	}
}

// The lazy-layout update applied inside the hash-grid backward (engine option fuse_opt): the bucket
// accumulation holds each grid entry's final fp16 gradient, so it updates that parameter pair's record
// directly instead of storing the gradient for k_adam_lazy4 to read back (C5: 210 MB written and 210 MB
// read per step). Pointers are offset to the grid's first parameter (an even index: records are pairs).
// Same fp32 operations, in the same order, as k_adam_lazy4's lazy_update for a non-matrix pair.
struct FusedAdam {
	f16* w16 = nullptr;
	AdamRec* rec = nullptr;  // null: no fused update (the backward stores the gradient); holds the fp32 weights
	float loss_scale = 1.f;
	AdamConfig cfg;
	const AdamConfig* cfg_dev = nullptr;
	const uint32_t* step_base = nullptr;
	uint32_t step_add = 0;
	const float* bias_tab = nullptr;
	// The MLP section's update too (mlp_n = its parameter count, a multiple of 4; 0: the optimizer launch
	// does it): the dW slab blocks of the grid backward's last kernel hold those parameters' final
	// gradients, so they run k_adam_lazy4's lazy_update on them (whole-model pointers; option fuse_mlp_opt)
	uint32_t mlp_n = 0;
	f16* mlp_w16 = nullptr;
	// no update (rec null), the gradient stored widened: the fp16-rounded sums as fp32 at g32 (grid-relative in
	// the grid backward, the whole model's buffer at the engine boundary) — the sharded optimizer's
	// reduce-scatter input written by the backward itself
	float* g32 = nullptr;
	AdamRec* mlp_rec = nullptr;
	f16* frags = nullptr;
	const uint32_t* fragmap = nullptr;
};
// One parameter pair's state between the load and the update (callers issue several pairs' loads
// before the first update: the record reads are the latency to hide).
struct FusedPair {
	float g[2];
	bool act[2];
	f32x4 q0, q1, q2;
};
__device__ __forceinline__ bool fused_adam_load(const FusedAdam& fa, uint32_t r, f16 g0h, f16 g1h, FusedPair& p) {
	p.g[0] = (float)g0h / fa.loss_scale;
	p.g[1] = (float)g1h / fa.loss_scale;
	p.act[0] = p.g[0] != 0.f;  // grid parameters: a zero gradient skips the parameter
	p.act[1] = p.g[1] != 0.f;
	if (!p.act[0] && !p.act[1]) return false;
	const f32x4* rp = (const f32x4*)(fa.rec + r);
	p.q0 = rp[0]; p.q1 = rp[1]; p.q2 = rp[2];
	return true;
}
__device__ __forceinline__ void fused_adam_store(const FusedAdam& fa, uint32_t r, FusedPair& p) {
	const AdamConfig c = fa.cfg_dev ? *fa.cfg_dev : fa.cfg;
	const uint32_t step = (fa.step_base ? *fa.step_base : 0u) + fa.step_add;
	const float lr = lr_schedule(c, step);
	const float d = c.ema_decay;
	float m1[2] = {p.q0[0], p.q0[1]}, m2[2] = {p.q0[2], p.q0[3]}, ema[2] = {p.q1[2], p.q1[3]};
	uint32_t steps[2] = {__float_as_uint(p.q1[0]), __float_as_uint(p.q1[1])};
	uint32_t done[2] = {__float_as_uint(p.q2[0]), __float_as_uint(p.q2[1])};
	float w[2] = {p.q2[2], p.q2[3]};
#pragma unroll
	for (int k = 0; k < 2; ++k) {
		if (!p.act[k]) continue;
		if (d > 0.f) ema[k] = ema_catch_up(ema[k], w[k], d, done[k], step, c.ema_closed_form);
		const float gk = p.g[k];
		const float mm = c.beta1 * m1[k] + (1.f - c.beta1) * gk;
		const float vv = c.beta2 * m2[k] + (1.f - c.beta2) * (gk * gk);
		m1[k] = mm;
		m2[k] = vv;
		const uint32_t sk = steps[k] + 1;
		steps[k] = sk;
		const float lr_s = adam_step_size(c, lr, sk, fa.bias_tab);
		w[k] = w[k] - lr_s / (sqrtf(vv) + c.eps) * mm;
		if (d > 0.f) ema[k] = ema_step(ema[k], d, (1.f - d) * w[k]);
		done[k] = step + 1;
	}
	f32x4* rp = (f32x4*)(fa.rec + r);
	rp[0] = f32x4{m1[0], m1[1], m2[0], m2[1]};
	rp[1] = f32x4{__uint_as_float(steps[0]), __uint_as_float(steps[1]), ema[0], ema[1]};
	rp[2] = f32x4{__uint_as_float(done[0]), __uint_as_float(done[1]), w[0], w[1]};
	*(f16x2*)(fa.w16 + 2 * (size_t)r) = f16x2{(f16)w[0], (f16)w[1]};
}
__device__ __forceinline__ void fused_adam_pair(const FusedAdam& fa, uint32_t r, f16 g0h, f16 g1h) {
	FusedPair p;
	if (fused_adam_load(fa, r, g0h, g1h, p)) fused_adam_store(fa, r, p);
}

// The trainer's device control block: ctl[0] optimizer step, ctl[1] block counter, AdamConfig at
// ctl + CTL_CFG. A graph launch rewrites step and config (set_device_ctl), so replayed steps follow
// set_learning_rate / set_option like eager ones.
constexpr uint32_t CTL_CFG = 16;
void adam_ema_update(const AdamConfig& c, uint32_t n, uint32_t n_matrix, float loss_scale, const AdamState& st, hipStream_t s);
// Lazy layout: the update of parameters [lo, hi) only (multiples of 4): one rank's slice under the sharded
// optimizer (st.g32 = the reduce-scattered fp32 gradient sums, indexed like the parameters)
void adam_lazy_range(const AdamConfig& c, uint32_t lo, uint32_t hi, uint32_t n_matrix, float loss_scale, const AdamState& st,
                     hipStream_t s);
void set_device_ctl(uint32_t* ctl, uint32_t step, const AdamConfig& c, hipStream_t s);
// Lazy layout: bring every parameter's EMA up to `steps_done` optimizer steps and write ema16 (the
// inference parameters) debiased as the eager update would have after step steps_done - 1.
void ema_materialize(const AdamConfig& c, uint32_t n, uint32_t steps_done, const AdamState& st, hipStream_t s);
// Lazy layout <-> the eager arrays (m1, m2, ema32 f32 and steps u32, each [n]), e.g. for serialize.
void adam_rec_to_soa(uint32_t n, const AdamRec* rec, float* m1, float* m2, float* ema32, uint32_t* steps, hipStream_t s);
void adam_soa_to_rec(uint32_t n, const float* m1, const float* m2, const float* ema32, const uint32_t* steps, uint32_t done,
                     AdamRec* rec, hipStream_t s);
// Lazy layout: the records' fp32 weights to the w32 mirror (to_rec false) or from it (to_rec true).
void adam_rec_weights(uint32_t n, AdamRec* rec, float* w32, bool to_rec, hipStream_t s);

}  // namespace ngp
