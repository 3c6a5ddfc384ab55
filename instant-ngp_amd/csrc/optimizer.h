// optimizer.h — Ema o ExponentialDecay o Adam (tcnn optimizer chain, restated).
#pragma once
#include "common.h"

namespace ngp {

struct AdamConfig {
	float lr = 1e-2f, beta1 = 0.9f, beta2 = 0.99f, eps = 1e-15f, l2 = 1e-6f;
	float ema_decay = 0.f;  // 0 => no Ema wrapper
	uint32_t decay_start = 0, decay_interval = 0;  // 0 interval => no ExponentialDecay wrapper
	float decay_base = 1.f;
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
// the inference (EMA) parameters are read (ema_materialize): bit-identical to the eager update.
struct AdamRec {
	float m1[2], m2[2];
	uint32_t steps[2];
	float ema[2];
	uint32_t done[2];
	uint32_t pad[2];
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
};
// The trainer's device control block: ctl[0] optimizer step, ctl[1] block counter, AdamConfig at
// ctl + CTL_CFG. A graph launch rewrites step and config (set_device_ctl), so replayed steps follow
// set_learning_rate / set_option like eager ones.
constexpr uint32_t CTL_CFG = 16;
void adam_ema_update(const AdamConfig& c, uint32_t n, uint32_t n_matrix, float loss_scale, const AdamState& st, hipStream_t s);
void set_device_ctl(uint32_t* ctl, uint32_t step, const AdamConfig& c, hipStream_t s);
// Lazy layout: bring every parameter's EMA up to `steps_done` optimizer steps and write ema16 (the
// inference parameters) debiased as the eager update would have after step steps_done - 1.
void ema_materialize(const AdamConfig& c, uint32_t n, uint32_t steps_done, const AdamState& st, hipStream_t s);
// Lazy layout <-> the eager arrays (m1, m2, ema32 f32 and steps u32, each [n]), e.g. for serialize.
void adam_rec_to_soa(uint32_t n, const AdamRec* rec, float* m1, float* m2, float* ema32, uint32_t* steps, hipStream_t s);
void adam_soa_to_rec(uint32_t n, const float* m1, const float* m2, const float* ema32, const uint32_t* steps, uint32_t done,
                     AdamRec* rec, hipStream_t s);

}  // namespace ngp
