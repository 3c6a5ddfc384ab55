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

// ctl: device optimizer step; the update reads it and then advances it (stream-ordered).
void adam_ema_step(const AdamConfig& c, uint32_t n, uint32_t n_matrix, float loss_scale, float* w32, f16* w16, const f16* g16,
                   float* m1, float* m2, uint32_t* steps, float* ema32, f16* ema16, uint32_t* ctl, hipStream_t s);

}  // namespace ngp
