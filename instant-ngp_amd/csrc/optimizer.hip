// optimizer.hip — fused Ema(ExponentialDecay(Adam)) step, one pass over the parameters.
//
// Replaces tcnn's Trainer::optimizer_step chain as configured by configs/nerf/base.json:5-22 and
// invoked at src/testbed_nerf.cu:3678. Semantics restated (tcnn absent):
// gradient /= loss_scale; non-matrix params with a zero gradient are skipped (lazy, per-parameter
// step counter); l2 only on matrix params; per-parameter bias correction; EMA debiased by the
// optimizer step. Oracle: orc_adam_step (oracle/ngp_oracle.c).
#include "optimizer.h"

#include <cmath>

namespace ngp {

// The optimizer step count lives on the device (ctl[0]) so the step can be replayed from a HIP graph:
// the update kernel reads it and a one-thread kernel after it advances it (a last-block counter would
// put ~13k same-address atomics on one L2 line: measured 330 us).
__device__ __forceinline__ float lr_schedule(const AdamConfig& c, uint32_t step) {
	float r = c.lr;
	if (c.decay_interval == 0 || step < c.decay_start) return r;
	const uint32_t k = (step - c.decay_start) / c.decay_interval + 1;
	for (uint32_t i = 0; i < k; ++i) r *= c.decay_base;
	return r;
}

__global__ void k_adam_ema(const uint32_t n, const uint32_t n_matrix, const float loss_scale, const AdamConfig c,
                           float* __restrict__ w32, f16* __restrict__ w16, const f16* __restrict__ g16,
                           float* __restrict__ m1, float* __restrict__ m2, uint32_t* __restrict__ steps,
                           float* __restrict__ ema32, f16* __restrict__ ema16, uint32_t* __restrict__ ctl) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t step = ctl[0];
	if (i < n) {
		const float lr = lr_schedule(c, step);
		float g = (float)g16[i] / loss_scale;
		float w = w32[i];
		if (!(i >= n_matrix && g == 0.f)) {
			if (i < n_matrix) g += c.l2 * w;
			const float mm = c.beta1 * m1[i] + (1.f - c.beta1) * g;
			const float vv = c.beta2 * m2[i] + (1.f - c.beta2) * (g * g);
			m1[i] = mm;
			m2[i] = vv;
			const uint32_t s = steps[i] + 1;
			steps[i] = s;
			const float lr_s = lr * sqrtf(1.f - powf(c.beta2, (float)s)) / (1.f - powf(c.beta1, (float)s));
			w = w - lr_s / (sqrtf(vv) + c.eps) * mm;
			w32[i] = w;
			w16[i] = (f16)w;
		}
		if (ema32) {
			const float debias = 1.f - powf(c.ema_decay, (float)(step + 1));
			const float v = c.ema_decay * ema32[i] + (1.f - c.ema_decay) * w;
			ema32[i] = v;
			ema16[i] = (f16)(v / debias);
		}
	}
}

__global__ void k_step_advance(uint32_t* ctl) { ctl[0] += 1; }

float AdamConfig::lr_at(uint32_t step) const {
	float r = lr;
	if (decay_interval == 0 || step < decay_start) return r;
	const uint32_t k = (step - decay_start) / decay_interval + 1;
	for (uint32_t i = 0; i < k; ++i) r *= decay_base;
	return r;
}

void adam_ema_step(const AdamConfig& c, uint32_t n, uint32_t n_matrix, float loss_scale, float* w32, f16* w16, const f16* g16,
                   float* m1, float* m2, uint32_t* steps, float* ema32, f16* ema16, uint32_t* ctl, hipStream_t s) {
	k_adam_ema<<<div_round_up(n, 256), 256, 0, s>>>(n, n_matrix, loss_scale, c, w32, w16, g16, m1, m2, steps,
	                                                 c.ema_decay > 0.f ? ema32 : nullptr, ema16, ctl);
	NGP_HIP(hipGetLastError());
	k_step_advance<<<1, 1, 0, s>>>(ctl);
	NGP_HIP(hipGetLastError());
}

}  // namespace ngp
