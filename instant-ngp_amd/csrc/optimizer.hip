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

// The optimizer step: eager launches pass it by value; a HIP graph of K captured steps reads a base
// from device memory (written once per graph launch by k_set_step) plus the step's index in the graph,
// so no per-step counter kernel is needed. lr_schedule, ema_catch_up: optimizer.h.

__global__ void k_adam_bias_table(float* __restrict__ tab, float beta1, float beta2) {
	const uint32_t sk = blockIdx.x * blockDim.x + threadIdx.x;
	if (sk >= BIAS_TAB_CAP) return;
	if (sk == 0) { tab[0] = beta1; tab[1] = beta2; return; }
	tab[2 * sk] = sqrtf(1.f - powf(beta2, (float)sk));
	tab[2 * sk + 1] = 1.f - powf(beta1, (float)sk);
}
void adam_bias_table(float* tab, float beta1, float beta2, hipStream_t s) {
	k_adam_bias_table<<<BIAS_TAB_CAP / 256, 256, 0, s>>>(tab, beta1, beta2);
	NGP_HIP(hipGetLastError());
}

__global__ void k_adam_ema(const uint32_t i0, const uint32_t n, const uint32_t n_matrix, const float loss_scale, const AdamConfig c_arg,
                           const AdamState st) {
	const AdamConfig c = st.cfg_dev ? *st.cfg_dev : c_arg;
	const uint32_t i = i0 + blockIdx.x * blockDim.x + threadIdx.x;
	const uint32_t step = (st.step_base ? *st.step_base : 0u) + st.step_add;
	if (i < n) {
		const float lr = lr_schedule(c, step);
		float g = (float)st.g16[i] / loss_scale;
		float w = st.w32[i];
		if (!(i >= n_matrix && g == 0.f)) {
			if (i < n_matrix) g += c.l2 * w;
			const float mm = c.beta1 * st.m1[i] + (1.f - c.beta1) * g;
			const float vv = c.beta2 * st.m2[i] + (1.f - c.beta2) * (g * g);
			st.m1[i] = mm;
			st.m2[i] = vv;
			const uint32_t s = st.steps[i] + 1;
			st.steps[i] = s;
			const float lr_s = adam_step_size(c, lr, s, st.bias_tab);
			w = w - lr_s / (sqrtf(vv) + c.eps) * mm;
			st.w32[i] = w;
			const f16 h = (f16)w;
			st.w16[i] = h;
			if (st.frags && i < n_matrix) {
				const uint32_t q0 = st.fragmap[2 * i], q1 = st.fragmap[2 * i + 1];
				if (q0 != ~0u) st.frags[q0] = h;
				if (q1 != ~0u) st.frags[q1] = h;
			}
		}
		if (st.ema32) {
			const float debias = 1.f - powf(c.ema_decay, (float)(step + 1));
			const float v = ema_step(st.ema32[i], c.ema_decay, (1.f - c.ema_decay) * w);
			st.ema32[i] = v;
			st.ema16[i] = (f16)(v / debias);
		}
	}
}

// Four consecutive parameters per thread with 16-B loads/stores (8-B for the fp16 arrays): the update
// is HBM-bound once the state outgrows the Infinity Cache (C5: 105 M params, 4.8 GB per step). A
// group whose four parameters are all lazily skipped (grid entries without gradient) reads only the
// gradient and the EMA inputs. Same per-parameter arithmetic as k_adam_ema.
__global__ void __launch_bounds__(256) k_adam_ema4(const uint32_t n4, const uint32_t n_matrix, const float loss_scale,
                                                   const AdamConfig c_arg, const AdamState st) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n4) return;
	const AdamConfig c = st.cfg_dev ? *st.cfg_dev : c_arg;
	const uint32_t i0 = 4 * t;
	const uint32_t step = (st.step_base ? *st.step_base : 0u) + st.step_add;
	const f16x4 gh = *(const f16x4*)(st.g16 + i0);
	float g[4];
	bool act[4], any = false;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		g[k] = (float)gh[k] / loss_scale;
		act[k] = !(i0 + k >= n_matrix && g[k] == 0.f);
		any |= act[k];
	}
	if (!any && !st.ema32) return;
	f32x4 w = *(const f32x4*)(st.w32 + i0);
	if (any) {
		const float lr = lr_schedule(c, step);
		f32x4 m1 = *(const f32x4*)(st.m1 + i0), m2 = *(const f32x4*)(st.m2 + i0);
		uint4 sp = *(const uint4*)(st.steps + i0);
		uint32_t sv[4] = {sp.x, sp.y, sp.z, sp.w};
		f16x4 wh = {};
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			if (act[k]) {
				float gk = g[k];
				if (i0 + k < n_matrix) gk += c.l2 * w[k];
				const float mm = c.beta1 * m1[k] + (1.f - c.beta1) * gk;
				const float vv = c.beta2 * m2[k] + (1.f - c.beta2) * (gk * gk);
				m1[k] = mm;
				m2[k] = vv;
				const uint32_t sk = sv[k] + 1;
				sv[k] = sk;
				const float lr_s = adam_step_size(c, lr, sk, st.bias_tab);
				w[k] = w[k] - lr_s / (sqrtf(vv) + c.eps) * mm;
			}
			wh[k] = (f16)w[k];
		}
		*(f32x4*)(st.m1 + i0) = m1;
		*(f32x4*)(st.m2 + i0) = m2;
		*(uint4*)(st.steps + i0) = uint4{sv[0], sv[1], sv[2], sv[3]};
		*(f32x4*)(st.w32 + i0) = w;
		*(f16x4*)(st.w16 + i0) = wh;
		if (st.frags && i0 < n_matrix) {
#pragma unroll
			for (int k = 0; k < 4; ++k) {
				if (i0 + k >= n_matrix || !act[k]) continue;
				const uint32_t q0 = st.fragmap[2 * (i0 + k)], q1 = st.fragmap[2 * (i0 + k) + 1];
				if (q0 != ~0u) st.frags[q0] = wh[k];
				if (q1 != ~0u) st.frags[q1] = wh[k];
			}
		}
	}
	if (st.ema32) {
		const float debias = 1.f - powf(c.ema_decay, (float)(step + 1));
		f32x4 e = *(const f32x4*)(st.ema32 + i0);
		f16x4 eh;
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			e[k] = ema_step(e[k], c.ema_decay, (1.f - c.ema_decay) * w[k]);
			eh[k] = (f16)(e[k] / debias);
		}
		*(f32x4*)(st.ema32 + i0) = e;
		*(f16x4*)(st.ema16 + i0) = eh;
	}
}

// ---- lazy-EMA layout ------------------------------------------------------------------------

__device__ __forceinline__ void lazy_load(const AdamState& st, uint32_t i0, uint32_t n_matrix, float loss_scale, LazyGroup& G) {
	G.i0 = i0;
	f16x4 gh;
	if (st.g32) {  // the ranks' fp32 sum, rounded to fp16 once (= the all-reduce path's narrowing)
		const f32x4 g = *(const f32x4*)(st.g32 + i0);
		gh = f16x4{(f16)g[0], (f16)g[1], (f16)g[2], (f16)g[3]};
	} else {
		gh = *(const f16x4*)(st.g16 + i0);
	}
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		G.g[k] = (float)gh[k] / loss_scale;
		G.act[k] = !(i0 + k >= n_matrix && G.g[k] == 0.f);
	}
	G.any[0] = G.act[0] || G.act[1];
	G.any[1] = G.act[2] || G.act[3];
#pragma unroll
	for (int r = 0; r < 2; ++r) {
		if (!G.any[r]) continue;
		const f32x4* rp = (const f32x4*)(st.rec + (i0 >> 1) + r);
		G.q[r][0] = rp[0]; G.q[r][1] = rp[1]; G.q[r][2] = rp[2];
	}
}

// groups [g0, g0 + n4) of 4 parameters
__global__ void __launch_bounds__(256) k_adam_lazy4(const uint32_t g0, const uint32_t n4, const uint32_t n_matrix, const float loss_scale,
                                                    const AdamConfig c_arg, const AdamState st) {
	const uint32_t half = (n4 + 1) / 2;
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= half) return;
	const AdamConfig c = st.cfg_dev ? *st.cfg_dev : c_arg;
	const uint32_t step = (st.step_base ? *st.step_base : 0u) + st.step_add;
	const bool two = t + half < n4;
	LazyGroup A, B;
	lazy_load(st, 4 * (g0 + t), n_matrix, loss_scale, A);
	if (two) lazy_load(st, 4 * (g0 + t + half), n_matrix, loss_scale, B);
	lazy_update(st, c, step, n_matrix, A);
	if (two) lazy_update(st, c, step, n_matrix, B);
}

__global__ void k_ema_materialize(uint32_t n, float d, uint32_t steps_done, uint32_t closed, const AdamState st) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const float debias = 1.f - powf(d, (float)steps_done);  // on the device, as the eager kernel computes it
	AdamRec* rp = st.rec + (i >> 1);
	const uint32_t k = i & 1u;
	float e = rp->ema[k];
	const uint32_t done = rp->done[k];
	if (done < steps_done) {
		e = ema_catch_up(e, rp->w[k], d, done, steps_done, closed);
		rp->ema[k] = e;
		rp->done[k] = steps_done;
	}
	st.ema16[i] = (f16)(e / debias);
}

__global__ void k_rec_to_soa(uint32_t n, const AdamRec* rec, float* m1, float* m2, float* ema32, uint32_t* steps) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const AdamRec& r = rec[i >> 1];
	const uint32_t k = i & 1u;
	m1[i] = r.m1[k]; m2[i] = r.m2[k]; ema32[i] = r.ema[k]; steps[i] = r.steps[k];
}

__global__ void k_soa_to_rec(uint32_t n, const float* m1, const float* m2, const float* ema32, const uint32_t* steps, uint32_t done,
                             AdamRec* rec) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	AdamRec& r = rec[i >> 1];
	const uint32_t k = i & 1u;
	r.m1[k] = m1[i]; r.m2[k] = m2[i]; r.ema[k] = ema32[i]; r.steps[k] = steps[i]; r.done[k] = done;
}

__global__ void k_rec_weights(uint32_t n, AdamRec* rec, float* w32, bool to_rec) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	if (to_rec) rec[i >> 1].w[i & 1u] = w32[i];
	else w32[i] = rec[i >> 1].w[i & 1u];
}

void ema_materialize(const AdamConfig& c, uint32_t n, uint32_t steps_done, const AdamState& st, hipStream_t s) {
	if (c.ema_decay <= 0.f || steps_done == 0 || n == 0) return;
	k_ema_materialize<<<div_round_up(n, 256), 256, 0, s>>>(n, c.ema_decay, steps_done, c.ema_closed_form, st);
	NGP_HIP(hipGetLastError());
}

void adam_rec_to_soa(uint32_t n, const AdamRec* rec, float* m1, float* m2, float* ema32, uint32_t* steps, hipStream_t s) {
	if (n) k_rec_to_soa<<<div_round_up(n, 256), 256, 0, s>>>(n, rec, m1, m2, ema32, steps);
	NGP_HIP(hipGetLastError());
}

void adam_soa_to_rec(uint32_t n, const float* m1, const float* m2, const float* ema32, const uint32_t* steps, uint32_t done,
                     AdamRec* rec, hipStream_t s) {
	if (n) k_soa_to_rec<<<div_round_up(n, 256), 256, 0, s>>>(n, m1, m2, ema32, steps, done, rec);
	NGP_HIP(hipGetLastError());
}

void adam_rec_weights(uint32_t n, AdamRec* rec, float* w32, bool to_rec, hipStream_t s) {
	if (n) k_rec_weights<<<div_round_up(n, 256), 256, 0, s>>>(n, rec, w32, to_rec);
	NGP_HIP(hipGetLastError());
}

__global__ void k_set_ctl(uint32_t* ctl, uint32_t step, const AdamConfig c) {
	ctl[0] = step;
	*(AdamConfig*)(ctl + CTL_CFG) = c;
}

float AdamConfig::lr_at(uint32_t step) const {
	float r = lr;
	if (decay_interval == 0 || step < decay_start) return r;
	const uint32_t k = (step - decay_start) / decay_interval + 1;
	for (uint32_t i = 0; i < k; ++i) r *= decay_base;
	return r;
}

void adam_ema_update(const AdamConfig& c, uint32_t n, uint32_t n_matrix, float loss_scale, const AdamState& st, hipStream_t s) {
	if (st.rec) {
		NGP_CHECK(n % 4 == 0 && ((uintptr_t)st.w32 | (uintptr_t)st.w16 | (uintptr_t)st.g16 | (uintptr_t)st.rec) % 16 == 0,
		          "lazy-EMA optimizer: parameters must be 16-B aligned groups of 4");
		k_adam_lazy4<<<div_round_up((n / 4 + 1) / 2, 256), 256, 0, s>>>(0, n / 4, n_matrix, loss_scale, c, st);
		NGP_HIP(hipGetLastError());
		return;
	}
	AdamState a = st;
	if (c.ema_decay <= 0.f) a.ema32 = nullptr;
	const bool aligned = ((uintptr_t)a.w32 | (uintptr_t)a.m1 | (uintptr_t)a.m2 | (uintptr_t)a.steps | (uintptr_t)a.ema32 |
	                      (uintptr_t)a.w16 | (uintptr_t)a.g16 | (uintptr_t)a.ema16) % 16 == 0;
	const uint32_t n4 = aligned ? n / 4 : 0;
	if (n4) k_adam_ema4<<<div_round_up(n4, 256), 256, 0, s>>>(n4, n_matrix, loss_scale, c, a);
	if (4 * n4 < n) k_adam_ema<<<div_round_up(n - 4 * n4, 256), 256, 0, s>>>(4 * n4, n, n_matrix, loss_scale, c, a);
	NGP_HIP(hipGetLastError());
}

void adam_lazy_range(const AdamConfig& c, uint32_t lo, uint32_t hi, uint32_t n_matrix, float loss_scale, const AdamState& st,
                     hipStream_t s) {
	NGP_CHECK(st.rec && lo % 4 == 0 && hi % 4 == 0 && lo <= hi, "lazy range update: record layout, groups of 4");
	NGP_CHECK(((uintptr_t)st.w16 | (uintptr_t)st.rec | (uintptr_t)(st.g32 ? (const void*)st.g32 : (const void*)st.g16)) % 16 == 0,
	          "lazy range update: 16-B aligned buffers");
	const uint32_t n4 = (hi - lo) / 4;
	if (n4) k_adam_lazy4<<<div_round_up((n4 + 1) / 2, 256), 256, 0, s>>>(lo / 4, n4, n_matrix, loss_scale, c, st);
	NGP_HIP(hipGetLastError());
}

void set_device_ctl(uint32_t* ctl, uint32_t step, const AdamConfig& c, hipStream_t s) {
	k_set_ctl<<<1, 1, 0, s>>>(ctl, step, c);
	NGP_HIP(hipGetLastError());
}

}  // namespace ngp
