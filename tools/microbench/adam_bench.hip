// adam_bench.hip — variants of the fused Ema o Adam update (optimizer.hip k_adam_ema4) on the C5 and C2
// parameter counts with a synthetic lazy-skip pattern (grid entries get a gradient with the touch
// probability the real batches produce: C5 ~28 % of entries, C2 ~96 %), timed with HIP events.
//   v0  k_adam_ema4 as in the engine (4 params / thread; w32 loaded after the skip test)
//   v1  g16, w32, ema32 issued together before the skip test
//   v2  v1 with 8 params / thread (two 4-groups interleaved: twice the loads in flight)
//   v3  v1 with nontemporal loads and stores on the streamed state
//   v4  v2 with nontemporal loads and stores
//   v5  v0 with m1, m2, steps, ema32 interleaved per 4-group (one 64-B record: 5 streams instead of 9)
// Prints one JSON line per (config, variant): avg/best ms and algorithmic GB/s (46 B per updated
// parameter, 16 B per skipped one). Also checks every variant leaves bit-identical state.
// Build: hipcc --offload-arch=gfx950 -O3 -o adam_bench adam_bench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef _Float16 f16;
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Cfg { float lr, beta1, beta2, eps, l2, ema_decay; };
struct St { float* w32; f16* w16; const f16* g16; float* m1; float* m2; uint32_t* steps; float* ema32; f16* ema16; f32x4* rec; };

template <bool NT, typename T> __device__ __forceinline__ T ld(const T* p) {
	if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT, typename T> __device__ __forceinline__ void st_(T* p, T v) {
	if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

// one 4-group: the engine's arithmetic
template <bool NT>
__device__ __forceinline__ void group(const St& s, const Cfg& c, uint32_t i0, uint32_t n_matrix, float ls, uint32_t step, f16x4 gh,
                                      f32x4 w, f32x4 e) {
	float g[4];
	bool act[4], any = false;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		g[k] = (float)gh[k] / ls;
		act[k] = !(i0 + k >= n_matrix && g[k] == 0.f);
		any |= act[k];
	}
	if (any) {
		f32x4 m1 = ld<NT>((const f32x4*)(s.m1 + i0)), m2 = ld<NT>((const f32x4*)(s.m2 + i0));
		u32x4 sp = ld<NT>((const u32x4*)(s.steps + i0));
		f16x4 wh;
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			if (act[k]) {
				float gk = g[k];
				if (i0 + k < n_matrix) gk += c.l2 * w[k];
				const float mm = c.beta1 * m1[k] + (1.f - c.beta1) * gk;
				const float vv = c.beta2 * m2[k] + (1.f - c.beta2) * (gk * gk);
				m1[k] = mm; m2[k] = vv;
				const uint32_t sk = sp[k] + 1;
				sp[k] = sk;
				const float lr_s = c.lr * sqrtf(1.f - powf(c.beta2, (float)sk)) / (1.f - powf(c.beta1, (float)sk));
				w[k] = w[k] - lr_s / (sqrtf(vv) + c.eps) * mm;
			}
			wh[k] = (f16)w[k];
		}
		st_<NT>((f32x4*)(s.m1 + i0), m1);
		st_<NT>((f32x4*)(s.m2 + i0), m2);
		st_<NT>((u32x4*)(s.steps + i0), sp);
		st_<NT>((f32x4*)(s.w32 + i0), w);
		st_<NT>((f16x4*)(s.w16 + i0), wh);
	}
	const float debias = 1.f - powf(c.ema_decay, (float)(step + 1));
	f16x4 eh;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		e[k] = c.ema_decay * e[k] + (1.f - c.ema_decay) * w[k];
		eh[k] = (f16)(e[k] / debias);
	}
	st_<NT>((f32x4*)(s.ema32 + i0), e);
	st_<NT>((f16x4*)(s.ema16 + i0), eh);
}

__global__ void __launch_bounds__(256) v0(uint32_t n4, uint32_t n_matrix, float ls, Cfg c, St s, uint32_t step) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n4) return;
	const uint32_t i0 = 4 * t;
	const f16x4 gh = *(const f16x4*)(s.g16 + i0);
	bool any = false;
#pragma unroll
	for (int k = 0; k < 4; ++k) any |= !(i0 + k >= n_matrix && (float)gh[k] == 0.f);
	if (!any) {  // the engine's order: w32 / ema32 are loaded after the test
		asm volatile("" ::: "memory");
	}
	const f32x4 w = *(const f32x4*)(s.w32 + i0);
	const f32x4 e = *(const f32x4*)(s.ema32 + i0);
	group<false>(s, c, i0, n_matrix, ls, step, gh, w, e);
}

template <bool NT>
__global__ void __launch_bounds__(256) v1(uint32_t n4, uint32_t n_matrix, float ls, Cfg c, St s, uint32_t step) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n4) return;
	const uint32_t i0 = 4 * t;
	const f16x4 gh = ld<NT>((const f16x4*)(s.g16 + i0));
	const f32x4 w = ld<NT>((const f32x4*)(s.w32 + i0));
	const f32x4 e = ld<NT>((const f32x4*)(s.ema32 + i0));
	group<NT>(s, c, i0, n_matrix, ls, step, gh, w, e);
}

// two groups per thread, 1024 params apart per wave-instruction (coalesced), all first loads issued together
template <bool NT>
__global__ void __launch_bounds__(256) v2(uint32_t n4, uint32_t n_matrix, float ls, Cfg c, St s, uint32_t step) {
	const uint32_t t = blockIdx.x * 512 + threadIdx.x;
	const uint32_t ta = t, tb = t + 256;
	const bool va = ta < n4, vb = tb < n4;
	const uint32_t ia = 4 * (va ? ta : 0), ib = 4 * (vb ? tb : 0);
	const f16x4 ga = ld<NT>((const f16x4*)(s.g16 + ia)), gb = ld<NT>((const f16x4*)(s.g16 + ib));
	const f32x4 wa = ld<NT>((const f32x4*)(s.w32 + ia)), wb = ld<NT>((const f32x4*)(s.w32 + ib));
	const f32x4 ea = ld<NT>((const f32x4*)(s.ema32 + ia)), eb = ld<NT>((const f32x4*)(s.ema32 + ib));
	if (va) group<NT>(s, c, ia, n_matrix, ls, step, ga, wa, ea);
	if (vb) group<NT>(s, c, ib, n_matrix, ls, step, gb, wb, eb);
}

// interleaved state: rec[4t + 0..3] = m1, m2, steps (as bits), ema32 of group t
__global__ void __launch_bounds__(256) v5(uint32_t n4, uint32_t n_matrix, float ls, Cfg c, St s, uint32_t step) {
	const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
	if (t >= n4) return;
	const uint32_t i0 = 4 * t;
	const f16x4 gh = *(const f16x4*)(s.g16 + i0);
	float g[4];
	bool act[4], any = false;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		g[k] = (float)gh[k] / ls;
		act[k] = !(i0 + k >= n_matrix && g[k] == 0.f);
		any |= act[k];
	}
	f32x4 w = *(const f32x4*)(s.w32 + i0);
	f32x4* r = s.rec + 4 * (size_t)t;
	f32x4 e = r[3];
	if (any) {
		f32x4 m1 = r[0], m2 = r[1];
		u32x4 sp = __builtin_bit_cast(u32x4, r[2]);
		f16x4 wh;
#pragma unroll
		for (int k = 0; k < 4; ++k) {
			if (act[k]) {
				float gk = g[k];
				if (i0 + k < n_matrix) gk += c.l2 * w[k];
				const float mm = c.beta1 * m1[k] + (1.f - c.beta1) * gk;
				const float vv = c.beta2 * m2[k] + (1.f - c.beta2) * (gk * gk);
				m1[k] = mm; m2[k] = vv;
				const uint32_t sk = sp[k] + 1;
				sp[k] = sk;
				const float lr_s = c.lr * sqrtf(1.f - powf(c.beta2, (float)sk)) / (1.f - powf(c.beta1, (float)sk));
				w[k] = w[k] - lr_s / (sqrtf(vv) + c.eps) * mm;
			}
			wh[k] = (f16)w[k];
		}
		r[0] = m1; r[1] = m2; r[2] = __builtin_bit_cast(f32x4, sp);
		*(f32x4*)(s.w32 + i0) = w;
		*(f16x4*)(s.w16 + i0) = wh;
	}
	const float debias = 1.f - powf(c.ema_decay, (float)(step + 1));
	f16x4 eh;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		e[k] = c.ema_decay * e[k] + (1.f - c.ema_decay) * w[k];
		eh[k] = (f16)(e[k] / debias);
	}
	r[3] = e;
	*(f16x4*)(s.ema16 + i0) = eh;
}

int main() {
	struct Conf { const char* name; uint32_t n, n_matrix; double p_active; } confs[] = {
		{"C5", 105462784u, 7168u, 0.28}, {"C2", 3302400u, 9216u, 0.96}};
	for (const Conf& cf : confs) {
		const uint32_t n = cf.n;
		std::vector<f16> g(n);
		uint64_t x = 88172645463325252ull;
		auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return (double)(x >> 11) / 9007199254740992.0; };
		uint64_t updated = 0;
		for (uint32_t i = 0; i < n; i += 2) {  // F = 2 (C5) / entries of 2 params: both or neither
			const bool a = i < cf.n_matrix || rnd() < cf.p_active;
			const f16 v = a ? (f16)(rnd() * 2.0 - 1.0) : (f16)0.f;
			g[i] = v;
			if (i + 1 < n) g[i + 1] = a ? (f16)(rnd() * 2.0 - 1.0) : (f16)0.f;
			updated += a ? 2 : 0;
		}
		std::vector<float> w0(n);
		for (uint32_t i = 0; i < n; ++i) w0[i] = (float)(rnd() * 2e-4 - 1e-4);
		St s;
		CHECK(hipMalloc(&s.w32, (size_t)n * 4)); CHECK(hipMalloc(&s.w16, (size_t)n * 2)); CHECK(hipMalloc((void**)&s.g16, (size_t)n * 2));
		CHECK(hipMalloc(&s.m1, (size_t)n * 4)); CHECK(hipMalloc(&s.m2, (size_t)n * 4)); CHECK(hipMalloc(&s.steps, (size_t)n * 4));
		CHECK(hipMalloc(&s.ema32, (size_t)n * 4)); CHECK(hipMalloc(&s.ema16, (size_t)n * 2));
		CHECK(hipMalloc(&s.rec, (size_t)n * 16));
		CHECK(hipMemcpy((void*)s.g16, g.data(), (size_t)n * 2, hipMemcpyHostToDevice));
		void* flush;
		const size_t flush_bytes = (size_t)512 << 20;
		CHECK(hipMalloc(&flush, flush_bytes));
		auto reset = [&]() {
			CHECK(hipMemcpy(s.w32, w0.data(), (size_t)n * 4, hipMemcpyHostToDevice));
			CHECK(hipMemcpy(s.ema32, w0.data(), (size_t)n * 4, hipMemcpyHostToDevice));
			CHECK(hipMemset(s.m1, 0, (size_t)n * 4)); CHECK(hipMemset(s.m2, 0, (size_t)n * 4)); CHECK(hipMemset(s.steps, 0, (size_t)n * 4));
			CHECK(hipMemset(s.rec, 0, (size_t)n * 16));
			CHECK(hipMemcpy2D((char*)s.rec + 48, 64, w0.data(), 16, 16, n / 4, hipMemcpyHostToDevice));
		};
		const Cfg c{1e-2f, 0.9f, 0.99f, 1e-15f, 1e-6f, 0.95f};
		const uint32_t n4 = n / 4;
		const double bytes = 46.0 * updated + 16.0 * (n - updated);
		hipEvent_t e0, e1;
		CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
		std::vector<float> ref;
		bool interleaved = false;
		auto run = [&](const char* name, auto launch) {
			reset();
			CHECK(hipDeviceSynchronize());
			float tot = 0.f, best = 1e30f;
			const int R = 10;
			for (int r = 0; r < R + 2; ++r) {
				if (cf.n < 20000000) CHECK(hipMemsetAsync(flush, r, flush_bytes));  // C2: run from a cold cache like the NeRF step
				CHECK(hipEventRecord(e0));
				launch(r);
				CHECK(hipEventRecord(e1));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (r >= 2) { tot += ms; best = ms < best ? ms : best; }
			}
			std::vector<float> out(n);
			if (interleaved) CHECK(hipMemcpy2D(out.data(), 16, (char*)s.rec + 48, 64, 16, n / 4, hipMemcpyDeviceToHost));
			else CHECK(hipMemcpy(out.data(), s.ema32, (size_t)n * 4, hipMemcpyDeviceToHost));
			bool same = true;
			if (ref.empty()) ref = out; else same = memcmp(ref.data(), out.data(), (size_t)n * 4) == 0;
			printf("{\"config\": \"%s\", \"variant\": \"%s\", \"n\": %u, \"updated\": %llu, \"avg_ms\": %.4f, \"best_ms\": %.4f, "
			       "\"algo_GBps\": %.1f, \"identical\": %s}\n",
			       cf.name, name, n, (unsigned long long)updated, tot / R, best, bytes / (tot / R) / 1e6, same ? "true" : "false");
			fflush(stdout);
		};
		const float ls = 128.f;
		run("v0", [&](int r) { v0<<<(n4 + 255) / 256, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		run("v1", [&](int r) { v1<false><<<(n4 + 255) / 256, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		run("v2", [&](int r) { v2<false><<<(n4 + 511) / 512, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		run("v3", [&](int r) { v1<true><<<(n4 + 255) / 256, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		run("v4", [&](int r) { v2<true><<<(n4 + 511) / 512, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		interleaved = true;
		run("v5", [&](int r) { v5<<<(n4 + 255) / 256, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		interleaved = false;
		run("v0", [&](int r) { v0<<<(n4 + 255) / 256, 256>>>(n4, cf.n_matrix, ls, c, s, r); });
		CHECK(hipFree(s.w32)); CHECK(hipFree(s.w16)); CHECK(hipFree((void*)s.g16)); CHECK(hipFree(s.m1)); CHECK(hipFree(s.m2));
		CHECK(hipFree(s.steps)); CHECK(hipFree(s.ema32)); CHECK(hipFree(s.ema16)); CHECK(hipFree(s.rec)); CHECK(hipFree(flush));
	}
	return 0;
}
