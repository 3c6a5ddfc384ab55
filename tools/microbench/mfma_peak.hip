// Microbenchmark: dense fp16 MFMA peak of the gfx950 chip, the denominator of the fused MLP's
// roofline (bench.py MFMA_F16_PEAK_TFLOPS). Every wave runs a chain of independent MFMAs on A
// accumulators held in registers (no memory traffic inside the loop), all CUs busy, 1-4 waves per
// SIMD; reports TFLOP/s for the two shapes the engine issues:
//   v_mfma_f32_32x32x16_f16  (layer chains of k_nerf_mlp*, 32768 FLOP per instruction)
//   v_mfma_f32_16x16x32_f16  (dW accumulation, 16384 FLOP per instruction)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench/bin/mfma_peak tools/microbench/mfma_peak.hip
// Output: one JSON line per (shape, accumulators, waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

template <int NACC>
__global__ void __launch_bounds__(256) k32(float* out, float seed) {
	f16x8 a, b;
	for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(seed * (threadIdx.x + i)); b[i] = (_Float16)(seed * (i - (int)threadIdx.x)); }
	f32x16 c[NACC];
	for (int k = 0; k < NACC; ++k) for (int i = 0; i < 16; ++i) c[k][i] = 0.f;
	for (int it = 0; it < ITERS; ++it) {
#pragma unroll
		for (int k = 0; k < NACC; ++k) c[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c[k], 0, 0, 0);
	}
	float s = 0.f;
	for (int k = 0; k < NACC; ++k) for (int i = 0; i < 16; ++i) s += c[k][i];
	if (s == 12345.f) out[blockIdx.x] = s;
}

template <int NACC>
__global__ void __launch_bounds__(256) k16(float* out, float seed) {
	f16x8 a, b;
	for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(seed * (threadIdx.x + i)); b[i] = (_Float16)(seed * (i - (int)threadIdx.x)); }
	f32x4 c[NACC];
	for (int k = 0; k < NACC; ++k) for (int i = 0; i < 4; ++i) c[k][i] = 0.f;
	for (int it = 0; it < ITERS; ++it) {
#pragma unroll
		for (int k = 0; k < NACC; ++k) c[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c[k], 0, 0, 0);
	}
	float s = 0.f;
	for (int k = 0; k < NACC; ++k) for (int i = 0; i < 4; ++i) s += c[k][i];
	if (s == 12345.f) out[blockIdx.x] = s;
}

template <typename K>
void run(const char* shape, K kern, int nacc, double flop_per_inst, int n_cu, float* out) {
	for (int wps = 1; wps <= 4; wps *= 2) {  // 256-thread blocks = one wave per SIMD each
		const int blocks = n_cu * wps;
		hipEvent_t e0, e1;
		CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
		kern<<<blocks, 256>>>(out, 1e-3f);  // warm-up
		CK(hipDeviceSynchronize());
		float best = 1e30f;
		for (int r = 0; r < 5; ++r) {
			CK(hipEventRecord(e0));
			kern<<<blocks, 256>>>(out, 1e-3f);
			CK(hipEventRecord(e1));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			if (ms < best) best = ms;
		}
		const double flop = (double)blocks * 4 * ITERS * nacc * flop_per_inst;
		printf("{\"shape\": \"%s\", \"accumulators\": %d, \"waves_per_simd\": %d, \"cus\": %d, \"best_ms\": %.4f, \"TFLOPs\": %.1f}\n",
		       shape, nacc, wps, n_cu, best, flop / (best * 1e-3) / 1e12);
		CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
	}
}

int main() {
	hipDeviceProp_t prop;
	CK(hipGetDeviceProperties(&prop, 0));
	const int n_cu = prop.multiProcessorCount;
	float* out;
	CK(hipMalloc(&out, 1 << 20));
	printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.gcnArchName, n_cu, prop.clockRate);
	run("32x32x16_f16", k32<1>, 1, 32768.0, n_cu, out);
	run("32x32x16_f16", k32<2>, 2, 32768.0, n_cu, out);
	run("32x32x16_f16", k32<4>, 4, 32768.0, n_cu, out);
	run("16x16x32_f16", k16<1>, 1, 16384.0, n_cu, out);
	run("16x16x32_f16", k16<4>, 4, 16384.0, n_cu, out);
	run("16x16x32_f16", k16<8>, 8, 16384.0, n_cu, out);
	CK(hipFree(out));
	return 0;
}
