// Microbenchmark 3: LDS throughput per op type with a tight loop (no mode branches), to calibrate
// the LDS-accumulation design of the hash-grid backward.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 1024;
constexpr int WIN = 8192;  // floats (32 KB)

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, uint32_t seed, uint32_t stride_mode) {
  __shared__ float s[WIN];
  for (int j = threadIdx.x; j < WIN; j += blockDim.x) s[j] = 0.f;
  __syncthreads();
  uint32_t x = (threadIdx.x * 2654435761u) ^ seed ^ (blockIdx.x << 16);
  float acc = 0.f;
#pragma unroll 8
  for (int it = 0; it < ITERS; ++it) {
    uint32_t a;
    if (stride_mode == 0) { x = x * 1664525u + 1013904223u; a = (x >> 10) & (WIN - 1); }
    else if (stride_mode == 1) a = (it * 64 + (threadIdx.x & 63) + (threadIdx.x >> 6) * 1024) & (WIN - 1);
    else if (stride_mode == 2) a = (it * 64 + (threadIdx.x >> 6) * 1024) & (WIN - 1);             // wave: one address
    else a = (it * 64 + ((threadIdx.x & 63) >> 3) * 2 + (threadIdx.x >> 6) * 1024) & (WIN - 1);  // 8 lanes/address
    if (OP == 0) __hip_atomic_fetch_add(s + a, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (OP == 1) __builtin_amdgcn_ds_atomic_fadd_v2f16((__attribute__((address_space(3))) h2*)(s + a), h2{(_Float16)1, (_Float16)1});
    else if (OP == 2) atomicAdd((uint32_t*)(s + a), 1u);
    else if (OP == 3) s[a] = (float)it;
    else if (OP == 4) acc += s[a];
    else if (OP == 5) { float v = s[a]; s[a] = v + 1.0f; }  // non-atomic RMW
    else if (OP == 6) atomicAdd((unsigned long long*)(s + (a & ~1u)), 1ull);
  }
  __syncthreads();
  if (acc == 12345.f) out[0] = acc;
  for (int j = threadIdx.x; j < WIN; j += blockDim.x) out[(size_t)blockIdx.x * WIN + j] = s[j];
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int blocks = 256 * 8;
  float* o; CK(hipMalloc(&o, (size_t)blocks * WIN * 4));
  const char* names[] = {"ds_add_f32", "ds_pk_add_f16", "ds_add_u32", "ds_write_b32", "ds_read_b32", "read+add+write (non-atomic)", "ds_add_u64"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int op = 0; op < 7; ++op) {
      float ms = 0;
      auto run = [&](auto kern) { ms = time_ms([&] { kern<<<blocks, 256>>>(o, 7, mode); }, 5); };
      switch (op) {
        case 0: run(k<0>); break; case 1: run(k<1>); break; case 2: run(k<2>); break;
        case 3: run(k<3>); break; case 4: run(k<4>); break; case 5: run(k<5>); break; case 6: run(k<6>); break;
      }
      double lanes = (double)blocks * 256 * ITERS;
      printf("%-30s %-10s %.3f ms  %.1f G lane-op/s  %.2f lane-op/clk/CU (2.4GHz)\n", names[op], (const char*[]){"random", "contig", "same/wave", "8 lanes/addr"}[mode],
             ms, lanes / ms / 1e6, lanes / ms / 1e6 / 256 / 2.4);
    }
  }
  return 0;
}
