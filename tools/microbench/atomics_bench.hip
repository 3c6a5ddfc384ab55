// Microbenchmark: rates that decide the hash-grid backward design on gfx950.
// (a) scattered f32 global atomics, (b) scattered packed-f16 atomics (lane pairs on one 8-B entry),
// (c) scattered plain stores, (d) random 8-B gathers (grid forward proxy), (e) stream copy,
// (f) LDS-privatised f32 accumulation (ds_add_f32) then one contiguous flush.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ void k_atomic_f32(float* t, uint32_t mask, uint32_t n, uint32_t seed) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t idx = hash32(i ^ seed) & mask;
  atomicAdd(t + idx, 1.0f);
}

__global__ void k_atomic_pkf16(h2* t, uint32_t mask, uint32_t n, uint32_t seed) {
  // lanes 2k and 2k+1 update the two halves of one 8-byte (4 x f16) entry
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t e = hash32((i >> 1) ^ seed) & mask;
  __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2*)(t + 2 * e + (i & 1)), h2{(_Float16)1.0f, (_Float16)1.0f});
}

__global__ void k_store_f32(float* t, uint32_t mask, uint32_t n, uint32_t seed) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t idx = hash32(i ^ seed) & mask;
  t[idx] = 1.0f;
}

__global__ void k_gather8(const uint2* t, uint32_t mask, uint32_t n, uint32_t seed, uint2* out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint2 acc = {0, 0};
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    uint32_t idx = hash32((i * 8 + c) ^ seed) & mask;
    uint2 v = t[idx];
    acc.x ^= v.x; acc.y += v.y;
  }
  out[i] = acc;
}

__global__ void k_copy(const float4* a, float4* b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) b[i] = a[i];
}

// LDS privatisation: each block owns a 16K-entry f32 chunk (64 KB), processes `per_block` random contributions
__global__ void k_lds_priv(float* t, uint32_t per_block, uint32_t seed) {
  extern __shared__ float s[];
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) s[j] = 0.f;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < per_block; k += blockDim.x) {
    uint32_t idx = hash32((blockIdx.x * per_block + k) ^ seed) & 16383;
    atomicAdd(s + idx, 1.0f);
  }
  __syncthreads();
  float* dst = t + (size_t)blockIdx.x * 16384;
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) dst[j] = s[j];
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
  const uint32_t N = 1u << 24;  // 16.8M ops
  const int reps = 10;
  for (uint32_t log2T : {20u, 22u, 26u}) {   // table entries: 4 MB, 16 MB, 256 MB (f32)
    uint32_t T = 1u << log2T;
    float* t; CK(hipMalloc(&t, (size_t)T * 8));
    CK(hipMemset(t, 0, (size_t)T * 8));
    float ms;
    ms = time_ms([&] { k_atomic_f32<<<N / 256, 256>>>(t, T - 1, N, 7); }, reps);
    printf("T=2^%u f32-atomic scattered : %.3f ms  %.2f G atom/s\n", log2T, ms, N / ms / 1e6);
    ms = time_ms([&] { k_atomic_pkf16<<<N / 256, 256>>>((h2*)t, (T / 2) - 1, N, 7); }, reps);
    printf("T=2^%u pkf16-atomic pairs   : %.3f ms  %.2f G lane-atom/s\n", log2T, ms, N / ms / 1e6);
    ms = time_ms([&] { k_store_f32<<<N / 256, 256>>>(t, T - 1, N, 7); }, reps);
    printf("T=2^%u f32 scattered store  : %.3f ms  %.2f G st/s\n", log2T, ms, N / ms / 1e6);
    uint2* o; CK(hipMalloc(&o, (size_t)N / 8 * 8));
    ms = time_ms([&] { k_gather8<<<N / 8 / 256, 256>>>((const uint2*)t, T - 1, N / 8, 7, o); }, reps);
    printf("T=2^%u random 8B gathers     : %.3f ms  %.2f G ld/s  %.1f GB/s\n", log2T, ms, N / ms / 1e6, N * 8.0 / ms / 1e6);
    CK(hipFree(o));
    CK(hipFree(t));
  }
  {
    size_t n = (size_t)1 << 28;  // 1 GiB per buffer in float4 units /4
    float4 *a, *b; CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 0, n * 4));
    float ms = time_ms([&] { k_copy<<<4096, 256>>>(a, b, n / 4); }, reps);
    printf("copy 1 GiB: %.3f ms  %.1f GB/s (r+w)\n", ms, 2.0 * n * 4 / ms / 1e6);
    CK(hipFree(a)); CK(hipFree(b));
  }
  {
    uint32_t blocks = 1024, per_block = N / blocks;
    float* t; CK(hipMalloc(&t, (size_t)blocks * 16384 * 4));
    float ms = time_ms([&] { k_lds_priv<<<blocks, 512, 65536>>>(t, per_block, 7); }, reps);
    printf("LDS-private f32 accumulate: %.3f ms  %.2f G add/s\n", ms, N / ms / 1e6);
    CK(hipFree(t));
  }
  return 0;
}
