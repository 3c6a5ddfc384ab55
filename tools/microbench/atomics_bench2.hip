// Microbenchmark 2: how many memory-side atomic requests does one wave-instruction cost when its lanes
// share addresses / 64-B segments? And LDS atomic variants. Decides the hash-grid backward design.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// lanes_per_addr lanes share one dword address; addrs_per_seg distinct dwords per 64-B segment.
__global__ void k_global(float* t, uint32_t mask_seg, uint32_t n, uint32_t lanes_per_addr, uint32_t addrs_per_seg, uint32_t seed) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t lane = threadIdx.x & 63;
  uint32_t group = lane / (lanes_per_addr * addrs_per_seg);        // segment group within the wave
  uint32_t within = (lane / lanes_per_addr) % addrs_per_seg;        // dword within segment
  uint32_t wave = i >> 6;
  uint32_t seg = hash32((wave * 64 + group) ^ seed) & mask_seg;
  atomicAdd(t + seg * 16 + within, 1.0f);
}

__global__ void k_global_pk(h2* t, uint32_t mask_seg, uint32_t n, uint32_t lanes_per_addr, uint32_t addrs_per_seg, uint32_t seed) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t lane = threadIdx.x & 63;
  uint32_t group = lane / (lanes_per_addr * addrs_per_seg);
  uint32_t within = (lane / lanes_per_addr) % addrs_per_seg;
  uint32_t wave = i >> 6;
  uint32_t seg = hash32((wave * 64 + group) ^ seed) & mask_seg;
  __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2*)(t + seg * 16 + within), h2{(_Float16)1.0f, (_Float16)1.0f});
}

// LDS: per block a 16K-float window; mode 0 random, 1 all lanes same address, 2 contiguous lanes
__global__ void k_lds(float* out, uint32_t iters, uint32_t mode, uint32_t seed) {
  __shared__ float s[16384];
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) s[j] = 0.f;
  __syncthreads();
  uint32_t x = hash32(threadIdx.x ^ seed ^ (blockIdx.x << 12));
  for (uint32_t k = 0; k < iters; ++k) {
    uint32_t a;
    if (mode == 0) { x = x * 1664525u + 1013904223u; a = (x >> 8) & 16383; }
    else if (mode == 1) a = (k * 64) & 16383;
    else a = ((k * 64) + (threadIdx.x & 63)) & 16383;
    atomicAdd(s + a, 1.0f);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) out[blockIdx.x * 16384 + j] = s[j];
}

__global__ void k_lds_pk(float* out, uint32_t iters, uint32_t seed) {
  __shared__ h2 s[16384];
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) s[j] = h2{0, 0};
  __syncthreads();
  uint32_t x = hash32(threadIdx.x ^ seed ^ (blockIdx.x << 12));
  for (uint32_t k = 0; k < iters; ++k) {
    x = x * 1664525u + 1013904223u;
    uint32_t a = (x >> 8) & 16383;
    __builtin_amdgcn_ds_atomic_fadd_v2f16((__attribute__((address_space(3))) h2*)(s + a), h2{(_Float16)1.0f, (_Float16)1.0f});
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 16384; j += blockDim.x) out[blockIdx.x * 16384 + j] = (float)s[j][0];
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
  const uint32_t N = 1u << 24;
  const uint32_t segs = 1u << 18;  // 16 MB table of 64-B segments
  float* t; CK(hipMalloc(&t, (size_t)segs * 64));
  CK(hipMemset(t, 0, (size_t)segs * 64));
  struct { uint32_t lpa, aps; const char* what; } cases[] = {
    {1, 1, "1 lane / segment (scattered)"},
    {1, 16, "16 distinct dwords / segment (contiguous 64 B)"},
    {4, 4, "4 lanes x 4 dwords / segment"},
    {16, 1, "16 lanes same dword"},
    {64, 1, "64 lanes same dword"},
    {4, 1, "4 lanes same dword, 16 segments"},
    {2, 1, "2 lanes same dword, 32 segments"},
  };
  for (auto& c : cases) {
    float ms = time_ms([&] { k_global<<<N / 256, 256>>>(t, segs - 1, N, c.lpa, c.aps, 7); }, 10);
    uint32_t segs_per_wave = 64 / (c.lpa * c.aps);
    double reqs = (double)(N / 64) * segs_per_wave;
    printf("f32  %-48s %.3f ms  %.1f G lane-atom/s  %.1f G seg/s\n", c.what, ms, N / ms / 1e6, reqs / ms / 1e6);
  }
  for (auto& c : cases) {
    float ms = time_ms([&] { k_global_pk<<<N / 256, 256>>>((h2*)t, segs - 1, N, c.lpa, c.aps, 7); }, 10);
    uint32_t segs_per_wave = 64 / (c.lpa * c.aps);
    double reqs = (double)(N / 64) * segs_per_wave;
    printf("pk16 %-48s %.3f ms  %.1f G lane-atom/s  %.1f G seg/s\n", c.what, ms, N / ms / 1e6, reqs / ms / 1e6);
  }
  float* o; CK(hipMalloc(&o, (size_t)1024 * 16384 * 4));
  for (uint32_t mode = 0; mode < 3; ++mode) {
    float ms = time_ms([&] { k_lds<<<1024, 256>>>(o, 256, mode, 3); }, 10);
    printf("LDS ds_add_f32 mode %u (0 random,1 same addr,2 contiguous): %.3f ms  %.1f G lane-atom/s\n", mode, ms, 1024.0 * 256 * 256 / ms / 1e6);
  }
  float ms = time_ms([&] { k_lds_pk<<<1024, 256>>>(o, 256, 3); }, 10);
  printf("LDS ds_pk_add_f16 random: %.3f ms  %.1f G lane-atom/s\n", ms, 1024.0 * 256 * 256 / ms / 1e6);
  return 0;
}
