#include <hip/hip_runtime.h>
__global__ void k(float* p, float v, unsigned* o) {
  unsigned x; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  o[blockIdx.x] = x;
  __hip_atomic_fetch_add(p + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_add(p + threadIdx.x+64, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicAdd(p + threadIdx.x + 128, v);
  __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) _Float16 __attribute__((ext_vector_type(2)))*)(p+256+threadIdx.x), (_Float16 __attribute__((ext_vector_type(2)))){(_Float16)v,(_Float16)v});
}
