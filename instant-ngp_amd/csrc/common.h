// common.h — shared types and helpers for the gfx950 engine (HIP only, no CUDA paths).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <unordered_map>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace ngp {

typedef _Float16 f16;
typedef f16 f16x2 __attribute__((ext_vector_type(2)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVE = 64;

struct Error : std::runtime_error {
	using std::runtime_error::runtime_error;
};

#define NGP_HIP(x)                                                                                    \
	do {                                                                                              \
		hipError_t e_ = (x);                                                                          \
		if (e_ != hipSuccess)                                                                         \
			throw ::ngp::Error(std::string(#x " failed: ") + hipGetErrorString(e_) + " @" + __FILE__ + \
			                   ":" + std::to_string(__LINE__));                                       \
	} while (0)

#define NGP_CHECK(cond, msg)                           \
	do {                                                \
		if (!(cond)) throw ::ngp::Error(std::string(msg)); \
	} while (0)

inline uint32_t div_round_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
inline uint32_t next_multiple(uint32_t a, uint32_t b) { return (a + b - 1) / b * b; }

// Number of compute units of the current device (256 on MI355X); cached per process.
int device_cu_count();

// ---- device helpers ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// fp32 -> fp16 of a value that has been rounded to fp32 first. LLVM folds fptrunc(fmul(a, b)) into
// v_fma_mixlo_f16, which rounds the exact product once to fp16 instead of rounding it to fp32 first as
// tcnn's `(__half)(a * b)` (and the oracle) do; the empty asm makes the fp32 value opaque to that fold.
__device__ __forceinline__ f16 to_f16(float x) {
	asm("" : "+v"(x));
	return (f16)x;
}

// Packed fp16 atomic add (global_atomic_pk_add_f16, no return). Address must be 4-byte aligned.
__device__ __forceinline__ void atomic_add_f16x2(f16* addr, f16x2 v) {
	__builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) f16x2*)addr, v);
}

// 64-lane transposed LDS read: see DESIGN.md §MLP (4 rows x 16 cols block per 16-lane group).
__device__ __forceinline__ f16x4 lds_read_tr16(const f16* p) {
	s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
	return __builtin_bit_cast(f16x4, v);
}

// hipFuncSetAttribute is a host-side driver call (microseconds); set each kernel's dynamic-LDS limit once.
inline void ensure_dynamic_lds(const void* kern, size_t bytes) {
	static std::mutex mu;
	static std::unordered_map<const void*, size_t> done;
	std::lock_guard<std::mutex> lock(mu);
	auto it = done.find(kern);
	if (it != done.end() && it->second >= bytes) return;
	NGP_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
	done[kern] = bytes;
}

}  // namespace ngp
