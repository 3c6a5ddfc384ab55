// Does a CU mask on a HIP stream (hipExtStreamCreateWithCUMask) restrict where its kernels run?
// A kernel of 256 x 4 blocks, each spinning for a fixed number of clock ticks at one block per SIMD, is
// timed on an unmasked stream and on streams masked to 1/2 and 1/8 of the CUs; every block also records
// its hardware CU id (HW_ID) so the distinct CUs used are counted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_spin(unsigned long long ticks, unsigned* ids) {
	__shared__ char big[96 * 1024];  // one block per CU
	const unsigned long long t0 = wall_clock64();
	while (wall_clock64() - t0 < ticks) {}
	if (threadIdx.x == 0) {
		unsigned xcc = 0, hw = 0;
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
		asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
		big[0] = 1;
		ids[blockIdx.x] = (xcc << 16) | ((hw >> 8) & 0xFFF);  // CU_ID | SH_ID | SE_ID bits
	}
}

int main() {
	int n_cu = 0;
	CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
	const int blocks = 1024;
	unsigned* d_ids;
	CHECK(hipMalloc(&d_ids, blocks * 4));
	for (int keep : {8, 4, 1}) {
		hipStream_t s;
		std::vector<uint32_t> mask((n_cu + 31) / 32, 0u);
		for (int c = 0; c < n_cu; ++c)
			if (c % 8 < keep) mask[c / 32] |= 1u << (c % 32);
		if (keep == 8) CHECK(hipStreamCreate(&s));
		else CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
		hipEvent_t a, b;
		CHECK(hipEventCreate(&a));
		CHECK(hipEventCreate(&b));
		k_spin<<<blocks, 256, 0, s>>>(1000, d_ids);
		CHECK(hipEventRecord(a, s));
		k_spin<<<blocks, 256, 0, s>>>(20000, d_ids);  // 200 us at 100 MHz
		CHECK(hipEventRecord(b, s));
		CHECK(hipStreamSynchronize(s));
		float ms = 0;
		CHECK(hipEventElapsedTime(&ms, a, b));
		std::vector<unsigned> ids(blocks);
		CHECK(hipMemcpy(ids.data(), d_ids, blocks * 4, hipMemcpyDeviceToHost));
		std::set<unsigned> u(ids.begin(), ids.end());
		printf("{\"keep_of_8\": %d, \"ms\": %.3f, \"distinct_cus\": %zu, \"n_cu\": %d}\n", keep, ms, u.size(), n_cu);
		CHECK(hipStreamDestroy(s));
	}
	return 0;
}
