// hbm_calib.hip — known-byte kernels for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950.
//
// MI355X_MICROARCH.md §HBM: FETCH_SIZE = TCC_EA0_RDREQ x 64 B reports half the bytes of a 16-B/lane
// streaming read; other widths are uncalibrated. Each kernel here touches a 1 GiB buffer (4x the
// Infinity Cache, so nothing is served on-die) with one access pattern the engine uses, and prints the
// exact bytes it reads and writes; tools/hbm_calib.py divides the counters by those bytes.
//   r16/r8/r4/r2: coalesced streaming reads at 16/8/4/2 B per lane (engine: optimizer, items, positions)
//   g8: random 8-B gathers (grid-forward F=4 rows) — counted as the 64-B segments they touch
//   w16/w4/w2: coalesced streaming stores; s8: scattered 8-B stores
// Build: hipcc --offload-arch=gfx950 -O3 -o hbm_calib hbm_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <typename T>
__global__ void k_read(const T* __restrict__ a, size_t n, float* __restrict__ sink) {
	float acc = 0.f;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const T v = a[i];
		acc += __builtin_bit_cast(float, ((const uint32_t*)&v)[0] & 0x3fffffffu);
	}
	if (acc == 1234.5f) sink[0] = acc;  // keeps the loads
}
__global__ void k_read2(const uint16_t* __restrict__ a, size_t n, float* __restrict__ sink) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
	if (acc == 12345u) sink[0] = (float)acc;
}
template <typename T>
__global__ void k_write(T* __restrict__ a, size_t n) {
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		T v;
		for (size_t k = 0; k < sizeof(T) / 2; ++k) ((uint16_t*)&v)[k] = (uint16_t)(i + k);
		a[i] = v;
	}
}
__global__ void k_gather8(const uint2* __restrict__ a, size_t n_entries, size_t n, float* __restrict__ sink) {
	float acc = 0.f;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7) * 805459861u;
		const uint2 v = a[h % n_entries];
		acc += __builtin_bit_cast(float, v.x & 0x3fffffffu);
	}
	if (acc == 1234.5f) sink[0] = acc;
}
__global__ void k_scatter8(uint2* __restrict__ a, size_t n_entries, size_t n) {
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 7) * 805459861u;
		a[h % n_entries] = uint2{(uint32_t)i, 1u};
	}
}

int main() {
	const size_t bytes = (size_t)1 << 30;
	void* buf;
	float* sink;
	CHECK(hipMalloc(&buf, bytes));
	CHECK(hipMalloc(&sink, 4));
	CHECK(hipMemset(buf, 1, bytes));
	const dim3 grid(256 * 16), block(256);
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	auto timed = [&](const char* name, double rd, double wr, auto launch) {
		launch();  // warm
		CHECK(hipDeviceSynchronize());
		CHECK(hipEventRecord(e0));
		launch();
		CHECK(hipEventRecord(e1));
		CHECK(hipEventSynchronize(e1));
		float ms;
		CHECK(hipEventElapsedTime(&ms, e0, e1));
		printf("{\"kernel\": \"%s\", \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", name, rd, wr,
		       ms, (rd + wr) / ms / 1e6);
	};
	timed("r16", bytes, 0, [&] { k_read<uint4><<<grid, block>>>((const uint4*)buf, bytes / 16, sink); });
	timed("r8", bytes, 0, [&] { k_read<uint2><<<grid, block>>>((const uint2*)buf, bytes / 8, sink); });
	timed("r4", bytes, 0, [&] { k_read<uint32_t><<<grid, block>>>((const uint32_t*)buf, bytes / 4, sink); });
	timed("r2", bytes, 0, [&] { k_read2<<<grid, block>>>((const uint16_t*)buf, bytes / 2, sink); });
	// 2^24 random 8-B gathers: every one touches its own 64-B segment of the 1 GiB table (128 M segments)
	const size_t ng = (size_t)1 << 24;
	timed("g8", (double)ng * 64, 0, [&] { k_gather8<<<grid, block>>>((const uint2*)buf, bytes / 8, ng, sink); });
	timed("w16", 0, bytes, [&] { k_write<uint4><<<grid, block>>>((uint4*)buf, bytes / 16); });
	timed("w4", 0, bytes, [&] { k_write<uint32_t><<<grid, block>>>((uint32_t*)buf, bytes / 4); });
	timed("w2", 0, bytes, [&] { k_write<uint16_t><<<grid, block>>>((uint16_t*)buf, bytes / 2); });
	timed("s8", 0, (double)ng * 8, [&] { k_scatter8<<<grid, block>>>((uint2*)buf, bytes / 8, ng); });
	CHECK(hipFree(buf));
	CHECK(hipFree(sink));
	return 0;
}
