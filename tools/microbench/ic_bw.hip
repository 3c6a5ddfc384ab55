// ic_bw.hip — streaming bandwidth of a working set that the Infinity Cache (256 MiB) holds vs one it
// does not, for pricing cache-resident kernels (the optimizer's ~150 MB of state at C2) against a
// measured ceiling instead of the HBM spec.
//
// For each working-set size: a read-only stream (16 B/lane), a write-only stream and a copy (read one
// half, write the other), each launched back to back 20 times after a warm launch; prints the best
// launch as JSON lines (bytes moved / kernel time, HIP events).
// Build: hipcc --offload-arch=gfx950 -O3 -o ic_bw ic_bw.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_read(const uint4* __restrict__ a, size_t n, float* __restrict__ sink) {
	uint32_t acc = 0;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		const uint4 v = a[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u) sink[0] = 1.f;
}
__global__ void k_write(uint4* __restrict__ a, size_t n) {
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
		a[i] = uint4{(uint32_t)i, 1u, 2u, 3u};
}
// 8 independent 16-B loads per lane in flight
__global__ void k_read8(const uint4* __restrict__ a, size_t n, float* __restrict__ sink) {
	uint32_t acc = 0;
	const size_t stride = (size_t)gridDim.x * blockDim.x;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 8 * stride) {
		uint4 v[8];
#pragma unroll
		for (int u = 0; u < 8; ++u) v[u] = i + u * stride < n ? a[i + u * stride] : uint4{0, 0, 0, 0};
#pragma unroll
		for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (acc == 0x12345678u) sink[0] = 1.f;
}
__global__ void k_copy8(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
	const size_t stride = (size_t)gridDim.x * blockDim.x;
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
		uint4 v[4];
#pragma unroll
		for (int u = 0; u < 4; ++u) v[u] = i + u * stride < n ? a[i + u * stride] : uint4{0, 0, 0, 0};
#pragma unroll
		for (int u = 0; u < 4; ++u) if (i + u * stride < n) { v[u].x += 1u; b[i + u * stride] = v[u]; }
	}
}
// one 16-B element per thread, no loop (the optimizer's shape: n/256 blocks, every block resident once)
__global__ void k_read_flat(const uint4* __restrict__ a, size_t n, float* __restrict__ sink) {
	const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
	if (i >= n) return;
	const uint4 v = a[i];
	if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) sink[0] = 1.f;
}
__global__ void k_copy_flat(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
	const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
	if (i >= n) return;
	uint4 v = a[i];
	v.x += 1u;
	b[i] = v;
}
// read-modify-write of 4 arrays of 16 B per thread (the optimizer's state streams)
__global__ void k_rmw4_flat(uint4* __restrict__ a, size_t n) {
	const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
	if (i >= n) return;
	uint4 v[4];
#pragma unroll
	for (int k = 0; k < 4; ++k) v[k] = a[k * n + i];
#pragma unroll
	for (int k = 0; k < 4; ++k) { v[k].x += 1u; a[k * n + i] = v[k]; }
}
__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		uint4 v = a[i];
		v.x += 1u;
		b[i] = v;
	}
}

int main() {
	const size_t sizes_mb[] = {32, 96, 150, 200, 1024};
	const size_t max_bytes = (size_t)1024 << 20;
	uint4* buf;
	float* sink;
	CHECK(hipMalloc(&buf, max_bytes));
	CHECK(hipMalloc(&sink, 4));
	CHECK(hipMemset(buf, 1, max_bytes));
	const dim3 grid(256 * 8), block(256);
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	for (size_t mb : sizes_mb) {
		const size_t bytes = mb << 20, n = bytes / 16;
		auto timed = [&](const char* name, double moved, auto launch) {
			launch();
			CHECK(hipDeviceSynchronize());
			float best = 1e30f;
			for (int r = 0; r < 20; ++r) {
				CHECK(hipEventRecord(e0));
				launch();
				CHECK(hipEventRecord(e1));
				CHECK(hipEventSynchronize(e1));
				float ms;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				if (ms < best) best = ms;
			}
			printf("{\"kernel\": \"%s\", \"working_set_MB\": %zu, \"bytes\": %.0f, \"best_ms\": %.4f, \"GBps\": %.1f}\n", name, mb,
			       moved, best, moved / best / 1e6);
			fflush(stdout);
		};
		timed("read16", (double)bytes, [&] { k_read<<<grid, block>>>(buf, n, sink); });
		timed("write16", (double)bytes, [&] { k_write<<<grid, block>>>(buf, n); });
		timed("copy16", (double)bytes, [&] { k_copy<<<grid, block>>>(buf, buf + n / 2, n / 2); });
		timed("read16_flat", (double)bytes, [&] { k_read_flat<<<(unsigned)((n + 255) / 256), block>>>(buf, n, sink); });
		timed("copy16_flat", (double)bytes, [&] { k_copy_flat<<<(unsigned)((n / 2 + 255) / 256), block>>>(buf, buf + n / 2, n / 2); });
		timed("rmw4_flat", 2.0 * bytes, [&] { k_rmw4_flat<<<(unsigned)((n / 4 + 255) / 256), block>>>(buf, n / 4); });
		timed("read16x8", (double)bytes, [&] { k_read8<<<grid, block>>>(buf, n, sink); });
		timed("copy16x4", (double)bytes, [&] { k_copy8<<<grid, block>>>(buf, buf + n / 2, n / 2); });
	}
	CHECK(hipFree(buf));
	CHECK(hipFree(sink));
	return 0;
}
