// dp_comm.hip — the engine's own RCCL communicator for data-parallel training over xGMI.
//
// The reference trains on one GPU; §8e's exchange step (sum of the fp16 gradient buffer
// before the replicated optimizer, plus the density-grid max and three counters in NeRF training)
// is issued here directly on the engine's stream, so a captured training step (forward/backward ->
// ncclAllReduce -> Adam/EMA) is one HIP graph on one queue: no host callback and no cross-queue graph
// edge per step. The unique id travels over any host channel (torch.distributed in dp.py).
// The fp16 gradient sum travels as fp32 by default (ngp_dp_comm_set_wire), so it is rounded once.
// Links librccl.so.1; inside a PyTorch process that is the RCCL instance torch already loaded (same
// SONAME), so both communicators live in one library.
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "../../include/ngp_engine.h"
#include "common.h"
#include "profiler.h"

namespace ngp { void set_last_error(const char* msg); }

struct ngp_dp_comm {
	ncclComm_t comm = nullptr;
	int rank = 0, world = 1;
	// fp16 sums travel as fp32 (default): RCCL's fp16 ring rounds the partial sum to fp16 at every hop,
	// so the result depends on N and on each rank's ring position. Widened, the N fp16 addends are summed
	// in fp32 and rounded to fp16 once (ngp_dp_comm_set_wire).
	int wire = NGP_DTYPE_F32;
	float* stage = nullptr;  // fp32 staging of the widened buffer
	uint64_t stage_count = 0;
};

namespace ngp {
// fp16 -> fp32 widening and the single fp32 -> fp16 rounding around a widened all-reduce; 8 elements per
// thread (16-B loads when the fp16 buffer is 16-B aligned, else 8 scalar ones), scalar tail
__global__ void k_widen_f16(const f16* __restrict__ a, float* __restrict__ b, uint64_t n, bool vec) {
	const uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 8;
	if (vec && i + 8 <= n) {
		const f16x8 v = *(const f16x8*)(a + i);
		f32x4 lo = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
		f32x4 hi = {(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
		*(f32x4*)(b + i) = lo;
		*(f32x4*)(b + i + 4) = hi;
	} else {
		for (uint64_t j = i; j < n && j < i + 8; ++j) b[j] = (float)a[j];
	}
}
__global__ void k_narrow_f32(const float* __restrict__ b, f16* __restrict__ a, uint64_t n, bool vec) {
	const uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 8;
	if (vec && i + 8 <= n) {
		const f32x4 lo = *(const f32x4*)(b + i), hi = *(const f32x4*)(b + i + 4);
		f16x8 v;
		for (int k = 0; k < 4; ++k) { v[k] = (f16)lo[k]; v[k + 4] = (f16)hi[k]; }
		*(f16x8*)(a + i) = v;
	} else {
		for (uint64_t j = i; j < n && j < i + 8; ++j) a[j] = (f16)b[j];
	}
}
void widen_f16(const f16* a, float* b, uint64_t n, hipStream_t s) {
	if (n == 0) return;
	k_widen_f16<<<(uint32_t)((n + 8 * 256 - 1) / (8 * 256)), 256, 0, s>>>(a, b, n, (uintptr_t)a % 16 == 0 && (uintptr_t)b % 16 == 0);
	NGP_HIP(hipGetLastError());
}
}  // namespace ngp

namespace {
int fail(const char* what, ncclResult_t r) {
	ngp::set_last_error((std::string(what) + ": " + ncclGetErrorString(r)).c_str());
	return NGP_ERROR;
}
}  // namespace

extern "C" {

int ngp_dp_comm_unique_id(uint8_t* id_out) {
	if (!id_out) return NGP_INVALID;
	ncclUniqueId id;
	const ncclResult_t r = ncclGetUniqueId(&id);
	if (r != ncclSuccess) return fail("ncclGetUniqueId", r);
	std::memcpy(id_out, id.internal, NGP_DP_UNIQUE_ID_BYTES);
	return NGP_OK;
}

int ngp_dp_comm_create(uint32_t rank, uint32_t world, const uint8_t* id_in, ngp_dp_comm** out) {
	if (!id_in || !out || world == 0 || rank >= world) return NGP_INVALID;
	static_assert(NGP_DP_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
	ncclUniqueId id;
	std::memcpy(id.internal, id_in, NGP_DP_UNIQUE_ID_BYTES);
	auto* c = new ngp_dp_comm;
	c->rank = (int)rank;
	c->world = (int)world;
	const ncclResult_t r = ncclCommInitRank(&c->comm, (int)world, id, (int)rank);
	if (r != ncclSuccess) {
		delete c;
		return fail("ncclCommInitRank", r);
	}
	*out = c;
	return NGP_OK;
}

void ngp_dp_comm_destroy(ngp_dp_comm* c) {
	if (!c) return;
	if (c->comm) (void)ncclCommDestroy(c->comm);
	if (c->stage) (void)hipFree(c->stage);
	delete c;
}

int ngp_dp_comm_set_wire(ngp_dp_comm* c, int dtype) {
	if (!c || (dtype != NGP_DTYPE_F32 && dtype != NGP_DTYPE_F16)) return NGP_INVALID;
	c->wire = dtype;
	return NGP_OK;
}

int ngp_dp_comm_reserve(ngp_dp_comm* c, uint64_t count) {
	if (!c) return NGP_INVALID;
	if (count <= c->stage_count) return NGP_OK;
	hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
	if (hipStreamIsCapturing(nullptr, &st) == hipSuccess && st != hipStreamCaptureStatusNone) return NGP_ERROR;
	if (c->stage) (void)hipFree(c->stage);
	c->stage = nullptr;
	c->stage_count = 0;
	if (hipMalloc(&c->stage, count * sizeof(float)) != hipSuccess) {
		ngp::set_last_error("ngp_dp_comm_reserve: hipMalloc of the fp32 staging buffer failed");
		return NGP_ERROR;
	}
	c->stage_count = count;
	return NGP_OK;
}

// ngp_allreduce_fn: user = ngp_dp_comm*
int ngp_dp_comm_allreduce(void* user, void* buf, uint64_t count, int dtype, int op, void* stream) {
	auto* c = (ngp_dp_comm*)user;
	if (!c || (!buf && count)) return NGP_INVALID;
	if (count == 0) return NGP_OK;
	const ncclRedOp_t o = op == NGP_REDUCE_MAX ? ncclMax : ncclSum;
	hipStream_t s = (hipStream_t)stream;
	if (op == NGP_REDUCE_SCATTER_SUM || op == NGP_ALL_GATHER) {
		// in place: rank r's slice [r c, (r + 1) c) of the count = world c elements
		if (count % (uint64_t)c->world) {
			ngp::set_last_error("ngp_dp_comm_allreduce: reduce-scatter / all-gather count must be a multiple of world");
			return NGP_INVALID;
		}
		const size_t per = (size_t)(count / (uint64_t)c->world), esz = dtype == NGP_DTYPE_F16 ? 2 : 4;
		const ncclDataType_t t = dtype == NGP_DTYPE_F16 ? ncclFloat16 : ncclFloat32;
		char* mine = (char*)buf + (size_t)c->rank * per * esz;
		if (op == NGP_REDUCE_SCATTER_SUM) {
			ngp::ProfScope ps("reduce_scatter", s);
			const ncclResult_t r = ncclReduceScatter(buf, mine, per, t, ncclSum, c->comm, s);
			return r == ncclSuccess ? NGP_OK : fail("ncclReduceScatter", r);
		}
		ngp::ProfScope ps("all_gather", s);
		const ncclResult_t r = ncclAllGather(mine, buf, per, t, c->comm, s);
		return r == ncclSuccess ? NGP_OK : fail("ncclAllGather", r);
	}
	ngp::ProfScope ps("allreduce", s);
	if (dtype == NGP_DTYPE_F16 && op == NGP_REDUCE_SUM && c->wire == NGP_DTYPE_F32) {
		// widened sum: fp16 -> fp32 staging, fp32 ring all-reduce, one rounding back to fp16. The staging
		// buffer is sized outside graph capture (ngp_dp_comm_reserve, called when a trainer binds the
		// communicator); it is grown here only on a stream that is not being captured
		if (count > c->stage_count) {
			hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
			if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) {
				ngp::set_last_error("ngp_dp_comm_allreduce: fp32 staging too small inside a graph capture (ngp_dp_comm_reserve first)");
				return NGP_ERROR;
			}
			if (hipStreamSynchronize(s) != hipSuccess) return NGP_ERROR;
			const int rc = ngp_dp_comm_reserve(c, count);
			if (rc != NGP_OK) return rc;
		}
		const uint32_t blocks = (uint32_t)((count + 8 * 256 - 1) / (8 * 256));
		const bool vec = (uintptr_t)buf % 16 == 0;  // any tensor view may come in (EngineComm.allreduce)
		ngp::k_widen_f16<<<blocks, 256, 0, s>>>((const ngp::f16*)buf, c->stage, count, vec);
		if (hipGetLastError() != hipSuccess) return NGP_ERROR;
		const ncclResult_t r = ncclAllReduce(c->stage, c->stage, (size_t)count, ncclFloat32, o, c->comm, s);
		if (r != ncclSuccess) return fail("ncclAllReduce", r);
		ngp::k_narrow_f32<<<blocks, 256, 0, s>>>(c->stage, (ngp::f16*)buf, count, vec);
		if (hipGetLastError() != hipSuccess) return NGP_ERROR;
		return NGP_OK;
	}
	const ncclDataType_t t = dtype == NGP_DTYPE_F16 ? ncclFloat16 : ncclFloat32;
	const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, t, o, c->comm, s);
	if (r != ncclSuccess) return fail("ncclAllReduce", r);
	return NGP_OK;
}

}  // extern "C"
