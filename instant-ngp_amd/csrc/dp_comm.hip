// dp_comm.hip — the engine's own RCCL communicator for data-parallel training over xGMI.
//
// The reference trains on one GPU; §8e's exchange step (sum of the fp16 gradient buffer
// before the replicated optimizer, plus the density-grid max and three counters in NeRF training)
// is issued here directly on the engine's stream, so a captured training step (forward/backward ->
// ncclAllReduce -> Adam/EMA) is one HIP graph on one queue: no host callback and no cross-queue graph
// edge per step. The unique id travels over any host channel (torch.distributed in dp.py).
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
};

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
	delete c;
}

// ngp_allreduce_fn: user = ngp_dp_comm*
int ngp_dp_comm_allreduce(void* user, void* buf, uint64_t count, int dtype, int op, void* stream) {
	auto* c = (ngp_dp_comm*)user;
	if (!c || (!buf && count)) return NGP_INVALID;
	if (count == 0) return NGP_OK;
	const ncclDataType_t t = dtype == NGP_DTYPE_F16 ? ncclFloat16 : ncclFloat32;
	const ncclRedOp_t o = op == NGP_REDUCE_MAX ? ncclMax : ncclSum;
	ngp::ProfScope ps("allreduce", (hipStream_t)stream);
	const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, t, o, c->comm, (hipStream_t)stream);
	if (r != ncclSuccess) return fail("ncclAllReduce", r);
	return NGP_OK;
}

}  // extern "C"
