// engine_internal.h — engine entry points shared between translation units (not part of the C-ABI).
#pragma once
#include "../../include/ngp_engine.h"

#include <hip/hip_runtime.h>

namespace ngp {
struct FusedAdam;
// The gradient exchange of a data-parallel training step (ngp_trainer_set_allreduce / set_data_parallel,
// ngp_nerf_trainer_set_data_parallel): `fn` (NULL: none) with its user pointer; the optimizer divides by
// loss_scale * world_factor; shard: reduce-scatter, the rank's slice of the optimizer, all-gather of the fp16
// weights (the trainer's lazy layout and option shard_opt), else one all-reduce of the fp16 gradients.
struct Exchange {
	ngp_allreduce_fn fn = nullptr;
	void* user = nullptr;
	uint32_t rank = 0, world = 1;
	float world_factor = 1.f;
	bool rank_known = false;  // set_data_parallel (sharding possible) vs set_allreduce (all-reduce only)
};
void widen_f16(const _Float16* a, float* b, uint64_t n, hipStream_t s);  // dp_comm.hip
// ngp_forward_backward with the grid's lazy optimizer update fused into the backward (fopt may be NULL)
int forward_backward_with(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                          uint32_t output_stride, const void* dL_doutput, uint32_t dL_stride, int grad_mode, const FusedAdam* fopt);
// ngp_trainer_capture_training_step with an explicit gradient exchange hook: `allreduce` (may be NULL)
// runs on the gradient buffer between backward and optimizer, which scales by loss_scale * world.
int capture_training_step_with(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                               const void* dL_doutput, uint32_t dL_stride, float loss_scale, uint32_t n_steps, int with_optimizer,
                               const Exchange& ex, ngp_graph** out);
// The values ngp_graph_launch writes into the trainer's device control block before a launch of its graph (set_device_ctl:
// step at ctl[0], the AdamConfig at ctl + CTL_CFG), for a caller that writes them in a kernel of its own, and
// the launch without that write (the rest of ngp_graph_launch: workspace check, step and staleness bookkeeping).
void trainer_ctl_values(const ngp_trainer* t, uint32_t** ctl, uint32_t* step, uint32_t* cfg_off, uint32_t* cfg_words, uint32_t* cfg);
void graph_launch_ctl_written(ngp_graph* g, void* stream);
// ngp_density with the internal output layout DENSITY_LAYOUT_ROW0 allowed besides AoS / SoA: row 0 only, a flat
// array of n (the density grid update reads nothing else)
constexpr uint32_t DENSITY_LAYOUT_ROW0 = 3;  // == MLP_LAYOUT_ROW0 (mlp.h)
int density_impl(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                 uint32_t output_stride, uint32_t output_layout, int use_inference_params);
// One eager step of what capture_training_step_with records (the host-callback exchange of gloo ranks)
int train_step_with(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride, const void* dL_doutput,
                    uint32_t dL_stride, float loss_scale, const Exchange& ex);
}  // namespace ngp
