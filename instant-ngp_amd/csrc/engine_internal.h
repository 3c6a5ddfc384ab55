// engine_internal.h — engine entry points shared between translation units (not part of the C-ABI).
#pragma once
#include "../../include/ngp_engine.h"

namespace ngp {
struct FusedAdam;
// ngp_forward_backward with the grid's lazy optimizer update fused into the backward (fopt may be NULL)
int forward_backward_with(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                          uint32_t output_stride, const void* dL_doutput, uint32_t dL_stride, int grad_mode, const FusedAdam* fopt);
// ngp_trainer_capture_training_step with an explicit gradient exchange hook: `allreduce` (may be NULL)
// runs on the gradient buffer between backward and optimizer, which scales by loss_scale * world.
int capture_training_step_with(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                               const void* dL_doutput, uint32_t dL_stride, float loss_scale, uint32_t n_steps, int with_optimizer,
                               ngp_allreduce_fn allreduce, void* allreduce_user, uint32_t world, ngp_graph** out);
}  // namespace ngp
