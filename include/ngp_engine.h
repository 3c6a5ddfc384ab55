/*
 * ngp_engine.h — C-ABI of the MI355X (gfx950) instant-ngp hot-path engine.
 *
 * The engine is a drop-in for the tiny-cuda-nn model/trainer objects the reference's Testbed drives:
 *   tcnn::NetworkWithInputEncoding  (src/testbed.cu:4110, image/SDF primitives)
 *   ngp::NerfNetwork                (include/neural-graphics-primitives/nerf_network.h:77-578)
 *   tcnn::Trainer + Optimizer chain (src/testbed.cu:4129; configs/nerf/base.json:5-22)
 * plus the NeRF training kernels of src/testbed_nerf.cu (ngp_nerf_* below).
 *
 * Conventions
 *  - Plain C types only; half-precision buffers are `void*` holding IEEE binary16.
 *  - Device pointers unless a name says _host. `stream` is a hipStream_t (NULL = default stream).
 *  - Matrices follow tcnn's naming: input  element (i, d) at input[i * input_stride + d] ("CM"/AoS,
 *    the NerfCoordinate layout, nerf.h:85-128); outputs AoS (layout 0: out[i * stride + f]) or
 *    SoA (layout 1: out[f * stride + i], tcnn "RM").
 *  - Errors: every int-returning function returns 0 on success and a negative code on failure;
 *    ngp_last_error() gives the message (the reference throws std::runtime_error /
 *    CUDA_CHECK_THROW, e.g. nerf_network.h:338-340). Handles are not internally synchronised:
 *    one host thread per (device, stream) handle, as the reference's one-stream-per-device Testbed
 *    (testbed.h:989).
 */
#ifndef NGP_ENGINE_H
#define NGP_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

typedef struct ngp_model ngp_model;     /* a network: NerfNetwork or NetworkWithInputEncoding */
typedef struct ngp_ctx ngp_ctx;         /* forward context (tcnn::Context, nerf_network.h:566-577) */
typedef struct ngp_trainer ngp_trainer; /* params + gradients + optimizer state (tcnn::Trainer) */

enum { NGP_OK = 0, NGP_ERROR = -1, NGP_INVALID = -2 };
enum { NGP_LAYOUT_AOS = 0, NGP_LAYOUT_SOA = 1 };
/* Engine extension for NerfNetwork inference outputs: only the 4 live rows (raw rgb, raw density) as
 * AoS [n x stride >= 4], skipping the 12 padded outputs of padded_output_width 16 (nerf_network.h:463). */
enum { NGP_LAYOUT_AOS_RGBD = 2 };
enum { NGP_GRAD_OVERWRITE = 0, NGP_GRAD_ACCUMULATE = 1, NGP_GRAD_IGNORE = 2 }; /* tcnn::EGradientMode */

/* ---- library ------------------------------------------------------------------------------ */
const char* ngp_last_error(void);
const char* ngp_version(void);
/* device name and CU count of the current HIP device */
int ngp_device_info(int* cu_count, char* name, size_t name_len);
/* device memory helpers for FFI callers without their own allocator */
int ngp_malloc(void** ptr, size_t bytes);
int ngp_free(void* ptr);
int ngp_memcpy(void* dst, const void* src, size_t bytes, int kind /* hipMemcpyKind */);
int ngp_stream_synchronize(void* stream);
/* per-kernel HIP-event timing on each kernel's launch stream (off by default). read() fills a JSON
 * object {"phase": {"calls": n, "ms": total}} and returns the length needed (incl. NUL). */
int ngp_profiler_enable(int enable);
int ngp_profiler_reset(void);
int ngp_profiler_read(char* json_buf, size_t len);
/* Verification (engine extension): the device forms of the shared math (csrc/ngp_math.h) against the reference
 * operations they replace, over the whole input range, on the GPU. which 0: ngp_div_2pf (the logf's f / (2 + f),
 * reciprocal + Newton + residual step) against the IEEE quotient for all 2^23 reduced arguments. *mismatches =
 * the number of inputs whose results differ in any bit (0 is the contract the sampler's bit-exactness rests on). */
int ngp_debug_math_check(int which, void* stream, uint64_t* mismatches);

/* ---- models (tcnn::Network<float, __half> surface) ------------------------------------------ */
/* NerfNetwork ctor (nerf_network.h:81-112); JSON strings are the config sections the Testbed passes
 * (src/testbed.cu:4029-4042: "encoding", "dir_encoding", "network", "rgb_network"). */
int ngp_nerf_network_create(uint32_t n_pos_dims, uint32_t n_dir_dims, uint32_t n_extra_dims, uint32_t dir_offset,
                            const char* pos_encoding_json, const char* dir_encoding_json,
                            const char* density_network_json, const char* rgb_network_json, ngp_model** out);
/* tcnn::NetworkWithInputEncoding(n_input_dims, n_output_dims, encoding, network) (src/testbed.cu:4101-4110) */
int ngp_network_with_input_encoding_create(uint32_t n_input_dims, uint32_t n_output_dims, const char* encoding_json,
                                           const char* network_json, ngp_model** out);
void ngp_model_destroy(ngp_model* m);

uint64_t ngp_model_n_params(const ngp_model* m);           /* n_params()            nerf_network.h:459 */
uint64_t ngp_model_n_matrix_params(const ngp_model* m);    /* sum of layer_sizes()  nerf_network.h:483, testbed.cu:3834-3846 */
uint32_t ngp_model_input_width(const ngp_model* m);        /* input_width()         nerf_network.h:467 */
uint32_t ngp_model_padded_output_width(const ngp_model* m);/* padded_output_width() nerf_network.h:463 */
uint32_t ngp_model_output_width(const ngp_model* m);       /* output_width()        nerf_network.h:471 */

/* Parameter layout: [density MLP | rgb MLP | position grid | dir encoding] (nerf_network.h:430-443);
 * NetworkWithInputEncoding: [MLP | grid]. Grid level offsets in entries (GridEncoding
 * level_params_offset / level_n_params, src/testbed.cu:4849-4856). */
typedef struct {
	uint64_t density_mlp_offset, density_mlp_params;
	uint64_t rgb_mlp_offset, rgb_mlp_params;
	uint64_t grid_offset, grid_params;
	uint32_t grid_dims, grid_levels, grid_features, grid_log2_hashmap, grid_base_resolution;
	float grid_per_level_scale;
	uint32_t grid_level_offsets[33]; /* entries; params = entries * grid_features */
	uint32_t grid_resolution[32];
	float grid_scale[32];
	uint32_t encoding_width;         /* padded encoding output width (density MLP input) */
} ngp_param_layout;
int ngp_model_param_layout(const ngp_model* m, ngp_param_layout* out);

/* set_params(params, inference_params, gradients) (nerf_network.h:430): fp16 device buffers of n_params */
int ngp_model_set_params(ngp_model* m, void* params, void* inference_params, void* gradients);
/* initialize_params(rnd, params_full_precision, scale) (nerf_network.h:445-457), host fp32 buffer */
int ngp_model_initialize_params(const ngp_model* m, uint64_t seed, float* params_full_precision_host, float scale);
/* GridEncoding::set_max_level / set_max_level_gpu (src/testbed.cu:3856-3864; testbed_nerf.cu:3996,4004) */
int ngp_model_set_max_level(ngp_model* m, float max_level, const float* max_level_per_sample);
/* engine knobs: "grid_backward_mode" = 0 auto, 1 direct packed-f16 atomics (tcnn-style),
 * 3 destination-bucketed exact sums (auto picks 3 for n >= 4096); "grid_bricks" (bucketed backward: dense
 * levels summed per brick where that moves fewer bytes, default 0); "fuse_infer", "fused_hist",
 * "fuse_slabs", "fuse_opt", "fuse_mlp_opt", "overlap", "win_debug"  */
int ngp_model_set_option(ngp_model* m, const char* key, double value);
/* engine state for tests and tools: "grid_brick_levels" = how many dense levels the bucketed backward sums
 * per brick in its plan for the last batch size (0: all levels through items) */
int ngp_model_query(const ngp_model* m, const char* key, double* value);
/* pre-size internal workspaces for batches up to n (lets callers capture steps into HIP graphs) */
int ngp_model_reserve(ngp_model* m, uint32_t n);
/* Inspection of the last training pass's intermediates (the role of tcnn's forward_activations(ctx),
 * nerf_network.h:502-507): "encoding" = fp16 AoS [n x encoding_width] grid output of the last unfused
 * forward, "dL_dencoding" = fp16 AoS [n x encoding_width] input of the grid backward, "dL_dsh" = fp16
 * [n x 16] dL/d(SH encoding) of the last backward with input gradients, "dw_slabs" = the fp32 per-block
 * MLP weight-gradient partial sums. Device pointer
 * valid until the next call that grows the workspace. */
int ngp_model_workspace(ngp_model* m, const char* name, void** ptr, uint64_t* bytes);
/* Counts workspace reallocations. A graph from ngp_trainer_capture_training_step holds workspace
 * pointers: ngp_graph_launch fails (instead of touching freed memory) once the epoch moved past the
 * capture's; callers re-capture when it changes. */
uint64_t ngp_model_workspace_epoch(const ngp_model* m);

/* inference_mixed_precision (nerf_network.h:116-174): output fp16 [n x padded_output_width] */
int ngp_inference(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                  uint32_t output_stride, uint32_t output_layout, int use_inference_params);
/* NerfNetwork::density (nerf_network.h:337-353): density MLP output fp16 [n x 16] */
int ngp_density(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                uint32_t output_stride, uint32_t output_layout, int use_inference_params);
/* forward_impl (nerf_network.h:179-254) -> context; output may be NULL */
int ngp_forward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                uint32_t output_stride, int use_inference_params, ngp_ctx** ctx);
/* backward_impl (nerf_network.h:256-335): param gradients into the gradient buffer given to set_params
 * (grad_mode NGP_GRAD_IGNORE: untouched). dL_dinput (nullable, the reference's `GPUMatrixDynamic<float>*
 * dL_dinput`): fp32 AoS [n x dL_dinput_stride]; rows 0..n_pos_dims-1 receive dL/dposition through the
 * grid encoding, a NerfNetwork's rows dir_offset..+2 dL/ddirection through the SH encoding
 * (nerf_network.h:282-299, 317-333); other rows are not written. A context from a forward with
 * use_inference_params runs the backward on the inference (EMA) parameters too (backward_impl's
 * use_inference_params, nerf_network.h:256-335). */
int ngp_backward(ngp_model* m, void* stream, ngp_ctx* ctx, const void* dL_doutput, uint32_t dL_stride, float* dL_dinput,
                 uint32_t dL_dinput_stride, int grad_mode);
void ngp_ctx_destroy(ngp_ctx* ctx);
/* NerfNetwork::density_forward (nerf_network.h:355-382) -> context; output (nullable): the density
 * network's fp16 output AoS [n x output_stride] (16 rows) */
int ngp_density_forward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                        uint32_t output_stride, int use_inference_params, ngp_ctx** ctx);
/* NerfNetwork::density_backward (nerf_network.h:384-428): dL_doutput = dL/d(density network output),
 * fp16 AoS [n x dL_stride] (16 rows, stride a multiple of 4). Gradients of the density MLP and the grid
 * (the rgb MLP's are left as they are); dL_dinput as in ngp_backward (position rows only). */
int ngp_density_backward(ngp_model* m, void* stream, ngp_ctx* ctx, const void* dL_doutput, uint32_t dL_stride, float* dL_dinput,
                         uint32_t dL_dinput_stride, int grad_mode);
/* tcnn Network::input_gradient(stream, dim, input, d_dinput, backprop_scale) — the reference's normals
 * (testbed_nerf.cu:2616, dim 3 = density; testbed.cu:4621, SDF dim 0): forward, backward of a one-hot
 * dL/doutput (row `dim` = backprop_scale) with parameter gradients ignored, result / backprop_scale.
 * d_dinput fp32 AoS [n x d_dinput_stride] (may alias `input` with the same stride, as the reference
 * passes positions_matrix for both: only the position/direction rows are written, after every read). */
int ngp_input_gradient(ngp_model* m, void* stream, uint32_t dim, uint32_t n, const float* input, uint32_t input_stride,
                       float* d_dinput, uint32_t d_dinput_stride, float backprop_scale);
/* fused training pass = forward_impl + backward_impl (src/testbed_nerf.cu:4077-4078) in one call */
int ngp_forward_backward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                         uint32_t output_stride, const void* dL_doutput, uint32_t dL_stride, int grad_mode);

/* Raw position-encoding access (tcnn GridEncoding forward / backward). out fp16 [n x encoding_width]. */
int ngp_encoding_forward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride, void* output,
                         uint32_t output_stride, uint32_t output_layout, int use_inference_params);
/* dL_dinput (nullable; needs dL_layout AoS): fp32 [n x dL_dinput_stride], rows 0..n_pos_dims-1 */
int ngp_encoding_backward(ngp_model* m, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                          const void* dL_doutput, uint32_t dL_stride, uint32_t dL_layout, float* dL_dinput,
                          uint32_t dL_dinput_stride, int grad_mode);

/* ---- trainer (tcnn::Trainer<float, __half, __half>, src/testbed.cu:4129) -------------------- */
/* optimizer_json: the "optimizer" config section (Ema / ExponentialDecay / Adam nesting).
 * Allocates fp32 master params, fp16 params / inference(EMA) params / gradients and Adam state,
 * initialises parameters from `seed` (default_rng_t, src/testbed.cu:3906) and calls set_params. */
int ngp_trainer_create(ngp_model* m, const char* optimizer_json, uint64_t seed, ngp_trainer** out);
void ngp_trainer_destroy(ngp_trainer* t);
/* Trainer::optimizer_step(stream, loss_scale) (src/testbed_nerf.cu:3678) */
int ngp_trainer_optimizer_step(ngp_trainer* t, void* stream, float loss_scale);
void* ngp_trainer_gradients(ngp_trainer* t);               /* fp16 [n_params], the DP all-reduce buffer */
/* 1 when the gradient buffer holds the last training pass's whole gradient. 0 after a step whose backward did
 * not write it: the grid's optimizer update fused into the backward (ngp_trainer_fused_update_active, captured
 * or training_step steps on the lazy layout) or the sharded data-parallel step, whose backward stores the
 * gradient as fp32 for the reduce-scatter. The buffer then holds an older gradient. ngp_forward_backward and
 * steps without the fused update write it again (engine extension; tcnn's gradients() is always current) */
int ngp_trainer_gradients_valid(const ngp_trainer* t);
void* ngp_trainer_params(ngp_trainer* t);                  /* fp16 [n_params] */
void* ngp_trainer_inference_params(ngp_trainer* t);        /* fp16 [n_params] (EMA when configured) */
/* fp32 [n_params]; large-table trainers keep the master weights in their optimizer records and refresh this
   mirror on each call (synchronizes the device; NULL + ngp_last_error on failure). For those trainers the
   buffer is read-only: writes into it never reach training or serialize (which reads the records); change
   weights with ngp_trainer_set_params_full_precision. For eager-layout trainers it is the live master copy. */
float* ngp_trainer_params_full_precision(ngp_trainer* t);
uint32_t ngp_trainer_step(const ngp_trainer* t);
uint64_t ngp_trainer_n_params(const ngp_trainer* t);
float ngp_trainer_learning_rate(const ngp_trainer* t);     /* optimizer->learning_rate() (testbed_nerf.cu:3771) */
int ngp_trainer_set_learning_rate(ngp_trainer* t, float lr);
/* Engine extension: trainer options. "ema_closed_form" 0 (default) / 1: how the large-table (lazy-EMA) layout
 * applies the EMA steps a skipped parameter owes: exact replay to the recurrence's fixed point, bit for bit the
 * per-step Ema of tcnn's chain (configs/nerf/base.json:5-8), or a closed form past 32 steps (within 1 fp16 ulp).
 * "shard_opt" 1 (default) / 0: the sharded optimizer under ngp_trainer_set_data_parallel (see there). */
int ngp_trainer_set_option(ngp_trainer* t, const char* key, double value);
/* set_params_full_precision (src/testbed.cu:4146): host fp32 -> master, fp16 params and inference params */
int ngp_trainer_set_params_full_precision(ngp_trainer* t, const float* params_host, uint64_t n);
/* serialize / deserialize (src/testbed.cu:4874,5040): flat little-endian blob, size query with buf=NULL */
int ngp_trainer_serialize(ngp_trainer* t, void* buf_host, uint64_t* size);
int ngp_trainer_deserialize(ngp_trainer* t, const void* buf_host, uint64_t size);

/* Engine extension (no reference counterpart): capture n_steps of {forward_backward(input, dL/doutput)
 * [+ optimizer_step(loss_scale) if with_optimizer]} on `stream` (not the null stream) into one HIP
 * graph, replayed by ngp_graph_launch. Inputs are read from the captured device pointers at every
 * launch. The optimizer step counter lives on the device, so replays follow the same learning-rate/EMA
 * schedule as eager steps. For launch-bound training loops (one launch instead of ~15 per step). */
typedef struct ngp_graph ngp_graph;
int ngp_trainer_capture_training_step(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                                      const void* dL_doutput, uint32_t dL_stride, float loss_scale, uint32_t n_steps,
                                      int with_optimizer, ngp_graph** out);
/* Engine extension: ONE step of exactly what a captured step runs, launched eagerly: forward_backward
 * (with the grid's lazy update fused into the backward when ngp_trainer_fused_update_active), the
 * trainer's gradient exchange hook if set (ngp_trainer_set_allreduce), then optimizer_step(loss_scale x
 * world). The per-kernel profile of this call is the profile of a replayed graph step. */
int ngp_trainer_train_step(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                           const void* dL_doutput, uint32_t dL_stride, float loss_scale);
/* 1 when a training step of n_batch samples runs the grid's optimizer update inside the backward (lazy-EMA
 * layout, model option fuse_opt, no exchange hook): the grid part of the gradient buffer is then not written. */
int ngp_trainer_fused_update_active(const ngp_trainer* t, uint32_t n_batch);
int ngp_graph_launch(ngp_graph* g, void* stream);
void ngp_graph_destroy(ngp_graph* g);

typedef struct { uint64_t state, inc; } ngp_rng; /* tcnn::pcg32 state (default_rng_t) */

/* ---- losses and the generic training step (tcnn::Trainer::training_step) ------------------- */
/* tcnn Loss otypes as named in the configs (configs/image/base.json:2-4 "L2", configs/sdf/base.json
 * "MAPE"): value = l(pred, target) / (n * dims), gradient = loss_scale * dl/dpred / (n * dims) rounded
 * to fp16; output columns >= dims get a zero gradient. */
enum { NGP_LOSS_L2 = 0, NGP_LOSS_L1 = 1, NGP_LOSS_MAPE = 2, NGP_LOSS_SMAPE = 3, NGP_LOSS_RELATIVE_L2 = 4 };
/* output fp16 AoS [n x output_stride], target fp32 AoS [n x target_stride], dL_doutput fp16 AoS;
 * values (optional, device [n]): per-sample loss; loss_sum (optional, device scalar): += total */
int ngp_loss_evaluate(int loss_type, void* stream, uint32_t n, uint32_t dims, const void* output, uint32_t output_stride,
                      const float* target, uint32_t target_stride, float loss_scale, void* dL_doutput, uint32_t dL_stride,
                      float* values, float* loss_sum);
/* tcnn::Trainer::training_step(stream, input, target, data_pdf = nullptr, run_optimizer)
 * (src/testbed_image.cu:276, src/testbed_sdf.cu:1304): forward, loss over the model's output_width
 * columns, backward into the gradient buffer (overwrite) and, if run_optimizer, optimizer_step. With
 * run_optimizer on the lazy-EMA layout and model option "fuse_opt" (default), the grid's update runs
 * inside the backward (bit-identical) and the grid part of the gradient buffer is not written. */
int ngp_trainer_training_step(ngp_trainer* t, void* stream, uint32_t n, const float* input, uint32_t input_stride,
                              const float* target, uint32_t target_stride, int loss_type, float loss_scale, int run_optimizer,
                              float* loss_sum);

/* ---- image primitive (BASELINE C1; src/testbed_image.cu) -------------------------------------- */
typedef struct ngp_image ngp_image;
enum { NGP_IMAGE_RANDOM = 0, NGP_IMAGE_STRATIFIED = 3 };  /* ERandomMode (common.h:124-130) */
typedef struct {
	uint32_t random_mode;            /* Stratified (testbed.h:875) */
	uint32_t snap_to_pixel_centers;  /* 1 (testbed.h:871) */
	uint32_t linear_colors;          /* 0 (testbed.h:872): targets are sRGB-encoded */
} ngp_image_config;
int ngp_image_default_config(ngp_image_config* out);
/* texture: RGBA fp32 [height x width x 4] in linear colours (EDataType::Float, e.g. albert.exr) */
int ngp_image_create(uint32_t width, uint32_t height, const float* rgba_host, ngp_image** out);
void ngp_image_destroy(ngp_image* img);
/* generate_training_data of Testbed::train_image (testbed_image.cu:223-265): generate_random_uniform
 * (advances *rng by 2n), stratify2_kernel (:62-76), eval_image_kernel_and_snap<float, 3> (:167-212).
 * positions [n x 2], targets [n x 3] (device). */
int ngp_image_generate_training_samples(const ngp_image* img, void* stream, uint32_t n, ngp_rng* rng, const ngp_image_config* cfg,
                                        float* positions, float* targets);
/* Testbed::train_image (testbed_image.cu:214-285): samples, training_step (L2, no optimizer), optimizer_step(128) */
int ngp_image_train_step(ngp_image* img, ngp_trainer* t, void* stream, uint32_t batch, ngp_rng* rng, const ngp_image_config* cfg,
                         float* loss_sum);

/* ---- SDF primitive (BASELINE C5; src/testbed_sdf.cu) ------------------------------------------ */
typedef struct ngp_sdf_mesh ngp_sdf_mesh;
/* triangles [n x 9] already normalised to the unit cube (Testbed::load_mesh, testbed_sdf.cu:1120-1150);
 * builds the surface-area CDF (triangle_distribution, :1167-1175) */
int ngp_sdf_mesh_create(uint32_t n_triangles, const float* tris_host, ngp_sdf_mesh** out);
void ngp_sdf_mesh_destroy(ngp_sdf_mesh* m);
/* the mesh's triangles in the order the BVH build left them (TriangleBvh4::build reorders
 * m_sdf.triangles_cpu, testbed_sdf.cu:1157; the surface CDF follows that order): [n x 9] host floats */
int ngp_sdf_mesh_triangles(const ngp_sdf_mesh* m, float* tris_out);
/* host-only TriangleBvh4::build (triangle_bvh.cu:540-617) for inspection: reorders tris [n x 9] in place
 * and writes the nodes, 32 bytes each {float lo[3], hi[3]; int32 left, right} (negative = leaf
 * triangle range [-left-1, -right-1)). nodes_out = NULL: *n_nodes = the node count, tris untouched. */
int ngp_sdf_bvh_build(float* tris, uint32_t n_triangles, uint32_t n_primitives_per_leaf, void* nodes_out, uint32_t* n_nodes);
/* generate_training_samples_sdf (testbed_sdf.cu:1187-1275), non-octree branch: n/8 * {4 on the surface,
 * 3 surface + logistic offset, 1 uniform in aabb}; n must be a multiple of 8; advances *rng by
 * 3n + 3 * (3n/8). Signed distances by brute force over the triangles (the BVH is SURVEY §8f). */
int ngp_sdf_generate_training_samples(ngp_sdf_mesh* m, void* stream, uint32_t n, ngp_rng* rng, const float* aabb_min,
                                      const float* aabb_max, float stddev, float* positions, float* distances);
/* signed_distance_raystab semantics (triangle_bvh.cu:415-433) over every triangle */
int ngp_sdf_signed_distance(ngp_sdf_mesh* m, void* stream, uint32_t n, const float* positions, float* distances);
/* shuffle<vec3> / shuffle<float> (testbed_sdf.cu:1295-1296): a bijection seeded by the training step */
int ngp_sdf_shuffle(void* stream, uint32_t n, uint32_t seed, const float* positions, const float* distances,
                    float* positions_shuffled, float* distances_shuffled);
/* Testbed::train_sdf (testbed_sdf.cu:1289-1312): shuffle, training_step (MAPE, loss scale 128, optimizer) */
int ngp_sdf_train_step(ngp_trainer* t, void* stream, uint32_t n, const float* positions, const float* distances, uint32_t step,
                       float* positions_shuffled, float* distances_shuffled, float* loss_sum);

/* ---- NeRF training kernels (src/testbed_nerf.cu), without OptiX --------------------------- */
typedef struct ngp_nerf_dataset ngp_nerf_dataset;  /* training images on device + cameras */
typedef struct ngp_nerf_trainer ngp_nerf_trainer;  /* Testbed NeRF training state (grid, counters, rng) */

/* One training image (TrainingImageMetadata, nerf_loader.h; xform after nerf_matrix_to_ngp):
 * camera-to-world mat4x3, column-major {x axis, y axis, z axis, origin}. */
typedef struct {
	uint32_t width, height;
	float focal_length[2];
	float principal_point[2];
	float xform[12];
	uint32_t lens_mode;      /* Lens (common_device.cuh:288-378, nerf_loader.cu:160-224): 0 perspective,
	                            1 OpenCV {k1, k2, p1, p2}, 2 OpenCV fisheye {k1, k2, k3, k4} */
	float lens_params[4];
} ngp_nerf_image;

/* Training knobs with the reference defaults (testbed.h:716-785; load_nerf_post testbed_nerf.cu:3093-3109). */
typedef struct {
	float aabb_min[3], aabb_max[3];   /* m_aabb */
	float cone_angle_constant;        /* 0 when aabb_scale <= 1, else 1/256 */
	uint32_t max_cascade;             /* ceil(log2(aabb_scale)) */
	uint32_t snap_to_pixel_centers;   /* 1 */
	uint32_t random_bg_color;         /* 1 */
	uint32_t linear_colors;           /* 0 */
	uint32_t color_space_linear;      /* 1 (m_color_space = Linear) */
	float background_color[3];        /* 0 */
	uint32_t rgb_activation;          /* 0 None, 1 ReLU, 2 Logistic, 3 Exponential; default 3 */
	uint32_t density_activation;      /* default 3 */
	uint32_t loss_type;               /* 0 L2, 1 L1, 2 MAPE, 3 SMAPE, 4 Huber, 5 LogL1, 6 RelativeL2; base.json: Huber */
	float near_distance;              /* 0.1 */
	uint32_t target_batch_size;       /* 2^18 */
} ngp_nerf_config;


typedef struct {
	uint32_t step, rays_per_batch, measured_batch_size, measured_batch_size_before_compaction;
	float loss;
} ngp_nerf_stats;

int ngp_nerf_default_config(float aabb_scale, ngp_nerf_config* out);
/* images: RGBA8 sRGB (EImageDataType::Byte; 0x00FF00FF marks masked pixels, common_device.cuh:893) */
int ngp_nerf_dataset_create(uint32_t n_images, const ngp_nerf_image* images, const void* const* rgba8_host,
                            ngp_nerf_dataset** out);
void ngp_nerf_dataset_destroy(ngp_nerf_dataset* ds);

/* generate_training_samples_nerf (testbed_nerf.cu:1382-1658); deterministic slots (prefix scans).
 * rays: [n_rays x 6] {o, d}; numsteps: [n_rays x 2] {n, base}; coords: [max_samples x 7];
 * counters: [2] = {rays kept, total steps incl. dropped rays}. */
int ngp_nerf_generate_training_samples(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream,
                                       uint32_t n_rays, uint32_t ray_offset, uint32_t n_rays_total, ngp_rng rng,
                                       uint32_t max_samples, const uint8_t* bitfield, uint32_t* ray_indices, float* rays,
                                       uint32_t* numsteps, float* coords, uint32_t* counters);
/* compute_loss_kernel_train_nerf (testbed_nerf.cu:1660-2012): composite, loss, compaction, dL/doutput */
int ngp_nerf_compute_loss(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                          uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted, const uint32_t* ray_counter,
                          const void* network_output, const uint32_t* ray_indices, const float* rays, uint32_t* numsteps,
                          const float* coords_in, float* coords_out, void* dloss_doutput, float* loss,
                          uint32_t* compacted_counter, const float* mean_density, float loss_scale);
/* The same with the training error map (testbed_nerf.cu:1869-1899, the kernel's error_map argument): every
 * compacted ray adds its mean loss, split bilinearly around uv * res - 0.5, into error_map
 * [n_images][em_height][em_width] (device floats, float atomics as in the reference). */
/* Engine extension: ngp_nerf_compute_loss with pass 1 keeping each composited sample's state (weight, transmittance
 * after it, rgb prefix through it) in sample_state ([5][state_capacity] floats, indexed like the samples: state_capacity
 * at least the sample buffer's length) for pass 2, which then does not composite each ray again. The same float
 * operations: outputs equal ngp_nerf_compute_loss's bit for bit. The training step uses this form. */
int ngp_nerf_compute_loss_state(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                                uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted, const uint32_t* ray_counter,
                                const void* network_output, const uint32_t* ray_indices, const float* rays, uint32_t* numsteps,
                                const float* coords_in, float* coords_out, void* dloss_doutput, float* loss,
                                uint32_t* compacted_counter, const float* mean_density, float loss_scale, float* sample_state,
                                uint64_t state_capacity);
int ngp_nerf_compute_loss_error_map(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                                    uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted,
                                    const uint32_t* ray_counter, const void* network_output, const uint32_t* ray_indices,
                                    const float* rays, uint32_t* numsteps, const float* coords_in, float* coords_out,
                                    void* dloss_doutput, float* loss, uint32_t* compacted_counter, const float* mean_density,
                                    float loss_scale, float* error_map, uint32_t em_width, uint32_t em_height);
/* tcnn fill_rollover / fill_rollover_and_rescale (testbed_nerf.cu:4061-4069); dtype 0 f32, 1 f16 */
int ngp_nerf_fill_rollover(void* stream, uint32_t n_elements, uint32_t stride, const uint32_t* n_input, void* data,
                           int dtype, int rescale);
/* occupancy grid (testbed_nerf.cu:635-809, 3412-3567) */
int ngp_nerf_grid_generate_samples(void* stream, const ngp_nerf_config* cfg, uint32_t n, ngp_rng rng, uint32_t step,
                                   const float* grid, uint32_t n_cascades, float thresh, float* positions,
                                   uint32_t* indices);
int ngp_nerf_grid_splat_max(void* stream, uint32_t n, const uint32_t* indices, const void* density_rm,
                            uint32_t density_activation, float* grid_tmp);
// The reference's memset(grid_tmp, 0) + splat_grid_samples_nerf_max_nearest_neighbor (testbed_nerf.cu:3476, :678-702)
// in one call: grid_tmp[c] = the max over the samples in cell c (0 where none) for all n_cells cells (a multiple of
// 8192), computed as a counting sort by cell bin instead of scattered atomics; bit-identical.
int ngp_nerf_grid_splat_max_cells(void* stream, uint32_t n, const uint32_t* indices, const void* density_rm,
                                  uint32_t density_activation, float* grid_tmp, uint32_t n_cells);
int ngp_nerf_grid_ema(void* stream, uint32_t n, float decay, float* grid, const float* grid_tmp);
int ngp_nerf_grid_mean_and_bitfield(void* stream, const float* grid, uint32_t max_cascade, float* mean, uint8_t* bitfield);

/* Testbed-level NeRF training (Testbed::train -> training_prep_nerf + train_nerf, src/testbed.cu:4285-4370,
 * testbed_nerf.cu:3611-3862, 4137-4152). The model/trainer must be a NerfNetwork and its Trainer. */
int ngp_nerf_trainer_create(ngp_model* model, ngp_trainer* trainer, const ngp_nerf_dataset* ds,
                            const ngp_nerf_config* cfg, uint64_t seed, ngp_nerf_trainer** out);
void ngp_nerf_trainer_destroy(ngp_nerf_trainer* t);
/* The training knobs of a live trainer (Testbed::Nerf::Training members the pybind surface writes, e.g.
 * random_bg_color, loss_type, near_distance, target batch size). max_cascade and the aabb size the density
 * grid and cannot change (recreate the trainer). */
int ngp_nerf_trainer_get_config(const ngp_nerf_trainer* t, ngp_nerf_config* out);
int ngp_nerf_trainer_set_config(ngp_nerf_trainer* t, const ngp_nerf_config* cfg);
int ngp_nerf_train_step(ngp_nerf_trainer* t, void* stream, int get_loss, ngp_nerf_stats* out);
int ngp_nerf_trainer_buffers(ngp_nerf_trainer* t, float** density_grid, uint8_t** bitfield, float** mean_density);
/* The same pointers for READING only: keeps a prelaunched (pipelined) sampler, which reads the bitfield
 * and writes none of the three. Writes through these pointers are not seen by an already prelaunched
 * sampler: use ngp_nerf_trainer_buffers to modify them. */
int ngp_nerf_trainer_buffers_read(const ngp_nerf_trainer* t, const float** density_grid, const uint8_t** bitfield,
                                  const float** mean_density);

/* Rendering (NerfTracer::init_rays_from_camera + trace + shade, testbed_nerf.cu:2229-2659,
 * 948-1196, 2164-2226; ERenderMode::Shade, pinhole). camera: the view (xform after
 * nerf_matrix_to_ngp, focal length in pixels, principal point); the screen centre is
 * render_screen_center(1 - principal point) = the principal point (set_camera_to_training_view,
 * testbed.cu:852, 4376-4379). spp samples starting at sample_index are averaged;
 * out_rgba: device float [height x width x 4], linear colours composited over background_rgba
 * (host, linear; NULL = transparent black). bitfield: the occupancy bitfield (NULL = march everywhere). */
typedef struct ngp_nerf_renderer ngp_nerf_renderer;
int ngp_nerf_renderer_create(ngp_nerf_renderer** out);
void ngp_nerf_renderer_destroy(ngp_nerf_renderer* r);
/* ERenderMode of the following renders (common.h:110-119): 1 Shade (default), 2 Normals (testbed_nerf.cu:
 * 1183-1188, 2179-2181, 2615-2617: the density output's input gradient per step, ngp_input_gradient with
 * backprop_scale 128, composited as normalize(-density'(raw) * gradient), shaded as (0.5 n + 0.5) * alpha),
 * 0 AO (each step's alpha), 3 Positions ((pos - 0.5) / 2 + 0.5, show_accel off), 4 Depth (dot(camera forward,
 * pos - ray origin) * depth_scale): :1189-1208, composited like Shade, no sRGB decoding in the shade step (:2183).
 * depth_scale: 1 / the dataset's scale (render_nerf, testbed_nerf.cu:2822); default 1. */
int ngp_nerf_renderer_set_mode(ngp_nerf_renderer* r, int render_mode);
int ngp_nerf_renderer_set_depth_scale(ngp_nerf_renderer* r, float depth_scale);
/* render_mode 9 = ERenderMode::EncodingVis (common.h:120): each step's warped position, the network's input
 * (testbed_nerf.cu:1202-1203). show_accel (Testbed::Nerf::show_accel, testbed.cu:1678; -1 = off, else 0..7): the
 * march tests the occupancy grid from that mip up (:2497, 2594), every step is opaque (:1078-1080), and Positions
 * colours the step's occupancy cell (:1190-1199) */
int ngp_nerf_renderer_set_show_accel(ngp_nerf_renderer* r, int show_accel);
int ngp_nerf_render(ngp_nerf_renderer* r, ngp_model* model, const ngp_nerf_config* cfg, void* stream, const ngp_nerf_image* camera,
                    const uint8_t* bitfield, uint32_t spp, uint32_t sample_index, float min_transmittance,
                    const float* background_rgba, int use_inference_params, float* out_rgba);

/* Data-parallel NeRF training (no counterpart in the reference, which trains on one GPU: SURVEY F7,
 * §8e). `allreduce` reduces a device buffer in place across the ranks, ordered on `stream` (the
 * caller's RCCL/torch.distributed binding); it is called for the fp16 gradient buffer (sum, before
 * the optimizer), the density-grid splat (max) and three f32 counters (sum). Rank r traces the global
 * rays [R r / N, R (r+1) / N) with their global ids and compacts to B / N samples. */
enum { NGP_DTYPE_F32 = 0, NGP_DTYPE_F16 = 1 };
enum { NGP_REDUCE_SUM = 0, NGP_REDUCE_MAX = 1 };
/* Collectives of the sharded optimizer (ngp_trainer_set_data_parallel), passed in `op` of the same hook. `count`
 * is the whole buffer, a multiple of world; rank r's slice is [r count / world, (r + 1) count / world).
 * NGP_REDUCE_SCATTER_SUM: every rank's buffer summed, the sum of rank r's slice left in rank r's slice (other
 * slices undefined afterwards). NGP_ALL_GATHER: every rank's slice copied into that slice of every rank. */
enum { NGP_REDUCE_SCATTER_SUM = 2, NGP_ALL_GATHER = 3 };
typedef int (*ngp_allreduce_fn)(void* user, void* device_buf, uint64_t count, int dtype, int op, void* stream);
int ngp_nerf_trainer_set_data_parallel(ngp_nerf_trainer* t, uint32_t rank, uint32_t world, ngp_allreduce_fn allreduce, void* user);
// Sampler pipelining (default on, single GPU): when no density-grid update is due before the next
// step, ngp_nerf_train_step launches the next step's ray sampling on an internal stream right after
// this step's loss pass, so it runs under this step's training pass (identical samples: the sampler
// reads only the occupancy bitfield, the rng and the ray count). Disable before modifying the density
// grid or bitfield between steps (ngp_nerf_trainer_buffers discards a prelaunched sampler). No reference counterpart (the
// Testbed runs the step serially, testbed_nerf.cu:3867-4132).
int ngp_nerf_trainer_set_pipeline(ngp_nerf_trainer* t, int enable);

/* The training error map (Testbed::Nerf::Training::ErrorMap, testbed.h:668-677, 736-738). Every step
 * deposits the compacted rays' losses into it (accumulate_error, testbed_nerf.cu:3951-3953, 4044); it is
 * zeroed and resized to min(3.5 (n_steps_between * rays_per_batch / n_images)^(1/4), image size) when a
 * window starts (:3659-3666), and after n_steps_between steps its CDFs are built (construct_cdf_2d/1d and
 * the host pass over the per-image totals, :3700-3748) and the window grows by 1.5x. which: 0 data
 * [n_images][height][width], 1 cdf_x_cond_y (cdf resolution), 2 cdf_y [n_images][cdf_height], 3 cdf_img
 * [n_images] (the normalised image CDF), 4 pmf_img [n_images] (host). Copies min(cap, size) floats to
 * host memory `out` (NULL: only *info) after the trainer's stream work. */
typedef struct {
	uint32_t width, height;          /* error_map.resolution */
	uint32_t cdf_width, cdf_height;  /* error_map.cdf_resolution */
	uint32_t n_images;
	uint32_t cdf_valid;              /* error_map.is_cdf_valid */
	uint32_t n_steps_since_update, n_steps_between_updates;
	uint64_t size;                   /* floats held by the requested array */
} ngp_nerf_error_map_info;
int ngp_nerf_trainer_error_map(ngp_nerf_trainer* t, int which, float* out, uint64_t cap, ngp_nerf_error_map_info* info);

/* Snapshots (Testbed::save_snapshot / load_snapshot, src/testbed.cu:4873-5057; python_api.cu:446-447):
 * msgpack of the network config (network_config_json, the Testbed's m_network_config; NULL = {}) with
 * a "snapshot" member holding tcnn Trainer::serialize (n_params, params_type "__half", params_binary),
 * [optimizer state], version 1, mode "nerf", density_grid_size, density_grid_binary (fp16), nerf.aabb_scale,
 * nerf.rgb counters, training_step, loss, aabb. Paths ending in .ingp are gzip streams (zstr; level 0
 * unless compress), others raw msgpack; loading accepts gzip, zlib or raw. Loading restores the params
 * (and the optimizer state if present), the density grid (mean and bitfield recomputed), the
 * rays-per-batch counters and the training step; the network must have the snapshot's n_params. */
int ngp_nerf_save_snapshot(ngp_nerf_trainer* t, void* stream, const char* path, const char* network_config_json,
                           int include_optimizer_state, int compress);
int ngp_nerf_load_snapshot(ngp_nerf_trainer* t, void* stream, const char* path);
/* Testbed::save_snapshot / load_snapshot for the image and SDF testbeds (testbed.cu:4873-5057): the trainer's
 * Trainer::serialize members (as in the NeRF snapshot), version, mode (e.g. "sdf", "image"), training_step, loss,
 * aabb {min, max} and bounding_radius. Loading restores the parameters (and the optimizer state if present; an
 * optimizer member lacking some arrays fills them from the parameters / zeros) and returns the scalars (each output
 * nullable; bounding_radius keeps its value when the snapshot has none). ngp_snapshot_mode: the snapshot's mode
 * (a NeRF snapshot without one: "nerf"), for a Testbed to switch mode before reset_network. */
int ngp_save_snapshot(ngp_trainer* t, void* stream, const char* path, const char* network_config_json, const char* mode,
                      const float* aabb_min, const float* aabb_max, float bounding_radius, uint32_t training_step, float loss,
                      int include_optimizer_state, int compress);
int ngp_load_snapshot(ngp_trainer* t, void* stream, const char* path, uint32_t* training_step, float* loss, float* aabb_min,
                      float* aabb_max, float* bounding_radius);
int ngp_snapshot_mode(const char* path, char* mode_buf, uint64_t cap);
/* Testbed::load_network_config (testbed.cu:246) of a snapshot: the config as JSON text without the
 * "snapshot" member (binaries as {"binary_bytes": n}); size query with json_buf = NULL. */
int ngp_snapshot_network_config(const char* path, char* json_buf, uint64_t* size);

/* The engine's own RCCL communicator (engine extension; SURVEY §8e exchange step). Rank 0 makes the
 * id, every rank passes the same bytes (any host channel) to ngp_dp_comm_create, which blocks until
 * all `world` ranks have joined; call it with the rank's HIP device current. ngp_dp_comm_allreduce
 * is an ngp_allreduce_fn (user = the communicator): ncclAllReduce in place on `stream`, graph-capturable. */
#define NGP_DP_UNIQUE_ID_BYTES 128
typedef struct ngp_dp_comm ngp_dp_comm;
int ngp_dp_comm_unique_id(uint8_t* id_out);
int ngp_dp_comm_create(uint32_t rank, uint32_t world, const uint8_t* id_in, ngp_dp_comm** out);
void ngp_dp_comm_destroy(ngp_dp_comm* c);
int ngp_dp_comm_allreduce(void* user, void* device_buf, uint64_t count, int dtype, int op, void* stream);
/* Wire type of fp16 sums (default NGP_DTYPE_F32: widened to fp32, all-reduced, rounded to fp16 once —
 * RCCL's fp16 ring rounds at every hop, so its sum depends on N and ring order; NGP_DTYPE_F16: half the
 * bytes). ngp_dp_comm_reserve sizes the fp32 staging buffer for `count` elements; it must run outside
 * graph capture (the trainers call it when the communicator is bound). */
int ngp_dp_comm_set_wire(ngp_dp_comm* c, int dtype);
int ngp_dp_comm_reserve(ngp_dp_comm* c, uint64_t count);
/* Gradient exchange inside the trainer's step (network-level data parallelism, bench.py --gpus N):
 * after every forward_backward captured by ngp_trainer_capture_training_step, and before the
 * optimizer, the fp16 gradient buffer is all-reduced (sum) with `allreduce`; the optimizer divides
 * by `world` (mean gradient) on top of its loss scale. allreduce = NULL turns it off. */
int ngp_trainer_set_allreduce(ngp_trainer* t, uint32_t world, ngp_allreduce_fn allreduce, void* user);
/* The same exchange with this process's rank, so that large-table (lazy-EMA) trainers shard the optimizer
 * (trainer option "shard_opt", default 1): the fp16 gradients, widened to fp32, are reduce-scattered; rank r
 * updates the optimizer records of its 1/world slice of the parameters from the fp32 sums rounded to fp16
 * once (bit for bit the all-reduce path's update) and the fp16 weights are all-gathered: half the wire bytes
 * of an fp32 all-reduce and 1/world of the update per rank. Other trainers, and shard_opt 0, all-reduce.
 * With world > 1 the records of other ranks' slices are stale on this rank after a sharded step: the EMA
 * (inference) parameters, the full-precision weights and serialize need ngp_trainer_gather_shards first,
 * called on every rank (they fail otherwise); the fp16 training parameters are always complete. */
int ngp_trainer_set_data_parallel(ngp_trainer* t, uint32_t rank, uint32_t world, ngp_allreduce_fn fn, void* user);
/* Collective (every rank, same order): all-gather the sharded optimizer records so that every rank holds the
 * whole optimizer state again. A no-op unless a sharded step left them partial. */
int ngp_trainer_gather_shards(ngp_trainer* t, void* stream);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif

#endif /* NGP_ENGINE_H */
