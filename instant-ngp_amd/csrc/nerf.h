// nerf.h — NeRF training kernels (sampling, loss + compaction, rollover, occupancy grid) for gfx950.
//
// Re-implements src/testbed_nerf.cu's training kernels without OptiX.
// Difference by design: the reference assigns sample / ray / compacted slots with
// atomicAdd counters, so its sample order is nondeterministic; here slots come from exclusive
// prefix scans in ray order, so the output is deterministic and equal to the reference's as a
// multiset keyed by (ray, step). Counters keep the reference's meaning (totals include rays that
// were dropped for exceeding the sample budget).
#pragma once
#include "../../include/ngp_engine.h"
#include "common.h"
#include "lens.h"

#include <functional>

namespace ngp {
namespace nerf {

constexpr uint32_t GRIDSIZE = 128;                         // NERF_GRIDSIZE (nerf.h:24-30)
constexpr uint32_t GRID_N_CELLS = GRIDSIZE * GRIDSIZE * GRIDSIZE;
constexpr uint32_t CASCADES = 8;                           // NERF_CASCADES (testbed_nerf.cu:59)
constexpr uint32_t STEPS = 1024;                           // NERF_STEPS (:58)
constexpr float SQRT3 = 1.73205080757f;
constexpr float MIN_CONE_STEPSIZE = SQRT3 / STEPS;         // STEPSIZE() (:65-71)
constexpr float MAX_CONE_STEPSIZE = MIN_CONE_STEPSIZE * (1 << (CASCADES - 1)) * STEPS / GRIDSIZE;  // (:76-79)
constexpr uint32_t N_MAX_RANDOM_SAMPLES_PER_RAY = 16;      // (:85-87)
constexpr float MIN_OPTICAL_THICKNESS = 0.01f;             // (:92-94)
constexpr uint32_t BITFIELD_BYTES = GRID_N_CELLS * CASCADES / 8;  // grid_mip_offset(NERF_CASCADES)/8

enum Activation : uint32_t { ACT_NONE = 0, ACT_RELU = 1, ACT_LOGISTIC = 2, ACT_EXP = 3 };
enum LossType : uint32_t { LOSS_L2 = 0, LOSS_L1 = 1, LOSS_MAPE = 2, LOSS_SMAPE = 3, LOSS_HUBER = 4, LOSS_LOGL1 = 5, LOSS_RELL2 = 6 };

struct Camera {          // per image, device side
	uint32_t width, height;
	float focal[2], principal[2];
	float m[12];         // effective camera matrix (rolling-shutter slerp at t=0 applied on the host)
	uint64_t pixel_offset;  // first RGBA8 pixel of this image in the packed image buffer
	uint32_t lens_mode;  // LensMode (lens.h)
	float lens[4];
};

struct Rng { uint64_t state, inc; };  // tcnn::pcg32 state

// Host: effective camera matrix = get_xform_given_rolling_shutter(start == end, t = 0)
// (common_device.cuh:401-408): rotation goes through glm quat_cast / slerp / normalize / mat3_cast.
void effective_camera_matrix(const float xform[12], float out[12]);

struct Dataset {
	uint32_t n_images = 0;
	Camera* d_cams = nullptr;
	uint32_t* d_pixels = nullptr;  // RGBA8 packed, sRGB
	std::vector<Camera> cams;
	~Dataset();
};

struct SampleArgs {
	uint32_t n_rays, ray_offset, n_rays_total_for_image_idx;  // image_idx uses the global ray id
	uint32_t max_samples;
	Rng rng;
	const uint8_t* bitfield;
	uint32_t* ray_indices;     // [n_rays] compacted
	float* rays;               // [n_rays x 6] {o, d} (unnormalized d)
	uint32_t* numsteps;        // [n_rays x 2] {numsteps, base}
	float* coords;             // [max_samples x 7] NerfCoordinate
	uint32_t* counters;        // [2]: rays kept, numsteps total (incl. dropped)
};

struct LossArgs {
	uint32_t n_rays;           // rays_per_batch (kernel grid); rays kept are counters[0]
	uint32_t n_rays_total_for_image_idx;
	Rng rng;
	uint32_t max_samples_compacted;
	const uint32_t* ray_counter;
	const f16* network_output;  // [n x out_stride] rows 0..2 raw rgb, 3 raw density
	uint32_t out_stride;       // 16 (padded_output_width) or 4 (NGP_LAYOUT_AOS_RGBD)
	const uint32_t* ray_indices;
	const float* rays;
	uint32_t* numsteps;        // in: {numsteps, base}; out: {compacted numsteps, compacted base}
	const float* coords_in;
	float* coords_out;         // [max_samples_compacted x 7]
	f16* dloss_doutput;        // [max_samples_compacted x 16]
	float* loss;               // [n_rays]
	bool zero_loss;            // pass 1 zeroes loss[0, n_rays) (the Testbed step's memset, testbed_nerf.cu:3579)
	uint32_t* compacted_counter;  // [1]
	const float* mean_density;    // [1]
	float loss_scale;
	float bg[3];
	// training error map (testbed_nerf.cu:1869-1899): each compacted ray adds its mean loss, bilinearly
	// split, into [n_images][em_h][em_w] floats; null: off
	float* error_map;
	uint32_t em_w, em_h;
	// optional (null: off): pass 1 stores, per sample it composites, the weight, the transmittance after it and
	// the rgb prefix through it ([5][state_cap] floats, indexed by the pre-compaction sample), and pass 2 reads
	// them instead of compositing each ray again. Same float operations, so the same bits either way.
	float* state;
	uint64_t state_cap;
	// optional (null: off): the loss's compaction scan also publishes the step's counters to host-mapped memory
	// ({ray_counter[0], ray_counter[1], compacted total, 0}, then pub_seq at [4] after a system-scope fence), as soon
	// as they are final: the host sizes the next step while pass 2, the rollover and the training pass run
	volatile uint32_t* pub_host;
	uint32_t pub_seq;
};

// The kernels (each cites its reference kernel in nerf.hip).
void sample_rays(const Dataset& ds, const ngp_nerf_config& cfg, const SampleArgs& a, uint32_t* tmp_u32, float* tmp_f32, hipStream_t s);
size_t sample_tmp_u32(uint32_t n_rays);  // u32 of sample_rays' tmp_u32 (counts, count-wave sums and prefixes)
void compute_loss(const Dataset& ds, const ngp_nerf_config& cfg, const LossArgs& a, uint32_t* tmp_u32, float* tmp_f32, hipStream_t s);
void fill_rollover_f16(uint32_t n_elements, uint32_t stride, const uint32_t* n_input, f16* data, bool rescale, hipStream_t s);
void fill_rollover_f32(uint32_t n_elements, uint32_t stride, const uint32_t* n_input, float* data, hipStream_t s);
void fill_rollover_pair(uint32_t n_elements, const uint32_t* n_input, f16* dloss, uint32_t stride16, float* coords,
                        uint32_t stride32, hipStream_t s);
// What the single-GPU NeRF step does right after the rollover, in the same launch (block 0, thread 0): publish the
// step's counters ctr[0..3] to host-mapped memory (then seq, after a system-scope fence; host null: published
// earlier, by the loss's scan), and write the optimizer control block the training graph reads ({ctl[0] = step,
// ctl[CTL_CFG..] = cfg}, set_device_ctl). bytes: cfg.
struct StepPublish {
	const uint32_t* ctr; volatile uint32_t* host; uint32_t seq;
	uint32_t* ctl; uint32_t step; uint32_t cfg_off, cfg_words; uint32_t cfg[32];  // cfg at ctl + cfg_off (words)
};
void fill_rollover_pair_publish(uint32_t n_elements, const uint32_t* n_input, f16* dloss, uint32_t stride16, float* coords,
                                uint32_t stride32, const StepPublish& pub, hipStream_t s);
void grid_generate_samples(uint32_t n, Rng rng, uint32_t step, const ngp_nerf_config& cfg, const float* grid_in,
                           uint32_t n_cascades, float thresh, float* positions, uint32_t* indices, uint32_t* mask, hipStream_t s);
size_t grid_mask_words(uint32_t n_cascades);  // u32 of grid_generate_samples' cell mask
void grid_splat_max(uint32_t n, const uint32_t* indices, const f16* density_rm, uint32_t density_activation, float* grid_tmp,
                    hipStream_t s);
// memset(grid_tmp, 0) + grid_splat_max as a counting sort by cell bin: writes all n_cells of grid_tmp; scratch holds
// grid_splat_scratch_u32(n, n_cells) words
size_t grid_splat_scratch_u32(uint32_t n, uint32_t n_cells);
void grid_splat_max_binned(uint32_t n, const uint32_t* indices, const f16* density_rm, uint32_t density_activation,
                           float* grid_tmp, uint32_t n_cells, uint32_t* scratch, hipStream_t s);
// The update's samples in bin order before the density evaluation (which then runs ~1.8x faster on grouped positions):
// grid_sort_samples writes 16-B records (x, y, z, cell within the bin) sorted by 8192-cell bin (order within a bin
// arbitrary; recs: 4 n floats) and keeps the bins' offsets in scratch (grid_sort_scratch_u32 words); the density reads
// the records with stride 4; grid_splat_sorted then writes every cell of grid_tmp from the densities of the sorted
// samples [lo, hi) (density_rm[k - lo]) = memset + splat of those samples.
size_t grid_sort_scratch_u32(uint32_t n, uint32_t n_cells);
void grid_sort_samples(uint32_t n, const float* positions, const uint32_t* indices, uint32_t n_cells, uint32_t* scratch,
                       float* recs, hipStream_t s);
void grid_splat_sorted(uint32_t n_cells, const uint32_t* scratch, const float* recs, const f16* density_rm, uint32_t lo, uint32_t hi,
                       uint32_t density_activation, float* grid_tmp, hipStream_t s);
void grid_ema(uint32_t n, float decay, float* grid, const float* grid_tmp, hipStream_t s);
void grid_mean_bitfield(const float* grid, uint32_t max_cascade, float* mean_out, uint8_t* bitfield, hipStream_t s);
// grid_ema then grid_mean_bitfield in three launches (the density grid update's finalization; n_el >= GRID_N_CELLS)
void grid_ema_mean_bitfield(uint32_t n_el, float decay, float* grid, const float* tmp, uint32_t max_cascade, float* mean_out,
                            uint8_t* bitfield, hipStream_t s);
size_t sample_tmp_f32(uint32_t n_rays);  // floats of sample_rays' tmp_f32 (stored t per step + ray geometry)
size_t loss_tmp_f32(uint32_t n_rays);    // floats of compute_loss' tmp_f32 (per-ray pass-1 results)
// construct_cdf_2d / construct_cdf_1d (testbed_nerf.cu:2356-2410) over the error map
void error_map_cdfs(uint32_t n_images, uint32_t w, uint32_t h, const float* data, float* cdf_x_cond_y, float* cdf_y,
                    float* cdf_img, hipStream_t s);

// ---- rendering (NerfTracer) ------------------------------------------------------------------
struct RenderArgs {
	uint32_t width, height;
	float focal[2], screen_center[2];
	float cam[12];                 // camera-to-world mat4x3 (column-major)
	uint32_t lens_mode;            // render_lens of the training view (testbed.cu:846)
	float lens[4];
	float near_distance;
	float aabb_min[3], aabb_max[3];
	float cone_angle_constant;
	uint32_t max_mip;              // max_cascade
	const uint8_t* bitfield;
	uint32_t sample_index, snap_to_pixel_centers, linear_colors;
	uint32_t rgb_activation, density_activation;
	float min_transmittance;
	float background[4];           // linear rgba
	uint32_t render_mode;          // ERenderMode (common.h:110-121): 0 AO, 1 Shade, 2 Normals, 3 Positions, 4 Depth, 9 EncodingVis
	float depth_scale;             // ERenderMode::Depth: 1 / dataset scale (testbed_nerf.cu:2822)
	int32_t show_accel;            // Testbed::Nerf::show_accel (-1 off): the march's minimum mip, alpha 1, Positions by cell
};
enum : uint32_t { RENDER_AO = 0, RENDER_SHADE = 1, RENDER_NORMALS = 2, RENDER_POSITIONS = 3, RENDER_DEPTH = 4, RENDER_ENCODING_VIS = 9 };
struct RenderWorkspace {
	void* payload[2]; void* payload_hit;
	float* rgba[2]; float* rgba_hit;
	float* coords;                 // [2^21 + 256 x 7]
	f16* out;                      // [16 x (2^21 + 256)] RM
	float* frame;                  // [W*H x 4]
	uint32_t* counters;            // device [2]
	uint32_t* host_counters;       // pinned [2]
};
size_t render_payload_bytes();
// spp samples of one view, averaged into out (linear RGBA [H x W x 4]); infer(n, coords, out_rm)
// evaluates the network on n NerfCoordinates (output RM, row stride n). Normals: grad(n, coords) then
// overwrites the coordinates' position rows with d(density output)/d(position) (Network::input_gradient,
// testbed_nerf.cu:2615-2617).
void render_frame(const RenderArgs& a, uint32_t spp, RenderWorkspace& ws,
                  const std::function<void(uint32_t, const float*, f16*)>& infer, float* out, hipStream_t s,
                  const std::function<void(uint32_t, float*)>& grad = nullptr);

}  // namespace nerf
}  // namespace ngp
