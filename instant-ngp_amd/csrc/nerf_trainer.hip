// nerf_trainer.hip — C-ABI for the NeRF kernels and the Testbed-level NeRF training step.
//
// ngp_nerf_train_step mirrors Testbed::train for NeRF (src/testbed.cu:4285-4370): training_prep_nerf
// (occupancy-grid update every clamp(step/16, 1, 16) steps, testbed_nerf.cu:4137-4152) then
// train_nerf (testbed_nerf.cu:3611-3862): sample -> inference over every sample -> loss/compaction
// -> rollover -> forward/backward on the compacted batch -> optimizer step -> counters (host sync) ->
// rays_per_batch adaptation.
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <zlib.h>

#include <chrono>
#include <fstream>
#include <sstream>

#include "engine_internal.h"
#include "json.h"
#include "msgpack.h"
#include "nerf.h"
#include "profiler.h"

using namespace ngp;
using namespace ngp::nerf;

struct ngp_nerf_dataset {
	Dataset ds;
};

namespace {

struct HostPcg {  // tcnn::pcg32 (host) for the Testbed's m_rng / density_grid_rng
	uint64_t state, inc;
	explicit HostPcg(uint64_t initstate, uint64_t initseq = 1u) {
		state = 0u; inc = (initseq << 1u) | 1u; next_uint(); state += initstate; next_uint();
	}
	uint32_t next_uint() {
		const uint64_t old = state;
		state = old * 0x5851f42d4c957f2dULL + inc;
		const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u), rot = (uint32_t)(old >> 59u);
		return (xs >> rot) | (xs << ((~rot + 1u) & 31));
	}
	void advance(uint64_t delta = (1ull << 32)) {
		uint64_t cm = 0x5851f42d4c957f2dULL, cp = inc, am = 1u, ap = 0u;
		while (delta > 0) {
			if (delta & 1) { am *= cm; ap = ap * cm + cp; }
			cp = (cm + 1) * cp; cm *= cm; delta /= 2;
		}
		state = am * state + ap;
	}
	Rng dev() const { return Rng{state, inc}; }
};

struct Buf {
	void* p = nullptr;
	size_t n = 0;
	template <typename T> T* get(size_t count) {
		const size_t need = count * sizeof(T);
		if (need > n) {
			if (p) NGP_HIP(hipFree(p));
			NGP_HIP(hipMalloc(&p, need));
			n = need;
		}
		return (T*)p;
	}
	~Buf() { if (p) (void)hipFree(p); }
};

}  // namespace

// external engine entry points used by the orchestrator
extern "C" int ngp_inference(ngp_model*, void*, uint32_t, const float*, uint32_t, void*, uint32_t, uint32_t, int);
extern "C" int ngp_density(ngp_model*, void*, uint32_t, const float*, uint32_t, void*, uint32_t, uint32_t, int);
extern "C" int ngp_forward_backward(ngp_model*, void*, uint32_t, const float*, uint32_t, void*, uint32_t, const void*, uint32_t, int);
extern "C" int ngp_trainer_optimizer_step(ngp_trainer*, void*, float);
extern "C" void* ngp_trainer_gradients(ngp_trainer*);
extern "C" uint64_t ngp_model_n_params(const ngp_model*);
extern "C" const char* ngp_last_error(void);

struct ngp_nerf_renderer {
	Buf pay0, pay1, payh, rgba0, rgba1, rgbah, coords, out, frame, counters;
	uint32_t* host_counters = nullptr;
	uint32_t render_mode = RENDER_SHADE;  // ngp_nerf_renderer_set_mode
	int32_t show_accel = -1;             // ngp_nerf_renderer_set_show_accel
	float depth_scale = 1.0f;             // ngp_nerf_renderer_set_depth_scale
	~ngp_nerf_renderer() { if (host_counters) (void)hipHostFree(host_counters); }
};

struct ngp_nerf_trainer {
	ngp_model* model;
	ngp_trainer* trainer;
	const ngp_nerf_dataset* data;
	ngp_nerf_config cfg;
	HostPcg rng{1337}, grid_rng{1};
	uint32_t training_step = 0, ema_step = 0;
	uint32_t rays_per_batch = 1u << 12;  // testbed.h:440
	uint32_t n_rays_total = 0;
	uint32_t measured_batch_size = 0, measured_before_compaction = 0;
	uint32_t measured_before_compaction_local = 0;  // this rank's pre-compaction count (inference sizing)
	float loss_scalar = 0.f;  // m_loss_scalar (last step that computed the loss)
	// the training pass (forward_backward + optimizer over the fixed compacted batch) replayed as one
	// HIP graph per step; re-captured if its buffers move
	ngp_graph* train_graph = nullptr;
	const void* graph_in = nullptr;
	const void* graph_dl = nullptr;
	uint32_t graph_n = 0;
	uint64_t graph_epoch = 0;  // model workspace epoch at capture (ngp_model_workspace_epoch)
	hipStream_t own_stream = nullptr;  // used when the caller passes the null stream (graphs need a stream)
	// per-step counters published by the step's last kernel into host-coherent pinned memory, read by
	// spinning on a sequence number (no copy-engine transfer, no blocking stream synchronize)
	volatile uint32_t* host_ctr = nullptr;
	uint32_t publish_seq = 0;
	// Sampler pipelining: the next step's ray sampling depends on the occupancy bitfield, the rng and the
	// rays-per-batch count, not on the network, so (when no density-grid update is due before it) it is
	// launched on `sample_stream` as soon as this step's loss pass has released the sample buffers and
	// runs concurrently with this step's training pass. Same kernels, same inputs: same samples.
	bool pipeline = true;                // ngp_nerf_trainer_set_pipeline
	bool prelaunched = false;
	uint32_t pre_R = 0, pre_max_inference = 0;
	hipStream_t sample_stream = nullptr;
	hipEvent_t ev_free = nullptr, ev_samp = nullptr;
	// The sampler -> inference handoff as hipStreamWriteValue32 / hipStreamWaitValue32 on signal memory: a queue
	// idling on a pending event wait starts its next kernel ~10 us after the event's work ends, on a pending value
	// wait ~6 us
	// (tools/microbench/queue_handoff.hip, profiles/r06s_queue_handoff.jsonl): Lego step 0.433 -> 0.428 ms, fox
	// 0.542 -> 0.535 ms (gpurun_out/r06t; the release handoff by value too, NGP_NERF_WAITVAL=2: Lego 0.427, fox 0.538).
	// NGP_NERF_WAITVAL=0: the events (A/B)
	uint32_t* sig_samp = nullptr;
	uint32_t* sig_free = nullptr;
	uint32_t seq_samp = 0, seq_free = 0;
	void ensure_signals() {
		if (sig_samp) return;
		NGP_HIP(hipExtMallocWithFlags((void**)&sig_samp, 8, hipMallocSignalMemory));
		NGP_HIP(hipExtMallocWithFlags((void**)&sig_free, 8, hipMallocSignalMemory));
		NGP_HIP(hipMemset(sig_samp, 0, 8));
		NGP_HIP(hipMemset(sig_free, 0, 8));
	}
	// Density-grid update pipelining: when the next step is due an update, its sample generation and bin sort read
	// only the grid (unchanged until that update) and the grid rng, so they run on `sample_stream` under this step's
	// training pass; the update then starts at the density evaluation (ev_gen). Discarding them restores the rng.
	bool grid_pregen = false;
	uint32_t pregen_nu = 0, pregen_nn = 0;
	hipEvent_t ev_gen = nullptr;
	HostPcg pregen_rng{1};  // grid_rng before the pregenerated samples
	void drain() {  // the prelaunched sampler finished and discarded (state is about to change)
		if (sample_stream) (void)hipStreamSynchronize(sample_stream);
		prelaunched = false;
		if (grid_pregen) grid_rng = pregen_rng;
		grid_pregen = false;
	}
	~ngp_nerf_trainer() {
		drain();
		if (train_graph) ngp_graph_destroy(train_graph);
		if (own_stream) (void)hipStreamDestroy(own_stream);
		if (sample_stream) (void)hipStreamDestroy(sample_stream);
		for (hipEvent_t e : {ev_free, ev_samp, ev_gen})
			if (e) (void)hipEventDestroy(e);
		for (uint32_t* p : {sig_samp, sig_free})
			if (p) (void)hipFree(p);
		if (host_ctr) (void)hipHostFree((void*)host_ctr);
	}
	// data parallelism: rank r traces global rays [R r / N, R (r+1) / N), compacts to B / N,
	// evaluates 1/N of the density-grid samples; the exchange steps go through `allreduce`
	uint32_t rank = 0, world = 1;
	ngp_allreduce_fn allreduce = nullptr;
	void* allreduce_user = nullptr;
	bool dp_capturable = false;  // the hook is the engine's RCCL communicator: the DP training pass is a graph
	Buf dp_scalars;
	bool dp() const { return allreduce != nullptr; }
	// the training pass's exchange: the shards' dL/doutput is already scaled by 128 / R_global, so the summed
	// gradient is the 1-GPU gradient (world factor 1)
	ngp::Exchange exchange() const {
		ngp::Exchange e;
		e.fn = allreduce; e.user = allreduce_user; e.rank = rank; e.world = world; e.world_factor = 1.f;
		e.rank_known = allreduce != nullptr;
		return e;
	}
	// occupancy grid
	Buf grid, grid_tmp, bitfield, mean, gpos, gidx, gdens, grid_mask, splat_scratch, gpos_sorted;
	// training workspaces
	Buf ray_indices, rays, numsteps, coords, mlp_out, dloss, coords_c, loss, counters, scan_tmp, tmp_u32, tmp_f32;
	// Early publish (one GPU): the counters are published by the loss's scan, so the host launches the next step's
	// sampler while this step's loss pass 2, rollover and training pass still run; the sampler's outputs then
	// alternate between two sets by step parity (the set it writes was last read two steps before), so it waits on
	// nothing. Default under cone stepping only (aabb_scale > 1: the count pass, ~1.5x the training pass, is the
	// step's critical path; fox 0.517 -> 0.499 ms); at cone 0 the two are balanced and a count pass already resident
	// when the training pass starts keeps its one-wave-per-SIMD MLP kernel off the SIMDs (Lego 0.421 -> 0.440 ms,
	// gpurun_out/r06bd). NGP_NERF_EARLY=1: always, 0: never (publish in the rollover, one set, the sampler waits
	// for this step's release).
	Buf ray_indices_b, rays_b, numsteps_b, coords_b, counters_b;
	bool early() const {
		static const int knob = getenv("NGP_NERF_EARLY") ? atoi(getenv("NGP_NERF_EARLY")) : -1;
		const bool on = knob < 0 ? cfg.cone_angle_constant > 1e-5f : knob != 0;
		return on && !dp();
	}
	Buf loss_state;  // compute_loss: pass 1's per-sample compositing state for pass 2 (LossArgs::state)
	// training error map (Testbed::Nerf::Training::ErrorMap and its update window, testbed.h:668-677, 736-738)
	Buf em_data, em_cdf_x, em_cdf_y, em_cdf_img;
	uint32_t em_w = 0, em_h = 0, em_cdf_w = 0, em_cdf_h = 0;
	uint32_t em_steps_since = 0, em_steps_between = 128;
	bool em_cdf_valid = false;
	std::vector<float> em_pmf_img;  // pmf_img_cpu
};

static hipStream_t S(void* s) { return (hipStream_t)s; }

#define NERF_TRY(...)                                  \
	try {                                              \
		__VA_ARGS__;                                   \
		return NGP_OK;                                 \
	} catch (const std::exception& e) {                \
		nerf_set_error(e.what());                      \
		return NGP_ERROR;                              \
	}

// share the engine's thread-local error string through a tiny hook in engine.hip
namespace ngp { void set_last_error(const char* msg); }
static void nerf_set_error(const char* m) { ngp::set_last_error(m); }

// mark_untrained_density_grid (testbed_nerf.cu:503-592) for perspective and OpenCV(-fisheye) cameras
__global__ void k_mark_untrained(uint32_t n_elements, float* __restrict__ grid, uint32_t n_images, const Camera* __restrict__ cams,
                                 const float* __restrict__ raw_xforms, bool clear_visible) {
	const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n_elements) return;
	if (grid[i] == -1.0f) return;
	const uint32_t level = i / GRID_N_CELLS, pos_idx = i % GRID_N_CELLS;
	auto inv = [](uint32_t x) {
		x = x & 0x49249249u; x = (x | (x >> 2)) & 0xc30c30c3u; x = (x | (x >> 4)) & 0x0f00f00fu;
		x = (x | (x >> 8)) & 0xff0000ffu; x = (x | (x >> 16)) & 0x0000ffffu; return x;
	};
	const uint32_t x = inv(pos_idx >> 0), y = inv(pos_idx >> 1), z = inv(pos_idx >> 2);
	const float vs = scalbnf(1.0f / GRIDSIZE, (int)level), sc = scalbnf(1.0f, (int)level);
	const float px = ((float)x / (float)GRIDSIZE - 0.5f) * sc + 0.5f;
	const float py = ((float)y / (float)GRIDSIZE - 0.5f) * sc + 0.5f;
	const float pz = ((float)z / (float)GRIDSIZE - 0.5f) * sc + 0.5f;
	uint32_t count = 0;
	for (uint32_t j = 0; j < n_images && count < 1; ++j) {
		const float* m = raw_xforms + 12 * j;  // training_xforms[j].start
		const Camera& cam = cams[j];
		// inverse(mat3(m)) via the adjugate (glm::inverse)
		const float a00 = m[0], a01 = m[1], a02 = m[2], a10 = m[3], a11 = m[4], a12 = m[5], a20 = m[6], a21 = m[7], a22 = m[8];
		const float det = a00 * (a11 * a22 - a21 * a12) - a10 * (a01 * a22 - a21 * a02) + a20 * (a01 * a12 - a11 * a02);
		const float id = 1.0f / det;
		float I[9];
		I[0] = (a11 * a22 - a21 * a12) * id; I[3] = -(a10 * a22 - a20 * a12) * id; I[6] = (a10 * a21 - a20 * a11) * id;
		I[1] = -(a01 * a22 - a21 * a02) * id; I[4] = (a00 * a22 - a20 * a02) * id; I[7] = -(a00 * a21 - a20 * a01) * id;
		I[2] = (a01 * a12 - a11 * a02) * id; I[5] = -(a00 * a12 - a10 * a02) * id; I[8] = (a00 * a11 - a10 * a01) * id;
		for (uint32_t k = 0; k < 8; ++k) {
			const float cx = px + ((k & 1) ? vs : 0.f), cy = py + ((k & 2) ? vs : 0.f), cz = pz + ((k & 4) ? vs : 0.f);
			float dx = cx - m[9], dy = cy - m[10], dz = cz - m[11];
			const float il = 1.0f / sqrtf(dx * dx + dy * dy + dz * dz);
			const float nx = dx * il, ny = dy * il, nz = dz * il;
			if (nx * m[6] + ny * m[7] + nz * m[8] < 1e-4f) continue;
			// pos_to_uv (common_device.cuh:547-585): perspective projection + forward lens distortion
			float ex = I[0] * dx + I[3] * dy + I[6] * dz, ey = I[1] * dx + I[4] * dy + I[7] * dz, ez = I[2] * dx + I[5] * dy + I[8] * dz;
			ex /= ez; ey /= ez;
			float du, dv;
			lens_delta(cam.lens_mode, cam.lens, ex, ey, &du, &dv);
			ex += du; ey += dv;
			const float u = ex * cam.focal[0] / (float)cam.width + cam.principal[0];
			const float v = ey * cam.focal[1] / (float)cam.height + cam.principal[1];
			// uv_to_ray with the raw xform (pos_to_uv is not injective under distortion), compare directions
			float rx = (u - cam.principal[0]) * (float)cam.width / cam.focal[0];
			float ry = (v - cam.principal[1]) * (float)cam.height / cam.focal[1];
			lens_undistort(cam.lens_mode, cam.lens, &rx, &ry);
			const float ddx = m[0] * rx + m[3] * ry + m[6], ddy = m[1] * rx + m[4] * ry + m[7], ddz = m[2] * rx + m[5] * ry + m[8];
			const float rl = 1.0f / sqrtf(ddx * ddx + ddy * ddy + ddz * ddz);
			const float qx = ddx * rl - nx, qy = ddy * rl - ny, qz = ddz * rl - nz;
			if (u > 0.0f && v > 0.0f && u < 1.0f && v < 1.0f && sqrtf(qx * qx + qy * qy + qz * qz) < 1e-3f) { ++count; break; }
		}
	}
	if (clear_visible || (grid[i] < 0) != (count < 1)) grid[i] = count >= 1 ? 1.f : -1.f;
	else grid[i] = 1.0f;
}

extern "C" {

int ngp_nerf_default_config(float aabb_scale, ngp_nerf_config* o) {
	if (!o || !(aabb_scale >= 1.0f)) return NGP_INVALID;
	memset(o, 0, sizeof(*o));
	const float inflate = 0.5f * std::min((float)(1 << (CASCADES - 1)), aabb_scale);  // testbed_nerf.cu:3093-3094
	for (int k = 0; k < 3; ++k) { o->aabb_min[k] = 0.5f - inflate; o->aabb_max[k] = 0.5f + inflate; }
	uint32_t mc = 0;
	while ((float)(1u << mc) < aabb_scale) ++mc;  // :3102-3105
	o->max_cascade = mc;
	o->cone_angle_constant = aabb_scale <= 1.0f ? 0.0f : 1.0f / 256.0f;  // :3109
	o->snap_to_pixel_centers = 1;
	o->random_bg_color = 1;
	o->linear_colors = 0;
	o->color_space_linear = 1;
	o->rgb_activation = ACT_EXP;
	o->density_activation = ACT_EXP;
	o->loss_type = LOSS_HUBER;  // configs/nerf/base.json "loss": Huber
	o->near_distance = 0.1f;
	o->target_batch_size = 1u << 18;
	return NGP_OK;
}

int ngp_nerf_dataset_create(uint32_t n_images, const ngp_nerf_image* images, const void* const* rgba8, ngp_nerf_dataset** out) {
	if (!out || !images || !rgba8 || n_images == 0) return NGP_INVALID;
	NERF_TRY({
		auto d = std::make_unique<ngp_nerf_dataset>();
		d->ds.n_images = n_images;
		uint64_t total = 0;
		std::vector<Camera> cams(n_images);
		for (uint32_t i = 0; i < n_images; ++i) {
			const ngp_nerf_image& im = images[i];
			Camera& c = cams[i];
			c.width = im.width; c.height = im.height;
			c.focal[0] = im.focal_length[0]; c.focal[1] = im.focal_length[1];
			c.principal[0] = im.principal_point[0]; c.principal[1] = im.principal_point[1];
			NGP_CHECK(im.lens_mode <= LENS_OPENCV_FISHEYE, "nerf dataset: unsupported lens mode");
			c.lens_mode = im.lens_mode;
			for (int k = 0; k < 4; ++k) c.lens[k] = im.lens_params[k];
			effective_camera_matrix(im.xform, c.m);
			c.pixel_offset = total;
			total += (uint64_t)im.width * im.height;
		}
		NGP_HIP(hipMalloc(&d->ds.d_pixels, total * 4 + 12 * 4 * n_images));
		for (uint32_t i = 0; i < n_images; ++i)
			NGP_HIP(hipMemcpy(d->ds.d_pixels + cams[i].pixel_offset, rgba8[i], (size_t)images[i].width * images[i].height * 4,
			                  hipMemcpyHostToDevice));
		// raw (start) transforms after the pixels, for mark_untrained_density_grid
		std::vector<float> raw(12 * n_images);
		for (uint32_t i = 0; i < n_images; ++i) memcpy(&raw[12 * i], images[i].xform, 48);
		NGP_HIP(hipMemcpy(d->ds.d_pixels + total, raw.data(), raw.size() * 4, hipMemcpyHostToDevice));
		NGP_HIP(hipMalloc(&d->ds.d_cams, n_images * sizeof(Camera)));
		NGP_HIP(hipMemcpy(d->ds.d_cams, cams.data(), n_images * sizeof(Camera), hipMemcpyHostToDevice));
		d->ds.cams = cams;
		*out = d.release();
	});
}

void ngp_nerf_dataset_destroy(ngp_nerf_dataset* d) { delete d; }

static const float* raw_xforms(const Dataset& ds) {
	const Camera& last = ds.cams.back();
	return (const float*)(ds.d_pixels + last.pixel_offset + (uint64_t)last.width * last.height);
}

int ngp_nerf_generate_training_samples(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                                       uint32_t ray_offset, uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples,
                                       const uint8_t* bitfield, uint32_t* ray_indices, float* rays, uint32_t* numsteps,
                                       float* coords, uint32_t* counters) {
	if (!ds || !cfg || !bitfield || !ray_indices || !rays || !numsteps || !coords || !counters) return NGP_INVALID;
	NERF_TRY({
		SampleArgs a{};
		a.n_rays = n_rays; a.ray_offset = ray_offset; a.n_rays_total_for_image_idx = n_rays_total ? n_rays_total : n_rays;
		a.max_samples = max_samples; a.rng = Rng{rng.state, rng.inc}; a.bitfield = bitfield;
		a.ray_indices = ray_indices; a.rays = rays; a.numsteps = numsteps; a.coords = coords; a.counters = counters;
		static thread_local Buf tmp, tmpf;
		if (n_rays == 0) { NGP_HIP(hipMemsetAsync(counters, 0, 8, S(stream))); return NGP_OK; }
		sample_rays(ds->ds, *cfg, a, tmp.get<uint32_t>(sample_tmp_u32(n_rays)), tmpf.get<float>(sample_tmp_f32(n_rays)), S(stream));
	});
}

static int nerf_compute_loss(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                             uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted, const uint32_t* ray_counter,
                             const void* network_output, uint32_t out_stride, const uint32_t* ray_indices, const float* rays,
                             uint32_t* numsteps, const float* coords_in, float* coords_out, void* dloss_doutput, float* loss,
                             uint32_t* compacted_counter, const float* mean_density, float loss_scale, bool zero_loss = false,
                             float* error_map = nullptr, uint32_t em_w = 0, uint32_t em_h = 0, float* state = nullptr,
                             uint64_t state_cap = 0, volatile uint32_t* pub_host = nullptr, uint32_t pub_seq = 0);

int ngp_nerf_compute_loss(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                          uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted, const uint32_t* ray_counter,
                          const void* network_output, const uint32_t* ray_indices, const float* rays, uint32_t* numsteps,
                          const float* coords_in, float* coords_out, void* dloss_doutput, float* loss,
                          uint32_t* compacted_counter, const float* mean_density, float loss_scale) {
	return nerf_compute_loss(ds, cfg, stream, n_rays, n_rays_total, rng, max_samples_compacted, ray_counter, network_output, 16,
	                         ray_indices, rays, numsteps, coords_in, coords_out, dloss_doutput, loss, compacted_counter, mean_density,
	                         loss_scale);
}

int ngp_nerf_compute_loss_error_map(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                                    uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted,
                                    const uint32_t* ray_counter, const void* network_output, const uint32_t* ray_indices,
                                    const float* rays, uint32_t* numsteps, const float* coords_in, float* coords_out,
                                    void* dloss_doutput, float* loss, uint32_t* compacted_counter, const float* mean_density,
                                    float loss_scale, float* error_map, uint32_t em_width, uint32_t em_height) {
	if (error_map && (em_width < 2 || em_height < 2)) return NGP_INVALID;  // the bilinear deposit needs a 2x2 texel block
	return nerf_compute_loss(ds, cfg, stream, n_rays, n_rays_total, rng, max_samples_compacted, ray_counter, network_output, 16,
	                         ray_indices, rays, numsteps, coords_in, coords_out, dloss_doutput, loss, compacted_counter, mean_density,
	                         loss_scale, false, error_map, em_width, em_height);
}

int ngp_nerf_compute_loss_state(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                                uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted, const uint32_t* ray_counter,
                                const void* network_output, const uint32_t* ray_indices, const float* rays, uint32_t* numsteps,
                                const float* coords_in, float* coords_out, void* dloss_doutput, float* loss,
                                uint32_t* compacted_counter, const float* mean_density, float loss_scale, float* sample_state,
                                uint64_t state_capacity) {
	if (!sample_state || state_capacity == 0) return NGP_INVALID;
	return nerf_compute_loss(ds, cfg, stream, n_rays, n_rays_total, rng, max_samples_compacted, ray_counter, network_output, 16,
	                         ray_indices, rays, numsteps, coords_in, coords_out, dloss_doutput, loss, compacted_counter, mean_density,
	                         loss_scale, false, nullptr, 0, 0, sample_state, state_capacity);
}

static int nerf_compute_loss(const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg, void* stream, uint32_t n_rays,
                             uint32_t n_rays_total, ngp_rng rng, uint32_t max_samples_compacted, const uint32_t* ray_counter,
                             const void* network_output, uint32_t out_stride, const uint32_t* ray_indices, const float* rays,
                             uint32_t* numsteps, const float* coords_in, float* coords_out, void* dloss_doutput, float* loss,
                             uint32_t* compacted_counter, const float* mean_density, float loss_scale, bool zero_loss,
                             float* error_map, uint32_t em_w, uint32_t em_h, float* state, uint64_t state_cap,
                             volatile uint32_t* pub_host, uint32_t pub_seq) {
	if (!ds || !cfg || !ray_counter || !network_output || !numsteps || !coords_in || !coords_out || !dloss_doutput ||
	    !compacted_counter || !mean_density)
		return NGP_INVALID;
	NERF_TRY({
		LossArgs a{};
		a.n_rays = n_rays; a.n_rays_total_for_image_idx = n_rays_total ? n_rays_total : n_rays; a.rng = Rng{rng.state, rng.inc};
		a.max_samples_compacted = max_samples_compacted; a.ray_counter = ray_counter; a.network_output = (const f16*)network_output;
		a.out_stride = out_stride;
		a.ray_indices = ray_indices; a.rays = rays; a.numsteps = numsteps; a.coords_in = coords_in; a.coords_out = coords_out;
		a.dloss_doutput = (f16*)dloss_doutput; a.loss = loss; a.compacted_counter = compacted_counter;
		a.mean_density = mean_density; a.loss_scale = loss_scale; a.zero_loss = zero_loss;
		a.error_map = error_map; a.em_w = em_w; a.em_h = em_h;
		a.state = state; a.state_cap = state ? state_cap : 0;
		a.pub_host = pub_host; a.pub_seq = pub_seq;
		NGP_CHECK(n_rays > 0 || !pub_host, "compute_loss: the counters are published by the scan, which needs rays");
		if (n_rays == 0) { NGP_HIP(hipMemsetAsync(compacted_counter, 0, 4, S(stream))); return NGP_OK; }
		static thread_local Buf tmp, tmpf;
		compute_loss(ds->ds, *cfg, a, tmp.get<uint32_t>(2 * (size_t)n_rays), tmpf.get<float>(loss_tmp_f32(n_rays)), S(stream));
	});
}

int ngp_nerf_fill_rollover(void* stream, uint32_t n_elements, uint32_t stride, const uint32_t* n_input, void* data, int dtype,
                           int rescale) {
	if (!n_input || !data) return NGP_INVALID;
	NERF_TRY({
		if (dtype == 1) fill_rollover_f16(n_elements, stride, n_input, (f16*)data, rescale != 0, S(stream));
		else fill_rollover_f32(n_elements, stride, n_input, (float*)data, S(stream));
	});
}

int ngp_nerf_grid_generate_samples(void* stream, const ngp_nerf_config* cfg, uint32_t n, ngp_rng rng, uint32_t step,
                                   const float* grid, uint32_t n_cascades, float thresh, float* positions, uint32_t* indices) {
	if (!cfg || !grid || !positions || !indices) return NGP_INVALID;
	NERF_TRY({
		static thread_local Buf mask;
		grid_generate_samples(n, Rng{rng.state, rng.inc}, step, *cfg, grid, n_cascades, thresh, positions, indices,
		                      mask.get<uint32_t>(grid_mask_words(n_cascades)), S(stream));
	});
}
int ngp_nerf_grid_splat_max(void* stream, uint32_t n, const uint32_t* indices, const void* density_rm, uint32_t act, float* tmp) {
	if (!indices || !density_rm || !tmp) return NGP_INVALID;
	NERF_TRY(grid_splat_max(n, indices, (const f16*)density_rm, act, tmp, S(stream)));
}
int ngp_nerf_grid_splat_max_cells(void* stream, uint32_t n, const uint32_t* indices, const void* density_rm, uint32_t act,
                                  float* tmp, uint32_t n_cells) {
	if ((n && (!indices || !density_rm)) || !tmp || n_cells == 0 || n_cells % 8192 || n_cells > 8 * GRID_N_CELLS) return NGP_INVALID;
	NERF_TRY({
		static thread_local Buf scratch;
		grid_splat_max_binned(n, indices, (const f16*)density_rm, act, tmp, n_cells,
		                      scratch.get<uint32_t>(grid_splat_scratch_u32(n, n_cells)), S(stream));
	});
}
int ngp_nerf_grid_ema(void* stream, uint32_t n, float decay, float* grid, const float* tmp) {
	if (!grid || !tmp) return NGP_INVALID;
	NERF_TRY(grid_ema(n, decay, grid, tmp, S(stream)));
}
int ngp_nerf_grid_mean_and_bitfield(void* stream, const float* grid, uint32_t max_cascade, float* mean, uint8_t* bitfield) {
	if (!grid || !mean || !bitfield || max_cascade >= CASCADES) return NGP_INVALID;
	NERF_TRY(grid_mean_bitfield(grid, max_cascade, mean, bitfield, S(stream)));
}

// ---- Testbed-level ---------------------------------------------------------------------------
int ngp_nerf_trainer_create(ngp_model* model, ngp_trainer* trainer, const ngp_nerf_dataset* ds, const ngp_nerf_config* cfg,
                            uint64_t seed, ngp_nerf_trainer** out) {
	if (!model || !trainer || !ds || !cfg || !out) return NGP_INVALID;
	NERF_TRY({
		auto t = std::make_unique<ngp_nerf_trainer>();
		t->model = model; t->trainer = trainer; t->data = ds; t->cfg = *cfg;
		t->rng = HostPcg(seed);                          // m_rng = default_rng_t{m_seed} (testbed.cu:3906)
		t->grid_rng = HostPcg(t->rng.next_uint());       // density_grid_rng (testbed.cu:3919)
		const uint32_t n_el = GRID_N_CELLS * (cfg->max_cascade + 1);
		NGP_HIP(hipMemset(t->grid.get<float>(n_el), 0, (size_t)n_el * 4));
		NGP_HIP(hipMemset(t->bitfield.get<uint8_t>(BITFIELD_BYTES), 0, BITFIELD_BYTES));
		NGP_HIP(hipMemset(t->mean.get<float>(1 + 512), 0, (1 + 512) * 4));
		*out = t.release();
	});
}

void ngp_nerf_trainer_destroy(ngp_nerf_trainer* t) { delete t; }

int ngp_nerf_trainer_get_config(const ngp_nerf_trainer* t, ngp_nerf_config* out) {
	if (!t || !out) return NGP_INVALID;
	*out = t->cfg;
	return NGP_OK;
}

int ngp_nerf_trainer_set_config(ngp_nerf_trainer* t, const ngp_nerf_config* cfg) {
	if (!t || !cfg) return NGP_INVALID;
	NERF_TRY({
		NGP_CHECK(cfg->max_cascade == t->cfg.max_cascade, "set_config: max_cascade sizes the density grid (reset the trainer)");
		for (int k = 0; k < 3; ++k)
			NGP_CHECK(cfg->aabb_min[k] == t->cfg.aabb_min[k] && cfg->aabb_max[k] == t->cfg.aabb_max[k],
			          "set_config: the aabb is fixed for the trainer's lifetime (reset the trainer)");
		NGP_CHECK(cfg->target_batch_size > 0 && cfg->target_batch_size % 256 == 0, "set_config: target_batch_size");
		t->drain();  // a prelaunched sampler ran with the old knobs
		const bool early_was = t->early();
		t->cfg = *cfg;
		// the sample-set choice changes with the cone (ngp_nerf_trainer::early): let the last step's passes finish
		// reading their set first
		if (t->early() != early_was) NGP_HIP(hipDeviceSynchronize());
	});
}

static void check_rc(int rc) { if (rc != NGP_OK) throw Error(ngp_last_error()); }

// ---- rendering ---------------------------------------------------------------------------------
int ngp_nerf_renderer_create(ngp_nerf_renderer** out) {
	if (!out) return NGP_INVALID;
	NERF_TRY({ *out = new ngp_nerf_renderer(); });
}
void ngp_nerf_renderer_destroy(ngp_nerf_renderer* r) { delete r; }
int ngp_nerf_renderer_set_mode(ngp_nerf_renderer* r, int render_mode) {
	if (!r || render_mode < (int)RENDER_AO || (render_mode > (int)RENDER_DEPTH && render_mode != (int)RENDER_ENCODING_VIS))
		return NGP_INVALID;
	r->render_mode = (uint32_t)render_mode;
	return NGP_OK;
}
int ngp_nerf_renderer_set_show_accel(ngp_nerf_renderer* r, int show_accel) {
	if (!r || show_accel < -1 || show_accel >= (int)CASCADES) return NGP_INVALID;
	r->show_accel = show_accel;
	return NGP_OK;
}
int ngp_nerf_renderer_set_depth_scale(ngp_nerf_renderer* r, float depth_scale) {
	if (!r) return NGP_INVALID;
	r->depth_scale = depth_scale;
	return NGP_OK;
}

int ngp_nerf_render(ngp_nerf_renderer* r, ngp_model* model, const ngp_nerf_config* cfg, void* stream, const ngp_nerf_image* camera,
                    const uint8_t* bitfield, uint32_t spp, uint32_t sample_index, float min_transmittance, const float* background_rgba,
                    int use_inference_params, float* out_rgba) {
	if (!r || !model || !cfg || !camera || !out_rgba || spp == 0) return NGP_INVALID;
	NERF_TRY({
		hipStream_t s = S(stream);
		RenderArgs a{};
		a.width = camera->width; a.height = camera->height;
		a.focal[0] = camera->focal_length[0]; a.focal[1] = camera->focal_length[1];
		// m_screen_center = 1 - principal point (set_camera_to_training_view, testbed.cu:852), then
		// render_screen_center (testbed.cu:4376-4379, zoom 1): (0.5 - m_screen_center) + 0.5 = principal point
		for (int k = 0; k < 2; ++k) a.screen_center[k] = (0.5f - (1.0f - camera->principal_point[k])) * 1.0f + 0.5f;
		effective_camera_matrix(camera->xform, a.cam);
		NGP_CHECK(camera->lens_mode <= LENS_OPENCV_FISHEYE, "render: unsupported lens mode");
		a.lens_mode = camera->lens_mode;
		for (int k = 0; k < 4; ++k) a.lens[k] = camera->lens_params[k];
		a.near_distance = 0.0f;  // m_render_near_distance (testbed.h:914)
		for (int k = 0; k < 3; ++k) { a.aabb_min[k] = cfg->aabb_min[k]; a.aabb_max[k] = cfg->aabb_max[k]; }
		a.cone_angle_constant = cfg->cone_angle_constant;
		a.max_mip = cfg->max_cascade;
		a.bitfield = bitfield;
		a.sample_index = sample_index;
		a.snap_to_pixel_centers = cfg->snap_to_pixel_centers;
		a.linear_colors = cfg->linear_colors;
		a.rgb_activation = cfg->rgb_activation;
		a.density_activation = cfg->density_activation;
		a.min_transmittance = min_transmittance;
		for (int k = 0; k < 4; ++k) a.background[k] = background_rgba ? background_rgba[k] : 0.f;
		const uint32_t n_px = a.width * a.height;
		const size_t max_q = (size_t)std::max(n_px, 2u * 1024 * 1024) + 256;
		RenderWorkspace ws{};
		const size_t pb = render_payload_bytes();
		ws.payload[0] = r->pay0.get<char>(pb * n_px);
		ws.payload[1] = r->pay1.get<char>(pb * n_px);
		ws.payload_hit = r->payh.get<char>(pb * n_px);
		ws.rgba[0] = r->rgba0.get<float>(4 * (size_t)n_px);
		ws.rgba[1] = r->rgba1.get<float>(4 * (size_t)n_px);
		ws.rgba_hit = r->rgbah.get<float>(4 * (size_t)n_px);
		ws.coords = r->coords.get<float>(7 * max_q);
		ws.out = r->out.get<f16>(16 * max_q);
		ws.frame = r->frame.get<float>(4 * (size_t)n_px);
		ws.counters = r->counters.get<uint32_t>(2);
		if (!r->host_counters) NGP_HIP(hipHostMalloc(&r->host_counters, 16));
		ws.host_counters = r->host_counters;
		a.render_mode = r->render_mode;
		a.depth_scale = r->depth_scale;
		a.show_accel = r->show_accel;
		auto infer = [&](uint32_t n, const float* coords, f16* out) {
			check_rc(ngp_inference(model, s, n, coords, 7, out, n, NGP_LAYOUT_SOA, use_inference_params));
		};
		// Normals: tcnn input_gradient's default backprop_scale (128); it reads the inference parameters
		auto grad = [&](uint32_t n, float* coords) {
			check_rc(ngp_input_gradient(model, s, 3, n, coords, 7, coords, 7, 128.0f));
		};
		render_frame(a, spp, ws, infer, out_rgba, s, grad);
	});
}

int ngp_nerf_trainer_set_data_parallel(ngp_nerf_trainer* t, uint32_t rank, uint32_t world, ngp_allreduce_fn allreduce, void* user) {
	if (!t || world == 0 || rank >= world || (world > 1 && !allreduce)) return NGP_INVALID;
	t->drain();
	// the sample-set choice (ngp_nerf_trainer::early) depends on the exchange: the last step's passes finish first
	if (hipDeviceSynchronize() != hipSuccess) return NGP_ERROR;
	t->rank = rank;
	t->world = world;
	t->allreduce = allreduce;
	t->allreduce_user = user;
	// an RCCL hook is stream-ordered and graph-capturable; a host callback (gloo) is not
	t->dp_capturable = allreduce == ngp_dp_comm_allreduce;
	if (t->dp_capturable && user && ngp_dp_comm_reserve((ngp_dp_comm*)user, ngp_model_n_params(t->model)) != NGP_OK) return NGP_ERROR;
	// the trainer's exchange with this rank: large tables shard the optimizer (reduce-scatter, slice update,
	// all-gather of the weights; trainer option shard_opt)
	const int rc = ngp_trainer_set_data_parallel(t->trainer, allreduce ? rank : 0, allreduce ? world : 1, allreduce, user);
	if (rc != NGP_OK) return rc;
	if (t->train_graph) ngp_graph_destroy(t->train_graph);  // re-captured with (or without) the exchange
	t->train_graph = nullptr;
	return NGP_OK;
}

int ngp_nerf_trainer_buffers_read(const ngp_nerf_trainer* t, const float** grid, const uint8_t** bitfield, const float** mean) {
	if (!t) return NGP_INVALID;
	if (grid) *grid = (const float*)t->grid.p;
	if (bitfield) *bitfield = (const uint8_t*)t->bitfield.p;
	if (mean) *mean = (const float*)t->mean.p;
	return NGP_OK;
}

int ngp_nerf_trainer_buffers(ngp_nerf_trainer* t, float** grid, uint8_t** bitfield, float** mean) {
	if (!t) return NGP_INVALID;
	// the caller may write these: a prelaunched sampler (pipelining) read the bitfield before any such
	// write, so discard it and let the next step sample serially after the caller's writes
	t->drain();
	if (grid) *grid = (float*)t->grid.p;
	if (bitfield) *bitfield = (uint8_t*)t->bitfield.p;
	if (mean) *mean = (float*)t->mean.p;
	return NGP_OK;
}


// update_density_grid_nerf (testbed_nerf.cu:3412-3536), in two parts: the samples (generation and, on one GPU, the
// sort by cell bin: they read only the grid and the grid rng), then their density, splat, EMA, mean and bitfield.
// One GPU: the samples sorted by cell bin before the density evaluation, and the splat from the sorted order, which
// writes every cell. Data parallel: the order within a bin is not deterministic, so the ranks' shards of it would not
// partition the samples; there each rank evaluates its shard of the generated order and splats it by the binned
// counting sort (every cell too). A/B knob NGP_SPLAT_SORT=0: memset, generated order, atomics.
static int splat_mode() {
	static const int m = getenv("NGP_SPLAT_SORT") ? atoi(getenv("NGP_SPLAT_SORT")) : 1;
	return m;
}
static void grid_update_samples(ngp_nerf_trainer* t, hipStream_t s, uint32_t n_uniform, uint32_t n_nonuniform) {
	const ngp_nerf_config& cfg = t->cfg;
	const uint32_t n_cascades = cfg.max_cascade + 1;
	const uint32_t n_el = GRID_N_CELLS * n_cascades;
	const uint32_t n = n_uniform + n_nonuniform;
	const float* grid = (const float*)t->grid.p;
	// every rank generates the same sample set (same density rng); each evaluates its 1/N shard
	float* pos = t->gpos.get<float>((size_t)n * 3);
	uint32_t* idx = t->gidx.get<uint32_t>(n);
	uint32_t* mask = t->grid_mask.get<uint32_t>(grid_mask_words(n_cascades));
	grid_generate_samples(n_uniform, t->grid_rng.dev(), t->ema_step, cfg, grid, n_cascades, -0.01f, pos, idx, mask, s);
	t->grid_rng.advance();
	grid_generate_samples(n_nonuniform, t->grid_rng.dev(), t->ema_step, cfg, grid, n_cascades, MIN_OPTICAL_THICKNESS,
	                      pos + (size_t)n_uniform * 3, idx + n_uniform, mask, s);
	t->grid_rng.advance();
	if (splat_mode() != 0 && t->world == 1)
		grid_sort_samples(n, pos, idx, n_el, t->splat_scratch.get<uint32_t>(grid_sort_scratch_u32(n, n_el)),
		                  t->gpos_sorted.get<float>((size_t)n * 4), s);
}
static void grid_update_finish(ngp_nerf_trainer* t, hipStream_t s, float decay, uint32_t n_uniform, uint32_t n_nonuniform) {
	const ngp_nerf_config& cfg = t->cfg;
	const uint32_t n_cascades = cfg.max_cascade + 1;
	const uint32_t n_el = GRID_N_CELLS * n_cascades;
	const uint32_t n = n_uniform + n_nonuniform;
	float* grid = (float*)t->grid.p;
	float* tmp = t->grid_tmp.get<float>(n_el);
	const bool sorted = splat_mode() != 0 && t->world == 1, binned = splat_mode() != 0 && t->world > 1;
	if (splat_mode() == 0) NGP_HIP(hipMemsetAsync(tmp, 0, (size_t)n_el * 4, s));
	const uint32_t* idx = t->gidx.get<uint32_t>(n);
	const uint32_t lo = (uint32_t)((uint64_t)n * t->rank / t->world), hi = (uint32_t)((uint64_t)n * (t->rank + 1) / t->world);
	const uint32_t ns = hi - lo;
	f16* dens = t->gdens.get<f16>((size_t)std::max(ns, 1u) * 16);
	const float* dpos = sorted ? t->gpos_sorted.get<float>((size_t)n * 4) : t->gpos.get<float>((size_t)n * 3);
	const uint32_t dstride = sorted ? 4 : 3;
	if (ns) {
		// row 0 (raw density) only: the other 15 rows of the density network's output are not read
		check_rc(ngp::density_impl(t->model, s, ns, dpos + (size_t)lo * dstride, dstride, dens, ns, ngp::DENSITY_LAYOUT_ROW0, 0));
		if (splat_mode() == 0) grid_splat_max(ns, idx + lo, dens, cfg.density_activation, tmp, s);
	}
	if (sorted)
		grid_splat_sorted(n_el, t->splat_scratch.get<uint32_t>(grid_sort_scratch_u32(n, n_el)), dpos, dens, lo, hi,
		                  cfg.density_activation, tmp, s);
	if (binned)
		grid_splat_max_binned(ns, idx + lo, dens, cfg.density_activation, tmp, n_el,
		                      t->splat_scratch.get<uint32_t>(grid_splat_scratch_u32(ns, n_el)), s);
	if (t->world > 1) {
		// splatted maxima of all shards (values are >= 0: float max == max of the shards' atomicMax)
		NGP_CHECK(t->allreduce(t->allreduce_user, tmp, n_el, NGP_DTYPE_F32, NGP_REDUCE_MAX, s) == 0,
		          "data parallel: density-grid all-reduce failed");
	}
	static const bool fused = !getenv("NGP_GRID_FINAL_FUSED") || atoi(getenv("NGP_GRID_FINAL_FUSED")) != 0;  // A/B knob
	if (fused) {
		grid_ema_mean_bitfield(n_el, decay, grid, tmp, cfg.max_cascade, (float*)t->mean.p, (uint8_t*)t->bitfield.p, s);
	} else {
		grid_ema(n_el, decay, grid, tmp, s);
		grid_mean_bitfield(grid, cfg.max_cascade, (float*)t->mean.p, (uint8_t*)t->bitfield.p, s);
	}
	++t->ema_step;
}
static void update_density_grid(ngp_nerf_trainer* t, hipStream_t s, float decay, uint32_t n_uniform, uint32_t n_nonuniform) {
	if (t->training_step == 0) {
		t->ema_step = 0;
		const Dataset& ds = t->data->ds;
		const uint32_t n_el = GRID_N_CELLS * (t->cfg.max_cascade + 1);
		k_mark_untrained<<<div_round_up(n_el, 128), 128, 0, s>>>(n_el, (float*)t->grid.p, ds.n_images, ds.d_cams, raw_xforms(ds), true);
		NGP_HIP(hipGetLastError());
	}
	grid_update_samples(t, s, n_uniform, n_nonuniform);
	grid_update_finish(t, s, decay, n_uniform, n_nonuniform);
}
// the update's sample counts at a step (training_prep_nerf, testbed_nerf.cu:3622-3630)
static void grid_update_counts(const ngp_nerf_trainer* t, uint32_t step, uint32_t* nu, uint32_t* nn) {
	const uint32_t nc = t->cfg.max_cascade + 1;
	*nu = step < 256 ? GRID_N_CELLS * nc : GRID_N_CELLS / 4 * nc;
	*nn = step < 256 ? 0u : GRID_N_CELLS / 4 * nc;
}

// Data parallel: this shard's counters and loss as five floats for one all-reduce (sum). The u32
// counters travel as 16-bit halves so their sums stay exact in fp32 for up to 256 ranks; the per-ray
// losses are normalised by the shard's ray count (compute_loss), rescaled here to 1 / R_global.
__global__ void k_dp_pack(const uint32_t* __restrict__ ctr, const float* __restrict__ loss, uint32_t n_loss, float loss_rescale,
                          float* __restrict__ out) {
	__shared__ float part[16];
	float sum = 0.f;
	for (uint32_t i = threadIdx.x; i < n_loss; i += blockDim.x) sum += loss[i];
	for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
	__syncthreads();
	if (threadIdx.x == 0) {
		float t = 0.f;
		for (uint32_t w = 0; w < blockDim.x / 64; ++w) t += part[w];
		out[0] = (float)(ctr[1] >> 16); out[1] = (float)(ctr[1] & 0xffffu);
		out[2] = (float)(ctr[2] >> 16); out[3] = (float)(ctr[2] & 0xffffu);
		out[4] = t * loss_rescale;
	}
}
// the all-reduced counters -> host-coherent memory (host[1] steps, host[2] compacted, host[5] loss bits;
// host[6] this shard's own step count, which sizes its next inference)
__global__ void k_dp_publish(const float* __restrict__ red, const uint32_t* __restrict__ ctr, volatile uint32_t* host, uint32_t seq) {
	if (threadIdx.x == 0) {
		host[6] = ctr[1];
		host[1] = ((uint32_t)red[0] << 16) + (uint32_t)red[1];
		host[2] = ((uint32_t)red[2] << 16) + (uint32_t)red[3];
		host[5] = __float_as_uint(red[4]);
		__threadfence_system();
		host[4] = seq;
	}
}

// Wait until the step's counters are published (k_rollover_pair_publish, or k_dp_publish; or the stream failed /
// stalled for a minute).
static void wait_published(volatile uint32_t* host, uint32_t seq, hipStream_t s) {
	const auto t0 = std::chrono::steady_clock::now();
	for (uint64_t spin = 0;; ++spin) {
		if (__atomic_load_n(&host[4], __ATOMIC_ACQUIRE) == seq) return;
		if ((spin & 1023) == 1023) {
			const hipError_t q = hipStreamQuery(s);
			if (q != hipSuccess && q != hipErrorNotReady) NGP_HIP(q);
			if (q == hipSuccess) {  // the stream drained: the publishing kernel ran, so its write is visible
				if (__atomic_load_n(&host[4], __ATOMIC_ACQUIRE) == seq) return;
				const hipError_t e = hipGetLastError();
				throw Error(std::string("nerf train step: stream idle but counters not published (") + hipGetErrorString(e) + ")");
			}
			NGP_CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60), "nerf train step: counters not published");
		}
		__builtin_ia32_pause();
	}
}

// Sizes and buffers of one step's sampling (train_nerf_step, testbed_nerf.cu:3867-3953), from the
// trainer's current rays-per-batch and measured counts.
struct SamplePlan {
	uint32_t R, Rl, r_lo, Bl, max_samples, max_inference, Ra;
	uint32_t* ray_indices;
	float* rays;
	uint32_t* numsteps;
	float* coords;
	uint32_t* ctr;
};
static SamplePlan sample_plan(ngp_nerf_trainer* t) {
	SamplePlan p;
	const uint32_t B = t->cfg.target_batch_size, W = t->world, rk = t->rank;
	p.R = t->rays_per_batch;
	p.r_lo = (uint32_t)((uint64_t)p.R * rk / W);
	p.Rl = (uint32_t)((uint64_t)p.R * (rk + 1) / W) - p.r_lo;
	p.Bl = (uint32_t)((uint64_t)B * (rk + 1) / W - (uint64_t)B * rk / W);
	p.max_samples = p.Bl * 16;
	if (t->measured_before_compaction_local == 0) p.max_inference = p.max_samples;
	else p.max_inference = next_multiple(std::min(t->measured_before_compaction_local, p.max_samples), 256);
	p.Ra = std::max(p.Rl, 1u);
	const bool b = t->early() && (t->training_step & 1u);  // the step's sample set (ngp_nerf_trainer::early)
	p.ray_indices = (b ? t->ray_indices_b : t->ray_indices).get<uint32_t>(p.Ra);
	p.rays = (b ? t->rays_b : t->rays).get<float>((size_t)p.Ra * 6);
	p.numsteps = (b ? t->numsteps_b : t->numsteps).get<uint32_t>((size_t)p.Ra * 2);
	p.coords = (b ? t->coords_b : t->coords).get<float>((size_t)p.max_samples * 7);
	p.ctr = (b ? t->counters_b : t->counters).get<uint32_t>(4);  // rays kept, steps, compacted steps
	return p;
}
static void launch_sampler(ngp_nerf_trainer* t, const SamplePlan& p, hipStream_t s) {
	ProfScope ps("nerf_sample", s);
	const ngp_rng rng{t->rng.state, t->rng.inc};
	check_rc(ngp_nerf_generate_training_samples(t->data, &t->cfg, s, p.Rl, p.r_lo, p.R, rng, p.max_inference,
	                                            (const uint8_t*)t->bitfield.p, p.ray_indices, p.rays, p.numsteps, p.coords, p.ctr));
}
static bool density_grid_update_due(uint32_t step) {
	const uint32_t skip = std::min(std::max(step / 16u, 1u), 16u);
	return step % skip == 0;
}

// Testbed::train_nerf's error map window (testbed_nerf.cu:3659-3666): at its first step the map is
// resized to min(3.5 (n_steps_between * rays_per_batch / n_images)^(1/4), image 0's size) per image and
// zeroed (uint32 arithmetic as in the reference). Returns the map the step's loss pass deposits into.
static float* error_map_window(ngp_nerf_trainer* t, hipStream_t s) {
	const Dataset& ds = t->data->ds;
	if (ds.n_images == 0 || ds.cams.empty()) return nullptr;
	if (t->em_steps_since == 0) {
		const uint32_t n_samples_per_image = (t->em_steps_between * t->rays_per_batch) / ds.n_images;
		const int k = (int)(std::sqrt(std::sqrt((float)n_samples_per_image)) * 3.5f);
		t->em_w = (uint32_t)std::min(k, (int)ds.cams[0].width);
		t->em_h = (uint32_t)std::min(k, (int)ds.cams[0].height);
		const size_t n = (size_t)t->em_w * t->em_h * ds.n_images;
		NGP_HIP(hipMemsetAsync(t->em_data.get<float>(std::max<size_t>(n, 1)), 0, n * sizeof(float), s));
	}
	return t->em_w >= 2 && t->em_h >= 2 ? (float*)t->em_data.p : nullptr;
}

// After the step (testbed_nerf.cu:3700-3748): when the window is full, the CDFs of the map
// (construct_cdf_2d/1d on the stream; with data parallelism the ranks' maps are summed first), the
// host pass over the per-image totals, then a 1.5x longer window.
static void error_map_step_done(ngp_nerf_trainer* t, hipStream_t s) {
	const Dataset& ds = t->data->ds;
	if (ds.n_images == 0 || ds.cams.empty()) return;
	t->em_steps_since += 1;
	if (t->em_steps_since < t->em_steps_between) return;
	t->em_cdf_w = t->em_w;
	t->em_cdf_h = t->em_h;
	const uint32_t n_img = ds.n_images, w = t->em_cdf_w, h = t->em_cdf_h;
	float* data = (float*)t->em_data.p;
	if (t->dp() && data && w && h)
		NGP_CHECK(t->allreduce(t->allreduce_user, data, (uint64_t)w * h * n_img, NGP_DTYPE_F32, NGP_REDUCE_SUM, s) == 0,
		          "data parallel: error map all-reduce failed");
	float* cdf_x = t->em_cdf_x.get<float>(std::max<size_t>((size_t)w * h * n_img, 1));
	float* cdf_y = t->em_cdf_y.get<float>(std::max<size_t>((size_t)h * n_img, 1));
	float* cdf_img = t->em_cdf_img.get<float>(n_img);
	error_map_cdfs(n_img, w, h, data, cdf_x, cdf_y, cdf_img, s);
	// the image CDF on the host (single-threaded in the reference too)
	std::vector<float> pmf(n_img), cdf(n_img);
	NGP_HIP(hipMemcpyAsync(pmf.data(), cdf_img, n_img * sizeof(float), hipMemcpyDeviceToHost, s));
	NGP_HIP(hipStreamSynchronize(s));
	float cum = 0.f;
	for (uint32_t i = 0; i < n_img; ++i) cdf[i] = cum += pmf[i];
	const float norm = 1.0f / cum;
	constexpr float MIN_PMF = 0.1f;
	for (uint32_t i = 0; i < n_img; ++i) {
		pmf[i] = (1.0f - MIN_PMF) * pmf[i] * norm + MIN_PMF / (float)n_img;
		cdf[i] = (1.0f - MIN_PMF) * cdf[i] * norm + MIN_PMF * (float)(i + 1) / (float)n_img;
	}
	NGP_HIP(hipMemcpyAsync(cdf_img, cdf.data(), n_img * sizeof(float), hipMemcpyHostToDevice, s));
	NGP_HIP(hipStreamSynchronize(s));
	t->em_pmf_img = std::move(pmf);
	t->em_steps_since = 0;
	t->em_cdf_valid = true;
	t->em_steps_between = (uint32_t)(t->em_steps_between * 1.5f);
}

int ngp_nerf_trainer_error_map(ngp_nerf_trainer* t, int which, float* out, uint64_t cap, ngp_nerf_error_map_info* info) {
	if (!t || which < 0 || which > 4) return NGP_INVALID;
	NERF_TRY({
		const uint32_t n_img = t->data->ds.n_images;
		const uint64_t sizes[5] = {(uint64_t)t->em_w * t->em_h * n_img, (uint64_t)t->em_cdf_w * t->em_cdf_h * n_img,
		                           (uint64_t)t->em_cdf_h * n_img, t->em_cdf_valid ? n_img : 0u, t->em_pmf_img.size()};
		const void* src[5] = {t->em_data.p, t->em_cdf_x.p, t->em_cdf_y.p, t->em_cdf_img.p, t->em_pmf_img.data()};
		if (info) {
			info->width = t->em_w; info->height = t->em_h;
			info->cdf_width = t->em_cdf_w; info->cdf_height = t->em_cdf_h;
			info->n_images = n_img;
			info->cdf_valid = t->em_cdf_valid ? 1u : 0u;
			info->n_steps_since_update = t->em_steps_since;
			info->n_steps_between_updates = t->em_steps_between;
			info->size = sizes[which];
		}
		const uint64_t n = std::min(cap, sizes[which]);
		if (out && n) {
			if (which == 4) {
				memcpy(out, src[4], n * sizeof(float));
			} else {
				NGP_HIP(hipDeviceSynchronize());
				NGP_HIP(hipMemcpy(out, src[which], n * sizeof(float), hipMemcpyDeviceToHost));
			}
		}
	});
}

int ngp_nerf_trainer_set_pipeline(ngp_nerf_trainer* t, int enable) {
	if (!t) return NGP_INVALID;
	NERF_TRY({
		t->drain();
		t->pipeline = enable != 0;
	});
}

// The pipelined sampler's stream. Experiment knobs (A/B): NGP_SAMPLER_PRIO / NGP_MAIN_PRIO -1 low,
// 1 high (HSA queue priority: which queue's workgroups the dispatcher places first); NGP_SAMPLER_CU_KEEP k in 1..7:
// the sampler's queue may use k of every 8 CUs (CU mask), so the training pass's one-block-per-CU MLP kernel
// finds whole CUs free on the rest.
static int env_prio(const char* name) {
	const char* v = getenv(name);
	if (!v || !*v) return 0;
	const int p = atoi(v);
	int least = 0, greatest = 0;
	NGP_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
	return p < 0 ? least : (p > 0 ? greatest : 0);  // lower number = higher priority
}
static hipStream_t make_sampler_stream() {
	hipStream_t s = nullptr;
	const char* keep = getenv("NGP_SAMPLER_CU_KEEP");
	const int k = keep ? atoi(keep) : 0;
	if (k > 0 && k < 8) {
		int dev = 0, n_cu = 0;
		NGP_HIP(hipGetDevice(&dev));
		NGP_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
		std::vector<uint32_t> mask((n_cu + 31) / 32, 0u);
		for (int c = 0; c < n_cu; ++c)
			if (c % 8 < k) mask[c / 32] |= 1u << (c % 32);
		NGP_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
		return s;
	}
	const int prio = env_prio("NGP_SAMPLER_PRIO");
	if (prio) NGP_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
	else NGP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
	return s;
}

// 1: the sampler -> inference handoff by value (default); 2: the buffer release too; 0: events only (A/B)
static int nerf_waitval() {
	static const int v = getenv("NGP_NERF_WAITVAL") ? atoi(getenv("NGP_NERF_WAITVAL")) : 1;
	return v;
}

int ngp_nerf_train_step(ngp_nerf_trainer* t, void* stream, int get_loss, ngp_nerf_stats* st) {
	if (!t) return NGP_INVALID;
	NERF_TRY({
		hipStream_t s = S(stream);
		if (!s) {  // a private blocking stream (ordered after the null stream's earlier work)
			if (!t->own_stream) {
				const int prio = env_prio("NGP_MAIN_PRIO");
				if (prio) NGP_HIP(hipStreamCreateWithPriority(&t->own_stream, hipStreamDefault, prio));
				else NGP_HIP(hipStreamCreate(&t->own_stream));
			}
			s = t->own_stream;
		}
		const ngp_nerf_config& cfg = t->cfg;
		const uint32_t B = cfg.target_batch_size;
		const bool pre = t->prelaunched;
		t->prelaunched = false;
		// training_prep_nerf (a prelaunched sampler implies no update was due at this step)
		if (!pre && density_grid_update_due(t->training_step)) {
			ProfScope ps("nerf_density_grid", s);
			uint32_t nu, nn;
			grid_update_counts(t, t->training_step, &nu, &nn);
			if (t->grid_pregen) {  // the samples were generated (and sorted) under the last step's training pass
				NGP_CHECK(nu == t->pregen_nu && nn == t->pregen_nn, "nerf: pregenerated density-grid samples are stale");
				t->grid_pregen = false;
				NGP_HIP(hipStreamWaitEvent(s, t->ev_gen, 0));
				grid_update_finish(t, s, 0.95f, nu, nn);
			} else {
				update_density_grid(t, s, 0.95f, nu, nn);
			}
		}
		// train_nerf_step (testbed_nerf.cu:3867-4132)
		const SamplePlan sp = sample_plan(t);
		const uint32_t R = sp.R, Rl = sp.Rl, Bl = sp.Bl, max_inference = sp.max_inference, Ra = sp.Ra;
		if (t->training_step == 0) t->n_rays_total = 0;
		t->n_rays_total += R;
		uint32_t* ray_indices = sp.ray_indices;
		float* rays = sp.rays;
		uint32_t* numsteps = sp.numsteps;
		float* coords = sp.coords;
		uint32_t* ctr = sp.ctr;
		f16* mlp_out = t->mlp_out.get<f16>((size_t)std::max(Bl, sp.max_samples) * 16);
		f16* dloss = t->dloss.get<f16>((size_t)Bl * 16);
		float* coords_c = t->coords_c.get<float>((size_t)Bl * 7);
		float* loss = t->loss.get<float>(Ra);
		ngp_rng rng{t->rng.state, t->rng.inc};
		// global ray ids (rng.advance(i * 16), image_idx(i, R)) so the shards draw the 1-GPU rays;
		// dL/doutput is scaled by 128 / R (global), so the summed gradient is the 1-GPU gradient
		if (pre) {
			NGP_CHECK(sp.R == t->pre_R && sp.max_inference == t->pre_max_inference, "nerf: prelaunched sampler is stale");
			if (nerf_waitval()) NGP_HIP(hipStreamWaitValue32(s, t->sig_samp, t->seq_samp, hipStreamWaitValueGte, 0xFFFFFFFFu));
			else NGP_HIP(hipStreamWaitEvent(s, t->ev_samp, 0));
		} else {
			launch_sampler(t, sp, s);
		}
		{
		ProfScope ps("nerf_inference", s);
		// only the 4 live outputs (raw rgb, raw density): compute_loss reads nothing else
		check_rc(ngp_inference(t->model, s, max_inference, coords, 7, mlp_out, 4, NGP_LAYOUT_AOS_RGBD, 0));
		}
		const bool dp = t->dp();
		const float loss_scale_local = 128.0f * (float)Rl / (float)R;
		float* error_map = error_map_window(t, s);
		if (!t->host_ctr) {
			void* p = nullptr;
			NGP_HIP(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
			t->host_ctr = (volatile uint32_t*)p;
			memset(p, 0, 64);
		}
		const bool early_pub = t->early() && Rl > 0;
		const uint32_t pub_seq = dp ? 0u : ++t->publish_seq;
		{
		ProfScope ps("nerf_loss", s);
		// pass 1 keeps each composited sample's state for pass 2 (indexed like the sampler's samples, at most max_samples)
		static const bool keep_state = !getenv("NGP_LOSS_STATE") || atoi(getenv("NGP_LOSS_STATE")) != 0;  // A/B knob
		float* lstate = keep_state ? t->loss_state.get<float>((size_t)5 * sp.max_samples) : nullptr;
		check_rc(nerf_compute_loss(t->data, &cfg, s, Rl, R, rng, Bl, ctr, mlp_out, 4, ray_indices, rays, numsteps, coords, coords_c,
		                               dloss, loss, ctr + 2, (const float*)t->mean.p, dp ? loss_scale_local : 128.0f, true,
		                               error_map, t->em_w, t->em_h, lstate, sp.max_samples, early_pub ? t->host_ctr : nullptr,
		                               pub_seq));
		}
		// the step's counters are final here (the training pass does not touch them): publish them before
		// the training pass so the host can size the next step while it runs (early_pub: already published)
		if (!dp) {
			// single GPU: the rollover launch (fill_rollover_and_rescale + fill_rollover) also publishes the counters
			// and writes the optimizer control block the training graph reads (a separate publish kernel and
			// ngp_graph_launch's k_set_ctl before: two launches less per step)
			StepPublish pub{};
			pub.ctr = ctr;
			pub.host = early_pub ? nullptr : t->host_ctr;
			pub.seq = pub_seq;
			trainer_ctl_values(t->trainer, &pub.ctl, &pub.step, &pub.cfg_off, &pub.cfg_words, pub.cfg);
			fill_rollover_pair_publish(Bl, ctr + 2, dloss, 16, coords_c, 7, pub, s);
		} else {
			fill_rollover_pair(Bl, ctr + 2, dloss, 16, coords_c, 7, s);  // fill_rollover_and_rescale + fill_rollover
		}
		if (dp) {
			// NerfCounters::update_after_training on the global batch: this shard's counters and loss
			// all-reduced on the stream, then published like the single-GPU counters (no copies, no sync)
			ProfScope ps("nerf_dp_counters", s);
			float* d = t->dp_scalars.get<float>(8);
			k_dp_pack<<<1, 1024, 0, s>>>(ctr, loss, get_loss ? Rl : 0u, (float)Rl / (float)R, d);
			NGP_HIP(hipGetLastError());
			NGP_CHECK(t->allreduce(t->allreduce_user, d, 5, NGP_DTYPE_F32, NGP_REDUCE_SUM, s) == 0,
			          "data parallel: counter all-reduce failed");
			k_dp_publish<<<1, 64, 0, s>>>(d, ctr, t->host_ctr, ++t->publish_seq);
		}
		NGP_HIP(hipGetLastError());
		// the next step's sampler may run under this step's training pass when the exchange is
		// stream-ordered (single GPU, or the engine's RCCL communicator)
		const bool can_pipeline = t->pipeline && (!dp || t->dp_capturable);
		if (can_pipeline) {
			if (!t->sample_stream) {
				t->sample_stream = make_sampler_stream();
				NGP_HIP(hipEventCreateWithFlags(&t->ev_free, hipEventDisableTiming));
				NGP_HIP(hipEventCreateWithFlags(&t->ev_samp, hipEventDisableTiming));
			}
			// sample buffers and counters released: an event (by the time the host launches the next sampler this
			// is long done, and a completed event's wait costs ~1.3 us against ~3.6 for a value wait)
			if (t->early()) {
				// nothing to release: the next sampler writes the other sample set
			} else if (nerf_waitval() == 2) {
				t->ensure_signals();
				NGP_HIP(hipStreamWriteValue32(s, t->sig_free, ++t->seq_free, 0));
			} else {
				NGP_HIP(hipEventRecord(t->ev_free, s));
			}
		}
		{
		ProfScope ps("nerf_train_pass", s);
		if (!dp || t->dp_capturable) {
			// one HIP graph per step: forward_backward [+ the gradient all-reduce, RCCL] + optimizer. Re-record
			// when the graph's buffers moved: the sample buffers, or any model workspace (a density-grid
			// update through ngp_density can grow the encoding workspace after a snapshot load)
			if (!t->train_graph || t->graph_in != coords_c || t->graph_dl != dloss || t->graph_n != Bl ||
			    t->graph_epoch != ngp_model_workspace_epoch(t->model)) {
				if (t->train_graph) ngp_graph_destroy(t->train_graph);
				t->train_graph = nullptr;
				// data parallel: the shards' dL/doutput is scaled by 128 / R_global, so the summed gradient is the
				// 1-GPU gradient: world factor 1 in the optimizer
				check_rc(capture_training_step_with(t->trainer, s, Bl, coords_c, 7, dloss, 16, 128.0f, 1, 1, t->exchange(),
				                                    &t->train_graph));
				t->graph_in = coords_c;
				t->graph_dl = dloss;
				t->graph_n = Bl;
				t->graph_epoch = ngp_model_workspace_epoch(t->model);
			}
			if (dp) check_rc(ngp_graph_launch(t->train_graph, s));
			else graph_launch_ctl_written(t->train_graph, s);  // the control block was written by the rollover launch
		} else {
			// host-callback exchange (gloo): not capturable; the same step body, launched eagerly
			check_rc(train_step_with(t->trainer, s, Bl, coords_c, 7, dloss, 16, 128.0f, t->exchange()));
		}
		t->rng.advance();  // m_rng.advance() (testbed_nerf.cu:4127)
		}
		++t->training_step;
		// NerfCounters::update_after_training (testbed_nerf.cu:3583-3609): host sync
		uint32_t h[4];
		double loss_sum = 0;
		if (get_loss && Rl && !dp) {
			std::vector<float> hl(Rl);
			NGP_HIP(hipMemcpyAsync(hl.data(), loss, (size_t)Rl * 4, hipMemcpyDeviceToHost, s));
			NGP_HIP(hipStreamSynchronize(s));
			for (float v : hl) loss_sum += v;
		} else {
			wait_published(t->host_ctr, t->publish_seq, s);
		}
		for (int k = 0; k < 4; ++k) h[k] = t->host_ctr[k];
		if (dp) {
			const uint32_t lb = t->host_ctr[5];
			float lv;
			memcpy(&lv, &lb, 4);
			loss_sum = lv;
			t->measured_before_compaction_local = t->host_ctr[6];
		} else {
			t->measured_before_compaction_local = h[1];
		}
		float loss_scalar = 0.f;
		t->measured_batch_size = 0;
		t->measured_before_compaction = 0;
		if (h[1] != 0 && h[2] != 0) {
			t->measured_before_compaction = h[1];
			t->measured_batch_size = h[2];
			if (get_loss) t->loss_scalar = loss_scalar = (float)(loss_sum * (double)t->measured_batch_size / (double)B);
			uint32_t r = (uint32_t)((float)t->rays_per_batch * (float)B / (float)t->measured_batch_size);
			t->rays_per_batch = std::min(next_multiple(r, 256), 1u << 18);
		}
		error_map_step_done(t, s);
		// next step's sampler, concurrent with this step's training pass (no density-grid update due first)
		if (can_pipeline && t->measured_batch_size > 0 && !density_grid_update_due(t->training_step)) {
			const SamplePlan np = sample_plan(t);
			// early(): the sampler writes the other sample set, which the step before last read (complete: this step's
			// counters are published), so it waits on nothing
			if (!t->early()) {
				if (nerf_waitval() == 2) NGP_HIP(hipStreamWaitValue32(t->sample_stream, t->sig_free, t->seq_free, hipStreamWaitValueGte, 0xFFFFFFFFu));
				else NGP_HIP(hipStreamWaitEvent(t->sample_stream, t->ev_free, 0));
			}
			launch_sampler(t, np, t->sample_stream);
			if (nerf_waitval()) {
				t->ensure_signals();
				NGP_HIP(hipStreamWriteValue32(t->sample_stream, t->sig_samp, ++t->seq_samp, 0));
			} else {
				NGP_HIP(hipEventRecord(t->ev_samp, t->sample_stream));
			}
			t->pre_R = np.R;
			t->pre_max_inference = np.max_inference;
			t->prelaunched = true;
		}
		// next step's density-grid update: its samples now, under this step's training pass (one GPU)
		static const bool pregen_on = !getenv("NGP_GRID_PREGEN") || atoi(getenv("NGP_GRID_PREGEN")) != 0;  // A/B knob
		if (pregen_on && can_pipeline && !dp && t->training_step > 0 && density_grid_update_due(t->training_step)) {
			if (!t->ev_gen) NGP_HIP(hipEventCreateWithFlags(&t->ev_gen, hipEventDisableTiming));
			grid_update_counts(t, t->training_step, &t->pregen_nu, &t->pregen_nn);
			t->pregen_rng = t->grid_rng;
			grid_update_samples(t, t->sample_stream, t->pregen_nu, t->pregen_nn);
			NGP_HIP(hipEventRecord(t->ev_gen, t->sample_stream));
			t->grid_pregen = true;
		}
		if (st) {
			st->step = t->training_step;
			st->rays_per_batch = t->rays_per_batch;
			st->measured_batch_size = t->measured_batch_size;
			st->measured_batch_size_before_compaction = t->measured_before_compaction;
			st->loss = loss_scalar;
		}
		NGP_CHECK(t->measured_batch_size > 0, "Nerf training generated 0 samples (testbed_nerf.cu:3693-3697)");
	});
}


// ---- snapshots (.ingp) ---------------------------------------------------------------------------
// Testbed::save_snapshot / load_snapshot (src/testbed.cu:4873-5057) for a NeRF testbed: msgpack of the
// network config with a "snapshot" member; .ingp files are gzip streams (zstr), others raw msgpack.
// tcnn Trainer::serialize writes n_params / params_type / params_binary (fp16 params); the optimizer
// member (include_optimizer_state) is this engine's own layout (tcnn absent: parity unpinned).
}  // extern "C"

namespace {
using ngp::mp::Value;

constexpr uint32_t SNAPSHOT_FORMAT_VERSION = 1;  // testbed.cu:80

bool ends_with_ci(const std::string& s, const std::string& suf) {
	return s.size() >= suf.size() && ngp::iequals(s.substr(s.size() - suf.size()), suf);
}

std::string gzip_bytes(const std::string& in, int level) {
	z_stream z{};
	NGP_CHECK(deflateInit2(&z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) == Z_OK, "snapshot: deflateInit2 failed");
	std::string out(deflateBound(&z, in.size()) + 64, '\0');
	z.next_in = (Bytef*)in.data();
	z.avail_in = (uInt)in.size();
	z.next_out = (Bytef*)out.data();
	z.avail_out = (uInt)out.size();
	const int rc = deflate(&z, Z_FINISH);
	const size_t n = out.size() - z.avail_out;
	deflateEnd(&z);
	NGP_CHECK(rc == Z_STREAM_END, "snapshot: deflate failed");
	out.resize(n);
	return out;
}

std::string maybe_inflate(const std::string& in) {
	const bool gz = in.size() >= 2 && (uint8_t)in[0] == 0x1f && (uint8_t)in[1] == 0x8b;
	const bool zl = in.size() >= 2 && ((uint8_t)in[0] & 0x0f) == 8 && (((uint8_t)in[0] << 8) | (uint8_t)in[1]) % 31 == 0;
	if (!gz && !zl) return in;  // raw msgpack
	z_stream z{};
	NGP_CHECK(inflateInit2(&z, 15 + 32) == Z_OK, "snapshot: inflateInit2 failed");
	z.next_in = (Bytef*)in.data();
	z.avail_in = (uInt)in.size();
	std::string out;
	char buf[1 << 16];
	int rc;
	do {
		z.next_out = (Bytef*)buf;
		z.avail_out = sizeof buf;
		rc = inflate(&z, Z_NO_FLUSH);
		NGP_CHECK(rc == Z_OK || rc == Z_STREAM_END, "snapshot: corrupt compressed stream");
		out.append(buf, sizeof buf - z.avail_out);
	} while (rc != Z_STREAM_END);
	inflateEnd(&z);
	return out;
}

std::string read_file(const char* path) {
	std::ifstream f(path, std::ios::binary);
	NGP_CHECK(f.good(), std::string("snapshot: cannot open '") + path + "'");
	std::stringstream ss;
	ss << f.rdbuf();
	return ss.str();
}

Value load_network_config(const char* path) {  // Testbed::load_network_config (testbed.cu:246): msgpack branch
	return ngp::mp::decode(maybe_inflate(read_file(path)));
}

Value vec3(const float* v) {
	Value a = Value::array();
	for (int k = 0; k < 3; ++k) a.arr.push_back(Value::real(v[k]));
	return a;
}

template <typename T> std::vector<T> device_to_host(const void* d, size_t n) {
	std::vector<T> h(n);
	if (n) NGP_HIP(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
	return h;
}

void check_ok(int rc) {
	if (rc != NGP_OK) throw ngp::Error(ngp_last_error());
}

const char* const OPT_NAMES[5] = {"full_precision_params_binary", "first_moments_binary", "second_moments_binary",
                                  "ema_params_binary", "param_steps_binary"};

// tcnn Trainer::serialize(include_optimizer_state) (testbed.cu:4874): n_params, params_type, params_binary (the fp16
// parameters) and, with the optimizer state, an "optimizer" member: the Adam moments and per-parameter steps, the
// EMA weights and the fp32 master weights under tcnn-style names (tcnn absent: the member names are a restatement,
// parity unpinned)
void trainer_to_snapshot(ngp_trainer* tr, uint64_t n, bool include_optimizer_state, Value& snap) {
	snap["n_params"] = Value::uint(n);
	snap["params_type"] = Value::str("__half");
	{
		auto p = device_to_host<uint16_t>(ngp_trainer_params(tr), n);
		snap["params_binary"] = Value::bin(p.data(), p.size() * 2);
	}
	if (!include_optimizer_state) return;
	uint64_t bytes = 0;
	check_ok(ngp_trainer_serialize(tr, nullptr, &bytes));
	std::string blob(bytes, '\0');
	check_ok(ngp_trainer_serialize(tr, blob.data(), &bytes));
	uint64_t hdr[4];
	memcpy(hdr, blob.data(), 32);
	Value opt = Value::object();
	opt["otype"] = Value::str("Ema(ExponentialDecay(Adam))");
	opt["current_step"] = Value::uint(hdr[3]);
	for (int k = 0; k < 5; ++k) opt[OPT_NAMES[k]] = Value::bin(blob.data() + 32 + (size_t)k * n * 4, (size_t)n * 4);
	snap["optimizer"] = opt;
}

// tcnn Trainer::deserialize (testbed.cu:5040): the parameters, then the optimizer state when the snapshot has one.
// An optimizer member without some of this engine's arrays (one written by another implementation of the chain)
// fills them from what is there: fp32 master weights and EMA from the parameters, moments and steps from 0.
void trainer_from_snapshot(ngp_trainer* tr, uint64_t n, const Value& snap) {
	NGP_CHECK((uint64_t)snap.at("n_params").number() == n, "snapshot: parameter count differs from this network");
	const Value& pb = snap.at("params_binary");
	const std::string type = snap.find("params_type") ? snap.at("params_type").s : std::string("__half");
	std::vector<float> w(n);
	if (type == "float") {
		NGP_CHECK(pb.s.size() == n * 4, "snapshot: params_binary size");
		memcpy(w.data(), pb.s.data(), n * 4);
	} else {
		NGP_CHECK(type == "__half" && pb.s.size() == n * 2, "snapshot: params_binary size/type");
		const ngp::f16* h = (const ngp::f16*)pb.s.data();
		for (uint64_t k = 0; k < n; ++k) w[k] = (float)h[k];
	}
	check_ok(ngp_trainer_set_params_full_precision(tr, w.data(), n));
	const Value* opt = snap.find("optimizer");
	if (!opt) return;
	std::string blob(32 + (size_t)n * 20, '\0');
	const uint64_t hdr[4] = {0x4e47504d49333535ULL, 1, n, (uint64_t)opt->number_or("current_step", 0.0)};
	memcpy(blob.data(), hdr, 32);
	for (int k = 0; k < 5; ++k) {
		char* dst = blob.data() + 32 + (size_t)k * n * 4;
		if (const Value* b = opt->find(OPT_NAMES[k])) {
			NGP_CHECK(b->s.size() == n * 4, std::string("snapshot: optimizer ") + OPT_NAMES[k] + " size");
			memcpy(dst, b->s.data(), n * 4);
		} else if (k == 0 || k == 3) {
			memcpy(dst, w.data(), n * 4);  // master weights / EMA: the parameters
		}  // moments, steps: 0
	}
	check_ok(ngp_trainer_deserialize(tr, blob.data(), blob.size()));
}

void write_snapshot(const char* path, Value& root, Value& snap, int compress) {
	root["snapshot"] = snap;
	std::string bytes;
	ngp::mp::encode(root, bytes);
	if (ends_with_ci(path, ".ingp")) bytes = gzip_bytes(bytes, compress ? Z_DEFAULT_COMPRESSION : Z_NO_COMPRESSION);
	std::ofstream f(path, std::ios::binary);
	NGP_CHECK(f.good(), std::string("snapshot: cannot write '") + path + "'");
	f.write(bytes.data(), (std::streamsize)bytes.size());
	NGP_CHECK(f.good(), "snapshot: write failed");
}

Value snapshot_root(const char* network_config_json) {
	Value root = network_config_json && *network_config_json ? ngp::mp::from_json(ngp::Json::parse(network_config_json))
	                                                          : Value::object();
	root.erase("snapshot");
	return root;
}
}  // namespace

extern "C" {

int ngp_nerf_save_snapshot(ngp_nerf_trainer* t, void* stream, const char* path, const char* network_config_json,
                           int include_optimizer_state, int compress) {
	if (!t || !path) return NGP_INVALID;
	NERF_TRY({
		NGP_HIP(hipStreamSynchronize(S(stream)));
		Value root = snapshot_root(network_config_json);
		Value snap = Value::object();
		trainer_to_snapshot(t->trainer, ngp_model_n_params(t->model), include_optimizer_state != 0, snap);
		snap["version"] = Value::uint(SNAPSHOT_FORMAT_VERSION);
		snap["mode"] = Value::str("nerf");
		snap["density_grid_size"] = Value::uint(GRIDSIZE);
		{
			const uint32_t n_el = GRID_N_CELLS * (t->cfg.max_cascade + 1);
			auto g = device_to_host<float>(t->grid.p, n_el);
			std::vector<f16> h(n_el);
			for (uint32_t k = 0; k < n_el; ++k) h[k] = (f16)g[k];  // (__half)density_grid[i]
			snap["density_grid_binary"] = Value::bin(h.data(), h.size() * 2);
		}
		Value& nerf = snap["nerf"];
		nerf["aabb_scale"] = Value::real(t->cfg.aabb_max[0] - t->cfg.aabb_min[0]);
		nerf["rgb"]["rays_per_batch"] = Value::uint(t->rays_per_batch);
		nerf["rgb"]["measured_batch_size"] = Value::uint(t->measured_batch_size);
		nerf["rgb"]["measured_batch_size_before_compaction"] = Value::uint(t->measured_before_compaction);
		snap["training_step"] = Value::uint(t->training_step);
		snap["loss"] = Value::real(t->loss_scalar);
		snap["aabb"]["min"] = vec3(t->cfg.aabb_min);
		snap["aabb"]["max"] = vec3(t->cfg.aabb_max);
		snap["density_grid_ema_step"] = Value::uint(t->ema_step);
		write_snapshot(path, root, snap, compress);
	});
}

int ngp_nerf_load_snapshot(ngp_nerf_trainer* t, void* stream, const char* path) {
	if (!t || !path) return NGP_INVALID;
	NERF_TRY({
		t->drain();
		hipStream_t s = S(stream);
		NGP_HIP(hipStreamSynchronize(s));
		const Value root = load_network_config(path);
		NGP_CHECK(root.find("snapshot"), std::string("File '") + path + "' does not contain a snapshot.");
		const Value& snap = root.at("snapshot");
		NGP_CHECK(snap.number_or("version", 0) >= SNAPSHOT_FORMAT_VERSION, "Snapshot uses an old format and can not be loaded.");
		if (const Value* m = snap.find("mode")) NGP_CHECK(m->type == Value::Str && m->s == "nerf", "snapshot: not a NeRF snapshot");
		NGP_CHECK((uint32_t)snap.at("density_grid_size").number() == GRIDSIZE, "Incompatible grid size.");
		trainer_from_snapshot(t->trainer, ngp_model_n_params(t->model), snap);  // tcnn Trainer::deserialize
		// density grid (fp16 in the file)
		const Value& gb = snap.at("density_grid_binary");
		const uint32_t n_el = GRID_N_CELLS * (t->cfg.max_cascade + 1);
		const size_t n_file = gb.s.size() / 2;
		if (n_file == n_el) {
			std::vector<float> g(n_el);
			const f16* h = (const f16*)gb.s.data();
			for (uint32_t k = 0; k < n_el; ++k) g[k] = (float)h[k];
			NGP_HIP(hipMemcpy(t->grid.p, g.data(), (size_t)n_el * 4, hipMemcpyHostToDevice));
			grid_mean_bitfield((const float*)t->grid.p, t->cfg.max_cascade, (float*)t->mean.p, (uint8_t*)t->bitfield.p, s);
		} else {
			// a size of 0 is a never-populated grid (testbed.cu:5000-5005)
			NGP_CHECK(n_file == 0, "Incompatible number of grid cascades.");
		}
		const Value& rgb = snap.at("nerf").at("rgb");
		t->rays_per_batch = (uint32_t)rgb.at("rays_per_batch").number();
		t->measured_batch_size = (uint32_t)rgb.at("measured_batch_size").number();
		t->measured_before_compaction = (uint32_t)rgb.at("measured_batch_size_before_compaction").number();
		t->measured_before_compaction_local = t->measured_before_compaction / t->world;
		t->training_step = (uint32_t)snap.at("training_step").number();
		t->loss_scalar = (float)snap.number_or("loss", 0.0);
		t->ema_step = (uint32_t)snap.number_or("density_grid_ema_step", (double)t->training_step);
		NGP_HIP(hipStreamSynchronize(s));
	});
}

// Testbed::save_snapshot / load_snapshot for the image and SDF testbeds (testbed.cu:4873-4937, 4939-5057): the
// mode-independent members (Trainer::serialize, version, mode, training_step, loss, aabb, bounding_radius).
int ngp_save_snapshot(ngp_trainer* t, void* stream, const char* path, const char* network_config_json, const char* mode,
                      const float* aabb_min, const float* aabb_max, float bounding_radius, uint32_t training_step, float loss,
                      int include_optimizer_state, int compress) {
	if (!t || !path || !mode) return NGP_INVALID;
	NERF_TRY({
		NGP_HIP(hipStreamSynchronize(S(stream)));
		Value root = snapshot_root(network_config_json);
		Value snap = Value::object();
		trainer_to_snapshot(t, ngp_trainer_n_params(t), include_optimizer_state != 0, snap);
		snap["version"] = Value::uint(SNAPSHOT_FORMAT_VERSION);
		snap["mode"] = Value::str(mode);
		snap["training_step"] = Value::uint(training_step);
		snap["loss"] = Value::real(loss);
		const float zero[3] = {0.f, 0.f, 0.f}, one[3] = {1.f, 1.f, 1.f};
		snap["aabb"]["min"] = vec3(aabb_min ? aabb_min : zero);
		snap["aabb"]["max"] = vec3(aabb_max ? aabb_max : one);
		snap["bounding_radius"] = Value::real(bounding_radius);
		write_snapshot(path, root, snap, compress);
	});
}

int ngp_load_snapshot(ngp_trainer* t, void* stream, const char* path, uint32_t* training_step, float* loss, float* aabb_min,
                      float* aabb_max, float* bounding_radius) {
	if (!t || !path) return NGP_INVALID;
	NERF_TRY({
		NGP_HIP(hipStreamSynchronize(S(stream)));
		const Value root = load_network_config(path);
		NGP_CHECK(root.find("snapshot"), std::string("File '") + path + "' does not contain a snapshot.");
		const Value& snap = root.at("snapshot");
		NGP_CHECK(snap.number_or("version", 0) >= SNAPSHOT_FORMAT_VERSION, "Snapshot uses an old format and can not be loaded.");
		trainer_from_snapshot(t, ngp_trainer_n_params(t), snap);
		if (training_step) *training_step = (uint32_t)snap.number_or("training_step", 0.0);
		if (loss) *loss = (float)snap.number_or("loss", 0.0);
		if (bounding_radius) *bounding_radius = (float)snap.number_or("bounding_radius", (double)*bounding_radius);
		if (const Value* a = snap.find("aabb")) {
			for (int d = 0; d < 3; ++d) {
				if (aabb_min) aabb_min[d] = (float)a->at("min").arr.at(d).number();
				if (aabb_max) aabb_max[d] = (float)a->at("max").arr.at(d).number();
			}
		}
	});
}

// The snapshot's mode ("nerf", "sdf", "image", ...; testbed.cu:4950-4957: a snapshot without one but with a "nerf"
// member is a NeRF snapshot), so that a Testbed can switch mode before reset_network
int ngp_snapshot_mode(const char* path, char* mode_buf, uint64_t cap) {
	if (!path || !mode_buf || cap == 0) return NGP_INVALID;
	NERF_TRY({
		const Value root = load_network_config(path);
		NGP_CHECK(root.find("snapshot"), std::string("File '") + path + "' does not contain a snapshot.");
		const Value& snap = root.at("snapshot");
		std::string m;
		if (const Value* v = snap.find("mode")) m = v->s;
		else if (snap.find("nerf")) m = "nerf";
		NGP_CHECK(!m.empty(), "Unknown snapshot mode. Snapshot must be regenerated with a new version of instant-ngp.");
		NGP_CHECK(m.size() + 1 <= cap, "snapshot mode: buffer too small");
		memcpy(mode_buf, m.c_str(), m.size() + 1);
	});
}

int ngp_snapshot_network_config(const char* path, char* json_buf, uint64_t* size) {
	if (!path || !size) return NGP_INVALID;
	NERF_TRY({
		Value root = load_network_config(path);
		NGP_CHECK(root.is_map(), "snapshot: top level is not a map");
		root.erase("snapshot");
		std::string text;
		ngp::mp::to_json_text(root, text);
		if (!json_buf) { *size = text.size() + 1; return NGP_OK; }
		NGP_CHECK(*size >= text.size() + 1, "snapshot: buffer too small");
		memcpy(json_buf, text.c_str(), text.size() + 1);
		*size = text.size() + 1;
	});
}

}  // extern "C"
