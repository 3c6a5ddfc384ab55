// training_abi.hip — C-ABI for the image (BASELINE C1) and SDF (BASELINE C5) primitives:
// Testbed::train_image (src/testbed_image.cu:214-285) and Testbed::train_sdf +
// generate_training_samples_sdf (src/testbed_sdf.cu:1187-1312), over the engine's training_step.
#include <algorithm>
#include <cmath>
#include <memory>
#include <string>
#include <vector>

#include "../../include/ngp_engine.h"
#include "training.h"

using namespace ngp;

extern "C" int ngp_trainer_training_step(ngp_trainer*, void*, uint32_t, const float*, uint32_t, const float*, uint32_t, int, float,
                                         int, float*);
extern "C" int ngp_trainer_optimizer_step(ngp_trainer*, void*, float);
extern "C" const char* ngp_last_error(void);
namespace ngp { void set_last_error(const char* msg); }

namespace {
struct Buf {
	void* p = nullptr;
	size_t n = 0;
	template <typename T> T* get(size_t count) {
		const size_t need = std::max<size_t>(count * sizeof(T), 16);
		if (need > n) {
			if (p) NGP_HIP(hipFree(p));
			NGP_HIP(hipMalloc(&p, need));
			n = need;
		}
		return (T*)p;
	}
	~Buf() { if (p) (void)hipFree(p); }
};
void check_rc(int rc) { if (rc != 0) throw Error(ngp_last_error()); }
hipStream_t S(void* s) { return (hipStream_t)s; }
}  // namespace

struct ngp_image {
	uint32_t width = 0, height = 0;
	float* texture = nullptr;  // RGBA fp32, linear colours (EDataType::Float)
	Buf positions, targets;
	~ngp_image() { if (texture) (void)hipFree(texture); }
};

struct ngp_sdf_mesh {
	uint32_t n_triangles = 0;
	float* tris = nullptr;  // [n x 9], BVH order
	float* cdf = nullptr;   // [n]
	BvhNode* nodes = nullptr;
	uint32_t n_nodes = 0;
	uint32_t depth = 0;
	BvhNode* qnodes = nullptr;  // query tree (4 triangles per leaf) over qtris, and its child blocks
	float* qtris = nullptr;
	uint32_t qdepth = 0;
	BvhChildBlock* blocks = nullptr;
	std::vector<float> tris_host;
	Buf perturbations;
	~ngp_sdf_mesh() {
		if (tris) (void)hipFree(tris);
		if (cdf) (void)hipFree(cdf);
		if (nodes) (void)hipFree(nodes);
		if (blocks) (void)hipFree(blocks);
		if (qnodes) (void)hipFree(qnodes);
		if (qtris) (void)hipFree(qtris);
	}
	SdfMeshDev dev() const { return SdfMeshDev{n_triangles, tris, cdf, nodes, depth, qnodes, qtris, qdepth, blocks}; }
};

#define TRY(...)                                   \
	try {                                          \
		__VA_ARGS__;                               \
		return NGP_OK;                             \
	} catch (const std::exception& e) {            \
		ngp::set_last_error(e.what());              \
		return NGP_ERROR;                          \
	}
#define ARG(cond)                                                    \
	do {                                                             \
		if (!(cond)) {                                               \
			ngp::set_last_error("invalid argument: " #cond);          \
			return NGP_INVALID;                                      \
		}                                                            \
	} while (0)

extern "C" {

// ---- image ---------------------------------------------------------------------------------------
int ngp_image_default_config(ngp_image_config* out) {
	ARG(out);
	out->random_mode = NGP_IMAGE_STRATIFIED;  // testbed.h:875
	out->snap_to_pixel_centers = 1;           // testbed.h:871
	out->linear_colors = 0;                   // testbed.h:872
	return NGP_OK;
}

int ngp_image_create(uint32_t width, uint32_t height, const float* rgba_host, ngp_image** out) {
	ARG(out && rgba_host && width >= 2 && height >= 2);
	TRY({
		auto img = std::make_unique<ngp_image>();
		img->width = width;
		img->height = height;
		const size_t bytes = (size_t)width * height * 4 * sizeof(float);
		NGP_HIP(hipMalloc(&img->texture, bytes));
		NGP_HIP(hipMemcpy(img->texture, rgba_host, bytes, hipMemcpyHostToDevice));
		*out = img.release();
	});
}

void ngp_image_destroy(ngp_image* img) { delete img; }

static ImageSampleArgs image_args(const ngp_image* img, uint32_t n, const ngp_rng* rng, const ngp_image_config* cfg, float* pos,
                                  float* tgt) {
	ImageSampleArgs a{};
	a.n = n;
	a.random_mode = cfg->random_mode;
	a.snap_to_pixel_centers = cfg->snap_to_pixel_centers;
	a.linear_colors = cfg->linear_colors;
	a.width = img->width;
	a.height = img->height;
	a.texture = img->texture;
	a.rng = HostPcg32{rng->state, rng->inc};
	a.positions = pos;
	a.targets = tgt;
	return a;
}

int ngp_image_generate_training_samples(const ngp_image* img, void* stream, uint32_t n, ngp_rng* rng, const ngp_image_config* cfg,
                                        float* positions, float* targets) {
	ARG(img && rng && cfg && (n == 0 || (positions && targets)));
	ARG(cfg->random_mode == NGP_IMAGE_RANDOM || cfg->random_mode == NGP_IMAGE_STRATIFIED);
	TRY({
		image_generate_samples(image_args(img, n, rng, cfg, positions, targets), S(stream));
		HostPcg32 r{rng->state, rng->inc};
		r.advance(2ull * n);  // generate_random_uniform advances m_rng by n_elements
		rng->state = r.state;
	});
}

int ngp_image_train_step(ngp_image* img, ngp_trainer* t, void* stream, uint32_t batch, ngp_rng* rng, const ngp_image_config* cfg,
                         float* loss_sum) {
	ARG(img && t && rng && cfg && batch > 0);
	TRY({
		float* pos = img->positions.get<float>((size_t)batch * 2);
		float* tgt = img->targets.get<float>((size_t)batch * 3);
		check_rc(ngp_image_generate_training_samples(img, stream, batch, rng, cfg, pos, tgt));
		// training_step(stream, positions, targets, nullptr, run_optimizer = false), L2 loss
		// (configs/image/base.json:2-4), then optimizer_step(stream, 128) (testbed_image.cu:276-283)
		check_rc(ngp_trainer_training_step(t, stream, batch, pos, 2, tgt, 3, NGP_LOSS_L2, 128.0f, 0, loss_sum));
		check_rc(ngp_trainer_optimizer_step(t, stream, 128.0f));
	});
}

// ---- SDF -----------------------------------------------------------------------------------------
int ngp_sdf_mesh_create(uint32_t n_triangles, const float* tris_host, ngp_sdf_mesh** out) {
	ARG(out && tris_host && n_triangles > 0);
	TRY({
		auto m = std::make_unique<ngp_sdf_mesh>();
		m->n_triangles = n_triangles;
		// Testbed::load_mesh (testbed_sdf.cu:1155-1172): the BVH build reorders the triangles, then the
		// surface-area distribution is built over that order
		m->tris_host.assign(tris_host, tris_host + (size_t)n_triangles * 9);
		std::vector<BvhNode> nodes;
		build_bvh4(m->tris_host.data(), n_triangles, 8, nodes);
		tris_host = m->tris_host.data();
		m->n_nodes = (uint32_t)nodes.size();
		m->depth = bvh_depth(nodes);
		{
			// the query tree: the same median-split build with 4 triangles per leaf over a copy of the
			// triangles (the reference's 8-triangle tree above keeps ordering them for surface sampling).
			// Signed distances do not depend on the tree; on the armadillo batch this one is 19 % faster
			// (ground truth 6.2 -> 5.0 ms, profiles/r03q_sdf_gt_leaf{8,4}.json)
			std::vector<float> q(m->tris_host);
			std::vector<BvhNode> qn;
			build_bvh4(q.data(), n_triangles, 4, qn);
			m->qdepth = bvh_depth(qn);
			std::vector<BvhChildBlock> cb;
			bvh_child_blocks(qn, cb);
			NGP_HIP(hipMalloc(&m->qnodes, qn.size() * sizeof(BvhNode)));
			NGP_HIP(hipMemcpy(m->qnodes, qn.data(), qn.size() * sizeof(BvhNode), hipMemcpyHostToDevice));
			NGP_HIP(hipMalloc(&m->qtris, q.size() * sizeof(float)));
			NGP_HIP(hipMemcpy(m->qtris, q.data(), q.size() * sizeof(float), hipMemcpyHostToDevice));
			NGP_HIP(hipMalloc(&m->blocks, cb.size() * sizeof(BvhChildBlock)));
			NGP_HIP(hipMemcpy(m->blocks, cb.data(), cb.size() * sizeof(BvhChildBlock), hipMemcpyHostToDevice));
		}
		NGP_HIP(hipMalloc(&m->nodes, nodes.size() * sizeof(BvhNode)));
		NGP_HIP(hipMemcpy(m->nodes, nodes.data(), nodes.size() * sizeof(BvhNode), hipMemcpyHostToDevice));
		// triangle_distribution.build(surface areas) (testbed_sdf.cu:1167-1172, discrete_distribution.h:20-36)
		std::vector<float> w(n_triangles), cdf(n_triangles);
		float total = 0.f;
		for (uint32_t i = 0; i < n_triangles; ++i) {
			const float* t = tris_host + 9 * (size_t)i;
			const float e1[3] = {t[3] - t[0], t[4] - t[1], t[5] - t[2]}, e2[3] = {t[6] - t[0], t[7] - t[1], t[8] - t[2]};
			const float c[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
			w[i] = 0.5f * std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
			total += w[i];
		}
		const float inv = 1.0f / total;
		float acc = 0.f;
		for (uint32_t i = 0; i < n_triangles; ++i) {
			acc += w[i] * inv;
			cdf[i] = acc;
		}
		cdf.back() = 1.0f;
		NGP_HIP(hipMalloc(&m->tris, (size_t)n_triangles * 9 * sizeof(float)));
		NGP_HIP(hipMalloc(&m->cdf, (size_t)n_triangles * sizeof(float)));
		NGP_HIP(hipMemcpy(m->tris, tris_host, (size_t)n_triangles * 9 * sizeof(float), hipMemcpyHostToDevice));
		NGP_HIP(hipMemcpy(m->cdf, cdf.data(), (size_t)n_triangles * sizeof(float), hipMemcpyHostToDevice));
		*out = m.release();
	});
}

void ngp_sdf_mesh_destroy(ngp_sdf_mesh* m) { delete m; }

int ngp_sdf_bvh_build(float* tris, uint32_t n_triangles, uint32_t n_primitives_per_leaf, void* nodes_out, uint32_t* n_nodes) {
	ARG(tris && n_nodes && n_primitives_per_leaf >= 1);
	TRY({
		std::vector<float> work(tris, tris + (size_t)n_triangles * 9);
		std::vector<BvhNode> nodes;
		build_bvh4(work.data(), n_triangles, n_primitives_per_leaf, nodes);
		if (!nodes_out) { *n_nodes = (uint32_t)nodes.size(); return NGP_OK; }
		NGP_CHECK(*n_nodes >= nodes.size(), "bvh: node buffer too small");
		std::copy(work.begin(), work.end(), tris);
		std::copy(nodes.begin(), nodes.end(), (BvhNode*)nodes_out);
		*n_nodes = (uint32_t)nodes.size();
	});
}

int ngp_sdf_mesh_triangles(const ngp_sdf_mesh* m, float* tris_out) {
	ARG(m && tris_out);
	TRY({ std::copy(m->tris_host.begin(), m->tris_host.end(), tris_out); });
}

int ngp_sdf_generate_training_samples(ngp_sdf_mesh* m, void* stream, uint32_t n, ngp_rng* rng, const float* aabb_min,
                                      const float* aabb_max, float stddev, float* positions, float* distances) {
	ARG(m && rng && aabb_min && aabb_max && n % 8 == 0 && (n == 0 || (positions && distances)));
	TRY({
		const uint32_t n_offset = n / 8 * 3;
		SdfSampleArgs a{};
		a.n = n;
		a.rng = HostPcg32{rng->state, rng->inc};
		for (int d = 0; d < 3; ++d) { a.aabb_min[d] = aabb_min[d]; a.aabb_max[d] = aabb_max[d]; }
		a.stddev = stddev;
		a.positions = positions;
		a.distances = distances;
		a.perturbations = m->perturbations.get<float>((size_t)std::max(n_offset, 1u) * 3);
		sdf_generate_samples(m->dev(), a, S(stream));
		HostPcg32 r{rng->state, rng->inc};
		r.advance(3ull * n + 3ull * n_offset);  // uniform positions, then the logistic perturbations
		rng->state = r.state;
	});
}

int ngp_sdf_signed_distance(ngp_sdf_mesh* m, void* stream, uint32_t n, const float* positions, float* distances) {
	ARG(m && (n == 0 || (positions && distances)));
	TRY({ sdf_signed_distance(m->dev(), n, positions, distances, false, S(stream)); });
}

int ngp_sdf_shuffle(void* stream, uint32_t n, uint32_t seed, const float* positions, const float* distances,
                    float* positions_shuffled, float* distances_shuffled) {
	ARG(n == 0 || (positions && distances && positions_shuffled && distances_shuffled));
	TRY({ sdf_shuffle(n, seed, positions, distances, positions_shuffled, distances_shuffled, S(stream)); });
}

int ngp_sdf_train_step(ngp_trainer* t, void* stream, uint32_t n, const float* positions, const float* distances, uint32_t step,
                       float* positions_shuffled, float* distances_shuffled, float* loss_sum) {
	ARG(t && n > 0 && positions && distances && positions_shuffled && distances_shuffled);
	TRY({
		// shuffle<vec3>/shuffle<float> seeded by m_training_step (testbed_sdf.cu:1295-1296), then
		// training_step(stream, positions, distances) with the MAPE loss (configs/sdf/base.json) and
		// the optimizer step (run_optimizer defaults to true), loss scale 128
		check_rc(ngp_sdf_shuffle(stream, n, step, positions, distances, positions_shuffled, distances_shuffled));
		check_rc(ngp_trainer_training_step(t, stream, n, positions_shuffled, 3, distances_shuffled, 1, NGP_LOSS_MAPE, 128.0f, 1,
		                                   loss_sum));
	});
}

}  // extern "C"
