// training.h — loss functions and the image / SDF training-data kernels for gfx950.
//
// Losses restate tcnn's Loss classes (tiny-cuda-nn absent: SURVEY F1; configs name them, e.g.
// configs/image/base.json:2-4 "L2", configs/sdf/base.json "MAPE"), as evaluated by
// tcnn::Trainer::training_step (src/testbed_image.cu:276, src/testbed_sdf.cu:1304). Image sampling
// follows Testbed::train_image (src/testbed_image.cu:214-285); SDF sampling follows
// Testbed::generate_training_samples_sdf (src/testbed_sdf.cu:1187-1275).
#pragma once
#include <vector>
#include "common.h"
#include "rng.h"

namespace ngp {

// tcnn loss otypes (the engine's numbering is the C-ABI's NGP_LOSS_*)
enum TcnnLoss : uint32_t { TL_L2 = 0, TL_L1 = 1, TL_MAPE = 2, TL_SMAPE = 3, TL_RELATIVE_L2 = 4 };

struct LossEvalArgs {
	uint32_t n, dims;                 // samples, target dims (<= out_stride)
	const f16* out; uint32_t out_stride;     // network output AoS fp16
	const float* target; uint32_t target_stride;  // AoS fp32
	float loss_scale;
	f16* dL_dout; uint32_t dL_stride;        // AoS fp16; columns >= dims are zeroed
	float* values;                    // optional [n]: per-sample loss (sum over dims, already / n_total)
	float* loss_sum;                  // optional device scalar, += sum of values (zero it first)
};
void loss_evaluate(uint32_t type, const LossEvalArgs& a, hipStream_t s);

// ---- image (BASELINE config C1) ---------------------------------------------------------------
enum ImageRandomMode : uint32_t { IMG_RANDOM = 0, IMG_STRATIFIED = 3 };  // ERandomMode (common.h:124-130)
struct ImageSampleArgs {
	uint32_t n;
	uint32_t random_mode, snap_to_pixel_centers, linear_colors;
	uint32_t width, height;
	const float* texture;             // RGBA fp32 [height x width x 4], linear colours
	HostPcg32 rng;                    // draws 2n floats (generate_random_uniform)
	float* positions;                 // [n x 2]
	float* targets;                   // [n x 3]
};
void image_generate_samples(const ImageSampleArgs& a, hipStream_t s);

// ---- SDF (BASELINE config C5) -----------------------------------------------------------------
struct BvhNode {                  // TriangleBvhNode (triangle_bvh.cuh:28-32)
	float lo[3], hi[3];               // bounding box
	int32_t left, right;              // children [left, right) or, negative, leaf triangles [-left-1, -right-1)
};
// The four children of a BVH node as the signed-distance kernels read them: boxes as fp16 rounded
// outward (lo down, hi up: every box contains its float box, so pruning tests stay conservative) and
// the traversal entry of each child (bvh.hip node_entry). 64 B per node instead of 4 x 32 B.
struct BvhChildBlock {
	_Float16 lo[4][3], hi[4][3];
	int32_t entry[4];
};
static_assert(sizeof(BvhChildBlock) == 64, "child block: one 64-B read");
// child blocks of build_bvh4's nodes: block j holds nodes 1 + 4j .. 4 + 4j
void bvh_child_blocks(const std::vector<BvhNode>& nodes, std::vector<BvhChildBlock>& blocks);
struct SdfMeshDev {
	uint32_t n_triangles;
	const float* tris;                // [n x 9] vertices a, b, c, in BVH order
	const float* cdf;                 // [n] inclusive area CDF normalised to 1 (triangle_cdf)
	const BvhNode* nodes;             // 4-ary BVH (bvh.hip)
	uint32_t depth;                   // internal nodes on the longest root-to-leaf path (bvh_depth)
	// the query tree the signed-distance kernels traverse: build_bvh4 with 4 triangles per leaf over its
	// own copy of the triangles (closest triangle and stab-ray hits do not depend on the tree)
	const BvhNode* qnodes;
	const float* qtris;
	uint32_t qdepth;
	const BvhChildBlock* blocks;      // bvh_child_blocks(qnodes)
};
// internal levels of a build_bvh4 tree (sizes the traversal stacks)
uint32_t bvh_depth(const std::vector<BvhNode>& nodes);
// TriangleBvh4::build (triangle_bvh.cu:540-617): reorders tris [n x 9] in place, fills nodes
void build_bvh4(float* tris, uint32_t n_triangles, uint32_t n_primitives_per_leaf, std::vector<BvhNode>& nodes);
// signed_distance_gpu, EMeshSdfMode::Raystab (triangle_bvh.cu:436-476): upper_bounds = the distances
// already hold upper bounds of the true distances (use_existing_distances_as_upper_bounds)
void sdf_signed_distance(const SdfMeshDev& m, uint32_t n, const float* positions, float* distances, bool upper_bounds,
                         hipStream_t s);
struct SdfSampleArgs {
	uint32_t n;                       // multiple of 8 (n/8 * {4 exact, 3 offset, 1 uniform})
	HostPcg32 rng;
	float aabb_min[3], aabb_max[3];   // m_aabb inflated by zero_offset
	float stddev;                     // bounding_radius / 1024 * surface_offset_scale
	float* positions;                 // [n x 3]
	float* distances;                 // [n]
	float* perturbations;             // workspace [n x 3]
};
// uniform draws, surface samples, offsets, uniform-in-AABB samples; unsigned upper bounds in distances
void sdf_generate_samples(const SdfMeshDev& m, const SdfSampleArgs& a, hipStream_t s);
// tcnn shuffle (src/testbed_sdf.cu:1295-1296): out[perm(i)] = in[i], perm a bijection seeded by step.
void sdf_shuffle(uint32_t n, uint32_t seed, const float* pos_in, const float* dist_in, float* pos_out, float* dist_out,
                 hipStream_t s);
uint32_t sdf_shuffle_index(uint32_t i, uint32_t n, uint32_t seed);

}  // namespace ngp
