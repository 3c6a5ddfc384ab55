// grid_scatter.h — destination-bucketed hash-grid backward (see grid_scatter.hip).
#pragma once
#include "grid.h"
#include "optimizer.h"
#include "slab_reduce.h"

namespace ngp {

// gradient store modes of the bucketed backward's last kernels (template parameter MODE)
enum : uint32_t { SC_STORE_F16 = 0, SC_FUSED_ADAM = 1, SC_STORE_F32 = 2 };

// Brick-summed dense levels (3D grids): dense levels LB..LD-1 are not sent through items. Samples are
// counting-sorted by brick (K^3 cells of the finest of those levels, f = LD - 1; one item per sample: its
// index), each brick part sums its samples' contributions to levels 0..LD-1 in LDS over the brick's region
// (a box of corners per level, W[l]^3 entries at regoff[l]) and stores the exact int64 sums as a slab; the
// finalize adds, per entry, the slabs of every brick whose region holds it. Corners outside the region
// (positions outside [0, 1]) go to an int64 fallback table with global atomics.
struct BrickConst {
	uint32_t LB = 0, LD = 0;  // brick levels [LB, LD) (coarser ones stay items: too few corners per brick, LDS contention)
	uint32_t vb0 = 0;         // bricks are vbs [vb0, vb0 + NBK), owned by level LB's range
	uint32_t K = 8, NB = 0, NBK = 0, R = 0;
	uint32_t W[4] = {}, regoff[4] = {};
	uint16_t lo[4][32] = {};  // region's first corner coordinate per level and brick coordinate
};

struct ScatterPlan {
	uint32_t B = 0;          // log2 entries per bucket (a bucket's accumulators fill one LDS tile)
	uint32_t n_buckets = 0;  // buckets are level-aligned: a bucket never spans two levels
	uint32_t spb = 0;        // samples per chunk (hist/scatter blocks are (chunk, level))
	uint32_t n_chunks = 0;
	uint32_t max_lb = 0;     // most buckets any one level spans
	uint64_t n_items = 0;    // n * L * 2^D contributions
	uint32_t split_limit = 0;// buckets with more items are summed in parts (k_sc_plan)
	uint32_t part = 0;
	uint32_t max_split_blocks = 0;
	uint32_t max_split_buckets = 0;
	uint32_t xcd_map = 2;    // scatter block order: 2 = a chunk's level blocks and neighbouring chunks share an XCD
	uint32_t bt = 1024;      // bucket accumulation block threads (experiment knob NGP_SC_BT)
	BrickConst bk;           // bk.LD = 0: every level through items
	uint32_t brick_part = 1024;  // samples per brick part (parts of one brick each store a slab)
	// workspace layout (bytes)
	size_t off_hist = 0, off_cur = 0, off_tot = 0, off_split = 0, off_lo = 0, off_splitb = 0, off_scratch = 0, off_idx = 0, off_val = 0,
	       off_bp = 0,    // bricks: {first part, parts} per brick
	       off_fb = 0,    // bricks: int64 fallback table [offsets[LD] x F] + flag; zero between steps
	       total = 0;
};

// bricks: allow the brick-summed dense levels (ScatterPlan::bk; chosen only where they move fewer bytes)
ScatterPlan make_scatter_plan(const GridDesc& g, uint32_t n, bool bricks = true);
// Phase 1 (positions only, so it can run on a side stream while the forward pass and the MLP run):
// bucket histogram per block of samples + per-bucket scans.
// hist_done: the histogram was produced by the training forward (scatter_hist, grid_forward).
void grid_scatter_prepare(const GridDesc& g, const GridBwdArgs& b, const ScatterPlan& p, void* workspace, hipStream_t s,
                          bool hist_done = false);
// The forward-fused histogram for this plan, or false when it does not apply (row kernel needed,
// the bucket counts of all levels must fit the forward block's LDS).
bool scatter_hist(const GridDesc& g, const ScatterPlan& p, void* workspace, GridHist& h);
// Phase 2: dL/dy -> gradient. overwrite: b.grad's grid section is fully written (no memset needed);
// otherwise the sums are added to it. Same level masking as grid_backward.
// slab (optional): the MLP's dW slab reduction, run in extra blocks of the last backward kernel
// (same arithmetic as reduce_slabs, no launch of its own).
// fused (optional, overwrite only): apply the lazy optimizer update to every entry with a nonzero
// gradient instead of storing the gradient (optimizer.h FusedAdam); the grid part of b.grad is then
// left unwritten.
// parts (optional): the bucket accumulation in bucket ranges, so that a consumer of the gradient (the sharded
// data-parallel exchange) can start on some parameters while the rest is still summed. Range j = buckets
// [j ? vb_end[j - 1] : 0, vb_end[j]) (the last one ends at the last bucket); the ranges run from the last to the
// first, each as a k_sc_accumulate launch (its split buckets' parts and its other buckets) and a k_sc_split_reduce
// launch (its split buckets; range 0 also the MLP's dW slabs), then `after(user, j, s)` is called: every gradient
// of the range's entries and of every higher range's (range 0: and the MLP's) is final on s. Integer sums:
// bit-identical to the one-launch form. Not with bricks or a fused update.
struct BwdParts {
	static constexpr uint32_t MAX = 8;
	uint32_t k = 0;
	uint32_t vb_end[MAX] = {};
	void (*after)(void* user, uint32_t part, hipStream_t s) = nullptr;
	void* user = nullptr;
};
// the first bucket whose entries reach past grid parameter `param` (entry * F, grid-relative): the bucket holding
// it (n_buckets when none). A range boundary there puts a bucket that straddles a part boundary in the higher
// range, which the parted backward sums first (BwdParts)
uint32_t scatter_bucket_at_param(const GridDesc& g, const ScatterPlan& p, uint64_t param);
void grid_backward_sorted(const GridDesc& g, const GridBwdArgs& b, const ScatterPlan& p, void* workspace,
                          hipStream_t s, bool overwrite, uint32_t debug = 0, const SlabJob* slab = nullptr,
                          const FusedAdam* fused = nullptr, const BwdParts* parts = nullptr);

}  // namespace ngp
