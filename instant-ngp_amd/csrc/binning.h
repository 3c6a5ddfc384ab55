// binning.h — spatial binning of samples + LDS-windowed hash-grid backward (see binning.hip).
#pragma once
#include <algorithm>

#include "grid.h"

namespace ngp {

constexpr uint32_t BIN_BLOCK = 1024;  // samples per histogram block

struct WinPlan {
	uint32_t R = 0;        // bins per axis
	uint32_t n_bins = 0;   // R^D
	uint32_t n_win = 0;    // levels 0..n_win-1 are accumulated in LDS windows
	uint32_t W[16] = {};   // window width (vertices per axis) per level
	uint32_t max_verts = 0;// largest window (vertices); LDS holds one level's window at a time
	uint32_t debug = 0;    // timing experiments only: 1 skip accumulate, 2 skip flush
};

struct WinArgs {
	uint32_t n;
	const float* pos; uint32_t pos_stride;
	const f16* dL_dy; uint32_t dy_stride;  // AoS
	f16* grad;
	const uint32_t* sorted;                // sample ids grouped by bin
	const uint32_t* offs;                  // exclusive-scanned bin-major histogram [bin][hist block]
	uint32_t n_hist_blocks;
	uint32_t R, n_bins, n_win;
	uint32_t W[16];
	uint32_t debug;
};

// Choose R and the windowed level prefix by a request-count cost model (0 windowed levels => none).
// lds_budget_bytes bounds one level's window (int32 fixed point, F per vertex).
WinPlan make_win_plan(const GridDesc& g, uint32_t n, size_t lds_budget_bytes);
inline uint32_t bin_hist_len(const WinPlan& p, uint32_t n) { return p.n_bins * ((n + BIN_BLOCK - 1) / BIN_BLOCK); }
// workspace (u32 count) for bin_samples' histogram + scanned offsets + scan temp; sorted: [n] u32
size_t bin_workspace_u32(const WinPlan& p, uint32_t n);
const uint32_t* bin_offsets(const WinPlan& p, uint32_t n, const uint32_t* ws);
void bin_samples(uint32_t D, uint32_t n, const float* pos, uint32_t stride, const WinPlan& p, uint32_t* hist,
                 uint32_t* sorted, hipStream_t s);
void grid_backward_windowed(const GridDesc& g, const WinPlan& p, const GridBwdArgs& b, const uint32_t* hist,
                            const uint32_t* sorted, hipStream_t s);

}  // namespace ngp
