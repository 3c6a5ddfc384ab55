"""Phase clock of the training MLP kernel k_nerf_mlp_train (mlp.hip built with -DNGP_TRAIN_CLOCK): runs the C2 (or
C2') training pass a few times on the variant library NGP_ENGINE_LIB and prints, for the last launch, the mean time
(us, from each block's entry) at which every phase boundary is reached over the blocks (wave 0 of each block), and
the per-iteration phase durations averaged over iterations. Timing experiments only.

    make -C instant-ngp_amd/csrc OUT=../../build/train_clock EXTRA=-DNGP_TRAIN_CLOCK
    NGP_ENGINE_LIB=build/train_clock/libngp_engine.so python tools/train_clock.py [--variant C2] [--steps 5]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["inputs", "density_fwd", "rgb_fwd_out", "images", "bwd_rgb", "bwd_density", "denc_store", "barrier1", "dW",
          "barrier2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="C2")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import bench
    from __graft_entry__ import load_package
    pkg = load_package()
    n = bench.B
    step, _, net, trainer, _ = bench.nerf_pass(pkg, args.variant, n, 0, 1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    lib = pkg.lib()
    f = lib.ngp_debug_train_clock
    f.argtypes = [C.c_void_p, C.c_uint32]
    S = 128
    buf = np.zeros(1024 * S, np.uint64)
    assert f(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(1024, S).astype(np.int64)
    blocks = int((t[:, 0] > 0).sum())
    t = t[:blocks]
    rel = (t - t[:, 0:1]) * 0.01  # 100 MHz ticks -> us
    n_it = 0
    while 2 + 10 * n_it + 9 < S - 1 and (t[:, 2 + 10 * n_it + 9] > 0).all():
        n_it += 1
    per = {p: [] for p in PHASES}
    for i in range(n_it):
        for k, p in enumerate(PHASES):
            a = 2 + 10 * i + k
            prev = a - 1
            per[p].append(float((rel[:, a] - rel[:, prev]).mean()))
    out = {"variant": args.variant, "blocks": blocks, "iterations": n_it,
           "weights_loaded_us": round(float(rel[:, 1].mean()), 3),
           "first_iteration_start_us": round(float(rel[:, 2].mean() - per["inputs"][0]), 3) if n_it else None,
           "exit_us": round(float(rel[:, 127].mean()), 3),
           "per_iteration_us": {p: round(float(np.mean(v)), 3) for p, v in per.items()},
           "iteration_total_us": round(float(sum(np.mean(v) for v in per.values())), 3)}
    out["after_loop_us"] = round(float((rel[:, 127] - rel[:, 2 + 10 * (n_it - 1) + 9]).mean()), 3) if n_it else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
