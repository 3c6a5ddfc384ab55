"""Phase clock of the two-waves-per-SIMD MLP training kernel (mlp_train16.hip built with -DNGP_T16_CLOCK):
runs the C2 training step a few times on the variant library NGP_ENGINE_LIB and prints, for the last step,
the mean time (us, from the block's entry) at which each phase boundary is reached over the blocks, and
the spread of the blocks' entry/exit times. Timing experiments only.

    NGP_ENGINE_LIB=build/t16_clock/libngp_engine.so python tools/t16_clock.py [--variant C2] [--steps 5]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="C2")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import bench
    from __graft_entry__ import load_package
    pkg = load_package()
    n = bench.B
    step, _, net, trainer, _ = bench.nerf_pass(pkg, args.variant, n, 0, 1, opts=("mlp_train16=1",))
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    lib = pkg._capi.lib()
    f = lib.ngp_debug_t16_clock
    f.argtypes = [C.c_void_p, C.c_uint32]
    S = 128
    buf = np.zeros(1024 * S, np.uint64)
    assert f(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(1024, S).astype(np.int64)
    blocks = int((t[:, 0] > 0).sum())
    t = t[:blocks]
    t0 = t[:, 0:1]
    rel = (t - t0) * 0.01  # 100 MHz ticks -> us
    names = {0: "entry", 1: "staged", 2: "loop"}
    ks = ["inputs", "d0", "dout_sh", "r0", "rh", "img", "bwd_rgb", "bwd_density", "denc", "sync1", "dW", "sync2"]
    for i in range(3, S - 1):
        names[i] = f"it{(i - 3) // 12}.{ks[(i - 3) % 12]}"
    names[S - 1] = "exit"
    out = {"blocks": blocks, "n": n}
    prev = 0.0
    phases = {}
    for i in range(S):
        col = t[:, i]
        ok = col >= t0[:, 0]
        if i > 0 and (col == 0).all():
            continue
        m = float(rel[ok, i].mean())
        phases[names[i]] = {"at_us": round(m, 3), "delta_us": round(m - prev, 3)}
        prev = m
    out["phases"] = phases
    start = (t[:, 0] - t[:, 0].min()) * 0.01
    end = (t[:, S - 1] - t[:, 0].min()) * 0.01
    out["entry_spread_us"] = [round(float(np.percentile(start, q)), 3) for q in (0, 50, 100)]
    out["exit_spread_us"] = [round(float(np.percentile(end, q)), 3) for q in (0, 50, 100)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
