"""Debug: where does the F=1 bucketed grid backward differ from the exact oracle? (GPU box)"""
import os, sys, zlib
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
from __graft_entry__ import load_package
import pyoracle as orc
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_grid_exact import positions, run_backward, encoding_width
pkg = load_package()
for (D, L, F, T, kind) in [(3, 8, 1, 16, "nerf"), (3, 8, 1, 16, "uniform"), (3, 8, 2, 16, "nerf"), (3, 2, 1, 16, "nerf"),
                           (3, 8, 1, 19, "nerf")]:
    n = 1 << 18
    x = positions(kind, n, D, seed=zlib.crc32(f"F1/{kind}".encode()) & 0xffff)
    W = encoding_width(L, F)
    g = np.random.default_rng(n + L)
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = g.uniform(-1, 1, (n, L * F)).astype(np.float16)
    _, _, got = run_backward(pkg, D, L, F, T, x, dy)
    _, _, got2 = run_backward(pkg, D, L, F, T, x, dy)
    grid = orc.make_grid(D, L, F, T)
    ref = orc.grid_backward_exact(grid, x, dy)
    bad = np.nonzero(got != ref)[0]
    offs = np.array(grid.offsets[:L + 1])
    lv = np.searchsorted(offs, bad // F, side="right") - 1
    print(D, L, F, T, kind, "bad", bad.size, "deterministic", np.array_equal(got, got2), "levels", np.bincount(lv, minlength=L).tolist(),
          "diff ulps", (got[bad].astype(np.int32) - ref[bad].astype(np.int32))[:10].tolist(), flush=True)
