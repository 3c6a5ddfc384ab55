"""The trainer's density-grid update (update_density_grid_nerf, testbed_nerf.cu:3412-3536) in its two splat forms:
the default sorts the update's samples by 8192-cell bin before the density evaluation and takes each bin's maxima in
LDS (every cell written, no memset); NGP_SPLAT_SORT=0 is the reference's form (memset, density in generated order,
scattered atomicMax). Max is order-independent and each sample's density does not depend on its neighbours, so 300
training steps (every-step updates, then the step-256 switch to every 16th with the 0.01 threshold) must leave the
density grid, bitfield, mean and parameters bit-identical. Each mode runs in its own process (the knob is read once)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from __graft_entry__ import load_package
pkg = load_package()
ds = pkg.synthetic.lego_like_dataset(n_images=8, width=96, height=96, seed=5)
cfg = pkg.nerf.default_config(float(sys.argv[3]))
net = pkg.create_nerf_network(pkg.nerf_config("C2"))
tr = pkg.Trainer(net, pkg.nerf_config("C2")["optimizer"])
run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
for _ in range(300):
    run.train_step(get_loss=False)
torch.cuda.synchronize()
np.savez(sys.argv[2], grid=run.density_grid.cpu().numpy(), bitfield=run.bitfield.cpu().numpy(),
         mean=run.mean_density.cpu().numpy(), params=tr.params.cpu().numpy())
"""


def _run(tmp_path, mode, aabb):
    out = str(tmp_path / f"m{mode}_{aabb}.npz")
    env = dict(os.environ, NGP_SPLAT_SORT=str(mode))
    subprocess.run([sys.executable, "-c", SCRIPT, ROOT, out, str(aabb)], env=env, check=True, timeout=300)
    return np.load(out)


@pytest.mark.gpu
@pytest.mark.parametrize("aabb", [1.0, 4.0])
def test_sorted_splat_training_bitwise(tmp_path, aabb):
    a = _run(tmp_path, 1, aabb)
    b = _run(tmp_path, 0, aabb)
    for k in ("grid", "bitfield", "mean", "params"):
        np.testing.assert_array_equal(a[k].view(np.uint8), b[k].view(np.uint8), err_msg=k)
    assert (a["grid"] > 0).any()
