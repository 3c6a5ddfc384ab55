"""Brick-summed dense levels of the bucketed grid backward (csrc/grid_scatter.hip, ScatterPlan::bk).

At 2^18 samples the C2 (L4 F4) and C2' (L16 F2) grids send their dense levels 1-2 through bricks
(each sample's index sorted by brick, its contributions summed in LDS over the brick's region, the exact
int64 slabs added per entry) instead of 8 items per sample and level. The contributions and their
fixed-point sums are those of the item path, so training must be bit for bit the same with the bricks
switched off (model option grid_bricks = 0): the NeRF training step with
the forward-fused histogram, on the eager optimizer layout (gradient stored, separate optimizer launch) and on
the lazy layout (the grid's and the MLP's optimizer update fused into the backward; the default for C2 and
C2'), each forced with NGP_LAZY_EMA, on uniform and on concentrated sample clouds whose bricks split into
parts, with positions on and past the unit cube's faces (the exact global fallback table). A second test
alternates batch sizes and toggles the option on one model (each re-plan moves the fallback table within
the reused workspace). The oracle comparison of the same path is tests/test_gpu_grid_exact.py.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
N = 1 << 18


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


def batch(kind, n, seed):
    g = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3), dtype=np.float32)
    if kind == "blob":  # NeRF-like: 80 % of the samples in a small blob -> a few bricks of thousands of samples
        blob = np.clip(0.5 + 0.05 * g.standard_normal((n, 3)), 0.0, 1.0).astype(np.float32)
        keep = g.random(n) < 0.8
        c[keep, :3] = blob[keep]
    c[:64, :3] = np.round(c[:64, :3] * 8) / 8   # brick and cell boundaries
    c[64:72, :3] = 1.0                          # the upper faces
    c[72:80, :3] = np.float32(1.0 + 2e-2)       # past the cube: corners outside every brick region
    c[80:88, :3] = np.float32(-1e-2)
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1e-2, 1e-2, (n, 4))
    return torch.from_numpy(c).cuda(), torch.from_numpy(dL).cuda()


def make(pkg, variant, lazy):
    old = os.environ.get("NGP_LAZY_EMA")
    os.environ["NGP_LAZY_EMA"] = "1" if lazy else "0"
    try:
        cfg = pkg.nerf_config(variant)
        net = pkg.create_nerf_network(cfg)
        tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
    finally:
        if old is None:
            del os.environ["NGP_LAZY_EMA"]
        else:
            os.environ["NGP_LAZY_EMA"] = old
    return net, tr


def result(tr):
    torch.cuda.synchronize()
    return tr.params.cpu().numpy().view(np.uint16).copy(), tr.params_full_precision.cpu().numpy().view(np.uint32).copy()


def train(pkg, variant, kind, bricks, lazy, steps=4):
    net, tr = make(pkg, variant, lazy)
    net.set_option("grid_bricks", 1 if bricks else 0)
    net.reserve(N)
    assert tr.fused_update_active(N) == lazy
    for s in range(steps):
        x, dL = batch(kind, N, 100 + s)
        tr.train_step(x, dL, 128.0)
    torch.cuda.synchronize()
    assert net.query("grid_brick_levels") == (2 if bricks else 0)  # C2 and C2': levels 1-2 (res 32, 64)
    return result(tr)


@pytest.mark.parametrize("lazy", [False, True], ids=["eager", "lazy_fused"])
@pytest.mark.parametrize("variant", ["C2", "C2p"])
@pytest.mark.parametrize("kind", ["uniform", "blob"])
def test_bricks_train_bitwise_like_items(pkg, variant, kind, lazy):
    p1, w1 = train(pkg, variant, kind, True, lazy)
    p0, w0 = train(pkg, variant, kind, False, lazy)
    assert np.isfinite(p1.view(np.float16).astype(np.float32)).all()
    np.testing.assert_array_equal(p1, p0)
    np.testing.assert_array_equal(w1, w0)


# (batch, grid_bricks) per step on ONE model: every change of either re-plans in the same workspace
SCHEDULE = ((N, 1), (N // 2, 1), (N, 1), (N, 0), (N // 4 * 3, 1), (N, 1), (N // 2, 0), (N // 2, 1))


@pytest.mark.parametrize("lazy", [False, True], ids=["eager", "lazy_fused"])
def test_bricks_replan_alternating_batches(pkg, lazy):
    runs = []
    for bricks_on in (True, False):
        net, tr = make(pkg, "C2", lazy)
        net.reserve(N)
        for s, (n, b) in enumerate(SCHEDULE):
            net.set_option("grid_bricks", b if bricks_on else 0)
            x, dL = batch("blob" if s % 2 else "uniform", n, 300 + s)
            tr.train_step(x, dL, 128.0)
        runs.append(result(tr))
        del net, tr
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
