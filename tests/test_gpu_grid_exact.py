"""Hash-grid backward bit for bit against the oracle at the BASELINE configs' real sizes.

The engine's destination-bucketed backward (csrc/grid_scatter.hip, used for n >= 4096) rounds every
contribution w * dL/dy to fp16 exactly as tcnn's kernel_grid_backward does before its half2 atomicAdd,
sums those fp16 values exactly (int64 in units of 2^-24) and rounds once. oracle/ngp_oracle.c
orc_grid_backward_exact restates that contract on the CPU, so the comparison is np.array_equal over the
whole gradient table: C2 (L4 F4 T2^19), C2' (L16 F2 T2^19), C5 (L16 F2 T2^22) and C1 (2D) at the full
2^18-sample batch, uniform points and a NeRF-like concentrated cloud (hot coarse entries, split
buckets), per-sample max_level, gradient accumulation, and points on/outside the unit cube.
"""
import zlib

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

MLP2 = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}
ADAM = {"otype": "Adam", "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6}


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


def enc_cfg(L, F, T):
    return {"otype": "HashGrid", "n_levels": L, "n_features_per_level": F, "log2_hashmap_size": T, "base_resolution": 16,
            "per_level_scale": 2.0}


def positions(kind, n, D, seed):
    g = np.random.default_rng(seed)
    if kind == "uniform":
        x = g.random((n, D), dtype=np.float32)
    else:  # NeRF-like: most samples in a small blob (hot coarse entries), the rest uniform
        x = np.clip(0.5 + 0.06 * g.standard_normal((n, D)), 0.0, 1.0).astype(np.float32)
        m = g.random(n) < 0.2
        x[m] = g.random((int(m.sum()), D), dtype=np.float32)
    x[:64] = np.round(x[:64] * 4) / 4      # exact cell boundaries
    x[64:72] = 1.0                         # the upper faces
    x[72:80] = np.float32(1.0 + 1e-3)      # outside the unit cube (tcnn wraps the index)
    return x


def run_backward(pkg, D, L, F, T, x, dy16, grad_mode=None, init=None, bricks=None):
    net = pkg.NetworkWithInputEncoding(D, 1, enc_cfg(L, F, T), MLP2)
    if bricks is not None:
        net.set_option("grid_bricks", bricks)
    tr = pkg.Trainer(net, ADAM)
    nm = net.n_matrix_params
    if init is not None:
        tr.gradients[nm:] = torch.from_numpy(init.view(np.float16)).cuda()
    kw = {} if grad_mode is None else {"grad_mode": grad_mode}
    net.encoding_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy16).cuda(), **kw)
    torch.cuda.synchronize()
    got = tr.gradients[nm:].cpu().numpy().view(np.uint16).copy()
    return net, tr, got


def dy_batch(net, n, L, F, seed, scale=1.0):
    W = net.layout().encoding_width if net is not None else L * F
    g = np.random.default_rng(seed)
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = (g.uniform(-1, 1, (n, L * F)) * scale).astype(np.float16)
    return dy


def encoding_width(L, F):
    return (L * F + 15) // 16 * 16


@pytest.mark.parametrize("name,D,L,F,T,kind", [
    ("C2", 3, 4, 4, 19, "uniform"), ("C2", 3, 4, 4, 19, "nerf"),
    ("C2p", 3, 16, 2, 19, "uniform"), ("C2p", 3, 16, 2, 19, "nerf"),
    ("C5", 3, 16, 2, 22, "uniform"), ("C5", 3, 16, 2, 22, "nerf"),
    ("C1", 2, 4, 2, 14, "uniform"), ("F1", 3, 8, 1, 16, "nerf"), ("F8", 3, 4, 8, 14, "uniform"),
])
def test_grid_backward_bitexact_full_batch(pkg, orc, name, D, L, F, T, kind):
    n = 1 << 18
    x = positions(kind, n, D, seed=zlib.crc32(f"{name}/{kind}".encode()) & 0xffff)
    W = encoding_width(L, F)
    g = np.random.default_rng(n + L)
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = g.uniform(-1, 1, (n, L * F)).astype(np.float16)
    _, _, got = run_backward(pkg, D, L, F, T, x, dy)
    ref = orc.grid_backward_exact(orc.make_grid(D, L, F, T), x, dy)
    assert got.shape == ref.shape
    bad = np.nonzero(got != ref)[0]
    detail = [(int(i), hex(got[i]), hex(ref[i])) for i in bad[:6]]
    assert bad.size == 0, f"{name}/{kind}: {bad.size} of {ref.size} gradient entries differ: {detail}"
    assert np.count_nonzero(ref) > 0


@pytest.mark.parametrize("name,L,F,T,kind", [("C2", 4, 4, 19, "uniform"), ("C2", 4, 4, 19, "nerf"),
                                              ("C2p", 16, 2, 19, "nerf"), ("C5", 16, 2, 22, "uniform")])
def test_grid_backward_bricks_bitexact(pkg, orc, name, L, F, T, kind):
    """The brick-summed dense levels (model option grid_bricks): the same table as the oracle, with points on
    the unit cube's faces (the upper corners at coordinate res) and outside it (the global fallback)."""
    n = 1 << 18
    x = positions(kind, n, 3, seed=zlib.crc32(f"bricks/{name}/{kind}".encode()) & 0xffff)
    x[80:88] = np.float32(1.0 + 2e-2)
    x[88:96] = np.float32(-1e-2)
    W = encoding_width(L, F)
    g = np.random.default_rng(n + L + 1)
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = g.uniform(-1, 1, (n, L * F)).astype(np.float16)
    net, _, got = run_backward(pkg, 3, L, F, T, x, dy, bricks=1)
    assert net.query("grid_brick_levels") == 2  # levels 1-2 (C5: res 32, 64; level 0 has too few cells per brick)
    ref = orc.grid_backward_exact(orc.make_grid(3, L, F, T), x, dy)
    bad = np.nonzero(got != ref)[0]
    detail = [(int(i), hex(got[i]), hex(ref[i])) for i in bad[:6]]
    assert bad.size == 0, f"{name}/{kind}: {bad.size} of {ref.size} gradient entries differ: {detail}"


def test_grid_backward_bitexact_small_values(pkg, orc):
    """dL/dy near the fp16 subnormal range: contributions round to subnormals or to zero exactly as in
    tcnn, and sums of subnormals are still exact."""
    D, L, F, T, n = 3, 16, 2, 19, 1 << 16
    x = positions("nerf", n, D, seed=3)
    dy = np.zeros((n, encoding_width(L, F)), np.float16)
    dy[:, :L * F] = (np.random.default_rng(1).uniform(-1, 1, (n, L * F)) * 3e-5).astype(np.float16)
    _, _, got = run_backward(pkg, D, L, F, T, x, dy)
    ref = orc.grid_backward_exact(orc.make_grid(D, L, F, T), x, dy)
    np.testing.assert_array_equal(got, ref)


def test_grid_backward_bitexact_max_level(pkg, orc):
    """Per-sample max_level (set_max_level_gpu, testbed_nerf.cu:3996,4004): the backward skips levels
    l > max_level * L (tcnn's '>' — the forward zeroes at '>=')."""
    D, L, F, T, n = 3, 16, 2, 19, 100000
    x = positions("uniform", n, D, seed=4)
    ml = np.random.default_rng(5).random(n).astype(np.float32)
    ml[:100] = np.float32(7 / 16)  # exactly on a level boundary
    net = pkg.NetworkWithInputEncoding(D, 1, enc_cfg(L, F, T), MLP2)
    tr = pkg.Trainer(net, ADAM)
    net.set_max_level(1.0, torch.from_numpy(ml).cuda())
    dy = dy_batch(net, n, L, F, seed=6)
    net.encoding_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy).cuda())
    torch.cuda.synchronize()
    got = tr.gradients[net.n_matrix_params:].cpu().numpy().view(np.uint16)
    ref = orc.grid_backward_exact(orc.make_grid(D, L, F, T), x, dy, 1.0, ml)
    np.testing.assert_array_equal(got, ref)


def test_grid_backward_bitexact_accumulate(pkg, orc):
    """GRAD_ACCUMULATE: old + exact sum, rounded once (tcnn accumulate semantics); entries without
    contributions keep their value."""
    D, L, F, T, n = 3, 8, 2, 16, 30000
    x = positions("nerf", n, D, seed=7)
    grid = orc.make_grid(D, L, F, T)
    np_ = orc.grid_n_entries(grid) * F
    init = (np.random.default_rng(8).uniform(-0.5, 0.5, np_)).astype(np.float16).view(np.uint16)
    dy = dy_batch(None, n, L, F, seed=9)
    dy = np.concatenate([dy, np.zeros((n, encoding_width(L, F) - L * F), np.float16)], axis=1)
    _, _, got = run_backward(pkg, D, L, F, T, x, dy, grad_mode=pkg.GRAD_ACCUMULATE, init=init)
    ref = orc.grid_backward_exact(grid, x, dy, grad16=init)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("D,L,F,T", [(3, 4, 4, 19), (3, 16, 2, 22)])
def test_grid_backward_ragged_sizes(pkg, orc, D, L, F, T):
    """Batch sizes that are not multiples of the scatter chunk (512 samples at C2; 1024 at C5, whose
    sparse 2^22 tables take the larger chunk), at the bucketed threshold."""
    grid = orc.make_grid(D, L, F, T)
    for n in (4096, 4097, 5000, 65535):
        x = positions("nerf", n, D, seed=n)
        dy = dy_batch(None, n, L, F, seed=n)
        dy = np.concatenate([dy, np.zeros((n, encoding_width(L, F) - L * F), np.float16)], axis=1)
        _, _, got = run_backward(pkg, D, L, F, T, x, dy)
        ref = orc.grid_backward_exact(grid, x, dy)
        np.testing.assert_array_equal(got, ref, err_msg=f"n={n}")
