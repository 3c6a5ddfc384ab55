"""How far the engine sits from tiny-cuda-nn's own fp16 arithmetic, at BASELINE's full sizes.

The engine's contract is stricter than tcnn's: fp32 blends and MLP accumulation rounded once to fp16,
and an exact grid-gradient sum. The oracle's tcnn mode (oracle/ngp_tcnn_mode.c, pinned on the CPU by
tests/test_oracle_tcnn_mode.py) computes what tcnn would on the same inputs: fp16 FMA chains in the grid blend,
fp16 WMMA accumulators in the MLPs, sequential fp16 atomics in the grid backward. tcnn itself is absent from the
reference (parity unpinned); its call sites are nerf_network.h:143-153, 201-216, 236-241, 324-333, and
the in-tree analogue of its fp16 atomics is takikawa_encoding.cuh:184-264.

Bars, written out:
* grid features (the encoding): every element within tcnn's own rounding-error bound of its fp16 chain plus half an
  fp16 spacing (the engine rounds the blend once): |e_gpu - e_tcnn| <= bound_tcnn + ulp16(e_gpu) / 2. The share
  within SURVEY's "1 ulp-fp16 + 1e-4" is reported (measured ~98.3 % at full size: tcnn's chain itself strays
  further from the exact blend; at least 95 % asserted);
* network outputs and dL/d(encoding): |x_gpu - x_tcnn| <= 1e-2 * max|x_tcnn| ("rel <= 1e-2, fp16 accumulate vs
  fp32"). A ReLU whose pre-activation lies within the fp16 accumulation noise of zero switches between the two
  arithmetics and masks a whole term: elements beyond the bar only in samples with such a ReLU (smallest
  |pre-activation| / sum |W a| below 2^-10, orc_*_train_ex margin), and in at most 2.5 % of the samples (measured
  1.4-1.7 % for dL/d(encoding) at C2, C2' and C5: fp16 accumulators round each 16-wide k-step, 2^-11 of the partial
  sum, so a 64-deep chain moves a pre-activation by up to ~2^-10 of its conditioning);
* grid gradient, from the engine's own dL/d(encoding): within the sequential fp16 sum's own bound (half a spacing
  per add) plus half a spacing: |g_gpu - g_tcnn| <= bound_tcnn + ulp16(g_gpu) / 2, every parameter.
The measured maxima go to the test report (record_property) and DESIGN §4.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FLIP_MARGIN = 2.0 ** -10


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


def coords_batch(n, seed):
    g = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    return c


def ulp16(x):
    return np.spacing(np.abs(x).astype(np.float16)).astype(np.float64)


def features_within(got, ref, bound):
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    assert np.all(err <= bound.astype(np.float64) * (1 + 1e-6) + 0.5 * ulp16(got) + 1e-9), float(err.max())
    # SURVEY's "1 ulp-fp16 + 1e-4" is tighter than tcnn's own chain of 8 fp16 FMAs (each rounds its partial blend,
    # and the weight is rounded to fp16 first): with table values of a trained size (|v| ~ 0.5) a few per cent of
    # tcnn's features are 2-4 ulp from the exact blend, which the engine rounds once (bit-exact with the oracle's
    # exact-blend restatement, tests/test_gpu_parity.py). The share is reported, with a floor
    survey = float(np.mean(err <= ulp16(ref) + 1e-4))
    ulps = err / ulp16(ref)
    assert survey >= 0.95, survey
    return (f"features max |d| {err.max():.3g} (max {ulps.max():.2f} ulp16, 99.9th pct {np.quantile(ulps, 0.999):.2f}), "
            f"within 1 ulp16 + 1e-4: {survey:.6f}")


def rel_within(name, got, ref, margin):
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    scale = float(np.abs(ref).max())
    bad = np.unique(np.where(err > 1e-2 * scale)[0])
    assert np.all(margin[bad] < FLIP_MARGIN), (name, float(margin[bad].max()))
    assert bad.size <= 0.025 * got.shape[0], (name, bad.size)
    ok = np.setdiff1d(np.arange(got.shape[0]), bad)
    return (f"{name} max |d| / max|ref| {err.max() / scale:.3g} (outside flip samples {err[ok].max() / scale:.3g}), "
            f"{bad.size} flip samples of {got.shape[0]}")


def grad_within(got16, ref16, bound):
    got = got16.view(np.float16).astype(np.float64)
    ref = ref16.view(np.float16).astype(np.float64)
    err = np.abs(got - ref)
    assert np.all(err <= bound * (1 + 1e-6) + 0.5 * ulp16(got) + 1e-12), float(err.max())
    nz = bound > 0
    return (f"grid gradient max |d| {err.max():.3g}, max |d| / bound {np.max(err[nz] / bound[nz]):.3g}, "
            f"bitwise equal {np.mean(got16 == ref16):.4f}")


@pytest.mark.parametrize("cfg_name,log2T,L,F", [("C2", 19, 4, 4), ("C2p", 19, 16, 2)])
def test_nerf_network_vs_tcnn_arithmetic(pkg, orc, cfg_name, log2T, L, F, record_property):
    cfg = pkg.nerf_config(cfg_name)
    cfg["encoding"]["log2_hashmap_size"] = log2T
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"])
    nm = net.n_matrix_params
    p = net.initialize_params(1337)
    p[nm:] = np.random.default_rng(3).uniform(-0.5, 0.5, p.size - nm).astype(np.float32)  # trained-looking grid
    tr.set_params_full_precision(p)
    torch.cuda.synchronize()
    p16 = tr.params.cpu().numpy().view(np.uint16).copy()
    n = 1 << 18
    c = coords_batch(n, seed=31)
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = np.random.default_rng(32).uniform(-1, 1, (n, 4))
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    net.forward_backward(torch.from_numpy(c).cuda(), torch.from_numpy(dL).cuda(), output=out)
    torch.cuda.synchronize()
    assert tr.gradients_valid
    got_out = out.float().cpu().numpy()
    got_enc = net.workspace("encoding", n).float().cpu().numpy()[:, :L * F]
    got_denc16 = net.workspace("dL_dencoding", n).cpu().numpy()
    got_g = tr.gradients.cpu().numpy().view(np.uint16)[nm:]

    m = orc.make_nerf(L=L, F=F, log2T=log2T)
    table = p16[nm:]
    ref_enc, bound = orc.grid_forward_tcnn(m.grid, c, table, stride=7)
    t = orc.nerf_tcnn(m, p16, c, dL.astype(np.float32))
    margin = orc.nerf_train_ex(m, p16, c, dL.astype(np.float32))["margin"]
    ref_g, gbound = orc.grid_backward_tcnn(m.grid, c, got_denc16, stride=7)
    msgs = [features_within(got_enc, ref_enc, bound),
            rel_within("output", got_out[:, :4], t["out"][:, :4], margin),
            rel_within("dL/dencoding", got_denc16.view(np.float16).astype(np.float32)[:, :L * F], t["denc"][:, :L * F], margin),
            grad_within(got_g, ref_g, gbound)]
    record_property("tcnn_mode", "; ".join(msgs))
    print(f"\n{cfg_name}: " + "\n".join(msgs))


SDF_MLP = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}
ADAM = {"otype": "Adam", "learning_rate": 1e-4, "beta1": 0.9, "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6}


def test_sdf_network_c5_vs_tcnn_arithmetic(pkg, orc, record_property):
    """C5 (configs/sdf/base.json, T = 2^22): NetworkWithInputEncoding forward and backward at 2^18 samples."""
    enc = {"otype": "HashGrid", "n_levels": 16, "n_features_per_level": 2, "log2_hashmap_size": 22,
           "base_resolution": 16, "per_level_scale": 2.0}
    net = pkg.NetworkWithInputEncoding(3, 1, enc, SDF_MLP)
    tr = pkg.Trainer(net, ADAM)
    nm = net.n_matrix_params
    p = net.initialize_params(1337)
    p[nm:] = np.random.default_rng(8).uniform(-0.5, 0.5, p.size - nm).astype(np.float32)
    tr.set_params_full_precision(p)
    torch.cuda.synchronize()
    p16 = tr.params.cpu().numpy().view(np.uint16).copy()
    n = 1 << 18
    g = np.random.default_rng(9)
    x = g.random((n, 3), dtype=np.float32)
    x[: n // 2] = np.clip(0.5 + 0.1 * g.standard_normal((n // 2, 3)), 0, 1).astype(np.float32)
    dy = np.zeros((n, 16), np.float16)
    dy[:, :1] = g.uniform(-1, 1, (n, 1))
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    net.forward_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy).cuda(), output=out)
    torch.cuda.synchronize()
    got_out = out.float().cpu().numpy()
    got_enc = net.workspace("encoding", n).float().cpu().numpy()[:, :32]
    got_denc16 = net.workspace("dL_dencoding", n).cpu().numpy()
    got_g = tr.gradients.cpu().numpy().view(np.uint16)[nm:]

    grid = orc.make_grid(3, 16, 2, 22)
    mlp = orc.make_mlp(32, 64, 2, 16)
    ref_enc, bound = orc.grid_forward_tcnn(grid, x, p16[nm:])
    t_out, t_denc = orc.net_tcnn(grid, mlp, p16, x, dy.astype(np.float32))
    margin = orc.net_train_ex(grid, mlp, p16, x, dy.astype(np.float32))["margin"]
    ref_g, gbound = orc.grid_backward_tcnn(grid, x, got_denc16)
    msgs = [features_within(got_enc, ref_enc, bound),
            rel_within("output", got_out[:, :1], t_out[:, :1], margin),
            rel_within("dL/dencoding", got_denc16.view(np.float16).astype(np.float32), t_denc, margin),
            grad_within(got_g, ref_g, gbound)]
    record_property("tcnn_mode", "; ".join(msgs))
    print("\nC5: " + "\n".join(msgs))
