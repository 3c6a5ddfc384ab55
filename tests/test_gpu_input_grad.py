"""Input gradients and the density-only network pass on the GPU (SURVEY §8b boundary):

* tcnn Encoding::backward's dL_dinput through the hash grid (ngp_encoding_backward): the engine's fp32
  kernel against the oracle's analytic float64 restatement (orc_grid_input_grad) on the same fp16 dL/dy;
* NerfNetwork::backward with dL_dinput (nerf_network.h:256-335): the position rows through the grid and the
  direction rows through the SH encoding, first against the oracle applied to the engine's own
  intermediates (dL/d(encoding), dL/d(SH)) — the kernel alone — then end to end against the oracle;
* tcnn Network::input_gradient, the reference's normals (testbed_nerf.cu:2616 dim 3; testbed.cu:4621
  SDF dim 0): parameter gradients untouched, the output may alias the input (positions_matrix twice);
* NerfNetwork::density_forward / density_backward (nerf_network.h:355-428).

Bars: the input-gradient kernel is fp32 with a fixed order against float64: per element
|gpu - ref| <= 1e-5 (|ref| + cond), cond = sum_l scale_l sum_f |dL/dy_lf| max|T| (the size of the terms
it sums). End to end, the MLP's dL/d(encoding) and dL/d(SH) are fp16 values whose last bit can differ
from the oracle's (fp32 MFMA accumulation vs double): per element 2 fp16 ulp + 1e-6 there,
and 1e-2 relative (+ 1e-3 of the column's largest value) on dL/dinput."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


def coords(n, seed):
    g = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    return c


def nerf_with_params(pkg, orc, log2T=15, L=4, F=4, seed=3, grid_scale=0.5):
    """A NerfNetwork whose grid holds O(1) values (the initial U(+-1e-4) table gives vanishing input
    gradients), its fp16 parameters uploaded through set_params."""
    cfg = pkg.nerf_config("C2")
    cfg["encoding"].update({"log2_hashmap_size": log2T, "n_levels": L, "n_features_per_level": F})
    net = pkg.create_nerf_network(cfg)
    m = orc.make_nerf(L=L, F=F, log2T=log2T)
    p32 = orc.nerf_init(m, seed)
    nm = orc.mlp_n_params(m.density) + orc.mlp_n_params(m.rgb)
    g = np.random.default_rng(seed)
    p32[nm:] = g.uniform(-grid_scale, grid_scale, p32.size - nm)
    p16 = orc.f32_to_f16_bits(p32)
    params = torch.from_numpy(p16.view(np.float16).copy()).cuda()
    grads = torch.zeros_like(params)
    net.set_params(params, params, grads)
    return net, m, p16, params, grads


@pytest.mark.parametrize("D,L,F,log2T,max_level", [(3, 4, 4, 19, 1.0), (3, 16, 2, 19, 1.0), (2, 4, 2, 14, 1.0),
                                                   (3, 8, 1, 12, 0.6), (3, 4, 8, 10, 1.0), (3, 16, 2, 22, 1.0)])
def test_encoding_input_gradient_vs_oracle(pkg, orc, D, L, F, log2T, max_level):
    enc = {"otype": "HashGrid", "n_levels": L, "n_features_per_level": F, "log2_hashmap_size": log2T,
           "base_resolution": 16, "per_level_scale": 2.0}
    net = pkg.NetworkWithInputEncoding(D, 1, enc, {"otype": "FullyFusedMLP", "activation": "ReLU",
                                                   "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 1})
    g = orc.make_grid(D, L, F, log2T)
    rng = np.random.default_rng(L * F + D)
    nm = net.n_matrix_params
    p16 = np.zeros(net.n_params, np.float16)
    p16[nm:] = rng.uniform(-1, 1, net.n_params - nm).astype(np.float16)
    params = torch.from_numpy(p16).cuda()
    grads = torch.zeros_like(params)
    net.set_params(params, params, grads)
    net.set_max_level(max_level)
    n = 20000
    pos = rng.random((n, D), dtype=np.float32)
    pos[:3] = np.array([0.0, 1.0, 0.5], np.float32)[:, None]
    W = net.layout().encoding_width
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = rng.standard_normal((n, L * F)).astype(np.float16)
    out = torch.full((n, D + 1), 7.0, device="cuda")  # the extra column must stay untouched
    net.encoding_backward(torch.from_numpy(pos).cuda(), torch.from_numpy(dy).cuda(), grad_mode=pkg.GRAD_IGNORE,
                          dL_dinput=out)
    got = out.cpu().numpy()
    assert np.all(got[:, D] == 7.0)
    ref = orc.grid_input_grad(g, pos, p16[nm:].view(np.uint16), dy.astype(np.float32), max_level)
    scales = np.array([g.scale[l] for l in range(L)])
    active = np.arange(L) < max_level * L + 1e-3
    cond = (np.abs(dy[:, :L * F].astype(np.float64)).reshape(n, L, F).sum(2) * (scales * active)).sum(1) * 2 ** D
    bar = 1e-5 * (np.abs(ref) + cond[:, None])
    err = np.abs(got[:, :D] - ref)
    assert np.all(err <= bar), (err.max(), np.unravel_index(np.argmax(err / bar), err.shape))
    assert int(torch.count_nonzero(grads).item()) == 0  # NGP_GRAD_IGNORE: no parameter gradient written


def test_nerf_backward_input_gradients(pkg, orc):
    net, m, p16, params, grads = nerf_with_params(pkg, orc)
    n = 6000  # ragged: not a multiple of the 32-sample tile
    c = coords(n, 9)
    g = np.random.default_rng(9)
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1, 1, (n, 4))
    x = torch.from_numpy(c).cuda()
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    ctx, _ = net.forward(x, out)
    din = torch.full((n, 7), 7.0, device="cuda")
    net.backward(ctx, torch.from_numpy(dL).cuda(), dL_dinput=din)
    torch.cuda.synchronize()
    got = din.cpu().numpy()
    assert np.all(got[:, 3] == 7.0)  # the dt row is not an input of either encoding: not written
    denc = net.workspace("dL_dencoding", n).cpu().numpy().astype(np.float32)
    dsh = net.workspace("dL_dsh", n).cpu().numpy().astype(np.float32)
    # (1) the input-gradient kernel on the engine's own intermediates
    nm = orc.mlp_n_params(m.density) + orc.mlp_n_params(m.rgb)
    ref_pos = orc.grid_input_grad(m.grid, c, p16[nm:], denc, 1.0, stride=7)
    ref_dir = np.stack([orc.sh4_input_grad(c[i, 4:], dsh[i]) for i in range(n)])
    cond = (np.abs(denc[:, :16]).reshape(n, 4, 4).sum(2) * np.array([m.grid.scale[l] for l in range(4)])).sum(1) * 8
    assert np.all(np.abs(got[:, :3] - ref_pos) <= 1e-5 * (np.abs(ref_pos) + cond[:, None]))
    cond_d = np.abs(dsh).sum(1) * 12.0
    assert np.all(np.abs(got[:, 4:] - ref_dir) <= 1e-5 * (np.abs(ref_dir) + cond_d[:, None]))
    # (2) end to end: the intermediates and the result against the oracle's NerfNetwork backward
    r = orc.nerf_input_grad(m, p16, c, dL.astype(np.float32))
    ulp = lambda a: np.spacing(np.abs(a).astype(np.float16)).astype(np.float32)
    keep = orc.nerf_train_ex(m, p16, c, dL.astype(np.float32))["margin"] > 1e-4  # no ReLU within 1e-4 of switching
    assert keep.mean() > 0.3
    for name, a, b in (("dL_dsh", dsh, r["dsh"]), ("dL_dencoding", denc[:, :16], r["denc"][:, :16])):
        bad = np.abs(a[keep] - b[keep]) > 2 * ulp(b[keep]) + 1e-6
        assert bad.mean() < 1e-3, (name, bad.mean())
    for cols in (slice(0, 3), slice(4, 7)):
        a, b = got[keep, cols], r["dinput"][keep, cols]
        bad = np.abs(a - b) > 1e-2 * np.abs(b) + 1e-3 * np.abs(b).max(axis=0)
        assert bad.mean() < 2e-3, bad.mean()
    # parameter gradients were written (Overwrite) as by a plain backward
    assert int(torch.count_nonzero(grads).item()) > 0


def test_input_gradient_normals_ignores_params_and_aliases(pkg, orc):
    """testbed_nerf.cu:2616: network.input_gradient(stream, 3, positions_matrix, positions_matrix) — the
    density's gradient written over the positions it was computed from. Same values as a separate output
    buffer; the dt row (3) keeps its value; the gradient buffer is untouched (EGradientMode::Ignore)."""
    net, m, p16, params, grads = nerf_with_params(pkg, orc, seed=4)
    n = 4099
    c = coords(n, 4)
    grads.fill_(3.0)
    sep = net.input_gradient(3, torch.from_numpy(c).cuda())
    x = torch.from_numpy(c).cuda()
    net.input_gradient(3, x, d_dinput=x)  # aliased, as the reference calls it
    torch.cuda.synchronize()
    a, b = sep.cpu().numpy(), x.cpu().numpy()
    np.testing.assert_array_equal(a[:, :3], b[:, :3])
    np.testing.assert_array_equal(a[:, 4:], b[:, 4:])
    np.testing.assert_array_equal(b[:, 3], c[:, 3])
    assert bool(torch.all(grads == 3.0))
    # d density / d input: the oracle with a one-hot dL/doutput (row 3), backprop scale 128 divided out
    dL = np.zeros((n, 16), np.float32)
    dL[:, 3] = 128.0
    r = orc.nerf_input_grad(m, p16, c, dL, scale=1.0 / 128.0)
    keep = orc.nerf_train_ex(m, p16, c, dL)["margin"] > 1e-4
    for cols in (slice(0, 3), slice(4, 7)):
        bad = np.abs(a[keep, cols] - r["dinput"][keep, cols]) > 1e-2 * np.abs(r["dinput"][keep, cols]) + \
            1e-3 * np.abs(r["dinput"][keep, cols]).max(axis=0) + 1e-7
        assert bad.mean() < 2e-3, bad.mean()
    # density alone depends on the direction only through nothing: its direction gradient is exactly 0
    assert np.all(a[:, 4:] == 0.0)


def test_density_forward_backward(pkg, orc):
    """NerfNetwork::density_forward + density_backward (nerf_network.h:355-428): the density network's
    16-row output, density-MLP and grid gradients from a full 16-row dL/d(density output), dL/dposition;
    the rgb MLP's gradients are left as they were."""
    net, m, p16, params, grads = nerf_with_params(pkg, orc, seed=6, grid_scale=1e-1)
    n = 5000
    c = coords(n, 6)
    g = np.random.default_rng(6)
    dL = g.uniform(-1, 1, (n, 16)).astype(np.float16)
    x = torch.from_numpy(c).cuda()
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    nd, nr = orc.mlp_n_params(m.density), orc.mlp_n_params(m.rgb)
    grads.fill_(5.0)
    ctx, _ = net.density_forward(x, out)
    din = torch.zeros((n, 7), device="cuda")
    net.density_backward(ctx, torch.from_numpy(dL).cuda(), dL_dinput=din)
    torch.cuda.synchronize()
    ref_out = orc.nerf_density(m, p16, c)
    o = out.cpu().numpy().astype(np.float32)
    assert np.abs(o - ref_out).max() <= 1e-2 * np.abs(ref_out).max()
    gg = grads.cpu().numpy().astype(np.float32)
    assert np.all(gg[nd:nd + nr] == 5.0)  # rgb MLP untouched
    ref_g, ref_din = orc.nerf_density_backward(m, p16, c, dL.astype(np.float32))
    for name, lo, hi in (("density", 0, nd), ("grid", nd + nr, gg.size)):
        err = np.abs(gg[lo:hi] - ref_g[lo:hi]).max()
        assert err <= 2e-2 * np.abs(ref_g[lo:hi]).max() + 1e-4, (name, err)
    d = din.cpu().numpy()
    bad = np.abs(d[:, :3] - ref_din[:, :3]) > 1e-2 * np.abs(ref_din[:, :3]) + 1e-3 * np.abs(ref_din[:, :3]).max(axis=0)
    assert bad.mean() < 2e-3, bad.mean()
    assert np.all(d[:, 3:] == 0.0)
    # the wrong context kind is refused (the reference's dynamic_cast<const ForwardContext&> contract)
    ctx2, _ = net.forward(x, torch.zeros((n, 16), dtype=torch.float16, device="cuda"))
    with pytest.raises(RuntimeError):
        net.density_backward(ctx2, torch.from_numpy(dL).cuda())


def _sh4_np(d):
    """Real spherical harmonics of degree 4 (16 values) of unit-cube-warped directions in float64: the
    published closed forms tcnn's SH encoding evaluates on d = 2 in - 1 (independent of the engine and of
    the oracle's derivative code)."""
    x, y, z = (2.0 * d[..., k] - 1.0 for k in range(3))
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    return np.stack([
        np.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
        -0.48860251190291987 * x, 1.0925484305920792 * xy, -1.0925484305920792 * yz,
        0.94617469575755997 * z2 - 0.31539156525251999, -1.0925484305920792 * xz,
        0.54627421529603959 * x2 - 0.54627421529603959 * y2, 0.59004358992664352 * y * (-3.0 * x2 + y2),
        2.8906114426405538 * xy * z, 0.45704579946446572 * y * (1.0 - 5.0 * z2),
        0.3731763325901154 * z * (5.0 * z2 - 3.0), 0.45704579946446572 * x * (1.0 - 5.0 * z2),
        1.4453057213202769 * z * (x2 - y2), 0.59004358992664352 * x * (-x2 + 3.0 * y2)], axis=-1)


def test_input_gradients_against_finite_differences(pkg, orc):
    """An independent check of the input-gradient formulas (the oracle restates the same ones).

    Grid rows: the encoding is trilinear inside a cell, so for points whose cells at every level are the
    same at x - h and x + h the central difference of sum_f dy_f enc_f(x) (enc from the GPU forward, fp16) is
    the exact derivative up to the fp16 rounding of the features, which bounds the difference element by
    element. SH rows: the central difference (float64, h = 1e-4) of sum_j dL/dsh_j SH_j(2 dir - 1) with the
    published degree-4 closed forms, against the direction rows of the NerfNetwork backward (its own dL/dsh):
    the factor 2 of d = 2 dir - 1 and every polynomial term."""
    L, F, D = 4, 2, 3
    enc = {"otype": "HashGrid", "n_levels": L, "n_features_per_level": F, "log2_hashmap_size": 19,
           "base_resolution": 16, "per_level_scale": 2.0}
    net = pkg.NetworkWithInputEncoding(D, 1, enc, {"otype": "FullyFusedMLP", "activation": "ReLU",
                                                   "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 1})
    rng = np.random.default_rng(21)
    nm = net.n_matrix_params
    p16 = np.zeros(net.n_params, np.float16)
    p16[nm:] = rng.uniform(-1, 1, net.n_params - nm).astype(np.float16)
    params = torch.from_numpy(p16).cuda()
    net.set_params(params, params, torch.zeros_like(params))
    n, h = 8192, np.float32(2.0 ** -12)
    pos = rng.uniform(0.05, 0.95, (n, D)).astype(np.float32)
    W = net.layout().encoding_width
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = rng.standard_normal((n, L * F)).astype(np.float16)
    got = torch.zeros((n, D), device="cuda")
    net.encoding_backward(torch.from_numpy(pos).cuda(), torch.from_numpy(dy).cuda(), grad_mode=pkg.GRAD_IGNORE, dL_dinput=got)
    got = got.cpu().numpy().astype(np.float64)
    scales = np.float32(16.0) * np.float32(2.0) ** np.arange(L, dtype=np.float32) - np.float32(1.0)
    dyf = dy[:, :L * F].astype(np.float64)
    checked = 0
    for d in range(D):
        xs = []
        for sgn in (1, -1):
            x = pos.copy()
            x[:, d] = pos[:, d] + np.float32(sgn) * h
            xs.append(x)
        # cells of every level at both points (pos = scale * x + 0.5, floor: the engine's grid arithmetic)
        same = np.ones(n, bool)
        for sc in scales:
            same &= np.all(np.floor(xs[0] * sc + np.float32(0.5)) == np.floor(xs[1] * sc + np.float32(0.5)), axis=1)
        e = [net.encode(torch.from_numpy(x).cuda()).cpu().numpy()[:, :L * F] for x in xs]
        step = (xs[0][:, d].astype(np.float64) - xs[1][:, d].astype(np.float64))
        fd = ((e[0].astype(np.float64) - e[1].astype(np.float64)) * dyf).sum(1) / step
        ulp = lambda a: np.spacing(np.abs(a).astype(np.float16)).astype(np.float64)
        bound = (np.abs(dyf) * (ulp(e[0]) + ulp(e[1])) / 2).sum(1) / step + 1e-4 * np.abs(got[:, d]) + 1e-6
        err = np.abs(fd - got[:, d])
        assert np.all(err[same] <= bound[same]), (d, float((err / bound)[same].max()))
        checked += int(same.sum())
    assert checked > n  # most points stay inside their cells at every level

    # SH rows through the NerfNetwork backward
    net2, m, p16b, params2, grads2 = nerf_with_params(pkg, orc, seed=8)
    c = coords(3000, 8)
    g = np.random.default_rng(8)
    dL = np.zeros((3000, 16), np.float16)
    dL[:, :4] = g.uniform(-1, 1, (3000, 4))
    x = torch.from_numpy(c).cuda()
    ctx, _ = net2.forward(x, torch.zeros((3000, 16), dtype=torch.float16, device="cuda"))
    din = torch.zeros((3000, 7), device="cuda")
    net2.backward(ctx, torch.from_numpy(dL).cuda(), dL_dinput=din)
    torch.cuda.synchronize()
    dsh = net2.workspace("dL_dsh", 3000).cpu().numpy().astype(np.float64)
    dirs = c[:, 4:].astype(np.float64)
    assert np.allclose(_sh4_np(dirs[:5]), np.stack([orc.sh4(d) for d in c[:5, 4:]]), atol=1e-6)
    hh = 1e-4
    fd = np.zeros((3000, 3))
    for k in range(3):
        dp, dm = dirs.copy(), dirs.copy()
        dp[:, k] += hh
        dm[:, k] -= hh
        fd[:, k] = ((_sh4_np(dp) - _sh4_np(dm)) * dsh).sum(1) / (2 * hh)
    gd = din.cpu().numpy()[:, 4:].astype(np.float64)
    scale = (np.abs(dsh).sum(1) * 12.0)[:, None]
    assert np.all(np.abs(gd - fd) <= 1e-5 * scale + 1e-6), float(np.abs(gd - fd).max())


def test_backward_honours_inference_params(pkg, orc):
    """nerf_network.h:256-335: backward_impl runs every sub-backward with the forward's use_inference_params.
    A forward on the inference parameters followed by backward must give the input and parameter gradients
    of a network whose training parameters ARE those inference parameters, bit for bit."""
    net, m, p16, params, grads = nerf_with_params(pkg, orc, seed=11)
    g = np.random.default_rng(11)
    other = torch.from_numpy((p16.view(np.float16).astype(np.float32) *
                              g.uniform(0.5, 1.5, p16.size).astype(np.float32)).astype(np.float16)).cuda()
    n = 5000
    c = torch.from_numpy(coords(n, 11)).cuda()
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1, 1, (n, 4))
    dL = torch.from_numpy(dL).cuda()
    res = []
    for train_p, inf_p, use_inf in ((other, params, True), (params, params, False)):
        gr = torch.zeros_like(params)
        net.set_params(train_p, inf_p, gr)
        out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
        ctx, _ = net.forward(c, out, use_inference_params=use_inf)
        din = torch.zeros((n, 7), device="cuda")
        net.backward(ctx, dL, dL_dinput=din)
        torch.cuda.synchronize()
        res.append((out.cpu().numpy().view(np.uint16), din.cpu().numpy(), gr.cpu().numpy().view(np.uint16)))
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a, b)
