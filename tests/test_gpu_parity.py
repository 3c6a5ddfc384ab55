"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on identical seeded inputs.

Bars: hash-grid indices / forward encoding bit-exact (same fp32 formula and corner
order, then one RNE rounding to fp16); MLP and network outputs within 1e-2 of the output scale
(fp16 activations, fp32 accumulation order differs); gradients within 2e-2 of the gradient scale
(fp16 atomics / fp16 rounding of per-layer gradients); optimizer within 1e-5 relative.
"""
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


def coords_batch(n, seed=0, dirs=True):
    g = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    return c


def enc_cfg(L, F, T, b=2.0):
    return {"otype": "HashGrid", "n_levels": L, "n_features_per_level": F, "log2_hashmap_size": T, "base_resolution": 16,
            "per_level_scale": b}


MLP2 = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}
ADAM = {"otype": "Adam", "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6}


def random_params(trainer, model, orc_n_matrix, grid_scale=1.0, seed=3):
    g = np.random.default_rng(seed)
    n = model.n_params
    p = model.initialize_params(1337)
    p[orc_n_matrix:] = g.uniform(-grid_scale, grid_scale, n - orc_n_matrix).astype(np.float32)
    trainer.set_params_full_precision(p)
    torch.cuda.synchronize()
    return trainer.params.cpu().numpy().view(np.uint16).copy()


@pytest.mark.parametrize("D,L,F,T", [(3, 4, 4, 19), (3, 16, 2, 19), (2, 16, 2, 14), (3, 8, 1, 12), (3, 4, 8, 14), (2, 4, 2, 14),
                                     (3, 16, 2, 22)])
def test_encoding_forward_bitexact(pkg, orc, D, L, F, T):
    net = pkg.NetworkWithInputEncoding(D, 1, enc_cfg(L, F, T), MLP2)
    tr = pkg.Trainer(net, ADAM)
    p16 = random_params(tr, net, net.n_matrix_params)
    n = 3001
    x = np.random.default_rng(D * L).random((n, D), dtype=np.float32)
    x[:8] = np.array([0, 1, 0.5, 0.25, 0.999999, 1e-7, 0.75, 0.125], np.float32)[:, None]
    xt = torch.from_numpy(x).cuda()
    got = net.encode(xt).cpu().numpy().view(np.uint16)
    g = orc.make_grid(D, L, F, T)
    ref = orc.f32_to_f16_bits(orc.grid_forward(g, x, p16[net.n_matrix_params:]))
    LF = L * F
    bad = np.argwhere(got[:, :LF] != ref)
    detail = [(int(i), int(f), hex(got[i, f]), hex(ref[i, f]), x[i].tolist()) for i, f in bad[:5]]
    assert len(bad) == 0, f"{len(bad)} mismatching fp16 features: {detail}"
    assert np.all(got[:, LF:] == 0)
    # SoA (tcnn RM) layout gives the same values
    soa = net.encode(xt, layout=pkg.LAYOUT_SOA).cpu().numpy().view(np.uint16)
    assert np.array_equal(soa[:LF].T, ref)


def test_encoding_max_level(pkg, orc):
    net = pkg.NetworkWithInputEncoding(3, 1, enc_cfg(8, 2, 14), MLP2)
    tr = pkg.Trainer(net, ADAM)
    p16 = random_params(tr, net, net.n_matrix_params)
    x = np.random.default_rng(5).random((777, 3), dtype=np.float32)
    ml = np.random.default_rng(6).random(777).astype(np.float32)
    net.set_max_level(1.0, torch.from_numpy(ml).cuda())
    got = net.encode(torch.from_numpy(x).cuda()).cpu().numpy().view(np.uint16)
    ref = orc.f32_to_f16_bits(orc.grid_forward(orc.make_grid(3, 8, 2, 14), x, p16[net.n_matrix_params:], 1.0, ml))
    assert np.array_equal(got, ref)
    net.set_max_level(0.5)
    got = net.encode(torch.from_numpy(x).cuda()).cpu().numpy().view(np.uint16)
    ref = orc.f32_to_f16_bits(orc.grid_forward(orc.make_grid(3, 8, 2, 14), x, p16[net.n_matrix_params:], 0.5))
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("D,L,F,T", [(3, 4, 4, 19), (3, 16, 2, 14), (2, 4, 2, 14), (3, 8, 1, 12)])
def test_encoding_backward(pkg, orc, D, L, F, T):
    net = pkg.NetworkWithInputEncoding(D, 1, enc_cfg(L, F, T), MLP2)
    tr = pkg.Trainer(net, ADAM)
    random_params(tr, net, net.n_matrix_params)
    n = 2048
    g = np.random.default_rng(11)
    x = g.random((n, D), dtype=np.float32)
    W = net.layout().encoding_width
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = g.uniform(-1, 1, (n, L * F))
    net.encoding_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy).cuda())
    torch.cuda.synchronize()
    got = tr.gradients.float().cpu().numpy()[net.n_matrix_params:]
    ref = orc.grid_backward(orc.make_grid(D, L, F, T), x, dy[:, :L * F].astype(np.float32))
    # fp16 atomics (tcnn's half2 atomicAdd semantics): each add rounds the running sum to fp16, so the
    # error bound grows with adds per entry; coarse 2D levels here take ~30 adds of up to 0.4
    tol = 3e-2 * np.abs(ref).max() + 1e-3
    assert np.abs(got - ref).max() <= tol, np.abs(got - ref).max()
    assert np.allclose(got[ref == 0], 0)


@pytest.fixture(scope="module")
def nerf_setup(pkg, orc):
    cfg = pkg.nerf_config("C2")
    cfg["encoding"]["log2_hashmap_size"] = 14
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"])
    p16 = random_params(tr, net, net.n_matrix_params, grid_scale=0.5)
    m = orc.make_nerf(L=4, F=4, log2T=14)
    return net, tr, p16, m


@pytest.mark.parametrize("n", [1, 31, 32, 1000, 4099])
def test_nerf_inference(pkg, orc, nerf_setup, n):
    net, tr, p16, m = nerf_setup
    c = coords_batch(n, seed=n)
    out = net.inference(torch.from_numpy(c).cuda(), use_inference_params=False).float().cpu().numpy()
    ref = orc.nerf_forward(m, p16, c)
    sc = np.abs(ref).max()
    assert np.abs(out - ref).max() <= 1e-2 * sc, (np.abs(out - ref).max(), sc)


def test_nerf_density(pkg, orc, nerf_setup):
    net, tr, p16, m = nerf_setup
    c = coords_batch(2000, seed=4)
    out = net.density(torch.from_numpy(c).cuda(), use_inference_params=False).float().cpu().numpy()
    ref = orc.nerf_density(m, p16, c)
    assert np.abs(out - ref).max() <= 1e-2 * np.abs(ref).max()
    soa = net.density(torch.from_numpy(c).cuda(), layout=pkg.LAYOUT_SOA, use_inference_params=False).float().cpu().numpy()
    assert np.array_equal(soa.T, out)


@pytest.mark.parametrize("n", [32, 777, 4096])
def test_nerf_forward_backward(pkg, orc, nerf_setup, n):
    net, tr, p16, m = nerf_setup
    c = coords_batch(n, seed=100 + n)
    g = np.random.default_rng(n)
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1, 1, (n, 4))
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    net.forward_backward(torch.from_numpy(c).cuda(), torch.from_numpy(dL).cuda(), output=out)
    torch.cuda.synchronize()
    ref_out = orc.nerf_forward(m, p16, c)
    assert np.abs(out.float().cpu().numpy() - ref_out).max() <= 1e-2 * np.abs(ref_out).max()
    ref = orc.nerf_backward(m, p16, c, dL.astype(np.float32))
    got = tr.gradients.float().cpu().numpy()
    nd = orc.mlp_n_params(m.density)
    nr = orc.mlp_n_params(m.rgb)
    for name, lo, hi in [("density", 0, nd), ("rgb", nd, nd + nr), ("grid", nd + nr, got.size)]:
        err = np.abs(got[lo:hi] - ref[lo:hi]).max()
        sc = np.abs(ref[lo:hi]).max()
        assert err <= 2e-2 * sc + 1e-4, f"{name}: max err {err} vs scale {sc}"


def test_forward_then_backward_equals_fused(pkg, nerf_setup):
    net, tr, p16, m = nerf_setup
    n = 2000
    c = torch.from_numpy(coords_batch(n, seed=9)).cuda()
    dL = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    dL[:, :4] = torch.rand((n, 4), device="cuda").half() - 0.5
    net.forward_backward(c, dL)
    g1 = tr.gradients.clone()
    ctx, _ = net.forward(c)
    net.backward(ctx, dL)
    torch.cuda.synchronize()
    # the MLP part is deterministic (slab reduction); the grid part uses atomics (order may differ)
    nm = net.n_matrix_params
    assert torch.equal(g1[:nm], tr.gradients[:nm])
    assert torch.allclose(g1[nm:].float(), tr.gradients[nm:].float(), atol=3e-3)  # fp16 atomic order


def test_nerf_c2prime_l16(pkg, orc):
    cfg = pkg.nerf_config("C2p")
    cfg["encoding"]["log2_hashmap_size"] = 15
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"])
    p16 = random_params(tr, net, net.n_matrix_params, grid_scale=0.5)
    m = orc.make_nerf(L=16, F=2, log2T=15)
    n = 1500
    c = coords_batch(n, seed=21)
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = np.random.default_rng(2).uniform(-1, 1, (n, 4))
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    net.forward_backward(torch.from_numpy(c).cuda(), torch.from_numpy(dL).cuda(), output=out)
    torch.cuda.synchronize()
    ref_out = orc.nerf_forward(m, p16, c)
    assert np.abs(out.float().cpu().numpy() - ref_out).max() <= 1e-2 * np.abs(ref_out).max()
    ref = orc.nerf_backward(m, p16, c, dL.astype(np.float32))
    got = tr.gradients.float().cpu().numpy()
    nm = net.n_matrix_params
    assert np.abs(got[:nm] - ref[:nm]).max() <= 2e-2 * np.abs(ref[:nm]).max()
    assert np.abs(got[nm:] - ref[nm:]).max() <= 2e-2 * np.abs(ref[nm:]).max() + 1e-4


@pytest.mark.parametrize("D,hidden", [(2, 2), (3, 2), (3, 3)])
def test_network_with_input_encoding(pkg, orc, D, hidden):
    enc = enc_cfg(16, 2, 14)
    mlp = dict(MLP2, n_hidden_layers=hidden)
    net = pkg.NetworkWithInputEncoding(D, 3, enc, mlp)
    tr = pkg.Trainer(net, ADAM)
    p16 = random_params(tr, net, net.n_matrix_params, grid_scale=0.5)
    n = 1234
    x = np.random.default_rng(D).random((n, D), dtype=np.float32)
    g = orc.make_grid(D, 16, 2, 14)
    mm = orc.make_mlp(32, 64, hidden, 16)
    nm = orc.mlp_n_params(mm)
    e = orc.f16_bits_to_f32(orc.f32_to_f16_bits(orc.grid_forward(g, x, p16[nm:])))
    ref = orc.mlp_forward(mm, p16[:nm], e)
    got = net.inference(torch.from_numpy(x).cuda(), use_inference_params=False).float().cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-2 * np.abs(ref).max()
    dy = np.zeros((n, 16), np.float16)
    dy[:, :3] = np.random.default_rng(7).uniform(-1, 1, (n, 3))
    net.forward_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy).cuda())
    torch.cuda.synchronize()
    dW, dx = orc.mlp_backward(mm, p16[:nm], e, dy.astype(np.float32))
    gg = tr.gradients.float().cpu().numpy()
    assert np.abs(gg[:nm] - dW).max() <= 2e-2 * np.abs(dW).max()
    gref = orc.grid_backward(g, x, dx[:, :32])
    assert np.abs(gg[nm:] - gref).max() <= 2e-2 * np.abs(gref).max() + 1e-4


@pytest.mark.parametrize("D,L,F,width,hidden", [(2, 4, 2, 16, 2), (3, 16, 2, 32, 2), (2, 16, 2, 16, 1), (3, 4, 4, 32, 3),
                                                 (3, 8, 2, 16, 3)])
def test_fully_fused_mlp_widths(pkg, orc, D, L, F, width, hidden):
    """tcnn FullyFusedMLP widths 16 and 32 (BASELINE C1: 2D L=4 F=2 T=2^14 with a 2x16 MLP): forward and
    the parameter / encoding gradients against the oracle, same bars as the 64-wide network."""
    enc = enc_cfg(L, F, 14)
    mlp = dict(MLP2, n_neurons=width, n_hidden_layers=hidden)
    net = pkg.NetworkWithInputEncoding(D, 3, enc, mlp)
    tr = pkg.Trainer(net, ADAM)
    p16 = random_params(tr, net, net.n_matrix_params, grid_scale=0.5)
    n = 2345
    x = np.random.default_rng(D + width).random((n, D), dtype=np.float32)
    g = orc.make_grid(D, L, F, 14)
    ew = -(-L * F // 16) * 16
    mm = orc.make_mlp(ew, width, hidden, 16)
    nm = orc.mlp_n_params(mm)
    assert nm == net.n_matrix_params == width * ew + (hidden - 1) * width * width + 16 * width
    e = np.zeros((n, ew), np.float32)
    e[:, :L * F] = orc.f16_bits_to_f32(orc.f32_to_f16_bits(orc.grid_forward(g, x, p16[nm:])))
    ref = orc.mlp_forward(mm, p16[:nm], e)
    got = net.inference(torch.from_numpy(x).cuda(), use_inference_params=False).float().cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-2 * np.abs(ref).max()
    dy = np.zeros((n, 16), np.float16)
    dy[:, :3] = np.random.default_rng(7).uniform(-1, 1, (n, 3))
    net.forward_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy).cuda())
    torch.cuda.synchronize()
    dW, dx = orc.mlp_backward(mm, p16[:nm], e, dy.astype(np.float32))
    gg = tr.gradients.float().cpu().numpy()
    assert np.abs(gg[:nm] - dW).max() <= 2e-2 * np.abs(dW).max()
    gref = orc.grid_backward(g, x, dx[:, :L * F])
    assert np.abs(gg[nm:] - gref).max() <= 2e-2 * np.abs(gref).max() + 1e-4


def test_optimizer_matches_oracle(pkg, orc, nerf_setup):
    net, tr, p16, m = nerf_setup
    cfg = orc.AdamCfg(1e-2, 0.9, 0.99, 1e-15, 1e-6, 0.95, 20000, 10000, 0.33)
    n = net.n_params
    nm = net.n_matrix_params
    g = np.random.default_rng(1)
    grad = (g.standard_normal(n) * 10).astype(np.float16)
    grad[nm::5] = 0
    w32 = tr.params_full_precision.cpu().numpy().copy()
    step0 = tr.step
    w16 = orc.f32_to_f16_bits(w32)
    m1 = np.zeros(n, np.float32); m2 = np.zeros(n, np.float32); steps = np.zeros(n, np.uint32)
    e32 = np.zeros(n, np.float32); e16 = np.zeros(n, np.uint16)
    tr.gradients.copy_(torch.from_numpy(grad).cuda())
    tr.optimizer_step(128.0)
    torch.cuda.synchronize()
    orc.adam_step(cfg, step0, nm, 128.0, w32, w16, grad.view(np.uint16), m1, m2, steps, e32, e16)
    got = tr.params_full_precision.cpu().numpy()
    np.testing.assert_allclose(got, w32, rtol=1e-5, atol=1e-7)
    got_inf = tr.inference_params.float().cpu().numpy()
    np.testing.assert_allclose(got_inf, orc.f16_bits_to_f32(e16), rtol=2e-3, atol=1e-5)


def test_trainer_serialize_roundtrip(pkg, nerf_setup):
    net, tr, p16, m = nerf_setup
    blob = tr.serialize()
    before = tr.params_full_precision.clone()
    tr.params_full_precision.zero_()
    tr.deserialize(blob)
    torch.cuda.synchronize()
    assert torch.equal(before, tr.params_full_precision)


def test_zero_batch_and_errors(pkg, nerf_setup):
    net, tr, p16, m = nerf_setup
    x = torch.zeros((0, 7), dtype=torch.float32, device="cuda")
    out = net.inference(x)
    assert out.shape == (0, 16)
    with pytest.raises(pkg.NgpError):
        pkg.NerfNetwork(3, 3, 0, 4, {"otype": "Frequency"}, None, MLP2, MLP2)


def test_large_batch_properties(pkg, nerf_setup):
    """Full BASELINE batch (2^18): finite outputs; linearity of the gradient in dL/doutput."""
    net, tr, p16, m = nerf_setup
    n = 1 << 18
    c = torch.from_numpy(coords_batch(n, seed=77)).cuda()
    dL = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    dL[:, :4] = (torch.rand((n, 4), device="cuda") - 0.5).half() * 0.01
    out = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    net.forward_backward(c, dL, output=out)
    g1 = tr.gradients.float().clone()
    net.forward_backward(c, dL * 2, output=out)
    g2 = tr.gradients.float().clone()
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    nm = net.n_matrix_params
    assert torch.allclose(g2[:nm], 2 * g1[:nm], rtol=2e-3, atol=1e-3)
    # k_nerf_mlp_train lays out and sums each layer like the inference kernel: the same output bit for bit
    ref_out = net.inference(c, use_inference_params=False)
    torch.cuda.synchronize()
    assert torch.equal(ref_out, out)


@pytest.mark.parametrize("mode", [1, 3])
@pytest.mark.parametrize("D,L,F,T,n", [(3, 4, 4, 19, 20000), (3, 16, 2, 19, 12000), (2, 16, 2, 14, 9000), (3, 4, 8, 14, 8192),
                                       (3, 8, 1, 12, 6000)])
def test_encoding_backward_modes(pkg, orc, mode, D, L, F, T, n):
    """Destination-bucketed backward (mode 3): bit-exact with the oracle's exact-sum restatement. Direct
    tcnn-style packed-fp16 atomics (mode 1): every atomic rounds the running sum to fp16 in arrival
    order, so parameter e may move by up to k_e * 2^-11 * sum|w dL/dy| (k_e = its contribution count)
    from the exactly rounded sum, checked per element. Positions include the cube faces/edges and a few
    outside [0,1]."""
    net = pkg.NetworkWithInputEncoding(D, 1, enc_cfg(L, F, T), MLP2)
    tr = pkg.Trainer(net, ADAM)
    net.set_option("grid_backward_mode", mode)
    g = np.random.default_rng(n + mode)
    x = g.random((n, D), dtype=np.float32)
    x[:64] = np.round(x[:64] * 4) / 4           # exact bin boundaries
    x[64:72] = 1.0
    x[72:80] = np.float32(1.0 + 1e-3)           # outside the unit cube
    W = net.layout().encoding_width
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = g.uniform(-1, 1, (n, L * F))
    net.encoding_backward(torch.from_numpy(x).cuda(), torch.from_numpy(dy).cuda())
    torch.cuda.synchronize()
    got = tr.gradients.cpu().numpy()[net.n_matrix_params:]
    grid = orc.make_grid(D, L, F, T)
    ref, absum = orc.grid_backward_exact(grid, x, dy, with_abs_sum=True)
    if mode == 3:
        np.testing.assert_array_equal(got.view(np.uint16), ref)
        return
    idx = orc.grid_indices(grid, x).reshape(-1)
    k = np.repeat(np.bincount(idx, minlength=orc.grid_n_entries(grid)), F).astype(np.float64)
    err = np.abs(got.astype(np.float64) - orc.f16_bits_to_f32(ref))
    tol = k * 2.0 ** -11 * absum + 2.0 ** -24
    assert np.all(err <= tol), (float((err / tol).max()), int((err > tol).sum()))


@pytest.mark.parametrize("mode", [1, 3])
def test_encoding_backward_accumulate(pkg, orc, mode):
    """GRAD_ACCUMULATE adds to the existing grid gradient (tcnn accumulate semantics); overwrite replaces it."""
    D, L, F, T, n = 3, 8, 2, 16, 30000
    net = pkg.NetworkWithInputEncoding(D, 1, enc_cfg(L, F, T), MLP2)
    tr = pkg.Trainer(net, ADAM)
    net.set_option("grid_backward_mode", mode)
    g = np.random.default_rng(5)
    x = torch.from_numpy(g.random((n, D), dtype=np.float32)).cuda()
    W = net.layout().encoding_width
    dy = np.zeros((n, W), np.float16)
    dy[:, :L * F] = g.uniform(-1, 1, (n, L * F))
    dy = torch.from_numpy(dy).cuda()
    nm = net.n_matrix_params
    tr.gradients[nm:] = 5.0  # stale values must be overwritten
    net.encoding_backward(x, dy)
    g1 = tr.gradients[nm:].clone()
    net.encoding_backward(x, dy, grad_mode=pkg.GRAD_ACCUMULATE)
    g2 = tr.gradients[nm:].clone()
    torch.cuda.synchronize()
    grid = orc.make_grid(D, L, F, T)
    xs, dys = x.cpu().numpy(), dy.cpu().numpy()
    ref1 = orc.grid_backward_exact(grid, xs, dys)
    if mode == 3:  # exact: overwrite, then old + exact sum rounded once
        np.testing.assert_array_equal(g1.cpu().numpy().view(np.uint16), ref1)
        np.testing.assert_array_equal(g2.cpu().numpy().view(np.uint16), orc.grid_backward_exact(grid, xs, dys, grad16=ref1))
        return
    ref = orc.grid_backward(grid, xs, dys[:, :L * F].astype(np.float32))
    scale = np.abs(ref).max()
    tol = 3e-2 * scale + 1e-3  # fp16 atomics in arrival order (tcnn's half2 atomicAdd)
    assert np.abs(g1.float().cpu().numpy() - ref).max() <= tol
    assert np.abs(g2.float().cpu().numpy() - 2 * ref).max() <= 2 * tol


def test_training_graph_matches_eager(pkg):
    """A captured training step (forward_backward + optimizer, one HIP graph) replays the eager steps:
    same learning-rate/EMA schedule from the device-side step counter, bit-identical parameters. At
    n = 2^13 no bucket of the grid backward is split, so the whole step is deterministic (exact integer
    sums, fixed-order MLP reductions); larger batches add fp16 atomics of partial sums on coarse levels."""
    cfg = pkg.nerf_config("C2")
    n = 1 << 13
    x = torch.from_numpy(coords_batch(n, 9)).cuda()
    dL = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    dL[:, :4] = (torch.rand((n, 4), device="cuda") - 0.5) * 0.02
    runs = []
    for use_graph in (False, True):
        net = pkg.create_nerf_network(cfg)
        tr = pkg.Trainer(net, cfg["optimizer"], seed=7)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            net.forward_backward(x, dL)  # first step eager in both runs (allocations)
            tr.optimizer_step(128.0)
            if use_graph:
                g = tr.capture_training_step(x, dL, 128.0, n_steps=2)
                for _ in range(2):
                    g.launch()
            else:
                for _ in range(4):
                    net.forward_backward(x, dL)
                    tr.optimizer_step(128.0)
        s.synchronize()
        assert tr.step == 5
        runs.append((tr.params_full_precision.cpu().numpy().copy(), tr.inference_params.float().cpu().numpy().copy()))
    np.testing.assert_array_equal(runs[1][0], runs[0][0])
    np.testing.assert_array_equal(runs[1][1], runs[0][1])


@pytest.mark.parametrize("grad_accumulate", [False, True])
def test_fused_slab_reduction_matches_separate(pkg, nerf_setup, grad_accumulate):
    """The MLP dW slab reduction run inside the grid backward's last kernel (option fuse_slabs, on by
    default) writes the same gradients bit for bit as the separate k_reduce_slabs launch, overwriting
    and accumulating (tcnn's GradientMode::Accumulate)."""
    net, tr, p16, m = nerf_setup
    n = 50000
    c = torch.from_numpy(coords_batch(n, seed=123)).cuda()
    dL = torch.zeros((n, 16), dtype=torch.float16, device="cuda")
    dL[:, :4] = torch.rand((n, 4), device="cuda").half() - 0.5
    res = {}
    for fuse in (1, 0):
        net.set_option("fuse_slabs", fuse)
        net.forward_backward(c, dL)
        if grad_accumulate:
            net.forward_backward(c, dL, grad_mode=pkg.GRAD_ACCUMULATE)
        torch.cuda.synchronize()
        res[fuse] = tr.gradients.clone()
    net.set_option("fuse_slabs", 1)
    assert torch.equal(res[1], res[0])
    assert res[1][: net.n_matrix_params].abs().sum() > 0
