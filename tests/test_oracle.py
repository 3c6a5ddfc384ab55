"""CPU tests pinning the oracle (oracle/ngp_oracle.c) before it is trusted as the checker.

- pcg32 against the published PCG known-answer vector (tests/golden/pcg32_kat.json);
- fp16 conversion against numpy's IEEE binary16 (all 65536 patterns + random floats);
- hash-grid forward/backward, MLP forward/backward and the NerfNetwork composition against an
  independent PyTorch (CPU, float64 autograd) restatement. That cross-check is independent of the
  oracle's code, not of tiny-cuda-nn (absent: parity unpinned).
"""
import json
import os

import numpy as np
import pytest
import torch

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_pcg32_kat(orc):
    kat = json.load(open(os.path.join(GOLDEN, "pcg32_kat.json")))
    r = orc.Rng(kat["initstate"], kat["initseq"])
    assert [r.next_uint() for _ in range(len(kat["outputs"]))] == [int(x, 16) for x in kat["outputs"]]


def test_pcg32_advance_matches_stepping(orc):
    a = orc.Rng(1337)
    b = orc.Rng(1337)
    for _ in range(1000):
        a.next_uint()
    b.advance(1000)
    assert a.next_uint() == b.next_uint()
    # negative advance (two's complement) goes back
    b.advance(-1)
    c = orc.Rng(1337)
    c.advance(1000)
    assert b.next_uint() == c.next_uint()


def test_pcg32_next_float_range(orc):
    r = orc.Rng(7)
    v = np.array([r.next_float() for _ in range(10000)])
    assert v.min() >= 0.0 and v.max() < 1.0
    assert abs(v.mean() - 0.5) < 0.02


def test_f16_roundtrip_all_patterns(orc):
    bits = np.arange(65536, dtype=np.uint16)
    ref = bits.view(np.float16).astype(np.float32)
    got = orc.f16_bits_to_f32(bits)
    finite = np.isfinite(ref)
    assert np.array_equal(got[finite].view(np.uint32), ref[finite].view(np.uint32))
    assert np.all(np.isnan(got[np.isnan(ref)]))


def test_f32_to_f16_matches_numpy(orc):
    rng = np.random.default_rng(0)
    x = np.concatenate([
        rng.standard_normal(200000).astype(np.float32) * np.float32(10.0) ** rng.integers(-9, 6, 200000).astype(np.float32),
        np.array([0.0, -0.0, 65504.0, 65519.0, 65520.0, 1e-8, 2.0 ** -25, 2.0 ** -24, 3 * 2.0 ** -26, 6.1e-5], np.float32),
    ])
    got = orc.f32_to_f16_bits(x)
    with np.errstate(over="ignore"):
        ref = x.astype(np.float16).view(np.uint16)
    assert np.array_equal(got, ref)


def test_grid_offsets_match_survey(orc):
    # SURVEY §8 parameter table (tcnn offset-table rules)
    assert orc.grid_n_entries(orc.make_grid(3, 4, 4, 19)) == 823296
    assert orc.grid_n_entries(orc.make_grid(3, 16, 2, 19)) == 7114752
    assert orc.grid_n_entries(orc.make_grid(3, 16, 2, 22)) == 52727808
    assert orc.grid_n_entries(orc.make_grid(2, 4, 2, 14)) == 21760


def test_nerf_param_count_matches_survey(orc):
    assert orc.nerf_n_params(orc.make_nerf()) == 3302400
    assert orc.nerf_n_params(orc.make_nerf(L=16, F=2)) == 14239744


# ------------------------------------------------------------------------------------------------
# Independent torch restatement of the hash grid (float64), for forward + autograd backward
# ------------------------------------------------------------------------------------------------
PRIMES = [1, 2654435761, 805459861]


def torch_grid(g, pos, table):
    """pos: (n, D) float32; table: (entries, F) float64 tensor requiring grad. Returns (n, L*F)."""
    n, D = pos.shape
    outs = []
    for l in range(g.n_levels):
        scale = np.float32(g.scale[l])
        res = int(g.resolution[l])
        T = int(g.offsets[l + 1] - g.offsets[l])
        p = np.float32(scale) * pos.astype(np.float32) + np.float32(0.5)  # fmaf may differ by 1ulp: use float64 check below
        p = (pos.astype(np.float64) * np.float64(scale) + 0.5).astype(np.float32)
        base = np.floor(p)
        frac = (p - base).astype(np.float32)
        base = base.astype(np.int64).astype(np.uint64)
        acc = 0
        for c in range(1 << D):
            w = np.ones(n, np.float32)
            pc = []
            for d in range(D):
                if c & (1 << d):
                    w = w * frac[:, d]
                    pc.append(base[:, d] + 1)
                else:
                    w = w * (np.float32(1) - frac[:, d])
                    pc.append(base[:, d])
            # index
            stride = 1
            index = np.zeros(n, np.uint64)
            dense = True
            for d in range(D):
                if stride > T:
                    break
                index = (index + pc[d] * np.uint64(stride)) & np.uint64(0xFFFFFFFF)
                stride *= res
            if T < stride:
                index = np.zeros(n, np.uint64)
                for d in range(D):
                    index ^= (pc[d] * np.uint64(PRIMES[d])) & np.uint64(0xFFFFFFFF)
            index = (index % np.uint64(T)).astype(np.int64) + int(g.offsets[l])
            acc = acc + torch.from_numpy(w.astype(np.float64))[:, None] * table[torch.from_numpy(index)]
        outs.append(acc)
    return torch.cat(outs, dim=1)


@pytest.mark.parametrize("D,L,F,log2T", [(3, 4, 4, 19), (3, 16, 2, 14), (2, 4, 2, 14), (3, 8, 1, 12), (3, 6, 8, 10)])
def test_grid_forward_backward_vs_torch(orc, D, L, F, log2T):
    g = orc.make_grid(D, L, F, log2T)
    rng = np.random.default_rng(D * 100 + L)
    n = 512
    pos = rng.random((n, D), dtype=np.float32)
    pos[:4] = np.array([0.0, 1.0, 0.5, 0.999999], np.float32)[:, None]  # edges: wraparound in dense levels
    E = orc.grid_n_entries(g)
    table32 = (rng.random(E * F, dtype=np.float32) * 2 - 1).astype(np.float16).astype(np.float32)
    table16 = table32.astype(np.float16).view(np.uint16)
    out = orc.grid_forward(g, pos, table16)
    t = torch.from_numpy(table32.astype(np.float64).reshape(E, F)).requires_grad_(True)
    ref = torch_grid(g, pos, t)
    np.testing.assert_allclose(out, ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    # indices are integers: the oracle's hashing must agree bit-exactly with the restatement above
    dy = rng.standard_normal((n, L * F)).astype(np.float32)
    ref.backward(torch.from_numpy(dy.astype(np.float64)))
    grad = orc.grid_backward(g, pos, dy)
    np.testing.assert_allclose(grad, t.grad.numpy().reshape(-1), rtol=1e-5, atol=1e-6)


def test_grid_max_level_zeroes_levels(orc):
    g = orc.make_grid(3, 8, 2, 14)
    rng = np.random.default_rng(1)
    pos = rng.random((64, 3), dtype=np.float32)
    E = orc.grid_n_entries(g)
    table16 = (rng.random(E * 2, dtype=np.float32) - 0.5).astype(np.float16).view(np.uint16)
    full = orc.grid_forward(g, pos, table16, 1.0)
    half = orc.grid_forward(g, pos, table16, 0.5)  # tcnn: level >= 0.5*8 + 1e-3 zeroed -> levels 5..7
    np.testing.assert_array_equal(half[:, :10], full[:, :10])
    assert np.all(half[:, 10:] == 0)


def test_sh4_orthonormal(orc):
    # Monte-Carlo orthonormality of the 16 real SH basis functions over the sphere
    rng = np.random.default_rng(3)
    d = rng.standard_normal((20000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    Y = np.stack([orc.sh4((v + 1) / 2) for v in d])
    G = Y.T @ Y / len(d) * 4 * np.pi
    np.testing.assert_allclose(G, np.eye(16), atol=0.06)


# ------------------------------------------------------------------------------------------------
# MLP vs torch float64 (tolerance covers the oracle's per-layer fp16 rounding)
# ------------------------------------------------------------------------------------------------
def torch_mlp(m, w, x):
    h = x
    off = 0
    nl = m.n_hidden + 1
    for l in range(nl):
        i = m.in_pad if l == 0 else m.width
        o = m.out_pad if l == nl - 1 else m.width
        W = w[off:off + i * o].view(o, i)
        off += i * o
        h = (h @ W.T).half().double()  # fp16 activations (cast is straight-through for grads)
        if l < nl - 1:
            h = torch.relu(h)
    return h


@pytest.mark.parametrize("in_pad,width,n_hidden,out_pad", [(16, 64, 1, 16), (32, 64, 2, 16), (32, 64, 3, 16), (16, 16, 2, 16)])
def test_mlp_vs_torch(orc, in_pad, width, n_hidden, out_pad):
    m = orc.make_mlp(in_pad, width, n_hidden, out_pad)
    npar = orc.mlp_n_params(m)
    rng = orc.Rng(11)
    w32 = np.zeros(npar, np.float32)
    orc.lib().orc_mlp_init(orc.C.byref(m), orc.C.byref(rng.s), orc.ptr(w32))
    w16 = orc.f32_to_f16_bits(w32)
    wq = orc.f16_bits_to_f32(w16)
    r = np.random.default_rng(5)
    x = orc.f16_bits_to_f32(orc.f32_to_f16_bits(r.standard_normal((256, in_pad)).astype(np.float32)))
    y = orc.mlp_forward(m, w16, x)
    wt = torch.from_numpy(wq.astype(np.float64)).requires_grad_(True)
    xt = torch.from_numpy(x.astype(np.float64)).requires_grad_(True)
    yt = torch_mlp(m, wt, xt)
    scale = np.abs(yt.detach().numpy()).max()
    np.testing.assert_allclose(y, yt.detach().numpy(), atol=2e-3 * scale)
    dy = orc.f16_bits_to_f32(orc.f32_to_f16_bits(r.standard_normal((256, out_pad)).astype(np.float32)))
    dW, dx = orc.mlp_backward(m, w16, x, dy)
    yt.backward(torch.from_numpy(dy.astype(np.float64)))
    gW = wt.grad.numpy()
    np.testing.assert_allclose(dW, gW, atol=1e-2 * np.abs(gW).max())
    gx = xt.grad.numpy()
    np.testing.assert_allclose(dx, gx, atol=1e-2 * np.abs(gx).max())


def test_nerf_composition_vs_torch(orc):
    """NerfNetwork fwd/bwd (nerf_network.h:116-335) vs torch restatement of the same composition."""
    m = orc.make_nerf(L=4, F=4, log2T=12)
    p32 = orc.nerf_init(m, 1337)
    # make the grid larger so the encoding matters
    nd, nr = orc.mlp_n_params(m.density), orc.mlp_n_params(m.rgb)
    r = np.random.default_rng(9)
    p32[nd + nr:] = r.uniform(-1, 1, p32.size - nd - nr).astype(np.float32)
    p16 = orc.f32_to_f16_bits(p32)
    pq = orc.f16_bits_to_f32(p16).astype(np.float64)
    n = 128
    coords = np.zeros((n, 7), np.float32)
    coords[:, :3] = r.random((n, 3))
    coords[:, 3] = 0.01
    d = r.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    coords[:, 4:7] = (d + 1) / 2
    out = orc.nerf_forward(m, p16, coords)

    pt = torch.from_numpy(pq).requires_grad_(True)
    E = orc.grid_n_entries(m.grid)
    table = pt[nd + nr:].view(E, 4)
    enc = torch_grid(m.grid, coords[:, :3], table)
    dout = torch_mlp(m.density, pt[:nd], enc)
    sh = torch.from_numpy(np.stack([orc.sh4(c[4:7]) for c in coords]).astype(np.float64))
    rout = torch_mlp(m.rgb, pt[nd:nd + nr], torch.cat([dout, sh], 1))
    ref = torch.cat([rout[:, :3], dout[:, :1], rout[:, 4:]], 1)
    sc = np.abs(ref.detach().numpy()).max()
    np.testing.assert_allclose(out, ref.detach().numpy(), atol=5e-3 * sc)

    dL = np.zeros((n, 16), np.float32)
    dL[:, :4] = orc.f16_bits_to_f32(orc.f32_to_f16_bits(r.standard_normal((n, 4)).astype(np.float32)))
    grads = orc.nerf_backward(m, p16, coords, dL)
    ref.backward(torch.from_numpy(dL.astype(np.float64)))
    g = pt.grad.numpy()
    for lo, hi in [(0, nd), (nd, nd + nr), (nd + nr, g.size)]:
        np.testing.assert_allclose(grads[lo:hi], g[lo:hi], atol=2e-2 * np.abs(g[lo:hi]).max())


def test_adam_matches_numpy(orc):
    cfg = orc.AdamCfg(1e-2, 0.9, 0.99, 1e-15, 1e-6, 0.95, 20000, 10000, 0.33)
    n, nm = 1000, 300
    r = np.random.default_rng(2)
    w32 = r.standard_normal(n).astype(np.float32)
    w16 = orc.f32_to_f16_bits(w32)
    m1 = np.zeros(n, np.float32); m2 = np.zeros(n, np.float32); steps = np.zeros(n, np.uint32)
    ema32 = np.zeros(n, np.float32); ema16 = np.zeros(n, np.uint16)
    g = r.standard_normal(n).astype(np.float32) * 128
    g[nm::7] = 0  # lazily skipped non-matrix params
    g16 = orc.f32_to_f16_bits(g)
    w0 = w32.copy()
    orc.adam_step(cfg, 0, nm, 128.0, w32, w16, g16, m1, m2, steps, ema32, ema16)
    gr = orc.f16_bits_to_f32(g16) / 128
    gr[:nm] += 1e-6 * w0[:nm]
    mm = 0.1 * gr
    vv = 0.01 * gr * gr
    lr = 1e-2 * np.sqrt(1 - 0.99) / (1 - 0.9)
    exp = w0 - lr / (np.sqrt(vv) + 1e-15) * mm
    skip = np.zeros(n, bool); skip[nm::7] = True
    np.testing.assert_allclose(w32[~skip], exp[~skip], rtol=1e-5)
    np.testing.assert_array_equal(w32[skip], w0[skip])
    assert np.all(steps[~skip] == 1) and np.all(steps[skip] == 0)
    # EMA debiased after one step equals the weights
    np.testing.assert_allclose(orc.f16_bits_to_f32(ema16), w32, rtol=1e-3, atol=1e-4)


def test_lr_schedule(orc):
    cfg = orc.AdamCfg(1e-2, 0.9, 0.99, 1e-15, 1e-6, 0.95, 20000, 10000, 0.33)
    assert orc.lib().orc_lr_at_step(orc.C.byref(cfg), 0) == pytest.approx(1e-2)
    assert orc.lib().orc_lr_at_step(orc.C.byref(cfg), 19999) == pytest.approx(1e-2)
    assert orc.lib().orc_lr_at_step(orc.C.byref(cfg), 20000) == pytest.approx(3.3e-3)
    assert orc.lib().orc_lr_at_step(orc.C.byref(cfg), 30000) == pytest.approx(3.3e-3 * 0.33)


def test_morton_and_srgb(orc):
    # x in bit 0: morton3D_invert(i) / (i >> 1) / (i >> 2) recovers x / y / z (testbed_nerf.cu:518-520)
    assert orc.lib().orc_morton3D(1, 0, 0) == 1
    assert orc.lib().orc_morton3D(0, 1, 0) == 2
    assert orc.lib().orc_morton3D(0, 0, 1) == 4
    assert orc.lib().orc_morton3D(127, 127, 127) == 128 ** 3 - 1
    inv = orc.lib().orc_morton3D_invert
    for x, y, z in [(3, 77, 120), (127, 0, 64), (5, 5, 5)]:
        i = orc.lib().orc_morton3D(x, y, z)
        assert (inv(i), inv(i >> 1), inv(i >> 2)) == (x, y, z)
    for v in [0.0, 0.01, 0.04045, 0.5, 1.0]:
        assert orc.lib().orc_linear_to_srgb(orc.lib().orc_srgb_to_linear(v)) == pytest.approx(v, abs=1e-3)


def test_shared_math_accuracy(orc):
    """ngp_math.h (the one expf/logf both the engine kernels and the oracle evaluate, so cone stepping
    and compaction are bit-exact) is within 1 ulp of float64 over the ranges the NeRF path uses and
    over random positive bit patterns; special values follow IEEE."""
    g = np.random.default_rng(0)

    def ulps(y, ref):
        sp = np.abs(np.spacing(ref.astype(np.float32))).astype(np.float64)
        return np.abs(y.astype(np.float64) - ref) / sp

    x = np.concatenate([g.uniform(-87.0, 88.7, 1 << 20), g.uniform(-15, 15, 1 << 20)]).astype(np.float32)
    assert ulps(orc.math_eval(0, x), np.exp(x.astype(np.float64))).max() <= 1.0
    bits = g.integers(0x00800000, 0x7f800000, 1 << 21, dtype=np.uint32)
    x = np.concatenate([bits.view(np.float32), np.float32(1) + g.uniform(-0.3, 0.4, 1 << 20).astype(np.float32)])
    assert ulps(orc.math_eval(1, x), np.log(x.astype(np.float64))).max() <= 1.0
    sub = orc.math_eval(0, np.array([-100.0, -103.0], np.float32))
    assert np.all(np.abs(sub.astype(np.float64) - np.exp([-100.0, -103.0])) <= 1.5e-45)
    sp = orc.math_eval(0, np.array([0, -200, 200, np.nan], np.float32))
    assert sp[0] == 1 and sp[1] == 0 and np.isinf(sp[2]) and np.isnan(sp[3])
    sp = orc.math_eval(1, np.array([0, -1, np.inf, np.nan, 1, 1e-40], np.float32))
    assert np.isneginf(sp[0]) and np.isnan(sp[1]) and np.isinf(sp[2]) and np.isnan(sp[3]) and sp[4] == 0
    assert abs(sp[5] - np.log(1e-40)) < 1e-5 * abs(np.log(1e-40))


def test_shared_math_fast_variants_equal_full(orc):
    """The kernels call ngp_math.h's unchecked cores where the argument is bounded (stepping-space
    segments, clamped activations) and a fast path for |x| <= 80 elsewhere: each returns the same bits
    as the full function on its domain, and the stepping-space division by log(1 + 1/256) equals IEEE
    division (tools/microbench/div_check.c checks it exhaustively)."""
    g = np.random.default_rng(5)
    x = np.concatenate([g.uniform(-80, 80, 1 << 20), g.uniform(-15, 15, 1 << 18)]).astype(np.float32)
    assert np.array_equal(orc.math_eval(2, x).view(np.uint32), orc.math_eval(0, x).view(np.uint32))
    bits = g.integers(0x00800000, 0x7f800000, 1 << 20, dtype=np.uint32)
    x = np.concatenate([bits.view(np.float32), g.uniform(0.4, 60, 1 << 18).astype(np.float32)])
    assert np.array_equal(orc.math_eval(3, x).view(np.uint32), orc.math_eval(1, x).view(np.uint32))
    x = np.concatenate([g.uniform(-200, 200, 1 << 20).astype(np.float32),
                        np.array([np.nan, np.inf, -np.inf, 80.0, -80.0, 88.7, -103.9, -120.0], np.float32)])
    assert np.array_equal(orc.math_eval(4, x).view(np.uint32), orc.math_eval(0, x).view(np.uint32))
    x = np.concatenate([g.uniform(-2, 5, 1 << 20), g.uniform(-1e3, 1e3, 1 << 18)]).astype(np.float32)
    l = np.float32(orc.math_eval(1, np.array([1 + 1 / 256], np.float32))[0])
    assert np.array_equal(orc.math_eval(5, x), (x / l).astype(np.float32))


def test_grid_backward_exact_vs_double(orc):
    """The contribution-exact backward (per-contribution fp16 rounding, exact sum, one rounding) agrees
    with the float64 backward within the per-contribution rounding it adds: <= sum of half an fp16 ulp
    per contribution + half an ulp of the result."""
    D, L, F, T, n = 3, 4, 2, 12, 4000
    g = orc.make_grid(D, L, F, T)
    rng = np.random.default_rng(2)
    x = rng.random((n, D), dtype=np.float32)
    dy = rng.uniform(-1, 1, (n, L * F)).astype(np.float16)
    exact, absum = orc.grid_backward_exact(g, x, dy, with_abs_sum=True)
    ref = orc.grid_backward(g, x, dy.astype(np.float32))
    got = exact.view(np.float16).astype(np.float64)
    tol = absum * 2.0 ** -11 + np.abs(ref) * 2.0 ** -11 + 2.0 ** -24
    assert np.all(np.abs(got - ref) <= tol)
    # accumulate: old + sum
    init = rng.uniform(-1, 1, exact.size).astype(np.float16).view(np.uint16)
    acc = orc.grid_backward_exact(g, x, dy, grad16=init)
    want = (init.view(np.float16).astype(np.float64) + ref)
    assert np.all(np.abs(acc.view(np.float16).astype(np.float64) - want) <= tol + np.abs(want) * 2.0 ** -10)


def test_nerf_train_ex_matches_serial(orc):
    """The parallel full-batch oracle pass equals the serial restatement: outputs, MLP gradients (up
    to float64 summation order), dL/d(encoding); its grid gradient (exact contract) stays within the
    per-contribution fp16 rounding of the float64 grid gradient."""
    m = orc.make_nerf(L=4, F=4, log2T=12)
    p = orc.nerf_init(m, 7)
    p16 = orc.f32_to_f16_bits(p)
    n = 600
    g = np.random.default_rng(0)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 4:] = g.random((n, 3))
    dL = np.zeros((n, 16), np.float32)
    dL[:, :4] = g.uniform(-1, 1, (n, 4)).astype(np.float16)
    r = orc.nerf_train_ex(m, p16, c, dL)
    np.testing.assert_array_equal(r["out"], orc.nerf_forward(m, p16, c))
    ref, denc = orc.nerf_backward(m, p16, c, dL, want_denc=True)
    nm = r["grads"].size
    np.testing.assert_allclose(r["grads"], ref[:nm], rtol=1e-12, atol=1e-15)
    np.testing.assert_array_equal(orc.f16_bits_to_f32(r["denc16"]), denc)
    assert np.all(r["grads_abs"] >= np.abs(r["grads"]) * (1 - 1e-12))
    assert np.all(r["out_abs"][:, :4] >= np.abs(r["out"][:, :4]) * (1 - 1e-6))
    gx, absum = orc.grid_backward_exact(m.grid, c[:, :3].copy(), r["denc16"], stride=3, with_abs_sum=True)
    tol = absum * 2.0 ** -11 + np.abs(ref[nm:]) * 2.0 ** -11 + 2.0 ** -24
    assert np.all(np.abs(orc.f16_bits_to_f32(gx) - ref[nm:]) <= tol)


# ------------------------------------------------------------------------------------------------
# Input gradients (orc_grid_input_grad, orc_sh4_input_grad) vs torch float64 autograd
# ------------------------------------------------------------------------------------------------
def torch_grid_pos(g, pos, table, max_level=1.0):
    """The grid forward as a function of the positions (float64 autograd through the trilinear weights;
    corner indices fixed by the float32 floor, as the forward's). pos: (n, D) float32."""
    n, D = pos.shape
    x = torch.from_numpy(pos.astype(np.float64)).requires_grad_(True)
    outs = []
    for l in range(g.n_levels):
        if l >= max_level * g.n_levels + 1e-3:
            outs.append(torch.zeros((n, g.n_features), dtype=torch.float64))
            continue
        scale = float(np.float32(g.scale[l]))
        res = int(g.resolution[l])
        T = int(g.offsets[l + 1] - g.offsets[l])
        # the forward's float32 fractions as values (fmaf: one rounding), d frac / dx = scale as derivative
        p32 = (pos.astype(np.float64) * scale + 0.5).astype(np.float32)
        base = np.floor(p32)
        frac32 = torch.from_numpy((p32 - base).astype(np.float64))
        frac = frac32 + (x - x.detach()) * scale
        base = base.astype(np.int64).astype(np.uint64)
        acc = 0
        for c in range(1 << D):
            w = torch.ones(n, dtype=torch.float64)
            pc = []
            for d in range(D):
                if c & (1 << d):
                    w = w * frac[:, d]
                    pc.append(base[:, d] + 1)
                else:
                    w = w * (1 - frac[:, d])
                    pc.append(base[:, d])
            stride, index = 1, np.zeros(n, np.uint64)
            for d in range(D):
                if stride > T:
                    break
                index = (index + pc[d] * np.uint64(stride)) & np.uint64(0xFFFFFFFF)
                stride *= res
            if T < stride:
                index = np.zeros(n, np.uint64)
                for d in range(D):
                    index ^= (pc[d] * np.uint64(PRIMES[d])) & np.uint64(0xFFFFFFFF)
            index = (index % np.uint64(T)).astype(np.int64) + int(g.offsets[l])
            acc = acc + w[:, None] * table[torch.from_numpy(index)]
        outs.append(acc)
    return x, torch.cat(outs, dim=1)


@pytest.mark.parametrize("D,L,F,log2T,max_level", [(3, 4, 4, 19, 1.0), (3, 16, 2, 14, 1.0), (2, 4, 2, 14, 1.0),
                                                   (3, 8, 1, 12, 0.6), (3, 6, 8, 10, 1.0)])
def test_grid_input_grad_vs_torch(orc, D, L, F, log2T, max_level):
    g = orc.make_grid(D, L, F, log2T)
    rng = np.random.default_rng(7 * D + L)
    n = 256
    pos = rng.random((n, D), dtype=np.float32)
    E = orc.grid_n_entries(g)
    table32 = (rng.random(E * F, dtype=np.float32) * 2 - 1).astype(np.float16).astype(np.float32)
    table16 = table32.astype(np.float16).view(np.uint16)
    dy = rng.standard_normal((n, L * F)).astype(np.float32)
    got = orc.grid_input_grad(g, pos, table16, dy, max_level)
    x, y = torch_grid_pos(g, pos, torch.from_numpy(table32.astype(np.float64).reshape(E, F)), max_level)
    y.backward(torch.from_numpy(dy.astype(np.float64)))
    ref = x.grad.numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-12 * np.abs(ref).max())


def torch_sh4(d):
    x, y, z = d[:, 0] * 2 - 1, d[:, 1] * 2 - 1, d[:, 2] * 2 - 1
    xy, xz, yz, x2, y2, z2 = x * y, x * z, y * z, x * x, y * y, z * z
    return torch.stack([
        torch.full_like(x, 0.28209479177387814), -0.48860251190291987 * y, 0.48860251190291987 * z,
        -0.48860251190291987 * x, 1.0925484305920792 * xy, -1.0925484305920792 * yz,
        0.94617469575755997 * z2 - 0.31539156525251999, -1.0925484305920792 * xz,
        0.54627421529603959 * x2 - 0.54627421529603959 * y2, 0.59004358992664352 * y * (-3.0 * x2 + y2),
        2.8906114426405538 * xy * z, 0.45704579946446572 * y * (1.0 - 5.0 * z2), 0.3731763325901154 * z * (5.0 * z2 - 3.0),
        0.45704579946446572 * x * (1.0 - 5.0 * z2), 1.4453057213202769 * z * (x2 - y2),
        0.59004358992664352 * x * (-x2 + 3.0 * y2)], dim=1)


def test_sh4_matches_torch_and_input_grad(orc):
    rng = np.random.default_rng(11)
    n = 200
    d = rng.standard_normal((n, 3))
    d = ((d / np.linalg.norm(d, axis=1, keepdims=True)) + 1) / 2
    d32 = d.astype(np.float32)
    dt = torch.from_numpy(d32.astype(np.float64)).requires_grad_(True)
    sh = torch_sh4(dt)
    np.testing.assert_allclose(np.stack([orc.sh4(v) for v in d32]), sh.detach().numpy(), rtol=1e-5, atol=1e-6)
    g = rng.standard_normal((n, 16)).astype(np.float32)
    sh.backward(torch.from_numpy(g.astype(np.float64)))
    got = np.stack([orc.sh4_input_grad(d32[i], g[i]) for i in range(n)])
    np.testing.assert_allclose(got, dt.grad.numpy(), rtol=1e-9, atol=1e-9)


def test_nerf_input_grad_vs_torch(orc):
    """The NerfNetwork input gradient (nerf_network.h:256-335 with dL_dinput) vs torch autograd of the
    composition w.r.t. positions and directions (float64; the oracle rounds intermediates to fp16)."""
    m = orc.make_nerf(L=4, F=4, log2T=12)
    p32 = orc.nerf_init(m, 5)
    rng = np.random.default_rng(5)
    p32[orc.mlp_n_params(m.density) + orc.mlp_n_params(m.rgb):] = rng.uniform(-0.5, 0.5, orc.grid_n_entries(m.grid) * 4)
    p16 = orc.f32_to_f16_bits(p32)
    pq = orc.f16_bits_to_f32(p16).astype(np.float64)
    n = 128
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = rng.random((n, 3))
    c[:, 3] = 0.01
    dd = rng.standard_normal((n, 3))
    c[:, 4:] = (dd / np.linalg.norm(dd, axis=1, keepdims=True) + 1) / 2
    dL = np.zeros((n, 16), np.float32)
    dL[:, :4] = rng.uniform(-1, 1, (n, 4)).astype(np.float16)
    r = orc.nerf_input_grad(m, p16, c, dL)
    nd, nr = orc.mlp_n_params(m.density), orc.mlp_n_params(m.rgb)
    table = torch.from_numpy(pq[nd + nr:].reshape(-1, 4))
    x, enc = torch_grid_pos(m.grid, c[:, :3], table)
    enc = torch.cat([enc.half().double(), torch.zeros((n, m.density.in_pad - enc.shape[1]), dtype=torch.float64)], 1)
    dout = torch_mlp(m.density, torch.from_numpy(pq[:nd]), enc)
    dt = torch.from_numpy(c[:, 4:].astype(np.float64)).requires_grad_(True)
    rout = torch_mlp(m.rgb, torch.from_numpy(pq[nd:nd + nr]), torch.cat([dout, torch_sh4(dt)], 1))
    out = torch.cat([rout[:, :3], dout[:, :1]], 1)
    out.backward(torch.from_numpy(dL[:, :4].astype(np.float64)))
    # samples with a hidden pre-activation within 1e-4 (relative) of a ReLU switch are excluded: the torch
    # encoding (float64, rounded once) can differ from the oracle's fp32 blend by one fp16 ulp and flip it
    keep = orc.nerf_train_ex(m, p16, c, dL)["margin"] > 1e-4
    assert keep.mean() > 0.5
    for got, ref in ((r["dinput"][:, :3], x.grad.numpy()), (r["dinput"][:, 4:], dt.grad.numpy())):
        # the oracle rounds activations and back-propagated gradients to fp16 (the kernel's contract)
        np.testing.assert_allclose(got[keep], ref[keep], rtol=2e-2, atol=2e-2 * np.abs(ref).max())
