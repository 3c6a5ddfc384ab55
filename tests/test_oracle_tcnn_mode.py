"""CPU tests pinning the oracle's tcnn mode (oracle/ngp_tcnn_mode.c) before the GPU test bounds the engine with it.

The tcnn mode restates tiny-cuda-nn's fp16 arithmetic (tcnn is absent from the reference: parity unpinned, SURVEY
§8c): half FMA chains in the grid blend, fp16 WMMA accumulators in the MLP, fp16 atomics in the grid backward.
Here each piece is checked against an independent numpy restatement of the same arithmetic (numpy rounds float64 to
float16 directly, correctly rounded, so the numpy side has no double rounding), and its stated rounding-error bounds
against float64 sums."""
import numpy as np
import pytest


def _pos(n, D, seed):
    g = np.random.default_rng(seed)
    x = g.random((n, D), dtype=np.float32)
    x[:8] = np.round(x[:8] * 4) / 4  # cell corners
    return x


def _np_corners(g, l, x):
    """numpy restatement of the corner setup and hash (tcnn grid_index with primes 1, 2654435761, 805459861)."""
    D = g.n_dims
    p = np.fma(np.float32(g.scale[l]), x.astype(np.float32), np.float32(0.5)) if hasattr(np, "fma") else None
    if p is None:
        p = (np.float64(g.scale[l]) * x.astype(np.float64) + 0.5).astype(np.float32)  # fma: one rounding
    t = np.floor(p)
    base = t.astype(np.int64).astype(np.uint32)
    frac = (p - t).astype(np.float32)
    T = g.offsets[l + 1] - g.offsets[l]
    res = g.resolution[l]
    out = []
    for c in range(1 << D):
        w = np.ones(x.shape[0], np.float32)
        pp = []
        for d in range(D):
            if c & (1 << d):
                w = (w * frac[:, d]).astype(np.float32)
                pp.append(base[:, d] + np.uint32(1))
            else:
                w = (w * (np.float32(1) - frac[:, d])).astype(np.float32)
                pp.append(base[:, d])
        stride, idx = 1, np.zeros(x.shape[0], np.uint64)
        dense = True
        for d in range(D):
            if stride > T:
                break
            idx += pp[d].astype(np.uint64) * np.uint64(stride)
            stride *= res
        if T < stride:
            primes = [1, 2654435761, 805459861]
            h = np.zeros(x.shape[0], np.uint32)
            for d in range(D):
                h ^= (pp[d].astype(np.uint64) * np.uint64(primes[d]) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
            idx = h.astype(np.uint64)
            dense = False
        else:
            idx = idx & np.uint64(0xFFFFFFFF)
        out.append((w, (g.offsets[l] + idx % np.uint64(T)).astype(np.int64), dense))
    return out


@pytest.mark.parametrize("D,L,F,log2T", [(3, 4, 4, 14), (3, 8, 2, 12), (2, 4, 2, 10)])
def test_grid_forward_tcnn_matches_numpy_half_fma(orc, D, L, F, log2T):
    g = orc.make_grid(D, L, F, log2T)
    n = 3000
    x = _pos(n, D, D + L)
    rng = np.random.default_rng(L)
    table = rng.uniform(-0.5, 0.5, orc.grid_n_entries(g) * F).astype(np.float16)
    got, bound = orc.grid_forward_tcnn(g, x, table.view(np.uint16))
    tab = table.astype(np.float64).reshape(-1, F)
    for l in range(L):
        acc = np.zeros((n, F), np.float16)
        exact = np.zeros((n, F), np.float64)
        for w, e, _ in _np_corners(g, l, x):
            wh = w.astype(np.float16).astype(np.float64)
            acc = (wh[:, None] * tab[e] + acc.astype(np.float64)).astype(np.float16)  # one rounding per fp16 FMA
            exact += w.astype(np.float64)[:, None] * tab[e]
        np.testing.assert_array_equal(got[:, l * F:(l + 1) * F], acc.astype(np.float32))
        # the chain's stated bound holds against the exact blend
        err = np.abs(got[:, l * F:(l + 1) * F].astype(np.float64) - exact)
        assert np.all(err <= bound[:, l * F:(l + 1) * F].astype(np.float64) * (1 + 1e-6) + 1e-12)


def test_grid_backward_tcnn_matches_numpy_sequential_fp16(orc):
    D, L, F, log2T = 3, 4, 2, 10
    g = orc.make_grid(D, L, F, log2T)
    n = 1500
    x = _pos(n, D, 5)
    dy = np.random.default_rng(6).uniform(-1, 1, (n, L * F)).astype(np.float16)
    got, bound = orc.grid_backward_tcnn(g, x, dy.view(np.uint16))
    acc = np.zeros(orc.grid_n_entries(g) * F, np.float16)
    corners = [_np_corners(g, l, x) for l in range(L)]
    for i in range(n):  # sample order, then level, corner, feature: the oracle's order
        for l in range(L):
            for w, e, _ in corners[l]:
                for f in range(F):
                    c = np.float16(np.float32(dy[i, l * F + f]) * w[i])
                    if c == 0:
                        continue
                    k = e[i] * F + f
                    acc[k] = np.float16(np.float64(acc[k]) + np.float64(c))
    np.testing.assert_array_equal(got, acc.view(np.uint16))
    exact = orc.f16_bits_to_f32(orc.grid_backward_exact(g, x, dy.view(np.uint16))).astype(np.float64)
    # the engine's contract rounds the exact sum once; the sequential fp16 sum stays within its summed half-spacings
    # of the exact sum, so the two differ by at most that plus half a spacing of the engine's value
    ulp = np.spacing(np.abs(exact).astype(np.float16)).astype(np.float64)
    assert np.all(np.abs(orc.f16_bits_to_f32(got).astype(np.float64) - exact) <= bound + 0.5 * ulp + 1e-12)


def test_nerf_tcnn_close_to_engine_contract(orc):
    """The fp16-accumulate forward and the fp32-accumulate one (the engine's contract, orc.nerf_forward) of the same
    small C2-shaped network agree to SURVEY §8(c)'s colour/MLP-output bar; dL/d(encoding) likewise."""
    m = orc.make_nerf(L=4, F=4, log2T=12)
    p = orc.nerf_init(m, seed=3)
    nm = orc.mlp_n_params(m.density) + orc.mlp_n_params(m.rgb)
    p[nm:] = np.random.default_rng(4).uniform(-0.5, 0.5, p.size - nm)
    p16 = orc.f32_to_f16_bits(p)
    n = 2000
    g = np.random.default_rng(5)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dl = np.zeros((n, 16), np.float32)
    dl[:, :4] = g.uniform(-1, 1, (n, 4)).astype(np.float16)
    t = orc.nerf_tcnn(m, p16, c, dl)
    ref = orc.nerf_forward(m, p16, c)
    assert np.abs(t["out"] - ref).max() <= 1e-2 * np.abs(ref).max()
    assert np.abs(t["out"] - ref).max() > 0  # the two arithmetics are distinguishable at this size
    # dL/d(encoding): a ReLU whose pre-activation is within the fp16 accumulation noise of zero can switch between
    # the two arithmetics and mask a whole term of the backward. Beyond the bar only in such samples (smallest
    # |pre-activation| / sum |W a| under 2^-10), and in at most 3 % of the samples
    _, denc = orc.nerf_backward(m, p16, c, dl, want_denc=True)
    err = np.abs(t["denc"] - denc)
    bad = np.unique(np.where(err > 1e-2 * np.abs(denc).max())[0])
    margin = orc.nerf_train_ex(m, p16, c, dl)["margin"]
    assert np.all(margin[bad] < 2.0 ** -10), margin[bad].max()
    assert bad.size <= 0.03 * n, bad.size
