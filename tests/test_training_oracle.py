"""CPU tests of the image / SDF / loss restatements (oracle/ngp_train_oracle.c) and the host-side
mesh normalisation. The reference holds no vectors for these paths: the checks are
properties the reference code implies (stratum membership, pixel-centre snapping, sRGB targets,
samples on the surface, inside/outside signs) and independent numpy restatements."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    return load_package()


def test_loss_matches_numpy(orc):
    g = np.random.default_rng(0)
    n, dims = 257, 3
    out = g.uniform(-2, 2, (n, 16)).astype(np.float16)
    tgt = g.uniform(-2, 2, (n, dims)).astype(np.float32)
    p = out[:, :dims].astype(np.float32)
    d = p - tgt
    N = np.float32(n * dims)
    ref = {
        "L2": (d * d / N, 2 * d / N),
        "L1": (np.abs(d) / N, np.where(d >= 0, 1.0, -1.0) / N),
        "MAPE": (np.abs(d) / (np.abs(tgt) + 1e-2) / N, np.where(d >= 0, 1.0, -1.0) / (np.abs(tgt) + 1e-2) / N),
        "SMAPE": (np.abs(d) * 2 / (np.abs(p) + np.abs(tgt) + 1e-2) / N,
                  np.where(d >= 0, 1.0, -1.0) * 2 / (np.abs(p) + np.abs(tgt) + 1e-2) / N),
        "RelativeL2": (d * d / (p * p + 1e-2) / N, 2 * d / (p * p + 1e-2) / N),
    }
    for name, (v, gr) in ref.items():
        tot, dl, vals = orc.loss(name, out.view(np.uint16), tgt, dims, loss_scale=128.0)
        got = orc.f16_bits_to_f32(dl)
        np.testing.assert_allclose(vals, v.sum(1), rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(got[:, :dims], (128 * gr).astype(np.float16).astype(np.float32), rtol=2e-3, atol=1e-6)
        assert np.all(got[:, dims:] == 0)
        assert abs(tot - v.sum()) <= 1e-4 * abs(v.sum())


def srgb(x):
    return np.where(x < 0.0031308, 12.92 * x, 1.055 * np.power(x, 0.41666) - 0.055)


@pytest.mark.parametrize("snap", [True, False])
def test_image_samples_properties(orc, snap):
    W, H = 48, 32
    tex = np.random.default_rng(1).random((H, W, 4)).astype(np.float32)
    n = 1 << 10  # square power of two: stratified
    rng = orc.Rng(1337)
    state0 = rng.s.state
    pos, tgt = orc.image_samples(n, rng, tex, random_mode=3, snap=snap)
    # the stream advanced by 2n draws (generate_random_uniform)
    r2 = orc.Rng(1337)
    r2.advance(2 * n)
    assert rng.s.state == r2.s.state and state0 != rng.s.state
    if snap:
        ix = np.floor(pos[:, 0] * W).astype(int)
        iy = np.floor(pos[:, 1] * H).astype(int)
        np.testing.assert_allclose(pos[:, 0], (ix + 0.5) / W, rtol=1e-6)
        np.testing.assert_allclose(tgt, srgb(tex[iy, ix, :3]), rtol=1e-5, atol=1e-6)
    else:
        # stratification: sample i lies in cell (i % 32, i // 32) of the 32x32 strata
        i = np.arange(n)
        assert np.all(np.floor(pos[:, 0] * 32) == i % 32)
        assert np.all(np.floor(pos[:, 1] * 32) == i // 32)
        lo = srgb(tex[..., :3]).min(axis=(0, 1)) - 1e-5
        hi = srgb(tex[..., :3]).max(axis=(0, 1)) + 1e-5
        assert np.all((tgt >= lo) & (tgt <= hi))


def test_sdf_samples_and_signs(orc, pkg):
    verts = pkg.synthetic.icosphere(2, radius=0.3, center=(0.5, 0.5, 0.5))
    tris, amin, amax, brad = pkg.sdf.load_mesh(verts)
    n = 512
    rng = orc.Rng(7)
    pos, dist = orc.sdf_samples(n, rng, tris, amin, amax, brad / 1024)
    base = n // 8
    sd = orc.sdf_signed_distance(pos, tris)
    # exact surface samples: distance 0 written, true distance ~0
    assert np.all(dist[:4 * base] == 0)
    assert np.abs(sd[:4 * base]).max() < 1e-5
    # offset samples: the upper bound holds
    assert np.all(np.abs(sd[4 * base:7 * base]) <= dist[4 * base:7 * base] + 1e-6)
    # uniform samples inside the aabb
    u = pos[7 * base:]
    assert np.all(u >= amin - 1e-6) and np.all(u <= amax + 1e-6)
    # signs: centre inside (negative), corners outside (positive), magnitude ~ | |p - c| - r |
    c = tris.reshape(-1, 3).mean(axis=0)
    q = np.array([c, c + [0.6, 0, 0], [0.02, 0.02, 0.02], c + [0.1, 0.05, 0]], np.float32)
    s = orc.sdf_signed_distance(q, tris)
    r = np.linalg.norm(tris.reshape(-1, 3) - c, axis=1).mean()
    assert s[0] < 0 and s[1] > 0 and s[2] > 0 and s[3] < 0
    np.testing.assert_allclose(np.abs(s), np.abs(np.linalg.norm(q - c, axis=1) - r), atol=0.02 * r)


def test_load_mesh_normalisation(pkg):
    verts = pkg.synthetic.icosphere(1, radius=3.0, center=(10, -4, 2))
    tris, amin, amax, brad = pkg.sdf.load_mesh(verts)
    v = tris.reshape(-1, 3)
    # longest axis spans 1 / (1 + 2 * 0.005 * sqrt(3)) of the unit cube, centred on 0.5
    ext = v.max(0) - v.min(0)
    np.testing.assert_allclose(ext.max(), 1 / (1 + 2 * 0.005 * np.sqrt(3)), rtol=1e-3)
    np.testing.assert_allclose((v.max(0) + v.min(0)) / 2, 0.5, atol=1e-5)
    assert np.all(amin >= 0) and np.all(amax <= 1) and np.all(amin < v.min(0)) and np.all(amax > v.max(0))
    assert abs(brad - np.sqrt(0.75)) < 1e-6


def test_bvh_build_structure():
    """TriangleBvh4::build (host, csrc/bvh.hip): 4-ary nodes, every triangle in exactly one leaf of at
    most 8, child boxes contain their triangles, and the reordering is a permutation."""
    from __graft_entry__ import load_package
    pkg = load_package()
    verts = pkg.synthetic.icosphere(3, radius=0.3, bumps=0.3)
    tris, _, _, _ = pkg.sdf.load_mesh(verts)
    out, nodes = pkg.sdf.build_bvh(tris, 8)
    assert sorted(map(bytes, out)) == sorted(map(bytes, tris))
    seen = np.zeros(len(out), bool)
    for n in nodes:
        if n["left"] < 0:
            lo, hi = -n["left"] - 1, -n["right"] - 1
            assert 0 < hi - lo <= 8
            assert not seen[lo:hi].any()
            seen[lo:hi] = True
            v = out[lo:hi].reshape(-1, 3)
            assert np.all(v >= n["lo"]) and np.all(v <= n["hi"])
        else:
            assert n["right"] - n["left"] == 4
    assert seen.all()
