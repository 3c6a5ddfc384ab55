"""CPU tests of the NeRF host side and of the NeRF oracle's own invariants (no GPU calls)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    return load_package()


def test_default_config_matches_reference_defaults(pkg):
    c = pkg.nerf.default_config(1.0)
    assert list(c.aabb_min) == [0, 0, 0] and list(c.aabb_max) == [1, 1, 1]
    assert c.cone_angle_constant == 0.0 and c.max_cascade == 0
    assert (c.snap_to_pixel_centers, c.random_bg_color, c.linear_colors, c.color_space_linear) == (1, 1, 0, 1)
    assert (c.rgb_activation, c.density_activation, c.loss_type) == (3, 3, 4)
    assert c.near_distance == pytest.approx(0.1) and c.target_batch_size == 1 << 18
    c = pkg.nerf.default_config(16.0)
    assert list(c.aabb_min) == [-7.5] * 3 and list(c.aabb_max) == [8.5] * 3
    assert c.max_cascade == 4 and c.cone_angle_constant == pytest.approx(1 / 256)
    c = pkg.nerf.default_config(256.0)  # inflation capped at 2^(cascades-1) = 128 (testbed_nerf.cu:3093)
    assert list(c.aabb_max) == [64.5] * 3 and c.max_cascade == 8
    c = pkg.nerf.default_config(2.0, loss_type=0, background_color=(1, 0.5, 0))
    assert c.loss_type == 0 and list(c.background_color) == [1, 0.5, 0]


def test_pcg32_seeding_matches_oracle(pkg, orc):
    r = pkg.nerf.pcg32(1337)
    o = orc.Rng(1337)
    assert (r.state, r.inc) == (o.s.state, o.s.inc)


def test_nerf_matrix_to_ngp(pkg):
    m = np.eye(4)
    m[:3, 3] = [1.0, 2.0, 3.0]
    x = pkg.nerf.nerf_matrix_to_ngp(m).reshape(4, 3)  # columns
    # column 1/2 negated, translation scaled + offset, rows cycled xyz <- yzx
    np.testing.assert_allclose(x[0], [0, 0, 1])
    np.testing.assert_allclose(x[1], [-1, 0, 0])
    np.testing.assert_allclose(x[2], [0, -1, 0])
    np.testing.assert_allclose(x[3], [2 * 0.33 + 0.5, 3 * 0.33 + 0.5, 1 * 0.33 + 0.5], rtol=1e-6)


def test_camera_matrix_of_rotation_is_identity_map(pkg, orc):
    S = pkg.synthetic
    for c2w in S.camera_poses(5, seed=4):
        x = pkg.nerf.nerf_matrix_to_ngp(c2w)
        np.testing.assert_allclose(orc.camera_matrix(x), x, atol=2e-6)


def test_synthetic_render(pkg):
    S = pkg.synthetic
    px = S.render(S.camera_poses(1)[0], 64, 48)
    assert px.shape == (48, 64, 4) and px.dtype == np.uint8
    a = px[..., 3]
    assert 0.05 < (a == 255).mean() < 0.9 and set(np.unique(a)) <= {0, 255}
    assert (px[a == 0][:, :3] == 0).all()


def _scene(pkg, n=3, w=40, h=30):
    S = pkg.synthetic
    ims, pix = [], []
    for c2w in S.camera_poses(n, seed=9):
        ims.append(pkg.nerf.make_image(w, h, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X))
        pix.append(S.render(c2w, w, h))
    return ims, pix


def test_oracle_sampler_invariants(pkg, orc):
    ims, pix = _scene(pkg)
    cfg = pkg.nerf.default_config(1.0)
    full = np.full(128 ** 3, 1.0, np.float32)
    bf = orc.nerf_grid_bitfield(np.concatenate([full] + [np.zeros_like(full)] * 7), 0, 0.005)
    out = orc.nerf_generate_samples(cfg, ims, pix, 64, orc.pcg(*_st(pkg.nerf.pcg32(5))), 1 << 16, bf)
    kept, total = out["counters"]
    assert 0 < kept <= 64
    ns = out["numsteps"][:kept]
    assert ns[:, 0].sum() == total and (ns[:, 1] == np.concatenate([[0], np.cumsum(ns[:-1, 0])])).all()
    c = out["coords"][:total]
    assert (c[:, :3] >= 0).all() and (c[:, :3] <= 1).all()
    np.testing.assert_allclose(c[:, 3], 0.0, atol=1e-6)  # dt = MIN_CONE_STEPSIZE at cone 0 -> warped 0
    assert (np.diff(out["ray_indices"][:kept].astype(np.int64)) > 0).all()
    empty = orc.nerf_generate_samples(cfg, ims, pix, 64, orc.pcg(*_st(pkg.nerf.pcg32(5))), 1 << 16, np.zeros_like(bf))
    assert list(empty["counters"]) == [0, 0]


def _st(r):
    return r.state, r.inc


def test_oracle_bitfield_max_pool(orc):
    g = np.zeros(128 ** 3 * 8, np.float32)
    x, y, z = 70, 3, 127
    g[orc.lib().orc_morton3D(x, y, z)] = 1.0
    bf = orc.nerf_grid_bitfield(g, 0, 0.005)
    bits = np.unpackbits(bf, bitorder="little").reshape(8, -1)
    assert bits[0].sum() == 1
    for level in range(1, 8):
        assert bits[level].sum() == 1
        x, y, z = x // 2 + 32, y // 2 + 32, z // 2 + 32
        assert bits[level][orc.lib().orc_morton3D(x, y, z)] == 1


def test_oracle_rollover(orc):
    a = np.arange(40, dtype=np.float32).reshape(10, 4)
    orc.fill_rollover(a, 3)
    np.testing.assert_array_equal(a[3:6], a[0:3])
    np.testing.assert_array_equal(a[9], a[0])


def test_counters_update_oracle_hand_cases(orc):
    """NerfCounters::update_after_training (testbed_nerf.cu:3583-3609), cases worked by hand."""
    B = 1 << 18
    # 4096 * 262144 / 100000 = 10737.4 -> 10737 -> next multiple of 256 = 10752
    assert orc.nerf_counters_update(4096, B, 500000, 100000, 2.0) == (10752, 100000, 500000, pytest.approx(2.0 * 100000 / B))
    # either counter zero: early return, rays_per_batch unchanged, measured sizes zeroed
    assert orc.nerf_counters_update(4096, B, 0, 0)[:3] == (4096, 0, 0)
    assert orc.nerf_counters_update(7936, B, 123, 0)[:3] == (7936, 0, 0)
    # clamp to 2^18 rays
    assert orc.nerf_counters_update(1 << 18, B, 4 << 18, 1000)[0] == 1 << 18
    # exact fit keeps R (already a multiple of 256)
    assert orc.nerf_counters_update(8192, B, 9 << 18, B)[0] == 8192
    # the step's inference size (testbed_nerf.cu:3923-3930)
    assert orc.nerf_max_inference(0, 1 << 22) == 1 << 22
    assert orc.nerf_max_inference(300001, 1 << 22) == 300032
    assert orc.nerf_max_inference(5 << 22, 1 << 22) == 1 << 22


def test_oracle_error_map_deposit_and_cdfs(pkg, orc):
    """The error map (testbed_nerf.cu:1869-1899, 2356-2410, 3730-3745) in the oracle: every compacted ray's
    mean loss is split over 4 texels with weights summing to 1, so the map's total is the sum of the per-ray
    losses; the CDF restatement equals a scalar float32 loop of the kernels; the image pmf sums to 1."""
    ims, pix = _scene(pkg, n=3, w=40, h=30)
    cfg = pkg.nerf.default_config(1.0)
    full = np.full(128 ** 3, 1.0, np.float32)
    bf = orc.nerf_grid_bitfield(np.concatenate([full] + [np.zeros_like(full)] * 7), 0, 0.005)
    n_rays = 256
    s = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc.pcg(*_st(pkg.nerf.pcg32(5))), 1 << 16, bf)
    out = np.random.default_rng(1).uniform(-2, 2, (1 << 16, 16)).astype(np.float16)
    res = orc.nerf_compute_loss(cfg, ims, pix, n_rays, orc.pcg(*_st(pkg.nerf.pcg32(5))), 1 << 15, s, out.view(np.uint16),
                                0.01, error_map_res=(9, 7))
    em = res["error_map"]
    assert em.shape == (3, 7, 9) and (em >= 0).all() and em.sum() > 0
    np.testing.assert_allclose(em.sum(dtype=np.float64), res["loss"].sum(dtype=np.float64) * n_rays, rtol=1e-5)
    cx, cy, ci = orc.error_map_cdfs(em)
    n, h, w = em.shape
    f = np.float32
    for i in range(n):
        cum_y = f(0)
        rows = []
        for y in range(h):
            cum = f(0)
            row = []
            for x in range(w):
                cum = f(cum + f(em[i, y, x] + f(1e-10)))
                row.append(cum)
            rows.append(cum)
            norm = f(1) / cum
            for x in range(w):
                want = f(f(f(f(1) - f(0.01)) * row[x]) * norm) + f(f(f(0.01) * f(x + 1)) / f(w))
                assert cx[i, y, x] == want
        for y in range(h):
            cum_y = f(cum_y + rows[y])
            assert cy[i, y] == f(f(f(f(1) - f(0.01)) * cum_y) * (f(1) / ci[i])) + f(f(f(0.01) * f(y + 1)) / f(h))
        assert ci[i] == cum_y
    assert (np.diff(cx, axis=2) > 0).all() and np.allclose(cx[:, :, -1], 1.0) and np.allclose(cy[:, -1], 1.0)
    pmf, cdf = orc.error_map_image_pmf(ci)
    assert abs(float(pmf.sum(dtype=np.float64)) - 1.0) < 1e-6 and abs(float(cdf[-1]) - 1.0) < 1e-6
