"""GPU parity of the NeRF renderer (NerfTracer) against the oracle's per-ray restatement.

Bars: ray marching is integer/stepping work identical to the oracle (same coordinates); colours are
composited from fp16 network outputs whose fp32 accumulation order differs, with __expf on the GPU,
so the image is compared within 2e-2 absolute per channel and 2e-3 on the mean."""
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


def _setup(pkg, orc, seed, grid_frac, aabb_scale=1.0):
    S = pkg.synthetic
    c2w = S.camera_poses(3, seed=seed)[1]
    cam = pkg.nerf.make_image(40, 30, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X)
    cfg = pkg.nerf.default_config(aabb_scale)
    ncfg = pkg.nerf_config("C2")
    ncfg["encoding"]["log2_hashmap_size"] = 14
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"], seed=seed)
    g = np.random.default_rng(seed)
    p = net.initialize_params(seed)
    nm = net.n_matrix_params
    p[nm:] = g.uniform(-0.5, 0.5, p.size - nm).astype(np.float32)
    tr.set_params_full_precision(p)
    torch.cuda.synchronize()
    p16 = tr.params.cpu().numpy().view(np.uint16).copy()
    grid = np.where(g.random(128 ** 3 * 8) < grid_frac, 1.0, 0.0).astype(np.float32)
    bf = orc.nerf_grid_bitfield(grid, cfg.max_cascade, 0.005)
    m = orc.make_nerf(L=4, F=4, log2T=14)
    net._trainer = tr  # the trainer owns the parameter buffers
    return cam, cfg, net, p16, bf, m


@pytest.mark.parametrize("seed,frac,sample_index,aabb_scale", [(0, 1.0, 0, 1.0), (1, 0.3, 3, 1.0), (5, 0.3, 0, 8.0),
                                                                (6, 0.15, 2, 4.0), (7, 0.05, 1, 16.0)])
def test_render_matches_oracle(pkg, orc, seed, frac, sample_index, aabb_scale):
    """aabb_scale > 1 (fox is 8: 4 cascades): the tracer marches with cone stepping through the shared
    ngp_math.h logf/expf and mips up to max_cascade (testbed_nerf.cu:948-1240,2504-2659)."""
    cam, cfg, net, p16, bf, m = _setup(pkg, orc, seed, frac, aabb_scale)
    r = pkg.nerf.NerfRenderer()
    bg = (0.1, 0.2, 0.3, 1.0)
    img = r.render(net, cfg, cam, torch.from_numpy(bf).cuda(), spp=1, sample_index=sample_index, min_transmittance=1e-4,
                   background=bg, use_inference_params=False).cpu().numpy()
    ref, counts = orc.nerf_render(cfg, cam, m, p16, bf, sample_index=sample_index, min_transmittance=1e-4, bg=bg)
    assert (counts > 0).mean() > 0.2  # the view sees the volume
    d = np.abs(img - ref)
    assert d.max() < 2e-2, d.max()
    assert d.mean() < 2e-3, d.mean()


@pytest.mark.parametrize("mode,k", [(1, (0.0578421, -0.0805099, -0.000980296, 0.00015575)), (2, (0.05, -0.01, 0.002, 0.0))])
def test_render_with_lens_matches_oracle(pkg, orc, mode, k):
    """render_with_lens_distortion with the training view's lens (testbed.cu:845-846): OpenCV and
    OpenCV fisheye (atanf: an ulp apart from the oracle's, inside the colour tolerance)."""
    cam, cfg, net, p16, bf, m = _setup(pkg, orc, 4, 0.5)
    cam.lens_mode = mode
    cam.lens_params[:] = list(k)
    cam.principal_point[:] = [0.47, 0.53]
    r = pkg.nerf.NerfRenderer()
    img = r.render(net, cfg, cam, torch.from_numpy(bf).cuda(), spp=1, min_transmittance=1e-4, background=(0, 0, 0, 1),
                   use_inference_params=False).cpu().numpy()
    ref, counts = orc.nerf_render(cfg, cam, m, p16, bf, sample_index=0, min_transmittance=1e-4, bg=(0, 0, 0, 1))
    assert (counts > 0).mean() > 0.2
    d = np.abs(img - ref)
    assert d.max() < 2e-2, d.max()
    assert d.mean() < 2e-3, d.mean()


@pytest.mark.parametrize("seed,frac", [(3, 1.0), (8, 0.3)])
def test_render_normals_matches_oracle(pkg, orc, seed, frac):
    """ERenderMode::Normals (testbed_nerf.cu:1183-1188, 2179-2181, 2615-2617): per step the density output's
    input gradient (ngp_input_gradient, backprop scale 128) composited as normalize(-density'(raw) * gradient),
    shaded (0.5 n + 0.5) * alpha. The gradient goes through fp16 intermediates whose fp32 sums are ordered
    differently from the oracle's and each step's normal is normalised, so a step whose gradient nearly
    vanishes can turn: pixels are compared within 2e-2, 98 % of them, mean 5e-3."""
    cam, cfg, net, p16, bf, m = _setup(pkg, orc, seed, frac)
    r = pkg.nerf.NerfRenderer()
    bg = (0.1, 0.2, 0.3, 1.0)
    img = r.render(net, cfg, cam, torch.from_numpy(bf).cuda(), spp=1, min_transmittance=1e-4, background=bg,
                   use_inference_params=False, render_mode="Normals").cpu().numpy()
    ref, counts = orc.nerf_render_normals(cfg, cam, m, p16, bf, min_transmittance=1e-4, bg=bg)
    assert (counts > 0).mean() > 0.2
    assert np.isfinite(img).all()
    d = np.abs(img - ref).max(axis=2)
    assert (d < 2e-2).mean() > 0.98, (d < 2e-2).mean()
    assert d.mean() < 5e-3, d.mean()
    # a Shade render with the same renderer afterwards is unaffected by the mode switch
    shade = r.render(net, cfg, cam, torch.from_numpy(bf).cuda(), spp=1, min_transmittance=1e-4, background=bg,
                     use_inference_params=False).cpu().numpy()
    ref_s, _ = orc.nerf_render(cfg, cam, m, p16, bf, min_transmittance=1e-4, bg=bg)
    assert np.abs(shade - ref_s).max() < 2e-2


def test_render_spp_average_and_background(pkg, orc):
    cam, cfg, net, p16, bf, m = _setup(pkg, orc, 2, 0.0)  # empty grid: every ray misses -> background
    r = pkg.nerf.NerfRenderer()
    img = r.render(net, cfg, cam, torch.from_numpy(bf).cuda(), spp=4, background=(0.25, 0.5, 0.75, 1.0),
                   use_inference_params=False).cpu().numpy()
    np.testing.assert_allclose(img, np.broadcast_to(np.array([0.25, 0.5, 0.75, 1.0], np.float32), img.shape), atol=1e-6)


def test_psnr_after_training(pkg):
    """The metric's second half: train on the procedural Lego stand-in, render held-out views, PSNR
    (scripts/run.py protocol: black background, snapped pixels, min transmittance 1e-4)."""
    S = pkg.synthetic
    ds, ims, pix = S.lego_like_dataset(n_images=24, width=96, height=96, seed=4, return_host=True)
    cfg = pkg.nerf.default_config(1.0)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    for _ in range(400):
        run.train_step(get_loss=False)
    r = pkg.nerf.NerfRenderer()
    test_poses = S.camera_poses(30, seed=99)[-3:]
    ps = []
    for c2w in test_poses:
        cam = pkg.nerf.make_image(96, 96, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X)
        img = r.render(net, cfg, cam, run.bitfield, spp=2, min_transmittance=1e-4, background=(0, 0, 0, 1))
        ref = pkg.nerf.ground_truth_linear(S.render(c2w, 96, 96))
        ps.append(pkg.nerf.psnr(img, ref)[0])
    assert np.mean(ps) > 20.0, ps


@pytest.mark.parametrize("mode,seed,frac,aabb_scale,show_accel", [
    ("Depth", 3, 1.0, 1.0, -1), ("Positions", 8, 0.3, 1.0, -1), ("AO", 6, 0.3, 4.0, -1), ("Depth", 5, 0.3, 8.0, -1),
    ("EncodingVis", 7, 0.3, 1.0, -1), ("EncodingVis", 4, 0.3, 8.0, -1),
    ("Positions", 9, 0.3, 1.0, 0), ("Positions", 10, 0.3, 8.0, 2), ("Shade", 11, 0.3, 4.0, 1)])
def test_render_modes_match_oracle(pkg, orc, mode, seed, frac, aabb_scale, show_accel):
    """ERenderMode AO, Positions, Depth and EncodingVis (testbed_nerf.cu:1189-1208: each step's alpha, (pos - 0.5) / 2
    + 0.5, dot(camera forward, pos - origin) * depth_scale with depth_scale = 1 / dataset scale, :2822, the warped
    position), composited like Shade and shaded without sRGB decoding (:2183-2186). show_accel >= 0 (the GUI's
    "Show acceleration", testbed.cu:1678): the march from that mip up (:2497, 2594), opaque steps (:1078-1080) and
    Positions coloured by the step's occupancy cell (:1190-1199: 1 - mip / 7 and two pcg32 draws seeded by the
    cell). Same march and bars as the Shade comparison."""
    cam, cfg, net, p16, bf, m = _setup(pkg, orc, seed, frac, aabb_scale)
    r = pkg.nerf.NerfRenderer()
    bg = (0.1, 0.2, 0.3, 1.0)
    ds = 1.0 / 0.33  # nerf_synthetic's scale (nerf_loader.cu:388)
    img = r.render(net, cfg, cam, torch.from_numpy(bf).cuda(), spp=1, min_transmittance=1e-4, background=bg,
                   use_inference_params=False, render_mode=mode, depth_scale=ds, show_accel=show_accel).cpu().numpy()
    ref, counts = orc.nerf_render(cfg, cam, m, p16, bf, min_transmittance=1e-4, bg=bg, render_mode=mode, depth_scale=ds,
                                  show_accel=show_accel)
    assert (counts > 0).mean() > 0.2
    assert np.isfinite(img).all()
    scale = max(1.0, float(np.abs(ref).max()))  # depth values grow with the scene's size
    d = np.abs(img - ref)
    assert d.max() < 2e-2 * scale, (d.max(), scale)
    assert d.mean() < 2e-3 * scale, d.mean()
    if mode == "Positions":  # a hit pixel's colour is a weighted mean of positions inside the unit cube
        hit = counts > 0
        assert np.all(img.reshape(-1, 4)[hit, :3] > -0.5)
