"""GPU parity of the NeRF training kernels (src/testbed_nerf.cu) against oracle/ngp_nerf_oracle.c.

Bars: sample generation (ray indices, per-ray step counts and bases, ray origins/directions, sample
coordinates) bit-exact with cone_angle 0 (no transcendental on that path; slots from prefix scans
equal the oracle's ray-order slots); density-grid sample positions/indices, splat+EMA grid, mean
(fixed reduction tree) and bitfields bit-exact;
rollover bit-exact. Cone-angle stepping and compositing evaluate ngp_math.h's expf/logf on both sides,
so sample indices, compacted counts, bases and coordinates are bit-exact at every aabb_scale; losses
agree to 1e-4 relative and fp16 loss gradients to 2 fp16 ulp (sRGB targets use powf).
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


@pytest.fixture(scope="module")
def scene(pkg):
    S = pkg.synthetic
    ims, pix = [], []
    for i, c2w in enumerate(S.camera_poses(6, seed=1)):
        w, h = 96 + 8 * i, 80 + 4 * i  # ragged image sizes
        ims.append(pkg.nerf.make_image(w, h, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X))
        px = S.render(c2w, w, h)
        px[3:5, 7:40] = np.array([255, 0, 255, 0], np.uint8)  # masked pixels (0x00FF00FF)
        pix.append(px)
    ds = pkg.nerf.NerfDataset(ims, pix)
    return ds, ims, pix


FOX_LENS = (0.0578421, -0.0805099, -0.000980296, 0.00015575)  # data/nerf/fox/transforms.json k1 k2 p1 p2


@pytest.fixture(scope="module")
def scene_lens(pkg):
    """OpenCV-distorted cameras (fox coefficients, and a stronger one) with off-centre principal points."""
    S = pkg.synthetic
    ims, pix = [], []
    for i, c2w in enumerate(S.camera_poses(4, seed=3)):
        w, h = 90 + 6 * i, 120 - 4 * i
        k = FOX_LENS if i % 2 == 0 else (-0.21, 0.05, 0.002, -0.001)
        ims.append(pkg.nerf.make_image(w, h, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X,
                                       principal=(0.48 + 0.01 * i, 0.52 - 0.01 * i), lens_mode=pkg.nerf.LENS_OPENCV,
                                       lens_params=k))
        pix.append(S.render(c2w, w, h))
    return pkg.nerf.NerfDataset(ims, pix), ims, pix


def occupancy(orc, seed=0, frac=0.3, max_cascade=0):
    g = np.random.default_rng(seed)
    grid = np.where(g.random(128 ** 3 * 8) < frac, 1.0, 0.0).astype(np.float32)
    return grid, orc.nerf_grid_bitfield(grid, max_cascade, 0.005)


def rng(pkg, seed):
    r = pkg.nerf.pcg32(seed)
    return r


def orc_rng(orc, r):
    return orc.pcg(r.state, r.inc)


@pytest.mark.parametrize("n_rays,max_samples,frac", [(1, 4096, 1.0), (777, 1 << 16, 0.3), (4096, 1 << 15, 0.5),
                                                     (4096, 1 << 18, 0.02)])
def test_generate_training_samples_bitexact(pkg, orc, scene, n_rays, max_samples, frac):
    ds, ims, pix = scene
    cfg = pkg.nerf.default_config(1.0)
    _, bf = occupancy(orc, seed=n_rays, frac=frac)
    r = rng(pkg, 1337 + n_rays)
    got = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, max_samples, torch.from_numpy(bf).cuda(),
                                             n_rays_total=n_rays)
    ref = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc_rng(orc, r), max_samples, bf)
    got = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(got["counters"].view(np.uint32), ref["counters"])
    kept = int(ref["counters"][0])
    assert kept > 0
    np.testing.assert_array_equal(got["ray_indices"][:kept].view(np.uint32), ref["ray_indices"][:kept])
    np.testing.assert_array_equal(got["numsteps"][:kept].view(np.uint32), ref["numsteps"][:kept])
    np.testing.assert_array_equal(got["rays"][:kept], ref["rays"][:kept])
    used = min(int(ref["counters"][1]), max_samples)
    np.testing.assert_array_equal(got["coords"][:used], ref["coords"][:used])


@pytest.mark.parametrize("aabb_scale,n_rays,max_samples", [
    (1.0, 1, 2), (1.0, 3, 40), (1.0, 17, 300), (1.0, 1 << 16, 1 << 17), (1.0, 50001, 123457),
    (8.0, 5, 100), (8.0, 1 << 16, 1 << 17), (8.0, 40000, 99999)])
def test_sampler_sample_budget(pkg, orc, scene, aabb_scale, n_rays, max_samples):
    """The sample budget cuts the batch inside a count wave (k_sample_bscan finds the crossing wave and counts
    its rays; k_sample_write keeps a ray only while its inclusive prefix fits): counters, kept rays, bases and
    coordinates bit-exact with the oracle's sequential atomicAdd order (testbed_nerf.cu:1616-1619), at cone 0 (16
    rays per count wave) and with cone stepping (8), ragged and tiny batches included."""
    ds, ims, pix = scene
    cfg = pkg.nerf.default_config(aabb_scale)
    _, bf = occupancy(orc, seed=n_rays % 1000 + 3, frac=0.3, max_cascade=cfg.max_cascade)
    r = rng(pkg, 77 + n_rays)
    got = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, max_samples, torch.from_numpy(bf).cuda(), n_rays_total=n_rays)
    ref = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc_rng(orc, r), max_samples, bf)
    got = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(got["counters"].view(np.uint32), ref["counters"])
    kept = int(ref["counters"][0])
    if n_rays > 100:
        assert int(ref["counters"][1]) > max_samples and kept < n_rays  # the budget cuts the batch
    np.testing.assert_array_equal(got["ray_indices"][:kept].view(np.uint32), ref["ray_indices"][:kept])
    np.testing.assert_array_equal(got["numsteps"][:kept].view(np.uint32), ref["numsteps"][:kept])
    np.testing.assert_array_equal(got["rays"][:kept], ref["rays"][:kept])
    used = int(ref["numsteps"][kept - 1][0] + ref["numsteps"][kept - 1][1]) if kept else 0
    np.testing.assert_array_equal(got["coords"][:used], ref["coords"][:used])


@pytest.mark.parametrize("n_rays,frac", [(2048, 0.4), (4096, 1.0)])
def test_generate_training_samples_opencv_lens(pkg, orc, scene_lens, n_rays, frac):
    """uv_to_ray with OpenCV undistortion (iterative Newton, common_device.cuh:330-369): no
    transcendental, so rays and samples stay bit-exact with the oracle."""
    ds, ims, pix = scene_lens
    cfg = pkg.nerf.default_config(1.0)
    _, bf = occupancy(orc, seed=n_rays + 7, frac=frac)
    r = rng(pkg, 4242 + n_rays)
    got = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, 1 << 18, torch.from_numpy(bf).cuda(), n_rays_total=n_rays)
    ref = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc_rng(orc, r), 1 << 18, bf)
    got = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(got["counters"].view(np.uint32), ref["counters"])
    kept = int(ref["counters"][0])
    np.testing.assert_array_equal(got["rays"][:kept], ref["rays"][:kept])
    np.testing.assert_array_equal(got["numsteps"][:kept].view(np.uint32), ref["numsteps"][:kept])
    used = min(int(ref["counters"][1]), 1 << 18)
    np.testing.assert_array_equal(got["coords"][:used], ref["coords"][:used])


@pytest.mark.parametrize("aabb_scale,n_rays,frac", [(4.0, 2048, 0.4), (8.0, 4096, 0.3), (8.0, 3000, 1.0), (16.0, 2048, 0.2)])
def test_generate_training_samples_cone(pkg, orc, scene, aabb_scale, n_rays, frac):
    """aabb_scale > 1 (the fox config is 8: 4 cascades): cone-angle stepping through logf/expf
    (testbed_nerf.cu:114-184) and mips 0..max_cascade. Engine and oracle evaluate the same
    ngp_math.h expf/logf, so counts, bases, rays and every sample coordinate are bit-exact."""
    ds, ims, pix = scene
    cfg = pkg.nerf.default_config(aabb_scale)
    assert cfg.cone_angle_constant > 1e-5
    _, bf = occupancy(orc, seed=5 + n_rays, frac=frac, max_cascade=cfg.max_cascade)
    r = rng(pkg, 99 + n_rays)
    max_samples = 1 << 20
    got = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, max_samples, torch.from_numpy(bf).cuda(), n_rays_total=n_rays)
    ref = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc_rng(orc, r), max_samples, bf)
    got = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(got["counters"].view(np.uint32), ref["counters"])
    kept = int(ref["counters"][0])
    assert kept > 0
    np.testing.assert_array_equal(got["ray_indices"][:kept].view(np.uint32), ref["ray_indices"][:kept])
    np.testing.assert_array_equal(got["numsteps"][:kept].view(np.uint32), ref["numsteps"][:kept])
    np.testing.assert_array_equal(got["rays"][:kept], ref["rays"][:kept])
    used = min(int(ref["counters"][1]), max_samples)
    assert used > 0
    np.testing.assert_array_equal(got["coords"][:used], ref["coords"][:used])


@pytest.mark.parametrize("aabb_scale,cone,n_rays,frac", [
    (8.0, None, 1 << 16, 0.05), (32.0, None, 1 << 16, 0.03), (128.0, None, 1 << 16, 0.01),
    (8.0, 1e-4, 1 << 14, 0.05), (8.0, 5e-4, 1 << 14, 0.05), (16.0, 2e-5, 1 << 13, 0.05), (8.0, 0.02, 1 << 14, 0.1),
    # a ragged cone-0 batch
    (8.0, None, 1 << 15, 0.05), (1.0, None, 30001, 0.1)])
def test_sampler_and_loss_cone_at_scale(pkg, orc, scene, aabb_scale, cone, n_rays, frac):
    """Fox-scale and larger ray counts (64k rays at aabb_scale 8, 32, 128: 2-4 K count waves and 4 tiles of the
    loss's group scan; 32k and 30001 rays) and user-set cone angles
    from 2e-5 to 0.02: the sampler's hardware exp/log speculation in empty space (csrc/nerf.hip
    step_empty) falls back to the exact path near every integer decision, with margins that scale with
    1 / log(1 + cone), so sample sets, compacted counts and coordinates stay bit-exact with the oracle."""
    ds, ims, pix = scene
    kw = {} if cone is None else {"cone_angle_constant": cone}
    cfg = pkg.nerf.default_config(aabb_scale, **kw)
    _, bf = occupancy(orc, seed=int(aabb_scale) + n_rays, frac=frac, max_cascade=cfg.max_cascade)
    r = rng(pkg, 2024 + n_rays)
    max_samples = 1 << 22
    bf_t = torch.from_numpy(bf).cuda()
    got = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, max_samples, bf_t, n_rays_total=n_rays)
    ref = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc_rng(orc, r), max_samples, bf)
    gn = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(gn["counters"].view(np.uint32), ref["counters"])
    kept = int(ref["counters"][0])
    assert kept > n_rays // 8  # most rays fit the sample budget (the rest are dropped, as the reference does)
    np.testing.assert_array_equal(gn["ray_indices"][:kept].view(np.uint32), ref["ray_indices"][:kept])
    np.testing.assert_array_equal(gn["numsteps"][:kept].view(np.uint32), ref["numsteps"][:kept])
    used = min(int(ref["counters"][1]), max_samples)
    assert used > n_rays
    np.testing.assert_array_equal(gn["coords"][:used], ref["coords"][:used])
    # compaction of the same samples (testbed_nerf.cu:1660-2012)
    g = np.random.default_rng(n_rays)
    out = g.uniform(-3.0, 2.0, (max_samples, 16)).astype(np.float16)
    mean = torch.tensor([0.003], device="cuda")
    max_c = 1 << 18
    gl = pkg.nerf.compute_loss(ds, cfg, n_rays, r, max_c, got, torch.from_numpy(out).cuda(), mean)
    rl = orc.nerf_compute_loss(cfg, ims, pix, n_rays, orc_rng(orc, r), max_c, ref, out.view(np.uint16), 0.003)
    cc = int(gl["compacted_counter"].cpu().numpy().view(np.uint32)[0])
    assert cc == int(rl["compacted_counter"][0]) and cc > 0
    n_used = min(cc, max_c)
    np.testing.assert_array_equal(gl["coords_compacted"].cpu().numpy()[:n_used], rl["coords_compacted"][:n_used])


@pytest.mark.parametrize("loss_type,act,aabb_scale", [(4, 3, 1.0), (0, 2, 1.0), (1, 3, 1.0), (4, 3, 8.0), (0, 2, 4.0)])
def test_compute_loss(pkg, orc, scene, loss_type, act, aabb_scale):
    """compute_loss_kernel_train_nerf (testbed_nerf.cu:1660-2012). Compositing weights use the shared
    ngp_expf (the reference's __expf site :1744), so where each ray terminates, the compacted count,
    every compacted {n, base} and every compacted coordinate are bit-exact, cone stepping included.
    Losses and dL/doutput are floating point: the sRGB targets go through powf (ocml vs glibc), so
    losses agree to rtol 1e-4 and each fp16 gradient to 2 fp16 ulp (+1e-7 absolute)."""
    ds, ims, pix = scene
    cfg = pkg.nerf.default_config(aabb_scale, loss_type=loss_type, rgb_activation=act, density_activation=3)
    _, bf = occupancy(orc, seed=2, frac=0.5, max_cascade=cfg.max_cascade)
    n_rays, max_samples = 2000, 1 << 17
    r = rng(pkg, 7)
    samples = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, max_samples, torch.from_numpy(bf).cuda())
    ref_s = orc.nerf_generate_samples(cfg, ims, pix, n_rays, orc_rng(orc, r), max_samples, bf)
    g = np.random.default_rng(loss_type)
    out = g.uniform(-3.0, 2.0, (max_samples, 16)).astype(np.float16)
    out_t = torch.from_numpy(out).cuda()
    mean = torch.tensor([0.003], device="cuda")
    max_c = 1 << 15
    em = torch.zeros((len(ims), 11, 13), dtype=torch.float32, device="cuda")
    got = pkg.nerf.compute_loss(ds, cfg, n_rays, r, max_c, samples, out_t, mean, error_map=em)
    ref = orc.nerf_compute_loss(cfg, ims, pix, n_rays, orc_rng(orc, r), max_c, ref_s, out.view(np.uint16), 0.003,
                                error_map_res=(13, 11))
    kept = int(ref_s["counters"][0])
    # error map deposit (:1869-1899): float atomics in any order, losses to rtol 1e-4 (powf, see above)
    em_ref = ref["error_map"]
    assert em_ref.sum() > 0
    np.testing.assert_allclose(em.cpu().numpy(), em_ref, rtol=1e-4, atol=1e-6 * float(em_ref.max()))
    cc = int(got["compacted_counter"].cpu().numpy().view(np.uint32)[0])
    assert cc == int(ref["compacted_counter"][0])
    assert cc > 0
    ns_got = samples["numsteps"].cpu().numpy()[:kept].view(np.uint32)
    np.testing.assert_array_equal(ns_got, ref_s["numsteps"][:kept])
    n_used = min(cc, max_c)
    co_got = got["coords_compacted"].cpu().numpy()
    np.testing.assert_array_equal(co_got[:n_used], ref["coords_compacted"][:n_used])
    np.testing.assert_allclose(got["loss"].cpu().numpy()[:kept], ref["loss"][:kept], rtol=1e-4, atol=1e-9)
    dl_got = got["dloss_doutput"].cpu().numpy().astype(np.float32)[:n_used, :4]
    dl_ref = orc.f16_bits_to_f32(ref["dloss_doutput"])[:n_used, :4]
    tol = 2 * np.spacing(np.abs(dl_ref).astype(np.float16)).astype(np.float32) + 1e-7
    bad = np.abs(dl_got - dl_ref) > tol
    assert not bad.any(), (int(bad.sum()), dl_got[bad][:5], dl_ref[bad][:5])


@pytest.mark.parametrize("loss_type,act,aabb_scale", [(4, 3, 1.0), (0, 2, 4.0)])
def test_compute_loss_kept_state_is_bitwise_equal(pkg, scene, orc, loss_type, act, aabb_scale):
    """The training step's form of the loss (pass 1 keeps each composited sample's weight, transmittance and
    rgb prefix; pass 2 reads them instead of compositing each ray again) gives the same bits as the two
    compositing passes: compacted count, {n, base}, coordinates, losses and dL/doutput. Also with a state
    capacity shorter than the samples (a C-ABI caller's smaller buffer): pass 2 composites the rays past it
    again instead of reading unwritten state, with the same bits."""
    ds, ims, pix = scene
    cfg = pkg.nerf.default_config(aabb_scale, loss_type=loss_type, rgb_activation=act, density_activation=3)
    _, bf = occupancy(orc, seed=3, frac=0.5, max_cascade=cfg.max_cascade)
    n_rays, max_samples, max_c = 2000, 1 << 17, 1 << 15
    r = rng(pkg, 11)
    g = np.random.default_rng(loss_type + 7)
    out_t = torch.from_numpy(g.uniform(-3.0, 2.0, (max_samples, 16)).astype(np.float16)).cuda()
    mean = torch.tensor([0.003], device="cuda")
    res = []
    for keep, cap in ((False, None), (True, None), (True, "short")):
        samples = pkg.nerf.generate_training_samples(ds, cfg, n_rays, r, max_samples, torch.from_numpy(bf).cuda())
        if cap == "short":  # about a third of the generated samples
            cap = max(1, int(samples["counters"][1].item()) // 3)  # counters = {rays kept, samples}
        got = pkg.nerf.compute_loss(ds, cfg, n_rays, r, max_c, samples, out_t, mean, keep_state=keep, state_capacity=cap)
        torch.cuda.synchronize()
        res.append({"ns": samples["numsteps"].cpu().numpy(), **{k: v.cpu().numpy() for k, v in got.items()}})
    a = res[0]
    assert int(a["compacted_counter"][0]) > 0
    for b in res[1:]:
        for k in ("ns", "compacted_counter", "coords_compacted", "loss"):
            np.testing.assert_array_equal(a[k].view(np.uint32), b[k].view(np.uint32), err_msg=k)
        np.testing.assert_array_equal(a["dloss_doutput"].view(np.uint16), b["dloss_doutput"].view(np.uint16))


@pytest.mark.parametrize("dtype,rescale", [(torch.float32, False), (torch.float16, False), (torch.float16, True)])
def test_fill_rollover(pkg, orc, dtype, rescale):
    g = np.random.default_rng(1)
    n, stride, n_in = 1000, 7 if dtype == torch.float32 else 16, 333
    a = g.standard_normal((n, stride)).astype(np.float32 if dtype == torch.float32 else np.float16)
    t = torch.from_numpy(a.copy()).cuda()
    pkg.nerf.fill_rollover(t, torch.tensor([n_in], dtype=torch.int32, device="cuda"), rescale=rescale)
    ref = a.copy() if dtype == torch.float32 else a.view(np.uint16).copy()
    orc.fill_rollover(ref, n_in, rescale)
    got = t.cpu().numpy()
    np.testing.assert_array_equal(got if dtype == torch.float32 else got.view(np.uint16), ref)


@pytest.mark.parametrize("binned", [False, True])
def test_density_grid_update(pkg, orc, binned):
    """binned: the memset + splat as one counting sort by cell bin (ngp_nerf_grid_splat_max_cells, what the
    trainer's update runs); tmp starts as garbage there, since every cell is written."""
    cfg = pkg.nerf.default_config(4.0)
    g = np.random.default_rng(3)
    grid = np.where(g.random(128 ** 3 * 8) < 0.5, g.random(128 ** 3 * 8) * 0.02, 0.0).astype(np.float32)
    grid[:1000] = -1.0  # untrained cells stay negative through the EMA
    n_casc = cfg.max_cascade + 1
    n = 128 ** 3 * n_casc // 4
    r = rng(pkg, 11)
    grid_t = torch.from_numpy(grid).cuda()
    pos, idx = pkg.nerf.grid_generate_samples(cfg, n, r, 3, grid_t, n_casc, 0.01)
    pos_ref, idx_ref = orc.nerf_grid_samples(cfg, n, orc_rng(orc, r), 3, grid, n_casc, 0.01)
    np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), idx_ref)
    np.testing.assert_array_equal(pos.cpu().numpy(), pos_ref)
    dens = g.uniform(-8, 3, (n, 16)).astype(np.float16)
    tmp = torch.full_like(grid_t, float("nan")) if binned else torch.zeros_like(grid_t)
    # the density network output is row-major [16 x n] (feature-major), density in row 0 (testbed_nerf.cu:3488-3496)
    pkg.nerf.grid_splat_max(idx, torch.from_numpy(np.ascontiguousarray(dens.T)).cuda(), 3, tmp, binned=binned)
    pkg.nerf.grid_ema(0.95, grid_t, tmp)
    ref_grid = grid.copy()
    orc.nerf_grid_splat_ema(idx_ref, dens[:, 0].copy().view(np.uint16), 3, ref_grid, 0.95)
    got = grid_t.cpu().numpy()
    # splat (atomicMax on the uint bits) and the EMA max-filter are exact float operations on the same
    # density bits: the whole grid is bit-exact
    np.testing.assert_array_equal(got.view(np.uint32), ref_grid.view(np.uint32))
    mean, bf = pkg.nerf.grid_mean_and_bitfield(grid_t, cfg.max_cascade)
    m = np.float32(mean[0].item())
    m_ref = np.float32(orc.nerf_grid_mean(ref_grid))
    assert m.view(np.uint32) == m_ref.view(np.uint32), (m, m_ref)  # the fixed reduction tree, restated
    np.testing.assert_array_equal(bf.cpu().numpy(), orc.nerf_grid_bitfield(ref_grid, cfg.max_cascade, float(m_ref)))


@pytest.mark.parametrize("seed,frac,scale", [(0, 0.3, 0.02), (1, 1.0, 1e-3), (2, 0.05, 5.0)])
def test_density_grid_mean_bitfield_bitexact(pkg, orc, seed, frac, scale):
    """update_density_grid_mean_and_bitfield (testbed_nerf.cu:3538-3567): the mean over cascade 0 and
    all 8 bitfield mips bit-exact from the grid alone (no GPU-provided mean), with thresholds that land
    on both sides of min(0.01, mean)."""
    g = np.random.default_rng(seed)
    grid = np.where(g.random(128 ** 3 * 8) < frac, g.random(128 ** 3 * 8) * scale, 0.0).astype(np.float32)
    grid[g.integers(0, grid.size, 5000)] = -1.0
    for max_cascade in (0, 3, 7):
        mean, bf = pkg.nerf.grid_mean_and_bitfield(torch.from_numpy(grid).cuda(), max_cascade)
        m = np.float32(mean[0].item())
        m_ref = np.float32(orc.nerf_grid_mean(grid))
        assert m.view(np.uint32) == m_ref.view(np.uint32), (m, m_ref)
        np.testing.assert_array_equal(bf.cpu().numpy(), orc.nerf_grid_bitfield(grid, max_cascade, float(m_ref)))


def test_nerf_training_end_to_end(pkg, orc):
    """Testbed-style training on the procedural scene: loss falls, occupancy grid prunes, the
    bitfield agrees with the oracle's restatement of the trainer's own density grid."""
    ds = pkg.synthetic.lego_like_dataset(n_images=12, width=128, height=128, seed=2)
    cfg = pkg.nerf.default_config(1.0)
    net = pkg.create_nerf_network(pkg.nerf_config("C2"))
    tr = pkg.Trainer(net, pkg.nerf_config("C2")["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    losses, stats = [], []
    for _ in range(700):
        s = run.train_step(get_loss=True)
        stats.append(s)
        losses.append(s["loss"])
    assert stats[-1]["step"] == 700
    assert all(np.isfinite(losses))
    assert np.mean(losses[-20:]) < 0.5 * np.mean(losses[:20])
    # compacted count before clamping to the batch (testbed_nerf.cu:3598); rays_per_batch adapts toward it
    assert 0 < stats[-1]["measured_batch_size"] <= stats[-1]["measured_batch_size_before_compaction"]
    assert stats[-1]["rays_per_batch"] % 256 == 0
    grid = run.density_grid.cpu().numpy()
    m = np.float32(run.mean_density.cpu().numpy()[0])
    bf = run.bitfield.cpu().numpy()
    assert grid.size == 128 ** 3 * (cfg.max_cascade + 1)
    full = np.zeros(128 ** 3 * 8, np.float32)
    full[:grid.size] = grid
    # the trainer's mean is the oracle's fixed-tree mean of the trainer's grid, bit for bit, and the
    # bitfield follows from the grid alone
    m_ref = np.float32(orc.nerf_grid_mean(full))
    assert m.view(np.uint32) == m_ref.view(np.uint32), (m, m_ref)
    np.testing.assert_array_equal(bf, orc.nerf_grid_bitfield(full, cfg.max_cascade, float(m_ref)))
    occupied = np.unpackbits(bf[:128 ** 3 // 8]).mean()
    assert 0.0 < occupied < 0.5  # the grid prunes once step >= 256 switches to the 0.01 threshold (:3518)


def test_training_error_map_window(pkg, orc):
    """The trainer's error map (testbed_nerf.cu:3659-3666, 1869-1899, 3700-3748): the first window is
    sized from 128 steps of the initial 4096 rays, its CDFs after step 128 equal the oracle's
    construct_cdf_2d/1d and host pass of the same map bit for bit, the next window is 1.5x longer and is
    sized from the current ray count, and a step deposits exactly its rays' losses."""
    n_img, W = 8, 96
    ds = pkg.synthetic.lego_like_dataset(n_images=n_img, width=W, height=W, seed=5)
    cfg = pkg.nerf.default_config(1.0)
    net = pkg.create_nerf_network(pkg.nerf_config("C2"))
    tr = pkg.Trainer(net, pkg.nerf_config("C2")["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    f = np.float32

    def side(between, rays):
        n = (between * rays) // n_img
        return min(int(f(np.sqrt(f(np.sqrt(f(n))))) * f(3.5)), W)

    stats = [run.train_step(get_loss=False) for _ in range(128)]
    em = run.error_map()
    k0 = side(128, 4096)
    assert (em["width"], em["height"], em["cdf_width"], em["cdf_height"]) == (k0, k0, k0, k0)
    assert em["cdf_valid"] == 1 and em["n_steps_since_update"] == 0 and em["n_steps_between_updates"] == 192
    data = em["data"]
    assert data.shape == (n_img, k0, k0) and (data >= 0).all() and data.sum() > 0
    cx, cy, ci = orc.error_map_cdfs(data)
    np.testing.assert_array_equal(em["cdf_x_cond_y"], cx)
    np.testing.assert_array_equal(em["cdf_y"], cy)
    pmf, cdf = orc.error_map_image_pmf(ci)
    np.testing.assert_array_equal(em["pmf_img"], pmf)
    np.testing.assert_array_equal(em["cdf_img"], cdf)
    R = stats[-1]["rays_per_batch"]
    s = run.train_step(get_loss=True)
    em = run.error_map()
    k1 = side(192, R)
    assert (em["width"], em["height"], em["n_steps_since_update"]) == (k1, k1, 1)
    # loss_scalar = sum_i(mean_loss_i / R) * measured / B (testbed_nerf.cu:3583-3609): the map holds sum_i mean_loss_i
    B = cfg.target_batch_size
    want = s["loss"] * B / s["measured_batch_size"] * R
    np.testing.assert_allclose(em["data"].sum(dtype=np.float64), want, rtol=1e-4)


def test_counters_follow_oracle_recurrence(pkg, orc):
    """Row a11: every step's rays_per_batch is NerfCounters::update_after_training
    (testbed_nerf.cu:3583-3609, oracle orc_nerf_counters_update) of the rays it traced and its measured
    counts, from the initial 4096 (testbed.h:440); the counts themselves are bit-exact with the oracle's
    sampler and compaction (test_generate_training_samples_*, test_compute_loss)."""
    ds = pkg.synthetic.lego_like_dataset(n_images=8, width=96, height=96, seed=5)
    cfg = pkg.nerf.default_config(1.0)
    net = pkg.create_nerf_network(pkg.nerf_config("C2"))
    tr = pkg.Trainer(net, pkg.nerf_config("C2")["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    B = cfg.target_batch_size
    R = 4096
    seen = set()
    for k in range(60):
        s = run.train_step(get_loss=(k % 7 == 0))
        r, mb, mbc, _ = orc.nerf_counters_update(R, B, s["measured_batch_size_before_compaction"], s["measured_batch_size"])
        assert (s["rays_per_batch"], s["measured_batch_size"], s["measured_batch_size_before_compaction"]) == (r, mb, mbc), k
        R = r  # (the compacted counter may exceed B: it counts every ray's request, :1825-1835)
        seen.add(R)
    assert seen != {4096}  # the ray count adapted (down: the untrained density keeps every ray long)


def test_inference_rgbd_layout(pkg):
    """NGP_LAYOUT_AOS_RGBD (the NeRF trainer's inference output) = rows 0..3 of the padded AoS output."""
    cfg = pkg.nerf_config("C2")
    cfg["encoding"]["log2_hashmap_size"] = 15
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"], seed=3)  # noqa: F841 (owns the parameters)
    g = np.random.default_rng(4)
    n = 3000  # ragged tail
    x = np.zeros((n, 7), np.float32)
    x[:, :3] = g.random((n, 3))
    x[:, 4:] = g.random((n, 3))
    xt = torch.from_numpy(x).cuda()
    full = net.inference(xt, layout=pkg.LAYOUT_AOS, use_inference_params=False)
    rgbd = net.inference(xt, layout=pkg.LAYOUT_AOS_RGBD, use_inference_params=False)
    torch.cuda.synchronize()
    assert rgbd.shape == (n, 4)
    np.testing.assert_array_equal(rgbd.cpu().numpy().view(np.uint16), full[:, :4].cpu().numpy().view(np.uint16))


@pytest.mark.gpu
@pytest.mark.parametrize("log2_T,max_level", [(15, 1.0), (19, 1.0), (19, 0.6)])
def test_fused_encoding_inference_bitwise(pkg, log2_T, max_level):
    """NerfNetwork inference with the grid encoding inside the MLP kernel (option fuse_infer, default) is
    bit-identical to encode-then-MLP (fuse_infer=0) for every output layout, dense and hashed levels,
    positions outside the unit cube and a lowered max level."""
    cfg = pkg.nerf_config("C2")
    cfg["encoding"]["log2_hashmap_size"] = log2_T
    net = pkg.create_nerf_network(cfg)
    g = np.random.default_rng(log2_T)
    params = torch.from_numpy((g.standard_normal(net.n_params) * 0.3).astype(np.float16)).cuda()
    net.set_params(params, params)
    net.set_max_level(max_level)
    n = 5000  # ragged tail
    x = np.zeros((n, 7), np.float32)
    x[:, :3] = g.uniform(-0.1, 1.1, (n, 3))
    x[:, 4:] = g.standard_normal((n, 3))
    x[:, 4:] /= np.linalg.norm(x[:, 4:], axis=1, keepdims=True)
    xt = torch.from_numpy(x).cuda()
    outs = {}
    for fuse in (1, 0):
        net.set_option("fuse_infer", fuse)
        for layout in (pkg.LAYOUT_AOS, pkg.LAYOUT_SOA, pkg.LAYOUT_AOS_RGBD):
            outs[fuse, layout] = net.inference(xt, layout=layout).cpu().numpy().view(np.uint16)
    for layout in (pkg.LAYOUT_AOS, pkg.LAYOUT_SOA, pkg.LAYOUT_AOS_RGBD):
        np.testing.assert_array_equal(outs[1, layout], outs[0, layout])
    assert np.isfinite(outs[1, pkg.LAYOUT_AOS].view(np.float16)[:, :4].astype(np.float32)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("aabb_scale", [1.0, 4.0])
def test_sampler_pipelining_is_exact(pkg, aabb_scale):
    """Launching the next step's sampler under the training pass (default), and the next density-grid update's
    sample generation and sort, trains exactly like the serial step: same per-step counts, same parameters,
    density grid and bitfield, bit for bit, across density-grid updates, growing ray counts, steps that read the
    loss back and steps where the caller takes writable buffers (discarding pregenerated update samples: the
    grid rng is restored). aabb_scale 4 (cone stepping) also runs the early counter publish: the next sampler under
    this step's loss pass 2 and training pass, writing the other of two sample sets."""
    ds = pkg.synthetic.lego_like_dataset(n_images=12, width=128, height=128, seed=5)
    cfg = pkg.nerf.default_config(aabb_scale)
    runs = []
    for pipeline in (True, False):
        net = pkg.create_nerf_network(pkg.nerf_config("C2"))
        tr = pkg.Trainer(net, pkg.nerf_config("C2")["optimizer"], seed=7)
        run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
        run.set_pipeline(pipeline)
        stats = []
        for i in range(300):
            stats.append(run.train_step(get_loss=(i % 37 == 0)))
            if i in (47, 271):  # updates due at steps 48 and 272 were pregenerated: discarded here
                run.writable_buffers()
        torch.cuda.synchronize()
        runs.append((stats, tr.serialize(), run.density_grid.cpu().numpy(), run.bitfield.cpu().numpy(), (net, tr, run)))
    (s1, p1, g1, b1, _), (s0, p0, g0, b0, _) = runs
    assert s1 == s0
    assert p1 == p0
    np.testing.assert_array_equal(g1, g0)
    np.testing.assert_array_equal(b1, b0)


@pytest.mark.parametrize("world,aabb_scale", [(2, 1.0), (4, 8.0), (3, 1.0)])
def test_sharded_samples_equal_single_gpu(pkg, orc, scene, world, aabb_scale):
    """rank r samples global rays [R r/N, R (r+1)/N) with their global ids (rng.advance(i*16),
    image_idx(i, R), testbed_nerf.cu:1417-1421), so the shards concatenated in rank order ARE the 1-GPU
    batch bit for bit: kept ray ids, rays, per-ray step counts and every sample coordinate; after
    compaction (dL/doutput scaled by 128/R globally) the compacted coordinates are bit-identical too and
    dL/doutput agrees to one fp16 ulp (128*Rl/R/Rl vs 128/R rounding)."""
    ds, ims, pix = scene
    cfg = pkg.nerf.default_config(aabb_scale)
    _, bf = occupancy(orc, seed=17, frac=0.35, max_cascade=cfg.max_cascade)
    bf_t = torch.from_numpy(bf).cuda()
    R, max_samples = 3000, 1 << 22
    r = rng(pkg, 4321)
    full = pkg.nerf.generate_training_samples(ds, cfg, R, r, max_samples, bf_t, n_rays_total=R)
    f = {k: v.cpu().numpy() for k, v in full.items()}
    kept_full, used_full = int(f["counters"][0]), int(f["counters"][1])
    assert 0 < used_full <= max_samples  # no ray dropped: the shards see the same budget
    g = np.random.default_rng(1)
    out = torch.from_numpy(g.uniform(-3.0, 2.0, (max_samples, 16)).astype(np.float16)).cuda()
    mean = torch.tensor([0.003], device="cuda")
    full_loss = pkg.nerf.compute_loss(ds, cfg, R, r, max_samples, {k: v.clone() for k, v in full.items()}, out, mean,
                                      n_rays_total=R)
    shards, losses = [], []
    base = 0
    for rank in range(world):
        lo, hi = pkg.dp.shard_range(R, rank, world)
        s = pkg.nerf.generate_training_samples(ds, cfg, hi - lo, r, max_samples, bf_t, ray_offset=lo, n_rays_total=R)
        sn = {k: v.cpu().numpy() for k, v in s.items()}
        used = int(sn["counters"][1])
        # the shard's network outputs are the full batch's rows of its samples
        out_s = out[base:base + max_samples].contiguous() if base + max_samples <= out.shape[0] else \
            torch.cat([out[base:], out[:base + max_samples - out.shape[0]]]).contiguous()
        shards.append(sn)
        losses.append(pkg.nerf.compute_loss(ds, cfg, hi - lo, r, max_samples, s, out_s, mean,
                                            loss_scale=128.0 * (hi - lo) / R, n_rays_total=R))
        base += used
    assert base == used_full
    cat = lambda k: np.concatenate([sh[k][:int(sh["counters"][0])] for sh in shards])
    np.testing.assert_array_equal(cat("ray_indices"), f["ray_indices"][:kept_full])
    np.testing.assert_array_equal(cat("rays"), f["rays"][:kept_full])
    np.testing.assert_array_equal(cat("numsteps")[:, 0], f["numsteps"][:kept_full, 0])
    coords = np.concatenate([sh["coords"][:int(sh["counters"][1])] for sh in shards])
    np.testing.assert_array_equal(coords, f["coords"][:used_full])
    cc = [int(l["compacted_counter"].cpu().numpy()[0]) for l in losses]
    cc_full = int(full_loss["compacted_counter"].cpu().numpy()[0])
    assert sum(cc) == cc_full
    co = np.concatenate([l["coords_compacted"].cpu().numpy()[:c] for l, c in zip(losses, cc)])
    np.testing.assert_array_equal(co, full_loss["coords_compacted"].cpu().numpy()[:cc_full])
    dl = np.concatenate([l["dloss_doutput"].cpu().numpy()[:c, :4].astype(np.float32) for l, c in zip(losses, cc)])
    dl_full = full_loss["dloss_doutput"].cpu().numpy()[:cc_full, :4]
    tol = np.spacing(np.abs(dl_full)).astype(np.float32) + 1e-7
    assert np.all(np.abs(dl - dl_full.astype(np.float32)) <= tol)
