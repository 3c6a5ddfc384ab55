"""BASELINE C3 on the real capture: data/fox (tools/stage_fox.sh copies data/nerf/fox from the reference
tree; the 17 frames whose JPEGs are missing are dropped).

The fox loads through the dataset ingest (nerf_data.load_nerf: OpenCV lens, cx/cy, aabb_scale 8 -> 4
cascades) with every 10th frame held out as tools/fox_train.py does, so 45 frames are trained. A network is
trained for 1000 Testbed steps, which leaves a real occupancy grid and the adapted ray count. Then one
density-grid update of update_density_grid_nerf's step >= 256 form (testbed_nerf.cu:3412-3536: a quarter of
the cells uniformly, a quarter above the optical-thickness threshold, density network, splat, EMA, mean,
bitfield) and one sampling + compaction pass at that ray count (testbed_nerf.cu:1382-2012) run on the GPU
and are checked against the oracle on the same inputs: grid sample positions and cells, the splat+EMA grid
bits, the mean, all 8 bitfield mips, the sample counters, kept ray ids, rays, per-ray step counts and bases,
every sample coordinate, the compacted counter and every compacted coordinate, bit for bit. The density and
colour values fed to the oracle are the GPU network's (the MLP has its own per-element bars,
test_gpu_network_full.py), and dL/doutput is compared to 2 fp16 ulp (sRGB targets go through powf)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FOX = os.path.join(ROOT, "data", "fox")
N_CELLS = 128 ** 3


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


@pytest.fixture(scope="module")
def fox(pkg):
    if not os.path.isfile(os.path.join(FOX, "transforms.json")):
        pytest.skip("data/fox not staged (tools/stage_fox.sh)")
    d = pkg.nerf_data.load_nerf(FOX)
    test = [i for i in range(len(d)) if i % 10 == 5][:5]  # tools/fox_train.py's held-out frames
    train = [i for i in range(len(d)) if i not in test]
    ims = [d.images[i] for i in train]
    pix = [d.rgba8[i] for i in train]
    return d, pkg.nerf.NerfDataset(ims, pix), ims, pix


def _orc_rng(orc, r):
    return orc.pcg(r.state, r.inc)


def test_fox_capture_density_update_sampler_compaction(pkg, orc, fox):
    d, ds, ims, pix = fox
    assert len(d) == 50 and len(ims) == 45 and d.aabb_scale == 8
    assert ims[0].lens_mode == pkg.nerf.LENS_OPENCV
    cfg = pkg.nerf.default_config(d.aabb_scale)
    n_casc = cfg.max_cascade + 1
    assert n_casc == 4
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    for _ in range(1000):
        st = run.train_step(get_loss=False)
    torch.cuda.synchronize()
    R = int(st["rays_per_batch"])
    assert R % 256 == 0 and R != 4096  # adapted from the initial 4096 (testbed.h:440) toward B / samples per ray
    grid = np.zeros(N_CELLS * 8, np.float32)
    grid[:N_CELLS * n_casc] = run.density_grid.cpu().numpy()
    assert (grid[:N_CELLS * n_casc] < 0).any() and (grid > 0.01).any()  # untrained cells and occupied ones

    # ---- one density-grid update, step >= 256 form ----
    nq = N_CELLS // 4 * n_casc
    r_u, r_n = pkg.nerf.pcg32(77), pkg.nerf.pcg32(78)
    ema_step = 40
    grid_t = torch.from_numpy(grid).cuda()
    pos_u, idx_u = pkg.nerf.grid_generate_samples(cfg, nq, r_u, ema_step, grid_t, n_casc, -0.01)
    pos_n, idx_n = pkg.nerf.grid_generate_samples(cfg, nq, r_n, ema_step, grid_t, n_casc, 0.01)
    ref_pu, ref_iu = orc.nerf_grid_samples(cfg, nq, _orc_rng(orc, r_u), ema_step, grid, n_casc, -0.01)
    ref_pn, ref_in = orc.nerf_grid_samples(cfg, nq, _orc_rng(orc, r_n), ema_step, grid, n_casc, 0.01)
    np.testing.assert_array_equal(idx_u.cpu().numpy().view(np.uint32), ref_iu)
    np.testing.assert_array_equal(idx_n.cpu().numpy().view(np.uint32), ref_in)
    np.testing.assert_array_equal(pos_u.cpu().numpy(), ref_pu)
    np.testing.assert_array_equal(pos_n.cpu().numpy(), ref_pn)
    pos = torch.cat([pos_u, pos_n]).contiguous()
    idx = torch.cat([idx_u, idx_n]).contiguous()
    dens = net.density(pos, layout=pkg.LAYOUT_SOA, use_inference_params=False)  # [16 x n], density in row 0
    tmp = torch.full_like(grid_t, float("nan"))  # the trainer's binned splat writes every cell
    pkg.nerf.grid_splat_max(idx, dens, cfg.density_activation, tmp, binned=True)
    pkg.nerf.grid_ema(0.95, grid_t, tmp)
    ref_grid = grid.copy()
    orc.nerf_grid_splat_ema(np.concatenate([ref_iu, ref_in]), dens[0].cpu().numpy().view(np.uint16).copy(),
                            cfg.density_activation, ref_grid, 0.95)
    np.testing.assert_array_equal(grid_t.cpu().numpy().view(np.uint32), ref_grid.view(np.uint32))
    mean, bf = pkg.nerf.grid_mean_and_bitfield(grid_t, cfg.max_cascade)
    m = np.float32(mean[0].item())
    m_ref = np.float32(orc.nerf_grid_mean(ref_grid))
    assert m.view(np.uint32) == m_ref.view(np.uint32), (m, m_ref)
    bf_ref = orc.nerf_grid_bitfield(ref_grid, cfg.max_cascade, float(m_ref))
    np.testing.assert_array_equal(bf.cpu().numpy(), bf_ref)
    occ = np.unpackbits(bf_ref[:N_CELLS // 8]).mean()
    assert 0.0 < occ < 0.6, occ

    # ---- sampling at the trained ray count, on the new bitfield ----
    B = cfg.target_batch_size
    max_samples = 16 * B
    r = pkg.nerf.pcg32(4711)
    got = pkg.nerf.generate_training_samples(ds, cfg, R, r, max_samples, bf, n_rays_total=R)
    ref = orc.nerf_generate_samples(cfg, ims, pix, R, _orc_rng(orc, r), max_samples, bf_ref)
    g = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(g["counters"].view(np.uint32), ref["counters"])
    kept, steps = int(ref["counters"][0]), int(ref["counters"][1])
    assert kept > R // 2 and steps > B // 4
    np.testing.assert_array_equal(g["ray_indices"][:kept].view(np.uint32), ref["ray_indices"][:kept])
    np.testing.assert_array_equal(g["numsteps"][:kept].view(np.uint32), ref["numsteps"][:kept])
    np.testing.assert_array_equal(g["rays"][:kept], ref["rays"][:kept])
    used = min(steps, max_samples)
    np.testing.assert_array_equal(g["coords"][:used], ref["coords"][:used])

    # ---- loss and compaction with the trained network's outputs over those samples ----
    out = net.inference(got["coords"], layout=pkg.LAYOUT_AOS, use_inference_params=False)
    out_np = out.cpu().numpy()
    gl = pkg.nerf.compute_loss(ds, cfg, R, r, B, got, out, mean[:1].contiguous())
    rl = orc.nerf_compute_loss(cfg, ims, pix, R, _orc_rng(orc, r), B, ref, out_np.view(np.uint16), float(m_ref))
    cc = int(gl["compacted_counter"].cpu().numpy().view(np.uint32)[0])
    assert cc == int(rl["compacted_counter"][0]) and cc > B // 8
    np.testing.assert_array_equal(got["numsteps"].cpu().numpy()[:kept].view(np.uint32), ref["numsteps"][:kept])
    n_used = min(cc, B)
    np.testing.assert_array_equal(gl["coords_compacted"].cpu().numpy()[:n_used], rl["coords_compacted"][:n_used])
    np.testing.assert_allclose(gl["loss"].cpu().numpy()[:kept], rl["loss"][:kept], rtol=1e-4, atol=1e-9)
    dl_got = gl["dloss_doutput"].cpu().numpy().astype(np.float32)[:n_used, :4]
    dl_ref = orc.f16_bits_to_f32(rl["dloss_doutput"])[:n_used, :4]
    tol = 2 * np.spacing(np.abs(dl_ref).astype(np.float16)).astype(np.float32) + 1e-7
    bad = np.abs(dl_got - dl_ref) > tol
    assert not bad.any(), (int(bad.sum()), dl_got[bad][:5], dl_ref[bad][:5])
