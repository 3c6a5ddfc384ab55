"""Snapshot (.ingp) format: Testbed::save_snapshot / load_snapshot (src/testbed.cu:4873-5057).

CPU: the engine's msgpack/zlib reader against files written by the Python msgpack + gzip/zlib
libraries (the format nlohmann::json::to_msgpack + zstr produce). GPU: a trained NeRF saved and
loaded back (params bitwise, density grid as fp16, bitfield recomputed, counters and step)."""
import gzip
import zlib

import msgpack
import numpy as np
import pytest
import torch

@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    return load_package()


CONFIG = {
    "loss": {"otype": "Huber"},
    "optimizer": {"otype": "Ema", "decay": 0.95, "nested": {"otype": "ExponentialDecay", "decay_start": 20000,
                                                            "nested": {"otype": "Adam", "learning_rate": 1e-2}}},
    "encoding": {"otype": "HashGrid", "n_levels": 4, "n_features_per_level": 4, "log2_hashmap_size": 19,
                 "base_resolution": 16, "per_level_scale": 2.0},
    "network": {"otype": "FullyFusedMLP", "activation": "ReLU", "n_neurons": 64, "n_hidden_layers": 1},
}


def _snapshot_blob():
    snap = {"n_params": 3, "params_type": "__half", "params_binary": np.arange(3, dtype=np.float16).tobytes(),
            "version": 1, "mode": "nerf", "density_grid_size": 128, "training_step": 7, "loss": 0.25,
            "aabb": {"min": [0.0, 0.0, 0.0], "max": [1.0, 1.0, 1.0]}}
    return msgpack.packb(dict(CONFIG, snapshot=snap), use_bin_type=True)


@pytest.mark.parametrize("kind", ["gzip", "zlib", "raw"])
def test_network_config_from_snapshot(pkg, tmp_path, kind):
    blob = _snapshot_blob()
    data = {"gzip": gzip.compress, "zlib": zlib.compress, "raw": lambda b: b}[kind](blob)
    path = tmp_path / ("s.ingp" if kind != "raw" else "s.msgpack")
    path.write_bytes(data)
    assert pkg.nerf.snapshot_network_config(str(path)) == CONFIG


def test_snapshot_without_member_is_rejected(pkg, tmp_path):
    path = tmp_path / "cfg.msgpack"
    path.write_bytes(msgpack.packb(CONFIG))
    assert pkg.nerf.snapshot_network_config(str(path)) == CONFIG  # a plain config reads fine
    bad = tmp_path / "bad.ingp"
    bad.write_bytes(gzip.compress(b"\xc1"))  # reserved msgpack byte
    with pytest.raises(Exception):
        pkg.nerf.snapshot_network_config(str(bad))


def _scene(pkg):
    S = pkg.synthetic
    ims, pix = [], []
    for c2w in S.camera_poses(6, seed=2):
        ims.append(pkg.nerf.make_image(64, 64, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X))
        pix.append(S.render(c2w, 64, 64))
    return pkg.nerf.NerfDataset(ims, pix)


def _training(pkg, ds):
    cfg = pkg.nerf.default_config(1.0)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    return pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337), net, tr, ncfg


@pytest.mark.gpu
@pytest.mark.parametrize("with_opt", [False, True])
def test_nerf_snapshot_roundtrip(pkg, orc, tmp_path, with_opt):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ds = _scene(pkg)
    run, net, tr, ncfg = _training(pkg, ds)
    for _ in range(300):
        st = run.train_step(get_loss=True)
    torch.cuda.synchronize()
    path = tmp_path / "lego.ingp"
    run.save_snapshot(str(path), ncfg, include_optimizer_state=with_opt)
    raw = msgpack.unpackb(gzip.decompress(path.read_bytes()), raw=False)
    snap = raw.pop("snapshot")
    assert raw == ncfg
    assert snap["version"] == 1 and snap["mode"] == "nerf" and snap["density_grid_size"] == 128
    assert snap["params_type"] == "__half" and snap["n_params"] == net.n_params
    assert snap["params_binary"] == tr.params.cpu().numpy().tobytes()
    grid16 = run.density_grid.cpu().numpy().astype(np.float16)
    assert snap["density_grid_binary"] == grid16.tobytes()
    assert snap["training_step"] == st["step"] and snap["nerf"]["rgb"]["rays_per_batch"] == st["rays_per_batch"]
    assert ("optimizer" in snap) == with_opt

    run2, net2, tr2, _ = _training(pkg, ds)
    assert pkg.nerf.snapshot_network_config(str(path)) == ncfg
    run2.load_snapshot(str(path))
    torch.cuda.synchronize()
    assert tr2.params.cpu().numpy().tobytes() == tr.params.cpu().numpy().tobytes()
    np.testing.assert_array_equal(run2.density_grid.cpu().numpy(), grid16.astype(np.float32))
    m = float(run2.mean_density.cpu().numpy()[0])
    cfg = pkg.nerf.default_config(1.0)
    np.testing.assert_array_equal(run2.bitfield.cpu().numpy(),
                                  orc.nerf_grid_bitfield(grid16.astype(np.float32), cfg.max_cascade, m))
    if with_opt:
        assert tr2.step == tr.step
    st2 = run2.train_step(get_loss=True)
    assert st2["step"] == st["step"] + 1 and np.isfinite(st2["loss"])


@pytest.mark.gpu
def test_resume_past_density_update_rerecords_graph(pkg, tmp_path):
    """Loading a snapshot at step >= 256 and training past the next density-grid update: that update
    grows the encoding workspace the captured training graph points into, so the trainer must re-record
    (ngp_model_workspace_epoch). Control: the same resume on a model whose workspaces were reserved for
    the density pass up front (nothing reallocates) — both runs must match bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ds = _scene(pkg)
    run, net, tr, ncfg = _training(pkg, ds)
    for _ in range(300):
        run.train_step(get_loss=False)
    path = tmp_path / "resume.ingp"
    run.save_snapshot(str(path), ncfg, include_optimizer_state=True)
    results = []
    for reserve_first in (False, True):
        run2, net2, tr2, _ = _training(pkg, ds)
        if reserve_first:
            net2.reserve(128 ** 3 * (run2.cfg.max_cascade + 1))
        run2.load_snapshot(str(path))
        e0 = pkg.lib().ngp_model_workspace_epoch(net2.handle)
        for _ in range(40):  # density updates every 16 steps after step 256
            st = run2.train_step(get_loss=True)
            assert np.isfinite(st["loss"])
        torch.cuda.synchronize()
        if not reserve_first:
            assert pkg.lib().ngp_model_workspace_epoch(net2.handle) > e0  # the density pass did grow a workspace
        results.append((tr2.params_full_precision.cpu().numpy().copy(), run2.density_grid.cpu().numpy().copy()))
    np.testing.assert_array_equal(results[0][0], results[1][0])
    np.testing.assert_array_equal(results[0][1], results[1][1])


@pytest.mark.gpu
def test_learning_rate_change_reaches_captured_steps(pkg):
    """set_learning_rate after the NeRF training graph was captured changes the replayed optimizer
    steps (the captured Adam reads its hyperparameters from the device control block)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ds = _scene(pkg)
    out = []
    for lr in (None, 0.0):
        run, net, tr, ncfg = _training(pkg, ds)
        for _ in range(5):
            run.train_step(get_loss=False)
        if lr is not None:
            tr.learning_rate = lr
        w0 = tr.params_full_precision.cpu().numpy().copy()
        for _ in range(3):
            run.train_step(get_loss=False)
        torch.cuda.synchronize()
        out.append(np.abs(tr.params_full_precision.cpu().numpy() - w0).max())
    assert out[0] > 0
    assert out[1] == 0  # lr 0: the replayed steps leave the weights unchanged
