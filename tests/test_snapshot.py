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
