"""The pybind11 Testbed (`pyngp`, csrc/python_api.cpp over csrc/testbed_host.hpp) on the GPU: the reference's
scripting flow (scripts/run.py: Testbed(), load_training_data, shall_train, `while testbed.frame()`,
save_snapshot / load_snapshot, render) on a procedural NeRF scene written to disk as transforms.json + PNGs.

* 200 frames train the scene; the C++ Testbed trains bit for bit like the package's Python Testbed mirror
  (nerf.NerfTraining) on the same files and seeds: the renders of the two networks are identical.
* A snapshot written by one Testbed and loaded by another gives the same training step and the same render.
* SDF (armadillo.obj, when staged) and image (.npy) Testbeds train through the same surface."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


@pytest.fixture(scope="module")
def scene_dir(pkg, tmp_path_factory):
    from PIL import Image
    S = pkg.synthetic
    d = tmp_path_factory.mktemp("standin")
    frames = []
    for i, c2w in enumerate(S.camera_poses(16, seed=4)):
        Image.fromarray(S.render(c2w, 96, 96)).save(d / f"r_{i}.png")
        frames.append({"file_path": f"./r_{i}", "transform_matrix": np.asarray(c2w, np.float64).tolist()})
    (d / "transforms.json").write_text(json.dumps({"camera_angle_x": S.LEGO_CAMERA_ANGLE_X, "frames": frames}))
    return str(d)


def test_testbed_trains_like_the_python_mirror_and_round_trips_a_snapshot(pkg, scene_dir, tmp_path):
    ngp = pkg.pyngp()
    tb = ngp.Testbed()
    tb.load_training_data(scene_dir)
    assert tb.mode == ngp.TestbedMode.Nerf
    assert tb.nerf.training.dataset.n_images == 16
    tb.shall_train = True
    losses = []
    while tb.frame():
        if tb.training_step % 16 == 1:  # the loss is read back every 16 steps (testbed.cu:4346)
            losses.append(tb.loss)
        if tb.training_step >= 200:
            break
    assert tb.training_step == 200
    assert tb.n_params() == 3302400 and tb.n_encoding_params() == 3293184
    assert all(np.isfinite(losses)) and np.mean(losses[-3:]) < 0.5 * losses[0]
    tb.set_camera_to_training_view(3)
    img = tb.render(64, 48, spp=1, linear=True)
    assert img.shape == (48, 64, 4) and np.isfinite(img).all() and img[..., :3].max() > 0.05

    # the Python Testbed mirror on the same files and seeds (Trainer / NerfTraining seed 1337)
    d = pkg.nerf_data.load_nerf(scene_dir)
    ds = pkg.nerf.NerfDataset(d.images, d.rgba8)
    cfg = pkg.nerf.default_config(d.aabb_scale)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"], seed=1337)
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    for k in range(200):
        run.train_step(get_loss=(k % 16 == 0))
    im3 = d.images[3]
    # the Testbed's float arithmetic: relative focal length (set_camera_to_training_view) x the render height
    f32 = np.float32
    focal = tuple(float(f32(f32(im3.focal_length[k]) / f32(im3.height)) * f32(48)) for k in range(2))
    cam = pkg.nerf.make_image(64, 48, list(im3.xform), focal=focal, principal=tuple(im3.principal_point))
    ref = pkg.nerf.NerfRenderer().render(net, cfg, cam, run.bitfield, spp=1, background=(0, 0, 0, 1)).cpu().numpy()
    np.testing.assert_array_equal(img, ref)
    # ERenderMode::Depth through the Testbed: depth in the dataset's units (depth_scale = 1 / dataset scale,
    # testbed_nerf.cu:2822), the same frame as the renderer called directly
    tb.render_mode = ngp.RenderMode.Depth
    depth = tb.render(64, 48, spp=1, linear=True)
    tb.render_mode = ngp.RenderMode.Shade
    ref_d = pkg.nerf.NerfRenderer().render(net, cfg, cam, run.bitfield, spp=1, background=(0, 0, 0, 1), render_mode="Depth",
                                           depth_scale=1.0 / d.scale).cpu().numpy()
    np.testing.assert_array_equal(depth, ref_d)
    assert np.isfinite(depth).all() and depth[..., 0].max() > 0.1

    # snapshot round trip into a fresh Testbed: the parameters, optimizer state and fp16 density grid it
    # restores are the ones saved (its own snapshot carries them unchanged), and it renders what the
    # Python mirror renders after loading the same file (after a load the inference parameters are the
    # loaded parameters and the bitfield follows from the fp16 grid, testbed.cu:4939-5057)
    import gzip
    import msgpack
    snap, snap2 = str(tmp_path / "standin.ingp"), str(tmp_path / "standin2.ingp")
    tb.save_snapshot(snap, include_optimizer_state=True, compress=True)
    tb2 = ngp.Testbed()
    tb2.load_training_data(scene_dir)
    tb2.load_snapshot(snap)
    assert tb2.training_step == 200
    tb2.save_snapshot(snap2, include_optimizer_state=True, compress=True)
    a, b = (msgpack.unpackb(gzip.decompress(open(p, "rb").read()), raw=False) for p in (snap, snap2))
    for key in ("params_binary", "density_grid_binary"):
        va = a["snapshot"][key] if key in a["snapshot"] else a[key]
        vb = b["snapshot"][key] if key in b["snapshot"] else b[key]
        assert len(va) > 0 and va == vb, key
    tb2.set_camera_to_training_view(3)
    img2 = tb2.render(64, 48, spp=1, linear=True)
    run.load_snapshot(snap)
    ref2 = pkg.nerf.NerfRenderer().render(net, cfg, cam, run.bitfield, spp=1, background=(0, 0, 0, 1)).cpu().numpy()
    np.testing.assert_array_equal(img2, ref2)
    assert np.abs(img2 - img).mean() < 0.05  # the EMA (inference) parameters before saving vs the loaded ones
    # shall_train off: frame() renders nothing and trains nothing
    tb2.shall_train = False
    tb2.frame()
    assert tb2.training_step == 200
    # a live knob reaches the trainer: no random background, then training continues
    tb.nerf.training.random_bg_color = False
    assert tb.nerf.training.random_bg_color == 0
    tb.train(1 << 18)
    assert tb.training_step == 201
    tb.reset()
    assert tb.training_step == 0


def test_testbed_sdf_and_image_modes(pkg, tmp_path):
    ngp = pkg.pyngp()
    arm = os.path.join(ROOT, "data", "sdf", "armadillo.obj")
    if os.path.isfile(arm):
        tb = ngp.Testbed()
        tb.load_training_data(arm)
        assert tb.mode == ngp.TestbedMode.Sdf
        tb.shall_train = True
        tb.training_batch_size = 1 << 16
        for _ in range(33):
            tb.frame()
        assert tb.training_step == 33 and np.isfinite(tb.loss) and tb.loss > 0
        _snapshot_round_trip(ngp, tb, tmp_path / "arm.ingp", ngp.TestbedMode.Sdf, arm)
    img = pkg.synthetic.synthetic_image(64, 48, seed=2)
    path = tmp_path / "img.npy"
    np.save(path, img.astype(np.float32))
    tb = ngp.Testbed()
    tb.load_training_data(str(path))
    assert tb.mode == ngp.TestbedMode.Image
    tb.reload_network_from_json({**pkg.IMAGE_BASE, "encoding": {**pkg.IMAGE_BASE["encoding"], "log2_hashmap_size": 14}})
    tb.shall_train = True
    tb.training_batch_size = 1 << 14
    first = None
    for _ in range(200):
        tb.frame()
        if tb.training_step == 1:
            first = tb.loss
    out = tb.render(64, 48, spp=1, linear=True)
    assert out.shape == (48, 64, 4) and np.isfinite(out).all()
    assert tb.loss < first
    _snapshot_round_trip(ngp, tb, tmp_path / "img.ingp", ngp.TestbedMode.Image, str(path))
    # after a load the inference parameters are the loaded parameters (testbed.cu:5040): a fresh Testbed and the
    # first one reloading its own snapshot render the same frame
    tb3 = ngp.Testbed()
    tb3.load_training_data(str(path))
    tb3.load_snapshot(str(tmp_path / "img.ingp"))
    tb.load_snapshot(str(tmp_path / "img.ingp"))
    np.testing.assert_array_equal(tb3.render(64, 48, spp=1, linear=True), tb.render(64, 48, spp=1, linear=True))


def _snapshot_round_trip(ngp, tb, path, mode, data):
    """Testbed::save_snapshot / load_snapshot for the SDF and image testbeds (testbed.cu:4873-5057): a fresh Testbed
    loads the file (its mode from the snapshot), holds the same training step and network, writes the same
    parameters and optimizer state back, and trains on."""
    import gzip
    import msgpack
    tb.save_snapshot(str(path), include_optimizer_state=True, compress=True)
    tb2 = ngp.Testbed()
    tb2.load_training_data(data)
    tb2.load_snapshot(str(path))
    assert tb2.mode == mode and tb2.training_step == tb.training_step and tb2.n_params() == tb.n_params()
    path2 = str(path) + ".2.ingp"
    tb2.save_snapshot(path2, include_optimizer_state=True, compress=True)
    a, b = (msgpack.unpackb(gzip.decompress(open(p, "rb").read()), raw=False)["snapshot"] for p in (str(path), path2))
    assert a["mode"] == b["mode"] == {ngp.TestbedMode.Sdf: "sdf", ngp.TestbedMode.Image: "image"}[mode]
    assert a["params_binary"] == b["params_binary"] and len(a["params_binary"]) == 2 * tb.n_params()
    for k, v in a["optimizer"].items():
        assert b["optimizer"][k] == v, k
    assert a["aabb"] == b["aabb"] and a["training_step"] == b["training_step"]
    tb2.shall_train = True
    for _ in range(3):
        tb2.frame()
    assert tb2.training_step == tb.training_step + 3 and np.isfinite(tb2.loss)
    return tb2


def _dense_entries(levels, b, nmin=16, d=3):
    """tcnn's offset table for a DenseGrid: res^D rounded to 8 per level, no hashmap cap (float32 as the engine)."""
    f32 = np.float32
    total = 0
    for l in range(levels):
        s = f32(np.exp2(f32(l) * np.log2(f32(b)))) * f32(nmin) - f32(1)
        res = int(np.ceil(s)) + 1
        total += (res ** d + 7) // 8 * 8
    return total


def test_reload_network_keeps_the_configs_per_level_scale(pkg, scene_dir, tmp_path):
    """reset_network (testbed.cu:3975-3997, 4037): the fork writes 2.0 only into its log member, so a config's own
    per_level_scale reaches the encoding (configs/nerf/densegrid.json: DenseGrid, 8 levels, b = 1.405), and a
    missing base_resolution becomes 2^(log2_hashmap_size / 3)."""
    ngp = pkg.pyngp()
    (tmp_path / "base.json").write_text(ngp.default_network_config(ngp.TestbedMode.Nerf))
    (tmp_path / "densegrid.json").write_text(
        '{\t// multiresolution dense grid - 8 levels, from res 16 to 173\n\t"parent" : "base.json",\n'
        '\t"encoding": {"otype": "DenseGrid", "n_levels": 8, "base_resolution": 16, "per_level_scale": 1.405}\n}\n')
    tb = ngp.Testbed()
    tb.load_training_data(scene_dir)
    tb.reload_network_from_file(str(tmp_path / "densegrid.json"))
    assert tb.n_encoding_params() == 4 * _dense_entries(8, 1.405)  # base.json's 4 features per level
    tb.shall_train = True
    for _ in range(3):
        tb.frame()
    assert tb.training_step == 3 and np.isfinite(tb.loss)
    # a hash grid with its own scale and no base_resolution: N_min = 2^(15 / 3) = 32 with the default T = 2^15
    (tmp_path / "own.json").write_text('{"parent": "base.json", "encoding": {"otype": "HashGrid", "n_levels": 2, '
                                       '"n_features_per_level": 2, "log2_hashmap_size": 15, "base_resolution": 0, '
                                       '"per_level_scale": 1.5}}')
    tb.reload_network_from_file(str(tmp_path / "own.json"))
    res = [32, int(np.ceil(np.float32(1.5) * np.float32(32) - np.float32(1))) + 1]
    assert tb.n_encoding_params() == 2 * sum(min((r ** 3 + 7) // 8 * 8, 1 << 15) for r in res)
    assert json.loads(tb.network_config)["encoding"]["per_level_scale"] == 1.5
