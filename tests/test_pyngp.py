"""The pybind11 Testbed surface (csrc/python_api.cpp over csrc/testbed_host.hpp; the reference's
src/python_api.cu:258-698, `import pyngp as ngp` in scripts/run.py:25) without a GPU: the module loads, carries
the reference's names and argument defaults, and its mode logic and default network configs are the
reference's (configs/<mode>/base.json as restated in instant-ngp_amd/config.py)."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ngp():
    from __graft_entry__ import load_package
    return load_package().pyngp()


def test_module_surface(ngp):
    for name in ("Testbed", "TestbedMode", "RenderMode", "LossType", "NerfActivation", "RandomMode", "mode_from_scene",
                 "mode_from_string"):
        assert hasattr(ngp, name), name
    assert int(ngp.TestbedMode.Nerf) == 0 and int(ngp.TestbedMode.Sdf) == 1 and int(ngp.TestbedMode.Image) == 2
    assert int(ngp.TestbedMode.Volume) == 3 and int(getattr(ngp.TestbedMode, "None")) == 4  # common.h:186-192
    assert int(ngp.RenderMode.Shade) == 1 and int(ngp.RenderMode.Normals) == 2  # common.h:110-119
    assert int(ngp.LossType.Huber) == 4 and int(ngp.LossType.SmoothL1) == 4
    T = ngp.Testbed
    for meth in ("load_training_data", "clear_training_data", "frame", "train", "reset", "reload_network_from_file",
                 "reload_network_from_json", "n_params", "n_encoding_params", "save_snapshot", "load_snapshot", "load_file",
                 "render", "set_camera_to_training_view", "first_training_view", "next_training_view"):
        assert callable(getattr(T, meth)), meth
    for prop in ("shall_train", "training_batch_size", "loss", "training_step", "mode", "nerf", "sdf", "image",
                 "background_color", "camera_matrix", "render_mode"):
        assert isinstance(getattr(T, prop), property), prop
    doc = T.save_snapshot.__doc__
    assert "include_optimizer_state: bool = False" in doc and "compress: bool = True" in doc
    import re
    assert re.search(r"width: [^=]+= 1920", T.render.__doc__) and re.search(r"spp: [^=]+= 1\b", T.render.__doc__)
    assert "reset_density_grid: bool = True" in T.reset.__doc__


def test_testbed_defaults_without_gpu(ngp):
    tb = ngp.Testbed()
    assert tb.mode == getattr(ngp.TestbedMode, "None")
    assert tb.shall_train is False and tb.training_batch_size == 1 << 18  # testbed.h:568,1005
    assert tb.training_step == 0 and tb.loss == 0.0
    assert list(tb.background_color) == [0.0, 0.0, 0.0, 1.0]  # testbed.h:936
    assert tb.render_mode == ngp.RenderMode.Shade
    tb.shall_train = True
    assert tb.frame() is True
    assert tb.shall_train is False  # Testbed::train without training data turns training off (testbed.cu:4286-4289)
    tb.training_batch_size = 1 << 16
    assert tb.training_batch_size == 1 << 16
    cam = tb.camera_matrix
    assert cam.shape == (3, 4)
    cam[:, 3] = [0.1, 0.2, 0.3]
    tb.camera_matrix = cam
    assert list(tb.camera_matrix[:, 3]) == pytest.approx([0.1, 0.2, 0.3])
    with pytest.raises(RuntimeError):
        tb.render(8, 8)  # no network


def test_mode_from_scene(ngp, tmp_path):
    (tmp_path / "transforms.json").write_text("{}")
    (tmp_path / "m.obj").write_text("v 0 0 0\n")
    (tmp_path / "i.exr").write_bytes(b"")
    (tmp_path / "v.nvdb").write_bytes(b"")
    assert ngp.mode_from_scene(str(tmp_path)) == ngp.TestbedMode.Nerf
    assert ngp.mode_from_scene(str(tmp_path / "transforms.json")) == ngp.TestbedMode.Nerf
    assert ngp.mode_from_scene(str(tmp_path / "m.obj")) == ngp.TestbedMode.Sdf
    assert ngp.mode_from_scene(str(tmp_path / "i.exr")) == ngp.TestbedMode.Image
    assert ngp.mode_from_scene(str(tmp_path / "v.nvdb")) == ngp.TestbedMode.Volume
    assert ngp.mode_from_scene(str(tmp_path / "missing.obj")) == getattr(ngp.TestbedMode, "None")
    assert ngp.mode_from_string("NeRF") == ngp.TestbedMode.Nerf and ngp.mode_from_string("x") == getattr(ngp.TestbedMode, "None")
    with pytest.raises(RuntimeError):
        ngp.Testbed().load_training_data(str(tmp_path / "missing.obj"))


def test_default_network_configs_match_config_py(ngp):
    from __graft_entry__ import load_package
    pkg = load_package()
    for mode, ref in ((ngp.TestbedMode.Nerf, pkg.NERF_BASE), (ngp.TestbedMode.Sdf, pkg.SDF_BASE),
                      (ngp.TestbedMode.Image, pkg.IMAGE_BASE)):
        assert json.loads(ngp.default_network_config(mode)) == ref
        assert json.loads(ngp.Testbed(mode).network_config) == ref
