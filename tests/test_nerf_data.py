"""Dataset ingest (instant-ngp_amd/nerf_data.py, restating src/nerf_loader.cu load_nerf) and the lens
models of the oracle (oracle/ngp_nerf_oracle.c lens_undistort, common_device.cuh:288-378). CPU only:
the dataset is written to a temporary directory in the fox transforms.json format; nothing is read
from the reference tree."""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

FOX = {"camera_angle_x": 0.7481849417937728, "camera_angle_y": 1.2193576119562444, "fl_x": 1375.52, "fl_y": 1374.49,
       "k1": 0.0578421, "k2": -0.0805099, "p1": -0.000980296, "p2": 0.00015575, "cx": 554.558, "cy": 965.268,
       "w": 54.0, "h": 96.0, "aabb_scale": 8}


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    return load_package()


def _opencv_distort(k, u, v):
    """forward OpenCV model in float64 (independent of the restatement under test)"""
    r2 = u * u + v * v
    radial = k[0] * r2 + k[1] * r2 * r2
    return (u + u * radial + 2 * k[2] * u * v + k[3] * (r2 + 2 * u * u),
            v + v * radial + 2 * k[3] * u * v + k[2] * (r2 + 2 * v * v))


def _fisheye_distort(k, u, v):
    r = math.hypot(u, v)
    th = math.atan(r)
    thd = th * (1 + k[0] * th ** 2 + k[1] * th ** 4 + k[2] * th ** 6 + k[3] * th ** 8)
    return (u * thd / r, v * thd / r) if r > 0 else (u, v)


@pytest.mark.parametrize("mode,k,fwd", [(1, FOX["k1"], None), (1, -0.25, None), (2, 0.05, None)])
def test_oracle_undistort_inverts_distortion(orc, mode, k, fwd):
    kk = (FOX["k1"], FOX["k2"], FOX["p1"], FOX["p2"]) if k == FOX["k1"] else (k, 0.04, 0.001, -0.002)
    if mode == 2:
        kk = (k, -0.01, 0.002, 0.0)
    lib = orc.lib()
    f = lib.orc_lens_undistort
    f.restype = None
    f.argtypes = [C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    karr = (C.c_float * 4)(*kk)
    g = np.random.default_rng(mode)
    for u0, v0 in g.uniform(-0.6, 0.6, (200, 2)):
        u, v = C.c_float(u0), C.c_float(v0)
        f(mode, karr, C.byref(u), C.byref(v))
        du, dv = (_opencv_distort if mode == 1 else _fisheye_distort)(kk, u.value, v.value)
        assert abs(du - u0) < 2e-5 and abs(dv - v0) < 2e-5, (u0, v0, du, dv)
    u, v = C.c_float(0.3), C.c_float(-0.2)
    f(0, karr, C.byref(u), C.byref(v))  # perspective: untouched
    assert (u.value, v.value) == (np.float32(0.3), np.float32(-0.2))


def _write_dataset(tmp, frames, top=None, fmt="jpg"):
    from PIL import Image
    os.makedirs(os.path.join(tmp, "images"), exist_ok=True)
    g = np.random.default_rng(0)
    for fr in frames:
        if fr.get("_missing"):
            continue
        img = g.integers(0, 256, (96, 54, 3), dtype=np.uint8)
        Image.fromarray(img).save(os.path.join(tmp, fr["file_path"]))
    j = dict(FOX if top is None else top)
    j["frames"] = [{k: v for k, v in fr.items() if not k.startswith("_")} for fr in frames]
    with open(os.path.join(tmp, "transforms.json"), "w") as f:
        f.write("// comment line, as nlohmann ignore_comments allows\n" + json.dumps(j))
    return os.path.join(tmp, "transforms.json")


def _frame(i, missing=False, sharp=30.0, fmt="jpg"):
    a = 0.3 * i
    m = [[math.cos(a), 0, math.sin(a), 3 * math.sin(a)], [0, 1, 0, 0.2 * i], [-math.sin(a), 0, math.cos(a), 3 * math.cos(a)],
         [0, 0, 0, 1]]
    return {"file_path": f"images/{i:04d}.{fmt}", "sharpness": sharp, "transform_matrix": m, "_missing": missing}


def test_load_fox_format(pkg, tmp_path):
    frames = [_frame(i, missing=(i in (3, 7))) for i in (10, 2, 1, 3, 4, 5, 6, 7, 8, 9)]
    path = _write_dataset(str(tmp_path), frames)
    d = pkg.nerf_data.load_nerf(path)
    # missing files are dropped by the sharpness filter (nerf_loader.cu:365), frames in natural order
    names = [os.path.basename(p) for p in d.paths]
    assert names == ["0001.jpg", "0002.jpg", "0004.jpg", "0005.jpg", "0006.jpg", "0008.jpg", "0009.jpg", "0010.jpg"]
    assert d.aabb_scale == 8 and d.scale == pytest.approx(0.33) and d.offset == [0.5, 0.5, 0.5]
    im = d.images[0]
    assert (im.width, im.height) == (54, 96)
    assert im.lens_mode == pkg.nerf.LENS_OPENCV
    np.testing.assert_allclose(list(im.lens_params), [FOX["k1"], FOX["k2"], FOX["p1"], FOX["p2"]], rtol=1e-6)
    np.testing.assert_allclose(list(im.principal_point), [FOX["cx"] / FOX["w"], FOX["cy"] / FOX["h"]], rtol=1e-6)
    np.testing.assert_allclose(list(im.focal_length), [FOX["fl_x"], FOX["fl_y"]], rtol=1e-6)
    # nerf_matrix_to_ngp of frame 0001 (scale 0.33, offset 0.5)
    m = np.asarray(_frame(1)["transform_matrix"], np.float32)
    np.testing.assert_allclose(np.asarray(im.xform), pkg.nerf.nerf_matrix_to_ngp(m, 0.33, (0.5, 0.5, 0.5)), rtol=1e-6)
    assert d.rgba8[0].shape == (96, 54, 4) and np.all(d.rgba8[0][..., 3] == 255)


def test_load_overrides_and_transparency(pkg, tmp_path):
    top = {"camera_angle_x": 0.69, "white_transparent": True, "scale": 0.5, "offset": [0.4, 0.5, 0.6], "aabb_scale": 2}
    frames = [_frame(i, fmt="png") for i in range(1, 4)]
    for fr in frames:
        del fr["sharpness"]
    frames[1]["fl_x"] = 77.0  # per-frame intrinsics override
    frames[2].update({"k1": -0.1, "is_fisheye": True, "cx": 20.0, "w": 54.0})  # per-frame lens override
    path = _write_dataset(str(tmp_path), frames, top=top, fmt="png")
    from PIL import Image
    img = np.array(Image.open(os.path.join(str(tmp_path), "images/0001.png")).convert("RGB"))
    img[:4, :4] = 255
    Image.fromarray(img).save(os.path.join(str(tmp_path), "images/0001.png"))
    d = pkg.nerf_data.load_nerf(path)
    assert len(d) == 3 and d.scale == 0.5 and d.offset == [0.4, 0.5, 0.6]
    f0 = 0.5 * 54 / math.tan(0.5 * 0.69)
    assert d.images[0].focal_length[0] == pytest.approx(f0, rel=1e-6)
    assert d.images[1].focal_length[0] == pytest.approx(77.0)
    assert d.images[0].lens_mode == 0 and d.images[2].lens_mode == pkg.nerf.LENS_OPENCV_FISHEYE
    assert d.images[2].principal_point[0] == pytest.approx(20.0 / 54.0)
    assert np.all(d.rgba8[0][:4, :4, 3] == 0)  # white -> transparent (convert_rgba32)


def test_load_errors(pkg, tmp_path):
    frames = [_frame(1)]
    del frames[0]["sharpness"]
    frames[0]["_missing"] = True
    path = _write_dataset(str(tmp_path), frames)
    with pytest.raises(FileNotFoundError):
        pkg.nerf_data.load_nerf(path)
