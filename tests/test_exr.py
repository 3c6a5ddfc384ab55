"""CPU tests of the EXR reader (instant-ngp_amd/exr.py) behind the image primitive's load_exr_image
(src/testbed_image.cu:389-402 -> tinyexr LoadEXRFromMemory): round trips through the writer for every
supported compression and pixel type, and the reference's own albert.exr (BASELINE C1) when the
reference tree is present."""
import hashlib
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALBERT = [p for p in (os.path.join(ROOT, "data", "image", "albert.exr"), "/root/reference/data/image/albert.exr")
          if os.path.exists(p)]


@pytest.fixture(scope="module")
def exr():
    from __graft_entry__ import load_package
    return load_package().exr


@pytest.mark.parametrize("compression", [0, 2, 3])
@pytest.mark.parametrize("pixel_type", [1, 2])
@pytest.mark.parametrize("shape", [(37, 53), (16, 16), (1, 5), (33, 1)])
def test_round_trip(exr, tmp_path, compression, pixel_type, shape):
    rgba = np.random.default_rng(sum(shape)).uniform(-2, 5, shape + (4,)).astype(np.float32)
    p = tmp_path / "t.exr"
    exr.write_exr(p, rgba, compression, pixel_type)
    got = exr.read_exr(p)
    ref = rgba.astype(np.float16).astype(np.float32) if pixel_type == 1 else rgba
    assert got.dtype == np.float32 and np.array_equal(got, ref)


def test_rejects_other_files(exr, tmp_path):
    p = tmp_path / "x.exr"
    p.write_bytes(b"\x89PNG....")
    with pytest.raises(exr.ExrError):
        exr.read_exr(p)


@pytest.mark.skipif(not ALBERT, reason="albert.exr not staged (tools/stage_image.sh)")
def test_albert_exr():
    """configs[0]'s image: 1024^2, 4 FLOAT channels, ZIP. A wrong predictor or interleave would not
    survive as a smooth photograph; the digest pins the decode."""
    from __graft_entry__ import load_package
    im = load_package().exr.read_exr(ALBERT[0])
    assert im.shape == (1024, 1024, 4)
    assert np.all(im[..., 3] == 1.0)
    assert np.array_equal(im[..., 0], im[..., 1]) and np.array_equal(im[..., 1], im[..., 2])  # grey
    assert 0.0 < im[..., :3].min() and im[..., :3].max() < 1.0
    assert np.median(np.abs(np.diff(im[..., 0], axis=1))) < 0.01
    assert hashlib.sha1(im.tobytes()).hexdigest() == "6cffb407862605daa8fe3e594552a844c9e9f5d1"
