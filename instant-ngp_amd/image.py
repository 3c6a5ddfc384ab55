"""Host mirror of the Testbed's image primitive (BASELINE config C1, src/testbed_image.cu) over the C-ABI.

`ImageTraining` is Testbed::train_image (testbed_image.cu:214-285): stratified random positions from
m_rng, snapped / bilinear sRGB targets from the RGBA float texture, tcnn training_step with the L2
loss, then optimizer_step(128). The random stream is Testbed::m_rng = default_rng_t{m_seed}
(src/testbed.cu:3906). Every call runs HIP; there is no CPU path.
"""
import ctypes as C

import numpy as np
import torch

from ._capi import ImageConfig, check, lib
from .nerf import pcg32
from .network import _ptr, _stream

RANDOM, STRATIFIED = 0, 3  # ERandomMode (common.h:124-130)


def default_config(**overrides):
    cfg = ImageConfig()
    check(lib().ngp_image_default_config(C.byref(cfg)))
    for k, v in overrides.items():
        setattr(cfg, k, int(v))
    return cfg


class Image:
    """Training image: RGBA float32 [H, W, 4] in linear colours (EDataType::Float, e.g. albert.exr)."""

    def __init__(self, rgba):
        rgba = np.ascontiguousarray(rgba, dtype=np.float32)
        if rgba.ndim != 3 or rgba.shape[2] != 4:
            raise ValueError(f"expected an [H, W, 4] RGBA array, got {rgba.shape}")
        self.height, self.width = rgba.shape[:2]
        h = C.c_void_p()
        check(lib().ngp_image_create(self.width, self.height, rgba.ctypes.data, C.byref(h)))
        self.handle = h

    @classmethod
    def load(cls, path):
        """Testbed::load_image (testbed_image.cu:372-402): .exr through the EXR reader (exr.py, tinyexr's
        LoadEXRFromMemory semantics), .npy as an [H, W, 4] float array; other formats raise."""
        p = str(path).lower()
        if p.endswith(".exr"):
            from .exr import read_exr
            return cls(read_exr(path))
        if p.endswith(".npy"):
            return cls(np.load(path))
        raise ValueError(f"unsupported image format: {path} (EXR or .npy)")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().ngp_image_destroy(h)
            except Exception:
                pass
            self.handle = None


class ImageTraining:
    """Testbed::train_image over a NetworkWithInputEncoding (2 -> 3) and its Trainer."""

    def __init__(self, network, trainer, image, cfg=None, seed=1337, batch_size=1 << 18):
        self.network, self.trainer, self.image = network, trainer, image
        self.cfg = cfg if cfg is not None else default_config()
        self.rng = pcg32(seed)
        self.batch_size = batch_size
        self.training_step = 0
        self._loss = torch.zeros(1, dtype=torch.float32, device="cuda")

    def generate_training_samples(self, n, stream=None):
        """generate_training_data (testbed_image.cu:223-265): positions [n, 2], targets [n, 3]."""
        pos = torch.empty((n, 2), dtype=torch.float32, device="cuda")
        tgt = torch.empty((n, 3), dtype=torch.float32, device="cuda")
        check(lib().ngp_image_generate_training_samples(self.image.handle, _stream(stream), n, C.byref(self.rng),
                                                        C.byref(self.cfg), _ptr(pos), _ptr(tgt)))
        return pos, tgt

    def train_step(self, get_loss=True, stream=None):
        if get_loss:
            self._loss.zero_()
        check(lib().ngp_image_train_step(self.image.handle, self.trainer.handle, _stream(stream), self.batch_size,
                                         C.byref(self.rng), C.byref(self.cfg), _ptr(self._loss) if get_loss else None))
        self.training_step += 1
        return float(self._loss.item()) if get_loss else None
