"""instant-ngp hot path on MI355X (gfx950): HIP hash-grid encoding, MFMA fully-fused MLPs,
NeRF training kernels, behind the C-ABI in include/ngp_engine.h.

The directory name is not a Python identifier; load it as `instant_ngp_amd` via
__graft_entry__.load_package() (tests/conftest.py does the same).
"""
from . import dp, exr, image, nerf, nerf_data, sdf, synthetic  # noqa: F401
from ._capi import NgpError, lib  # noqa: F401
from .config import IMAGE_BASE, NERF_BASE, SDF_BASE, load_config, merge_patch, nerf_config  # noqa: F401
from .network import (GRAD_ACCUMULATE, GRAD_IGNORE, GRAD_OVERWRITE, LAYOUT_AOS, LAYOUT_AOS_RGBD, LAYOUT_SOA, Model, NerfNetwork,  # noqa: F401
                      NetworkWithInputEncoding, Trainer, TrainingGraph, loss_evaluate, wrap_device)


def create_nerf_network(cfg, n_pos_dims=3, n_dir_dims=3, n_extra_dims=0, dir_offset=4):
    """Testbed::reset_network's NerfNetwork construction (src/testbed.cu:4029-4042)."""
    return NerfNetwork(n_pos_dims, n_dir_dims, n_extra_dims, dir_offset, cfg["encoding"], cfg.get("dir_encoding"),
                       cfg["network"], cfg["rgb_network"])


def pyngp():
    """The pybind11 Testbed module (csrc/python_api.cpp, built into lib/ by build()): the reference's
    `import pyngp as ngp` surface (src/python_api.cu)."""
    import importlib
    import os
    import sys
    lib_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
    if lib_dir not in sys.path:
        sys.path.insert(0, lib_dir)
    return importlib.import_module("pyngp")
