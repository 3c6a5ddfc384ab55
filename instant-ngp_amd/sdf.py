"""Host mirror of the Testbed's SDF primitive (BASELINE config C5, src/testbed_sdf.cu) over the C-ABI.

`load_mesh` restates Testbed::load_mesh's normalisation (testbed_sdf.cu:1120-1165); `SdfTraining` is
training_prep_sdf + train_sdf (:1289-1330): every step regenerates the batch online
(generate_training_samples_sdf, :1187-1275, non-octree branch), shuffles it and runs tcnn
training_step with the MAPE loss (configs/sdf/base.json) and the optimizer. Signed distances come
from a 4-ary triangle BVH (TriangleBvh4, src/triangle_bvh.cu; csrc/bvh.hip) traversed on the GPU.
"""
import ctypes as C

import numpy as np
import torch

from ._capi import check, lib
from .nerf import pcg32
from .network import _ptr, _stream


def load_mesh(vertices):
    """Normalise triangle-soup vertices [3T, 3] into the unit cube as Testbed::load_mesh does.
    Returns (triangles [T, 9] float32, aabb_min, aabb_max, bounding_radius)."""
    v = np.asarray(vertices, dtype=np.float32).reshape(-1, 3)
    if v.shape[0] % 3 != 0 or v.shape[0] == 0:
        raise ValueError("vertices must hold whole triangles")
    inflation = np.float32(0.005)
    lo, hi = v.min(axis=0), v.max(axis=0)
    amount = np.float32(np.linalg.norm(hi - lo)) * inflation
    lo, hi = lo - amount, hi + amount
    diag = hi - lo
    scale = np.float32(diag.max())
    v = (v - lo - np.float32(0.5) * diag) / scale + np.float32(0.5)
    alo, ahi = v.min(axis=0), v.max(axis=0)
    amount = np.float32(np.linalg.norm(ahi - alo)) * inflation
    alo, ahi = np.maximum(alo - amount, 0.0), np.minimum(ahi + amount, 1.0)  # intersection with [0,1]^3
    bounding_radius = float(np.linalg.norm(np.full(3, 0.5, np.float32)))
    return (np.ascontiguousarray(v.reshape(-1, 9), dtype=np.float32), alo.astype(np.float32), ahi.astype(np.float32),
            bounding_radius)


BVH_NODE = np.dtype([("lo", np.float32, 3), ("hi", np.float32, 3), ("left", np.int32), ("right", np.int32)])


def build_bvh(triangles, n_primitives_per_leaf=8):
    """TriangleBvh4::build on the host (no GPU): (triangles in BVH order, nodes structured array)."""
    tris = np.array(triangles, dtype=np.float32).reshape(-1, 9)
    n = C.c_uint32(0)
    check(lib().ngp_sdf_bvh_build(tris.ctypes.data, tris.shape[0], n_primitives_per_leaf, None, C.byref(n)))
    nodes = np.zeros(n.value, dtype=BVH_NODE)
    check(lib().ngp_sdf_bvh_build(tris.ctypes.data, tris.shape[0], n_primitives_per_leaf, nodes.ctypes.data, C.byref(n)))
    return tris, nodes


class SdfMesh:
    """The mesh on the device with its BVH. `triangles` is the BVH order (the build reorders them, as
    TriangleBvh4::build reorders m_sdf.triangles_cpu; surface sampling draws from that order)."""

    def __init__(self, triangles):
        tris = np.ascontiguousarray(triangles, dtype=np.float32).reshape(-1, 9)
        h = C.c_void_p()
        check(lib().ngp_sdf_mesh_create(tris.shape[0], tris.ctypes.data, C.byref(h)))
        self.handle = h
        self.triangles = np.empty_like(tris)
        check(lib().ngp_sdf_mesh_triangles(h, self.triangles.ctypes.data))

    def signed_distance(self, positions, stream=None):
        out = torch.empty(positions.shape[0], dtype=torch.float32, device=positions.device)
        check(lib().ngp_sdf_signed_distance(self.handle, _stream(stream), positions.shape[0], _ptr(positions), _ptr(out)))
        return out

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().ngp_sdf_mesh_destroy(h)
            except Exception:
                pass
            self.handle = None


class SdfTraining:
    """Testbed SDF training (training_prep_sdf + train_sdf) over a NetworkWithInputEncoding (3 -> 1)."""

    def __init__(self, network, trainer, mesh, aabb_min, aabb_max, bounding_radius=float(np.sqrt(0.75)), seed=1337,
                 batch_size=1 << 18, surface_offset_scale=1.0, zero_offset=0.0):
        self.network, self.trainer, self.mesh = network, trainer, mesh
        self.rng = pcg32(seed)
        self.batch_size = batch_size
        # sdf_aabb = m_aabb inflated by zero_offset (testbed_sdf.cu:1238-1239)
        self.aabb_min = (np.asarray(aabb_min, np.float32) - np.float32(zero_offset)).astype(np.float32)
        self.aabb_max = (np.asarray(aabb_max, np.float32) + np.float32(zero_offset)).astype(np.float32)
        self.stddev = float(np.float32(bounding_radius) / np.float32(1024.0) * np.float32(surface_offset_scale))
        self.training_step = 0
        n = batch_size
        self.positions = torch.empty((n, 3), dtype=torch.float32, device="cuda")
        self.distances = torch.empty(n, dtype=torch.float32, device="cuda")
        self.positions_shuffled = torch.empty_like(self.positions)
        self.distances_shuffled = torch.empty_like(self.distances)
        self._loss = torch.zeros(1, dtype=torch.float32, device="cuda")

    def generate_training_samples(self, n=None, positions=None, distances=None, stream=None):
        n = n or self.batch_size
        pos = positions if positions is not None else torch.empty((n, 3), dtype=torch.float32, device="cuda")
        dist = distances if distances is not None else torch.empty(n, dtype=torch.float32, device="cuda")
        check(lib().ngp_sdf_generate_training_samples(self.mesh.handle, _stream(stream), n, C.byref(self.rng),
                                                      self.aabb_min.ctypes.data, self.aabb_max.ctypes.data, self.stddev,
                                                      _ptr(pos), _ptr(dist)))
        return pos, dist

    def train_step(self, get_loss=True, regenerate=True, stream=None):
        if regenerate:  # generate_sdf_data_online (training_prep_sdf)
            self.generate_training_samples(self.batch_size, self.positions, self.distances, stream=stream)
        if get_loss:
            self._loss.zero_()
        check(lib().ngp_sdf_train_step(self.trainer.handle, _stream(stream), self.batch_size, _ptr(self.positions),
                                       _ptr(self.distances), self.training_step, _ptr(self.positions_shuffled),
                                       _ptr(self.distances_shuffled), _ptr(self._loss) if get_loss else None))
        self.training_step += 1
        return float(self._loss.item()) if get_loss else None
