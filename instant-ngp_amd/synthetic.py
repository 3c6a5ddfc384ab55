"""Procedural stand-in for the NeRF synthetic Lego capture (no network, no datasets in this image).

Same shape as data/nerf/nerf_synthetic/lego/transforms_train.json: 100 RGBA views of 800x800,
camera_angle_x 0.6911112, cameras on a sphere of radius 4.03 looking at the origin, transparent
background, opaque object inside the unit cube after nerf_matrix_to_ngp (scale 0.33, offset 0.5).
The object is a handful of analytic spheres and boxes rendered with torch (CPU or GPU) — plumbing
for synthetic input, not part of the measured path.
"""
import math

import numpy as np
import torch

from .nerf import NerfDataset, make_image, nerf_matrix_to_ngp

LEGO_CAMERA_ANGLE_X = 0.6911112070083618
LEGO_RADIUS = 4.0311


def look_at_c2w(eye):
    """Blender/NeRF camera-to-world (camera looks down -z, y up) for a camera at `eye` facing the origin."""
    eye = np.asarray(eye, np.float64)
    fwd = -eye / np.linalg.norm(eye)
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    if np.linalg.norm(right) < 1e-6:
        right = np.array([1.0, 0.0, 0.0])
    right /= np.linalg.norm(right)
    true_up = np.cross(right, fwd)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = right, true_up, -fwd, eye
    return m


def camera_poses(n, seed=0, radius=LEGO_RADIUS):
    """Upper-hemisphere views like the Blender synthetic training split."""
    rs = np.random.RandomState(seed)
    poses = []
    for i in range(n):
        theta = 2 * math.pi * ((i * 0.618033988749895 + rs.uniform(0, 0.05)) % 1.0)
        z = rs.uniform(0.05, 0.95)
        rxy = math.sqrt(1 - z * z)
        poses.append(look_at_c2w(radius * np.array([rxy * math.cos(theta), rxy * math.sin(theta), z])))
    return poses


_SPHERES = [  # centre (Blender coords), radius, sRGB colour
    ((0.0, 0.0, 0.2), 0.55, (0.95, 0.75, 0.10)),
    ((0.7, 0.3, -0.1), 0.35, (0.85, 0.15, 0.10)),
    ((-0.6, -0.5, 0.0), 0.40, (0.15, 0.35, 0.85)),
    ((-0.2, 0.7, 0.5), 0.25, (0.20, 0.75, 0.25)),
]
_BOXES = [  # min, max, colour
    ((-1.0, -1.0, -0.7), (1.0, 1.0, -0.45), (0.55, 0.55, 0.55)),
    ((0.3, -0.9, -0.45), (0.9, -0.3, 0.35), (0.90, 0.90, 0.85)),
]


def render(c2w, width, height, camera_angle_x=LEGO_CAMERA_ANGLE_X, device="cpu"):
    """RGBA8 [H, W, 4] of the procedural scene from Blender pose c2w."""
    f = 0.5 * width / math.tan(0.5 * camera_angle_x)
    j, i = torch.meshgrid(torch.arange(height, device=device, dtype=torch.float32),
                          torch.arange(width, device=device, dtype=torch.float32), indexing="ij")
    d = torch.stack([(i + 0.5 - 0.5 * width) / f, -(j + 0.5 - 0.5 * height) / f, -torch.ones_like(i)], -1)
    R = torch.tensor(c2w[:3, :3], dtype=torch.float32, device=device)
    o = torch.tensor(c2w[:3, 3], dtype=torch.float32, device=device)
    d = d @ R.T
    d = d / d.norm(dim=-1, keepdim=True)
    best = torch.full(d.shape[:2], float("inf"), device=device)
    col = torch.zeros(d.shape, device=device)
    nrm = torch.zeros(d.shape, device=device)
    for c, r, rgb in _SPHERES:
        c = torch.tensor(c, device=device)
        oc = o - c
        b = (d * oc).sum(-1)
        disc = b * b - (oc * oc).sum() + r * r
        t = -b - torch.sqrt(disc.clamp(min=0))
        hit = (disc > 0) & (t > 0) & (t < best)
        best = torch.where(hit, t, best)
        p = o + t[..., None] * d
        col = torch.where(hit[..., None], torch.tensor(rgb, device=device), col)
        nrm = torch.where(hit[..., None], (p - c) / r, nrm)
    for lo, hi, rgb in _BOXES:
        lo, hi = torch.tensor(lo, device=device), torch.tensor(hi, device=device)
        inv = 1.0 / torch.where(d.abs() < 1e-9, torch.full_like(d, 1e-9), d)
        t0, t1 = (lo - o) * inv, (hi - o) * inv
        tmin = torch.minimum(t0, t1).max(-1).values
        tmax = torch.maximum(t0, t1).min(-1).values
        hit = (tmax >= tmin) & (tmin > 0) & (tmin < best)
        best = torch.where(hit, tmin, best)
        axis = torch.minimum(t0, t1).argmax(-1)
        n = torch.nn.functional.one_hot(axis, 3).float() * -torch.sign(d)
        col = torch.where(hit[..., None], torch.tensor(rgb, device=device), col)
        nrm = torch.where(hit[..., None], n, nrm)
    light = torch.tensor([0.4, 0.3, 0.85], device=device)
    light = light / light.norm()
    shade = 0.35 + 0.65 * (nrm * light).sum(-1).clamp(min=0)
    alpha = torch.isfinite(best)
    rgb = (col * shade[..., None]).clamp(0, 1)
    out = torch.cat([rgb, alpha[..., None].float()], -1) * alpha[..., None]
    return (out * 255 + 0.5).clamp(0, 255).to(torch.uint8).cpu().numpy()


def lego_like_dataset(n_images=100, width=800, height=800, seed=0, device="cpu", return_host=False):
    """NerfDataset of the procedural scene with the Lego capture's shape (aabb_scale 1)."""
    images, pixels = [], []
    for c2w in camera_poses(n_images, seed):
        images.append(make_image(width, height, nerf_matrix_to_ngp(c2w), camera_angle_x=LEGO_CAMERA_ANGLE_X))
        pixels.append(render(c2w, width, height, device=device))
    ds = NerfDataset(images, pixels)
    return (ds, images, pixels) if return_host else ds


# ---- image / SDF stand-ins (albert.exr and armadillo.obj are not on the GPU box) --------------
def synthetic_image(width=1024, height=1024, seed=0):
    """An RGBA float32 [H, W, 4] linear-colour test image with edges, gradients and fine texture
    (stand-in for data/image/albert.exr, 1024^2 RGBA float)."""
    rs = np.random.RandomState(seed)
    y, x = np.mgrid[0:height, 0:width].astype(np.float32)
    x /= width
    y /= height
    img = np.zeros((height, width, 4), np.float32)
    img[..., 0] = 0.5 + 0.5 * np.sin(12 * np.pi * x * (1 + y))
    img[..., 1] = ((x - 0.5) ** 2 + (y - 0.5) ** 2 < 0.1).astype(np.float32) * 0.8 + 0.1 * y
    img[..., 2] = np.clip(np.abs(np.sin(40 * x) * np.cos(33 * y)) + 0.05 * rs.standard_normal((height, width)), 0, 1)
    img[..., 3] = 1.0
    return np.ascontiguousarray(img ** 2.2)  # stored linear, like an EXR


def icosphere(subdivisions=2, radius=1.0, center=(0.0, 0.0, 0.0), bumps=0.0, seed=0):
    """Closed triangle mesh [T*3, 3] (outward winding). bumps > 0 displaces vertices radially by a
    smooth random field (an armadillo stand-in with concavities)."""
    t = (1.0 + 5 ** 0.5) / 2
    verts = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
             (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    faces = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
             (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
             (8, 6, 7), (9, 8, 1)]
    v = [np.array(p, np.float64) / np.linalg.norm(p) for p in verts]
    for _ in range(subdivisions):
        cache, nf = {}, []

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in cache:
                m = v[a] + v[b]
                v.append(m / np.linalg.norm(m))
                cache[k] = len(v) - 1
            return cache[k]
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    V = np.array(v)
    if bumps > 0:
        rs = np.random.RandomState(seed)
        dirs = rs.standard_normal((6, 3))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        field = sum(np.exp(4.0 * (V @ d - 1.0)) * rs.uniform(-1, 1) for d in dirs)
        V = V * (1.0 + bumps * field)[:, None]
    V = V * radius + np.asarray(center, np.float64)
    return V[np.array(faces).reshape(-1)].astype(np.float32)
