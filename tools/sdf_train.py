"""SDF primitive on a real mesh (BASELINE config C5: armadillo, configs/sdf/base.json with T=2^22).

Loads an OBJ (stage it first: tools/stage_sdf.sh; data/ is git-ignored and travels with the gpurun
snapshot), normalises it as Testbed::load_mesh, builds the triangle BVH, then runs Testbed::train_sdf
for --seconds: every step regenerates the 2^18-sample batch online (surface / perturbed / uniform
samples, BVH raystab signed distances), shuffles and trains (MAPE, Ema/Adam). Reports steps,
samples/s, the loss and two held-out checks: the sign agreement of the learned SDF with the BVH ground
truth on uniform points in the aabb, and the mean absolute error on near-surface points."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load_obj_triangles(path):
    """Triangle soup [3T, 3] from an OBJ (v / f lines; polygons fanned; 1-based and negative indices)."""
    verts, faces = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                verts.append([float(x) for x in line.split()[1:4]])
            elif line.startswith("f "):
                idx = []
                for tok in line.split()[1:]:
                    k = int(tok.split("/")[0])
                    idx.append(k - 1 if k > 0 else len(verts) + k)
                for j in range(1, len(idx) - 1):
                    faces.append((idx[0], idx[j], idx[j + 1]))
    v = np.asarray(verts, np.float32)
    return v[np.asarray(faces, np.int64).reshape(-1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mesh", default=os.path.join(ROOT, "data", "sdf", "armadillo.obj"))
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--log2-hashmap", type=int, default=22)
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    t0 = time.time()
    soup = load_obj_triangles(args.mesh)
    tris, amin, amax, brad = pkg.sdf.load_mesh(soup)
    mesh = pkg.sdf.SdfMesh(tris)
    t_mesh = time.time() - t0
    cfg = json.loads(json.dumps(pkg.SDF_BASE))
    cfg["encoding"].update({"log2_hashmap_size": args.log2_hashmap, "per_level_scale": 2.0})
    net = pkg.NetworkWithInputEncoding(3, 1, cfg["encoding"], cfg["network"])
    tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
    sdf = pkg.sdf.SdfTraining(net, tr, mesh, amin, amax, brad, seed=1337)
    torch.cuda.synchronize()
    steps, curve = 0, []
    t_start = time.time()
    while time.time() - t_start < args.seconds:
        get = steps % 100 == 0
        loss = sdf.train_step(get_loss=get)
        if get:
            curve.append((round(time.time() - t_start, 2), steps, round(float(loss), 6)))
        steps += 1
    torch.cuda.synchronize()
    t_train = time.time() - t_start
    # held-out checks against the BVH ground truth
    g = torch.Generator(device="cuda").manual_seed(7)
    lo, hi = torch.tensor(amin, device="cuda"), torch.tensor(amax, device="cuda")
    uni = lo + (hi - lo) * torch.rand((1 << 16, 3), device="cuda", generator=g)
    face = torch.from_numpy(mesh.triangles[np.random.default_rng(8).integers(0, len(mesh.triangles), 1 << 16)]).cuda()
    w = torch.rand((1 << 16, 2), device="cuda", generator=g)
    s = torch.sqrt(w[:, :1])
    surf = face[:, 0:3] * (1 - s) + face[:, 3:6] * (s * (1 - w[:, 1:])) + face[:, 6:9] * (s * w[:, 1:])
    near = surf + 0.005 * torch.randn(surf.shape, device="cuda", generator=g)
    res = {}
    for name, pts in (("uniform", uni), ("near_surface", near)):
        gt = mesh.signed_distance(pts.contiguous())
        pred = net.inference(pts.contiguous(), use_inference_params=True)[:, 0].float()
        res[name] = {"sign_agreement": float(((pred > 0) == (gt > 0)).float().mean()),
                     "mae": float((pred - gt).abs().mean())}
    print(json.dumps({
        "workload": "Testbed::train_sdf on %s (%d triangles), L=16 F=2 T=2^%d, 2x64 MLP, online sample regeneration"
                    % (os.path.basename(args.mesh), len(mesh.triangles), args.log2_hashmap),
        "steps": steps, "train_seconds": round(t_train, 2), "ms_per_step": 1e3 * t_train / max(steps, 1),
        "samples_per_s": steps * sdf.batch_size / t_train, "mesh_load_and_bvh_seconds": round(t_mesh, 2),
        "eval": res, "loss_curve": curve[:30]}), flush=True)


if __name__ == "__main__":
    main()
