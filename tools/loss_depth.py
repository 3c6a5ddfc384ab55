"""How deep into its samples the loss composites each ray, on a trained state: the data for deciding whether the
NeRF step's inference could evaluate only a prefix of every ray's samples first. Trains the C2
network for --steps Testbed steps (the Lego stand-in or --fox), samples one batch, runs the inference on every
sample and the loss, and reports, for prefix lengths K, the samples a first pass over min(n, K) per ray would
evaluate, the rays whose compositing reaches sample K (composited >= K and n > K: they need the rest), and the
samples of a second pass over those rays' remaining samples. One JSON object."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--fox", action="store_true")
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    if args.fox:
        d = pkg.nerf_data.load_nerf(os.path.join(ROOT, "data", "fox"))
        ds = pkg.nerf.NerfDataset(d.images, d.rgba8)
        cfg = pkg.nerf.default_config(d.aabb_scale)
    else:
        ds = pkg.synthetic.lego_like_dataset(n_images=100, width=800, height=800, seed=0, device="cuda")
        cfg = pkg.nerf.default_config(1.0)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    for _ in range(args.steps):
        st = run.train_step(get_loss=False)
    torch.cuda.synchronize()
    R = int(st["rays_per_batch"])
    B = cfg.target_batch_size
    mean, bf = pkg.nerf.grid_mean_and_bitfield(run.density_grid.clone(), cfg.max_cascade)
    r = pkg.nerf.pcg32(4711)
    got = pkg.nerf.generate_training_samples(ds, cfg, R, r, 16 * B, bf, n_rays_total=R)
    kept = int(got["counters"].cpu().numpy().view(np.uint32)[0])
    n = got["numsteps"].cpu().numpy().view(np.uint32).reshape(-1)[: 2 * kept].reshape(-1, 2)[:, 0].astype(np.int64)
    out = net.inference(got["coords"], layout=pkg.LAYOUT_AOS, use_inference_params=False)
    pkg.nerf.compute_loss(ds, cfg, R, r, B, got, out, mean[:1].contiguous(), keep_state=True)
    torch.cuda.synchronize()
    cn = got["numsteps"].cpu().numpy().view(np.uint32).reshape(-1)[: 2 * kept].reshape(-1, 2)[:, 0].astype(np.int64)
    res = {"scene": "fox" if args.fox else "lego_stand_in", "rays": R, "kept": kept, "samples": int(n.sum()),
           "composited": int(cn.sum()), "samples_per_ray": float(n.mean()), "composited_per_ray": float(cn.mean()),
           "composited_p50_p90_p99": np.percentile(cn, [50, 90, 99]).tolist(), "prefix": []}
    for K in (16, 32, 48, 64, 96, 128):
        more = (cn >= K) & (n > K)
        res["prefix"].append({"K": K, "first_pass_samples": int(np.minimum(n, K).sum()), "rays_needing_more": int(more.sum()),
                              "second_pass_samples": int((n - K)[more].sum())})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
