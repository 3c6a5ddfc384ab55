"""The fox loss passes on a trained state: per-ray sample counts (the compositing chain lengths) and the
loss launch's time. Trains the C2 network on data/fox for --steps Testbed steps, samples one batch at the
adapted ray count, then times compute_loss (torch events, --reps launches) and prints one JSON object."""
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
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--keep-state", type=int, default=1, help="pass 1 keeps the compositing state (the training step's form)")
    ap.add_argument("--flush-mb", type=int, default=0, help="write this many MB between launches (evicts the L2s)")
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    d = pkg.nerf_data.load_nerf(os.path.join(ROOT, "data", "fox"))
    ds = pkg.nerf.NerfDataset(d.images, d.rgba8)
    cfg = pkg.nerf.default_config(d.aabb_scale)
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
    ns = got["numsteps"].cpu().numpy().view(np.uint32).reshape(-1)[: 2 * kept].reshape(-1, 2)[:, 0].astype(np.int64)
    out = net.inference(got["coords"], layout=pkg.LAYOUT_AOS, use_inference_params=False)
    ks = bool(args.keep_state)
    ns0 = got["numsteps"].clone()  # compute_loss rewrites numsteps to the compacted {n, base}: restored per launch
    gl = pkg.nerf.compute_loss(ds, cfg, R, r, B, got, out, mean[:1].contiguous(), keep_state=ks)
    flush = torch.empty(max(args.flush_mb, 1) * (1 << 18), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = 0.0
    for _ in range(args.reps):
        got["numsteps"].copy_(ns0)
        if args.flush_mb:
            flush.fill_(1.0)
        ev0.record()
        pkg.nerf.compute_loss(ds, cfg, R, r, B, got, out, mean[:1].contiguous(), keep_state=ks)
        ev1.record()
        torch.cuda.synchronize()
        tot += ev0.elapsed_time(ev1)
    q = np.percentile(ns, [50, 90, 99, 99.9]).tolist()
    chunks = (ns + 15) // 16
    print(json.dumps({"rays": R, "kept": kept, "samples": int(ns.sum()), "numsteps_mean": float(ns.mean()),
                      "numsteps_p50_p90_p99_p999": q, "numsteps_max": int(ns.max()),
                      "chunks_max": int(chunks.max()), "chunks_mean": float(chunks.mean()),
                      "rays_over_256": int((ns > 256).sum()), "rays_over_512": int((ns > 512).sum()),
                      "keep_state": ks, "flush_mb": args.flush_mb, "compute_loss_ms": tot / args.reps}))


if __name__ == "__main__":
    main()
