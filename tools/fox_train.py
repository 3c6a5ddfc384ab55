"""Fox capture (BASELINE config C3): load data/fox with the dataset ingest (nerf_data.load_nerf,
restating src/nerf_loader.cu: OpenCV lens, cx/cy principal point, aabb_scale 8 -> 4 cascades), train
the full Testbed NeRF step for --seconds of wall clock on the non-held-out frames, then render the
held-out frames (every --holdout-th) through their own cameras and lenses and report PSNR.
Stage the data first: tools/stage_fox.sh (data/ is git-ignored and travels with the gpurun snapshot).
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


DEFAULT_DATA = os.path.join(ROOT, "data", "fox")


def run(pkg, data=DEFAULT_DATA, seconds=30.0, holdout=10, eval_views=5, spp=1):
    """Train on the fox capture for `seconds` of wall clock and evaluate; returns the result dict."""
    args = argparse.Namespace(data=data, seconds=seconds, holdout=holdout, eval_views=eval_views, spp=spp)
    t0 = time.time()
    d = pkg.nerf_data.load_nerf(args.data)
    t_load = time.time() - t0
    idx = list(range(len(d)))
    test = [i for i in idx if args.holdout and i % args.holdout == args.holdout // 2][:args.eval_views]
    train = [i for i in idx if i not in test]
    t0 = time.time()
    ds = pkg.nerf.NerfDataset([d.images[i] for i in train], [d.rgba8[i] for i in train])
    t_upload = time.time() - t0
    cfg = pkg.nerf.default_config(d.aabb_scale)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    torch.cuda.synchronize()
    samples, steps, curve, trained = 0, 0, [], 0
    t_start = time.time()
    while True:
        st = run.train_step(get_loss=(steps % 100 == 0))
        samples += st["measured_batch_size"]
        trained += min(st["measured_batch_size"], 1 << 18)  # the batch the step trains on (rollover truncates)
        steps += 1
        if steps % 100 == 1:
            curve.append((round(time.time() - t_start, 2), steps, round(st["loss"], 6)))
        if time.time() - t_start >= args.seconds:
            break
    torch.cuda.synchronize()
    t_train = time.time() - t_start
    r = pkg.nerf.NerfRenderer()
    ps, t_render = [], time.time()
    for i in test:
        img = r.render(net, cfg, d.images[i], run.bitfield, spp=args.spp, min_transmittance=1e-4, background=(0, 0, 0, 1))
        ref = pkg.nerf.ground_truth_linear(torch.from_numpy(d.rgba8[i]).cuda())
        ps.append(pkg.nerf.psnr(img, ref)[0])
    # training views through the same renderer (fit quality, as opposed to held-out generalisation)
    ps_train = []
    for i in train[::max(1, len(train) // 3)][:3]:
        img = r.render(net, cfg, d.images[i], run.bitfield, spp=args.spp, min_transmittance=1e-4, background=(0, 0, 0, 1))
        ref = pkg.nerf.ground_truth_linear(torch.from_numpy(d.rgba8[i]).cuda())
        ps_train.append(pkg.nerf.psnr(img, ref)[0])
    torch.cuda.synchronize()
    t_render = time.time() - t_render
    h, w = d.rgba8[0].shape[:2]
    return {
        "metric": "training samples/sec + PSNR, NeRF fox (C3) on 1 MI355X",
        "value": samples / t_train, "unit": "samples/s",
        "value_trained": trained / t_train,  # min(measured_batch_size, B) per step: the samples actually trained
        "psnr_heldout": float(np.mean(ps)) if ps else None, "psnr_views": [round(p, 2) for p in ps],
        "psnr_train_views": [round(p, 2) for p in ps_train],
        "train_seconds": round(t_train, 2), "steps": steps, "ms_per_step": 1e3 * t_train / steps,
        "n_gpus": 1, "dtype": "f16",
        "data": f"data/nerf/fox: {len(d)} frames present ({w}x{h} JPEG, OpenCV lens), {len(train)} trained, "
                f"{len(test)} held out (every {args.holdout}th)",
        "config": {"workload": "Testbed NeRF training (configs/nerf/base.json fork), aabb_scale "
                               f"{d.aabb_scale:g} ({cfg.max_cascade + 1} cascades) + NerfTracer eval (spp {args.spp})",
                   "batch": 1 << 18},
        "load_seconds": round(t_load, 2), "upload_seconds": round(t_upload, 2), "render_seconds": round(t_render, 2),
        "loss_curve": curve[:40],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=DEFAULT_DATA)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--holdout", type=int, default=10, help="every N-th frame is held out for evaluation (0: none)")
    ap.add_argument("--eval-views", type=int, default=5)
    ap.add_argument("--spp", type=int, default=1)
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    print(json.dumps(run(pkg, args.data, args.seconds, args.holdout, args.eval_views, args.spp)), flush=True)


if __name__ == "__main__":
    main()
