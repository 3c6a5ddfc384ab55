"""PSNR@30s on the procedural Lego stand-in (BASELINE metric, second half).

Trains the full Testbed NeRF step (occupancy-grid update, ray sampling, inference over every
sample, loss/compaction, fused forward/backward, Adam/EMA) for --seconds of wall clock on 100
800x800 views shaped like nerf_synthetic/lego (the real capture is not in this image: SURVEY F9),
then renders held-out views with the scripts/run.py protocol (black background, snapped pixels,
spp 8, min transmittance 1e-4) and prints one JSON line: full-pipeline training samples/s
(sum of compacted batch sizes / training wall time) and the mean PSNR."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(pkg, seconds=30.0, images=100, res=800, test_views=8, spp=8, rank=0, world=1, scaling="strong", dp_wire16=True):
    """Train the full NeRF step for `seconds` of wall clock on the procedural stand-in, then render the
    held-out views. Returns the result dict (samples/s over the training wall time, mean PSNR).
    world > 1 (torch.distributed initialised): data-parallel training (NerfTraining.set_data_parallel:
    rays sharded with their global ids, engine RCCL exchange); every rank stops after the same step
    (decided jointly every 32 steps) and rank 0 renders the held-out views. scaling "strong" (SURVEY §8e): the
    1-GPU batch of 2^18 samples split over the ranks, the 1-GPU ray set; "weak": 2^18 samples per rank (the global
    batch, target_batch_size, N x 2^18)."""
    S = pkg.synthetic
    t0 = time.time()
    ds = S.lego_like_dataset(n_images=images, width=res, height=res, seed=0, device="cuda")
    t_data = time.time() - t0
    cfg = pkg.nerf.default_config(1.0)
    if scaling == "weak":
        cfg.target_batch_size = (1 << 18) * world
    batch = int(cfg.target_batch_size)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    if world > 1:
        import torch.distributed as dist
        tr.set_option("dp_wire16", int(dp_wire16))  # the fp16 gradient buffer reduce-scattered as fp16
        run.set_data_parallel(rank, world)
        dist.barrier()
    torch.cuda.synchronize()
    samples, steps, trained = 0, 0, 0  # measured_batch_size is the global count under data parallelism (all-reduced)
    t_start = time.time()
    curve = []
    while True:
        st = run.train_step(get_loss=(steps % 100 == 0))
        samples += st["measured_batch_size"]
        trained += min(st["measured_batch_size"], batch)  # the batch the step trains on (rollover truncates)
        steps += 1
        if steps % 100 == 1:
            curve.append((round(time.time() - t_start, 2), steps, round(st["loss"], 6)))
        if world > 1:
            if steps % 32 == 0:  # the ranks must run the same number of steps (collectives inside)
                if pkg.dp.reduce_scalar(float(time.time() - t_start >= seconds), "max") > 0:
                    break
        elif time.time() - t_start >= seconds:
            break
    torch.cuda.synchronize()
    t_train = time.time() - t_start
    if world > 1:
        t_train = pkg.dp.reduce_scalar(t_train, "max")
        tr.gather_shards()  # collective: the sharded optimizer state (EMA records) whole on every rank
        if rank != 0:
            return {"value": samples / t_train, "steps": steps, "train_seconds": t_train}
    r = pkg.nerf.NerfRenderer()
    poses = S.camera_poses(images + test_views, seed=12345)[-test_views:]
    ps, t_render = [], time.time()
    for c2w in poses:
        cam = pkg.nerf.make_image(res, res, pkg.nerf.nerf_matrix_to_ngp(c2w), camera_angle_x=S.LEGO_CAMERA_ANGLE_X)
        img = r.render(net, cfg, cam, run.bitfield, spp=spp, min_transmittance=1e-4, background=(0, 0, 0, 1))
        ref = pkg.nerf.ground_truth_linear(S.render(c2w, res, res, device="cuda"))
        ps.append(pkg.nerf.psnr(img, ref)[0])
    torch.cuda.synchronize()
    t_render = time.time() - t_render
    return {
        "metric": "training samples/sec + PSNR@30s, NeRF Lego at 1/2/4/8 MI355X",
        "value": samples / t_train, "unit": "samples/s",
        "value_trained": trained / t_train,  # min(measured_batch_size, B) per step: the samples actually trained
        "psnr": float(np.mean(ps)), "psnr_views": [round(p, 2) for p in ps],
        "train_seconds": round(t_train, 2), "steps": steps, "ms_per_step": 1e3 * t_train / steps,
        "n_gpus": world, "dtype": "f16",
        "data": f"procedural Lego stand-in: {images} views {res}x{res} RGBA8, camera_angle_x of lego "
                "(nerf_synthetic is not in the image)",
        "config": {"workload": "Testbed NeRF training (configs/nerf/base.json fork, C2) + NerfTracer eval "
                               f"(black bg, snapped, spp {spp})", "batch": batch,
                   "parallelism": f"dp{world}", "scaling": scaling},
        "dataset_seconds": round(t_data, 2), "render_seconds": round(t_render, 2), "loss_curve": curve[:40],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--images", type=int, default=100)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--test-views", type=int, default=8)
    ap.add_argument("--spp", type=int, default=8)
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    print(json.dumps(run(pkg, args.seconds, args.images, args.res, args.test_views, args.spp)), flush=True)


if __name__ == "__main__":
    main()
