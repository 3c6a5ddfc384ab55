"""Per-phase timing of the full Testbed NeRF training step (training_prep_nerf + train_nerf_step).

Trains --steps steps on the procedural Lego stand-in, then records --measure more steps with the
engine's HIP-event profiler (events on the launch stream) and prints one JSON object: wall ms per
step, mean rays / pre-compaction samples / compacted samples per step, and each phase's mean ms per
call and per step (nerf_density_grid runs every clamp(step/16, 1, 16) steps)."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--measure", type=int, default=200)
    ap.add_argument("--images", type=int, default=100)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--pipeline", type=int, default=1, help="1: next step's sampler under the training pass (default), 0: serial step")
    ap.add_argument("--option", action="append", default=[], help="model option key=value (ngp_model_set_option)")
    ap.add_argument("--option-after-warmup", action="append", default=[],
                    help="model option key=value set after the warm-up steps (timing experiments: win_debug)")
    ap.add_argument("--fox", action="store_true", help="the fox capture (data/fox, tools/stage_fox.sh) instead of the stand-in")
    ap.add_argument("--profiler", type=int, default=1, help="0: no engine HIP-event profiler in the measured steps (wall time only)")
    ap.add_argument("--env-after-warmup", action="append", default=[],
                    help="KEY=VALUE set in the environment after the warm-up steps (engine timing switches read per step)")
    ap.add_argument("--sampler-stats", action="store_true",
                    help="read the march statistics of a -DNGP_SAMPLER_DIAG=4 build (NGP_ENGINE_LIB) over the measured steps")
    args = ap.parse_args()
    from __graft_entry__ import load_package
    pkg = load_package()
    if args.fox:
        d = pkg.nerf_data.load_nerf(os.path.join(ROOT, "data", "fox"))
        ds = pkg.nerf.NerfDataset(d.images, d.rgba8)
        cfg = pkg.nerf.default_config(d.aabb_scale)
    else:
        S = pkg.synthetic
        ds = S.lego_like_dataset(n_images=args.images, width=args.res, height=args.res, seed=0, device="cuda")
        cfg = pkg.nerf.default_config(1.0)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    for kv in args.option:
        key, value = kv.split("=")
        net.set_option(key, float(value))
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    run.set_pipeline(args.pipeline)
    lib = pkg.lib()
    t0 = time.time()
    for i in range(args.steps):
        run.train_step(get_loss=False)
        if i % 500 == 0:
            print(f"step {i} {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    t_warm = time.time() - t0
    for kv in args.option_after_warmup:
        key, value = kv.split("=")
        net.set_option(key, float(value))
    for kv in args.env_after_warmup:
        key, value = kv.split("=", 1)
        os.environ[key] = value
    lib.ngp_profiler_reset()
    lib.ngp_profiler_enable(args.profiler)
    if args.sampler_stats:
        lib.ngp_debug_sampler_stats(None, 0)
    rays, pre, comp = [], [], []
    t0 = time.time()
    for _ in range(args.measure):
        st = run.train_step(get_loss=False)
        rays.append(st["rays_per_batch"])
        pre.append(st["measured_batch_size_before_compaction"])
        comp.append(st["measured_batch_size"])
    torch.cuda.synchronize()
    dt = time.time() - t0
    lib.ngp_profiler_enable(0)
    need = lib.ngp_profiler_read(None, 0)
    buf = ctypes.create_string_buffer(need)
    lib.ngp_profiler_read(buf, need)
    k = json.loads(buf.value.decode())
    stats = None
    if args.sampler_stats:
        raw = (ctypes.c_uint64 * 48)()
        lib.ngp_debug_sampler_stats(raw, 48)
        n = max(raw[3], 1)
        stats = {"rays": raw[3], "empty_iters_per_ray": raw[0] / n, "occ_iters_per_ray": raw[1] / n,
                 "occ_rounds_per_occ_iter": raw[2] / max(raw[1], 1), "occ_states_per_ray": raw[4] / n,
                 "max_iters_one_ray": raw[5], "empty_exits_per_ray": raw[6] / n,
                 "empty_rounds_per_empty_iter": raw[7] / max(raw[0], 1),
                 "wall_ticks_per_ray": {"setup_ray": raw[40] / n, "sampling_end": raw[41] / n, "guess_verify": raw[42] / n,
                                        "occupancy_test": raw[43] / n, "march_loop": raw[44] / n,
                                        "initial_guess": raw[46] / n},
                 "max_wall_ticks_one_ray": raw[45],
                 "iters_log2_hist": {f"{1 << b}": raw[8 + b] for b in range(32) if raw[8 + b]}}
    phases = {n: {"calls": v["calls"], "ms_per_call": round(v["ms"] / max(v["calls"], 1), 4),
                  "ms_per_step": round(v["ms"] / args.measure, 4)} for n, v in sorted(k.items())}
    print(json.dumps({
        "warm_steps": args.steps, "warm_seconds": round(t_warm, 2), "measured_steps": args.measure,
        "ms_per_step_wall": round(1e3 * dt / args.measure, 4),
        "rays_per_batch": float(np.mean(rays)),
        "rays_per_batch_changed": float(np.mean(np.diff(np.asarray(rays)) != 0)) if len(rays) > 1 else 0.0,
        # how predictable the next step's ray count is (a speculative sampler must guess it): the step-to-step
        # differences in units of 256 rays, and the hit rate of R_{k+1} = R_{k-1} and of R_{k+1} in {R_k, R_{k-1}}
        "rays_delta_hist": {str(int(k)): int(v) for k, v in zip(*np.unique(np.diff(np.asarray(rays)) // 256, return_counts=True))},
        "rays_hit_prev2": float(np.mean(np.asarray(rays)[2:] == np.asarray(rays)[:-2])) if len(rays) > 2 else 0.0,
        "rays_hit_last_two": float(np.mean((np.asarray(rays)[2:] == np.asarray(rays)[1:-1]) |
                                           (np.asarray(rays)[2:] == np.asarray(rays)[:-2]))) if len(rays) > 2 else 0.0, "samples_before_compaction": float(np.mean(pre)),
        "compacted_samples": float(np.mean(comp)),
        "samples_per_s": float(np.sum(comp) / dt), "phases": phases, "sampler_stats": stats}, indent=1), flush=True)


if __name__ == "__main__":
    main()
