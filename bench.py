"""Training-throughput benchmark of the instant-ngp hot path on MI355X.

A step = one NerfNetwork training pass over one synthetic batch of B = 2^18 samples per GPU:
hash-grid encoding forward -> fused density+rgb MLP forward/backward (MFMA) -> hash-grid backward
(destination-bucketed exact reduction; its histogram overlaps the forward on a side stream) -> [RCCL all-reduce of the fp16 gradient buffer when N > 1] -> fused
Adam/EMA optimizer step. Config C2 = the fork's configs/nerf/base.json (L=4, F=4, T=2^19,
64-wide MLPs, fp16) — BASELINE.json configs[1]. Inputs are resident in HBM before timing starts.

Multi-GPU: one process per GPU (torch.distributed.run), weak scaling (each rank trains its own
2^18-sample shard per step), gradients summed with one RCCL all-reduce per step.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

B = 1 << 18
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA spec

# Algorithmic work per sample (SURVEY §8d / BASELINE.md): encoding bytes, MLP FLOPs
ALGO = {
    "C2": {"enc_fwd_B": 300, "enc_bwd_B": 556, "mlp_train_flop": 55296, "mlp_fwd_flop": 18432},
    "C2p": {"enc_fwd_B": 588, "enc_bwd_B": 1100, "mlp_train_flop": 61440, "mlp_fwd_flop": 20480},
    # SDF C5 (3D, L=16 F=2 T=2^22, 32 -> 64 -> 64 -> 16): training_step = inference + train pass
    "C5": {"enc_fwd_B": 588, "enc_bwd_B": 1100, "mlp_train_flop": 43008, "mlp_fwd_flop": 14336},
    # image (configs/image/base.json: 2D, L=16 F=2 T=2^24): 8 + 4*L*F*2 + L*F*2 fwd, 8 + 64 + 2*4*64 bwd
    "IMG": {"enc_fwd_B": 328, "enc_bwd_B": 584, "mlp_train_flop": 43008, "mlp_fwd_flop": 14336},
}
WORKLOADS = {
    "C2": "NerfNetwork training pass, C2 (configs/nerf/base.json fork: L=4 F=4 T=2^19, density 1x64 + rgb 2x64 fp16 MLPs), "
          "fwd+bwd+Adam/EMA",
    "C2p": "NerfNetwork training pass, C2' (L=16 F=2 T=2^19, density 1x64 + rgb 2x64 fp16 MLPs), fwd+bwd+Adam/EMA",
    "C5": "Testbed::train_sdf step, C5 (configs/sdf/base.json with T=2^22: L=16 F=2, 2x64 MLP): shuffle + "
          "training_step (inference, MAPE loss, fwd+bwd, Ema/Adam) on a resident synthetic batch",
    "IMG": "Testbed::train_image step (configs/image/base.json: 2D L=16 F=2 T=2^24, 2x64 MLP): stratified samples, "
           "sRGB targets, training_step (L2), optimizer_step",
}


def synthetic_batch(n, seed, device):
    """Positions U[0,1)^3, directions uniform on S^2 warped by (d+1)/2, constant dt (NerfCoordinate),
    dL/doutput U(+-1e-2) on the 4 live rows (rgb + density)."""
    g = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3), dtype=np.float32)
    c[:, 3] = 0.0
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1e-2, 1e-2, (n, 4))
    return torch.from_numpy(c).to(device), torch.from_numpy(dL).to(device)


# profiler region -> the HIP kernels it launches (substrings of the rocprofv3 kernel names)
REGION_KERNELS = {
    "grid_forward": ["k_grid_forward"],
    "grid_backward": ["k_grid_backward"],
    "grid_backward_sorted": ["k_sc_scatter", "k_sc_accumulate", "k_sc_split_reduce"],
    "mlp_train": ["k_nerf_mlp<1,", "k_mlp<1,"],
    "mlp_infer": ["k_nerf_mlp<0,", "k_mlp<0,"],
}


def pmc_traffic(variant, region):
    """HBM bytes per launch of `region` from the newest committed rocprofv3 PMC summary
    (profiles/<round>_pmc_<variant>.json, written by tools/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE passes of this bench, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM). None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{variant.lower()}.json")))
    if not files or region not in REGION_KERNELS:
        return None, None
    summ = json.load(open(files[-1]))
    tot, hit = 0.0, False
    for name, v in summ.items():
        compact = name.replace(" ", "")
        if any(k.replace(" ", "") in compact for k in REGION_KERNELS[region]):
            tot += v["hbm_bytes"]
            hit = True
    return (tot if hit else None), os.path.relpath(files[-1], ROOT)


def cpu_baseline(variant, budget_s=12.0):
    """The oracle (a naive C port of the same encoding + MLP fwd/bwd, fp32/fp64, no SIMD intrinsics) timed
    on the host: one thread for a third of the budget, then one thread per host core for the rest
    (ctypes releases the GIL, each thread owns its chunk and gradient buffer: the OpenMP-over-samples
    baseline of SURVEY §8d). `value` is the all-cores rate."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as orc
    L, F = (4, 4) if variant == "C2" else (16, 2)
    m = orc.make_nerf(L=L, F=F, log2T=19)
    p32 = orc.nerf_init(m, 1337)
    p16 = orc.f32_to_f16_bits(p32)
    chunk = 8192
    x, dL = synthetic_batch(chunk, 7, "cpu")
    x, dL = x.numpy(), dL.float().numpy()

    def run(seconds):
        # one OpenMP thread per caller (the oracle's forward is an omp loop): thread-per-chunk scaling,
        # output and gradient buffers allocated once per thread
        orc.set_num_threads(1)
        out = np.zeros((chunk, 16), np.float32)
        grads = np.zeros(orc.nerf_n_params(m), np.float64)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            orc.nerf_forward(m, p16, x, out=out)
            orc.nerf_backward(m, p16, x, dL, grads=grads)
            done += chunk
        return done, time.perf_counter() - t0

    n1, t1 = run(budget_s / 3)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        res = list(ex.map(run, [2 * budget_s / 3] * threads))
        dt = time.perf_counter() - t0
    nt = sum(r[0] for r in res)
    return {"value": nt / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "single_thread_value": n1 / t1,
            "sample": f"NerfNetwork fwd+bwd ({variant}) of an {chunk}-sample synthetic batch in the C oracle: "
                      f"{n1} samples on 1 thread in {t1:.1f} s, then {nt} samples on {threads} threads in {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variant", default="C2", choices=["C2", "C2p", "C5", "IMG"])
    ap.add_argument("--batch", type=int, default=B)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", type=int, default=1, help="1: time the K steps as one captured HIP graph (N=1)")
    ap.add_argument("--overlap", type=int, default=None, help="engine side-stream overlap bitmask (engine.hip)")
    ap.add_argument("--opt", action="append", default=[], help="model option key=value (ngp_model_set_option)")
    args = ap.parse_args()

    from __graft_entry__ import load_package
    pkg = load_package()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    rank, world, local_rank = pkg.dp.init_from_env()

    n = args.batch
    loss_scale = 128.0
    if args.variant in ("C2", "C2p"):
        cfg = pkg.nerf_config(args.variant)
        net = pkg.create_nerf_network(cfg)
        if args.overlap is not None:
            net.set_option("overlap", args.overlap)
        for kv in args.opt:
            k, v = kv.split("=")
            net.set_option(k, float(v))
        trainer = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        net.reserve(n)
        x, dL = synthetic_batch(n, 1337 + rank, "cuda")
        grads = trainer.gradients
        comm = None
        if world > 1:
            # the engine's own RCCL communicator: the gradient all-reduce is enqueued by the engine on
            # its stream, between the backward and the optimizer, and captured into the step's graph
            comm = pkg.dp.EngineComm(rank, world)
            trainer.set_allreduce(comm)

        def step():
            net.forward_backward(x, dL)
            if comm is not None:
                comm.allreduce(grads)  # RCCL over xGMI; 1/N folded into the loss scale
            trainer.optimizer_step(loss_scale * world)
        graphable = True
    elif args.variant == "C5":
        cfg = json.loads(json.dumps(pkg.SDF_BASE))
        cfg["encoding"].update({"log2_hashmap_size": 22, "per_level_scale": 2.0})
        net = pkg.NetworkWithInputEncoding(3, 1, cfg["encoding"], cfg["network"])
        trainer = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        verts = pkg.synthetic.icosphere(4, radius=0.35, bumps=0.3, seed=rank)
        tris, amin, amax, brad = pkg.sdf.load_mesh(verts)
        mesh = pkg.sdf.SdfMesh(tris)
        sdf = pkg.sdf.SdfTraining(net, trainer, mesh, amin, amax, brad, seed=1337 + rank, batch_size=n)
        sdf.generate_training_samples(n, sdf.positions, sdf.distances)  # resident batch (online regeneration untimed)
        torch.cuda.synchronize()
        if world > 1:
            raise SystemExit("C5 bench is single-GPU")

        def step():
            sdf.train_step(get_loss=False, regenerate=False)
        graphable = False
    else:  # IMG
        cfg = json.loads(json.dumps(pkg.IMAGE_BASE))
        cfg["encoding"]["per_level_scale"] = 2.0
        net = pkg.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"])
        trainer = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        img = pkg.image.Image(pkg.synthetic.synthetic_image(1024, 1024, seed=rank))
        it = pkg.image.ImageTraining(net, trainer, img, seed=1337 + rank, batch_size=n)
        if world > 1:
            raise SystemExit("IMG bench is single-GPU")

        def step():
            it.train_step(get_loss=False)
        graphable = False

    lib = pkg.lib()
    stream = torch.cuda.Stream()
    use_graph = bool(args.graph) and graphable
    graph_note = None
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        graph = None
        if use_graph:
            # the K timed steps as one HIP graph launch (forward_backward + optimizer per step)
            try:
                graph = trainer.capture_training_step(x, dL, loss_scale, n_steps=args.steps)
                graph.launch()  # untimed replay: graph upload / first-launch costs
                torch.cuda.synchronize()
            except Exception as e:  # same HIP kernels, launched one by one
                graph, graph_note = None, f"graph capture failed ({e}); eager launches"
                print(f"[bench] {graph_note}", file=sys.stderr, flush=True)
        if graph is None:
            lib.ngp_profiler_reset()
            lib.ngp_profiler_enable(1)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graph is not None:
            graph.launch()
        else:
            for _ in range(args.steps):
                step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        if graph is not None:
            # per-kernel HIP-event timing: the same K steps replayed eagerly, queued behind one more
            # graph launch so the host is ahead of the GPU and the events bracket kernels only
            lib.ngp_profiler_reset()
            for _ in range(3):  # ~3x the host's enqueue time of K eager steps
                graph.launch()
            lib.ngp_profiler_enable(1)
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
        lib.ngp_profiler_enable(0)
    dt = t1 - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    import ctypes
    need = lib.ngp_profiler_read(None, 0)
    cbuf = ctypes.create_string_buffer(need)
    lib.ngp_profiler_read(cbuf, need)
    kernels = json.loads(cbuf.value.decode())

    if rank == 0:
        a = ALGO[args.variant]
        per_kernel = {k: v["ms"] / max(v["calls"], 1) for k, v in kernels.items()}
        roof = {
            "grid_forward": ("hbm", a["enc_fwd_B"] * n / 1e9, HBM_PEAK_GBS, "GB/s"),
            "grid_backward": ("hbm", a["enc_bwd_B"] * n / 1e9, HBM_PEAK_GBS, "GB/s"),
            "grid_backward_sorted": ("hbm", a["enc_bwd_B"] * n / 1e9, HBM_PEAK_GBS, "GB/s"),
            "mlp_train": ("mfma", a["mlp_train_flop"] * n / 1e12, MFMA_F16_PEAK_TFLOPS, "TFLOP/s"),
            "mlp_infer": ("mfma", a["mlp_fwd_flop"] * n / 1e12, MFMA_F16_PEAK_TFLOPS, "TFLOP/s"),
        }
        dom = max((k for k in roof if k in per_kernel), key=lambda k: per_kernel[k])
        bound, work, peak, unit = roof[dom]
        achieved = work / (per_kernel[dom] / 1e3)
        traffic, traffic_src = pmc_traffic(args.variant, dom)
        kern_summary = {}
        for k, ms in per_kernel.items():
            e = {"avg_ms": round(ms, 4)}
            if k in roof:
                b2, w2, p2, u2 = roof[k]
                e.update({"achieved": round(w2 / (ms / 1e3), 1), "unit": u2, "frac": round(w2 / (ms / 1e3) / p2, 4)})
            kern_summary[k] = e
        res = {
            "metric": "training samples/sec + PSNR@30s, NeRF Lego at 1/2/4/8 MI355X",
            "value": n * world * args.steps / dt,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f16",
            "data": "synthetic (U[0,1)^3 positions, uniform S^2 directions, U(+-1e-2) dL/dout; random-init weights)",
            "config": {"workload": WORKLOADS[args.variant],
                       "batch_per_gpu": n, "global_batch": n * world, "parallelism": f"dp{world}",
                       "launch": "hip_graph" if graph is not None else (graph_note or "eager"),
                       "exchange": "engine RCCL all-reduce of the fp16 gradient buffer per step" if world > 1 else None},
            "kernel_timing": ("HIP events per kernel on the launch stream, eager replay of the same K steps queued "
                              "behind a graph launch" if graph is not None else "HIP events per kernel over the timed region"),
            "roofline": {"kernel": dom, "bound": bound, "achieved": round(achieved, 1), "peak": peak, "unit": unit,
                         "frac": round(achieved / peak, 4),
                         "traffic": None if traffic is None else round(traffic / 1e6, 2),
                         "traffic_unit": "MB/launch (HBM, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                         "traffic_source": traffic_src,
                         "algorithmic": round(work * (1e3 if unit == "GB/s" else 1e6), 2),
                         "algorithmic_unit": "MB/launch" if unit == "GB/s" else "MFLOP/launch"},
            "kernels": kern_summary,
        }
        if world == 1 and not args.no_cpu_baseline and args.variant in ("C2", "C2p"):
            res["cpu_baseline"] = cpu_baseline(args.variant)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
