"""Training-throughput benchmark of the instant-ngp hot path on MI355X.

A step = one NerfNetwork training pass over one synthetic batch of B = 2^18 samples per GPU:
hash-grid encoding forward -> fused density+rgb MLP forward/backward (MFMA) -> hash-grid backward
(destination-bucketed exact reduction; its histogram overlaps the forward on a side stream) -> [RCCL all-reduce of the fp16 gradient buffer when N > 1] -> fused
Adam/EMA optimizer step. Config C2 = the fork's configs/nerf/base.json (L=4, F=4, T=2^19,
64-wide MLPs, fp16) — BASELINE.json configs[1]. Inputs are resident in HBM before timing starts.

Multi-GPU: one process per GPU (torch.distributed.run); --scaling weak (default: each rank trains its
own 2^18-sample batch per step) or strong (one global 2^18 batch sharded over the ranks); gradients
summed with one RCCL all-reduce per step, inside the step's HIP graph.

At N=1 the JSON line also carries (rank 0, after the timed region):
  roofline      the dominant region's algorithmic bytes (or FLOPs) per launch / its HIP-event time;
                regions: grid forward, grid backward (bucket scan + plan + scatter + accumulate + split
                reduce), fused MLP training kernel, optimizer (46 B per updated parameter, 16 B per
                lazily skipped one); `traffic` = bytes that left L2 for the fabric (Infinity Cache + HBM)
                per launch, from the committed rocprofv3 summary of sized read requests + WRITE_SIZE
  cpu_baseline  the C oracle's encoding + MLP fwd/bwd on every host core this process may use
  e2e           the full Testbed NeRF step for 30 s on the procedural Lego stand-in: samples/s and PSNR
  c2p           the same training pass at C2' (L=16 F=2 T=2^19), BASELINE's literal "L=16"
  c5            the SDF training step at C5 (L=16 F=2 T=2^22, 105 M parameters: the HBM-bound config)
  c5_online     the reference's default SDF step on armadillo (online sample + BVH ground-truth
                regeneration every step), when data/sdf is staged
  c3            the fox capture trained for 15 s (samples/s, held-out PSNR), when data/fox is staged
"""
import argparse
import json
import math
import os
import re
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

B = 1 << 18
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
IC_BYTES = 256 * 2 ** 20     # Infinity Cache (MI355X_MICROARCH.md)
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
    if os.environ.get("NGP_BENCH_POINTS") == "blob":  # NeRF-like concentration (hot coarse entries)
        blob = np.clip(0.5 + 0.06 * g.standard_normal((n, 3)), 0.0, 1.0).astype(np.float32)
        keep = g.random(n) < 0.8
        c[keep, :3] = blob[keep]
    if os.environ.get("NGP_BENCH_POINTS") == "sorted":  # experiment: spatially coherent batch (Morton order)
        q = np.minimum((c[:, :3] * 128).astype(np.uint64), 127)
        key = np.zeros(n, np.uint64)
        for b in range(7):
            for d in range(3):
                key |= ((q[:, d] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + d)
        c[:, :3] = c[np.argsort(key, kind="stable"), :3]
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
    "grid_backward_total": ["k_sc_scan", "k_sc_plan", "k_sc_scatter", "k_sc_accumulate", "k_sc_split_reduce"],
    # k_nerf_mlp / k_mlp carry the mode as their LAST template argument (1 = training, 0 = inference)
    "mlp_train": ["k_nerf_mlp_train<", "1>(ngp::NerfMlpArgs)", "1>(ngp::MlpArgs)"],
    "mlp_infer": ["0>(ngp::NerfMlpArgs)", "0>(ngp::MlpArgs)"],
    "optimizer": ["k_adam_ema", "k_adam_lazy"],
}
# engine profiler phases that make up a roofline region (each runs once per training step)
REGION_PHASES = {"grid_backward_total": ["grid_bwd_prepare", "grid_backward_sorted"]}
# optimizer bytes per parameter (optimizer.hip k_adam_ema4): updated = read g16 w32 m1 m2 steps ema32
# (22 B) + write w32 m1 m2 steps w16 ema32 ema16 (24 B) = 46 B; lazily skipped grid entry (zero
# gradient) = read g16 w32 ema32 (10 B) + write ema32 ema16 (6 B) = 16 B
OPT_B_UPDATED, OPT_B_SKIPPED = 46, 16
# the grid's lazy-layout update fused into the bucketed backward (engine option fuse_opt: C5, C2'): a parameter
# pair's optimizer state AND fp32 master weights are one AdamRec (optimizer.h: {m1, m2, steps, ema, w, done}
# for two parameters, static_assert sizeof == 48), so an updated parameter reads and writes its half of the
# record and writes its fp16 weight; skipped parameters are not touched, no gradient is stored or re-read
ADAMREC_BYTES, ADAMREC_PARAMS = 48, 2
OPT_B_FUSED = ADAMREC_BYTES // ADAMREC_PARAMS * 2 + 2  # = 50 B per updated parameter
L2_PEAK_GBS = 34500.0  # aggregate L2 bandwidth (MI355X_MICROARCH.md, L2): no fabric rate can exceed it


def newest_profile(suffix):
    """profiles/<round>_<suffix> of the latest round tag: r<NN> then a letter sequence that grows like
    spreadsheet columns (r02z < r02aa < r02br), so plain string order is wrong past z."""
    import glob
    import re

    def key(path):
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    files = glob.glob(os.path.join(ROOT, "profiles", f"*_{suffix}"))
    return max(files, key=key) if files else None


# the bucketed backward's store mode (grid_scatter.h: 0 fp16 gradient, 1 fused optimizer update, 2 fp32 gradient)
# is the second template argument of k_sc_accumulate / k_sc_split_reduce: ...ILj<F>ELj<MODE>E...
_SC_MODE = re.compile(r"k_sc_(?:accumulate|split_reduce)ILj\d+ELj(\d+)E")


def pmc_traffic(variant, region, sc_mode=None):
    """Bytes per launch of `region` that left L2 for the fabric (Infinity Cache + HBM), from the newest
    committed rocprofv3 summary profiles/<round>_pmc_<variant>.json (tools/pmc_summary.py: reads =
    32/64/128 x TCC_EA0_RDREQ_{32B,64B,128B}, writes = WRITE_SIZE; calibrated against known-byte kernels
    in profiles/r02_hbm_calib.json — FETCH_SIZE alone counts every 128-B request as 64 B). None if absent."""
    path = newest_profile(f"pmc_{variant.lower()}.json")
    if not path or region not in REGION_KERNELS:
        return None, None
    summ = json.load(open(path))
    tot, hit = 0.0, False
    for name, v in summ.items():
        compact = name.replace(" ", "")
        m = _SC_MODE.search(compact)
        if m and sc_mode is not None and int(m.group(1)) != sc_mode:
            continue  # another store mode's instantiation (a different path than the one timed)
        if any(k.replace(" ", "") in compact for k in REGION_KERNELS[region]) and "fabric_bytes" in v:
            tot += v["fabric_bytes"]
            hit = True
    return (tot if hit else None), os.path.relpath(path, ROOT)


def pmc_mfma_util(variant, region):
    """MFMA utilisation of `region`'s kernels (rocprofv3 MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES over the
    SIMD-cycles of the dispatch) from the newest committed PMC summary; None if absent."""
    path = newest_profile(f"pmc_{variant.lower()}.json")
    if not path or region not in REGION_KERNELS:
        return None
    summ = json.load(open(path))
    vals = [v["mfma_util"] for name, v in summ.items()
            if any(k.replace(" ", "") in name.replace(" ", "") for k in REGION_KERNELS[region]) and v.get("mfma_util")]
    return round(max(vals), 4) if vals else None


def host_cores():
    """CPU threads this process may use: the affinity mask, capped by a cgroup CPU quota if one is set."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(variant, budget_s=12.0):
    """The oracle (a naive C port of the same encoding + MLP fwd/bwd, fp32/fp64, no SIMD intrinsics) timed
    on the host: one thread for a third of the budget, then one thread per usable host core for the rest
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
    threads, affinity, quota = host_cores()
    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        res = list(ex.map(run, [2 * budget_s / 3] * threads))
        dt = time.perf_counter() - t0
    nt = sum(r[0] for r in res)
    return {"value": nt / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "single_thread_value": n1 / t1,
            "hardware_concurrency": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"NerfNetwork fwd+bwd ({variant}) of an {chunk}-sample synthetic batch in the C oracle: "
                      f"{n1} samples on 1 thread in {t1:.1f} s, then {nt} samples on {threads} threads "
                      f"(every usable core) in {dt:.1f} s"}


def read_profiler(lib):
    import ctypes
    need = lib.ngp_profiler_read(None, 0)
    cbuf = ctypes.create_string_buffer(need)
    lib.ngp_profiler_read(cbuf, need)
    return json.loads(cbuf.value.decode())


def timed_steps(lib, step, steps, warmup, world, capture=None, comm=None):
    """W untimed warmup steps, then K steps between barrier + synchronize on both sides (one captured
    HIP graph of K steps when `capture` gives one), then the same K steps replayed eagerly with the
    engine's per-kernel HIP events (queued behind graph launches so the events bracket kernels only).
    `step` must run what the graph runs (Trainer.train_step is the eager form of a captured step).
    comm: a host-side exchange (dp.HostComm) whose own round-trip timer stands in for the engine
    profiler's "allreduce" region. Returns (seconds for the K timed steps, launch mode, per-phase
    profiler dict)."""
    stream = torch.cuda.Stream()
    graph_note = None
    with torch.cuda.stream(stream):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        graph = None
        if capture is not None:
            try:
                graph = capture(steps)
                # untimed replays: graph upload / first-launch costs, then at least ~25 ms of GPU work before the
                # timed launch. A short warmup leaves the clocks ramping into the timed region: at K = 20 after 5
                # warmup steps the first timed launch ran 146 us/step and every later one 135-138
                # (tools/graph_probe.py, profiles/r05e_graph_probe.jsonl)
                t_w = time.perf_counter()
                for i in range(16):
                    graph.launch()
                    torch.cuda.synchronize()
                    if i >= 1 and time.perf_counter() - t_w > 0.025:
                        break
            except Exception as e:  # same HIP kernels, launched one by one
                graph, graph_note = None, f"graph capture failed ({e}); eager launches"
                print(f"[bench] {graph_note}", file=sys.stderr, flush=True)
        if graph is None:
            lib.ngp_profiler_reset()
            lib.ngp_profiler_enable(1)
        if hasattr(comm, "reset_timer"):
            comm.reset_timer()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graph is not None:
            graph.launch()
        else:
            for _ in range(steps):
                step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        if graph is not None:
            lib.ngp_profiler_reset()
            for _ in range(3):  # ~3x the host's enqueue time of K eager steps
                graph.launch()
            lib.ngp_profiler_enable(1)
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
        lib.ngp_profiler_enable(0)
    prof = read_profiler(lib)
    if hasattr(comm, "reset_timer") and comm.calls and "allreduce" not in prof:
        prof["allreduce"] = {"ms": comm.ms, "calls": comm.calls, "timer": "host round trip (gloo)"}
    return t1 - t0, ("hip_graph" if graph is not None else (graph_note or "eager")), prof


def nerf_pass(pkg, variant, n, rank, world, opts=(), overlap=None, wire="f32", shard=True, exchange_at_world_1=False,
              dp_parts=None, dp_wire16=False):
    """NerfNetwork + Trainer for C2/C2' with a resident synthetic batch; returns (step, capture, net, trainer,
    comm). step() is Trainer.train_step, the eager form of the captured step (the grid's update fused into
    the backward on the lazy layout, the exchange hook, the optimizer), so the per-kernel replay profiles
    the path the graph times. capture is None when the exchange is a host round trip (gloo)."""
    cfg = pkg.nerf_config(variant)
    net = pkg.create_nerf_network(cfg)
    if overlap is not None:
        net.set_option("overlap", overlap)
    for kv in opts:
        k, v = kv.split("=")
        net.set_option(k, float(v))
    trainer = pkg.Trainer(net, cfg["optimizer"], seed=1337)
    net.reserve(n)
    x, dL = synthetic_batch(n, 1337 + rank, "cuda")
    comm = None
    if world > 1 or exchange_at_world_1:
        # nccl: the engine's own RCCL communicator, the gradient exchange enqueued by the engine on its
        # stream between the backward and the optimizer and captured into the step's graph; gloo (ranks
        # sharing one GPU): a host round trip through torch.distributed, eager steps only. A world of one
        # (exchange_at_world_1, no process group): the engine communicator alone, for the dp1_overhead record
        comm = pkg.dp.EngineComm(0, 1, wire=wire) if world == 1 else pkg.dp.make_comm(rank, world, wire=wire)
        if shard:
            if dp_parts is not None:
                trainer.set_option("dp_parts", dp_parts)  # the exchange in parameter parts, overlapping the backward
            trainer.set_option("dp_wire16", int(dp_wire16))
            trainer.set_data_parallel(comm)  # sharded optimizer: reduce-scatter, slice update, all-gather
        else:
            trainer.set_allreduce(comm)
    loss_scale = 128.0

    def step():
        trainer.train_step(x, dL, loss_scale)  # 1/N of the all-reduced sum folded into the loss scale

    def capture(k):
        return trainer.capture_training_step(x, dL, loss_scale, n_steps=k)
    return step, (None if isinstance(comm, pkg.dp.HostComm) else capture), net, trainer, comm


def slab_reduction_bytes(lib, net):
    """Algorithmic bytes of the MLP dW slab reduction that runs inside the grid backward's last kernel
    (engine option fuse_slabs): every fp32 slab read once [blocks x n_matrix], the fp16 MLP gradient
    written once. 0 when the model has no slab workspace."""
    import ctypes
    p, nb = ctypes.c_void_p(), ctypes.c_uint64()
    if lib.ngp_model_workspace(net.handle, b"dw_slabs", ctypes.byref(p), ctypes.byref(nb)) != 0:
        return 0
    return int(nb.value) + 2 * int(net.n_matrix_params)


CHECK_L2_RATE = True  # bench.py --pmc-collect turns it off: a counter-collection run precedes its own summary


def roofline(variant, n, kernels, n_opt_updated, n_opt_skipped, slab_bytes=0, fused_grid_updated=None):
    """Per-region achieved rate and fraction of peak; returns (summary dict, dominant region).
    slab_bytes: the fused dW slab reduction's bytes, counted in the grid_backward_total region (its
    kernel runs them as extra blocks). fused_grid_updated: grid parameters updated by the optimizer fused
    into the backward (profiler phase grid_backward_adam); their OPT_B_FUSED bytes join that region and
    the optimizer region covers the MLP alone (n_opt_* are then the MLP's counts)."""
    a = ALGO[variant]
    per = {k: v["ms"] / max(v["calls"], 1) for k, v in kernels.items()}
    for region, phases in REGION_PHASES.items():
        if all(p in per for p in phases):
            per[region] = sum(per[p] for p in phases)
    fused_b = 0
    sc_mode = 1 if "grid_backward_adam" in per else 0  # the timed step's bucketed-backward store mode
    if "grid_backward_adam" in per and "grid_bwd_prepare" in per:
        per["grid_backward_total"] = per["grid_bwd_prepare"] + per["grid_backward_adam"]
        fused_b = OPT_B_FUSED * (fused_grid_updated or 0)
    roof = {
        "grid_forward": ("hbm", a["enc_fwd_B"] * n / 1e9, HBM_PEAK_GBS, "GB/s"),
        "grid_backward": ("hbm", a["enc_bwd_B"] * n / 1e9, HBM_PEAK_GBS, "GB/s"),
        # SURVEY §8(d)'s bytes (+ the fused dW slab reduction's); the fused optimizer update's bytes are reported
        # beside them (achieved_incl_fused_update), not in `frac`: §8(d) defines no bytes for them
        "grid_backward_total": ("hbm", (a["enc_bwd_B"] * n + slab_bytes) / 1e9, HBM_PEAK_GBS, "GB/s"),
        "mlp_train": ("mfma", a["mlp_train_flop"] * n / 1e12, MFMA_F16_PEAK_TFLOPS, "TFLOP/s"),
        "mlp_infer": ("mfma", a["mlp_fwd_flop"] * n / 1e12, MFMA_F16_PEAK_TFLOPS, "TFLOP/s"),
    }
    if n_opt_updated is not None:
        roof["optimizer"] = ("hbm", (OPT_B_UPDATED * n_opt_updated + OPT_B_SKIPPED * n_opt_skipped) / 1e9, HBM_PEAK_GBS, "GB/s")
    summary = {}
    for k, ms in per.items():
        e = {"avg_ms": round(ms, 4)}
        if k in roof:
            b, w, pk, u = roof[k]
            e.update({"achieved": round(w / (ms / 1e3), 1), "unit": u, "frac": round(w / (ms / 1e3) / pk, 4)})
            if k == "grid_backward_total" and fused_b:
                wf = w + fused_b / 1e9
                e.update({"achieved_incl_fused_update": round(wf / (ms / 1e3), 1),
                          "frac_incl_fused_update": round(wf / (ms / 1e3) / pk, 4)})
            if b == "hbm":
                traffic, src = pmc_traffic(variant, k, sc_mode)
                if traffic is not None:
                    # what actually left L2 for the fabric per launch, and its rate
                    e["fabric_MB"] = round(traffic / 1e6, 2)
                    e["fabric_GBs"] = round(traffic / 1e9 / (ms / 1e3), 1)
                    if e["fabric_GBs"] > L2_PEAK_GBS and CHECK_L2_RATE:
                        # more bytes per second leaving L2 than L2 can deliver: the committed PMC summary
                        # describes other kernels than the ones timed here (stale profile or a different path)
                        raise RuntimeError(f"roofline {variant}/{k}: {e['fabric_MB']} MB per launch from {src} in "
                                           f"{ms * 1e3:.1f} us = {e['fabric_GBs']} GB/s > L2 {L2_PEAK_GBS} GB/s")
                if k == "optimizer" and w * 1e9 < IC_BYTES:
                    # the optimizer's whole working set is re-touched every step and fits the Infinity Cache:
                    # its bytes are served on-die, so the HBM spec is not their ceiling and no fraction of it
                    # is printed. fabric_GBs stays as the measured rate.
                    e.update({"bound": "infinity_cache", "frac": None,
                              "note": "working set < Infinity Cache, re-touched every step: no HBM fraction; "
                                      "fabric_GBs = PMC bytes leaving L2 / time"})
        if k in ("mlp_train", "mlp_infer"):
            u = pmc_mfma_util(variant, k)
            if u is not None:
                e["mfma_util_pmc"] = u
        summary[k] = e
    cands = [k for k in roof if k in per and not (k == "grid_backward" and "grid_backward_total" in per)
             and summary[k].get("bound") != "infinity_cache"]
    dom = max(cands, key=lambda k: per[k])
    bound, work, peak, unit = roof[dom]
    achieved = work / (per[dom] / 1e3)
    traffic, src = pmc_traffic(variant, dom, sc_mode)
    rl = {"kernel": dom, "bound": bound, "achieved": round(achieved, 1), "peak": peak, "unit": unit,
          "frac": round(achieved / peak, 4), "traffic": None if traffic is None else round(traffic / 1e6, 2),
          "traffic_unit": "MB/launch leaving L2 for the fabric (Infinity Cache + HBM; rocprofv3 sized read requests "
                          "+ WRITE_SIZE)",
          "traffic_source": src,
          "algorithmic": round(work * (1e3 if unit == "GB/s" else 1e6), 2),
          "algorithmic_includes": (("SURVEY 8(d)'s per-sample bytes and the fused MLP dW slab reduction: %.2f MB"
                                    % (slab_bytes / 1e6)) if dom == "grid_backward_total" and slab_bytes else None),
          "algorithmic_unit": "MB/launch" if unit == "GB/s" else "MFLOP/launch"}
    if dom == "grid_backward_total" and fused_b:
        # the same kernels also apply the grid's optimizer update (records read and written once per updated
        # pair): real HBM work that 8(d) does not count, and that the PMC traffic above includes
        wf = work + fused_b / 1e9
        rl.update({"fused_update_algorithmic": round(fused_b / 1e6, 2),
                   "fused_update_note": "the grid's optimizer update fused into the backward: %d B per updated parameter; "
                                        "not in `algorithmic`/`frac` (SURVEY 8(d) defines no bytes for it), included in "
                                        "`traffic`" % OPT_B_FUSED,
                   "achieved_incl_fused_update": round(wf / (per[dom] / 1e3), 1),
                   "frac_incl_fused_update": round(wf / (per[dom] / 1e3) / peak, 4)})
    return summary, rl


ARMADILLO = os.path.join(ROOT, "data", "sdf", "armadillo.obj")


def c5_pass(pkg, n, rank, mesh_path=None, online=False):
    """Testbed::train_sdf at C5 (configs/sdf/base.json with T=2^22): returns (step, net, trainer).
    online=False: a resident batch on a synthetic mesh (the training step alone). online=True: the
    reference's default step (generate_sdf_data_online = true, testbed.h:842): every step regenerates the
    batch (surface/perturbed/uniform samples, BVH raystab signed distances, testbed_sdf.cu:1187-1324)."""
    cfg = json.loads(json.dumps(pkg.SDF_BASE))
    cfg["encoding"].update({"log2_hashmap_size": 22, "per_level_scale": 2.0})
    net = pkg.NetworkWithInputEncoding(3, 1, cfg["encoding"], cfg["network"])
    trainer = pkg.Trainer(net, cfg["optimizer"], seed=1337)
    if mesh_path:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import sdf_train
        verts = sdf_train.load_obj_triangles(mesh_path)
    else:
        verts = pkg.synthetic.icosphere(4, radius=0.35, bumps=0.3, seed=rank)
    tris, amin, amax, brad = pkg.sdf.load_mesh(verts)
    mesh = pkg.sdf.SdfMesh(tris)
    sdf = pkg.sdf.SdfTraining(net, trainer, mesh, amin, amax, brad, seed=1337 + rank, batch_size=n)
    sdf.generate_training_samples(n, sdf.positions, sdf.distances)  # resident batch (online regeneration untimed)
    torch.cuda.synchronize()

    def step():
        sdf.train_step(get_loss=False, regenerate=online)
    step.n_triangles = int(tris.shape[0])
    return step, net, trainer


def optimizer_counts(net, trainer, step, fused=False):
    """Parameters the optimizer updates vs lazily skips (grid entries with a zero gradient) in one step.
    fused: the step is Trainer::training_step, whose grid update runs inside the backward without storing
    the gradient (engine option fuse_opt); the counts come from one step with it off. Returns
    (updated, skipped) for the optimizer launch and the number of grid parameters the fused update
    touches (None when not fused)."""
    if fused:
        net.set_option("fuse_opt", 0)
    step()
    torch.cuda.synchronize()
    nm = net.n_matrix_params
    nz = int(torch.count_nonzero(trainer.gradients[nm:]).item())
    if fused:
        net.set_option("fuse_opt", 1)
        return nm, 0, nz
    return nm + nz, net.n_params - nm - nz, None


def exchange_ms(kernels):
    """Per-step time of the gradient exchange: the engine profiler's RCCL phases (allreduce, or reduce_scatter +
    all_gather) or, for gloo ranks, the host round-trip timer reported as "allreduce"."""
    ph = [kernels[k] for k in ("allreduce", "reduce_scatter", "all_gather") if k in kernels]
    return round(sum(v["ms"] / max(v["calls"], 1) for v in ph), 4) if ph else None


# engine profiler phases that enclose other phases (the NeRF step's outer scopes; not added in kernels_sum_ms)
NESTED_PHASES = {"nerf_sample", "nerf_density_grid", "nerf_inference", "nerf_loss", "nerf_train_pass"}


def kernels_sum_ms(kernels):
    """Sum of the per-step averages of the engine profiler's top-level phases: the device time of one step
    as the per-kernel replay saw it, to compare with ms_per_step."""
    return round(sum(v["ms"] / max(v["calls"], 1) for k, v in kernels.items() if k not in NESTED_PHASES), 4)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` without a torch.distributed environment: start N fresh rank processes
    (torch.distributed.run, rendezvous on 127.0.0.1) running this same command line, and return their exit
    code. Runs before this process touches the GPU (no HIP call has been made yet): the ranks are children,
    never an exec of this process."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def check_world(gpus, env=os.environ):
    """The rank layout bench.py runs with: (needs_launch, world). --gpus N > 1 without WORLD_SIZE means
    bench.py must start the N ranks itself; with WORLD_SIZE set, it must equal --gpus."""
    if "WORLD_SIZE" not in env:
        return gpus > 1, 1
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (torch.distributed.run --nproc-per-node must match)")
    return False, world


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variant", default="C2", choices=["C2", "C2p", "C5", "IMG"])
    ap.add_argument("--batch", type=int, default=B)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --batch samples per GPU; strong: --batch samples per step over all GPUs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-seconds", type=float, default=30.0, help="full NeRF step + PSNR sub-record (0: off)")
    ap.add_argument("--e2e-weak-seconds", type=float, default=15.0,
                    help="N > 1: the e2e NeRF step with 2^18 samples per rank (weak scaling) for this long (0: off)")
    ap.add_argument("--no-c2p", action="store_true", help="skip the C2' (L=16) sub-record")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (SDF, T=2^22) sub-records")
    ap.add_argument("--c5-online-steps", type=int, default=10,
                    help="steps of the online-regenerating armadillo SDF step (c5_online sub-record; 0: off)")
    ap.add_argument("--c3-seconds", type=float, default=15.0, help="fox (C3) training sub-record length (0: off)")
    ap.add_argument("--graph", type=int, default=1, help="1: time the K steps as one captured HIP graph (N=1)")
    ap.add_argument("--overlap", type=int, default=None, help="engine side-stream overlap bitmask (engine.hip)")
    ap.add_argument("--opt", action="append", default=[], help="model option key=value (ngp_model_set_option)")
    ap.add_argument("--wire", default="f32", choices=["f32", "f16"],
                    help="gradient all-reduce wire type (f32: fp16 sums widened, rounded once)")
    ap.add_argument("--no-strong", action="store_true", help="N > 1: skip the strong-scaling sub-record")
    ap.add_argument("--dp-shard", type=int, default=1,
                    help="N > 1: 1 = sharded optimizer (reduce-scatter fp32, slice update, all-gather fp16 weights), "
                         "0 = one fp32 all-reduce of the gradients and a replicated update")
    ap.add_argument("--no-dp1", action="store_true", help="N = 1: skip the dp1_overhead sub-record")
    ap.add_argument("--dp-parts", type=int, default=None,
                    help="sharded exchange: parameter parts, each reduce-scattered / updated / all-gathered while the "
                         "backward sums the next (trainer option dp_parts; default: the engine's)")
    ap.add_argument("--dp-wire16", type=int, default=1,
                    help="sharded exchange: 1 = reduce-scatter the fp16 gradient buffer as fp16, the gradients' own "
                         "precision (half the wire bytes of fp32; RCCL rounds each hop's partial sum to fp16), 0 = "
                         "widened to fp32 (sums rounded once)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "gloo"],
                    help="N > 1 exchange: rccl (engine RCCL communicator, one GPU per rank) or gloo (host round "
                         "trip through torch.distributed: ranks may share a GPU, eager steps only)")
    ap.add_argument("--device", type=int, default=None, help="GPU index for every rank (default: LOCAL_RANK)")
    ap.add_argument("--e2e-images", type=int, default=100, help="views of the e2e procedural scene")
    ap.add_argument("--e2e-res", type=int, default=800, help="resolution of the e2e procedural scene")
    ap.add_argument("--no-vs1", action="store_true", help="N > 1: skip the in-job 1-GPU reference pass")
    ap.add_argument("--no-opt-count", action="store_true",
                    help="skip the untimed step that counts updated parameters (PMC passes: at C5 that step runs "
                         "unfused and would mix into the per-dispatch counter averages)")
    ap.add_argument("--pmc-collect", action="store_true",
                    help="a rocprofv3 counter-collection run (tools/gpu_round.sh pmc): the committed PMC summaries it "
                         "replaces may describe older kernels, so the L2-rate check of the roofline is skipped")
    args = ap.parse_args()
    global CHECK_L2_RATE
    CHECK_L2_RATE = not args.pmc_collect

    need_launch, _ = check_world(args.gpus)
    if need_launch:
        sys.exit(launch_ranks(args.gpus))

    from __graft_entry__ import load_package
    pkg = load_package()
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank if args.device is None else args.device)
    rank, world, local_rank = pkg.dp.init_from_env("gloo" if args.comm == "gloo" else None)
    assert world == args.gpus, (world, args.gpus)
    lib = pkg.lib()

    vs1 = None
    if world > 1 and args.variant in ("C2", "C2p") and not args.no_vs1:
        # the 1-GPU reference for the N-vs-1 ratios, measured in this job: rank 0 alone trains the same
        # --batch per step with no exchange, launched like the N-rank passes; the other ranks wait
        if rank == 0:
            s1, c1, _, _, _ = nerf_pass(pkg, args.variant, args.batch, 0, 1, args.opt, args.overlap)
            use_graph = args.graph and args.comm == "rccl"
            dt1, launch1, _ = timed_steps(lib, s1, args.steps, args.warmup, 1, c1 if use_graph else None)
            vs1 = {"value": args.batch * args.steps / dt1, "ms_per_step": dt1 / args.steps * 1e3, "launch": launch1,
                   "batch": args.batch}
            del s1, c1
            torch.cuda.synchronize()
        dist.barrier()

    n = args.batch if args.scaling == "weak" else args.batch // world
    n_opt = (None, None)
    c5_fused = None
    comm = None
    if args.variant in ("C2", "C2p"):
        step, capture, net, trainer, comm = nerf_pass(pkg, args.variant, n, rank, world, args.opt, args.overlap,
                                                      args.wire, shard=bool(args.dp_shard), dp_parts=args.dp_parts,
                                                      dp_wire16=bool(args.dp_wire16))
        if not args.no_opt_count:
            *n_opt, c5_fused = optimizer_counts(net, trainer, step, fused=trainer.fused_update_active(n))
        if not args.graph:
            capture = None
    elif args.variant == "C5":
        if world > 1:
            raise SystemExit("C5 bench is single-GPU")
        step, net, trainer = c5_pass(pkg, n, rank)
        if not args.no_opt_count:
            *n_opt, c5_fused = optimizer_counts(net, trainer, step, fused=True)
        capture = None
    else:  # IMG
        if world > 1:
            raise SystemExit("IMG bench is single-GPU")
        cfg = json.loads(json.dumps(pkg.IMAGE_BASE))
        cfg["encoding"]["per_level_scale"] = 2.0
        net = pkg.NetworkWithInputEncoding(2, 3, cfg["encoding"], cfg["network"])
        trainer = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        img = pkg.image.Image(pkg.synthetic.synthetic_image(1024, 1024, seed=rank))
        it = pkg.image.ImageTraining(net, trainer, img, seed=1337 + rank, batch_size=n)

        def step():
            it.train_step(get_loss=False)
        capture = None

    n_params_total = net.n_params
    dt, launch, kernels = timed_steps(lib, step, args.steps, args.warmup, world, capture, comm)
    slab_b = slab_reduction_bytes(lib, net)
    param_hashes = None
    if world > 1:
        dt = pkg.dp.reduce_scalar(dt, "max")
        # data parallelism keeps every rank's parameters identical (same all-reduced gradient, same update)
        import hashlib
        torch.cuda.synchronize()
        param_hashes = [None] * world
        dist.all_gather_object(param_hashes, hashlib.sha1(trainer.params.cpu().numpy().tobytes()).hexdigest())

    strong = None
    if world > 1 and args.variant in ("C2", "C2p") and not args.no_strong:
        # the other scaling mode in the same line: weak = fixed batch per GPU (headline), strong = one
        # global --batch sharded over the N ranks
        n_s = args.batch // world if args.scaling == "weak" else args.batch
        s_s, c_s, _, _, comm_s = nerf_pass(pkg, args.variant, n_s, rank, world, args.opt, args.overlap, args.wire,
                                           shard=bool(args.dp_shard), dp_parts=args.dp_parts,
                                           dp_wire16=bool(args.dp_wire16))
        dts, launch_s, k_s = timed_steps(lib, s_s, args.steps, args.warmup, world, c_s if args.graph else None, comm_s)
        dts = pkg.dp.reduce_scalar(dts, "max")
        strong = {"scaling": "strong" if args.scaling == "weak" else "weak", "batch_per_gpu": n_s,
                  "global_batch": n_s * world, "value": n_s * world * args.steps / dts, "unit": "samples/s",
                  "ms_per_step": dts / args.steps * 1e3, "launch": launch_s,
                  "exchange_ms_per_step": exchange_ms(k_s)}
        del s_s, c_s, comm_s
    e2e_dp = e2e_dp_weak = None
    if world > 1 and args.variant == "C2" and args.e2e_seconds > 0:
        # the metric's full form on N GPUs: the Testbed NeRF step data-parallel (rays sharded with their
        # global ids, RCCL all-reduce of gradients, density-grid maxima and counters), then PSNR on rank 0.
        # strong: the 1-GPU batch over N ranks (the 1-GPU ray set); weak: 2^18 samples per rank
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import psnr30
        e2e_dp = psnr30.run(pkg, seconds=args.e2e_seconds, images=args.e2e_images, res=args.e2e_res, rank=rank,
                            world=world, dp_wire16=bool(args.dp_wire16))
        if args.e2e_weak_seconds > 0:
            e2e_dp_weak = psnr30.run(pkg, seconds=args.e2e_weak_seconds, images=args.e2e_images, res=args.e2e_res,
                                     rank=rank, world=world, scaling="weak", dp_wire16=bool(args.dp_wire16))

    if rank == 0:
        kern_summary, rl = roofline(args.variant, n, kernels, *n_opt, slab_bytes=slab_b, fused_grid_updated=c5_fused)
        res = {
            "metric": "training samples/sec + PSNR@30s, NeRF Lego at 1/2/4/8 MI355X",
            "value": n * world * args.steps / dt,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f16",
            "data": "synthetic (U[0,1)^3 positions, uniform S^2 directions, U(+-1e-2) dL/dout; random-init weights)",
            "config": {"workload": WORKLOADS[args.variant],
                       "batch_per_gpu": n, "global_batch": n * world, "parallelism": f"dp{world}",
                       "launch": launch,
                       "exchange": (("sharded optimizer: fp32 reduce-scatter of the widened gradients, 1/N of the "
                                     "optimizer records updated per rank, fp16 all-gather of the weights" if args.dp_shard else
                                     f"all-reduce of the gradient buffer ({args.wire} on the wire), replicated update")
                                    + (" (engine RCCL communicator, inside the step's graph)" if args.comm == "rccl" else
                                       " (gloo host round trips)")
                                    if world > 1 else None)},
            "kernel_timing": ("HIP events per kernel on the launch stream, eager replay of the same K steps queued "
                              "behind a graph launch" if launch == "hip_graph" else "HIP events per kernel over the timed region"),
            "roofline": rl,
            "optimizer_params": ({"updated": n_opt[0], "skipped": n_opt[1]} if c5_fused is None else
                                 {"mlp_updated": n_opt[0], "grid_updated_in_backward": c5_fused}),
            "kernels_sum_ms": kernels_sum_ms(kernels),
            "kernels": kern_summary,
        }
        if world > 1:
            res["exchange_ms_per_step"] = exchange_ms(kernels)
            q = 8 * world
            n_pad = (int(n_params_total) + q - 1) // q * q
            res["exchange_bytes"] = ({"reduce_scatter_f16" if args.dp_wire16 else "reduce_scatter_f32":
                                      (2 if args.dp_wire16 else 4) * n_pad, "all_gather_f16": 2 * n_pad} if args.dp_shard else
                                     {"all_reduce": (4 if args.wire == "f32" else 2) * int(n_params_total)})
            if strong is not None:
                res["strong"] = strong
            res["param_sha1_per_rank"] = param_hashes
            if vs1 is not None:
                # N-vs-1 from this job's own 1-GPU pass: weak = N x batch per step over N GPUs, strong = one
                # batch per step over N GPUs, both against one GPU training one batch per step
                res["vs_1gpu"] = {"one_gpu": vs1, "weak_ratio": None, "strong_ratio": None}
                for mode, v in ((args.scaling, res["value"]),
                                (strong["scaling"] if strong else None, strong["value"] if strong else None)):
                    if mode is not None:
                        res["vs_1gpu"][f"{mode}_ratio"] = round(v / vs1["value"], 4)
            if e2e_dp_weak is not None:
                res["e2e_weak"] = {k: e2e_dp_weak[k] for k in ("value", "value_trained", "unit", "psnr", "psnr_views",
                                                               "train_seconds", "steps", "ms_per_step", "n_gpus", "config")}
            if e2e_dp is not None:
                res["e2e"] = {k: e2e_dp[k] for k in ("value", "unit", "psnr", "psnr_views", "train_seconds", "steps",
                                                     "ms_per_step", "n_gpus", "data", "config")}
        if world == 1 and args.variant in ("C2", "C2p") and not args.no_dp1 and not args.pmc_collect and args.comm == "rccl":
            # (not in counter-collection runs: their summaries describe the headline step's kernels alone)
            # the data-parallel step's own cost, measured where it can be (one GPU): the same pass with the
            # engine's RCCL communicator attached at world 1, timed like the headline (one graph of K steps),
            # sharded (reduce-scatter + slice update + all-gather) and all-reduce, against the fused N = 1 step
            res["dp1_overhead"] = {"note": "world-1 RCCL exchange attached, vs the fused single-GPU step above. shard: "
                                           "the backward stores the fp32 gradient itself, reduce-scatter, the rank's "
                                           "slice of the optimizer (here all of it), all-gather of the fp16 weights; "
                                           "shard_p2: the same in two parameter parts, the higher one exchanged on a "
                                           "second stream while the backward sums the lower one (trainer option "
                                           "dp_parts); shard_wire16: fp16 reduce-scatter; allreduce: fp16 gradient, "
                                           "widen, all-reduce, narrow, replicated update"}
            for mode in ("shard", "shard_p2", "shard_wire16", "allreduce"):
                sd, cd, _, _, commd = nerf_pass(pkg, args.variant, n, 0, 1, args.opt, args.overlap, args.wire,
                                                shard=mode != "allreduce", exchange_at_world_1=True,
                                                dp_parts=2 if mode == "shard_p2" else args.dp_parts,
                                                dp_wire16=mode == "shard_wire16")
                dtd, launchd, kd = timed_steps(lib, sd, args.steps, args.warmup, 1, cd if args.graph else None)
                res["dp1_overhead"][mode] = {
                    "ms_per_step": dtd / args.steps * 1e3, "launch": launchd,
                    "overhead_us": round((dtd - dt) / args.steps * 1e6, 2),
                    "phases_us": {k: round(v["ms"] / max(v["calls"], 1) * 1e3, 2) for k, v in kd.items()}}
                del sd, cd, commd
            torch.cuda.synchronize()
        if world == 1 and args.variant == "C2":
            if not args.no_c2p:
                # BASELINE's literal "L=16": the same training pass at C2' (L=16 F=2 T=2^19)
                s2, c2, net2, tr2, _ = nerf_pass(pkg, "C2p", n, 0, 1)
                *o2, f2 = optimizer_counts(net2, tr2, s2, fused=tr2.fused_update_active(n))
                dt2, launch2, k2 = timed_steps(lib, s2, args.steps, args.warmup, 1, c2)
                ks2, rl2 = roofline("C2p", n, k2, *o2, slab_bytes=slab_reduction_bytes(lib, net2), fused_grid_updated=f2)
                res["c2p"] = {"workload": WORKLOADS["C2p"], "value": n * args.steps / dt2, "unit": "samples/s",
                              "ms_per_step": dt2 / args.steps * 1e3, "launch": launch2, "roofline": rl2, "kernels": ks2,
                              "kernels_sum_ms": kernels_sum_ms(k2),
                              "optimizer_params": ({"updated": o2[0], "skipped": o2[1]} if f2 is None else
                                                   {"mlp_updated": o2[0], "grid_updated_in_backward": f2})}
                del s2, c2, net2, tr2
            if not args.no_c5:
                # BASELINE configs[4]: the HBM-bound SDF step (T=2^22, 105 M parameters), same batch size
                s5, net5, tr5 = c5_pass(pkg, n, 0)
                *o5, f5 = optimizer_counts(net5, tr5, s5, fused=True)
                dt5, launch5, k5 = timed_steps(lib, s5, args.steps, args.warmup, 1, None)
                ks5, rl5 = roofline("C5", n, k5, *o5, slab_bytes=slab_reduction_bytes(lib, net5), fused_grid_updated=f5)
                res["c5"] = {"workload": WORKLOADS["C5"], "value": n * args.steps / dt5, "unit": "samples/s",
                             "ms_per_step": dt5 / args.steps * 1e3, "launch": launch5, "roofline": rl5, "kernels": ks5,
                             "kernels_sum_ms": kernels_sum_ms(k5),
                             "optimizer_params": {"mlp_updated": o5[0], "grid_updated_in_backward": f5}}
                del s5, net5, tr5
                torch.cuda.empty_cache()
            if not args.no_c5 and args.c5_online_steps > 0 and os.path.isfile(ARMADILLO):
                # the reference's default SDF step on its named mesh: online regeneration every step
                # (surface / perturbed / uniform samples + BVH raystab signs) + the training step
                s6, net6, tr6 = c5_pass(pkg, n, 0, mesh_path=ARMADILLO, online=True)
                dt6, launch6, k6 = timed_steps(lib, s6, args.c5_online_steps, 2, 1, None)
                per6 = {k: round(v["ms"] / max(v["calls"], 1), 4) for k, v in k6.items()}
                res["c5_online"] = {"workload": "Testbed::train_sdf with generate_sdf_data_online (testbed.h:842): "
                                                "sample generation + BVH raystab ground truth + training_step, C5",
                                    "mesh": f"armadillo.obj ({s6.n_triangles} triangles)", "value": n * args.c5_online_steps / dt6,
                                    "unit": "samples/s", "ms_per_step": dt6 / args.c5_online_steps * 1e3,
                                    "steps": args.c5_online_steps, "launch": launch6, "phases_ms": per6}
                del s6, net6, tr6
                torch.cuda.empty_cache()
            if args.e2e_seconds > 0:
                # the metric's full form: the Testbed NeRF step (occupancy grid, sampling, inference,
                # loss/compaction, training pass, optimizer) for 30 s, then PSNR on held-out views
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                import psnr30
                e = psnr30.run(pkg, seconds=args.e2e_seconds)
                res["e2e"] = {k: e[k] for k in ("value", "value_trained", "unit", "psnr", "psnr_views", "train_seconds", "steps",
                                                "ms_per_step", "data", "config")}
                res["e2e"]["value_note"] = ("value: sum of measured_batch_size (the reference's counter, "
                                            "testbed_nerf.cu:3598) / s; value_trained: sum of min(measured, 2^18)")
            if args.c3_seconds > 0:
                # BASELINE configs[2]: the fox capture (OpenCV lens, aabb_scale 8: 4 cascades), when staged
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                import fox_train
                if os.path.isfile(os.path.join(fox_train.DEFAULT_DATA, "transforms.json")):
                    f = fox_train.run(pkg, seconds=args.c3_seconds)
                    res["c3"] = {k: f[k] for k in ("value", "value_trained", "unit", "psnr_heldout", "psnr_views", "psnr_train_views",
                                                   "train_seconds", "steps", "ms_per_step", "data", "config")}
                else:
                    res["c3"] = {"skipped": "data/fox not staged (tools/stage_fox.sh copies it from the reference tree)"}
        if world == 1 and not args.no_cpu_baseline and args.variant in ("C2", "C2p"):
            res["cpu_baseline"] = cpu_baseline(args.variant)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
