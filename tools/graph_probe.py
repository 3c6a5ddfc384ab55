"""Where does a K-step graph launch lose time? (bench.py at K=20 measured 144.4 us/step,
K=50 133.9 us/step, with the same per-kernel sums.)

Builds bench.py's C2 pass, then for K in --ks: captures one K-step graph, launches it once untimed, and times
--reps launches one by one, each bracketed like bench.py's timed region (synchronize, perf_counter, launch,
synchronize). Also records HIP events on the launch stream around each launch (device-side span), and the
host time spent inside the launch call itself. Prints one JSON line per K."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="20,50")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variant", default="C2")
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between launches (GPU idle)")
    args = ap.parse_args()
    import bench
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    step, capture, net, trainer, _ = bench.nerf_pass(pkg, args.variant, bench.B, 0, 1)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        for k in [int(v) for v in args.ks.split(",")]:
            g = capture(k)
            g.launch()
            torch.cuda.synchronize()
            rows = []
            for _ in range(args.reps):
                if args.idle_ms:
                    time.sleep(args.idle_ms / 1e3)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e0.record(stream)
                g.launch()
                th = time.perf_counter()
                e1.record(stream)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                rows.append({"wall_us_per_step": round((t1 - t0) / k * 1e6, 2),
                             "event_us_per_step": round(e0.elapsed_time(e1) * 1e3 / k, 2),
                             "host_launch_us": round((th - t0) * 1e6, 1)})
            # back-to-back launches without a sync in between: the steady state
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                g.launch()
            torch.cuda.synchronize()
            bb = (time.perf_counter() - t0) / (k * args.reps) * 1e6
            print(json.dumps({"k": k, "launches": rows, "back_to_back_us_per_step": round(bb, 2)}), flush=True)
            del g


if __name__ == "__main__":
    main()
