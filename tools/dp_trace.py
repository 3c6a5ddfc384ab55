"""The sharded data-parallel C2 step at world 1 over the engine's RCCL communicator, captured and replayed, for a
rocprofv3 kernel trace: do the exchange's collectives and slice updates (exchange stream) run concurrently with the
grid backward's bucket accumulation (step stream)? Usage (on the GPU box):
  rocprofv3 --kernel-trace -f csv -d OUT -o run -- python3 tools/dp_trace.py [--parts 2] [--wire16 0] [--launches 20]
then python3 tools/trace_overlap.py OUT/.../run_kernel_trace.csv k_sc_accumulate"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=2)
    ap.add_argument("--wire16", type=int, default=0)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--steps-per-launch", type=int, default=4)
    ap.add_argument("--eager", type=int, default=0, help="1: time eager train_step calls instead of a captured graph")
    args = ap.parse_args()
    import bench
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    step, capture, net, trainer, comm = bench.nerf_pass(pkg, "C2", bench.B, 0, 1, exchange_at_world_1=True,
                                                        dp_parts=args.parts, dp_wire16=bool(args.wire16))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
        g = None if args.eager else capture(args.steps_per_launch)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        for _ in range(args.launches):
            if g is None:
                for _ in range(args.steps_per_launch):
                    step()
            else:
                g.launch()
        ev1.record(s)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / (args.launches * args.steps_per_launch)
    print(f"sharded C2 step, world 1, {args.parts} parts, wire16={args.wire16}, {'eager' if args.eager else 'graph'} "
          f"(DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')}, "
          f"DEBUG_HIP_FORCE_GRAPH_QUEUES={os.environ.get('DEBUG_HIP_FORCE_GRAPH_QUEUES')}): {ms * 1e3:.1f} us per step")


if __name__ == "__main__":
    main()
