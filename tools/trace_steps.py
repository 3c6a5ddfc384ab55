"""Per-step timeline from a rocprofv3 kernel trace (run_kernel_trace.csv).

Steps are delimited by a marker kernel (default: k_grid_forward). Prints each step's wall time and,
for the step given by --show, every kernel with start/end relative to the step start and its queue."""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--marker", default="k_grid_forward")
ap.add_argument("--show", type=int, nargs="*", default=[])
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
steps = []
for a, b in zip(starts, starts[1:]):
    t0 = int(rows[a]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    steps.append((a, b, t0, t1))
print("step durations (us):", " ".join(f"{(t1 - t0) / 1000:.0f}" for _, _, t0, t1 in steps))
for k in args.show:
    a, b, t0, t1 = steps[k]
    print(f"--- step {k}: {(t1 - t0) / 1000:.1f} us")
    for r in rows[a:b]:
        s = int(r["Start_Timestamp"]) - t0
        e = int(r["End_Timestamp"]) - t0
        print(f"{s / 1000:8.1f} {e / 1000:8.1f} {(e - s) / 1000:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:80]}")
