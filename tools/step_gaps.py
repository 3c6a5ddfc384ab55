"""Per-step queue occupancy from a rocprofv3 kernel trace of the NeRF step: steps start at the
fused-encoding inference kernel; for the last --last steps, the wall time, the busy time of the
main queue (union of its kernels), its idle gaps, and the largest gaps with the kernels around them."""
import argparse
import csv
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last", type=int, default=30)
ap.add_argument("--marker", default="k_nerf_mlp<1, 1, 2, 3>")
args = ap.parse_args()
rows = list(csv.DictReader(open(args.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if args.marker in r["Kernel_Name"]]
main_q = rows[starts[-1]]["Queue_Id"]
walls, busy, gaps = [], [], defaultdict(list)
for a, b in list(zip(starts, starts[1:]))[-args.last:]:
    t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    walls.append((t1 - t0) / 1e3)
    end, bsum = t0, 0
    prev = None
    for r in rows[a:b]:
        if r["Queue_Id"] != main_q:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end and prev is not None:
            gaps[(prev[:40], r["Kernel_Name"][:40])].append((s - end) / 1e3)
        bsum += max(0, e - max(s, end))
        end = max(end, e)
        prev = r["Kernel_Name"]
    busy.append(bsum / 1e3)
n = len(walls)
print(f"steps {n}: wall {sum(walls) / n:.1f} us, main-queue busy {sum(busy) / n:.1f} us, idle {(sum(walls) - sum(busy)) / n:.1f} us")
top = sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:12]
for (p, q), v in top:
    print(f"  gap {sum(v) / n:6.1f} us/step ({len(v)}x, mean {sum(v) / len(v):.1f})  {p} -> {q}")
# per-kernel device time per step over the same steps (all queues), largest first
per = defaultdict(float)
for a, b in list(zip(starts, starts[1:]))[-args.last:]:
    for r in rows[a:b]:
        per[(r["Queue_Id"], r["Kernel_Name"][:70])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("per-kernel us/step (queue, kernel):")
for (q, k), v in sorted(per.items(), key=lambda kv: -kv[1])[:25]:
    print(f"  {v / n:7.1f}  q{q}  {k}")
