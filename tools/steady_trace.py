"""Per-kernel durations over the last 40 % of a rocprofv3 kernel trace (the steady state of a NeRF run whose
first steps are the density-grid warm-up). Usage: python3 tools/steady_trace.py run_kernel_trace.csv [top]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
cut = t0 + (t1 - t0) * 0.6
d = collections.defaultdict(list)
for r in rows:
    if int(r["Start_Timestamp"]) >= cut:
        d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{k:70s} n={len(v):5d} avg_us={sum(v) / len(v):8.1f} total_ms={sum(v) / 1e3:8.2f}")
