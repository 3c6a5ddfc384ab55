"""Which kernels run concurrently with a given kernel in a rocprofv3 kernel trace (steady state: the last
40 %). Usage: python3 tools/trace_overlap.py run_kernel_trace.csv NAME_SUBSTRING"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
cut = t0 + (t1 - t0) * 0.6
rows = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
targets = [x for x in iv if sys.argv[2] in x[2]]
over = collections.Counter()
over_t = collections.Counter()
for s, e, _ in targets:
    for s2, e2, n2 in iv:
        if s2 < e and e2 > s and not (s2 == s and e2 == e):
            over[n2] += 1
            over_t[n2] += (min(e, e2) - max(s, s2)) / 1e3
tot = sum(e - s for s, e, _ in targets) / 1e3
print(f"{len(targets)} x {sys.argv[2]}: avg {tot / max(len(targets), 1):.1f} us")
for k, c in over.most_common(15):
    print(f"  {k:60s} overlaps {c:5d} times, {over_t[k] / max(len(targets), 1):7.1f} us per target")
