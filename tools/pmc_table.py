"""Average per-dispatch value of every counter in a rocprofv3 counter_collection.csv, per kernel."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0.0, 0])
for row in csv.DictReader(open(sys.argv[1])):
    k = (row["Kernel_Name"][:60], row["Counter_Name"])
    acc[k][0] += float(row["Counter_Value"])
    acc[k][1] += 1
for (kern, ctr), (v, n) in sorted(acc.items()):
    print(f"{kern:60s} {ctr:28s} {v / n:16.1f}  (n={n})")
