"""Per-kernel ratio of rocprofv3 memory counters to the exact bytes of tools/microbench/hbm_calib.hip.

Usage: python tools/hbm_calib.py gpurun_out/calib  -> JSON {kernel: {counter: value, ratio...}}
Counters are averaged over the kernel's dispatches (each kernel runs twice). FETCH_SIZE/WRITE_SIZE are
KiB; TCC_* request counts are per dispatch."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ORDER = ["r16", "r8", "r4", "r2", "g8", "w16", "w4", "w2", "s8"]


def load(path):
    per = defaultdict(lambda: defaultdict(list))  # dispatch -> counter -> values
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Kernel_Name"].startswith("__amd"):
                continue
            d = int(row["Dispatch_Id"])
            names[d] = row["Kernel_Name"]
            per[d][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return names, {d: {c: sum(v) for c, v in cs.items()} for d, cs in per.items()}


def main(root):
    times = [json.loads(l) for l in open(os.path.join(root, "calib_times.jsonl"))]
    known = {t["kernel"]: t for t in times}
    res = defaultdict(dict)
    for path in sorted(glob.glob(os.path.join(root, "counters_*.csv"))):
        names, vals = load(path)
        ds = sorted(vals)
        for i, d in enumerate(ds):  # two dispatches per kernel, in ORDER
            k = ORDER[i // 2]
            for c, v in vals[d].items():
                res[k].setdefault(c, []).append(v)
    out = {}
    for k in ORDER:
        r = {c: sum(v) / len(v) for c, v in res[k].items()}
        rd, wr = known[k]["read_bytes"], known[k]["write_bytes"]
        if "FETCH_SIZE" in r and rd:
            r["FETCH_SIZE_bytes_over_true"] = r["FETCH_SIZE"] * 1024 / rd
        if "WRITE_SIZE" in r and wr:
            r["WRITE_SIZE_bytes_over_true"] = r["WRITE_SIZE"] * 1024 / wr
        if "TCC_EA0_RDREQ_sum" in r and rd:
            b = r.get("TCC_BUBBLE_sum", 0.0)
            r32 = r.get("TCC_EA0_RDREQ_32B_sum", 0.0)
            r["rdreq_bytes_over_true"] = (32 * r32 + 64 * (r["TCC_EA0_RDREQ_sum"] - b - r32) + 128 * b) / rd
        if "TCC_EA0_RDREQ_128B_sum" in r and rd:
            r["sized_rdreq_bytes_over_true"] = (32 * r.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64 * r.get("TCC_EA0_RDREQ_64B_sum", 0.0) +
                                                128 * r["TCC_EA0_RDREQ_128B_sum"]) / rd
        if "TCC_EA0_WRREQ_sum" in r and wr:
            w64 = r.get("TCC_EA0_WRREQ_64B_sum", 0.0)
            r["wrreq_bytes_over_true"] = (64 * w64 + 32 * (r["TCC_EA0_WRREQ_sum"] - w64)) / wr
        out[k] = r
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
