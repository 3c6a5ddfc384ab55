"""Per-kernel HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs.

FETCH_SIZE and WRITE_SIZE are in KiB (rocprofv3 derived counters). Per MI355X_MICROARCH.md §HBM, on
gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so `fetch_bytes_corrected` doubles
it; WRITE_SIZE is exact for streaming stores and for float atomics. Output: one JSON object keyed by
kernel name with the per-dispatch averages (bytes).
"""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            acc[name][0] += float(row["Counter_Value"])
            acc[name][1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f_kib, nf = fetch.get(k, (0.0, 0))
        w_kib, nw = write.get(k, (0.0, 0))
        out[k] = {"dispatches": max(nf, nw),
                  "fetch_bytes_raw": f_kib * 1024, "fetch_bytes_corrected": 2 * f_kib * 1024,
                  "write_bytes": w_kib * 1024,
                  "hbm_bytes": 2 * f_kib * 1024 + w_kib * 1024}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
