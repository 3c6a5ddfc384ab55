"""Per-kernel memory traffic and MFMA utilisation per launch from rocprofv3 --pmc counter CSVs.

Inputs: counter_collection CSVs of separate passes (any order), e.g.
  sized reads : TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  writes      : WRITE_SIZE
  MFMA        : MfmaUtil SQ_INSTS_VALU_MFMA_MOPS_F16 (or SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE)
Calibration (tools/microbench/hbm_calib.hip, profiles/r02_hbm_calib.json): every read the L2 sends to
the fabric on gfx950 is a 128-B request (streaming reads of 2..16 B per lane and random 8-B gathers
alike), and FETCH_SIZE tallies each as 64 B; the sized request counters give the bytes exactly
(32/64/128 x count). WRITE_SIZE is exact for coalesced stores (64-B requests) and counts a scattered
sub-32-B store as its 32-B request. These are bytes between L2 and the fabric: Infinity Cache hits are
included, so a kernel whose working set stays in the 256 MiB Infinity Cache can show more than the HBM
peak. MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x SIMDs), the rocprofv3 MfmaUtil
formula; MFMA FLOPs = SQ_INSTS_VALU_MFMA_MOPS_F16 x 512.

Usage: python tools/pmc_summary.py [--simds 1024] CSV... > summary.json
"""
import argparse
import csv
import json
import sys
from collections import defaultdict


def load(paths):
    # (kernel name) -> counter -> list of per-dispatch values (summed over the rows of one dispatch)
    per_disp = defaultdict(lambda: defaultdict(float))
    names = {}
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                key = (path, int(row["Dispatch_Id"]))
                names[key] = row["Kernel_Name"]
                per_disp[key][row["Counter_Name"]] += float(row["Counter_Value"])
    acc = defaultdict(lambda: defaultdict(list))
    for key, cs in per_disp.items():
        for c, v in cs.items():
            acc[names[key]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} | {"_dispatches": max(len(v) for v in cs.values())}
            for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--simds", type=int, default=1024, help="SIMDs of the device (256 CUs x 4)")
    ap.add_argument("csv", nargs="+")
    args = ap.parse_args()
    out = {}
    for k, c in sorted(load(args.csv).items()):
        e = {"dispatches": c["_dispatches"]}
        if "TCC_EA0_RDREQ_128B_sum" in c:
            e["read_bytes"] = 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0.0) + \
                128 * c["TCC_EA0_RDREQ_128B_sum"]
        if "FETCH_SIZE" in c:
            e["fetch_size_bytes_raw"] = c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "read_bytes" in e and "write_bytes" in e:
            e["fabric_bytes"] = e["read_bytes"] + e["write_bytes"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE", 0) > 0:
            e["mfma_util"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] * args.simds)
            e["gpu_cycles"] = c["GRBM_GUI_ACTIVE"]
        if "MfmaUtil" in c:  # rocprofv3's derived counter (its own reductions over XCDs)
            e["mfma_util"] = c["MfmaUtil"] / 100.0
        if "SQ_INSTS_VALU_MFMA_MOPS_F16" in c:
            e["mfma_f16_flop"] = c["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512
        out[k] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
