#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (tools/microbench/hbm_calib.hip): one rocprofv3
# pass per counter group, each under its own time limit; summaries in gpurun_out/$1.
set -e -o pipefail
OUT=gpurun_out/${1:-calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 5 60 ./tools/microbench/hbm_calib > "$OUT/calib_times.jsonl"
pass() {
  local tag=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" -f csv -d "$OUT/pmc_$tag" -o run -- ./tools/microbench/hbm_calib > /dev/null 2> "$OUT/pmc_$tag.err"
  find "$OUT/pmc_$tag" -name '*counter_collection.csv' -exec cp {} "$OUT/counters_$tag.csv" \;
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum
pass wrreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
pass rdsize TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
pass dram TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum
