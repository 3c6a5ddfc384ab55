#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats and HBM PMC passes.
# Usage (on the box, from the repo root): bash tools/gpu_round.sh TAG [stages...]
#   stages: tests smoke bench prof pmc (default: all)
# Every GPU step runs under its own timeout and the script stops at the first failure.
set -e -o pipefail
TAG=${1:-r01}; shift || true
STAGES=${*:-"tests smoke bench prof pmc"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ " $STAGES " == *" $1 "* ]]; }

if has tests; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/gpu_tests.log" 2>&1
  tail -3 "$OUT/gpu_tests.log"
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  tail -2 "$OUT/smoke.log"
fi
if has bench; then
  timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
  cat "$OUT/bench.json"
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
      python3 bench.py --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  head -12 "$OUT/kernel_stats.csv"
fi
if has pmc; then
  # HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), eager launches
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -f csv -d "$OUT/pmc_$c" -o run -- \
        python3 bench.py --no-cpu-baseline --graph 0 --steps 5 --warmup 2 > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.err"
    find "$OUT/pmc_$c" -name '*counter_collection.csv' -exec cp {} "$OUT/counters_$c.csv" \;
  done
  python3 tools/pmc_summary.py "$OUT/counters_FETCH_SIZE.csv" "$OUT/counters_WRITE_SIZE.csv" > "$OUT/pmc_summary.json"
  cat "$OUT/pmc_summary.json"
fi
if has pmcx; then
  # extra counters for one pass, e.g. PMCX="TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  timeout -k 10 300 rocprofv3 --pmc ${PMCX} -f csv -d "$OUT/pmcx" -o run -- \
      python3 bench.py --no-cpu-baseline --graph 0 --steps 5 --warmup 2 > "$OUT/pmcx.json" 2> "$OUT/pmcx.err"
  find "$OUT/pmcx" -name '*counter_collection.csv' -exec cp {} "$OUT/counters_x.csv" \;
  python3 tools/pmc_table.py "$OUT/counters_x.csv" | tee "$OUT/pmcx_table.txt"
fi
