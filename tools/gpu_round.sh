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
  timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_ARGS:--x} -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -3 "$OUT/gpu_tests.log"
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  tail -2 "$OUT/smoke.log"
fi
if has bench; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err"
  cat "$OUT/bench.json"
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
      python3 bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c5 --pmc-collect ${PMC_ARGS} > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  rm -rf "$OUT/prof"
  head -12 "$OUT/kernel_stats.csv"
fi
if has pmc; then
  # separate passes (TCC slots): sized read requests, WRITE_SIZE, MFMA utilisation; eager launches; one
  # summary per variant (PMC_VARIANTS, default C2 C2p C5) -> $OUT/pmc_summary_<variant>.json
  for V in ${PMC_VARIANTS:-C2 C2p C5}; do
    BENCH_PMC="python3 bench.py --variant $V --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c2p --no-c5 --graph 0 --steps 5 --warmup 2 --no-opt-count --pmc-collect ${PMC_ARGS}"
    i=0
    for c in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "WRITE_SIZE" \
             "MfmaUtil SQ_INSTS_VALU_MFMA_MOPS_F16"; do
      i=$((i+1))
      timeout -k 10 300 rocprofv3 --pmc $c -f csv -d "$OUT/pmc_${V}_$i" -o run -- $BENCH_PMC > "$OUT/pmc_${V}_$i.json" 2> "$OUT/pmc_${V}_$i.err"
      find "$OUT/pmc_${V}_$i" -name '*counter_collection.csv' -exec cp {} "$OUT/counters_${V}_$i.csv" \;
      rm -rf "$OUT/pmc_${V}_$i"
    done
    python3 tools/pmc_summary.py "$OUT"/counters_${V}_[0-9].csv > "$OUT/pmc_summary_$V.json"
    python3 -c "import json; d=json.load(open('$OUT/pmc_summary_$V.json')); [print('$V', k[:60], {a: round(b, 4) if isinstance(b, float) else b for a, b in v.items()}) for k, v in d.items()]"
  done
fi
if has pmcx; then
  # extra counters for one pass, e.g. PMCX="TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
  timeout -k 10 300 rocprofv3 --pmc ${PMCX} -f csv -d "$OUT/pmcx" -o run -- \
      python3 bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c2p --no-c5 --graph 0 --steps 5 --warmup 2 --pmc-collect ${PMC_ARGS} > "$OUT/pmcx.json" 2> "$OUT/pmcx.err"
  find "$OUT/pmcx" -name '*counter_collection.csv' -exec cp {} "$OUT/counters_x.csv" \;
  rm -rf "$OUT/pmcx"
  python3 tools/pmc_table.py "$OUT/counters_x.csv" | tee "$OUT/pmcx_table.txt"
fi
