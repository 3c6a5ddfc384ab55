#!/bin/bash
# Run bench.py once per argument set (separated by ';' in $SWEEP), print value + per-kernel times.
# Usage: SWEEP="--overlap 0;--overlap 1;VAR=1 --overlap 0" bash tools/bench_sweep.sh TAG  (VAR=val tokens go to the environment)
set -e -o pipefail
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
IFS=';' read -ra CASES <<< "$SWEEP"
i=0
for c in "${CASES[@]}"; do
  envs=(); args=()
  for tok in $c; do
    if [[ "$tok" != --* && "$tok" == *=* ]]; then envs+=("$tok"); else args+=("$tok"); fi
  done
  timeout -k 10 300 env "${envs[@]}" python bench.py --no-cpu-baseline "${args[@]}" > "$OUT/case$i.json" 2> "$OUT/case$i.err"
  python3 -c "
import json,sys
d=json.load(open('$OUT/case$i.json'))
k=' '.join(f\"{n}={v['avg_ms']*1e3:.1f}\" for n,v in d['kernels'].items())
print(f\"[$c] {d['value']/1e6:.1f} M/s {d['ms_per_step']*1e3:.1f} us/step | {k}\")"
  i=$((i+1))
done
