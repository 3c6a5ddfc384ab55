#!/bin/bash
# Run bench.py once per argument set (separated by ';' in $SWEEP), print value + per-kernel times.
# Usage: SWEEP="--overlap 0;--overlap 1" bash tools/bench_sweep.sh TAG
set -e -o pipefail
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
IFS=';' read -ra CASES <<< "$SWEEP"
i=0
for c in "${CASES[@]}"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $c > "$OUT/case$i.json" 2> "$OUT/case$i.err"
  python3 -c "
import json,sys
d=json.load(open('$OUT/case$i.json'))
k=' '.join(f\"{n}={v['avg_ms']*1e3:.1f}\" for n,v in d['kernels'].items())
print(f\"[$c] {d['value']/1e6:.1f} M/s {d['ms_per_step']*1e3:.1f} us/step | {k}\")"
  i=$((i+1))
done
