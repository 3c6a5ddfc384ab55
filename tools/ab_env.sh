# A/B of grid-backward plan knobs on the in-tree build (C5 / C2 / C2' via bench.py): the fused/grid tests
# under the last variant's environment, then each variant twice. Variants: "name:VAR=val,VAR=val".
set -e -o pipefail
T=$1; shift; mkdir -p gpurun_out/$T; export TMPDIR=/tmp
apply() { unset NGP_SC_BT NGP_SC_LDS_KB NGP_SC_CHUNK NGP_SC_PART NGP_SC_LIMIT; local kv=${1#*:}; [ "$kv" = "$1" ] && return 0; for a in ${kv//,/ }; do export "$a"; done; }
last=${@: -1}; apply "$last"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lazy_ema.py tests/test_gpu_grid_exact.py tests/test_gpu_network_full.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
for R in 1 2; do for v in "$@"; do
  apply "$v"; n=${v%%:*}
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 > gpurun_out/$T/b_${n}_$R.json 2> gpurun_out/$T/b_${n}_$R.err
  python -c "
import json; d=json.load(open('gpurun_out/$T/b_${n}_$R.json')); f=d['c5']['kernels']
print('$n', 'C2', round(d['ms_per_step']*1e3,1), 'C2p', round(d['c2p']['ms_per_step']*1e3,1), 'C5', round(d['c5']['ms_per_step']*1e3,1), {a: round(f[a]['avg_ms']*1e3,1) for a in ('grid_backward_adam','grid_bwd_prepare')})"
done; done
