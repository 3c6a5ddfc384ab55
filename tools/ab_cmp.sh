# A/B of engine builds: the fused/lazy-EMA/grid/network GPU tests on the last variant, then bench.py (C2, C2', C5)
# of every variant twice. Usage: bash tools/ab_cmp.sh TAG VARIANT... ("intree" or a directory under build/).
# Earlier runs: r03bz intree/cmp, r03ca intree/cmp2, r03cb cmp/cmp3 (the compacted fused update).
set -e -o pipefail
T=$1; shift; mkdir -p gpurun_out/$T; export TMPDIR=/tmp
lib() { if [ "$1" = intree ]; then unset NGP_ENGINE_LIB; else export NGP_ENGINE_LIB=$PWD/build/$1/libngp_engine.so; fi; }
last=${@: -1}; lib $last
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lazy_ema.py tests/test_gpu_network_full.py tests/test_gpu_grid_exact.py > gpurun_out/$T/tests_$last.log 2>&1
tail -1 gpurun_out/$T/tests_$last.log
for R in 1 2; do for v in "$@"; do
  lib $v
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 > gpurun_out/$T/b_${v}_$R.json 2> gpurun_out/$T/b_${v}_$R.err
  python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_$R.json')); f=d['c5']['kernels']
print('$v', 'C2', round(d['ms_per_step']*1e3,1), 'C2p', round(d['c2p']['ms_per_step']*1e3,1), 'C5', round(d['c5']['ms_per_step']*1e3,1), {a: round(f[a]['avg_ms']*1e3,1) for a in f})"
done; done
