# A/B of engine builds on the synthetic C2 / C2' / C5 training passes (bench.py, no end-to-end runs), with the
# grid-exactness tests run against each variant first. bash tools/ab_bench.sh TAG VARIANT...
#   VARIANT: "intree" or a directory under build/ holding libngp_engine.so
set -e -o pipefail
T=$1; shift
V=${*:-"intree"}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for v in $V; do
  LIBV=""; if [ $v != intree ]; then LIBV=$PWD/build/$v/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_grid_exact.py tests/test_gpu_parity.py > gpurun_out/$T/tests_$v.log 2>&1
  echo "$v $(tail -1 gpurun_out/$T/tests_$v.log)"
done
for R in 1 2; do
  for v in $V; do
    LIBV=""; if [ $v != intree ]; then LIBV=$PWD/build/$v/libngp_engine.so; fi
    NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 > gpurun_out/$T/b_${v}_$R.json 2> gpurun_out/$T/b_${v}_$R.err
    python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_$R.json'))
k=d['kernels']; c=d['c2p']['kernels']; f=d['c5']['kernels']
print('$v', 'C2', round(d['ms_per_step']*1e3,1), {a: round(k[a]['avg_ms']*1e3,1) for a in k}, 'C2p', round(d['c2p']['ms_per_step']*1e3,1), round(c['grid_backward_total']['avg_ms']*1e3,1), 'C5', round(d['c5']['ms_per_step']*1e3,1), round(f['grid_backward_total']['avg_ms']*1e3,1))
"
  done
done
