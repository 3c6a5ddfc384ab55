# Fused grid update inside captured training steps: lazy-EMA tests on build/fcap, then C2 bench with the
# in-tree build (eager layout) against build/fcap with NGP_LAZY_EMA=1 (lazy layout, fused capture).
set -e -o pipefail
T=r03bw; mkdir -p gpurun_out/$T; export TMPDIR=/tmp
NGP_ENGINE_LIB=$PWD/build/fcap/libngp_engine.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lazy_ema.py > gpurun_out/$T/tests_fcap.log 2>&1
tail -1 gpurun_out/$T/tests_fcap.log
for R in 1 2; do for v in intree fcap; do
  unset NGP_LAZY_EMA NGP_ENGINE_LIB
  if [ $v != intree ]; then export NGP_ENGINE_LIB=$PWD/build/$v/libngp_engine.so NGP_LAZY_EMA=1; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c5 > gpurun_out/$T/b_${v}_$R.json 2> gpurun_out/$T/b_${v}_$R.err
  python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_$R.json')); k=d['kernels']
print('$v', 'C2', round(d['ms_per_step']*1e3,1), {a: round(k[a]['avg_ms']*1e3,1) for a in k}, 'C2p', round(d['c2p']['ms_per_step']*1e3,1))"
done; done
