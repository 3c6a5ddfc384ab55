set -e -o pipefail
T=r03bu; mkdir -p gpurun_out/$T; export TMPDIR=/tmp
NGP_ENGINE_LIB=$PWD/build/new/libngp_engine.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lazy_ema.py tests/test_gpu_network_full.py tests/test_gpu_grid_exact.py tests/test_gpu_parity.py tests/test_snapshot.py > gpurun_out/$T/tests_new.log 2>&1
tail -1 gpurun_out/$T/tests_new.log
for R in 1 2; do for v in prev new; do
  NGP_ENGINE_LIB=$PWD/build/$v/libngp_engine.so timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c2p > gpurun_out/$T/b_${v}_$R.json 2> gpurun_out/$T/b_${v}_$R.err
  python -c "
import json; d=json.load(open('gpurun_out/$T/b_${v}_$R.json')); f=d['c5']['kernels']
print('$v', 'C2', round(d['ms_per_step']*1e3,1), 'C5', round(d['c5']['ms_per_step']*1e3,1), {a: round(f[a]['avg_ms']*1e3,1) for a in f})"
done; done
