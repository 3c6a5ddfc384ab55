# Fused-update template split: grid backward / optimizer parity tests, then the default bench
# (C2, C2', C5) and the kernel stats of C2 + C2'. bash tools/r03_fusedtpl.sh TAG
set -e -o pipefail
T=${1:-r03ae}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_lazy_ema.py tests/test_gpu_grid_exact.py tests/test_gpu_training.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
BENCH_ARGS="--no-cpu-baseline --e2e-seconds 0 --c3-seconds 0" bash tools/gpu_round.sh $T bench prof > gpurun_out/$T/round.txt
python3 -c "
import json; d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1])
print('C2', d['value'] / 1e9, d['ms_per_step'], 'C2p', d['c2p']['ms_per_step'], 'C5', d['c5']['ms_per_step'], 'c5_online', d['c5_online']['ms_per_step'])"
grep -E "accumulate|split_reduce" gpurun_out/$T/kernel_stats.csv | cut -c1-40,150-220
