# fused grid optimizer: parity tests, the C5 bench and its PMC passes (bash tools/r03_fused.sh TAG)
set -e -o pipefail
T=${1:-r03fused}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lazy_ema.py tests/test_gpu_network_full.py tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python bench.py --variant C5 --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err
python -c "import json; d=json.load(open('gpurun_out/$T/bench_c5.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline']), json.dumps(d['optimizer_params']))"
PMC_VARIANTS=C5 bash tools/gpu_round.sh $T pmc
