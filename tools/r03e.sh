set -e -o pipefail
T=${1:-r03e}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
tail -3 gpurun_out/$T/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c2p > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
python -c "import json; d=json.load(open('gpurun_out/$T/bench.json')); print(d['value'], d['c5']['ms_per_step'], json.dumps(d.get('c5_online')))"
