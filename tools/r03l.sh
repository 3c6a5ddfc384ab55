set -e -o pipefail
T=${1:-r03l}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_network_full.py tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_input_grad.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
tail -3 gpurun_out/$T/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --c5-online-steps 0 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
python -c "import json; d=json.load(open('gpurun_out/$T/bench.json')); print(d['value'], d['ms_per_step'], d['kernels']['mlp_train'], d['c2p']['kernels']['mlp_train'], d['c5']['ms_per_step'])"
