set -e -o pipefail
T=${1:-r03m}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_network_full.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
tail -2 gpurun_out/$T/tests.log
for V in lib lib_b; do
NGP_ENGINE_LIB=$PWD/instant-ngp_amd/$V/libngp_engine.so timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --c5-online-steps 0 --no-c5 > gpurun_out/$T/bench_$V.json 2> gpurun_out/$T/bench_$V.err
python -c "import json; d=json.load(open('gpurun_out/$T/bench_$V.json')); print('$V', d['value'], d['ms_per_step'], d['kernels']['mlp_train'], d['c2p']['kernels']['mlp_train']['avg_ms'])"
done
