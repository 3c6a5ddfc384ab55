# Dynamically drawn partitions in the MLP training kernel: GPU tests of the NeRF network, training
# and data-parallel paths; C2 bench (no contention); Lego/fox pipelined step phases. bash tools/r03_mlpdyn.sh TAG
set -e -o pipefail
T=${1:-r03bc}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_nerf.py tests/test_gpu_dp.py tests/test_gpu_network_full.py tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_training.py tests/test_gpu_lazy_ema.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c5 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
python3 -c "import json; d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]); print('C2', d['value']/1e9, d['ms_per_step'], 'mlp', d['kernels']['mlp_train'], 'C2p', d['c2p']['ms_per_step'])"
for S in "" "--fox"; do
  timeout -k 10 300 python tools/nerf_step_profile.py $S > gpurun_out/$T/t$S.json 2> gpurun_out/$T/t$S.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t$S.json')); p=d['phases']; print('$S', d['ms_per_step_wall'], 'train', p['nerf_train_pass']['ms_per_step'], 'count', p['sample_count']['ms_per_step'])"
done
