# Single-workgroup scans (sampler base/keep/slot in one launch, loss compaction scan): NeRF parity
# tests, then fox and Lego step phases, serial and pipelined. bash tools/r03_scan1.sh TAG
set -e -o pipefail
T=${1:-r03ao}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py tests/test_gpu_dp.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
run() {  # name args
  timeout -k 10 300 python tools/nerf_step_profile.py $2 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); print('$1', d['ms_per_step_wall'], {k: v['ms_per_step'] for k, v in d['phases'].items()})"
}
run fox_serial "--fox --pipeline 0"
run fox "--fox"
run lego_serial "--pipeline 0"
run lego ""
