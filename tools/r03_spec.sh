# Speculative empty-space march (cone stepping): sampler parity tests, then the fox step phases (bash tools/r03_spec.sh TAG)
set -e -o pipefail
T=${1:-r03x}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python tools/nerf_step_profile.py --fox > gpurun_out/$T/fox_phases.json 2> gpurun_out/$T/fox_phases.err
timeout -k 10 300 python tools/nerf_step_profile.py --fox --pipeline 0 > gpurun_out/$T/fox_phases_serial.json 2> gpurun_out/$T/fox_phases_serial.err
for f in fox_phases fox_phases_serial; do python -c "
import json; d=json.load(open('gpurun_out/$T/$f.json')); print('$f', d['ms_per_step_wall'], {k: v['ms_per_step'] for k, v in d['phases'].items()})"; done
