# NeRF step phases on the Lego stand-in (pipelined and serial) and on fox (bash tools/r03_phases.sh TAG)
set -e -o pipefail
T=${1:-r03w}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python tools/nerf_step_profile.py > gpurun_out/$T/lego_phases.json 2> gpurun_out/$T/lego_phases.err
timeout -k 10 300 python tools/nerf_step_profile.py --pipeline 0 > gpurun_out/$T/lego_phases_serial.json 2> gpurun_out/$T/lego_phases_serial.err
timeout -k 10 300 python tools/nerf_step_profile.py --fox > gpurun_out/$T/fox_phases.json 2> gpurun_out/$T/fox_phases.err
for f in lego_phases lego_phases_serial fox_phases; do python -c "
import json; d=json.load(open('gpurun_out/$T/$f.json')); print('$f', d['ms_per_step_wall'], {k: v['ms_per_step'] for k, v in d['phases'].items()})"; done
