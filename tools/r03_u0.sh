# Unified guess-and-verify march at cone 0 (Lego stand-in): parity tests, then pipelined and serial
# step phases of the in-tree build against build/u0off (-DNGP_SAMPLER_UNIFIED0=0). bash tools/r03_u0.sh TAG
set -e -o pipefail
T=${1:-r03ab}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
for V in u0 u0off; do
  LIBV=""
  if [ $V = u0off ]; then LIBV=$PWD/build/u0off/libngp_engine.so; fi
  for P in 1 0; do
    NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py --pipeline $P > gpurun_out/$T/lego_${V}_p$P.json 2> gpurun_out/$T/lego_${V}_p$P.err
    python -c "import json; d=json.load(open('gpurun_out/$T/lego_${V}_p$P.json')); print('$V p$P', d['ms_per_step_wall'], {k: v['ms_per_step'] for k, v in d['phases'].items() if k in ('sample_count', 'nerf_train_pass', 'nerf_sample')})"
  done
done
