# Loss-pass prefetch depth A/B (NGP_LOSS_PF = 1, 2 in-tree, 4): parity tests of the in-tree build, then
# the Lego stand-in and fox steps with the engine's per-phase timing. bash tools/r03_losspf.sh TAG
set -e -o pipefail
T=${1:-r03be}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
for V in pf2 pf1 pf4; do
  LIBV=""
  if [ $V != pf2 ]; then LIBV=$PWD/build/$V/libngp_engine.so; fi
  for S in lego fox; do
    F=""; if [ $S = fox ]; then F=--fox; fi
    NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py $F > gpurun_out/$T/t_${S}_$V.json 2> gpurun_out/$T/t_${S}_$V.err
    python -c "import json; d=json.load(open('gpurun_out/$T/t_${S}_$V.json')); p=d['phases']; print('$S $V', d['ms_per_step_wall'], {k: p[k]['ms_per_call'] for k in ('loss_pass1','loss_pass2','nerf_loss','nerf_train_pass','nerf_sample')})"
  done
done
