# A/B of NeRF step builds: NeRF parity tests of the in-tree build, then the Lego stand-in and fox steps
# (pipelined, per-phase HIP-event timing) for each variant, interleaved.
# bash tools/ab_nerf_step.sh TAG VARIANT...   (VARIANT: "intree" or a directory under build/)
set -e -o pipefail
T=$1; shift
V=${*:-"intree head"}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/$T/tests.log 2>&1
[ -n "$SKIP_TESTS" ] || tail -1 gpurun_out/$T/tests.log
for R in 1 2; do
  for v in $V; do
    LIBV=""
    if [ $v != intree ]; then LIBV=$PWD/build/$v/libngp_engine.so; fi
    for S in lego fox; do
      F=""; if [ $S = fox ]; then F=--fox; fi
      NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py $F > gpurun_out/$T/t_${S}_${v}_$R.json 2> gpurun_out/$T/t_${S}_${v}_$R.err
      python -c "import json; d=json.load(open('gpurun_out/$T/t_${S}_${v}_$R.json')); p=d['phases']; print('$S $v', d['ms_per_step_wall'], {k: p[k]['ms_per_call'] for k in ('sample_count','sample_write','loss_pass1','loss_pass2','nerf_train_pass','nerf_inference','mlp_infer_enc')})"
    done
  done
done
