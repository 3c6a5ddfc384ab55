# Cost of the count pass's tbuf stores: in-tree build against build/diag5 (stores suppressed), fox and
# Lego serial steps. bash tools/r03_storecost.sh TAG
set -e -o pipefail
T=${1:-r03ag}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for S in --fox ""; do
for V in intree diag5; do
  LIBV=""
  if [ $V = diag5 ]; then LIBV=$PWD/build/diag5/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py $S --pipeline 0 --steps 1000 --measure 100 > gpurun_out/$T/t_$V$S.json 2> gpurun_out/$T/t_$V$S.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$V$S.json')); print('$V$S', d['ms_per_step_wall'], d['phases']['sample_count'])"
done
done
