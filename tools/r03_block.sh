# Sampler block size: 256 (in-tree) against 64 and 128 threads, fox and Lego serial steps.
# bash tools/r03_block.sh TAG
set -e -o pipefail
T=${1:-r03an}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1000 --measure 100 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); print('$1', d['ms_per_step_wall'], d['phases']['sample_count'])"
}
for B in b256 b64 b128; do
  LIBV=""
  if [ $B != b256 ]; then LIBV=$PWD/build/$B/libngp_engine.so; fi
  run fox_$B "$LIBV" "--fox --pipeline 0"
  run lego_$B "$LIBV" "--pipeline 0"
done
