# Occupancy byte prefetched before the verify step: parity tests, then fox/Lego serial and pipelined
# timing, in-tree against build/pf0 (-DNGP_SAMPLER_PREFETCH=0). bash tools/r03_carry.sh TAG
set -e -o pipefail
T=${1:-r03ax}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1500 --measure 150 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); p=d['phases']; print('$1', d['ms_per_step_wall'], 'count', p['sample_count']['ms_per_step'], 'train', p['nerf_train_pass']['ms_per_step'])"
}
for V in pf pf0; do
  LIBV=""
  if [ $V != pf ]; then LIBV=$PWD/build/$V/libngp_engine.so; fi
  run fox_serial_$V "$LIBV" "--fox --pipeline 0"
  run lego_serial_$V "$LIBV" "--pipeline 0"
  run fox_$V "$LIBV" "--fox"
  run lego_$V "$LIBV" ""
done
