# Count-pass waves per SIMD (grid-stride over rays): parity tests, then Lego/fox step timing,
# pipelined and serial, for 2 (in-tree), 0 (one group per ray, build/w0) and 3 (build/w3).
# bash tools/r03_waves.sh TAG
set -e -o pipefail
T=${1:-r03at}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1500 --measure 150 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); p=d['phases']; print('$1', d['ms_per_step_wall'], 'count', p['sample_count']['ms_per_step'], 'train', p['nerf_train_pass']['ms_per_step'], 'sample', p['nerf_sample']['ms_per_step'])"
}
for W in w2 w0 w3; do
  LIBV=""
  if [ $W != w2 ]; then LIBV=$PWD/build/$W/libngp_engine.so; fi
  run lego_$W "$LIBV" ""
  run fox_$W "$LIBV" "--fox"
done
run lego_w2_serial "" "--pipeline 0"
