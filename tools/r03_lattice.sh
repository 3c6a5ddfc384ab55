# Lattice march: NeRF/render parity tests, then serial and pipelined step timing (fox, Lego) of the
# in-tree build against build/lat0 (-DNGP_SAMPLER_LATTICE=0). bash tools/r03_lattice.sh TAG
set -e -o pipefail
T=${1:-r03am}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1000 --measure 100 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); print('$1', d['ms_per_step_wall'], d['phases']['sample_count'])"
}
run fox "" "--fox --pipeline 0"
run fox_lat0 $PWD/build/lat0/libngp_engine.so "--fox --pipeline 0"
run lego "" "--pipeline 0"
run lego_lat0 $PWD/build/lat0/libngp_engine.so "--pipeline 0"
run fox_pipe "" "--fox"
run lego_pipe "" ""
