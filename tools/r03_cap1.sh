# Verify-round cap 1 (in-tree): parity tests; fox timing in-tree vs RG 16 (build/rg16); Lego timing
# in-tree vs the unified loop at cone 0 (build/u0), serial and pipelined. bash tools/r03_cap1.sh TAG
set -e -o pipefail
T=${1:-r03ai}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py tests/test_gpu_render.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1000 --measure 100 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); print('$1', d['ms_per_step_wall'], d['phases']['sample_count'], d['phases'].get('nerf_train_pass'))"
}
run fox_cap1 "" "--fox --pipeline 0"
run fox_rg16 $PWD/build/rg16/libngp_engine.so "--fox --pipeline 0"
run fox_cap1_pipe "" "--fox"
run lego_cap1 "" "--pipeline 0"
run lego_u0 $PWD/build/u0/libngp_engine.so "--pipeline 0"
run lego_cap1_pipe "" ""
run lego_u0_pipe $PWD/build/u0/libngp_engine.so ""
