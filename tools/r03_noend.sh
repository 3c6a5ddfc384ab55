# sampling_end against the plain march to the aabb exit (build/diag2), Lego and fox serial steps.
# bash tools/r03_noend.sh TAG
set -e -o pipefail
T=${1:-r03ak}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1000 --measure 100 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); print('$1', d['ms_per_step_wall'], d['phases']['sample_count'])"
}
run lego "" "--pipeline 0"
run lego_noend $PWD/build/diag2/libngp_engine.so "--pipeline 0"
run fox "" "--fox --pipeline 0"
run fox_noend $PWD/build/diag2/libngp_engine.so "--fox --pipeline 0"
