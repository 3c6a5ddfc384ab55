# Lanes per ray in the fox sampler: in-tree build (RG 8) against build/rg16 (-DNGP_SAMPLER_RG=16):
# parity tests with the RG 16 build, then serial-step timing of both. bash tools/r03_rg.sh TAG
set -e -o pipefail
T=${1:-r03aa}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
NGP_ENGINE_LIB=$PWD/build/rg16/libngp_engine.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests_rg16.log 2>&1
tail -1 gpurun_out/$T/tests_rg16.log
for V in rg8 rg16; do
  LIBV=""
  if [ $V = rg16 ]; then LIBV=$PWD/build/rg16/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py --fox --pipeline 0 > gpurun_out/$T/t_$V.json 2> gpurun_out/$T/t_$V.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$V.json')); print('$V', d['ms_per_step_wall'], d['phases']['sample_count'])"
done
