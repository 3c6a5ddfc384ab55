# Verify-round cap of the unified cone march: parity tests (in-tree, cap 2), then fox serial-step timing
# of caps 0 (unlimited), 1, 2 (in-tree), 3. bash tools/r03_cap.sh TAG
set -e -o pipefail
T=${1:-r03ah}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
for V in cap2 cap0 cap1 cap3; do
  LIBV=""
  if [ $V != cap2 ]; then LIBV=$PWD/build/$V/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py --fox --pipeline 0 --steps 1000 --measure 100 > gpurun_out/$T/t_$V.json 2> gpurun_out/$T/t_$V.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$V.json')); print('$V', d['ms_per_step_wall'], d['phases']['sample_count'])"
done
