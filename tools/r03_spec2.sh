# Empty-space march A/B on fox: parity tests, march statistics (build/diag4), serial-step timing of the
# in-tree build against build/spec0 (exact chain). bash tools/r03_spec2.sh TAG
set -e -o pipefail
T=${1:-r03z}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
NGP_ENGINE_LIB=$PWD/build/diag4/libngp_engine.so timeout -k 10 300 python tools/nerf_step_profile.py --fox --sampler-stats > gpurun_out/$T/fox_stats.json 2> gpurun_out/$T/fox_stats.err
python -c "import json; print(json.load(open('gpurun_out/$T/fox_stats.json'))['sampler_stats'])"
for V in spec spec0; do
  LIBV=""
  if [ $V = spec0 ]; then LIBV=$PWD/build/spec0/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py --fox --pipeline 0 > gpurun_out/$T/t_$V.json 2> gpurun_out/$T/t_$V.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$V.json')); print('$V', d['ms_per_step_wall'], d['phases']['sample_count'])"
done
