# Lego stand-in sampler diagnostics: march statistics (build/diag4) and the cost of sampling_end
# (build/diag1 evaluates it twice) against the in-tree build. bash tools/r03_lego_diag.sh TAG
set -e -o pipefail
T=${1:-r03ac}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
NGP_ENGINE_LIB=$PWD/build/diag4/libngp_engine.so timeout -k 10 300 python tools/nerf_step_profile.py --sampler-stats --pipeline 0 > gpurun_out/$T/lego_stats.json 2> gpurun_out/$T/lego_stats.err
python -c "import json; d=json.load(open('gpurun_out/$T/lego_stats.json')); print(d['sampler_stats']); print({k: v for k, v in d.items() if k not in ('phases', 'sampler_stats')})"
for V in intree diag1; do
  LIBV=""
  if [ $V = diag1 ]; then LIBV=$PWD/build/diag1/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py --pipeline 0 > gpurun_out/$T/t_$V.json 2> gpurun_out/$T/t_$V.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$V.json')); print('$V', d['ms_per_step_wall'], d['phases']['sample_count'])"
done
