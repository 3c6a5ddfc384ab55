set -e -o pipefail
mkdir -p gpurun_out/r06ay
for S in lego fox; do
  F=""; [ $S = fox ] && F=--fox
  for d in 0 64 1; do
    timeout -k 10 200 python tools/nerf_step_profile.py $F --steps 1500 --measure 300 --profiler 1 --option-after-warmup win_debug=$d > gpurun_out/r06ay/${S}_$d.json 2> gpurun_out/r06ay/${S}_$d.err
    python3 -c "import json; d=json.load(open('gpurun_out/r06ay/${S}_$d.json')); p=d['phases']; print('$S', $d, d['ms_per_step_wall'], {k: p[k]['ms_per_call'] for k in p if 'grid' in k or 'train' in k})"
  done
done
