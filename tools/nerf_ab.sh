# A/B of the full Testbed NeRF step (Lego stand-in and fox) on one GPU box: wall ms per step of
# tools/nerf_step_profile.py without the engine profiler, each variant run twice, interleaved.
#
#   bash tools/nerf_ab.sh TAG [-a "nerf_step_profile.py args"] VARIANT...
#
# VARIANT = name[:KEY=VAL,KEY=VAL...] with KEY an environment variable for that run (as tools/ab.sh).
set -e -o pipefail
T=$1; shift
ARGS="--steps 2000 --measure 1000 --profiler 0"
while getopts "a:" o; do
  case $o in a) ARGS=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
mkdir -p gpurun_out/$T
SET_KEYS=""
apply() {
  unset $SET_KEYS
  local kv=${1#*:}
  [ "$kv" = "$1" ] && return 0
  IFS=',' read -ra pairs <<< "$kv"
  for a in "${pairs[@]}"; do export "${a//;/,}"; SET_KEYS="$SET_KEYS ${a%%=*}"; done
}
for R in 1 2; do
  for v in "$@"; do
    apply "$v"; n=${v%%:*}
    for S in lego fox; do
      F=""; [ $S = fox ] && F=--fox
      timeout -k 10 300 python tools/nerf_step_profile.py $F $ARGS > gpurun_out/$T/t_${S}_${n}_$R.json 2> gpurun_out/$T/t_${S}_${n}_$R.err
      python3 -c "import json; d=json.load(open('gpurun_out/$T/t_${S}_${n}_$R.json')); print('$S $n $R', d['ms_per_step_wall'], round(d['samples_per_s']/1e6,1), 'M/s')"
    done
  done
done
