# A/B runs on one GPU box: optional parity tests, then bench.py (and optionally the NeRF step profile) for each
# variant, interleaved twice so that clock drift hits every variant alike. One summary line per run.
#
#   bash tools/ab.sh TAG [-t "test files"] [-b "bench.py args"] [-n] VARIANT...
#
# VARIANT = name[:KEY=VAL,KEY=VAL...]. KEY is an environment variable for that run (NGP_MODEL_OPTS="k=v;k=v"
# sets engine options on every model, NGP_SC_* the grid-backward plan knobs, ...), or lib=DIR to load
# build/DIR/libngp_engine.so instead of the in-tree engine. -t runs the tests under the LAST variant's
# settings first; -n adds the Lego stand-in and fox step profiles (tools/nerf_step_profile.py). Outputs go to
# gpurun_out/TAG/.  Example: bash tools/ab.sh r04x -t tests/test_gpu_network_full.py new old:NGP_MODEL_OPTS="fuse_slabs=0"
set -e -o pipefail
T=$1; shift
TESTS=""; BENCH="--no-cpu-baseline --e2e-seconds 0 --c3-seconds 0"; NERF=""
while getopts "t:b:n" o; do
  case $o in t) TESTS=$OPTARG ;; b) BENCH=$OPTARG ;; n) NERF=1 ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
SET_KEYS=""
apply() {  # reset (every variable an earlier variant exported), then export the variant's settings
  unset NGP_ENGINE_LIB NGP_MODEL_OPTS NGP_SC_BT NGP_SC_LDS_KB NGP_SC_CHUNK NGP_SC_PART NGP_SC_LIMIT $SET_KEYS
  local kv=${1#*:}
  [ "$kv" = "$1" ] && return 0
  IFS=',' read -ra pairs <<< "$kv"
  for a in "${pairs[@]}"; do
    if [[ $a == lib=* ]]; then export NGP_ENGINE_LIB=$PWD/build/${a#lib=}/libngp_engine.so
    else export "${a//;/,}"; SET_KEYS="$SET_KEYS ${a%%=*}"; fi
  done
}
if [ -n "$TESTS" ]; then
  apply "${@: -1}"
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/$T/tests.log 2>&1
  tail -1 gpurun_out/$T/tests.log
fi
for R in 1 2; do
  for v in "$@"; do
    apply "$v"; n=${v%%:*}
    timeout -k 10 400 python bench.py $BENCH > gpurun_out/$T/b_${n}_$R.json 2> gpurun_out/$T/b_${n}_$R.err
    python3 - gpurun_out/$T/b_${n}_$R.json "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
out = {"C2": round(d["ms_per_step"] * 1e3, 1)}
for k in ("c2p", "c5"):
    if k in d:
        out[k] = round(d[k]["ms_per_step"] * 1e3, 1)
for k in ("e2e", "c3"):
    if k in d and "ms_per_step" in d[k]:
        out[k] = round(d[k]["ms_per_step"] * 1e3, 1)
ks = d.get("kernels", {})
out["kernels_us"] = {a: round(ks[a]["avg_ms"] * 1e3, 1) for a in ks}
print(sys.argv[2], json.dumps(out))
PY
    if [ -n "$NERF" ]; then
      for S in lego fox; do
        F=""; [ $S = fox ] && F=--fox
        timeout -k 10 300 python tools/nerf_step_profile.py $F > gpurun_out/$T/t_${S}_${n}_$R.json 2> gpurun_out/$T/t_${S}_${n}_$R.err
        python3 -c "import json; d=json.load(open('gpurun_out/$T/t_${S}_${n}_$R.json')); p=d['phases']; print('$S $n', d['ms_per_step_wall'], {k: p[k]['ms_per_call'] for k in p if k in ('sample_count','loss_pass1','loss_pass2','nerf_train_pass','nerf_inference','mlp_train')})"
      done
    fi
  done
done
