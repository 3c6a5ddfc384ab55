# A/B of engine builds on one GPU box: bench.py single-config records with NGP_ENGINE_LIB pointing at each
# build, each variant twice, interleaved.
#   bash tools/lib_ab.sh TAG "C5 C2p C2" name=path/libngp_engine.so ...
set -e -o pipefail
T=$1; CFGS=$2; shift 2
mkdir -p gpurun_out/$T
for R in 1 2; do
  for v in "$@"; do
    n=${v%%=*}; lib=${v#*=}
    for C in $CFGS; do
      NGP_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --variant $C --steps 30 --warmup 5 --no-cpu-baseline \
        --e2e-seconds 0 --no-c2p --no-c5 --c3-seconds 0 --no-dp1 > gpurun_out/$T/${C}_${n}_$R.json 2> gpurun_out/$T/${C}_${n}_$R.err
      python3 -c "import json; d=json.loads(open('gpurun_out/$T/${C}_${n}_$R.json').read().strip().splitlines()[-1]); print('$C $n $R', round(d['ms_per_step'], 4))"
    done
  done
done
