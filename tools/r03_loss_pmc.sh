# SQ counters of the Lego stand-in step's per-ray kernels (loss passes, sample write, inference MLP),
# and the sample-write LDS staging A/B (in-tree NGP_SW_STAGE=1 vs build/sw0). bash tools/r03_loss_pmc.sh TAG
set -e -o pipefail
T=${1:-r03bf}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d gpurun_out/$T/pmc -o run -- python3 tools/nerf_step_profile.py --steps 2000 --measure 20 > gpurun_out/$T/pmc.json 2> gpurun_out/$T/pmc.err
find gpurun_out/$T/pmc -name '*counter_collection.csv' -exec cp {} gpurun_out/$T/counters.csv \;
rm -rf gpurun_out/$T/pmc
python3 - gpurun_out/$T/counters.csv <<'PY' | tee gpurun_out/$T/pmc_summary.txt
import csv, sys
from collections import defaultdict
rows = defaultdict(lambda: defaultdict(dict))
for r in csv.DictReader(open(sys.argv[1])):
    for k in ("k_loss_pass1", "k_loss_pass2", "k_sample_write", "k_nerf_mlp<", "k_sample_count", "k_nerf_mlp_train"):
        if k in r["Kernel_Name"]:
            d = rows[k][int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, disp in rows.items():
    last = sorted(disp)[-20:]
    avg = {c: sum(disp[d][c] for d in last) / len(last) for c in disp[last[0]]}
    print(k, "last 20 dispatches", {a: round(b) for a, b in avg.items()})
PY
rm -f gpurun_out/$T/counters.csv
for V in sw1 sw0 sw1 sw0; do
  LIBV=""
  if [ $V = sw0 ]; then LIBV=$PWD/build/sw0/libngp_engine.so; fi
  for S in lego fox; do
    F=""; if [ $S = fox ]; then F=--fox; fi
    NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py $F > gpurun_out/$T/t_${S}_$V.json 2> gpurun_out/$T/t_${S}_$V.err
    python -c "import json; d=json.load(open('gpurun_out/$T/t_${S}_$V.json')); p=d['phases']; print('$S $V', d['ms_per_step_wall'], {k: p[k]['ms_per_call'] for k in ('sample_write','nerf_sample','loss_pass1','loss_pass2','nerf_train_pass')})"
  done
done
