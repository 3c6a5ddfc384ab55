# SQ counters of the fox sampler count pass, the speculative empty march against the exact chain
# (build/spec0: -DNGP_SAMPLER_EMPTY_SPEC=0). bash tools/r03_sampler_pmc.sh TAG
set -e -o pipefail
T=${1:-r03y}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for V in spec spec0; do
  LIBV=""
  if [ $V = spec0 ]; then LIBV=$PWD/build/spec0/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -s KILL 240 rocprofv3 --pmc $C -f csv -d gpurun_out/$T/pmc_$V -o run -- python3 tools/nerf_step_profile.py --fox --steps 2000 --measure 20 > gpurun_out/$T/$V.json 2> gpurun_out/$T/$V.err
  find gpurun_out/$T/pmc_$V -name '*counter_collection.csv' -exec cp {} gpurun_out/$T/counters_$V.csv \;
  rm -rf gpurun_out/$T/pmc_$V
  python3 - gpurun_out/$T/counters_$V.csv <<'PY'
import sys
sys.path.insert(0, "tools")
import csv
from collections import defaultdict
rows = defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    if "sample_count" in r["Kernel_Name"]:
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = rows[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
last = sorted(rows)[-20:]
avg = {c: sum(rows[d][c] for d in last) / len(last) for c in rows[last[0]]}
print(sys.argv[1], "last 20 sample_count dispatches", {a: round(b) for a, b in avg.items()})
PY
  rm -f gpurun_out/$T/counters_$V.csv  # large; the printed summary is the record
done
for V in spec spec0 spec; do
  LIBV=""
  if [ $V = spec0 ]; then LIBV=$PWD/build/spec0/libngp_engine.so; fi
  NGP_ENGINE_LIB=$LIBV timeout -k 10 300 python tools/nerf_step_profile.py --fox --pipeline 0 > gpurun_out/$T/t_$V.json 2> gpurun_out/$T/t_$V.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$V.json')); print('$V', d['ms_per_step_wall'], d['phases']['sample_count'])"
done
