# Kernel order of the last Lego steps (rocprofv3 kernel trace), to place the per-step buffer copies.
# bash tools/r03_ktrace.sh TAG
set -e -o pipefail
T=${1:-r03ay}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/$T/kt -o run -- python3 tools/nerf_step_profile.py --steps 300 --measure 5 > gpurun_out/$T/p.json 2> gpurun_out/$T/p.err
find gpurun_out/$T/kt -name '*kernel_trace.csv' -exec cp {} gpurun_out/$T/kernel_trace.csv \;
rm -rf gpurun_out/$T/kt
python3 - gpurun_out/$T/kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-90:]:
    print(r.get("Queue_Id", ""), r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) // 1000)
PY
