# Which training-pass kernels slow down under the pipelined sampler: rocprofv3 kernel stats of the Lego
# stand-in step, pipelined and serial. bash tools/r03_pipe_prof.sh TAG
set -e -o pipefail
T=${1:-r03as}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for P in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$T/prof_p$P -o run -- python3 tools/nerf_step_profile.py --pipeline $P --steps 1500 --measure 100 > gpurun_out/$T/p$P.json 2> gpurun_out/$T/p$P.err
  find gpurun_out/$T/prof_p$P -name '*kernel_stats.csv' -exec cp {} gpurun_out/$T/kernel_stats_p$P.csv \;
  rm -rf gpurun_out/$T/prof_p$P
done
python3 - gpurun_out/$T <<'PY'
import csv, sys
d = sys.argv[1]
st = {}
for P in (1, 0):
    for r in csv.DictReader(open(f"{d}/kernel_stats_p{P}.csv")):
        st.setdefault(r["Name"][:70], {})[P] = (int(r["Calls"]), float(r["AverageNs"]) / 1000)
for k, v in sorted(st.items(), key=lambda kv: -kv[1].get(1, (0, 0))[0] * kv[1].get(1, (0, 0))[1])[:25]:
    print(f"{k:70s} pipelined {v.get(1)} serial {v.get(0)}")
PY
