# Idle time of the NeRF step's queues at steady state: rocprofv3 kernel trace of the Lego stand-in and fox
# steps (engine profiler off), then per step: wall, the main queue's busy time and its idle gaps.
# bash tools/gaps.sh TAG
set -e -o pipefail
T=${1:-r03bk}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for S in lego fox; do
  F=""; if [ $S = fox ]; then F=--fox; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/$T/kt_$S -o run -- python3 tools/nerf_step_profile.py $F --steps 2000 --measure 40 --profiler 0 > gpurun_out/$T/p_$S.json 2> gpurun_out/$T/p_$S.err
  find gpurun_out/$T/kt_$S -name '*kernel_trace.csv' -exec cp {} gpurun_out/$T/kernel_trace_$S.csv \;
  rm -rf gpurun_out/$T/kt_$S
  python3 tools/step_gaps.py gpurun_out/$T/kernel_trace_$S.csv --last 30 | tee gpurun_out/$T/gaps_$S.txt
  python3 -c "import json; print('$S wall ms/step', json.load(open('gpurun_out/$T/p_$S.json'))['ms_per_step_wall'])"
done
