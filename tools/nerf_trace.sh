# Steady-state NeRF step under rocprofv3: per-kernel table over the last 40 % of the run (tools/steady_trace.py)
# and the kernel timeline of two steps (tools/trace_steps.py). Usage (on the GPU box):
#   bash tools/nerf_trace.sh TAG lego   (the stand-in, 10-s tools/psnr30.py run)
#   bash tools/nerf_trace.sh TAG fox    (data/fox, 3000 steps of tools/nerf_step_profile.py --fox)
# -> gpurun_out/TAG/<scene>_steady.txt, <scene>_steps.txt
set -e -o pipefail
T=${1:-nerf_trace}; S=${2:-lego}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
if [ "$S" = fox ]; then
  CMD="python3 tools/nerf_step_profile.py --fox --steps 3000 --measure 500 --profiler 0"; SHOW="3000 3001"
else
  CMD="python3 tools/psnr30.py --seconds 10 --test-views 1"; SHOW="15000 15001"
fi
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/$T/$S -o run -- $CMD > gpurun_out/$T/$S.json 2> gpurun_out/$T/$S.err
python3 tools/steady_trace.py gpurun_out/$T/$S/run_kernel_trace.csv 40 > gpurun_out/$T/${S}_steady.txt
python3 tools/trace_steps.py gpurun_out/$T/$S/run_kernel_trace.csv --show $SHOW > gpurun_out/$T/${S}_steps.txt
rm -f gpurun_out/$T/$S/run_kernel_trace.csv
