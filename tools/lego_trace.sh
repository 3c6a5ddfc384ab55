# Steady-state NeRF step on the Lego stand-in under rocprofv3: per-kernel table over the last 40 % of a 10-s run
# (tools/steady_trace.py) and the kernel timeline of two steps (tools/trace_steps.py). Usage (on the GPU box):
#   bash tools/lego_trace.sh TAG   -> gpurun_out/TAG/lego_steady.txt, lego_steps.txt
set -e -o pipefail
T=${1:-lego_trace}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/$T/lego -o run -- python3 tools/psnr30.py --seconds 10 --test-views 1 > gpurun_out/$T/lego.json 2> gpurun_out/$T/lego.err
python3 tools/steady_trace.py gpurun_out/$T/lego/run_kernel_trace.csv 40 > gpurun_out/$T/lego_steady.txt
python3 tools/trace_steps.py gpurun_out/$T/lego/run_kernel_trace.csv --show 15000 15001 > gpurun_out/$T/lego_steps.txt
rm -f gpurun_out/$T/lego/run_kernel_trace.csv
