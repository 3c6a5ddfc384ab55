# steady-state kernel trace of the full NeRF step on the Lego stand-in (e2e), and of the fox step (C3)
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d gpurun_out/r06i/lego -o run -- python3 tools/psnr30.py --seconds 10 --test-views 1 > gpurun_out/r06i/lego.json 2> gpurun_out/r06i/lego.err || exit 1
python3 tools/steady_trace.py gpurun_out/r06i/lego/run_kernel_trace.csv 40 > gpurun_out/r06i/lego_steady.txt
python3 tools/trace_steps.py gpurun_out/r06i/lego/run_kernel_trace.csv --show 15000 15001 > gpurun_out/r06i/lego_steps.txt
gzip -c gpurun_out/r06i/lego/run_kernel_trace.csv > /dev/null
rm -f gpurun_out/r06i/lego/run_kernel_trace.csv
