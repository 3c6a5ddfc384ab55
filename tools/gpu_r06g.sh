mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
for P in 1 2; do
  timeout -k 10 120 python3 tools/dp_trace.py --parts $P >> gpurun_out/r06g/dp.txt 2>&1 || exit 1
  NGP_XS_PRIORITY=0 timeout -k 10 120 python3 tools/dp_trace.py --parts $P >> gpurun_out/r06g/dp.txt 2>&1 || exit 1
  timeout -k 10 120 python3 tools/dp_trace.py --parts $P --eager 1 >> gpurun_out/r06g/dp.txt 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 tools/dp_trace.py --parts $P >> gpurun_out/r06g/dp.txt 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/r06g/trace_p2 -o run -- python3 tools/dp_trace.py --parts 2 > gpurun_out/r06g/trace.txt 2>&1
