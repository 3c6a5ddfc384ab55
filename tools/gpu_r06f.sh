mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcnn_mode.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r06f/tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
for P in 1 2; do
  for E in 0 1; do
    timeout -k 10 120 python3 tools/dp_trace.py --parts $P --eager $E >> gpurun_out/r06f/dp.txt 2>&1 || exit 1
  done
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python3 tools/dp_trace.py --parts $P >> gpurun_out/r06f/dp.txt 2>&1 || exit 1
  DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 120 python3 tools/dp_trace.py --parts $P >> gpurun_out/r06f/dp.txt 2>&1 || exit 1
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/r06f/trace_p2_nopc -o run -- python3 tools/dp_trace.py --parts 2 > gpurun_out/r06f/trace.txt 2>&1
