export TMPDIR=/tmp; mkdir -p gpurun_out/r04k
NGP_ENGINE_LIB=$PWD/build/t16t/libngp_engine.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_network_full.py > gpurun_out/r04k/tests_t16t.log 2>&1; rc=$?
tail -1 gpurun_out/r04k/tests_t16t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_grid_bricks.py tests/test_gpu_grid_exact.py tests/test_gpu_parity.py tests/test_gpu_network_full.py > gpurun_out/r04k/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04k/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for b in 0 1; do
  NGP_MODEL_OPTS=grid_bricks=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04k/prof_$b -o run -- python3 bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c5 --pmc-collect --steps 20 --warmup 3 > gpurun_out/r04k/b_$b.json 2> gpurun_out/r04k/b_$b.err || exit 1
  find gpurun_out/r04k/prof_$b -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04k/stats_$b.csv \;
  rm -rf gpurun_out/r04k/prof_$b
done
bash tools/ab.sh r04k2 -b "--no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c5" nostage0:NGP_MODEL_OPTS=grid_stage0=0 g16:lib=g16 t16t:lib=t16t base
