# rocprofv3 kernel stats of the C5 training step alone (bench.py --variant C5), then the PMC passes of C2'.
set -e -o pipefail
OUT=gpurun_out/${1:-r03by}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof5" -o run -- \
    python3 bench.py --variant C5 --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c2p --no-c5 --steps 20 --warmup 5 > "$OUT/prof5_bench.json" 2> "$OUT/prof5.err"
find "$OUT/prof5" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_c5.csv" \;
rm -rf "$OUT/prof5"
head -14 "$OUT/kernel_stats_c5.csv" | cut -d, -f1-8
PMC_VARIANTS=C2p bash tools/gpu_round.sh ${1:-r03by} pmc
