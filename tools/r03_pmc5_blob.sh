# C5 PMC passes (fused optimizer, no unfused counting step) and the C2 pass on NeRF-like concentrated
# points (NGP_BENCH_POINTS=blob) next to uniform ones (bash tools/r03_pmc5_blob.sh TAG)
set -e -o pipefail
T=${1:-r03v}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
PMC_VARIANTS=C5 bash tools/gpu_round.sh $T pmc > gpurun_out/$T/pmc_stdout.txt
grep -E "adam|accumul|split" gpurun_out/$T/pmc_stdout.txt | cut -c1-250
for P in uniform blob; do
NGP_BENCH_POINTS=$P timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-seconds 0 --c3-seconds 0 --no-c2p --no-c5 > gpurun_out/$T/bench_$P.json 2> gpurun_out/$T/bench_$P.err
python -c "import json; d=json.load(open('gpurun_out/$T/bench_$P.json')); print('$P', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
