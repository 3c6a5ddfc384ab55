# SDF ground-truth A/B: parity tests, then the armadillo profile (bash tools/r03_sdf.sh TAG)
set -e -o pipefail
T=${1:-r03sdf}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python tools/sdf_gt_profile.py > gpurun_out/$T/sdf_gt.json 2> gpurun_out/$T/sdf_gt.err
cat gpurun_out/$T/sdf_gt.json
