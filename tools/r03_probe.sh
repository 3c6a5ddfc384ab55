# one-off GPU probes used this round (SDF ground truth profile + statistics): bash tools/r03_probe.sh TAG
set -e -o pipefail
T=${1:-r03probe}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python tools/sdf_gt_profile.py > gpurun_out/$T/sdf_gt.json 2> gpurun_out/$T/sdf_gt.err
cat gpurun_out/$T/sdf_gt.json
NGP_SDF_STATS=1 timeout -k 10 300 python tools/sdf_gt_profile.py > gpurun_out/$T/sdf_gt_stats.json 2> gpurun_out/$T/sdf_gt_stats.err
grep sdf_sign_stats gpurun_out/$T/sdf_gt_stats.err | sort -u
