# s_setprio in the MLP training kernel: Lego/fox pipelined step timing and the pipelined kernel stats,
# in-tree (priority 3) against build/p0 (default priority). bash tools/r03_prio.sh TAG
set -e -o pipefail
T=${1:-r03au}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
run() {  # name lib args
  NGP_ENGINE_LIB=$2 timeout -k 10 300 python tools/nerf_step_profile.py $3 --steps 1500 --measure 150 > gpurun_out/$T/t_$1.json 2> gpurun_out/$T/t_$1.err
  python -c "import json; d=json.load(open('gpurun_out/$T/t_$1.json')); p=d['phases']; print('$1', d['ms_per_step_wall'], 'count', p['sample_count']['ms_per_step'], 'train', p['nerf_train_pass']['ms_per_step'], 'sample', p['nerf_sample']['ms_per_step'])"
}
for V in prio3 p0; do
  LIBV=""
  if [ $V != prio3 ]; then LIBV=$PWD/build/$V/libngp_engine.so; fi
  run lego_$V "$LIBV" ""
  run fox_$V "$LIBV" "--fox"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$T/prof -o run -- python3 tools/nerf_step_profile.py --steps 1500 --measure 100 > gpurun_out/$T/prof.json 2> gpurun_out/$T/prof.err
find gpurun_out/$T/prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/$T/kernel_stats_pipelined.csv \;
rm -rf gpurun_out/$T/prof
grep -E "mlp_train|sample_count|sc_scatter|sc_accum" gpurun_out/$T/kernel_stats_pipelined.csv | cut -c1-60,120-200
