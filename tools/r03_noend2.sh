# sampling_end off under cone stepping: NeRF parity tests, fox timing. bash tools/r03_noend2.sh TAG
set -e -o pipefail
T=${1:-r03al}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nerf.py > gpurun_out/$T/tests.log 2>&1
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 python tools/nerf_step_profile.py --fox --pipeline 0 --steps 1000 --measure 100 > gpurun_out/$T/t_fox.json 2> gpurun_out/$T/t_fox.err
python -c "import json; d=json.load(open('gpurun_out/$T/t_fox.json')); print('fox', d['ms_per_step_wall'], d['phases']['sample_count'])"
timeout -k 10 300 python tools/nerf_step_profile.py --fox --steps 1000 --measure 100 > gpurun_out/$T/t_fox_pipe.json 2> gpurun_out/$T/t_fox_pipe.err
python -c "import json; d=json.load(open('gpurun_out/$T/t_fox_pipe.json')); print('fox pipelined', d['ms_per_step_wall'], {k: v['ms_per_step'] for k, v in d['phases'].items()})"
