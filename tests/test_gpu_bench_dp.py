"""bench.py's N > 1 flow executed end to end on the box's one GPU (BASELINE C4).

`bench.py --gpus 2 --comm gloo --device 0` starts two rank processes itself (torch.distributed.run on
127.0.0.1) that share device 0 and exchange gradients through gloo (a host round trip per step), so every
line of the multi-rank code path runs: the in-job 1-GPU reference pass, the weak-scaling headline, the
strong-scaling sub-record, the all-reduce timing, the parameter hashes gathered from both ranks and the
data-parallel Testbed NeRF step (`e2e`, rays sharded with their global ids). The numbers are not scaling
measurements (two ranks on one GPU); the driver's 8-GPU run over RCCL is."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_line():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "gloo", "--device", "0", "--graph", "0",
           "--steps", "3", "--warmup", "1", "--e2e-seconds", "2", "--e2e-weak-seconds", "2", "--e2e-images", "8", "--e2e-res", "128",
           "--c3-seconds", "0", "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["scaling"] == "weak" and res["config"]["global_batch"] == 2 * res["config"]["batch_per_gpu"]
    assert res["value"] > 0 and res["ms_per_step"] > 0
    # the strong-scaling sub-record: one 2^18 batch sharded over the two ranks
    st = res["strong"]
    assert st is not None and st["scaling"] == "strong" and st["global_batch"] == res["config"]["batch_per_gpu"]
    assert st["exchange_ms_per_step"] is not None and st["exchange_ms_per_step"] > 0
    assert res["exchange_ms_per_step"] is not None and res["exchange_ms_per_step"] > 0
    # the sharded optimizer (default): C2's fp16 gradients reduce-scattered as fp16, the fp16 weights all-gathered
    assert res["exchange_bytes"] == {"reduce_scatter_f16": 2 * 3302400, "all_gather_f16": 2 * 3302400}
    # every rank ends with the same parameters (same summed gradient; each slice updated once, then gathered)
    h = res["param_sha1_per_rank"]
    assert len(h) == 2 and h[0] == h[1]
    # N-vs-1 ratios against this job's own 1-GPU pass
    v1 = res["vs_1gpu"]
    assert v1["one_gpu"]["value"] > 0
    assert v1["weak_ratio"] == pytest.approx(res["value"] / v1["one_gpu"]["value"], rel=1e-3, abs=6e-5)  # printed to 4 decimals
    assert v1["strong_ratio"] == pytest.approx(st["value"] / v1["one_gpu"]["value"], rel=1e-3, abs=6e-5)
    # the data-parallel Testbed NeRF step (e2e over the two ranks) and its held-out PSNR on rank 0
    e = res["e2e"]
    assert e["n_gpus"] == 2 and e["steps"] > 0 and e["value"] > 0 and e["psnr"] > 10.0
    # the same with 2^18 samples per rank (weak scaling: global batch 2 x 2^18)
    w = res["e2e_weak"]
    assert w["n_gpus"] == 2 and w["steps"] > 0 and w["value"] > 0 and w["config"]["batch"] == 2 << 18
