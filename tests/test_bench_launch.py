"""bench.py's multi-GPU plumbing on CPU: `--gpus N` without a torch.distributed environment starts N
rank processes itself (torch.distributed.run on 127.0.0.1), with one it checks WORLD_SIZE == --gpus; and
the N-rank gradient sum the engine's communicator performs (fp16 addends widened to fp32, rounded once)
does not depend on the ring order, unlike a sum rounded to fp16 at every hop."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bench():
    import importlib
    return importlib.import_module("bench")


def test_check_world_plumbing():
    b = _bench()
    assert b.check_world(1, env={}) == (False, 1)
    assert b.check_world(8, env={}) == (True, 1)  # bench.py must start the ranks itself
    assert b.check_world(4, env={"WORLD_SIZE": "4"}) == (False, 4)
    with pytest.raises(SystemExit):
        b.check_world(8, env={"WORLD_SIZE": "2"})


def test_launch_ranks_command(monkeypatch):
    b = _bench()
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20"])
    assert b.launch_ranks(8) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "20"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launched_ranks_see_world(tmp_path):
    """Real end-to-end launch on CPU: a tiny script using bench.launch_ranks' command shape reports
    the world size each rank sees (gloo, 2 ranks)."""
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "import bench\n"
        "need, world = bench.check_world(int(sys.argv[2]))\n"
        "assert not need and world == dist.get_world_size()\n"
        "print('rank', dist.get_rank(), 'world', world, flush=True)\n"
        "dist.destroy_process_group()\n")
    b = _bench()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", f"--master-port={b.free_port()}", str(script), "--gpus", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("world 2") == 2


def _ring_sum_f16(parts, start):
    """RCCL's fp16 ring: the partial sum is rounded to fp16 after every hop, starting at rank `start`."""
    n = len(parts)
    acc = parts[start].astype(np.float16)
    for k in range(1, n):
        acc = (acc.astype(np.float32) + parts[(start + k) % n].astype(np.float32)).astype(np.float16)
    return acc


def _ring_sum_wide(parts, start):
    """The engine communicator's wire: fp16 addends widened to fp32, summed in ring order, rounded once."""
    n = len(parts)
    acc = parts[start].astype(np.float32)
    for k in range(1, n):
        acc = acc + parts[(start + k) % n].astype(np.float32)
    return acc.astype(np.float16)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_widened_allreduce_is_ring_order_insensitive(world):
    g = np.random.default_rng(world)
    n = 1 << 16
    # gradient-like magnitudes: a few decades of spread, as the grid's fp16 gradients have
    parts = [(g.standard_normal(n) * 10.0 ** g.uniform(-4, -1, n)).astype(np.float16) for _ in range(world)]
    exact = np.sum([p.astype(np.float64) for p in parts], axis=0)
    ref = exact.astype(np.float16)  # the sum rounded once from exact
    wide = [_ring_sum_wide(parts, s) for s in range(world)]
    hop = [_ring_sum_f16(parts, s) for s in range(world)]
    # widened: every ring position gives the once-rounded exact sum except where fp32 itself rounds
    # on a fp16 tie (vanishingly rare); per-hop fp16 rounding differs between positions by whole ulps
    for w in wide:
        assert np.mean(w != ref) < 1e-4
    disagree_hop = np.mean(np.any(np.stack(hop) != hop[0], axis=0))
    if world > 2:  # two addends: one rounding whatever the order
        assert disagree_hop > 0.01
    # per-hop rounding: error bounded by one fp16 half-ulp of the largest partial sum per hop
    scale = np.max(np.abs(np.cumsum([p.astype(np.float64) for p in parts], axis=0)), axis=0) + np.abs(exact)
    for h in hop:
        assert np.all(np.abs(h.astype(np.float64) - exact) <= world * scale * 2.0 ** -11 + 2.0 ** -24 * world)
