"""World-size-2 data-parallel tests on CPU (gloo): the DP decomposition used by bench.py --gpus N
(shard by global sample index, sum gradients with one all-reduce, divide by N in the optimizer)
reproduces the single-process full-batch update. Gradients come from the CPU oracle here; on the
GPU box the same code path all-reduces the engine's fp16 gradient buffer over RCCL."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n):
    g = np.random.default_rng(0)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dL = np.zeros((n, 16), np.float32)
    dL[:, :4] = g.uniform(-1, 1, (n, 4))
    return c, dL


def _worker(rank, world, port, n, out_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    from __graft_entry__ import load_package
    pkg = load_package()
    import pyoracle as orc
    r, w, _ = pkg.dp.init_from_env(backend="gloo")
    m = orc.make_nerf(L=4, F=4, log2T=12)
    p16 = orc.f32_to_f16_bits(orc.nerf_init(m, 1337))
    c, dL = _batch(n)
    lo, hi = pkg.dp.shard_range(n, r, w)
    g = torch.from_numpy(orc.nerf_backward(m, p16, c[lo:hi], dL[lo:hi]))
    div = pkg.dp.allreduce_gradients(g, w)
    cnt = pkg.dp.allreduce_counters([hi - lo, float(dL[lo:hi].sum())], w)
    if r == 0:
        out_q.put((g.numpy(), div, cnt))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    from __graft_entry__ import load_package
    dp = load_package().dp
    for n in [0, 1, 7, 262144, 1000003]:
        for w in [1, 2, 3, 8]:
            rs = [dp.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_dp_allreduce_matches_full_batch():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as orc
    n, world = 256, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    g_dp, div, cnt = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = orc.make_nerf(L=4, F=4, log2T=12)
    p16 = orc.f32_to_f16_bits(orc.nerf_init(m, 1337))
    c, dL = _batch(n)
    g_full = orc.nerf_backward(m, p16, c, dL)
    np.testing.assert_allclose(g_dp, g_full, rtol=1e-9, atol=1e-12)
    assert div == world
    assert cnt[0] == n and abs(cnt[1] - float(dL.astype(np.float64).sum())) < 1e-4
