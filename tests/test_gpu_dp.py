"""Data-parallel NeRF training with two ranks sharing the box's GPU over gloo.

Checks the exchange steps by their invariants: after every step the ranks hold bitwise-identical
parameters and density grids (gradients, density-grid maxima and counters are all-reduced, the
optimizer is replicated), both ranks see the same global counters and loss, and the sharded run
trains like the single-process run on the same scene (its loss falls to within 1.5x of it)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 80


def _run(rank, world, port, out_dir, shard=True):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world)})
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ds = pkg.synthetic.lego_like_dataset(n_images=10, width=96, height=96, seed=3)
    cfg = pkg.nerf.default_config(1.0)
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"])
    run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
    tag = f"w{world}" + ("" if shard else "_ar")
    if world > 1:
        tr.set_option("shard_opt", int(shard))  # sharded optimizer (default) or one all-reduce per step
        run.set_data_parallel(rank, world)
    log = []
    for k in range(STEPS):
        s = run.train_step(get_loss=True)
        torch.cuda.synchronize()
        if k == 0:  # the step's gradient (all-reduced across the ranks on the all-reduce path)
            np.save(os.path.join(out_dir, f"grad0_{tag}_r{rank}.npy"), tr.gradients.float().cpu().numpy())
        log.append({"loss": s["loss"], "rays": s["rays_per_batch"], "measured": s["measured_batch_size"],
                    "params": hashlib.sha1(tr.params.cpu().numpy().tobytes()).hexdigest(),
                    "grid": hashlib.sha1(run.density_grid.cpu().numpy().tobytes()).hexdigest()})
    with open(os.path.join(out_dir, f"{tag}_r{rank}.json"), "w") as f:
        json.dump(log, f)
    if world > 1:
        dist.destroy_process_group()


def test_nerf_data_parallel_two_ranks(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    port = 29500 + os.getpid() % 1000
    mp.spawn(_run, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    mp.spawn(_run, args=(2, port + 2, str(tmp_path), False), nprocs=2, join=True)
    mp.spawn(_run, args=(1, port + 1, str(tmp_path)), nprocs=1, join=True)
    r0 = json.load(open(tmp_path / "w2_r0.json"))
    r1 = json.load(open(tmp_path / "w2_r1.json"))
    ar0 = json.load(open(tmp_path / "w2_ar_r0.json"))
    single = json.load(open(tmp_path / "w1_r0.json"))
    # all-reduce path: every rank holds the same summed gradient (the batches differ from the 1-GPU step's
    # wherever compaction truncates or rolls over per shard, so the sum is compared on a fixed batch below)
    assert np.array_equal(np.load(tmp_path / "grad0_w2_ar_r0.npy"), np.load(tmp_path / "grad0_w2_ar_r1.npy"))
    # the sharded optimizer trains bit for bit like the all-reduce path: same parameters, grid and counters
    assert r0 == ar0
    for a, b in zip(r0, r1):
        assert a["params"] == b["params"] and a["grid"] == b["grid"]
        assert a["rays"] == b["rays"] and a["measured"] == b["measured"]
        assert a["loss"] == pytest.approx(b["loss"], rel=1e-6)
    l_dp = np.mean([e["loss"] for e in r0[-10:]])
    l_1 = np.mean([e["loss"] for e in single[-10:]])
    l_0 = np.mean([e["loss"] for e in r0[:5]])
    assert l_dp < 0.7 * l_0
    assert l_dp < 1.5 * l_1, (l_dp, l_1)


def _engine_comm_run(_rank, port, out_dir):
    """One rank over the nccl backend (RCCL): the engine's communicator all-reduces the gradient buffer
    inside a captured 3-step training graph; a world of one must leave training bitwise unchanged."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": "0", "WORLD_SIZE": "1"})
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cfg = pkg.nerf_config("C2")
    cfg["encoding"]["log2_hashmap_size"] = 15
    g = np.random.default_rng(5)
    n = 4096
    x = np.zeros((n, 7), np.float32)
    x[:, :3] = g.random((n, 3))
    x[:, 4:] = g.random((n, 3))
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1e-2, 1e-2, (n, 4))
    x, dL = torch.from_numpy(x).cuda(), torch.from_numpy(dL).cuda()
    comm = pkg.dp.EngineComm(0, 1)
    s = torch.cuda.Stream()
    hashes = []
    for use_comm in (False, True):
        net = pkg.create_nerf_network(cfg)
        tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        net.reserve(n)
        if use_comm:
            tr.set_allreduce(comm)
        with torch.cuda.stream(s):
            graph = tr.capture_training_step(x, dL, 128.0, n_steps=3)
            graph.launch()
            graph.launch()
            # eager exchange on the same stream through the same communicator
            net.forward_backward(x, dL)
            if use_comm:
                comm.allreduce(tr.gradients)
            tr.optimizer_step(128.0)
        torch.cuda.synchronize()
        hashes.append(hashlib.sha1(tr.params.cpu().numpy().tobytes()).hexdigest())
    # a tensor view that is only 2-byte aligned: the widened path takes scalar loads there; at
    # world 1 the widened sum is the identity, bit for bit
    buf = torch.randn(4099, device="cuda").half()
    view = buf[1:]
    before = view.clone()
    comm.allreduce(view)
    torch.cuda.synchronize()
    hashes.append(bool(torch.equal(view.view(torch.int16), before.view(torch.int16))))
    del comm
    dist.destroy_process_group()
    with open(os.path.join(out_dir, "comm.json"), "w") as f:
        json.dump(hashes, f)


def test_engine_rccl_allreduce_in_captured_step(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    mp.spawn(_engine_comm_run, args=(29400 + os.getpid() % 1000, str(tmp_path)), nprocs=1, join=True)
    a, b, unaligned_ok = json.load(open(tmp_path / "comm.json"))
    assert a == b
    assert unaligned_ok


def _nerf_rccl_world1(_rank, port, out_dir):
    """The data-parallel NeRF step with the engine's RCCL communicator at world 1: counters and loss
    all-reduced on the stream and published (no copies), the training pass one captured graph with the
    gradient all-reduce inside, the next step's sampler pipelined under it. World 1 must train bitwise
    like the plain step (N > 1 over xGMI is the driver's scaling run)."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": "0", "WORLD_SIZE": "1"})
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    logs = []
    for dp_mode in (False, True):
        ds = pkg.synthetic.lego_like_dataset(n_images=10, width=96, height=96, seed=3)
        cfg = pkg.nerf.default_config(1.0)
        ncfg = pkg.nerf_config("C2")
        net = pkg.create_nerf_network(ncfg)
        tr = pkg.Trainer(net, ncfg["optimizer"])
        run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
        if dp_mode:
            run.set_data_parallel(0, 1, exchange_at_world_1=True)
        log = []
        for k in range(70):
            s = run.train_step(get_loss=(k % 5 == 0))
            log.append([s["rays_per_batch"], s["measured_batch_size"], s["measured_batch_size_before_compaction"],
                        round(float(s["loss"]), 5)])
        torch.cuda.synchronize()
        log.append([hashlib.sha1(tr.params.cpu().numpy().tobytes()).hexdigest(),
                    hashlib.sha1(run.density_grid.cpu().numpy().tobytes()).hexdigest()])
        logs.append(log)
        del run
    dist.destroy_process_group()
    with open(os.path.join(out_dir, "nerf_world1.json"), "w") as f:
        json.dump(logs, f)


def test_nerf_data_parallel_rccl_world1_is_exact(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    mp.spawn(_nerf_rccl_world1, args=(29700 + os.getpid() % 1000, str(tmp_path)), nprocs=1, join=True)
    plain, dp = json.load(open(tmp_path / "nerf_world1.json"))
    assert plain[-1] == dp[-1]  # parameters and density grid, bitwise
    for a, b in zip(plain[:-1], dp[:-1]):
        assert a[:3] == b[:3]  # counters
        assert b[3] == pytest.approx(a[3], rel=1e-4, abs=1e-7)  # loss (device float sum vs host double sum)


def test_sharded_gradient_sum_equals_full_batch():
    """SURVEY §8e collective 1: the shards' gradients (each rank's half of one fixed 2^15-sample batch,
    dL/doutput scaled by 1/2 as the NeRF step scales by 128 / R_global) sum to the gradient of the whole
    batch within the fp16 rounding of each partial and of the total (grid: exact sums rounded once per
    shard; MLP: fp32 slab sums rounded once) — the all-reduce then adds exactly those partials."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from __graft_entry__ import load_package
    pkg = load_package()
    cfg = pkg.nerf_config("C2")
    cfg["encoding"]["log2_hashmap_size"] = 16
    n = 1 << 15
    g = np.random.default_rng(9)
    x = np.zeros((n, 7), np.float32)
    x[:, :3] = g.random((n, 3))
    x[:, 4:] = g.random((n, 3))
    dL = np.zeros((n, 16), np.float32)
    dL[:, :4] = g.uniform(-1, 1, (n, 4))
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)

    def grad(lo, hi, scale):
        net.forward_backward(torch.from_numpy(x[lo:hi]).cuda(), torch.from_numpy((dL[lo:hi] * scale).astype(np.float16)).cuda())
        torch.cuda.synchronize()
        return tr.gradients.float().cpu().numpy().copy()

    full = grad(0, n, 0.5)  # the same 1/2 scale, so the halves' rounding of dL/doutput is the full batch's
    p0, p1 = grad(0, n // 2, 0.5), grad(n // 2, n, 0.5)
    tol = 2.0 ** -11 * (np.abs(p0) + np.abs(p1) + np.abs(full)) * 1.01 + 2.0 ** -24
    bad = np.abs((p0 + p1) - full) > tol
    assert not bad.any(), (int(bad.sum()), float(np.abs(p0 + p1 - full).max()))
