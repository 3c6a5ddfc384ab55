"""The sharded optimizer of the data-parallel step (ngp_trainer_set_data_parallel).

Each rank's fp16-rounded gradients are stored widened to fp32 (by the backward itself, or by a widening pass) and
reduce-scattered; rank r updates the lazy-EMA records of its
1/N slice of the parameters from the fp32 sums rounded to fp16 once, and the fp16 weights are all-gathered. The
all-reduce path (ngp_trainer_set_allreduce: fp32 all-reduce of the widened gradients, narrowed to fp16, every
rank updating every record) rounds the same sums the same way, so the two must train bit for bit alike:

* two ranks sharing the box's GPU over gloo (host round trips), eager steps, C2 (3.3 M parameters, lazy layout):
  fp16 weights after every step, and after ngp_trainer_gather_shards the serialized optimizer state and the EMA
  inference parameters, equal between the paths and between the ranks;
* one rank over the engine's RCCL communicator (world 1), captured steps: the sharded step trains bit for bit
  like the fused single-GPU step.

Both in every form of the exchange: in 1 (the default), 2 or 4 parameter parts, each exchanged on the exchange
stream as soon as the backward has summed it (trainer option dp_parts), and with the fp16 wire (dp_wire16: the
reduce-scatter sums fp16 gradients). gloo's reduce-scatter sums the fp16 values in fp32 and rounds once, and at
world 1 nothing is summed, so the fp16 wire is bit-exact here; RCCL's fp16 ring at world >= 3 rounds per hop
(DESIGN §7 gives that bar).

Reading the EMA parameters, the full-precision weights or serializing before the gather must fail loudly."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
STEPS = 6


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


def _h(t):
    return hashlib.sha1(t.cpu().numpy().tobytes()).hexdigest()


def _batch(rank, step, n=1 << 14):
    g = np.random.default_rng(100 * rank + step)
    x = np.zeros((n, 7), np.float32)
    x[:, :3] = g.random((n, 3))
    x[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    x[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dl = np.zeros((n, 16), np.float16)
    dl[:, :4] = g.uniform(-1, 1, (n, 4))
    if step % 2:  # every other step only the left half of the cube: skipped grid entries (lazy EMA gaps)
        x[:, 0] *= 0.5
    return torch.from_numpy(x).cuda(), torch.from_numpy(dl).cuda()


SHARD_MODES = ("shard", "shard_p2", "shard_p4", "shard_widen", "shard_wire16")


def _shard_options(tr, mode):
    tr.set_option("dp_parts", {"shard_p2": 2, "shard_p4": 4}.get(mode, 1))
    tr.set_option("dp_wire16", int(mode == "shard_wire16"))


def _gloo_rank(rank, world, port, out_dir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world)})
    import torch.distributed as dist
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for mode in SHARD_MODES + ("allreduce",):
        cfg = pkg.nerf_config("C2")
        net = pkg.create_nerf_network(cfg)
        if mode == "shard_widen":  # dW slab reduction in its own launch: the backward cannot store fp32 itself
            net.set_option("fuse_slabs", 0)
        tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        comm = pkg.dp.HostComm(rank, world)
        if mode.startswith("shard"):
            _shard_options(tr, mode)
            tr.set_data_parallel(comm)
        else:
            tr.set_allreduce(comm)
        log = []
        for k in range(STEPS):
            x, dl = _batch(rank, k)
            tr.train_step(x, dl, 128.0)
            torch.cuda.synchronize()
            log.append(_h(tr.params))
        errors = []
        if mode == "shard":  # partial records: these must refuse before the gather
            for what, fn in (("serialize", tr.serialize), ("inference_params", lambda: tr.inference_params.sum()),
                             ("params_full_precision", lambda: tr.params_full_precision.sum())):
                try:
                    fn()
                    errors.append(f"{what}: no error")
                except Exception as e:  # noqa: BLE001 - any engine error is the expected outcome
                    if "gather_shards" not in str(e):
                        errors.append(f"{what}: {e}")
        tr.gather_shards()
        blob = tr.serialize()
        out[mode] = {"params": log, "blob": hashlib.sha1(blob).hexdigest(), "inf": _h(tr.inference_params),
                     "w32": _h(tr.params_full_precision), "errors": errors}
        del tr, net, comm
    dist.barrier()
    dist.destroy_process_group()
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(out, f)


def test_sharded_optimizer_gloo_world2_equals_allreduce(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    mp.spawn(_gloo_rank, args=(2, 29100 + os.getpid() % 1000, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (json.load(open(tmp_path / f"r{r}.json")) for r in (0, 1))
    for r in (r0, r1):
        assert r["shard"]["errors"] == []
        for mode in SHARD_MODES:
            assert r[mode]["params"] == r["allreduce"]["params"], mode  # fp16 weights after every step
            for key in ("blob", "inf", "w32"):
                assert r[mode][key] == r["allreduce"][key], (mode, key)
    assert r0["shard"] == {**r1["shard"]}  # both ranks hold the same model


def _rccl_world1(_rank, out_dir):
    from __graft_entry__ import load_package
    pkg = load_package()
    torch.cuda.set_device(0)
    n = 1 << 15
    x, dl = _batch(0, 0, n)
    x1, dl1 = _batch(0, 1, n)
    res = {}
    for mode in ("plain", "shard", "shard_p2", "shard_p4", "shard_wire16"):
        cfg = pkg.nerf_config("C2")
        net = pkg.create_nerf_network(cfg)
        tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
        net.reserve(n)
        comm = None
        if mode != "plain":
            comm = pkg.dp.EngineComm(0, 1)  # a world of one: no process group
            _shard_options(tr, mode)
            tr.set_data_parallel(comm)
        assert tr.fused_update_active(n) == (mode == "plain")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            g0 = tr.capture_training_step(x, dl, 128.0, n_steps=3, stream=s)
            g1 = tr.capture_training_step(x1, dl1, 128.0, n_steps=2, stream=s)
            for _ in range(2):
                g0.launch(s)
                g1.launch(s)
            tr.train_step(x, dl, 128.0, stream=s)  # the eager form of the same step
        s.synchronize()
        tr.gather_shards()  # a no-op at world 1
        res[mode] = [_h(tr.params), hashlib.sha1(tr.serialize()).hexdigest(), _h(tr.inference_params), tr.step]
        del g0, g1, tr, net, comm
    with open(os.path.join(out_dir, "w1.json"), "w") as f:
        json.dump(res, f)


def test_sharded_optimizer_rccl_world1_equals_fused_step(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    mp.spawn(_rccl_world1, args=(str(tmp_path),), nprocs=1, join=True)
    r = json.load(open(tmp_path / "w1.json"))
    for mode in ("shard", "shard_p2", "shard_p4", "shard_wire16"):
        assert r["plain"] == r[mode], mode
    assert r["shard"][3] == 11


class _NoopComm:
    """A world-2 exchange that moves nothing (rank 0 of 2): capturable, so it drives the captured sharded step's
    host bookkeeping on one GPU. Numerically meaningless; only the staleness rules are checked with it."""

    def __init__(self, pkg):
        self.rank, self.world, self.handle = 0, 2, None
        self.fn = pkg.dp.ALLREDUCE_FN(lambda user, buf, count, dtype, op, stream: 0)


def test_captured_sharded_step_invalidates_state_at_every_launch(pkg):
    """A captured sharded step over world > 1 leaves the other ranks' records stale at EVERY launch, not only
    while it is recorded: after gather_shards, a further launch must make serialize / the EMA parameters fail
    again. Its backward stores the gradient as fp32 only, so gradients_valid is False after it and
    True again after a plain forward_backward."""
    n = 1 << 14
    x, dl = _batch(0, 0, n)
    cfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
    net.reserve(n)
    comm = _NoopComm(pkg)
    tr.set_data_parallel(comm)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        g = tr.capture_training_step(x, dl, 128.0, n_steps=1, stream=s)
    for _ in range(2):
        with torch.cuda.stream(s):
            g.launch(s)
        s.synchronize()
        with pytest.raises(pkg.NgpError, match="gather_shards"):
            tr.serialize()
        assert not tr.gradients_valid
        tr.gather_shards()  # the no-op all-gather "restores" the records: the reads are allowed again
        tr.serialize()
    net.forward_backward(x, dl)
    torch.cuda.synchronize()
    assert tr.gradients_valid
    del g
    tr.set_data_parallel(None)
