"""The lazy-EMA optimizer layout (optimizer.h AdamRec: per-pair records, EMA of untouched entries
completed when next updated or when the inference parameters are read) must train bit for bit like the
eager Ema(ExponentialDecay(Adam)) update of tcnn's chain (configs/nerf/base.json:5-22;
configs/sdf/base.json). Large tables (>= 2^23 parameters: BASELINE C5, C2') use it by default; NGP_LAZY_EMA
forces either layout here, on tables small enough to compare quickly, with batches small enough that
most grid entries get no gradient in a step (the lazy path's whole point)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pkg():
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_package()


def make_trainer(pkg, kind, lazy):
    old = os.environ.get("NGP_LAZY_EMA")
    os.environ["NGP_LAZY_EMA"] = "1" if lazy else "0"
    try:
        if kind == "nerf":
            cfg = pkg.nerf_config("C2")
            cfg["encoding"]["log2_hashmap_size"] = 15
            net = pkg.create_nerf_network(cfg)
            opt = cfg["optimizer"]
        else:  # SDF: configs/sdf/base.json with a smaller table
            cfg = dict(pkg.SDF_BASE)
            enc = dict(cfg["encoding"])
            enc.update({"log2_hashmap_size": 15, "per_level_scale": 2.0})
            net = pkg.NetworkWithInputEncoding(3, 1, enc, cfg["network"])
            opt = cfg["optimizer"]
        tr = pkg.Trainer(net, opt, seed=1337)
    finally:
        if old is None:
            del os.environ["NGP_LAZY_EMA"]
        else:
            os.environ["NGP_LAZY_EMA"] = old
    return net, tr


def batch(kind, n, step):
    g = np.random.default_rng(1000 + step)
    if kind == "nerf":
        c = np.zeros((n, 7), np.float32)
        c[:, :3] = g.random((n, 3))
        c[:, 3] = 0.01
        d = g.standard_normal((n, 3))
        c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
        dl = np.zeros((n, 16), np.float16)
        dl[:, :4] = g.uniform(-1, 1, (n, 4))
    else:
        c = g.random((n, 3)).astype(np.float32)
        dl = np.zeros((n, 16), np.float16)
        dl[:, 0] = g.uniform(-1, 1, n)
    return torch.from_numpy(c).cuda(), torch.from_numpy(dl).cuda()


@pytest.mark.parametrize("kind", ["nerf", "sdf"])
def test_lazy_ema_trains_bitwise_like_eager(pkg, kind):
    runs = {}
    for lazy in (False, True):
        net, tr = make_trainer(pkg, kind, lazy)
        snaps = []
        for step in range(24):
            # small batches on most steps: most fine-level entries get no gradient and are skipped
            n = 4096 if step % 5 else 1 << 15
            x, dl = batch(kind, n, step)
            net.forward_backward(x, dl)
            tr.optimizer_step(128.0)
            if step in (6, 23):  # reading the inference parameters mid-run completes the EMA; training continues
                torch.cuda.synchronize()
                snaps.append(tr.inference_params.cpu().numpy().view(np.uint16).copy())
        # one more step, then inference with the EMA parameters through the network (the engine brings
        # them up to date itself before the encoding and MLP read them)
        x, dl = batch(kind, 4096, 24)
        net.forward_backward(x, dl)
        tr.optimizer_step(128.0)
        xq, _ = batch(kind, 3000, 99)
        snaps.append(net.inference(xq, use_inference_params=True).cpu().numpy().view(np.uint16).copy())
        torch.cuda.synchronize()
        runs[lazy] = (tr.params_full_precision.cpu().numpy().view(np.uint32).copy(),
                      tr.params.cpu().numpy().view(np.uint16).copy(), snaps, tr.serialize())
        del net, tr
    (w_e, p_e, s_e, b_e), (w_l, p_l, s_l, b_l) = runs[False], runs[True]
    np.testing.assert_array_equal(w_l, w_e)
    np.testing.assert_array_equal(p_l, p_e)
    for a, b in zip(s_l, s_e):
        np.testing.assert_array_equal(a, b)
    assert b_l == b_e, "serialized optimizer state (w32, m1, m2, ema32, steps) differs"


def test_lazy_ema_deserialize_resumes_bitwise(pkg):
    """A blob written by the eager layout restores into the lazy one (and vice versa) and training
    continues identically."""
    net_e, tr_e = make_trainer(pkg, "sdf", False)
    for step in range(5):
        x, dl = batch("sdf", 4096, step)
        net_e.forward_backward(x, dl)
        tr_e.optimizer_step(128.0)
    blob = tr_e.serialize()
    net_l, tr_l = make_trainer(pkg, "sdf", True)
    tr_l.deserialize(blob)
    tr_e2 = tr_e
    for step in range(5, 12):
        x, dl = batch("sdf", 4096, step)
        for net, tr in ((net_e, tr_e2), (net_l, tr_l)):
            net.forward_backward(x, dl)
            tr.optimizer_step(128.0)
    torch.cuda.synchronize()
    assert tr_l.serialize() == tr_e2.serialize()
    np.testing.assert_array_equal(tr_l.inference_params.cpu().numpy().view(np.uint16),
                                  tr_e2.inference_params.cpu().numpy().view(np.uint16))


def test_lazy_ema_set_params_full_precision_bitwise(pkg):
    """Trainer::set_params_full_precision (testbed.cu:4146) mid-training: the lazy layout must first
    replay the EMA steps its skipped entries still owe on the OLD weights (the eager layout applied them
    every step), then take the new weights; training and a serialize afterwards match the eager layout."""
    runs = {}
    for lazy in (False, True):
        net, tr = make_trainer(pkg, "sdf", lazy)
        for step in range(6):
            x, dl = batch("sdf", 4096, step)
            net.forward_backward(x, dl)
            tr.optimizer_step(128.0)
        torch.cuda.synchronize()
        w = tr.params_full_precision.cpu().numpy().copy()
        w[::3] *= 0.5  # new weights for a third of the parameters
        tr.set_params_full_precision(w)
        blob_now = tr.serialize()
        for step in range(6, 10):
            x, dl = batch("sdf", 4096, step)
            net.forward_backward(x, dl)
            tr.optimizer_step(128.0)
        torch.cuda.synchronize()
        runs[lazy] = (blob_now, tr.serialize(), tr.inference_params.cpu().numpy().view(np.uint16).copy())
        del net, tr
    assert runs[True][0] == runs[False][0], "serialize right after set_params_full_precision differs"
    assert runs[True][1] == runs[False][1], "training after set_params_full_precision differs"
    np.testing.assert_array_equal(runs[True][2], runs[False][2])


def test_fused_optimizer_training_step_bitwise(pkg):
    """Trainer::training_step with the optimizer (train_sdf's call, testbed_sdf.cu:1304) on the lazy
    layout runs the grid's update inside the bucketed backward (model option fuse_opt, default on), and the
    MLP's in the backward's dW slab blocks (fuse_mlp_opt, default on): it must train bit for bit like the separate k_adam_lazy4 launch and like the eager layout, with steps
    whose batches leave most entries untouched and steps whose coarse buckets split into parts."""
    runs = {}
    for name, lazy, fuse, mlp in (("eager", False, 0, 1), ("lazy", True, 0, 1), ("fused", True, 1, 1), ("fused_mlp_launch", True, 1, 0)):
        net, tr = make_trainer(pkg, "sdf", lazy)
        net.set_option("fuse_opt", fuse)
        net.set_option("fuse_mlp_opt", mlp)  # the MLP's update in the slab blocks (1) or its own launch (0)
        snaps = []
        for step in range(20):
            n = 4096 if step % 3 else 1 << 16
            x, _ = batch("sdf", n, step)
            tgt = torch.from_numpy(np.random.default_rng(500 + step).uniform(-0.1, 0.1, (n, 1)).astype(np.float32)).cuda()
            tr.training_step(x, tgt, "MAPE", run_optimizer=True)
            if step == 9:
                torch.cuda.synchronize()
                snaps.append(tr.inference_params.cpu().numpy().view(np.uint16).copy())
        torch.cuda.synchronize()
        snaps.append(tr.inference_params.cpu().numpy().view(np.uint16).copy())
        runs[name] = (tr.params_full_precision.cpu().numpy().view(np.uint32).copy(),
                      tr.params.cpu().numpy().view(np.uint16).copy(), snaps, tr.serialize(), tr.step)
        del net, tr
    for name in ("lazy", "fused", "fused_mlp_launch"):
        w, p, s, b, st = runs[name]
        np.testing.assert_array_equal(w, runs["eager"][0])
        np.testing.assert_array_equal(p, runs["eager"][1])
        for a, e in zip(s, runs["eager"][2]):
            np.testing.assert_array_equal(a, e)
        assert b == runs["eager"][3], f"{name}: serialized optimizer state differs"
        assert st == runs["eager"][4] == 20


@pytest.mark.parametrize("kind", ["nerf", "sdf"])
def test_fused_optimizer_captured_steps_bitwise(pkg, kind):
    """Captured training steps (ngp_trainer_capture_training_step: forward_backward + optimizer_step replayed
    as one HIP graph) on the lazy layout run the grid's update inside the bucketed backward too, with the step
    and hyperparameters read from the trainer's device block: bit for bit the eager layout's graph, across
    launches, a learning-rate change between launches, and a mid-run read of the inference parameters."""
    runs = {}
    for name, lazy, fuse, mlp in (("eager", False, 0, 1), ("lazy", True, 0, 1), ("fused", True, 1, 1), ("fused_mlp_launch", True, 1, 0)):
        net, tr = make_trainer(pkg, kind, lazy)
        net.set_option("fuse_opt", fuse)
        net.set_option("fuse_mlp_opt", mlp)
        s = torch.cuda.Stream()
        snaps = []
        graphs = []
        for n, step in ((1 << 15, 1), (4096, 0)):  # the larger batch first: its workspaces serve both graphs
            x, dl = batch(kind, n, step)
            with torch.cuda.stream(s):
                graphs.append((tr.capture_training_step(x, dl, 128.0, n_steps=2, stream=s), x, dl))
        for it in range(6):
            graphs[it % 3 == 2][0].launch(s)
            if it == 3:
                s.synchronize()
                snaps.append(tr.inference_params.cpu().numpy().view(np.uint16).copy())
                tr.learning_rate = tr.learning_rate * 0.5
        s.synchronize()
        snaps.append(tr.inference_params.cpu().numpy().view(np.uint16).copy())
        runs[name] = (tr.params_full_precision.cpu().numpy().view(np.uint32).copy(),
                      tr.params.cpu().numpy().view(np.uint16).copy(), snaps, tr.serialize(), tr.step)
        del graphs, net, tr
    for name in ("lazy", "fused", "fused_mlp_launch"):
        w, p, sn, b, st = runs[name]
        np.testing.assert_array_equal(w, runs["eager"][0])
        np.testing.assert_array_equal(p, runs["eager"][1])
        for a, e in zip(sn, runs["eager"][2]):
            np.testing.assert_array_equal(a, e)
        assert b == runs["eager"][3], f"{name}: serialized optimizer state differs"
        assert st == runs["eager"][4] == 12


def test_lazy_mirror_is_read_only():
    """ngp_trainer_params_full_precision on the lazy layout hands out a mirror of the records' weights:
    writing into it reaches neither training nor serialize (which read the records), and the next read of
    the accessor shows the records again (the mirror used to be trusted once synced)."""
    from __graft_entry__ import load_package
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    pkg = load_package()
    net, tr = make_trainer(pkg, "sdf", True)
    for step in range(4):
        x, dl = batch("sdf", 4096, step)
        net.forward_backward(x, dl)
        tr.optimizer_step(128.0)
    torch.cuda.synchronize()
    blob = tr.serialize()
    w = tr.params_full_precision
    before = w.cpu().numpy().copy()
    w.mul_(2.0)  # a caller's write into the mirror
    torch.cuda.synchronize()
    assert tr.serialize() == blob
    np.testing.assert_array_equal(tr.params_full_precision.cpu().numpy(), before)


@pytest.mark.parametrize("lazy", [False, True])
def test_eager_train_step_equals_captured_step(pkg, lazy):
    """ngp_trainer_train_step (what bench.py's per-kernel replay runs) is one captured step launched eagerly:
    K eager steps and one K-step graph train bit for bit alike, with the grid's update fused into the
    backward on the lazy layout."""
    runs = []
    for mode in ("eager", "graph"):
        net, tr = make_trainer(pkg, "nerf", lazy)
        x, dl = batch("nerf", 1 << 15, 0)
        assert tr.fused_update_active(x.shape[0]) == lazy
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            if mode == "eager":
                for _ in range(3):
                    tr.train_step(x, dl, 128.0, stream=s)
            else:
                tr.capture_training_step(x, dl, 128.0, n_steps=3, stream=s).launch(s)
        s.synchronize()
        runs.append((tr.serialize(), tr.params.cpu().numpy().view(np.uint16).copy(), tr.step))
        del net, tr
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    assert runs[0][2] == runs[1][2] == 3
