"""The C++ drop-in caller (tests/cabi/drop_in.cpp over include/ngp_tcnn_adapter.hpp, g++ only) runs the
Testbed's per-step call sequence through the C-ABI — density (testbed_nerf.cu:3514), inference over the
samples (:4001), forward + backward (:4077-4078), optimizer_step (:3678), Trainer serialize/deserialize
(src/testbed.cu:4874,5040) — and the input-gradient surface: input_gradient for normals written over the
positions (testbed_nerf.cu:2616), backward with dL_dinput (nerf_network.h:262), density_forward /
density_backward (:355-428) — in its own process on the GPU; its outputs are checked against the CPU
oracle with the parity bars of test_gpu_parity.py (outputs 1e-2 of scale, gradients 2e-2 of scale) and
of test_gpu_input_grad.py (input gradients per element)."""
import json
import os
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_drop_in_matches_oracle(tmp_path, orc):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from __graft_entry__ import load_package
    pkg = load_package()
    cfg = pkg.nerf_config("C2")
    cfg["encoding"]["log2_hashmap_size"] = 15
    for k in ("encoding", "dir_encoding", "network", "rgb_network", "optimizer"):
        (tmp_path / f"{k}.json").write_text(json.dumps(cfg[k]))
    n = 3000
    g = np.random.default_rng(77)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3))
    c[:, 3] = 0.01
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dL = np.zeros((n, 16), np.float16)
    dL[:, :4] = g.uniform(-1, 1, (n, 4))
    c.tofile(tmp_path / "coords.bin")
    dL.tofile(tmp_path / "dL.bin")
    exe = os.path.join(ROOT, "tests", "cabi", "drop_in")
    r = subprocess.run([exe, str(tmp_path), str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    meta = json.loads((tmp_path / "meta.json").read_text())
    m = orc.make_nerf(L=4, F=4, log2T=15)
    assert meta["n_params"] == orc.nerf_n_params(m)
    assert meta["padded_output_width"] == 16 and meta["input_width"] == 7
    assert meta["step_after"] == 1 and meta["step_restored"] == 0
    assert "column major" in meta["rm_input_error"]

    p16 = np.fromfile(tmp_path / "params.bin", np.uint16)
    ref = orc.nerf_forward(m, p16, c)
    sc = np.abs(ref).max()
    infer = np.fromfile(tmp_path / "infer.bin", np.float16).reshape(n, 16).astype(np.float32)
    fwd = np.fromfile(tmp_path / "fwd.bin", np.float16).reshape(n, 16).astype(np.float32)
    assert np.abs(infer - ref).max() <= 1e-2 * sc
    assert np.array_equal(fwd, infer)
    den = np.fromfile(tmp_path / "density.bin", np.float16).reshape(16, n).T.astype(np.float32)
    ref_d = orc.nerf_density(m, p16, c)
    assert np.abs(den - ref_d).max() <= 1e-2 * np.abs(ref_d).max()

    grads = np.fromfile(tmp_path / "grads.bin", np.float16).astype(np.float32)
    ref_g = orc.nerf_backward(m, p16, c, dL.astype(np.float32))
    nd, nr = orc.mlp_n_params(m.density), orc.mlp_n_params(m.rgb)
    for name, lo, hi in [("density", 0, nd), ("rgb", nd, nd + nr), ("grid", nd + nr, grads.size)]:
        err = np.abs(grads[lo:hi] - ref_g[lo:hi]).max()
        assert err <= 2e-2 * np.abs(ref_g[lo:hi]).max() + 1e-4, name
    after = np.fromfile(tmp_path / "params_after.bin", np.uint16)
    changed = after != p16
    assert changed[:meta["n_matrix_params"]].mean() > 0.9  # every MLP weight with a gradient moves

    # input gradients and the density-only pass, on the restored (initial) parameters. The initial grid
    # is U(+-1e-4), so dL/dposition is small but not zero; bars per element (as test_gpu_input_grad.py)
    keep = orc.nerf_train_ex(m, p16, c, dL.astype(np.float32))["margin"] > 1e-4
    assert keep.mean() > 0.5
    assert meta["ctx_kind_error"] == "refused"

    def close(a, b, frac=2e-3):
        bad = np.abs(a - b) > 1e-2 * np.abs(b) + 1e-3 * np.abs(b).max(axis=0) + 1e-9
        return bad.mean() < frac
    normals = np.fromfile(tmp_path / "normals.bin", np.float32).reshape(n, 7)
    np.testing.assert_array_equal(normals[:, 3], c[:, 3])  # written over the coordinates: dt row kept
    oh = np.zeros((n, 16), np.float32)
    oh[:, 3] = 128.0
    r_n = orc.nerf_input_grad(m, p16, c, oh, scale=1.0 / 128.0)
    assert close(normals[keep, :3], r_n["dinput"][keep, :3])
    assert np.all(normals[:, 4:] == 0.0)  # the density does not depend on the direction
    din = np.fromfile(tmp_path / "dinput.bin", np.float32).reshape(n, 7)
    r_b = orc.nerf_input_grad(m, p16, c, dL.astype(np.float32))
    assert close(din[keep, :3], r_b["dinput"][keep, :3]) and close(din[keep, 4:], r_b["dinput"][keep, 4:])
    assert np.all(din[:, 3] == 0.0)
    dens = np.fromfile(tmp_path / "dens_out.bin", np.float16).reshape(n, 16).astype(np.float32)
    assert np.abs(dens - ref_d).max() <= 1e-2 * np.abs(ref_d).max()
    g2 = np.fromfile(tmp_path / "grads2.bin", np.float16).astype(np.float32)
    ref_dg, ref_ddin = orc.nerf_density_backward(m, p16, c, dL.astype(np.float32))
    for name, lo, hi, ref in [("density", 0, nd, ref_dg), ("rgb (from backward, untouched)", nd, nd + nr, ref_g),
                              ("grid", nd + nr, g2.size, ref_dg)]:
        err = np.abs(g2[lo:hi] - ref[lo:hi]).max()
        assert err <= 2e-2 * np.abs(ref[lo:hi]).max() + 1e-4, name
    ddin = np.fromfile(tmp_path / "dens_dinput.bin", np.float32).reshape(n, 7)
    assert close(ddin[:, :3], ref_ddin[:, :3]) and np.all(ddin[:, 3:] == 0.0)
