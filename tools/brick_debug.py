"""Brick-summed grid backward vs the item path on the same inputs (debugging aid): per level, how many grid
gradient entries differ, and where. Cases: NetworkWithInputEncoding (encoding_backward, histogram by
k_sc_hist) and the NeRF network's forward_backward (histogram fused into the forward), with and without
positions outside the unit cube.

    python tools/brick_debug.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def coords(n, seed, outside):
    g = np.random.default_rng(seed)
    c = np.zeros((n, 7), np.float32)
    c[:, :3] = g.random((n, 3), dtype=np.float32)
    c[:64, :3] = np.round(c[:64, :3] * 8) / 8
    c[64:72, :3] = 1.0
    if outside:
        c[72:80, :3] = np.float32(1.0 + 2e-2)
        c[80:88, :3] = np.float32(-1e-2)
    d = g.standard_normal((n, 3))
    c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    return c


def level_report(grid_desc_offsets, F, a, b):
    out = {}
    for l in range(len(grid_desc_offsets) - 1):
        lo, hi = grid_desc_offsets[l] * F, grid_desc_offsets[l + 1] * F
        d = np.nonzero(a[lo:hi] != b[lo:hi])[0]
        out[l] = {"diff": int(d.size), "of": int(hi - lo), "first": [int(x // F) for x in d[:6]]}
    return out


def main():
    from __graft_entry__ import load_package
    pkg = load_package()
    n = 1 << 18
    res = {}
    offs = [0, 4096, 4096 + 32768, 4096 + 32768 + 262144, 4096 + 32768 + 262144 + 524288]
    for outside in (False, True):
        c = coords(n, 5, outside)
        dy = (np.random.default_rng(6).uniform(-1, 1, (n, 16)) * 1e-2).astype(np.float16)
        # (1) encoding_backward through NetworkWithInputEncoding (k_sc_hist)
        grads = []
        for bricks in (1, 0):
            enc = {"otype": "HashGrid", "n_levels": 4, "n_features_per_level": 4, "log2_hashmap_size": 19,
                   "base_resolution": 16, "per_level_scale": 2.0}
            mlp = {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64,
                   "n_hidden_layers": 2}
            net = pkg.NetworkWithInputEncoding(3, 1, enc, mlp)
            net.set_option("grid_bricks", bricks)
            tr = pkg.Trainer(net, {"otype": "Adam", "learning_rate": 1e-2})
            nm = net.n_matrix_params
            x = torch.from_numpy(np.ascontiguousarray(c[:, :3])).cuda()
            net.encoding_backward(x, torch.from_numpy(dy).cuda())
            torch.cuda.synchronize()
            grads.append(tr.gradients[nm:].cpu().numpy().view(np.uint16).copy())
            res[f"enc_outside{int(outside)}_levels"] = net.query("grid_brick_levels") if bricks else None
        res[f"enc_outside{int(outside)}"] = level_report(offs, 4, grads[0], grads[1])
        # (2) NeRF forward_backward (forward-fused histogram), one call, gradient buffer compared
        grads = []
        for bricks in (1, 0):
            cfg = pkg.nerf_config("C2")
            net = pkg.create_nerf_network(cfg)
            net.set_option("grid_bricks", bricks)
            tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
            nm = net.n_matrix_params
            dL = np.zeros((n, 16), np.float16)
            dL[:, :4] = np.random.default_rng(7).uniform(-1e-2, 1e-2, (n, 4))
            net.forward_backward(torch.from_numpy(c).cuda(), torch.from_numpy(dL).cuda())
            torch.cuda.synchronize()
            grads.append(tr.gradients[nm:].cpu().numpy().view(np.uint16).copy())
            res[f"nerf_outside{int(outside)}_levels"] = net.query("grid_brick_levels") if bricks else None
        res[f"nerf_outside{int(outside)}"] = level_report(offs, 4, grads[0], grads[1])
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
