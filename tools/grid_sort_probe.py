"""Would the density-grid update's density evaluation run faster on samples grouped by cell? Times the C2 density
network (grid forward + density MLP, ngp_density) on fox-sized update samples (n_cascades * 128^3 / 2: the uniform and
the non-uniform half) in their generated order and sorted by cell index (Morton order within a cascade). One JSON
line: microseconds per call, median of 20, each order."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def main():
    from __graft_entry__ import load_package
    pkg = load_package()
    aabb = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    cfg = pkg.nerf.default_config(aabb)
    n_casc = cfg.max_cascade + 1
    n_el = 128 ** 3 * n_casc
    g = np.random.default_rng(0)
    grid = torch.from_numpy(np.where(g.random(n_el) < 0.1, 0.05, 0.0).astype(np.float32)).cuda()
    r = pkg.nerf.pcg32(7)
    pu, iu = pkg.nerf.grid_generate_samples(cfg, n_el // 4, r, 0, grid, n_casc, -0.01)
    pn, inn = pkg.nerf.grid_generate_samples(cfg, n_el // 4, r, 1, grid, n_casc, 0.01)
    pos = torch.cat([pu, pn]).contiguous()
    idx = torch.cat([iu, inn]).contiguous()
    perm = torch.argsort(idx.view(torch.int32).long(), stable=True)
    pos_s = pos[perm].contiguous()
    # grouped by bins of 2^b cells only, in random order within a bin (what a counting sort by bin gives)
    key = idx.view(torch.int32).long()
    noise = torch.randint(0, 1 << 22, key.shape, device=key.device)
    pos_b = {b: pos[torch.argsort(((key >> b) << 22) + noise)].contiguous() for b in (9, 13, 16)}
    ncfg = pkg.nerf_config("C2")
    net = pkg.create_nerf_network(ncfg)
    tr = pkg.Trainer(net, ncfg["optimizer"], seed=1)  # noqa: F841 (holds the parameters)
    out = torch.empty((16, pos.shape[0]), dtype=torch.float16, device="cuda")
    f = lambda p: net.density(p, output=out, layout=pkg.LAYOUT_SOA, use_inference_params=False)
    f(pos); f(pos_s); [f(v) for v in pos_b.values()]; torch.cuda.synchronize()
    res = {"aabb_scale": aabb, "n": int(pos.shape[0]), "generated_us": timed(lambda: f(pos)),
           "sorted_us": timed(lambda: f(pos_s)),
           **{f"bins_2^{b}_us": timed(lambda: f(pos_b[b])) for b in pos_b}, "generated_us_again": timed(lambda: f(pos))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
