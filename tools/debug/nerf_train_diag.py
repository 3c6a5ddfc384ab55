"""Training diagnostics on the procedural scene: loss, mean density, occupancy, batch stats."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
res = int(sys.argv[2]) if len(sys.argv) > 2 else 200
ds = pkg.synthetic.lego_like_dataset(n_images=50, width=res, height=res, seed=2, device="cuda")
cfg = pkg.nerf.default_config(1.0)
net = pkg.create_nerf_network(pkg.nerf_config("C2"))
tr = pkg.Trainer(net, pkg.nerf_config("C2")["optimizer"])
run = pkg.nerf.NerfTraining(net, tr, ds, cfg, seed=1337)
t0 = time.time()
for i in range(steps):
    s = run.train_step(get_loss=True)
    if i % 100 == 0 or i == steps - 1:
        torch.cuda.synchronize()
        bf = run.bitfield.cpu().numpy()
        occ = np.unpackbits(bf[:128 ** 3 // 8]).mean()
        g = run.density_grid.cpu().numpy()
        print(f"step {s['step']:5d} loss {s['loss']:.5f} rays {s['rays_per_batch']:6d} batch {s['measured_batch_size']:7d}"
              f"/{s['measured_batch_size_before_compaction']:7d} mean {run.mean_density.cpu().item():.4f} occ {occ:.3f}"
              f" grid[min {g.min():.3g} max {g.max():.3g}] t {time.time() - t0:.1f}s", flush=True)
