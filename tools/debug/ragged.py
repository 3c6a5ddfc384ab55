import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import numpy as np, torch
import pyoracle as orc
from __graft_entry__ import load_package
pkg = load_package()
cfg = pkg.nerf_config("C2"); cfg["encoding"]["log2_hashmap_size"] = 14
net = pkg.create_nerf_network(cfg); tr = pkg.Trainer(net, cfg["optimizer"])
p = net.initialize_params(1337); nm = net.n_matrix_params
p[nm:] = np.random.default_rng(3).uniform(-0.5, 0.5, p.size - nm).astype(np.float32)
tr.set_params_full_precision(p); torch.cuda.synchronize()
p16 = tr.params.cpu().numpy().view(np.uint16).copy()
m = orc.make_nerf(L=4, F=4, log2T=14)
for n in [32, 33, 777, 800]:
    g = np.random.default_rng(n)
    c = np.zeros((n, 7), np.float32); c[:, :3] = g.random((n, 3)); c[:, 3] = 0.01
    d = g.standard_normal((n, 3)); c[:, 4:] = (d / np.linalg.norm(d, axis=1, keepdims=True) + 1) / 2
    dL = np.zeros((n, 16), np.float16); dL[:, :4] = g.uniform(-1, 1, (n, 4))
    net.forward_backward(torch.from_numpy(c).cuda(), torch.from_numpy(dL).cuda()); torch.cuda.synchronize()
    got = tr.gradients.float().cpu().numpy()
    ref, denc = orc.nerf_backward(m, p16, c, dL.astype(np.float32), want_denc=True)
    e1 = np.abs(got[nm:] - ref[nm:]).max()
    # grid backward alone from the oracle's dL/denc
    net.encoding_backward(torch.from_numpy(c).cuda(), torch.from_numpy(denc.astype(np.float16)).cuda()); torch.cuda.synchronize()
    got2 = tr.gradients.float().cpu().numpy()
    e2 = np.abs(got2[nm:] - ref[nm:]).max()
    # which samples' contributions are wrong: recompute per-sample
    bad = []
    if e1 > 1e-2:
        for i in range(n):
            gi = orc.grid_backward(m.grid, c[i:i+1, :3].copy(), denc[i:i+1, :16].copy(), stride=3)
        diff = got[nm:] - ref[nm:]
        idx = np.argsort(-np.abs(diff))[:5]
        bad = [(int(k), float(diff[k]), float(ref[nm + k])) for k in idx]
    print(f"n={n} fused grid err={e1:.4g} grid-from-oracle-denc err={e2:.4g} scale={np.abs(ref[nm:]).max():.4g} worst={bad}", flush=True)
