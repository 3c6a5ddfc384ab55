"""Timing-only experiment: hash-grid backward variants and their phases (C2 / C2p, 2^18 samples)."""
import ctypes, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from __graft_entry__ import load_package
pkg = load_package()
L = pkg.lib()
for variant in ["C2", "C2p"]:
    cfg = pkg.nerf_config(variant)
    net = pkg.create_nerf_network(cfg)
    tr = pkg.Trainer(net, cfg["optimizer"])
    n = 1 << 18
    x = torch.rand((n, 7), device="cuda")
    W = net.layout().encoding_width
    dy = ((torch.rand((n, W), device="cuda") - 0.5) * 0.01).half()
    for mode, dbg in [(1, 0), (3, 0), (3, 1), (3, 8), (3, 1 | 4)]:
        net.set_option("grid_backward_mode", mode)
        net.set_option("win_debug", dbg)
        for _ in range(3):
            net.encoding_backward(x, dy)
        torch.cuda.synchronize()
        L.ngp_profiler_reset(); L.ngp_profiler_enable(1)
        for _ in range(10):
            net.encoding_backward(x, dy)
        torch.cuda.synchronize()
        L.ngp_profiler_enable(0)
        need = L.ngp_profiler_read(None, 0); buf = ctypes.create_string_buffer(need); L.ngp_profiler_read(buf, need)
        k = json.loads(buf.value.decode())
        print(variant, "mode", mode, "debug", dbg, {a: round(b["ms"] / b["calls"] * 1000, 1) for a, b in k.items()}, flush=True)
