"""Where the SDF ground-truth time goes (BASELINE C5 online step, testbed_sdf.cu:1187-1324): times
generate_training_samples on the armadillo batch (engine profiler phases sdf_samples / sdf_distance /
sdf_sign), then mesh.signed_distance (no upper bounds) on the perturbed-surface and the uniform parts of
that batch separately, and reports the inside fraction of each part. One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    from __graft_entry__ import load_package
    import sdf_train
    pkg = load_package()
    lib = pkg.lib()
    sys.path.insert(0, ROOT)
    from bench import read_profiler
    tris, amin, amax, brad = pkg.sdf.load_mesh(sdf_train.load_obj_triangles(os.path.join(ROOT, "data", "sdf", "armadillo.obj")))
    mesh = pkg.sdf.SdfMesh(tris)
    cfg = json.loads(json.dumps(pkg.SDF_BASE))
    net = pkg.NetworkWithInputEncoding(3, 1, cfg["encoding"], cfg["network"])
    tr = pkg.Trainer(net, cfg["optimizer"], seed=1337)
    n = 1 << 18
    st = pkg.sdf.SdfTraining(net, tr, mesh, amin, amax, brad, seed=1337, batch_size=n)
    for _ in range(2):
        st.generate_training_samples(n, st.positions, st.distances)
    torch.cuda.synchronize()
    lib.ngp_profiler_reset()
    lib.ngp_profiler_enable(1)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        st.generate_training_samples(n, st.positions, st.distances)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    lib.ngp_profiler_enable(0)
    ph = {k: round(v["ms"] / max(v["calls"], 1), 4) for k, v in read_profiler(lib).items()}
    base = n // 8
    pos = st.positions
    d = st.distances.cpu().numpy()
    res = {"wall_ms": round(wall * 1e3, 3), "phases_ms": ph, "n": n, "triangles": int(tris.shape[0]),
           "inside_frac_perturbed": float(np.mean(d[4 * base:7 * base] < 0)),
           "inside_frac_uniform": float(np.mean(d[7 * base:] < 0))}
    for name, sl in (("perturbed", slice(4 * base, 7 * base)), ("uniform", slice(7 * base, n))):
        p = pos[sl].contiguous()
        mesh.signed_distance(p)
        torch.cuda.synchronize()
        lib.ngp_profiler_reset()
        lib.ngp_profiler_enable(1)
        for _ in range(reps):
            mesh.signed_distance(p)
        torch.cuda.synchronize()
        lib.ngp_profiler_enable(0)
        res[name] = {k: round(v["ms"] / max(v["calls"], 1), 4) for k, v in read_profiler(lib).items()}
        res[name]["points"] = int(p.shape[0])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
