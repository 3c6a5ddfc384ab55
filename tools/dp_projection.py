"""DESIGN §7's projection of the data-parallel step at N GPUs from the one-GPU measurements (no 8-GPU node has been
available to measure it). Every input is on the command line, with the round-6 measurements as defaults.

Model (sharded exchange, one part):
  T_N = T_s1 - (rs_1 + ag_1) - upd_1 * (1 - 1/N) + E_N,   E_N = RS_N + AG_N
  RS_N = lat + (N-1)/N * bytes_rs / busbw,  AG_N = lat + (N-1)/N * bytes_ag / busbw
with T_s1 the measured world-1 sharded step (bench dp1_overhead.shard), rs_1/ag_1 its world-1 collective phases,
upd_1 its optimizer phase (all parameters at world 1, 1/N of them at N), bytes_rs = 4 P (fp32 wire) or 2 P (fp16
wire), bytes_ag = 2 P, P the padded parameter count. Weak scaling (each rank its own batch, the bench's headline):
ratio = N T_1 / T_N. Strong scaling (one global batch, the NeRF step's data parallelism): the compute
part divides by N (an upper bound: small per-rank batches run less efficiently), ratio = T_1e / (T_1e / N + E_N +
c_N) with c_N the per-step counter all-reduce.

    python3 tools/dp_projection.py [--n 8] [--busbw 150 250 400] [--lat 10]"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--busbw", type=float, nargs="*", default=[150.0, 250.0, 400.0], help="RCCL bus bandwidth, GB/s")
    ap.add_argument("--lat", type=float, default=10.0, help="latency per collective, us")
    ap.add_argument("--params", type=int, default=3302400, help="padded parameter count P (C2)")
    ap.add_argument("--t1", type=float, default=134.4, help="single-GPU fused C2 step, us (bench headline)")
    ap.add_argument("--ts1", type=float, default=139.4, help="world-1 sharded C2 step, us (dp1_overhead.shard)")
    ap.add_argument("--rs1", type=float, default=4.5, help="world-1 reduce-scatter phase, us")
    ap.add_argument("--ag1", type=float, default=4.5, help="world-1 all-gather phase, us")
    ap.add_argument("--upd1", type=float, default=11.0, help="world-1 slice update (all parameters), us")
    ap.add_argument("--t1e", type=float, default=467.0, help="single-GPU e2e NeRF step, us")
    ap.add_argument("--counters", type=float, default=10.0, help="NeRF counter all-reduce per step, us")
    a = ap.parse_args()
    N, P = a.n, a.params
    out = {"n": N, "lat_us": a.lat, "params": P, "rows": []}
    for bw in a.busbw:
        for wire, brs in (("f32", 4 * P), ("f16", 2 * P)):
            rs = a.lat + (N - 1) / N * brs / (bw * 1e3)  # bytes / (GB/s) -> us: bytes / (bw * 1e3)
            ag = a.lat + (N - 1) / N * 2 * P / (bw * 1e3)
            e = rs + ag
            tn = a.ts1 - (a.rs1 + a.ag1) - a.upd1 * (1 - 1 / N) + e
            weak = N * a.t1 / tn
            strong_e2e = a.t1e / (a.t1e / N + e + a.counters)
            weak_e2e = N * a.t1e / (a.t1e + e + a.counters)
            out["rows"].append({"busbw_GBs": bw, "wire": wire, "exchange_us": round(e, 1), "c2_step_us": round(tn, 1),
                                "c2_weak_ratio": round(weak, 2), "e2e_strong_ratio": round(strong_e2e, 2),
                                "e2e_weak_ratio": round(weak_e2e, 2)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
