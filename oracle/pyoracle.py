"""ctypes wrapper over oracle/build/libngp_oracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker. The product path (instant-ngp_amd) never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libngp_oracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


class Pcg32(C.Structure):
    _fields_ = [("state", C.c_uint64), ("inc", C.c_uint64)]


class Grid(C.Structure):
    _fields_ = [
        ("n_dims", C.c_uint32), ("n_levels", C.c_uint32), ("n_features", C.c_uint32),
        ("log2_hashmap", C.c_uint32), ("base_resolution", C.c_uint32), ("per_level_scale", C.c_float),
        ("offsets", C.c_uint32 * 33), ("scale", C.c_float * 32), ("resolution", C.c_uint32 * 32),
    ]


class Mlp(C.Structure):
    _fields_ = [("in_pad", C.c_uint32), ("width", C.c_uint32), ("n_hidden", C.c_uint32), ("out_pad", C.c_uint32)]


class Nerf(C.Structure):
    _fields_ = [("grid", Grid), ("density", Mlp), ("rgb", Mlp), ("dir_offset", C.c_uint32), ("in_stride", C.c_uint32)]


class AdamCfg(C.Structure):
    _fields_ = [("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("l2", C.c_float),
                ("ema_decay", C.c_float), ("decay_start", C.c_uint32), ("decay_interval", C.c_uint32),
                ("decay_base", C.c_float)]


P = C.c_void_p


def _declare(L):
    def d(name, res, *args):
        f = getattr(L, name)
        f.restype = res
        f.argtypes = list(args)
    u32, u64, i64, f32, sz = C.c_uint32, C.c_uint64, C.c_int64, C.c_float, C.c_size_t
    d("orc_f32_to_f16", C.c_uint16, f32)
    d("orc_f16_to_f32", f32, C.c_uint16)
    d("orc_f32_to_f16_array", None, P, P, sz)
    d("orc_f16_to_f32_array", None, P, P, sz)
    d("orc_pcg32_seed", None, P, u64, u64)
    d("orc_pcg32_default", None, P)
    d("orc_pcg32_next_uint", u32, P)
    d("orc_pcg32_next_float", f32, P)
    d("orc_pcg32_advance", None, P, i64)
    d("orc_generate_random_uniform", None, P, sz, P, f32, f32)
    d("orc_grid_init", u32, P, u32, u32, u32, u32, u32, f32)
    d("orc_grid_forward", None, P, sz, P, u32, P, f32, P, P)
    d("orc_grid_backward", None, P, sz, P, u32, P, f32, P, P)
    d("orc_grid_indices", None, P, sz, P, u32, P)
    d("orc_grid_backward_exact", None, P, sz, P, u32, P, u32, f32, P, C.c_int, P, P)
    d("orc_sh4", None, f32, f32, f32, P)
    d("orc_grid_input_grad", None, P, sz, P, u32, P, P, u32, f32, P)
    d("orc_sh4_input_grad", None, P, P, P)
    d("orc_nerf_input_grad", None, P, P, sz, P, P, f32, P, P, P)
    d("orc_nerf_density_backward", None, P, P, sz, P, P, P, P)
    d("orc_mlp_n_params", u32, P)
    d("orc_mlp_forward", None, P, P, sz, P, P)
    d("orc_mlp_backward", None, P, P, sz, P, P, P, P)
    d("orc_mlp_init", None, P, P, P)
    d("orc_nerf_n_params", u32, P)
    d("orc_set_num_threads", None, C.c_int)
    d("orc_nerf_forward", None, P, P, sz, P, P)
    d("orc_nerf_density", None, P, P, sz, P, u32, P)
    d("orc_nerf_backward", None, P, P, sz, P, P, P, P)
    d("orc_nerf_train_ex", None, P, P, sz, P, P, P, P, P, P, P, P, P)
    d("orc_net_train_ex", None, P, P, P, sz, P, u32, P, P, P, P, P, P, P, P)
    d("orc_nerf_init", None, P, u64, P)
    d("orc_lr_at_step", f32, P, u32)
    d("orc_adam_step", None, P, u32, sz, sz, f32, P, P, P, P, P, P, P, P)
    d("orc_ema_step", None, f32, u32, sz, P, P, P)
    d("orc_morton3D", u32, u32, u32, u32)
    d("orc_srgb_to_linear", f32, f32)
    d("orc_linear_to_srgb", f32, f32)
    d("orc_num_threads", C.c_int)
    d("orc_math_eval", None, C.c_int, sz, P, P)
    d("orc_loss", C.c_double, C.c_int, u32, u32, P, u32, P, u32, f32, P, u32, P)
    d("orc_image_samples", None, u32, P, C.c_int, C.c_int, C.c_int, u32, u32, P, P, P)
    d("orc_triangle_cdf", None, u32, P, P)
    d("orc_sdf_samples", None, u32, P, u32, P, P, P, P, f32, P, P)
    d("orc_sdf_signed_distance", None, u32, P, u32, P, P)
    d("orc_grid_forward_tcnn", None, P, sz, P, u32, P, P, P)
    d("orc_nerf_tcnn", None, P, P, sz, P, P, P, P, P)
    d("orc_net_tcnn", None, P, P, P, sz, P, u32, P, P, P)
    d("orc_grid_backward_tcnn", None, P, sz, P, u32, P, u32, P, P)
    _declare_nerf(L)


def ptr(a):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "oracle needs contiguous arrays"
    return a.ctypes.data_as(C.c_void_p)


# ---------------------------------------------------------------------------------------------
# Thin pythonic helpers
# ---------------------------------------------------------------------------------------------
def f32_to_f16_bits(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    out = np.empty(a.shape, dtype=np.uint16)
    lib().orc_f32_to_f16_array(ptr(a), ptr(out), a.size)
    return out


def f16_bits_to_f32(a):
    a = np.ascontiguousarray(a, dtype=np.uint16)
    out = np.empty(a.shape, dtype=np.float32)
    lib().orc_f16_to_f32_array(ptr(a), ptr(out), a.size)
    return out


class Rng:
    """tcnn::pcg32 restated (pcg32(initstate, initseq=1))."""

    def __init__(self, seed=None, seq=1):
        self.s = Pcg32()
        if seed is None:
            lib().orc_pcg32_default(C.byref(self.s))
        else:
            lib().orc_pcg32_seed(C.byref(self.s), seed, seq)

    def next_uint(self):
        return lib().orc_pcg32_next_uint(C.byref(self.s))

    def next_float(self):
        return lib().orc_pcg32_next_float(C.byref(self.s))

    def advance(self, delta):
        lib().orc_pcg32_advance(C.byref(self.s), delta)

    def uniform(self, n, lo=0.0, hi=1.0):
        out = np.empty(n, dtype=np.float32)
        lib().orc_generate_random_uniform(C.byref(self.s), n, ptr(out), lo, hi)
        return out


def make_grid(D, L, F, log2T, Nmin=16, b=2.0):
    g = Grid()
    lib().orc_grid_init(C.byref(g), D, L, F, log2T, Nmin, b)
    return g


def grid_n_entries(g):
    return g.offsets[g.n_levels]


def grid_forward(g, pos, table16, max_level=1.0, max_level_per_sample=None, stride=None):
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    n = pos.shape[0]
    stride = stride or pos.shape[1]
    out = np.zeros((n, g.n_levels * g.n_features), dtype=np.float32)
    mls = None if max_level_per_sample is None else np.ascontiguousarray(max_level_per_sample, np.float32)
    lib().orc_grid_forward(C.byref(g), n, ptr(pos), stride, ptr(np.ascontiguousarray(table16)), max_level, ptr(mls), ptr(out))
    return out


def grid_backward(g, pos, dL_dy, max_level=1.0, max_level_per_sample=None, stride=None):
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    n = pos.shape[0]
    stride = stride or pos.shape[1]
    grad = np.zeros(grid_n_entries(g) * g.n_features, dtype=np.float64)
    mls = None if max_level_per_sample is None else np.ascontiguousarray(max_level_per_sample, np.float32)
    lib().orc_grid_backward(C.byref(g), n, ptr(pos), stride, ptr(np.ascontiguousarray(dL_dy, np.float32)), max_level,
                            ptr(mls), ptr(grad))
    return grad


def math_eval(fn, x):
    """ngp_math.h evaluated on the host: fn 0 expf, 1 logf, 2 expf_mid, 3 logf_pos, 4 expf_fast, 5 div_rc by log(1+1/256)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.empty_like(x)
    lib().orc_math_eval(fn, x.size, ptr(x), ptr(y))
    return y


def grid_backward_exact(g, pos, dL_dy16, max_level=1.0, max_level_per_sample=None, stride=None, grad16=None,
                        with_abs_sum=False):
    """Contribution-exact backward (the engine's bucketed contract): fp16 bits of the gradient.
    dL_dy16: uint16 [n x W] (W >= L*F; only the first L*F columns are read). grad16: accumulate into
    these fp16 bits (tcnn GradientMode accumulate) instead of overwriting."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    dy = np.ascontiguousarray(dL_dy16).view(np.uint16)
    n = pos.shape[0]
    np_ = grid_n_entries(g) * g.n_features
    acc = grad16 is not None
    out = np.ascontiguousarray(grad16, dtype=np.uint16).copy() if acc else np.zeros(np_, np.uint16)
    absum = np.zeros(np_, np.float64) if with_abs_sum else None
    mls = None if max_level_per_sample is None else np.ascontiguousarray(max_level_per_sample, np.float32)
    lib().orc_grid_backward_exact(C.byref(g), n, ptr(pos), stride or pos.shape[1], ptr(dy), dy.shape[1], max_level, ptr(mls),
                                  int(acc), ptr(out), ptr(absum))
    return (out, absum) if with_abs_sum else out


def grid_indices(g, pos, stride=None):
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    n = pos.shape[0]
    idx = np.zeros((n, g.n_levels, 1 << g.n_dims), dtype=np.uint32)
    lib().orc_grid_indices(C.byref(g), n, ptr(pos), stride or pos.shape[1], ptr(idx))
    return idx


def sh4(d):
    out = np.zeros(16, dtype=np.float32)
    lib().orc_sh4(float(d[0]), float(d[1]), float(d[2]), ptr(out))
    return out


def grid_input_grad(g, pos, table16, dL_dy, max_level=1.0, stride=None):
    """Analytic dL/dposition through the grid (orc_grid_input_grad), float64 [n x D]. dL_dy float [n x W]
    (W >= L*F, only the first L*F columns read)."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    dy = np.ascontiguousarray(dL_dy, dtype=np.float32)
    out = np.zeros((pos.shape[0], g.n_dims), np.float64)
    lib().orc_grid_input_grad(C.byref(g), pos.shape[0], ptr(pos), stride or pos.shape[1], ptr(np.ascontiguousarray(table16)),
                              ptr(dy), dy.shape[1], max_level, ptr(out))
    return out


def sh4_input_grad(d, dL_dsh):
    out = np.zeros(3, np.float64)
    lib().orc_sh4_input_grad(ptr(np.ascontiguousarray(d, np.float32)), ptr(np.ascontiguousarray(dL_dsh, np.float32)), ptr(out))
    return out


def nerf_input_grad(m, params16, coords, dL_dout, scale=1.0):
    """NerfNetwork backward with dL_dinput (orc_nerf_input_grad): dict of dinput [n x in_stride] (position and
    direction rows), dsh [n x 16] and denc [n x encoding width] (the fp16-rounded intermediates)."""
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    n = coords.shape[0]
    r = {"dinput": np.zeros((n, m.in_stride), np.float32), "dsh": np.zeros((n, 16), np.float32),
         "denc": np.zeros((n, m.density.in_pad), np.float32)}
    lib().orc_nerf_input_grad(C.byref(m), ptr(np.ascontiguousarray(params16)), n, ptr(coords),
                              ptr(np.ascontiguousarray(dL_dout, np.float32)), float(scale), ptr(r["dinput"]), ptr(r["dsh"]),
                              ptr(r["denc"]))
    return r


def nerf_density_backward(m, params16, coords, dL_ddens):
    """NerfNetwork::density_backward (orc_nerf_density_backward): (grads float64 [n_params] with the density MLP
    and grid sections, dinput float32 [n x in_stride] position rows)."""
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    n = coords.shape[0]
    grads = np.zeros(nerf_n_params(m), np.float64)
    dinput = np.zeros((n, m.in_stride), np.float32)
    lib().orc_nerf_density_backward(C.byref(m), ptr(np.ascontiguousarray(params16)), n, ptr(coords),
                                    ptr(np.ascontiguousarray(dL_ddens, np.float32)), ptr(grads), ptr(dinput))
    return grads, dinput


def make_mlp(in_pad, width, n_hidden, out_pad):
    return Mlp(in_pad, width, n_hidden, out_pad)


def mlp_n_params(m):
    return lib().orc_mlp_n_params(C.byref(m))


def mlp_forward(m, w16, x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros((x.shape[0], m.out_pad), dtype=np.float32)
    lib().orc_mlp_forward(C.byref(m), ptr(np.ascontiguousarray(w16)), x.shape[0], ptr(x), ptr(y))
    return y


def mlp_backward(m, w16, x, dy, want_dx=True):
    x = np.ascontiguousarray(x, dtype=np.float32)
    dy = np.ascontiguousarray(dy, dtype=np.float32)
    dW = np.zeros(mlp_n_params(m), dtype=np.float64)
    dx = np.zeros_like(x) if want_dx else None
    lib().orc_mlp_backward(C.byref(m), ptr(np.ascontiguousarray(w16)), x.shape[0], ptr(x), ptr(dy), ptr(dW), ptr(dx))
    return dW, dx


def make_nerf(L=4, F=4, log2T=19, Nmin=16, b=2.0, width=64, density_hidden=1, rgb_hidden=2, dir_offset=4, in_stride=7):
    n = Nerf()
    lib().orc_grid_init(C.byref(n.grid), 3, L, F, log2T, Nmin, b)
    enc_pad = (L * F + 15) // 16 * 16
    n.density = Mlp(enc_pad, width, density_hidden, 16)
    n.rgb = Mlp(32, width, rgb_hidden, 16)
    n.dir_offset = dir_offset
    n.in_stride = in_stride
    return n


def nerf_n_params(m):
    return lib().orc_nerf_n_params(C.byref(m))


def nerf_init(m, seed=1337):
    p = np.zeros(nerf_n_params(m), dtype=np.float32)
    lib().orc_nerf_init(C.byref(m), seed, ptr(p))
    return p


def set_num_threads(n):
    """OpenMP threads of the calling thread's oracle parallel regions (omp_set_num_threads)."""
    lib().orc_set_num_threads(int(n))


def nerf_forward(m, params16, coords, out=None):
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    if out is None:
        out = np.zeros((coords.shape[0], 16), dtype=np.float32)
    lib().orc_nerf_forward(C.byref(m), ptr(np.ascontiguousarray(params16)), coords.shape[0], ptr(coords), ptr(out))
    return out


def nerf_density(m, params16, coords, stride=None):
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    out = np.zeros((coords.shape[0], 16), dtype=np.float32)
    lib().orc_nerf_density(C.byref(m), ptr(np.ascontiguousarray(params16)), coords.shape[0], ptr(coords),
                           stride or coords.shape[1], ptr(out))
    return out


def nerf_backward(m, params16, coords, dL_dout, want_denc=False, grads=None):
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    if grads is None:
        grads = np.zeros(nerf_n_params(m), dtype=np.float64)
    else:
        grads.fill(0.0)
    denc = np.zeros((coords.shape[0], m.density.in_pad), dtype=np.float32) if want_denc else None
    lib().orc_nerf_backward(C.byref(m), ptr(np.ascontiguousarray(params16)), coords.shape[0], ptr(coords),
                            ptr(np.ascontiguousarray(dL_dout, np.float32)), ptr(grads), ptr(denc))
    return (grads, denc) if want_denc else grads


def nerf_train_ex(m, params16, coords, dL_dout):
    """Full-batch forward + backward with conditioning companions (orc_nerf_train_ex): dict of out,
    out_abs [n x 16], grads, grads_abs (MLP section, float64), denc16 (fp16 bits) and denc_abs
    [n x encoding width]."""
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    n = coords.shape[0]
    nm = mlp_n_params(m.density) + mlp_n_params(m.rgb)
    r = {"out": np.zeros((n, 16), np.float32), "out_abs": np.zeros((n, 16), np.float32),
         "grads": np.zeros(nm, np.float64), "grads_abs": np.zeros(nm, np.float64),
         "denc16": np.zeros((n, m.density.in_pad), np.uint16), "denc_abs": np.zeros((n, m.density.in_pad), np.float32),
         "margin": np.zeros(n, np.float32)}
    lib().orc_nerf_train_ex(C.byref(m), ptr(np.ascontiguousarray(params16)), n, ptr(coords),
                            ptr(np.ascontiguousarray(dL_dout, np.float32)), ptr(r["out"]), ptr(r["out_abs"]), ptr(r["grads"]),
                            ptr(r["grads_abs"]), ptr(r["denc16"]), ptr(r["denc_abs"]), ptr(r["margin"]))
    return r


def net_train_ex(grid, mlp, params16, pos, dL_dout, stride=None):
    """orc_net_train_ex: NetworkWithInputEncoding full-batch pass with conditioning companions."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    n = pos.shape[0]
    nm = mlp_n_params(mlp)
    r = {"out": np.zeros((n, mlp.out_pad), np.float32), "out_abs": np.zeros((n, mlp.out_pad), np.float32),
         "grads": np.zeros(nm, np.float64), "grads_abs": np.zeros(nm, np.float64),
         "denc16": np.zeros((n, mlp.in_pad), np.uint16), "denc_abs": np.zeros((n, mlp.in_pad), np.float32),
         "margin": np.zeros(n, np.float32)}
    lib().orc_net_train_ex(C.byref(grid), C.byref(mlp), ptr(np.ascontiguousarray(params16)), n, ptr(pos),
                           stride or pos.shape[1], ptr(np.ascontiguousarray(dL_dout, np.float32)), ptr(r["out"]),
                           ptr(r["out_abs"]), ptr(r["grads"]), ptr(r["grads_abs"]), ptr(r["denc16"]), ptr(r["denc_abs"]),
                           ptr(r["margin"]))
    return r


# ---------------------------------------------------------------------------------------------
# tcnn mode (oracle/ngp_tcnn_mode.c): the reference's fp16 arithmetic (half FMAs in the grid blend, fp16 WMMA
# accumulators in the MLP, fp16 atomics in the grid backward), to bound the engine against it
# ---------------------------------------------------------------------------------------------
def grid_forward_tcnn(g, pos, table16, stride=None):
    """(out float32 [n x L*F] fp16 values, bound float32 [n x L*F]: the fp16 chain's own rounding-error bound)."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    n = pos.shape[0]
    out = np.zeros((n, g.n_levels * g.n_features), np.float32)
    bound = np.zeros_like(out)
    lib().orc_grid_forward_tcnn(C.byref(g), n, ptr(pos), stride or pos.shape[1], ptr(np.ascontiguousarray(table16)), ptr(out),
                                ptr(bound))
    return out, bound


def nerf_tcnn(m, params16, coords, dL_dout=None):
    """NerfNetwork forward (and dL/d(encoding) when dL_dout is given) in tcnn's arithmetic: dict out [n x 16],
    enc [n x encoding width], denc [n x encoding width] or None."""
    coords = np.ascontiguousarray(coords, dtype=np.float32)
    n = coords.shape[0]
    r = {"out": np.zeros((n, 16), np.float32), "enc": np.zeros((n, m.density.in_pad), np.float32),
         "denc": None if dL_dout is None else np.zeros((n, m.density.in_pad), np.float32)}
    dl = None if dL_dout is None else np.ascontiguousarray(dL_dout, np.float32)
    lib().orc_nerf_tcnn(C.byref(m), ptr(np.ascontiguousarray(params16)), n, ptr(coords), ptr(dl), ptr(r["out"]), ptr(r["denc"]),
                        ptr(r["enc"]))
    return r


def net_tcnn(grid, mlp, params16, pos, dL_dout=None, stride=None):
    """NetworkWithInputEncoding forward (and dL/d(encoding)) in tcnn's arithmetic: (out, denc or None)."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    n = pos.shape[0]
    out = np.zeros((n, mlp.out_pad), np.float32)
    denc = None if dL_dout is None else np.zeros((n, mlp.in_pad), np.float32)
    dl = None if dL_dout is None else np.ascontiguousarray(dL_dout, np.float32)
    lib().orc_net_tcnn(C.byref(grid), C.byref(mlp), ptr(np.ascontiguousarray(params16)), n, ptr(pos), stride or pos.shape[1],
                       ptr(dl), ptr(out), ptr(denc))
    return out, denc


def grid_backward_tcnn(g, pos, dL_dy16, stride=None):
    """tcnn's fp16-atomic grid backward in sample order: (grad16 uint16 [entries*F], bound float64: half a spacing
    per add, summed)."""
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    dy = np.ascontiguousarray(dL_dy16).view(np.uint16)
    np_ = grid_n_entries(g) * g.n_features
    out = np.zeros(np_, np.uint16)
    bound = np.zeros(np_, np.float64)
    lib().orc_grid_backward_tcnn(C.byref(g), pos.shape[0], ptr(pos), stride or pos.shape[1], ptr(dy), dy.shape[1], ptr(out),
                                 ptr(bound))
    return out, bound


def adam_step(cfg, step, n_matrix, loss_scale, w32, w16, g16, m1, m2, steps, ema32=None, ema16=None):
    lib().orc_adam_step(C.byref(cfg), step, w32.size, n_matrix, loss_scale, ptr(w32), ptr(w16), ptr(g16), ptr(m1),
                        ptr(m2), ptr(steps), ptr(ema32), ptr(ema16))


def ema_step(decay, step, w32, ema32, ema16):
    """tcnn Ema after optimizer step `step`: ema32 = d ema32 + (1 - d) w32, ema16 = fp16(ema32 / (1 - d^(step+1)))."""
    lib().orc_ema_step(decay, step, w32.size, ptr(np.ascontiguousarray(w32, np.float32)), ptr(ema32), ptr(ema16))


# ---------------------------------------------------------------------------------------------
# NeRF training kernels (oracle/ngp_nerf_oracle.c). cfg / images are ctypes structures with the
# layout of ngp_nerf_config / ngp_nerf_image (include/ngp_engine.h); they are passed by address.
# ---------------------------------------------------------------------------------------------
def _declare_nerf(L):
    def d(name, res, *args):
        f = getattr(L, name)
        f.restype = res
        f.argtypes = list(args)
    u32, f32 = C.c_uint32, C.c_float
    d("orc_morton3D_invert", u32, u32)
    d("orc_camera_matrix", None, P, P)
    d("orc_nerf_generate_samples", None, P, P, P, u32, u32, u32, u32, Pcg32, u32, P, P, P, P, P, P)
    d("orc_nerf_compute_loss", None, P, P, P, u32, u32, u32, Pcg32, u32, u32, P, P, P, P, P, P, P, P, P, f32, f32)
    d("orc_nerf_compute_loss_em", None, P, P, P, u32, u32, u32, Pcg32, u32, u32, P, P, P, P, P, P, P, P, P, f32, f32, P,
      u32, u32)
    d("orc_nerf_grid_samples", None, P, u32, Pcg32, u32, P, u32, f32, P, P)
    d("orc_nerf_grid_splat_ema", None, u32, P, P, u32, u32, f32, P)
    d("orc_nerf_grid_mean", C.c_float, P)
    d("orc_nerf_counters_update", u32, u32, u32, u32, u32, f32, P, P, P)
    d("orc_nerf_max_inference", u32, u32, u32)
    d("orc_nerf_grid_bitfield", None, P, u32, f32, P)
    d("orc_fill_rollover_f32", None, u32, u32, u32, P)
    d("orc_fill_rollover_f16", None, u32, u32, u32, P, C.c_int)
    d("orc_ld_random_val", f32, u32, u32, u32)
    d("orc_nerf_render_march", None, P, P, P, u32, u32, P, P, C.c_int)
    d("orc_nerf_render_composite", None, P, P, u32, u32, P, P, P, f32, P, P)
    d("orc_nerf_render_composite_mode", None, P, P, u32, u32, P, P, P, f32, P, C.c_int, f32, C.c_int, P)


N_CELLS = 128 ** 3


def _images_arg(images):
    arr_t = type(images[0]) * len(images)
    return arr_t(*images)


def _pixels_arg(pixels):
    pix = [np.ascontiguousarray(p, dtype=np.uint8) for p in pixels]
    return pix, (C.c_void_p * len(pix))(*[p.ctypes.data for p in pix])


def pcg(state, inc):
    return Pcg32(state, inc)


def camera_matrix(xform12):
    out = np.zeros(12, np.float32)
    lib().orc_camera_matrix(ptr(np.ascontiguousarray(xform12, np.float32)), ptr(out))
    return out


def nerf_generate_samples(cfg, images, pixels, n_rays, rng, max_samples, bitfield, ray_offset=0, n_div=None):
    ims = _images_arg(images)
    keep, pix = _pixels_arg(pixels)
    out = {
        "ray_indices": np.zeros(n_rays, np.uint32), "rays": np.zeros((n_rays, 6), np.float32),
        "numsteps": np.zeros((n_rays, 2), np.uint32), "coords": np.zeros((max_samples, 7), np.float32),
        "counters": np.zeros(2, np.uint32),
    }
    lib().orc_nerf_generate_samples(C.byref(cfg), ims, pix, len(images), n_rays, ray_offset, n_div or n_rays, rng,
                                    max_samples, ptr(np.ascontiguousarray(bitfield, np.uint8)), ptr(out["ray_indices"]),
                                    ptr(out["rays"]), ptr(out["numsteps"]), ptr(out["coords"]), ptr(out["counters"]))
    del keep
    return out


def nerf_compute_loss(cfg, images, pixels, n_rays, rng, max_compacted, samples, out16, mean_density, loss_scale=128.0,
                      n_div=None, error_map_res=None):
    """samples: dict from nerf_generate_samples (numpy; its numsteps is rewritten in place). error_map_res
    (w, h): also deposit every compacted ray's mean loss into a zeroed error map, res["error_map"]
    [n_images, h, w] (testbed_nerf.cu:1869-1899)."""
    ims = _images_arg(images)
    keep, pix = _pixels_arg(pixels)
    res = {
        "coords_compacted": np.zeros((max_compacted, 7), np.float32),
        "dloss_doutput": np.zeros((max_compacted, 16), np.uint16),
        "loss": np.zeros(n_rays, np.float32), "compacted_counter": np.zeros(1, np.uint32),
    }
    em_w, em_h = error_map_res or (0, 0)
    em = np.zeros((len(images), em_h, em_w), np.float32) if error_map_res else None
    lib().orc_nerf_compute_loss_em(C.byref(cfg), ims, pix, len(images), n_rays, n_div or n_rays, rng, max_compacted,
                                   int(samples["counters"][0]), ptr(np.ascontiguousarray(out16, np.uint16)),
                                   ptr(samples["ray_indices"]), ptr(samples["rays"]), ptr(samples["numsteps"]),
                                   ptr(samples["coords"]), ptr(res["coords_compacted"]), ptr(res["dloss_doutput"]),
                                   ptr(res["loss"]), ptr(res["compacted_counter"]), float(mean_density), float(loss_scale),
                                   ptr(em) if em is not None else None, em_w, em_h)
    if em is not None:
        res["error_map"] = em
    del keep
    return res


ERROR_MAP_MIN_PDF = np.float32(0.01)


def error_map_cdfs(data):
    """construct_cdf_2d + construct_cdf_1d (testbed_nerf.cu:2356-2410) in float32, sequential running sums
    like the kernels' loops (np.cumsum accumulates in order). data [n_images, h, w] -> (cdf_x_cond_y,
    cdf_y, cdf_img)."""
    data = np.asarray(data, np.float32)
    n, h, w = data.shape
    one, mp = np.float32(1.0), ERROR_MAP_MIN_PDF
    cum = np.cumsum(data + np.float32(1e-10), axis=2, dtype=np.float32)
    cdf_y_raw = cum[:, :, -1].copy()
    norm = one / cdf_y_raw
    xs = (mp * np.arange(1, w + 1, dtype=np.float32)) / np.float32(w)
    cdf_x = (one - mp) * cum * norm[:, :, None] + xs
    cy = np.cumsum(cdf_y_raw, axis=1, dtype=np.float32)
    cdf_img = cy[:, -1].copy()
    ys = (mp * np.arange(1, h + 1, dtype=np.float32)) / np.float32(h)
    cdf_y = (one - mp) * cy * (one / cdf_img)[:, None] + ys
    return cdf_x.astype(np.float32), cdf_y.astype(np.float32), cdf_img


def error_map_image_pmf(cdf_img):
    """The host pass over construct_cdf_1d's per-image totals (testbed_nerf.cu:3730-3745): (pmf, cdf)."""
    tot = np.asarray(cdf_img, np.float32)
    n = tot.size
    cum = np.cumsum(tot, dtype=np.float32)
    norm = np.float32(1.0) / cum[-1]
    mp = np.float32(0.1)
    pmf = (np.float32(1.0) - mp) * tot * norm + mp / np.float32(n)
    cdf = (np.float32(1.0) - mp) * cum * norm + (mp * np.arange(1, n + 1, dtype=np.float32)) / np.float32(n)
    return pmf.astype(np.float32), cdf.astype(np.float32)


def nerf_grid_samples(cfg, n, rng, step, grid, n_cascades, thresh):
    pos = np.zeros((n, 3), np.float32)
    idx = np.zeros(n, np.uint32)
    lib().orc_nerf_grid_samples(C.byref(cfg), n, rng, step, ptr(np.ascontiguousarray(grid, np.float32)), n_cascades,
                                thresh, ptr(pos), ptr(idx))
    return pos, idx


def nerf_grid_splat_ema(indices, density16, act, grid, decay=0.95):
    """density16: fp16 bits of the density output (one per sample). Updates grid (float32) in place."""
    lib().orc_nerf_grid_splat_ema(indices.size, ptr(np.ascontiguousarray(indices, np.uint32)),
                                  ptr(np.ascontiguousarray(density16, np.uint16)), act, grid.size, decay, ptr(grid))


def nerf_counters_update(rays_per_batch, target_batch_size, numsteps_counter, compacted_counter, loss_sum=0.0):
    """NerfCounters::update_after_training (testbed_nerf.cu:3583-3609): returns (rays_per_batch,
    measured_batch_size, measured_before_compaction, loss_scalar)."""
    ls = C.c_float(0)
    mb = C.c_uint32(0)
    mbc = C.c_uint32(0)
    r = lib().orc_nerf_counters_update(rays_per_batch, target_batch_size, numsteps_counter, compacted_counter, loss_sum,
                                       C.byref(ls), C.byref(mb), C.byref(mbc))
    return r, mb.value, mbc.value, ls.value


def nerf_max_inference(measured_before_compaction, max_samples):
    return lib().orc_nerf_max_inference(measured_before_compaction, max_samples)


def nerf_grid_mean(grid):
    return lib().orc_nerf_grid_mean(ptr(np.ascontiguousarray(grid, np.float32)))


def nerf_grid_bitfield(grid, max_cascade, mean):
    bf = np.zeros(N_CELLS // 8 * 8, np.uint8)
    lib().orc_nerf_grid_bitfield(ptr(np.ascontiguousarray(grid, np.float32)), max_cascade, mean, ptr(bf))
    return bf


def fill_rollover(data, n_in, rescale=False):
    n, stride = data.shape
    if data.dtype == np.float32:
        lib().orc_fill_rollover_f32(n, stride, n_in, ptr(data))
    else:
        lib().orc_fill_rollover_f16(n, stride, n_in, ptr(data), int(rescale))


# ---- image / SDF / losses (ngp_train_oracle.c) ------------------------------------------------
LOSSES = {"L2": 0, "L1": 1, "MAPE": 2, "SMAPE": 3, "RelativeL2": 4}


def loss(loss_type, out16_bits, target, dims, loss_scale=128.0, dL_stride=16):
    """tcnn loss restated: returns (total, dL/dout fp16 bits [n x dL_stride], per-sample values)."""
    out16_bits = np.ascontiguousarray(out16_bits, dtype=np.uint16)
    target = np.ascontiguousarray(target, dtype=np.float32)
    n = out16_bits.shape[0]
    dl = np.zeros((n, dL_stride), np.uint16)
    vals = np.zeros(n, np.float32)
    t = lib().orc_loss(LOSSES.get(loss_type, loss_type), n, dims, ptr(out16_bits), out16_bits.shape[1], ptr(target),
                       target.shape[1], loss_scale, ptr(dl), dL_stride, ptr(vals))
    return t, dl, vals


def image_samples(n, rng, texture, random_mode=3, snap=True, linear_colors=False):
    """Testbed::train_image's generate_training_data (testbed_image.cu:223-265). rng: Rng (advanced)."""
    texture = np.ascontiguousarray(texture, dtype=np.float32)
    H, W = texture.shape[:2]
    pos = np.zeros((n, 2), np.float32)
    tgt = np.zeros((n, 3), np.float32)
    lib().orc_image_samples(n, C.byref(rng.s), random_mode, int(snap), int(linear_colors), W, H, ptr(texture), ptr(pos),
                            ptr(tgt))
    return pos, tgt


def triangle_cdf(tris):
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    cdf = np.zeros(tris.shape[0], np.float32)
    lib().orc_triangle_cdf(tris.shape[0], ptr(tris), ptr(cdf))
    return cdf


def sdf_samples(n, rng, tris, aabb_min, aabb_max, stddev):
    """generate_training_samples_sdf positions + upper-bound distances (before the signed distance)."""
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    cdf = triangle_cdf(tris)
    pos = np.zeros((n, 3), np.float32)
    dist = np.zeros(n, np.float32)
    lo = np.asarray(aabb_min, np.float32)
    hi = np.asarray(aabb_max, np.float32)
    lib().orc_sdf_samples(n, C.byref(rng.s), tris.shape[0], ptr(tris), ptr(cdf), ptr(lo), ptr(hi), stddev, ptr(pos),
                          ptr(dist))
    return pos, dist


def sdf_signed_distance(pos, tris):
    pos = np.ascontiguousarray(pos, dtype=np.float32).reshape(-1, 3)
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    out = np.zeros(pos.shape[0], np.float32)
    lib().orc_sdf_signed_distance(pos.shape[0], ptr(pos), tris.shape[0], ptr(tris), ptr(out))
    return out


RENDER_MODES = {"AO": 0, "Shade": 1, "Positions": 3, "Depth": 4, "EncodingVis": 9}  # ERenderMode (common.h:110-121)


def nerf_render(cfg, cam, model, params16, bitfield, sample_index=0, min_transmittance=0.01, bg=(0, 0, 0, 0),
                max_per_ray=1024, render_mode="Shade", depth_scale=1.0, show_accel=-1):
    """NerfTracer restated per ray: march, oracle NerfNetwork on every sample, composite (the step colour of
    render_mode: AO, Shade, Positions, Depth or EncodingVis; show_accel >= 0: the march from that mip up, opaque
    steps, Positions by occupancy cell), shade. Returns linear rgba [H, W, 4] and the per-pixel sample counts."""
    W, H = cam.width, cam.height
    coords = np.zeros((W * H, max_per_ray, 7), np.float32)
    counts = np.zeros(W * H, np.int32)
    bfp = ptr(bitfield) if bitfield is not None else None
    lib().orc_nerf_render_march(C.byref(cfg), C.byref(cam), bfp, sample_index, max_per_ray, ptr(coords), ptr(counts),
                                int(show_accel))
    mask = np.arange(max_per_ray)[None, :] < counts[:, None]
    out16 = np.zeros((W * H, max_per_ray, 16), np.uint16)
    if mask.any():
        o = nerf_forward(model, params16, np.ascontiguousarray(coords[mask]))
        out16[mask] = f32_to_f16_bits(o)
    frame = np.zeros((W * H, 4), np.float32)
    bgv = np.asarray(bg, np.float32)
    lib().orc_nerf_render_composite_mode(C.byref(cfg), C.byref(cam), W * H, max_per_ray, ptr(coords), ptr(counts),
                                         ptr(out16), min_transmittance, ptr(bgv), RENDER_MODES[render_mode],
                                         float(depth_scale), int(show_accel), ptr(frame))
    return frame.reshape(H, W, 4), counts


def nerf_render_normals(cfg, cam, model, params16, bitfield, sample_index=0, min_transmittance=0.01, bg=(0, 0, 0, 0),
                        max_per_ray=1024):
    """ERenderMode::Normals restated (testbed_nerf.cu:2615-2617 input_gradient(3, positions) with backprop scale
    128; composite :1183-1188 normal = normalize(-density'(raw) * d raw / d position); shade :2179-2181
    (0.5 n + 0.5) * alpha, composited over bg). The same march as nerf_render. Linear rgba [H, W, 4], counts."""
    W, H = cam.width, cam.height
    coords = np.zeros((W * H, max_per_ray, 7), np.float32)
    counts = np.zeros(W * H, np.int32)
    bfp = ptr(bitfield) if bitfield is not None else None
    lib().orc_nerf_render_march(C.byref(cfg), C.byref(cam), bfp, sample_index, max_per_ray, ptr(coords), ptr(counts), -1)
    mask = np.arange(max_per_ray)[None, :] < counts[:, None]
    raw = np.zeros((W * H, max_per_ray), np.float32)
    grad = np.zeros((W * H, max_per_ray, 3), np.float32)
    if mask.any():
        c = np.ascontiguousarray(coords[mask])
        raw[mask] = f16_bits_to_f32(f32_to_f16_bits(nerf_forward(model, params16, c)[:, 3]))
        dL = np.zeros((c.shape[0], 16), np.float32)
        dL[:, 3] = 128.0
        grad[mask] = nerf_input_grad(model, params16, c, dL, scale=1.0 / 128.0)["dinput"][:, :3]
    act = cfg.density_activation
    dens = {0: lambda v: v, 1: lambda v: np.maximum(v, 0), 2: lambda v: 1 / (1 + np.exp(-v)), 3: np.exp}[act]
    ddens = {0: lambda v: np.ones_like(v), 1: lambda v: (v > 0).astype(np.float32),
             2: lambda v: (1 / (1 + np.exp(-v))) * (1 - 1 / (1 + np.exp(-v))), 3: lambda v: np.exp(np.clip(v, -15, 15))}[act]
    min_step = np.sqrt(3.0) / 1024
    frame = np.tile(np.asarray(bg, np.float64), (W * H, 1))
    for i in range(W * H):
        rgba = np.zeros(4)
        for k in range(counts[i]):
            dt = coords[i, k, 3] * (min_step * (1 << 7) - min_step) + min_step
            w = (1.0 - np.exp(-dens(np.float64(raw[i, k])) * dt)) * (1.0 - rgba[3])
            nrm = -ddens(np.float64(raw[i, k])) * grad[i, k].astype(np.float64)
            rgba[:3] += nrm / np.linalg.norm(nrm) * w
            rgba[3] += w
            if rgba[3] > 1.0 - min_transmittance:
                rgba /= rgba[3]
                break
        if rgba[3] > 0.001:  # the tracer's hit list (compact_kernel_nerf)
            n = rgba[:3] / np.linalg.norm(rgba[:3])
            rgba[:3] = (0.5 * n + 0.5) * rgba[3]
            frame[i] = rgba + frame[i] * (1.0 - rgba[3])
    return frame.reshape(H, W, 4).astype(np.float32), counts
