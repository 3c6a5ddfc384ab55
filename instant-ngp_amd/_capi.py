"""ctypes binding of include/ngp_engine.h (the engine's C-ABI).

This is the same binding a maintainer would add on the reference side; the
product path fails loudly when lib/libngp_engine.so is missing — there is no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libngp_engine.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "ngp_engine.h")

_lib = None


class NgpError(RuntimeError):
    pass


class ParamLayout(C.Structure):
    _fields_ = [
        ("density_mlp_offset", C.c_uint64), ("density_mlp_params", C.c_uint64),
        ("rgb_mlp_offset", C.c_uint64), ("rgb_mlp_params", C.c_uint64),
        ("grid_offset", C.c_uint64), ("grid_params", C.c_uint64),
        ("grid_dims", C.c_uint32), ("grid_levels", C.c_uint32), ("grid_features", C.c_uint32),
        ("grid_log2_hashmap", C.c_uint32), ("grid_base_resolution", C.c_uint32),
        ("grid_per_level_scale", C.c_float),
        ("grid_level_offsets", C.c_uint32 * 33), ("grid_resolution", C.c_uint32 * 32), ("grid_scale", C.c_float * 32),
        ("encoding_width", C.c_uint32),
    ]


P = C.c_void_p
u32, u64, f32, i32, sz = C.c_uint32, C.c_uint64, C.c_float, C.c_int, C.c_size_t

# name -> (restype, argtypes); must cover every function declared in include/ngp_engine.h
SIGNATURES = {
    "ngp_last_error": (C.c_char_p, []),
    "ngp_version": (C.c_char_p, []),
    "ngp_device_info": (i32, [C.POINTER(C.c_int), C.c_char_p, sz]),
    "ngp_malloc": (i32, [C.POINTER(P), sz]),
    "ngp_free": (i32, [P]),
    "ngp_memcpy": (i32, [P, P, sz, i32]),
    "ngp_stream_synchronize": (i32, [P]),
    "ngp_profiler_enable": (i32, [i32]),
    "ngp_profiler_reset": (i32, []),
    "ngp_profiler_read": (i32, [C.c_char_p, sz]),
    "ngp_nerf_network_create": (i32, [u32, u32, u32, u32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(P)]),
    "ngp_network_with_input_encoding_create": (i32, [u32, u32, C.c_char_p, C.c_char_p, C.POINTER(P)]),
    "ngp_model_destroy": (None, [P]),
    "ngp_model_n_params": (u64, [P]),
    "ngp_model_n_matrix_params": (u64, [P]),
    "ngp_model_input_width": (u32, [P]),
    "ngp_model_padded_output_width": (u32, [P]),
    "ngp_model_output_width": (u32, [P]),
    "ngp_model_param_layout": (i32, [P, C.POINTER(ParamLayout)]),
    "ngp_model_set_params": (i32, [P, P, P, P]),
    "ngp_model_initialize_params": (i32, [P, u64, P, f32]),
    "ngp_model_set_max_level": (i32, [P, f32, P]),
    "ngp_model_set_option": (i32, [P, C.c_char_p, C.c_double]),
    "ngp_model_reserve": (i32, [P, u32]),
    "ngp_inference": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_density": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_forward": (i32, [P, P, u32, P, u32, P, u32, i32, C.POINTER(P)]),
    "ngp_backward": (i32, [P, P, P, P, u32, i32]),
    "ngp_ctx_destroy": (None, [P]),
    "ngp_forward_backward": (i32, [P, P, u32, P, u32, P, u32, P, u32, i32]),
    "ngp_encoding_forward": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_encoding_backward": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_trainer_create": (i32, [P, C.c_char_p, u64, C.POINTER(P)]),
    "ngp_trainer_destroy": (None, [P]),
    "ngp_trainer_optimizer_step": (i32, [P, P, f32]),
    "ngp_trainer_gradients": (P, [P]),
    "ngp_trainer_params": (P, [P]),
    "ngp_trainer_inference_params": (P, [P]),
    "ngp_trainer_params_full_precision": (P, [P]),
    "ngp_trainer_step": (u32, [P]),
    "ngp_trainer_learning_rate": (f32, [P]),
    "ngp_trainer_set_learning_rate": (i32, [P, f32]),
    "ngp_trainer_set_params_full_precision": (i32, [P, P, u64]),
    "ngp_trainer_serialize": (i32, [P, P, C.POINTER(u64)]),
    "ngp_trainer_deserialize": (i32, [P, P, u64]),
}


def lib():
    """Load the engine. Raises if the HIP library was not built — never falls back to CPU."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NgpError(f"HIP engine library missing: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise NgpError(lib().ngp_last_error().decode())
    return rc
