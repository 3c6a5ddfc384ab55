"""ctypes binding of include/ngp_engine.h (the engine's C-ABI).

This is the same binding a maintainer would add on the reference side; the
product path fails loudly when lib/libngp_engine.so is missing — there is no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# NGP_ENGINE_LIB selects another build of the same library (A/B experiments); default is in-tree.
LIB_PATH = os.environ.get("NGP_ENGINE_LIB") or os.path.join(HERE, "lib", "libngp_engine.so")
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


class NerfImage(C.Structure):
    """ngp_nerf_image: TrainingImageMetadata + camera-to-world mat4x3 (column-major)."""
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("focal_length", C.c_float * 2),
                ("principal_point", C.c_float * 2), ("xform", C.c_float * 12), ("lens_mode", C.c_uint32),
                ("lens_params", C.c_float * 4)]


class NerfConfig(C.Structure):
    """ngp_nerf_config: Testbed NeRF training knobs (testbed.h:716-785)."""
    _fields_ = [
        ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("cone_angle_constant", C.c_float),
        ("max_cascade", C.c_uint32), ("snap_to_pixel_centers", C.c_uint32), ("random_bg_color", C.c_uint32),
        ("linear_colors", C.c_uint32), ("color_space_linear", C.c_uint32), ("background_color", C.c_float * 3),
        ("rgb_activation", C.c_uint32), ("density_activation", C.c_uint32), ("loss_type", C.c_uint32),
        ("near_distance", C.c_float), ("target_batch_size", C.c_uint32),
    ]


class Rng(C.Structure):
    """ngp_rng: tcnn::pcg32 state, passed by value."""
    _fields_ = [("state", C.c_uint64), ("inc", C.c_uint64)]


class ImageConfig(C.Structure):
    """ngp_image_config: Testbed image training knobs (testbed.h:871-875)."""
    _fields_ = [("random_mode", C.c_uint32), ("snap_to_pixel_centers", C.c_uint32), ("linear_colors", C.c_uint32)]


class NerfStats(C.Structure):
    _fields_ = [("step", C.c_uint32), ("rays_per_batch", C.c_uint32), ("measured_batch_size", C.c_uint32),
                ("measured_batch_size_before_compaction", C.c_uint32), ("loss", C.c_float)]


class NerfErrorMapInfo(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("cdf_width", C.c_uint32), ("cdf_height", C.c_uint32),
                ("n_images", C.c_uint32), ("cdf_valid", C.c_uint32), ("n_steps_since_update", C.c_uint32),
                ("n_steps_between_updates", C.c_uint32), ("size", C.c_uint64)]


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
    "ngp_debug_math_check": (i32, [i32, P, C.POINTER(C.c_uint64)]),
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
    "ngp_model_query": (i32, [P, C.c_char_p, C.POINTER(C.c_double)]),
    "ngp_model_reserve": (i32, [P, u32]),
    "ngp_model_workspace": (i32, [P, C.c_char_p, C.POINTER(P), C.POINTER(u64)]),
    "ngp_model_workspace_epoch": (u64, [P]),
    "ngp_inference": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_density": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_forward": (i32, [P, P, u32, P, u32, P, u32, i32, C.POINTER(P)]),
    "ngp_backward": (i32, [P, P, P, P, u32, P, u32, i32]),
    "ngp_density_forward": (i32, [P, P, u32, P, u32, P, u32, i32, C.POINTER(P)]),
    "ngp_density_backward": (i32, [P, P, P, P, u32, P, u32, i32]),
    "ngp_input_gradient": (i32, [P, P, u32, u32, P, u32, P, u32, f32]),
    "ngp_ctx_destroy": (None, [P]),
    "ngp_forward_backward": (i32, [P, P, u32, P, u32, P, u32, P, u32, i32]),
    "ngp_encoding_forward": (i32, [P, P, u32, P, u32, P, u32, u32, i32]),
    "ngp_encoding_backward": (i32, [P, P, u32, P, u32, P, u32, u32, P, u32, i32]),
    "ngp_trainer_create": (i32, [P, C.c_char_p, u64, C.POINTER(P)]),
    "ngp_trainer_destroy": (None, [P]),
    "ngp_trainer_optimizer_step": (i32, [P, P, f32]),
    "ngp_trainer_gradients": (P, [P]),
    "ngp_trainer_gradients_valid": (i32, [P]),
    "ngp_trainer_params": (P, [P]),
    "ngp_trainer_inference_params": (P, [P]),
    "ngp_trainer_params_full_precision": (P, [P]),
    "ngp_trainer_step": (u32, [P]),
    "ngp_trainer_learning_rate": (f32, [P]),
    "ngp_trainer_set_learning_rate": (i32, [P, f32]),
    "ngp_trainer_set_option": (i32, [P, C.c_char_p, C.c_double]),
    "ngp_trainer_set_params_full_precision": (i32, [P, P, u64]),
    "ngp_trainer_serialize": (i32, [P, P, C.POINTER(u64)]),
    "ngp_trainer_deserialize": (i32, [P, P, u64]),
    "ngp_trainer_capture_training_step": (i32, [P, P, u32, P, u32, P, u32, f32, u32, i32, C.POINTER(P)]),
    "ngp_trainer_train_step": (i32, [P, P, u32, P, u32, P, u32, f32]),
    "ngp_trainer_fused_update_active": (i32, [P, u32]),
    "ngp_graph_launch": (i32, [P, P]),
    "ngp_graph_destroy": (None, [P]),
    "ngp_loss_evaluate": (i32, [i32, P, u32, u32, P, u32, P, u32, f32, P, u32, P, P]),
    "ngp_trainer_training_step": (i32, [P, P, u32, P, u32, P, u32, i32, f32, i32, P]),
    "ngp_image_default_config": (i32, [C.POINTER(ImageConfig)]),
    "ngp_image_create": (i32, [u32, u32, P, C.POINTER(P)]),
    "ngp_image_destroy": (None, [P]),
    "ngp_image_generate_training_samples": (i32, [P, P, u32, C.POINTER(Rng), C.POINTER(ImageConfig), P, P]),
    "ngp_image_train_step": (i32, [P, P, P, u32, C.POINTER(Rng), C.POINTER(ImageConfig), P]),
    "ngp_sdf_mesh_create": (i32, [u32, P, C.POINTER(P)]),
    "ngp_sdf_mesh_destroy": (None, [P]),
    "ngp_sdf_mesh_triangles": (i32, [P, P]),
    "ngp_sdf_bvh_build": (i32, [P, u32, u32, P, C.POINTER(u32)]),
    "ngp_sdf_generate_training_samples": (i32, [P, P, u32, C.POINTER(Rng), P, P, f32, P, P]),
    "ngp_sdf_signed_distance": (i32, [P, P, u32, P, P]),
    "ngp_sdf_shuffle": (i32, [P, u32, u32, P, P, P, P]),
    "ngp_sdf_train_step": (i32, [P, P, u32, P, P, u32, P, P, P]),
    "ngp_nerf_default_config": (i32, [f32, C.POINTER(NerfConfig)]),
    "ngp_nerf_dataset_create": (i32, [u32, C.POINTER(NerfImage), C.POINTER(P), C.POINTER(P)]),
    "ngp_nerf_dataset_destroy": (None, [P]),
    "ngp_nerf_generate_training_samples": (i32, [P, C.POINTER(NerfConfig), P, u32, u32, u32, Rng, u32, P, P, P, P, P,
                                                 P]),
    "ngp_nerf_compute_loss": (i32, [P, C.POINTER(NerfConfig), P, u32, u32, Rng, u32, P, P, P, P, P, P, P, P, P, P, P,
                                    f32]),
    "ngp_nerf_compute_loss_error_map": (i32, [P, C.POINTER(NerfConfig), P, u32, u32, Rng, u32, P, P, P, P, P, P, P, P,
                                              P, P, P, f32, P, u32, u32]),
    "ngp_nerf_compute_loss_state": (i32, [P, C.POINTER(NerfConfig), P, u32, u32, Rng, u32, P, P, P, P, P, P, P, P, P, P, P,
                                          f32, P, C.c_uint64]),
    "ngp_nerf_fill_rollover": (i32, [P, u32, u32, P, P, i32, i32]),
    "ngp_nerf_grid_generate_samples": (i32, [P, C.POINTER(NerfConfig), u32, Rng, u32, P, u32, f32, P, P]),
    "ngp_nerf_grid_splat_max": (i32, [P, u32, P, P, u32, P]),
    "ngp_nerf_grid_splat_max_cells": (i32, [P, u32, P, P, u32, P, u32]),
    "ngp_nerf_grid_ema": (i32, [P, u32, f32, P, P]),
    "ngp_nerf_grid_mean_and_bitfield": (i32, [P, P, u32, P, P]),
    "ngp_nerf_trainer_create": (i32, [P, P, P, C.POINTER(NerfConfig), u64, C.POINTER(P)]),
    "ngp_nerf_trainer_destroy": (None, [P]),
    "ngp_nerf_trainer_get_config": (i32, [P, C.POINTER(NerfConfig)]),
    "ngp_nerf_trainer_set_config": (i32, [P, C.POINTER(NerfConfig)]),
    "ngp_nerf_train_step": (i32, [P, P, i32, C.POINTER(NerfStats)]),
    "ngp_nerf_trainer_buffers": (i32, [P, C.POINTER(P), C.POINTER(P), C.POINTER(P)]),
    "ngp_nerf_trainer_buffers_read": (i32, [P, C.POINTER(P), C.POINTER(P), C.POINTER(P)]),
    "ngp_nerf_trainer_set_pipeline": (i32, [P, i32]),
    "ngp_nerf_trainer_error_map": (i32, [P, i32, P, u64, C.POINTER(NerfErrorMapInfo)]),
    "ngp_nerf_trainer_set_data_parallel": (i32, [P, u32, u32, P, P]),
    "ngp_nerf_save_snapshot": (i32, [P, P, C.c_char_p, C.c_char_p, i32, i32]),
    "ngp_nerf_load_snapshot": (i32, [P, P, C.c_char_p]),
    "ngp_snapshot_network_config": (i32, [C.c_char_p, C.c_char_p, C.POINTER(u64)]),
    "ngp_dp_comm_unique_id": (i32, [P]),
    "ngp_dp_comm_create": (i32, [u32, u32, P, C.POINTER(P)]),
    "ngp_dp_comm_destroy": (None, [P]),
    "ngp_dp_comm_allreduce": (i32, [P, P, u64, i32, i32, P]),
    "ngp_dp_comm_set_wire": (i32, [P, i32]),
    "ngp_dp_comm_reserve": (i32, [P, u64]),
    "ngp_trainer_set_allreduce": (i32, [P, u32, P, P]),
    "ngp_trainer_set_data_parallel": (i32, [P, u32, u32, P, P]),
    "ngp_nerf_renderer_set_depth_scale": (i32, [P, f32]),
    "ngp_nerf_renderer_set_show_accel": (i32, [P, i32]),
    "ngp_trainer_n_params": (u64, [P]),
    "ngp_save_snapshot": (i32, [P, P, C.c_char_p, C.c_char_p, C.c_char_p, P, P, f32, u32, f32, i32, i32]),
    "ngp_load_snapshot": (i32, [P, P, C.c_char_p, P, P, P, P, P]),
    "ngp_snapshot_mode": (i32, [C.c_char_p, C.c_char_p, u64]),
    "ngp_trainer_gather_shards": (i32, [P, P]),
    "ngp_nerf_renderer_create": (i32, [C.POINTER(P)]),
    "ngp_nerf_renderer_destroy": (None, [P]),
    "ngp_nerf_renderer_set_mode": (i32, [P, i32]),
    "ngp_nerf_render": (i32, [P, P, C.POINTER(NerfConfig), P, C.POINTER(NerfImage), P, u32, u32, f32, P, i32, P]),
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
