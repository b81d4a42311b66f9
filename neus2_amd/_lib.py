"""ctypes binding of the C-ABI in include/neus2_hip.h (libneus2_hip.so, built in-tree).

The product path runs only through this library: if it is missing the import fails loudly
(there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# NEUS2_HIP_LIB: development override (bitwise A/B of two builds, scripts/golden_params.py); unset in use
LIB_PATH = os.environ.get("NEUS2_HIP_LIB") or os.path.join(_HERE, "libneus2_hip.so")


class NeusNetworkConfig(C.Structure):
    _fields_ = [
        ("n_levels", C.c_uint32), ("n_features_per_level", C.c_uint32), ("log2_hashmap_size", C.c_uint32),
        ("base_resolution", C.c_uint32), ("per_level_scale", C.c_float), ("top_resolution", C.c_float),
        ("valid_level_scale", C.c_float), ("base_valid_level_scale", C.c_float), ("base_training_step", C.c_uint32),
        ("n_neurons", C.c_uint32), ("n_density_hidden", C.c_uint32), ("n_rgb_hidden", C.c_uint32),
        ("learning_rate", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("epsilon", C.c_float), ("l2_reg", C.c_float),
        ("ema_decay", C.c_float), ("decay_start", C.c_uint32), ("decay_interval", C.c_uint32), ("decay_base", C.c_float),
        ("ek_loss_weight", C.c_float), ("mask_loss_weight", C.c_float), ("anneal_end", C.c_uint32), ("batch_size", C.c_uint32),
        ("sdf_bias", C.c_float), ("density_grid_decay", C.c_float), ("seed", C.c_uint32), ("fixed_rays_per_batch", C.c_uint32),
        ("predict_global_movement", C.c_uint32), ("global_movement_steps", C.c_uint32), ("finetune_global_movement", C.c_uint32),
        ("reset_density_grid_after_global_movement", C.c_uint32), ("after_learning_rate", C.c_float),
        ("gm_learning_rate", C.c_float), ("gm_beta1", C.c_float), ("gm_beta2", C.c_float), ("gm_epsilon", C.c_float),
        ("gm_decay_start", C.c_uint32), ("gm_decay_interval", C.c_uint32), ("gm_decay_base", C.c_float),
    ]


class NeusImage(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("rgba8", C.c_void_p),
        ("focal", C.c_float * 2), ("principal", C.c_float * 2), ("xform", C.c_float * 12),
    ]


class NeusTrainStats(C.Structure):
    _fields_ = [
        ("training_step", C.c_uint32), ("rays_per_batch", C.c_uint32), ("measured_batch_size", C.c_uint32),
        ("measured_batch_size_before_compaction", C.c_uint32), ("n_rays_total", C.c_uint32), ("valid_level", C.c_uint32),
        ("zero_records", C.c_uint32), ("loss", C.c_float), ("ek_loss", C.c_float), ("mask_loss", C.c_float),
        ("last_loss", C.c_float), ("density_grid_mean", C.c_float), ("ray_loss", C.c_float),
        ("n_rays_with_samples", C.c_uint32), ("trained_samples_total", C.c_uint64),
        ("march_first_pass_rays", C.c_uint32), ("kept_ray_extent", C.c_uint32), ("nonfinite_loss", C.c_uint32),
        ("training_aborted", C.c_uint32), ("pre_samples_total", C.c_uint64), ("rays_total", C.c_uint64),
        ("occ_samples_total", C.c_uint64), ("occ_updates", C.c_uint32), ("health_flags", C.c_uint32),
        ("evaluated_samples_total", C.c_uint64), ("progressive_steps", C.c_uint64), ("evaluated_samples_last", C.c_uint32),
        ("progressive_chunk_end", C.c_uint32), ("lookahead_steps", C.c_uint64), ("adam_split_steps", C.c_uint64),
        ("cut_steps", C.c_uint64), ("march_cut_steps", C.c_uint64), ("march_cut_reruns", C.c_uint64),
    ]


class NeusDataParallelInfo(C.Structure):
    _fields_ = [
        ("rank", C.c_uint32), ("world", C.c_uint32), ("has_communicator", C.c_uint32), ("local_group", C.c_uint32),
        ("collective_calls", C.c_uint64), ("allreduce_bytes", C.c_uint64), ("last_step_allreduce_bytes", C.c_uint64),
        ("host_group", C.c_uint32),
    ]


class NeusRestoreState(C.Structure):
    _fields_ = [
        ("training_step", C.c_uint32), ("rays_per_batch", C.c_uint32), ("measured_batch_size", C.c_uint32),
        ("measured_batch_size_before_compaction", C.c_uint32), ("loss", C.c_float), ("rebuild_bitfield", C.c_int32),
    ]


class NeusNetLayout(C.Structure):
    _fields_ = [
        ("n_params", C.c_uint64), ("n_density", C.c_uint64), ("n_rgb", C.c_uint64), ("grid_offset", C.c_uint64),
        ("n_grid_params", C.c_uint64), ("variance_offset", C.c_uint64), ("n_matrix", C.c_uint64),
        ("density_input_width", C.c_uint32), ("rgb_input_width", C.c_uint32),
        ("per_level_scale", C.c_float), ("n_levels", C.c_uint32),
    ]


class NeusRenderRequest(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_uint32), ("training_view", C.c_int32),
        ("xform", C.c_float * 12), ("focal", C.c_float * 2), ("screen_center", C.c_float * 2),
        ("snap_to_pixel_centers", C.c_int32), ("min_transmittance", C.c_float), ("use_ema", C.c_int32),
    ]


class NeusTrainingOptions(C.Structure):
    _fields_ = [
        ("random_bg_color", C.c_int32), ("background_color", C.c_float * 3), ("color_space", C.c_int32),
        ("linear_colors", C.c_int32), ("cone_angle_constant", C.c_float), ("near_distance", C.c_float),
        ("depth_supervision_lambda", C.c_float),
    ]


class NeusOptimizerState(C.Structure):
    _fields_ = [("n_params", C.c_uint32), ("current_step", C.c_uint32), ("learning_rate", C.c_float),
                ("learning_rate_factor", C.c_float)]


class NeusModuleInfo(C.Structure):
    _fields_ = [("n_params", C.c_uint64), ("n_input_dims", C.c_uint32), ("n_output_dims", C.c_uint32),
                ("param_precision", C.c_int32), ("output_precision", C.c_int32), ("gradient_precision", C.c_int32),
                ("batch_capacity", C.c_uint32), ("n_levels", C.c_uint32), ("grid_offset", C.c_uint64),
                ("per_level_scale", C.c_float)]


# Every symbol declared in include/neus2_hip.h (checked by tests/test_capi.py).
EXPORTS = [
    "neus_last_error", "neus_abi_version", "neus_device_count", "neus_device_synchronize",
    "neus_testbed_create", "neus_testbed_destroy", "neus_testbed_set_dataset", "neus_testbed_reload_network",
    "neus_testbed_layout", "neus_testbed_train", "neus_testbed_get_stats", "neus_testbed_get_params",
    "neus_testbed_set_params", "neus_testbed_get_gradients", "neus_testbed_get_ema_params",
    "neus_testbed_get_half_params",
    "neus_testbed_get_density_grid", "neus_testbed_set_density_grid", "neus_testbed_restore_state", "neus_testbed_get_rng", "neus_testbed_render", "neus_testbed_sdf_on_grid",
    "neus_testbed_marching_cubes", "neus_testbed_mc_density", "neus_testbed_get_mesh", "neus_testbed_mesh_vertex_colors", "neus_mc_table", "neus_prepare_image_rgba8", "neus_testbed_ray_counts", "neus_debug_time_kernel", "neus_debug_march_stats", "neus_debug_exclusive_scan", "neus_debug_scan_giveup", "neus_debug_inject_health", "neus_debug_set_lds_fill", "neus_debug_set_lds_fill_all", "neus_debug_set_xcd_shift", "neus_debug_denorm_probe", "neus_debug_get_batch", "neus_debug_get_buffer", "neus_debug_replay_loss_grad", "neus_debug_sample_rays_round0", "neus_debug_march_profile", "neus_debug_scatter_stats", "neus_debug_scatter_parts", "neus_testbed_time_kernel", "neus_testbed_stream",
    "neus_testbed_synchronize", "neus_testbed_set_profiling", "neus_testbed_kernel_times", "neus_testbed_set_infer_timing", "neus_testbed_infer_timing",
    "neus_testbed_set_exchange_timing", "neus_testbed_exchange_timing",
    "neus_nccl_unique_id", "neus_testbed_init_data_parallel", "neus_testbed_init_data_parallel_ex",
    "neus_testbed_data_parallel_info", "neus_testbed_set_exchange_overlap", "neus_local_group_create", "neus_local_group_destroy",
    "neus_testbed_init_local_group", "neus_host_group_create", "neus_host_group_destroy", "neus_testbed_init_host_group", "neus_debug_host_group_allreduce",
    "neus_grid_encode", "neus_net_forward", "neus_net_backward", "neus_sample_rays", "neus_loss_compact",
    "neus_optimizer_step", "neus_fill_rollover", "neus_occ_update", "neus_mfma_probe",
    "neus_testbed_next_frame", "neus_testbed_get_movement", "neus_testbed_set_movement", "neus_testbed_frame_state",
    "neus_testbed_change_frame", "neus_testbed_prepare_for_test", "neus_testbed_get_training_options",
    "neus_testbed_set_training_options", "neus_testbed_saved_transform", "neus_testbed_get_optimizer_state",
    "neus_testbed_set_optimizer_state", "neus_testbed_set_progressive_inference",
    "neus_module_create_network", "neus_module_create_nerf_network", "neus_module_create_encoding", "neus_module_create_network_with_input_encoding", "neus_module_destroy", "neus_context_destroy",
    "neus_module_info", "neus_module_hyperparams", "neus_module_set_training_step", "neus_module_set_indeed_batch_size",
    "neus_module_initialize_params", "neus_module_inference", "neus_module_forward", "neus_module_backward",
    "neus_module_backward_backward_input",
    "neus_net_backward_pos", "neus_delta_apply", "neus_delta_backward",
]

# include/neus2_hip.h's NEUS_ABI_VERSION this binding was written against: a library of another ABI fails to load
ABI_VERSION = 6

_lib = None


def lib():
    """Loads libneus2_hip.so. Raises if it has not been built (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    l = C.CDLL(LIB_PATH)
    l.neus_last_error.restype = C.c_char_p
    for name in EXPORTS:
        f = getattr(l, name)
        if name != "neus_last_error":
            f.restype = C.c_int
    v = C.c_uint32(0)
    if l.neus_abi_version(C.byref(v)) != 0 or v.value != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: C-ABI version {v.value}, this binding needs {ABI_VERSION} (rebuild the library)")
    _lib = l
    return l


class NeusError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        msg = lib().neus_last_error()
        raise NeusError(msg.decode() if msg else "neus error")
    return rc
