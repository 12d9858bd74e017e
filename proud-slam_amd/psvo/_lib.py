"""ctypes binding of libpsvo.so (include/psvo.h).

The library is built in-tree (proud-slam_amd/lib/libpsvo.so, see
csrc/Makefile).  There is NO fallback: if the library is missing or fails to
load, every psvo entry point raises — the product path never silently runs
PyTorch or CPU code in place of the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os

import torch

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PSVO_LIB_PATH: a diagnostic build of the same sources (A/B experiments); never set on the product path
LIB_PATH = os.environ.get("PSVO_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libpsvo.so")

_vp, _i32, _i64, _f32, _f64, _u64 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float,
                                      ctypes.c_double, ctypes.c_uint64)

# name -> (restype, argtypes); mirrors include/psvo.h
_SIGNATURES = {
    "psvo_last_error": (ctypes.c_char_p, []),
    "psvo_version": (ctypes.c_char_p, []),
    "psvo_svo_intersect": (_i32, [_vp, _i32, _i32, _i32, _f32, _i32] + [_vp] * 7),
    "psvo_inverse_cdf_sampling": (_i32, [_vp, _i32, _i32, _i32, _i32, _f32] + [_vp] * 9),
    "psvo_ball_intersect": (_i32, [_vp, _i32, _i32, _i32, _f32, _i32] + [_vp] * 6),
    "psvo_aabb_intersect": (_i32, [_vp, _i32, _i32, _i32, _f32, _i32] + [_vp] * 6),
    "psvo_triangle_intersect": (_i32, [_vp, _i32, _i32, _i32, _f32, _f32, _i32] + [_vp] * 6),
    "psvo_uniform_ray_sampling": (_i32, [_vp, _i32, _i32, _i32, _i32, _f32] + [_vp] * 7),
    "psvo_ray_intersect_sorted": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _f32, _f32, _f32] + [_vp] * 6),
    "psvo_hit_rank": (_i32, [_vp, _i64, _vp, _vp, _vp]),
    "psvo_sample_rays": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _u64, _vp, _vp, _vp, _vp,
                                _vp, _vp]),
    "psvo_sample_rays_range": (_i32, [_vp, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _u64, _vp,
                                      _vp, _vp, _vp, _vp, _vp]),
    "psvo_ray_stats": (_i32, [_vp, _i64, _vp, _vp, _f32, _vp]),
    "psvo_scan_counts": (_i32, [_vp, _i64, _vp, _vp]),
    "psvo_sample_points": (_i32, [_vp, _i64, _i32, _i32] + [_vp] * 9),
    "psvo_interp_fwd": (_i32, [_vp, _i64, _i32, _f32] + [_vp] * 9),
    "psvo_interp_bwd": (_i32, [_vp, _i64, _i32, _f32] + [_vp] * 12),
    "psvo_interp_bwd_workspace_floats": (_i64, [_i64, _i32]),
    "psvo_interp_bwd_chunked": (_i32, [_vp, _i64, _i32, _i32, _f32] + [_vp] * 13),
    "psvo_composite_fwd": (_i32, [_vp, _i64, _i32, _f32] + [_vp] * 10),
    "psvo_composite_bwd": (_i32, [_vp, _i64, _i32, _f32] + [_vp] * 12),
    "psvo_composite_loss": (_i32, [_vp, _i64, _i32, _f32, _f32] + [_vp] * 14),
    "psvo_criterion_coef": (_i32, [_vp, _i64, _i32, _f32, _f32, _vp, _vp, _vp, _f32, _f32, _f32, _f32, _i32, _vp,
                                   _vp, _vp]),
    "psvo_criterion_reduce": (_i32, [_vp, _i64, _vp, _vp]),
    "psvo_rows_workspace_ints": (_i64, [_i64]),
    "psvo_sample_pixels_workspace_ints": (_i64, [_i32, _i64]),
    "psvo_pack_tree_workspace_ints": (_i64, [_i64]),
    "psvo_adam_mark_rows": (_i32, [_vp, _i64, _vp, _vp, _vp]),
    "psvo_adam_flags_from_state": (_i32, [_vp, _i64, _vp, _vp, _vp]),
    "psvo_pack_tree": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "psvo_ray_intersect_sorted_packed": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _f32] + [_vp] * 6),
    "psvo_sample_pixels": (_i32, [_vp, _i32, _i64, _i64, _vp, _i32, _vp, _u64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "psvo_rows_compact": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "psvo_rows_scatter_add": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "psvo_rows_compact_flagged": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "psvo_rows_clear": (_i32, [_vp, _i64, _i32, _vp, _vp, _vp]),
    "psvo_rows_mark": (_i32, [_vp, _i64, _vp, _vp]),
    "psvo_rows_flags_from_grad": (_i32, [_vp, _i64, _i32, _vp, _vp]),
    "psvo_mlp_image_floats": (_i64, []),
    "psvo_mlp_image_floats_w": (_i64, [_i32]),
    "psvo_mlp_act_floats": (_i64, [_i64, _i32]),
    "psvo_mlp_mask_words": (_i64, [_i64, _i32]),
    "psvo_mlp_workspace_floats_w": (_i64, [_i64, _i32, _i32]),
    "psvo_map_grad_floats_w": (_i64, [_i64, _i32]),
    "psvo_mlp_fwd": (_i32, [_vp, _i64, _i32] + [_vp] * 16),
    "psvo_mlp_workspace_floats": (_i64, [_i64, _i32]),
    "psvo_mlp_bwd": (_i32, [_vp, _i64, _i32] + [_vp] * 28 + [_i32, _i32, _vp]),
    "psvo_criterion_workspace_floats": (_i64, [_i64]),
    "psvo_criterion_sums": (_i32, [_vp, _i64, _i32, _i32, _f32, _f32] + [_vp] * 9),
    "psvo_criterion_finalize": (_i32, [_vp, _vp, _i64, _i32, _f32, _f32, _f32, _f32, _f32, _i32, _vp]),
    "psvo_criterion_bwd": (_i32, [_vp, _i64, _i32, _f32, _f32] + [_vp] * 12),
    "psvo_adam_step": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _f64, _f64, _f64, _f64, _f64, _i64]),
    "psvo_engine_new": (_vp, []),
    "psvo_engine_free": (None, [_vp]),
    "psvo_engine_set_timing": (_i32, [_vp, _i32]),
    "psvo_engine_set_paths": (_i32, [_vp, _i32]),
    "psvo_engine_select_stats": (_i32, [_vp, _vp, _vp, _i32]),
    "psvo_engine_gate_stream": (_i32, [_vp, _vp]),
    "psvo_debug_set_lookback": (_i32, [_i32, _i32, _i32]),
    "psvo_debug_set_pixel_draw": (_i32, [_i32]),
    "psvo_debug_lb_helps": (_i32, [_vp, _i32]),
    "psvo_engine_queued": (_i32, [_vp]),
    "psvo_map_discard": (_i32, [_vp]),
    "psvo_engine_exchange_words": (_i64, [_i32, _i64, _i64]),
    "psvo_engine_set_exchange": (_i32, [_vp, _i32, _i32, _i64, _i64, _vp, _vp, _vp, _vp]),
    "psvo_engine_timing": (_i32, [_vp, _vp]),
    "psvo_engine_set_clock": (_i32, [_vp, _i32]),
    "psvo_engine_clock": (_i32, [_vp, _vp, _vp]),
    "psvo_host_wait_stats": (_i32, [_vp, _vp, _vp, _i32]),
    "psvo_map_step": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _u64, _i64, _i32, _vp, _vp]),
    "psvo_map_adam": (_i32, [_vp, _vp, _vp, _i64]),
    "psvo_map_adam_ex": (_i32, [_vp, _vp, _vp, _i64, _i32]),
    "psvo_map_join": (_i32, [_vp, _vp]),
    "psvo_map_side_wait": (_i32, [_vp, _vp]),
    "psvo_engine_grad_rays": (_i32, [_vp, _vp, _i64, _vp, _vp]),
    "psvo_map_query": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _u64]),
    "psvo_map_step_frames": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _i64, _i32, _vp, _vp]),
    "psvo_pose_rays_frames": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "psvo_pose_grad_frames": (_i32, [_vp, _i32, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "psvo_track_step": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _f64, _vp, _u64, _i64, _i32, _vp,
                               _vp, _vp]),
    "psvo_pose_rays": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "psvo_mesh_linspace": (_i32, [_i32, _vp]),
    "psvo_mesh_case_table": (_i32, [_vp, _vp]),
    "psvo_mesh_grid_feat": (_i32, [_vp, _i64, _i32, _f32, _vp, _vp, _vp, _vp]),
    "psvo_mesh_point_feat": (_i32, [_vp, _i64, _f32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "psvo_mesh_mc_count": (_i32, [_vp, _i64, _i32] + [_vp] * 6),
    "psvo_mesh_mc_emit": (_i32, [_vp, _i64, _i32, _f32] + [_vp] * 7),
    "psvo_mesh_vox_map_slots": (_i64, [_i64]),
    "psvo_mesh_vertex_rows": (_i32, [_vp, _i64, _vp, _i64, _vp, _f32, _vp, _vp]),
    "psvo_pose_grad": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "psvo_criterion_depth_filter": (_i32, [_vp, _i64, _i32] + [_vp] * 7),
    "psvo_criterion_sums_ex": (_i32, [_vp, _i64, _i32, _i32, _f32, _f32] + [_vp] * 11),
    "psvo_criterion_bwd_ex": (_i32, [_vp, _i64, _i32, _f32, _f32] + [_vp] * 14),
    "psvo_map_grad_floats": (_i64, [_i64]),
    "psvo_dtree_new": (_vp, [_vp, _i32, _i64]),
    "psvo_dtree_free": (None, [_vp]),
    "psvo_dtree_insert": (_i32, [_vp, _vp, _vp, _i64]),
    "psvo_dtree_count": (_i64, [_vp]),
    "psvo_dtree_count_leaves": (_i64, [_vp, _vp]),
    "psvo_dtree_export": (_i32, [_vp, _vp, _f32, _vp, _vp, _vp, _vp, _vp]),
    "psvo_dtree_probe": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "psvo_share_block_bytes": (_i64, []),
    "psvo_share_create": (_vp, [ctypes.c_char_p]),
    "psvo_share_attach": (_vp, [ctypes.c_char_p]),
    "psvo_share_detach": (None, [_vp]),
    "psvo_share_unlink": (_i32, [ctypes.c_char_p]),
    "psvo_share_set_flag": (_i32, [_vp, _i32, _i32]),
    "psvo_share_get_flag": (_i32, [_vp, _i32]),
    "psvo_share_push_pose": (_i32, [_vp, _vp, _i32]),
    "psvo_share_trajectory": (_i64, [_vp, _vp, _i64]),
    "psvo_share_publish": (_i32, [_vp, _vp, _i32, _i32, _vp, _vp, _vp, _i64, _i32, _vp, _vp]),
    "psvo_share_acquire": (_i32, [_vp, _i32, _u64, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "psvo_share_read": (_i32, [_vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "psvo_share_release": (_i32, [_vp, _i32, _i32]),
    "psvo_share_version": (_u64, [_vp, _i32]),
    "psvo_octree_new": (_vp, [_i32, _i32, _f64, _i32]),
    "psvo_octree_free": (None, [_vp]),
    "psvo_octree_insert": (_i32, [_vp, _vp, _i64]),
    "psvo_octree_count": (_i64, [_vp]),
    "psvo_octree_count_leaves": (_i64, [_vp]),
    "psvo_octree_export": (_i32, [_vp, _vp, _vp, _vp]),
    "psvo_build_octree": (_i32, [_vp, _vp, _i64, _i32, _i64, _vp, _vp, _vp, _vp]),
    "psvo_octree_has_voxel": (_i32, [_vp, _i32, _i32, _i32]),
    "psvo_octree_try_insert": (_f64, [_vp, _vp, _i64]),
    "psvo_octree_leaf_voxels": (_i64, [_vp, _vp, _i64]),
}

_lib = None

# Optional per-launch HIP-event timer (bench.py installs one): a callable
# name -> context manager recording events around launches on the current
# stream.  None (the default) costs nothing.
KERNEL_TIMER = None


def timed(name):
    if KERNEL_TIMER is None:
        return _NULL
    return KERNEL_TIMER(name)


class _Null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NULL = _Null()


class PsvoError(RuntimeError):
    pass


def lib():
    """Load libpsvo.so (after torch, so the HIP runtime is torch's)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PsvoError(f"libpsvo.so not built: {LIB_PATH} is missing (run `make -C proud-slam_amd/csrc` or "
                            f"__graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            if os.environ.get("PSVO_LIB_PATH") and not hasattr(L, name):
                continue  # an older diagnostic build (A/B runs) may predate an entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGNATURES)


def call(name, *args):
    """Call a psvo entry point; tensor arguments are passed as their data
    pointers and stay referenced (alive) until the call returns."""
    cargs = [ctypes.c_void_p(a.data_ptr()) if isinstance(a, torch.Tensor) else a for a in args]
    rc = getattr(lib(), name)(*cargs)
    if rc != 0:
        msg = lib().psvo_last_error().decode(errors="replace")
        raise PsvoError(f"{name} failed (code {rc}): {msg}")


def ptr(t):
    """Device/host pointer of a tensor (None → NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device=None):
    """Raw hipStream_t of torch's current stream on `device`."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_device_tensor(t, name, dtype=None):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous tensor")
    if dtype is not None and t.dtype != dtype:
        kind = {torch.float32: "float", torch.int32: "int"}.get(dtype, str(dtype))
        raise RuntimeError(f"{name} must be a {kind} tensor")
