"""ctypes binding of libmd2hip.so (include/md2.h).

The product path has NO fallback: if the HIP library is missing or fails to load, every call
raises.  Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``)."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MD2HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libmd2hip.so"))

MAX_SCALES = 5
ABI_VERSION = 2          # include/md2.h MD2_ABI_VERSION: the struct layouts below


class LossCfg(C.Structure):
    """``md2_loss_cfg``."""
    _fields_ = [
        ("n", C.c_int), ("c", C.c_int), ("width", C.c_int), ("height", C.c_int),
        ("nscales", C.c_int),
        ("scale_w", C.c_int * MAX_SCALES), ("scale_h", C.c_int * MAX_SCALES),
        ("smooth_weight", C.c_float * MAX_SCALES),
        ("divisor", C.c_float), ("smooth_normalize", C.c_int),
        ("K", C.c_float * 9), ("invK", C.c_float * 9),
        ("min_depth", C.c_float), ("max_depth", C.c_float),
        ("x_sample_stride", C.c_longlong), ("x_frame_stride", C.c_longlong),
        ("target", C.c_int), ("src0", C.c_int), ("src1", C.c_int),
        ("invert_mask", C.c_int), ("sigmoid_grad", C.c_int),
    ]


class LossOut(C.Structure):
    """``md2_loss_out``."""
    _fields_ = [
        ("loss", C.c_void_p), ("terms", C.c_void_p),
        ("d_disp", C.c_void_p * MAX_SCALES), ("d_pose", C.c_void_p),
        ("vis_loss", C.c_void_p), ("vis_sel", C.c_void_p), ("vis_warped", C.c_void_p),
        ("vis_cell", C.c_void_p),
    ]


class ConvDesc(C.Structure):
    """``md2_conv_desc``."""
    _fields_ = [(n, C.c_int) for n in ("n", "cin", "h", "w", "cout", "kh", "kw", "stride", "pad",
                                       "reflect", "act")]


class ModelCfg(C.Structure):
    """``md2_model_cfg``."""
    _fields_ = [
        ("arch", C.c_int), ("in_channels", C.c_int), ("batch", C.c_int),
        ("width", C.c_int), ("height", C.c_int),
        ("n_levels", C.c_int), ("scale_levels", C.c_int * MAX_SCALES),
        ("K", C.c_float * 9), ("invK", C.c_float * 9),
        ("min_depth", C.c_float), ("max_depth", C.c_float), ("disparity_smoothness", C.c_float),
        ("scales", C.c_float * MAX_SCALES),
        ("automasking", C.c_int), ("target", C.c_int), ("src0", C.c_int), ("src1", C.c_int),
        ("embedding_levels", C.c_int), ("num_bins", C.c_int),
    ]


class WarpCfg(C.Structure):
    """``md2_warp_cfg``."""
    _fields_ = [
        ("n", C.c_int), ("c", C.c_int), ("width", C.c_int), ("height", C.c_int),
        ("dw", C.c_int), ("dh", C.c_int),
        ("K", C.c_float * 9), ("invK", C.c_float * 9),
        ("min_depth", C.c_float), ("max_depth", C.c_float),
        ("x_sample_stride", C.c_longlong), ("x_frame_stride", C.c_longlong),
        ("target", C.c_int), ("src0", C.c_int), ("src1", C.c_int),
    ]


_lib = None
_load_error = None

CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
INCLUDE_H = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "md2.h")


def source_build_id():
    """The hash csrc/Makefile embeds as md2_build_id(): sha256 of the sorted csrc sources
    (*.hip *.cpp *.h *.inc), the Makefile and include/md2.h, concatenated; None without a tree."""
    import hashlib
    if not os.path.isdir(CSRC):
        return None
    names = sorted(set(n for n in os.listdir(CSRC)
                       if os.path.splitext(n)[1] in (".hip", ".cpp", ".h", ".inc")))
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, n) for n in names] + [os.path.join(CSRC, "Makefile"), INCLUDE_H]:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]

P = C.c_void_p
FP = C.POINTER(C.c_void_p)

_SIGS = {
    "md2_abi_version": (C.c_int, []),
    "md2_last_error": (C.c_char_p, []),
    "md2_build_id": (C.c_char_p, []),
    "md2_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "md2_memcpy_d2d": (C.c_int, [P, P, C.c_size_t, P]),
    "md2_loss_workspace_size": (C.c_size_t, [C.POINTER(LossCfg)]),
    "md2_loss_fwd_bwd": (C.c_int, [C.POINTER(LossCfg), FP, P, P, P, C.c_float, C.POINTER(LossOut), P, P]),
    "md2_so3_compose_fwd": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "md2_so3_compose_bwd": (C.c_int, [P, C.c_int, C.c_int, P, P, P]),
    "md2_conv2d_workspace_size": (C.c_size_t, [C.POINTER(ConvDesc)]),
    "md2_conv2d_fwd": (C.c_int, [C.POINTER(ConvDesc), P, P, P, P, P, P]),
    "md2_conv2d_dgrad": (C.c_int, [C.POINTER(ConvDesc), P, P, P, P, P]),
    "md2_conv2d_wgrad": (C.c_int, [C.POINTER(ConvDesc), P, P, P, P, P, P]),
    "md2_act_backward": (C.c_int, [P, P, P, C.c_longlong, C.c_int, P]),
    "md2_adam": (C.c_int, [P, P, P, P, C.c_longlong, C.c_float, C.c_float, C.c_float, C.c_float,
                            C.c_int, C.c_float, P]),
    "md2_maxpool3s2_fwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_maxpool3s2_bwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_upsample2_fwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_upsample2_bwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_arch_param_count": (C.c_int, [C.POINTER(ModelCfg), C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "md2_arch_param_info": (C.c_int, [C.POINTER(ModelCfg), C.c_int, C.c_char_p, C.c_int,
                                      C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_longlong)]),
    "md2_model_create": (C.c_int, [C.POINTER(ModelCfg), P, P, C.POINTER(C.c_void_p)]),
    "md2_model_destroy": (C.c_int, [P]),
    "md2_model_device_bytes": (C.c_size_t, [P]),
    "md2_model_repack": (C.c_int, [P, P]),
    "md2_model_forward_loss": (C.c_int, [P, P, P, P, P, P]),
    "md2_model_forward": (C.c_int, [P, P, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), P]),
    "md2_model_set_cotangents": (C.c_int, [P, FP, P, P]),
    "md2_model_backward_from": (C.c_int, [P, FP, P, P]),
    "md2_model_num_segments": (C.c_int, [P]),
    "md2_model_backward_segment": (C.c_int, [P, C.c_int, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong), P]),
    "md2_model_adam": (C.c_int, [P, P, P, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, C.c_float, P]),
    "md2_model_adam_segment": (C.c_int, [P, C.c_int, P, P, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int,
                                         C.c_float, P]),
    "md2_model_adam_join": (C.c_int, [P, P]),
    "md2_model_train_step": (C.c_int, [P, P, P, P, P, C.c_float, C.c_int, P, P]),
    "md2_model_train_step_graph": (C.c_int, [P, P, P, P, P, C.c_float, C.c_int, P, P]),
    "md2_model_set_params": (C.c_int, [P, P, P]),
    "md2_model_get_params": (C.c_int, [P, P, P]),
    "md2_model_get_grads": (C.c_int, [P, P, P]),
    "md2_model_loss_cotangent": (C.c_int, [P, C.c_float, P]),
    "md2_model_set_disparity_bins": (C.c_int, [P, P, P]),
    "md2_model_outputs": (C.c_int, [P, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                    C.POINTER(C.c_void_p)]),
    "md2_model_eval_disparity": (C.c_int, [P, P, C.c_int, C.POINTER(C.c_void_p), P]),
    "md2_model_debug_tensor": (C.c_int, [P, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_int)]),
    "md2_model_features": (C.c_int, [P, C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int)]),
    "md2_mpi_embed_features": (C.c_int, [P, C.c_longlong, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int,
                                         C.c_int, P, P]),
    "md2_concat_channels": (C.c_int, [P, C.c_int, P, C.c_int, C.c_int, C.c_longlong, P, P]),
    "md2_automasking_loss": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_static_scores_workspace_size": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "md2_static_scores": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_mine_src_xyz": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_mine_tgt_xyz": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_mine_sample": (C.c_int, [P, C.c_int, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P, P]),
    "md2_plane_volume_rendering": (C.c_int, [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P]),
    "md2_render_tgt_rgb_depth": (C.c_int, [P, P, P, P, P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P, P]),
    "md2_ssim_fwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_ssim_bwd": (C.c_int, [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_backproject_fwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_backproject_bwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_project_fwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, P, P, P, P, P]),
    "md2_project_workspace_size": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "md2_project_bwd": (C.c_int, [P, C.c_int, C.c_int, C.c_int, P, P, P, P, P, P, P, P, P]),
    "md2_grid_sample_border_fwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, P]),
    "md2_grid_sample_border_bwd": (C.c_int, [P, P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                             P, P, P]),
    "md2_unorm8_to_float": (C.c_int, [P, P, C.c_longlong, P]),
    "md2_png_info": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "md2_load_triplets_u8": (C.c_int, [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int, P, P, C.c_int]),
    "md2_load_kitti_u8": (C.c_int, [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int, P, P, C.c_int]),
    "md2_smooth_loss_workspace_size": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "md2_smooth_loss_fwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, P, P, P]),
    "md2_smooth_loss_bwd": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, P, P, P]),
    "md2_warp_photometric_workspace_size": (C.c_size_t, [C.POINTER(WarpCfg)]),
    "md2_warp_photometric_fwd": (C.c_int, [C.POINTER(WarpCfg), P, P, P, P, P, P, P, P]),
    "md2_warp_photometric_bwd": (C.c_int, [C.POINTER(WarpCfg), P, P, P, P, P, P, P, P, P]),
    "md2_model_set_profiling": (C.c_int, [P, C.c_int]),
    "md2_model_profile_read": (C.c_int, [P, C.POINTER(C.c_double), C.c_int]),
    "md2_model_profile_records": (C.c_int, [P, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                            C.POINTER(C.c_int), C.c_char_p, C.c_int, C.POINTER(C.c_int)]),
}


def lib():
    """Load libmd2hip.so once (raises if it is missing: there is no CPU fallback)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libmd2hip.so not found at {LIB_PATH}: run `make -C monodepth2.jl_amd/csrc` "
                           "(or __graft_entry__.build()); the HIP path has no fallback")
    # torch must be imported first so that its HIP runtime is the one in the process
    import torch  # noqa: F401
    l = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        f = getattr(l, name)
        f.restype = res
        f.argtypes = args
    got = l.md2_abi_version()
    if got != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH} has ABI version {got}, this binding expects {ABI_VERSION}: "
                           "rebuild the library or update md2hip")
    built = l.md2_build_id().decode()
    want = source_build_id()
    if want is not None and built != want and os.environ.get("MD2HIP_LIB") is None:
        raise RuntimeError(f"{LIB_PATH} was built from other sources (build id {built}, tree {want}): "
                           "stale library -- rebuild with `make -C monodepth2.jl_amd/csrc`")
    _lib = l
    return l


def declare(name, restype, argtypes):
    """Register the signature of an additional exported symbol."""
    _SIGS[name] = (restype, argtypes)
    if _lib is not None:
        f = getattr(_lib, name)
        f.restype = restype
        f.argtypes = argtypes


class MD2Error(RuntimeError):
    pass


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().md2_last_error().decode(errors="replace")
        raise MD2Error(f"{what} failed (code {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (or None -> NULL)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


def ptr_array(ts, n=MAX_SCALES):
    arr = (C.c_void_p * n)()
    for i, t in enumerate(ts):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def stream_of(device=None):
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
