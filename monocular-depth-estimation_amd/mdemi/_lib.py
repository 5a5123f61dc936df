"""ctypes binding of libmdemi.so (the C ABI declared in include/mdemi.h).

The library is built in-tree (``csrc/Makefile`` -> ``mdemi/libmdemi.so``) and
loaded *after* torch so that it binds the HIP runtime torch already mapped
(one runtime per process).  There is no fallback: if the library is missing
every op raises, which is what the GPU tests and ``smoke()`` rely on.

Error behaviour mirrors the reference: failures of the device library surface
as ``RuntimeError`` (as ``utils/dist_utils.py:29,37,57`` does for invalid
collectives); shape/config errors raised in Python stay ``ValueError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the HIP library is mapped)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MDEMI_LIB") or os.path.join(_HERE, "libmdemi.so")  # override: A/B benchmarking
HEADER_PATH = os.path.abspath(os.path.join(_HERE, "..", "..", "include", "mdemi.h"))
HEADER_PATHS = [HEADER_PATH, os.path.abspath(os.path.join(_HERE, "..", "..", "include", "mdemi_ext.h"))]

c_float_p = ctypes.POINTER(ctypes.c_float)
vp = ctypes.c_void_p
i32 = ctypes.c_int32
i64 = ctypes.c_int64
f32 = ctypes.c_float
sz = ctypes.c_size_t

# ---- constants (include/mdemi.h) ----
L_KCONTIG, L_MNCONTIG, L_CONV = 0, 1, 2
OP_NONE, OP_GELU = 0, 1
BIAS_NONE, BIAS_COL, BIAS_ROW = 0, 1, 2
ACT_NONE, ACT_GELU, ACT_RELU, ACT_LEAKY, ACT_GELU_GRAD, ACT_SIGMOID = 0, 1, 2, 3, 4, 5
ACT_SILU, ACT_RELU_GRAD, ACT_SILU_GRAD = 6, 7, 8
ACT_GRAD_OF = {ACT_GELU: ACT_GELU_GRAD, ACT_RELU: ACT_RELU_GRAD, ACT_SILU: ACT_SILU_GRAD}
BINS_RELU, BINS_ELU = 0, 1  # include/mdemi_ext.h
WL_OHWI, WL_OIHW, WL_DGRAD = 0, 1, 2  # include/mdemi_ext.h (mdemi_conv_weight_layout)
PAD_ZERO, PAD_REPLICATE = 0, 1
EW_ADD, EW_SIGMOID_SCALE, EW_SIGMOID_SCALE_BWD, EW_AXPBY, EW_ACT_BWD = 0, 1, 2, 3, 4


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, i32) for n in ("n", "h", "w", "c", "oh", "ow", "kh", "kw", "stride", "pad",
                                   "pad_mode", "_reserved")]


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("M", i32), ("N", i32), ("K", i32), ("batch", i32),
        ("A", vp), ("lda", i64), ("a_bstride", i64), ("a_layout", i32), ("a_op", i32),
        ("B", vp), ("ldb", i64), ("b_bstride", i64), ("b_layout", i32), ("b_op", i32),
        ("C", vp), ("ldc", i64), ("c_bstride", i64),
        ("alpha", f32), ("beta", f32),
        ("bias", vp), ("bias_mode", i32), ("act", i32),
        ("aux", vp), ("ldaux", i64), ("aux_bstride", i64),
        ("residual", vp), ("ldres", i64), ("res_bstride", i64),
        ("split_k", i32), ("_pad0", i32),
        ("workspace", vp), ("workspace_bytes", i64),
        ("conv", ConvGeom),
        ("preact", vp), ("ldpre", i64), ("pre_bstride", i64),
        ("rowsum_a", vp),
        ("batch_inner", i32), ("_pad1", i32),
        ("a_bstride_inner", i64), ("b_bstride_inner", i64), ("c_bstride_inner", i64),
        ("row_scale", vp), ("row_scale_group", i64),
    ]


class WinAttnDesc(ctypes.Structure):
    _fields_ = [
        ("B", i32), ("H", i32), ("W", i32), ("heads", i32), ("head_dim", i32), ("window", i32),
        ("shift", i32), ("_pad0", i32),
        ("scale", f32), ("_pad1", i32),
        ("q", vp), ("k", vp), ("qk_ld", i64),
        ("q_pad", vp), ("k_pad", vp),
        ("v", vp), ("v_ld", i64), ("v_pad", vp),
        ("rpb_table", vp),
        ("out", vp), ("out_ld", i64),
        ("lse", vp),
        ("dout", vp),
        ("dq", vp), ("dk", vp), ("dqk_ld", i64),
        ("dv", vp), ("dv_ld", i64),
        ("d_rpb_table", vp),
        ("dq_pad", vp), ("dk_pad", vp), ("dv_pad", vp),
        ("workspace", vp), ("workspace_bytes", i64),
    ]


class TensorRef(ctypes.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp),
                ("numel", i64), ("group", i32), ("step_slot", i32)]


class AdamWGroup(ctypes.Structure):
    _fields_ = [("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32),
                ("_pad", i32)]


AUG_MAX_SPANS = 8  # include/mdemi_ext.h MDEMI_AUG_MAX_SPANS


class AugSample(ctypes.Structure):  # include/mdemi_ext.h mdemi_aug_sample
    _fields_ = [("affine", ctypes.c_double * 6), ("fixed", i32 * 6), ("rotate", i32), ("crop_x", i32),
                ("crop_y", i32), ("flip", i32), ("gamma", f32), ("brightness", f32), ("color", f32 * 3),
                ("n_rows", i32), ("n_cols", i32), ("mask_keep", i32), ("rows", (i32 * 2) * AUG_MAX_SPANS),
                ("cols", (i32 * 2) * AUG_MAX_SPANS)]


# name -> (restype, argtypes)
_SIGS = {
    "mdemi_last_error": (ctypes.c_char_p, []),
    "mdemi_version": (ctypes.c_int, []),
    "mdemi_gemm_workspace_size": (sz, [ctypes.POINTER(GemmDesc)]),
    "mdemi_gemm_f32": (ctypes.c_int, [ctypes.POINTER(GemmDesc), vp]),
    "mdemi_gemm_bf16": (ctypes.c_int, [ctypes.POINTER(GemmDesc), vp]),
    "mdemi_gemm_f32e": (ctypes.c_int, [ctypes.POINTER(GemmDesc), vp]),
    "mdemi_gemm_set_variant": (ctypes.c_int, [i32, i32]),
    "mdemi_gemm_set_variant_m16": (ctypes.c_int, [i32]),
    "mdemi_gemm_bf16x": (ctypes.c_int, [ctypes.POINTER(GemmDesc), vp, vp, vp, vp]),
    "mdemi_gemm_bf16x_supported": (ctypes.c_int, [ctypes.POINTER(GemmDesc), vp, vp]),
    "mdemi_gemm_set_variant_b16": (ctypes.c_int, [i32]),
    "mdemi_cast_bf16": (ctypes.c_int, [vp, vp, i64, vp]),
    "mdemi_add16": (ctypes.c_int, [vp, vp, vp, vp, i64, vp]),
    "mdemi_bn_train_fwd16": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, i64, i32, f32, i32, vp,
                                            vp]),
    "mdemi_bn_train_fwd_pooled_workspace_size": (sz, [i32, i64, i32]),
    "mdemi_bn_train_fwd_pooled": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, i64, i32, f32, i32,
                                                 vp, vp]),
    "mdemi_chnorm_bwd16": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32,
                                          vp, vp]),
    "mdemi_chan_scale16": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i64, i32, vp]),
    "mdemi_gemm_set_options": (ctypes.c_int, [i32, i32]),
    "mdemi_colsum_workspace_size": (sz, [i64, i64]),
    "mdemi_colsum_f32": (ctypes.c_int, [vp, i64, i64, i64, vp, ctypes.c_int, vp, vp]),
    "mdemi_headconv_fwd": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_headconv_wgrad_workspace_size": (sz, [i32, i32, i32, i32, i32]),
    "mdemi_headconv_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp]),
    "mdemi_binhead_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i32, i64, i32, vp]),
    "mdemi_binhead_bwd_workspace_size": (sz, [i32, i32, i64]),
    "mdemi_binhead_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i64, i32, vp, vp]),
    "mdemi_layernorm_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, f32, vp]),
    "mdemi_layernorm_fwd16": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, i32, f32, vp]),
    "mdemi_layernorm_bwd_workspace_size": (sz, [i64, i32]),
    "mdemi_layernorm_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp, vp]),
    "mdemi_layernorm_bwd_add": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp, vp]),
    "mdemi_winattn_fwd_workspace_size": (sz, [ctypes.POINTER(WinAttnDesc)]),
    "mdemi_winattn_fwd": (ctypes.c_int, [ctypes.POINTER(WinAttnDesc), vp]),
    "mdemi_winattn_bwd_workspace_size": (sz, [ctypes.POINTER(WinAttnDesc)]),
    "mdemi_winattn_bwd": (ctypes.c_int, [ctypes.POINTER(WinAttnDesc), vp]),
    "mdemi_winattn_bwd_bias": (ctypes.c_int, [ctypes.POINTER(WinAttnDesc), vp, vp]),
    "mdemi_silog_workspace_size": (sz, [i32, i64]),
    "mdemi_silog_fwd": (ctypes.c_int, [vp, vp, vp, vp, i32, i64, f32, f32, f32, i32, i32, vp, vp]),
    "mdemi_silog_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i64, f32, f32, f32, i32, i32, vp]),
    "mdemi_bilinear_fwd": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, f32, i64, i64, vp]),
    "mdemi_bilinear_bwd": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, f32, i64, i64, i32, vp]),
    "mdemi_nchw_to_nhwc": (ctypes.c_int, [vp, vp, i32, i32, i64, vp]),
    "mdemi_nhwc_to_nchw": (ctypes.c_int, [vp, vp, i32, i32, i64, vp]),
    "mdemi_pixel_shuffle_nhwc": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_patchify_nchw": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_adaptive_avgpool_fwd": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_adaptive_avgpool_bwd": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_chnorm_workspace_size": (sz, [i32, i64, i32, i32, i32]),
    "mdemi_chnorm_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, f32, i32, vp, vp]),
    "mdemi_chnorm_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32,
                                        vp, vp]),
    "mdemi_elementwise": (ctypes.c_int, [i32, vp, vp, vp, i64, f32, f32, vp]),
    "mdemi_rowscale_add": (ctypes.c_int, [vp, vp, vp, vp, i64, i64, vp]),
    "mdemi_space_to_depth2": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, vp]),
    "mdemi_copy2d": (ctypes.c_int, [vp, i64, vp, i64, i64, i64, i32, vp]),
    "mdemi_chnorm_apply": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, i32, i32, vp]),
    "mdemi_bn_frozen_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, i32, vp, vp]),
    "mdemi_bn_train_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, i64, i32, f32, i32, vp, vp]),
    "mdemi_bn_running_update": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i64, f32, f32, vp]),
    "mdemi_multi_tensor_chunk": (ctypes.c_int, []),
    "mdemi_grad_norm_workspace_size": (sz, [i32]),
    "mdemi_grad_sumsq": (ctypes.c_int, [vp, i32, i64, f32, vp, vp, vp]),
    "mdemi_adamw_step": (ctypes.c_int, [vp, i32, ctypes.POINTER(AdamWGroup), i32, vp, f32, f32, i32, vp, i64, vp, vp]),
    "mdemi_adamw_step_dev": (ctypes.c_int, [vp, i32, vp, i32, i32, vp, vp, vp, f32, f32, i64, vp, vp]),
    "mdemi_adamw_step16": (ctypes.c_int, [vp, i32, ctypes.POINTER(AdamWGroup), i32, vp, f32, f32, i32, vp, i64, vp, vp,
                                          vp]),
    "mdemi_adamw_step_dev16": (ctypes.c_int, [vp, i32, vp, i32, i32, vp, vp, vp, f32, f32, i64, vp, vp, vp]),
    # ---- include/mdemi_ext.h ----
    "mdemi_dwconv_fwd": (ctypes.c_int, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_dwconv_bwd_workspace_size": (sz, [i32, i32, i32, i32, i32]),
    "mdemi_dwconv_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp,
                                        vp]),
    "mdemi_spatial_reduce_workspace_size": (sz, [i32, i64, i32]),
    "mdemi_spatial_reduce": (ctypes.c_int, [vp, vp, vp, i32, i64, i32, f32, vp, vp]),
    "mdemi_chan_scale": (ctypes.c_int, [vp, vp, vp, vp, i32, i64, i32, vp]),
    "mdemi_se_gate_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, vp]),
    "mdemi_se_gate_bwd_workspace_size": (sz, [i32, i32, i32]),
    "mdemi_se_gate_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, vp, vp]),
    "mdemi_softmax_fwd": (ctypes.c_int, [vp, vp, i64, i32, f32, vp]),
    "mdemi_softmax_bwd": (ctypes.c_int, [vp, vp, vp, i64, i32, f32, i32, vp]),
    "mdemi_softmax_fwd16": (ctypes.c_int, [vp, vp, vp, i64, i32, f32, vp]),
    "mdemi_softmax_bwd16": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, f32, i32, vp]),
    "mdemi_act_fwd": (ctypes.c_int, [vp, vp, i64, i32, vp]),
    "mdemi_dropout": (ctypes.c_int, [vp, vp, i64, f32, ctypes.c_uint64, ctypes.c_uint64, vp]),
    "mdemi_dropout_dev": (ctypes.c_int, [vp, vp, i64, f32, vp, ctypes.c_uint64, ctypes.c_uint64, vp]),
    "mdemi_dropout_dev16": (ctypes.c_int, [vp, vp, vp, i64, f32, vp, ctypes.c_uint64, ctypes.c_uint64, vp]),
    "mdemi_softmax_fwd_drop16": (ctypes.c_int, [vp, vp, vp, i64, i32, f32, f32, vp, ctypes.c_uint64, ctypes.c_uint64,
                                                vp]),
    "mdemi_binhead_nhwc_fwd": (ctypes.c_int, [vp, vp, vp, vp, i32, i64, i32, vp]),
    "mdemi_binhead_nhwc_bwd_workspace_size": (sz, [i32, i64, i32]),
    "mdemi_binhead_nhwc_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, vp, vp]),
    "mdemi_bins_fwd": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, i32, f32, f32, vp]),
    "mdemi_bins_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, vp]),
    "mdemi_nchw_to_nhwc_pad": (ctypes.c_int, [vp, vp, i32, i32, i64, i32, vp]),
    "mdemi_unpatchify_nhwc": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_pad_fold_replicate": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, vp]),
    "mdemi_depth_metrics_workspace_size": (sz, [i32, i32, i32]),
    "mdemi_depth_metrics": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, i32, f32, f32, i32, vp, vp, vp]),
    "mdemi_flip_w": (ctypes.c_int, [vp, vp, i64, i32, vp]),
    "mdemi_flip_avg_w": (ctypes.c_int, [vp, vp, vp, i64, i32, vp]),
    "mdemi_bins_chamfer_workspace_size": (sz, [i32, i32, i64]),
    "mdemi_bins_chamfer_fwd": (ctypes.c_int, [vp, vp, i32, i32, i32, i64, f32, vp, vp, vp, vp]),
    "mdemi_bins_chamfer_bwd": (ctypes.c_int, [vp, vp, vp, i32, i32, i32, vp]),
    "mdemi_conv_weight_layout": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, vp]),
    "mdemi_conv_weight_layout16": (ctypes.c_int, [vp, vp, vp, i32, i32, i32, i32, i32, vp]),
    "mdemi_augment": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, i32, i32,
                                     f32, f32, vp, vp, vp]),
    "mdemi_window_shuffle": (ctypes.c_int, [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, vp]),
    "mdemi_window_shuffle_i32": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, vp]),
    "mdemi_ordered_softmax_fwd": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, i32, i32, f32, vp]),
    "mdemi_ordered_softmax_bwd_workspace_size": (sz, [i32, i32, i32]),
    "mdemi_ordered_softmax_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp, vp]),
    "mdemi_glu_fwd": (ctypes.c_int, [vp, vp, i64, i32, vp]),
    "mdemi_glu_bwd": (ctypes.c_int, [vp, vp, vp, i64, i32, vp]),
    "mdemi_pad_replicate": (ctypes.c_int, [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp]),
}

_lib = None
_lock = threading.Lock()


class MdemiLibraryError(RuntimeError):
    pass


def load():
    """Map libmdemi.so and declare every entry point. Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise MdemiLibraryError(
                f"libmdemi.so not found at {LIB_PATH}; build it with "
                "`make -C monocular-depth-estimation_amd/csrc` (or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                if os.environ.get("MDEMI_LIB"):  # an A/B build of an older ABI
                    continue
                raise MdemiLibraryError(f"{LIB_PATH} does not export {name}")
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def exported_symbols():
    return list(_SIGS.keys())


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().mdemi_last_error().decode(errors="replace")
        raise RuntimeError(f"mdemi {what} failed (rc={rc}): {msg}")


def call(name: str, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


# ---- per-device scratch (the library never allocates) ----
_ws: dict = {}
# Once a hipGraph has been captured, a workspace buffer superseded by a larger one
# (a later eager call at a bigger shape) must never return to the allocator: the
# graph keeps the raw addresses it was recorded with.  Before any capture, a
# superseded buffer is freed only after the device has drained: workspaces are
# also used on side streams (GraphedPredictor's warm-up stream), and the caching
# allocator would otherwise hand the block to a new allocation on its origin
# stream while another stream's kernels still use it.  Growth happens in
# warm-up only, so the synchronisation is rare.
_ws_retired: list = []
_graph_captured = False


def note_graph_capture() -> None:
    """Called when a workspace is handed out during a capture (and by Trainer)."""
    global _graph_captured
    _graph_captured = True


def workspace(nbytes: int, device=None, slot: int = 0) -> torch.Tensor:
    """Return a cached uint8 device buffer of at least nbytes (stream-ordered reuse)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (device.index if device.index is not None else torch.cuda.current_device(), slot)
    buf = _ws.get(key)
    nbytes = max(int(nbytes), 256)
    capturing = torch.cuda.is_current_stream_capturing()
    if capturing:
        note_graph_capture()
    if buf is None or buf.numel() < nbytes:
        if capturing:
            raise RuntimeError(f"mdemi: workspace slot {slot} must grow to {nbytes} bytes during hipGraph capture; "
                               "run the captured step eagerly first (warm-up) so every workspace is sized")
        if buf is not None:
            if _graph_captured:
                _ws_retired.append(buf)
            else:
                torch.cuda.synchronize(device)
        buf = torch.empty(int(nbytes * 1.25) + 4096, dtype=torch.uint8, device=device)
        _ws[key] = buf
    return buf
