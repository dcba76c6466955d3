"""ctypes binding of libe2ep_hip.so (C ABI: include/e2ep.h).

The library is built in-tree by csrc/Makefile (or __graft_entry__.build()).  There is no
fallback: if it is missing or fails to load, every op raises — the product path never
silently degrades to PyTorch or CPU code.
"""
import ctypes
import os

import torch  # noqa: F401  (loads torch's libamdhip64 first, so the library binds to it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("E2EP_LIB", os.path.join(_HERE, "libe2ep_hip.so"))

_p, _i, _i64, _f, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_size_t
_d = ctypes.c_double
_fp3 = ctypes.POINTER(ctypes.c_float)

# name -> (restype, argtypes); must match include/e2ep.h
SIGNATURES = {
    "e2ep_abi_version": (_i, []),
    "e2ep_last_error": (ctypes.c_char_p, []),
    "e2ep_rig_transforms": (_i, [_p, _p, _i, _p, _p, _p]),
    "e2ep_geom_index": (_i, [_p, _p, _p, _fp3, _fp3, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p]),
    "e2ep_lss_plan_workspace": (_sz, [_i, _i]),
    "e2ep_lss_tiles": (_i, [_i]),
    "e2ep_debug_fwd_trace": (_i, [_p]),
    "e2ep_lss_plan": (_i, [_p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _sz, _p]),
    "e2ep_lss_fwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _i64, _p]),
    "e2ep_lss_bwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p]),
    "e2ep_transpose": (_i, [_p, _i64, _i, _i, _i, _p, _p]),
    "e2ep_transpose_multi": (_i, [_p, _i, _i, _p]),
    "e2ep_target_bev": (_i, [_p, _p, _i, _i, _i, _f, _f, _p, _i64, _p]),
    "e2ep_conv_fwd_workspace": (_sz, [_p]),
    "e2ep_conv_fwd": (_i, [_p, _p, _p, _p, _i, _i, _p, _p, _sz, _p, _i]),
    "e2ep_conv_fwd_stats_tiles": (_i, [_p, _i]),
    "e2ep_conv_fwd_stats": (_i, [_p, _p, _p, _p, _i, _i, _p, _p, _sz, _p, _sz, _p, _i]),
    "e2ep_conv_dgrad_workspace": (_sz, [_p, _i]),
    "e2ep_conv_dgrad": (_i, [_p, _p, _p, _i, _i, _p, _p, _sz, _p]),
    "e2ep_conv_dgrad_acc": (_i, [_p, _p, _p, _i, _i, _p, _p, _p, _sz, _p, _i]),
    "e2ep_conv_gemm_variant": (_i, [_i]),
    "e2ep_conv_split_params": (_i, [_i, _i, _i]),
    "e2ep_conv_precision": (_i, [_i]),
    "e2ep_gemm_precision": (_i, [_i]),
    "e2ep_fusion_tokens_fwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _f, _p, _p, _p]),
    "e2ep_fusion_tokens_bwd": (_i, [_p, _i, _i, _i, _i, _f, _p, _p, _p, _p, _p]),
    "e2ep_embed_tokens_fwd": (_i, [_p, _i, _p, _i, _p, _i, _i, _i, _f, _p, _p, _p]),
    "e2ep_embed_tokens_bwd": (_i, [_p, _p, _i, _i, _i, _i, _i, _f, _p, _p, _p, _p]),
    "e2ep_conv_wgrad_kstep": (_i, [_i]),
    "e2ep_conv_wgrad_splits": (_i, [_p]),
    "e2ep_conv_wgrad_workspace": (_sz, [_p, _i]),
    "e2ep_conv_wgrad": (_i, [_p, _p, _p, _i, _p, _sz, _p, _i, _p, _i]),
    "e2ep_conv_bwd_pair_ok": (_i, [_p, _i]),
    "e2ep_conv_bwd": (_i, [_p, _p, _p, _p, _i, _p, _p, _p, _sz, _i, _p, _sz, _p, _p, _i]),
    "e2ep_bias_grad": (_i, [_p, _i, _i, _i, _p, _p]),
    "e2ep_col_sum_workspace": (_sz, [_i, _i]),
    "e2ep_col_sum": (_i, [_p, _i, _i, _p, _p, _p]),
    "e2ep_skinny_gemm": (_i, [_p, _i, _i, _p, _i, _i, _p, _i, _i, _i, _p, _p]),
    "e2ep_bn_workspace": (_sz, [_i, _i, _i, _i]),
    "e2ep_bn_fwd": (_i, [_p, _p, _p, _p, _p, _f, _p, _p, _i, _i, _i, _i, _i, _f, _f, _i, _p, _p, _p, _p, _sz, _p]),
    "e2ep_bn_stats": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _f, _f, _p, _p, _p, _p, _p, _sz, _p, _i]),
    "e2ep_bn_fwd_split": (_i, [_i, _i, _i, _i]),
    "e2ep_bn_finalize_part_workspace": (_sz, [_i, _i]),
    "e2ep_bn_finalize_part": (_i, [_p, _i, _p, _p, _p, _p, _i, _i, _i, _i, _f, _f, _p, _p, _p, _p, _p, _sz, _p]),
    "e2ep_bn_apply": (_i, [_p, _p, _p, _p, _p, _f, _i, _i, _i, _i, _i, _p, _p]),
    "e2ep_bn_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _f, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _sz, _p, _i]),
    "e2ep_act_fwd": (_i, [_p, _i64, _i, _p, _p]),
    "e2ep_act_bwd": (_i, [_p, _p, _i64, _i, _p, _p]),
    "e2ep_cat_channels": (_i, [_p, _p, _i, _i, _i64, _p, _p]),
    "e2ep_split_channels": (_i, [_p, _p, _i, _i, _i64, _p, _p]),
    "e2ep_sum3": (_i, [_p, _p, _p, _p, _p]),
    "e2ep_add_f32": (_i, [_p, _p, _i64, _p, _p]),
    "e2ep_rng_draw": (_i, [_p, _i, _p, _i, _p, _p]),
    "e2ep_eq_mask_i64": (_i, [_p, _i64, _i, _i, _i64, _p, _p]),
    "e2ep_add_i64_multi": (_i, [_p, _i, _i64, _p]),
    "e2ep_resize_fwd": (_i, [_p, _i, _i, _i64, _i, _i, _i, _i, _f, _f, _p, _i64, _p]),
    "e2ep_resize_bwd_workspace": (_sz, [_i, _i, _i]),
    "e2ep_resize_bwd": (_i, [_p, _i64, _i, _i, _i, _i, _i, _f, _f, _p, _i, _p, _p]),
    "e2ep_resize_bwd_cl": (_i, [_p, _i64, _i, _i, _i, _i, _i, _i, _f, _f, _p, _p]),
    "e2ep_dwconv_fwd": (_i, [_p, _p, _p, _p, _p, _i, _p, _p]),
    "e2ep_dwconv_fwd_stats_tiles": (_i, [_p]),
    "e2ep_dwconv_fwd_stats": (_i, [_p, _p, _p, _p, _p, _i, _p, _p, _sz, _p, _i]),
    "e2ep_dwconv_dgrad": (_i, [_p, _p, _p, _p, _p, _i]),
    "e2ep_dwconv_wgrad_workspace": (_sz, [_p]),
    "e2ep_dwconv_wgrad": (_i, [_p, _p, _p, _p, _p, _i, _p, _sz, _p, _p, _i]),
    "e2ep_dwconv_bwd_pair_ok": (_i, [_p]),
    "e2ep_dwconv_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _p, _p, _sz, _p, _p, _i]),
    "e2ep_maxpool3s2_fwd": (_i, [_p, _i, _i, _i, _p, _p, _p]),
    "e2ep_maxpool3s2_bwd": (_i, [_p, _p, _i, _i, _i, _p, _p]),
    "e2ep_avgpool_fwd": (_i, [_p, _i, _i, _p, _p]),
    "e2ep_avgpool_bwd": (_i, [_p, _i, _i, _p, _p]),
    "e2ep_add_drop_ln_fwd": (_i, [_p, _p, _p, _f, _p, _p, _i, _i, _f, _p, _p, _p, _p, _p]),
    "e2ep_add_drop_ln_bwd_workspace": (_sz, [_i, _i]),
    "e2ep_add_drop_ln_fwd_seeded": (_i, [_p, _p, _p, _f, _p, _p, _i, _i, _f, _p, _p, _p, _p, _p]),
    "e2ep_add_drop_ln_bwd_seeded": (_i, [_p, _p, _p, _p, _p, _p, _f, _i, _i, _p, _p, _p, _p, _p, _p]),
    "e2ep_add_drop_ln_bwd": (_i, [_p, _p, _p, _p, _p, _p, _f, _i, _i, _p, _p, _p, _p, _p, _p]),
    "e2ep_attn_fwd": (_i, [_p, _p, _p] + [_i] * 11 + [_f, _i, _p, _f, _p, _p, _p, _p]),
    "e2ep_attn_bwd_workspace": (_sz, [_i, _i, _i]),
    "e2ep_attn_bwd": (_i, [_p] * 6 + [_i] * 11 + [_f, _i, _p, _f, _p, _p, _p, _p, _p, _p]),
    "e2ep_attn_bwd_part": (_i, [_p] * 6 + [_i] * 11 + [_f, _i, _p, _f, _p, _p, _p, _p, _p, _i, _p]),
    "e2ep_attn_keep_mask": (_i, [_p, _i, _i, _i, _f, _p, _p]),
    "e2ep_softmax_c_fwd": (_i, [_p, _i, _i, _i, _p, _p]),
    "e2ep_softmax_c_bwd": (_i, [_p, _p, _i, _i, _i, _p, _p]),
    "e2ep_relu_dropout_fwd": (_i, [_p, _i64, _f, _p, _p, _p]),
    "e2ep_relu_dropout_bwd": (_i, [_p, _p, _i64, _f, _p, _p, _p]),
    "e2ep_se_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i]),
    "e2ep_se_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i]),
    "e2ep_se_bwd_bn": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i]),
    "e2ep_bn_bwd_planes": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i]),
    "e2ep_bn_bwd_split": (_i, [_i, _i, _i, _i]),
    "e2ep_bn_eval_multi": (_i, [_p, _i, _p]),
    "e2ep_se_gate_fwd": (_i, [_p, _p, _i, _i, _p, _p]),
    "e2ep_se_gate_bwd": (_i, [_p, _p, _p, _i, _i, _p, _p, _p]),
    "e2ep_adam_chunk_elems": (_i, []),
    "e2ep_adam_step": (_i, [_p, _i, _p, _p, _p, _p, _p, _p, _p, _p, _d, _d, _d, _d, _f, _p, _p]),
    "e2ep_grad_gather": (_i, [_p, _i, _p, _p, _p, _p]),
    "e2ep_graph_replace_memsets": (_i, [_p, ctypes.POINTER(_i)]),
    "e2ep_graph_exec_create": (_i, [_p, _p]),
    "e2ep_graph_exec_launch": (_i, [_p, _p]),
    "e2ep_graph_exec_destroy": (_i, [_p]),
    "e2ep_capture_unjoined": (_i, [_p, _p, ctypes.POINTER(_i)]),
    "e2ep_tokens_init": (_i, [_p, _i, _i, _i, _p, _i, _i64, _p]),
    "e2ep_token_argmax_append": (_i, [_p, _i64, _i, _i, _p, _i, _i, _p]),
    "e2ep_dwconv_bf16_ok": (_i, [_p]),
    "e2ep_control_ce_workspace": (_sz, [_i]),
    "e2ep_control_ce_fwd": (_i, [_p, _p, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p]),
    "e2ep_control_ce_bwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _p, _p]),
    "e2ep_seg_ce_workspace": (_sz, [_i, _i]),
    "e2ep_seg_ce_fwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _p, _p, _p]),
    "e2ep_seg_ce_bwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _p, _p]),
    "e2ep_depth_bce_workspace": (_sz, [_i, _i, _i, _i]),
    "e2ep_depth_bce_fwd": (_i, [_p, _p, _i, _i, _i, _i, _i, _f, _f, _p, _p, _p, _p, _p]),
    "e2ep_depth_bce_fwd_f64": (_i, [_p, _p, _i, _i, _i, _i, _i, _d, _d, _p, _p, _p, _p, _p]),
    "e2ep_gemm_workspace": (_sz, [_i, _i, _i]),
    "e2ep_gemm_force": (_i, [_i, _i, _i]),
    "e2ep_gemm_skinny": (_i, [_i]),
    "e2ep_gemm_split_min": (_i, [_i]),
    "e2ep_bn_small": (_i, [_i]),
    "e2ep_bn_small_limits": (_i, [_i, _i]),
    "e2ep_tune": (_i, [_i, _i]),
    "e2ep_gemm": (_i, [_p, _i, _i, _p, _i, _i, _p, _p, _i, _p, _i, _i, _i, _i, _i, _p, _sz, _p]),
    "e2ep_gemm_rowsum_workspace": (_sz, [_i, _i, _i]),
    "e2ep_gemm_rowsum": (_i, [_p, _i, _p, _i, _p, _i, _p, _i, _i, _i, _p, _sz, _p]),
    "e2ep_linear_bwd": (_i, [_p, _i, _p, _i, _p, _i, _p, _i, _p, _i, _p, _i, _p, _i, _i, _i, _p, _sz, _p, _sz, _p]),
    "e2ep_decode_frames": (_i, [_p, _p, _p, _i64, _i, _p, _p, _p]),
    "e2ep_widen_u8_i64": (_i, [_p, _p, _i64, _i, _p, _p]),
    "e2ep_depth_bce_bwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p, _p]),
}

_LIB = None
_ERR = None


class E2EPError(RuntimeError):
    pass


def load():
    """Load and bind the library once; raise E2EPError if it is not there."""
    global _LIB, _ERR
    if _LIB is not None:
        return _LIB
    if _ERR is not None:
        raise _ERR
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    except (OSError, AttributeError) as e:
        _ERR = E2EPError(f"libe2ep_hip.so unavailable ({LIB_PATH}): {e}. Build it with "
                         f"`make -C e2e-parking-carla_amd/csrc` or __graft_entry__.build().")
        raise _ERR
    _LIB = lib
    if os.environ.get("E2EP_CONV_VARIANT"):  # A/B timing of the conv GEMM kernel choice
        lib.e2ep_conv_gemm_variant(int(os.environ["E2EP_CONV_VARIANT"]))
    if os.environ.get("E2EP_GEMM_SKINNY"):  # A/B timing of the few-row GEMM path
        lib.e2ep_gemm_skinny(int(os.environ["E2EP_GEMM_SKINNY"]))
    if os.environ.get("E2EP_CONV_SPLIT"):  # "target,thresh[,wgrad_target]" for A/B timing
        v = [int(x) for x in os.environ["E2EP_CONV_SPLIT"].split(",")] + [0]
        lib.e2ep_conv_split_params(v[0], v[1], v[2])
    if os.environ.get("E2EP_BN_SMALL_LIMITS"):  # "fwd_max_vec,bwd_max_vec" for A/B timing
        f, b = (int(x) for x in os.environ["E2EP_BN_SMALL_LIMITS"].split(","))
        lib.e2ep_bn_small_limits(f, b)
    if os.environ.get("E2EP_TUNE"):  # "key=value,..." launch-plan tunables for A/B timing
        for kv in os.environ["E2EP_TUNE"].split(","):
            k, v = kv.split("=")
            lib.e2ep_tune(int(k), int(v))
    if os.environ.get("E2EP_GEMM_SPLIT_MIN"):  # A/B timing of small-grid K splits
        lib.e2ep_gemm_split_min(int(os.environ["E2EP_GEMM_SPLIT_MIN"]))
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise E2EPError(f"{name} failed ({rc}): {lib.e2ep_last_error().decode()}")


def call_raw(name, *args):
    """Call an entry point that returns a value rather than a status."""
    return getattr(load(), name)(*args)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def nbytes(t):
    """Size in bytes of a workspace tensor (None -> 0), passed with it as workspace_bytes."""
    return 0 if t is None else t.numel() * t.element_size()


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dims(vals):
    """A host int32 array (kept alive by the caller for the duration of the call)."""
    return (ctypes.c_int * len(vals))(*[int(v) for v in vals])


def host3(vals):
    return (ctypes.c_float * 3)(*[float(v) for v in vals])
