"""ctypes binding of libsdk_amd.so — the C ABI declared in include/sdk_amd.h.

No fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SD_AMD_LIB selects another build of the same ABI (A/B benchmarking of kernel revisions only)
LIB_PATH = os.environ.get("SD_AMD_LIB") or os.path.join(_HERE, "libsdk_amd.so")

vp = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
f32 = C.c_float
fp = C.POINTER(C.c_float)


class ConvSrc(C.Structure):
    _fields_ = [("src0", vp), ("src1", vp), ("c_split", i32), ("cin", i32), ("ld0", i32), ("ld1", i32),
                ("h", i32), ("w", i32), ("ksize", i32), ("stride", i32), ("pad", i32), ("upsample", i32),
                ("gn_scale", vp), ("gn_shift", vp), ("silu", i32), ("pad_end", i32)]


class ConvArgs(C.Structure):
    _fields_ = [("batch", i32), ("ho", i32), ("wo", i32), ("cout", i32), ("nseg", i32), ("seg", ConvSrc * 2),
                ("weight", vp), ("k_total", i32), ("bias", vp), ("row_bias", vp), ("row_bias_ld", i32),
                ("residual", vp), ("res_ld", i32), ("out", vp), ("out_ld", i32), ("out_mode", i32),
                ("split_k", i32), ("workspace", vp), ("workspace_bytes", i64), ("variant_hint", i32),
                ("act", i32), ("gn_partial", vp), ("weight_batch_stride", i64), ("split_inlaunch", i32),
                ("tile_counters", vp), ("tile_group_m", i32)]


class ConvPlanInfo(C.Structure):
    _fields_ = [("split_k", i32), ("grid_tiles", i32), ("workspace_bytes", i64), ("variant", i32),
                ("flops", C.c_double), ("gn_chunks", i32)]


class GroupNormArgs(C.Structure):
    _fields_ = [("src0", vp), ("src1", vp), ("c_split", i32), ("ld0", i32), ("ld1", i32), ("batch", i32),
                ("hw", i32), ("channels", i32), ("groups", i32), ("eps", f32), ("gamma", vp), ("beta", vp),
                ("scale", vp), ("shift", vp), ("workspace", vp), ("workspace_bytes", i64)]


class AttentionArgs(C.Structure):
    _fields_ = [("q", vp), ("k", vp), ("v", vp), ("o", vp), ("q_ld", i32), ("k_ld", i32), ("v_ld", i32),
                ("o_ld", i32), ("batch", i32), ("heads", i32), ("nq", i32), ("nk", i32), ("head_dim", i32),
                ("scale", f32), ("causal", i32)]


class XAttnArgs(C.Structure):
    _fields_ = [("t", vp), ("kv", vp), ("wq", vp), ("wo", vp), ("bias", vp), ("res", vp), ("out", vp),
                ("t_ld", i32), ("kv_ld", i32), ("w_ld", i32), ("res_ld", i32), ("out_ld", i32), ("batch", i32),
                ("n_img", i32), ("nk", i32), ("channels", i32), ("head_dim", i32), ("scale", f32)]


class XAttnLnArgs(C.Structure):
    _fields_ = [("in_gamma", vp), ("in_beta", vp), ("in_eps", f32), ("out_gamma", vp), ("out_beta", vp),
                ("out_eps", f32), ("out_ln", vp), ("out_ln_ld", i32)]


class FfArgs(C.Structure):
    _fields_ = [("t", vp), ("res", vp), ("out", vp), ("packed", vp), ("b2", vp), ("t_ld", i32), ("res_ld", i32),
                ("out_ld", i32), ("rows", i32), ("channels", i32), ("features", i32)]


class TokenLinearArgs(C.Structure):
    _fields_ = [("x", vp), ("w", vp), ("bias", vp), ("res", vp), ("out", vp), ("x_ld", i32), ("res_ld", i32),
                ("out_ld", i32), ("rows", i32), ("in_features", i32), ("out_features", i32)]


class DdimArgs(C.Structure):
    _fields_ = [("x", vp), ("e", vp), ("e_uncond", vp), ("noise", vp), ("x_prev", vp), ("pred_x0", vp),
                ("n", i64), ("sqrt_one_minus_at", f32), ("sqrt_at", f32), ("dir_coef", f32), ("sqrt_a_prev", f32),
                ("sigma", f32), ("temperature", f32), ("guidance", f32), ("v_param", i32), ("v_sqrt_a", f32),
                ("v_sqrt_1ma", f32)]


OUT_NHWC_F16, OUT_NCHW_F32, OUT_GEGLU_F16, OUT_ROWS_F32 = 0, 1, 2, 3
ACT_NONE, ACT_QUICK_GELU = 0, 1

EXPORTS = ["sdk_conv2d_plan", "sdk_conv2d", "sdk_group_norm_workspace", "sdk_group_norm_affine", "sdk_group_norm_apply", "sdk_group_norm_apply_padded", "sdk_group_norm_apply_ex", "sdk_group_norm", "sdk_group_norm_finalize", "sdk_layer_norm",
           "sdk_attention", "sdk_cross_attention_block_supported", "sdk_xattn_pack_weight", "sdk_cross_attention_block", "sdk_cross_attention_block_ln", "sdk_segment_softmax", "sdk_ff_supported", "sdk_ff_packed_bytes", "sdk_ff_pack", "sdk_feed_forward", "sdk_token_linear_supported", "sdk_token_linear", "sdk_token_linear_ln", "sdk_ddim_step", "sdk_ddpm_step", "sdk_timestep_embedding", "sdk_nchw_to_nhwc",
           "sdk_diag_gaussian_sample", "sdk_stochastic_encode", "sdk_token_embedding", "sdk_extract_patches",
           "sdk_fold_patches", "sdk_upsample_bilinear2x", "sdk_upsample_nearest2x_padded", "sdk_gelu", "sdk_last_error", "sdk_version", "sdk_kernel_name",
           "sdk_probe_mfma_flops", "sdk_probe_mfma", "sdk_probe_copy", "sdk_probe_copy_ex"]

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"sd_amd: HIP library not built ({LIB_PATH} missing); run __graft_entry__.build()")
    # torch first: its HIP runtime (libamdhip64.so.7) is then the one this library binds to.  Loading
    # the library before torch pulls in a second runtime copy, and its first kernel launch reports
    # "no ROCm-capable device" once torch has initialised the GPU.
    import torch  # noqa: F401
    L = C.CDLL(LIB_PATH)
    L.sdk_conv2d_plan.argtypes = [C.POINTER(ConvArgs), C.POINTER(ConvPlanInfo)]
    L.sdk_conv2d.argtypes = [C.POINTER(ConvArgs), vp]
    L.sdk_group_norm_workspace.argtypes = [i32, i32, i32]
    L.sdk_group_norm_workspace.restype = i64
    L.sdk_group_norm_affine.argtypes = [C.POINTER(GroupNormArgs), vp]
    L.sdk_group_norm_apply.argtypes = [C.POINTER(GroupNormArgs), i32, vp, i32, vp]
    L.sdk_group_norm_apply_padded.argtypes = [C.POINTER(GroupNormArgs), i32, vp, i32, i32, i32, i32, vp]
    L.sdk_group_norm_apply_ex.argtypes = [C.POINTER(GroupNormArgs), i32, vp, i32, vp, i32, vp, i32, vp]
    L.sdk_group_norm.argtypes = [C.POINTER(GroupNormArgs), i32, vp, i32, i32, i32, i32, vp, i32, vp, i32, vp]
    L.sdk_group_norm_finalize.argtypes = [C.POINTER(GroupNormArgs), vp, i32, vp, i32, vp]
    L.sdk_upsample_bilinear2x.argtypes = [vp, vp, i32, i32, i32, i32, vp]
    L.sdk_upsample_nearest2x_padded.argtypes = [vp, i32, vp, i32, i32, i32, i32, i32, vp]
    L.sdk_gelu.argtypes = [vp, vp, i64, vp]
    L.sdk_layer_norm.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, f32, vp]
    L.sdk_attention.argtypes = [C.POINTER(AttentionArgs), vp]
    L.sdk_cross_attention_block_supported.argtypes = [i32, i32, i32, i32]
    L.sdk_xattn_pack_weight.argtypes = [vp, i32, vp, i32, vp]
    L.sdk_cross_attention_block.argtypes = [C.POINTER(XAttnArgs), vp]
    L.sdk_cross_attention_block_ln.argtypes = [C.POINTER(XAttnArgs), C.POINTER(XAttnLnArgs), vp]
    L.sdk_segment_softmax.argtypes = [vp, i32, vp, i32, i32, i32, i32, f32, vp]
    L.sdk_ff_supported.argtypes = [i32, i32]
    L.sdk_ff_packed_bytes.argtypes = [i32, i32]
    L.sdk_ff_packed_bytes.restype = i64
    L.sdk_ff_pack.argtypes = [vp, vp, vp, vp, i32, i32, vp]
    L.sdk_feed_forward.argtypes = [C.POINTER(FfArgs), vp]
    L.sdk_token_linear_supported.argtypes = [i32, i32]
    L.sdk_token_linear.argtypes = [C.POINTER(TokenLinearArgs), vp]
    L.sdk_token_linear_ln.argtypes = [C.POINTER(TokenLinearArgs), vp, vp, f32, vp, i32, vp]
    L.sdk_ddim_step.argtypes = [C.POINTER(DdimArgs), vp]
    L.sdk_ddpm_step.argtypes = [vp, vp, vp, vp, i64, f32, f32, f32, vp]
    L.sdk_timestep_embedding.argtypes = [vp, vp, vp, i32, i32, vp]
    L.sdk_nchw_to_nhwc.argtypes = [vp, vp, i32, i32, i32, i32, f32, vp]
    L.sdk_diag_gaussian_sample.argtypes = [vp, vp, vp, i32, i32, i32, f32, vp]
    L.sdk_stochastic_encode.argtypes = [vp, vp, vp, i64, f32, f32, vp]
    L.sdk_token_embedding.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp]
    L.sdk_extract_patches.argtypes = [vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]
    L.sdk_fold_patches.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp]
    L.sdk_probe_mfma_flops.argtypes = [i32, i32, i32]
    L.sdk_probe_mfma_flops.restype = C.c_double
    L.sdk_probe_mfma.argtypes = [i32, i32, i32, vp, vp, vp]
    L.sdk_probe_copy.argtypes = [vp, vp, i64, vp]
    L.sdk_probe_copy_ex.argtypes = [vp, vp, i64, i32, vp]
    L.sdk_last_error.restype = C.c_char_p
    L.sdk_kernel_name.restype = C.c_char_p
    L.sdk_kernel_name.argtypes = [i32]
    for name in EXPORTS:
        if not hasattr(L, name):
            raise RuntimeError(f"sd_amd: {LIB_PATH} does not export {name}")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().sdk_last_error().decode(errors="replace")
        raise RuntimeError(f"sd_amd.{what} failed ({rc}): {msg}")
