"""ctypes binding of the rankops C ABI (include/rankops.h, include/rankops_io.h).

This is the reference-side FFI a maintainer adds next to the reference's `nn.Module`
bodies: plain device pointers, sizes and the current HIP stream go in, nothing torch-typed
crosses the boundary.  The shared library is `librankops.so`, built in-tree by
`csrc/Makefile` (hipcc, gfx950).  There is no fallback: if the library is missing or fails
to load, every rankops op raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int32, c_int64, c_uint32, c_void_p

import torch  # noqa: F401  -- must be loaded first: librankops binds to torch's HIP runtime

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RANKOPS_LIB", os.path.join(_HERE, "librankops.so"))

RK_OK = 0
RK_ERR_UNSUPPORTED = 4  # include/rankops.h
RK_FLAG_INDEX_OOB = 1
RK_ACT_NONE, RK_ACT_RELU, RK_ACT_LEAKY, RK_ACT_DICE, RK_ACT_PRELU = 0, 1, 2, 3, 4
RK_MAX_SEGMENTS = 64
ABI_VERSION = 1


class Segment(ctypes.Structure):
    _fields_ = [
        ("src", c_void_p),
        ("idx", c_void_p),
        ("idx_stride", c_int64),
        ("src_ld", c_int64),
        ("rows", c_int64),
        ("dim", c_int32),
        ("out_col", c_int32),
    ]


class Epilogue(ctypes.Structure):
    _fields_ = [
        ("bias", c_void_p),
        ("residual", c_void_p),
        ("ld_residual", c_int64),
        ("residual_periodic", c_void_p),
        ("residual_period", c_int32),
        ("pre_scale", c_void_p),
        ("pre_shift", c_void_p),
        ("act", c_int32),
        ("slope", c_float),
        ("act_scale", c_void_p),
        ("act_shift", c_void_p),
        ("act_alpha", c_void_p),
        ("act_alpha_len", c_int32),
        ("post_scale", c_void_p),
        ("post_shift", c_void_p),
        ("ln_gamma", c_void_p),
        ("ln_beta", c_void_p),
        ("ln_eps", c_float),
        ("has_ln", c_int32),
        ("pool_out", c_void_p),
        ("ld_pool", c_int64),
        ("pool_rows", c_int32),
        ("pool_mean", c_int32),
        ("pool_len", c_void_p),
        ("head_w", c_void_p),
        ("head_b", c_void_p),
        ("head_partial", c_void_p),
        ("fm1", c_void_p),
        ("fm2", c_void_p),
        ("final_w", c_void_p),
        ("final_b", c_void_p),
        ("head_logit", c_void_p),
        ("head_prob", c_void_p),
        ("head_aux", c_void_p),
    ]


class MlpLayer(ctypes.Structure):
    _fields_ = [
        ("w", c_void_p),
        ("ldw", c_int64),
        ("n", c_int32),
        ("act", c_int32),
        ("slope", c_float),
        ("residual", c_int32),
        ("bias", c_void_p),
        ("pre_scale", c_void_p),
        ("pre_shift", c_void_p),
        ("act_scale", c_void_p),
        ("act_shift", c_void_p),
        ("act_alpha", c_void_p),
        ("act_alpha_len", c_int32),
        ("post_scale", c_void_p),
        ("post_shift", c_void_p),
        ("store", c_void_p),
        ("ld_store", c_int64),
    ]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("numel", c_int64), ("step", c_void_p)]


RK_MLP_MAX_LAYERS = 8
_SEG_P = POINTER(Segment)
_EPI_P = POINTER(Epilogue)
_MLP_P = POINTER(MlpLayer)

# name -> (restype, argtypes); the exact set declared in include/*.h
SIGNATURES = {
    "rk_abi_version": (c_int32, []),
    "rk_build_info": (c_char_p, []),
    "rk_last_error": (c_char_p, []),
    "rk_init": (ctypes.c_int, [c_int32]),
    "rk_error_flags": (ctypes.c_int, [c_int32, POINTER(c_uint32), c_int32]),
    "rk_concat_gather": (ctypes.c_int, [_SEG_P, c_int32, c_int64, c_void_p, c_int64, c_void_p]),
    "rk_dcn_cross": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int64, c_void_p,
         c_int64, c_void_p, c_int64, c_void_p, c_void_p],
    ),
    "rk_dcn_forward": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, _MLP_P, c_int32, _EPI_P, c_void_p],
    ),
    "rk_fm_gather": (
        ctypes.c_int,
        [_SEG_P, _SEG_P, c_int32, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p],
    ),
    "rk_fm_pack_table": (
        ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_void_p]),
    "rk_fm_gather_packed": (
        ctypes.c_int, [_SEG_P, c_int32, c_int32, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "rk_din_attention": (
        ctypes.c_int,
        [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_void_p],
    ),
    "rk_row_l2norm_mean": (
        ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p]),
    "rk_afm_forward": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int32, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
         c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "rk_din_attention_dense": (
        ctypes.c_int,
        [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_int32,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_void_p],
    ),
    "rk_dice_forward": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int64, c_void_p]),
    "rk_bst_attention": (
        ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_int64, c_void_p]),
    "rk_bst_attention_masked": (
        ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_int32, c_void_p, c_int64, c_void_p, c_int64,
                       c_void_p]),
    "rk_bst_small_forward": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32,
         c_int32, POINTER(c_void_p), POINTER(ctypes.c_float), c_int32, _MLP_P, c_int32, _EPI_P, c_void_p]),
    "rk_bst_forward_blocks": (
        ctypes.c_int,
        [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, c_int32, c_int32,
         POINTER(c_void_p), POINTER(ctypes.c_float), c_void_p, c_int64, c_int32, c_void_p]),
    "rk_bst_forward_blocks_packed": (
        ctypes.c_int,
        [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, c_int32, c_int32,
         POINTER(c_void_p), POINTER(ctypes.c_float), c_void_p, c_int64, c_int32, c_void_p]),
    "rk_bst_pack_block_weight": (ctypes.c_int, [c_void_p, c_void_p, c_void_p]),
    "rk_linear": (
        ctypes.c_int,
        [c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_int64, c_int64, c_int32, c_int32, _EPI_P, c_void_p,
         c_int64, c_void_p],
    ),
    "rk_din_forward": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int32, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32,
         c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, _MLP_P,
         c_int32, _EPI_P, c_int32, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_din_forward_ex": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int32, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32,
         c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, _MLP_P,
         c_int32, _EPI_P, c_int32, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_din_forward_plan": (
        ctypes.c_int,
        [_SEG_P, c_int32, c_int32, c_int32, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32,
         c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, _MLP_P,
         c_int32, _EPI_P, c_int32, c_float, c_void_p, c_void_p, c_void_p, POINTER(c_void_p)]),
    "rk_din_plan_launch": (ctypes.c_int, [c_void_p, c_void_p]),
    "rk_din_plan_set_epilogue_image": (ctypes.c_int, [c_void_p, c_void_p]),
    "rk_mlp_epilogue_image_floats": (ctypes.c_int, [_MLP_P, c_int32, c_int32]),
    "rk_mlp_pack_epilogue": (ctypes.c_int, [_MLP_P, c_int32, c_int32, c_void_p, c_void_p]),
    "rk_din_plan_destroy": (None, [c_void_p]),
    "rk_din_attention_image_floats": (c_int64, [c_int32]),
    "rk_din_pack_attention": (
        ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "rk_mlp_packed_size": (ctypes.c_int, [c_int32, c_int32, POINTER(c_int64), POINTER(c_int64)]),
    "rk_mlp_pack_weight": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p]),
    "rk_mlp_forward": (
        ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, _MLP_P, c_int32, _EPI_P, c_void_p, c_int64, c_void_p]),
    "rk_mlp_forward_gather": (ctypes.c_int, [POINTER(Segment), ctypes.c_int32, ctypes.c_int32, c_int64, _MLP_P,
                                             ctypes.c_int32, _EPI_P, c_void_p]),
    "rk_fwfm_forward": (ctypes.c_int, [POINTER(Segment), POINTER(Segment), ctypes.c_int32, ctypes.c_int32, c_int64,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_gemm": (ctypes.c_int, [c_int32, c_int32, c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                               c_int64, c_void_p, c_int64, c_void_p, c_int32, c_int32, c_void_p]),
    "rk_logit_head_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int32,
                                              c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int64, c_void_p,
                                              c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_rng_next": (ctypes.c_int, [c_void_p, c_void_p, c_void_p]),
    "rk_dropout_mask": (ctypes.c_int, [ctypes.c_uint64, c_void_p, c_int64, c_int32, ctypes.c_double, c_void_p,
                                       c_void_p]),
    "rk_bn_act_train_forward": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int32, c_void_p,
                                               c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_int32, c_float, ctypes.c_double, ctypes.c_uint64, c_void_p,
                                               c_void_p, c_int64, c_void_p]),
    "rk_bn_act_backward": (ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int32,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_float, ctypes.c_double,
                                          ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                          c_void_p]),
    "rk_fm_backward": (ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int32, c_int32,
                                      c_void_p, c_int64, c_void_p]),
    "rk_fm_combine_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p]),
    "rk_dice_train_forward": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_float,
                                             c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_int64, c_void_p]),
    "rk_dice_backward": (ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "rk_prelu_train_forward": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_int32,
                                              c_void_p, c_int64, c_void_p]),
    "rk_prelu_backward": (ctypes.c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p,
                                         c_int32, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "rk_din_att_cross": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64,
                                        c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "rk_din_att_pool_forward": (ctypes.c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                               c_int32, c_int32, c_int32, c_void_p, c_void_p, c_int64, c_int32,
                                               c_void_p]),
    "rk_din_att_pool_backward": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                                c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p,
                                                c_void_p, c_void_p]),
    "rk_din_cross_fold": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int64, c_int32, c_int32,
                                         c_void_p, c_void_p, c_int64, c_void_p]),
    "rk_row_l2norm_backward": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_float, c_void_p,
                                              c_void_p, c_int64, c_void_p]),
    "rk_fwfm_backward": (ctypes.c_int, [POINTER(Segment), ctypes.c_int32, ctypes.c_int32, c_int64, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_afm_pairs": (ctypes.c_int, [POINTER(Segment), c_int32, c_int32, c_int64, c_void_p, c_void_p, c_void_p]),
    "rk_afm_pool_forward": (ctypes.c_int, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                                           c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_afm_pool_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_int32, c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int64,
                                            c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_afm_pair_fold": (ctypes.c_int, [c_void_p, c_void_p, c_int32, c_int32, c_int64, c_void_p, c_void_p]),
    "rk_bst_add_pos": (ctypes.c_int, [c_void_p, c_void_p, c_int32, c_int64, c_int32, c_void_p, c_void_p]),
    "rk_bst_attn_train_forward": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                                 c_void_p, c_void_p]),
    "rk_bst_attn_train_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32,
                                                  c_void_p, c_void_p]),
    "rk_linear_res_dropout_ln": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int64, c_void_p,
                                                c_void_p, ctypes.c_double, ctypes.c_uint64, c_void_p, c_void_p,
                                                c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_bst_res_dropout_ln_forward": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_int32, ctypes.c_double,
                                                     ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                                                     c_void_p, c_void_p, c_void_p, c_void_p]),
    "rk_bst_ln_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32,
                                          ctypes.c_double, ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_int64, c_void_p]),
    "rk_bst_pool_ln_backward": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_int32, c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_int64, c_int32, ctypes.c_double,
                                               ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_int64, c_void_p]),
    "rk_bst_ln_backward_workspace_floats": (c_int64, [c_int32]),
    "rk_bst_gather_pos": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32, c_int32, c_void_p,
                                         c_void_p, c_void_p, c_void_p]),
    "rk_embedding_backward_seq": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_void_p, c_int64, c_void_p]),
    "rk_gemm_wgrad": (ctypes.c_int, [c_int64, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                                     c_void_p, c_int64, c_void_p, c_int32, c_void_p, c_int64, c_void_p]),
    "rk_gemm_wgrad_workspace_floats": (c_int64, [c_int64, c_int64, c_int64]),
    "rk_bst_pos_backward": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p]),
    "rk_bst_leaky_dropout": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_float, ctypes.c_double, ctypes.c_uint64,
                                            c_void_p, c_int32, c_void_p, c_void_p]),
    "rk_bst_pool": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_int32, c_void_p, c_int64, c_int32,
                                   c_void_p]),
    "rk_bst_pool_backward": (ctypes.c_int, [c_void_p, c_int64, c_int32, c_int64, c_int32, c_int32, c_void_p, c_int32,
                                            c_void_p, c_void_p]),
    "rk_embedding_backward_sorted_workspace_size": (ctypes.c_int, [c_int64, POINTER(c_int64)]),
    "rk_embedding_backward_sorted": (ctypes.c_int, [POINTER(Segment), c_int64, c_void_p, c_int64, c_void_p, c_int64,
                                                    c_void_p]),
    "rk_relu_backward": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int32, c_void_p]),
    "rk_dcn_cross_backward": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p, c_int32,
                                             c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p]),
    "rk_embedding_backward": (ctypes.c_int, [_SEG_P, c_int32, c_int64, c_void_p, c_int64, c_void_p]),
    "rk_adam_step": (ctypes.c_int, [POINTER(AdamTensor), c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double, c_int64, c_void_p]),
    "rk_eval_batch": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int64, ctypes.c_int32, c_void_p, c_void_p, c_void_p]),
    "rk_auc_workspace_size": (ctypes.c_int, [c_int64, POINTER(c_int64)]),
    "rk_auc": (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "rk_linear_tiled": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, _MLP_P, c_void_p, c_int64, c_void_p]),
    "rk_shard_pack_indices": (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_void_p, c_void_p]),
    "rk_shard_gather_rows": (ctypes.c_int, [_SEG_P, c_int32, c_int32, c_void_p, c_int32, c_int64, c_int64, c_int64,
                                            c_void_p, c_void_p]),
    "rk_fm_linear_packed": (ctypes.c_int, [_SEG_P, c_int32, c_int32, c_int64, _MLP_P, c_void_p, c_int64, c_void_p,
                                           c_void_p, c_void_p]),
    "rk_deepfm_forward": (ctypes.c_int, [_SEG_P, c_int32, c_int32, c_int64, _MLP_P, c_int32, _EPI_P, c_void_p,
                                         c_void_p, c_void_p]),
    "rk_deepfm_forward_fo": (ctypes.c_int, [_SEG_P, c_void_p, c_void_p, c_int32, c_int32, c_int64, _MLP_P, c_int32,
                                            _EPI_P, c_void_p, c_void_p, c_void_p]),
    "rk_shard_gather_rows_split": (ctypes.c_int, [_SEG_P, _SEG_P, c_int32, c_int32, c_void_p, c_int32, c_int64,
                                                  c_int64, c_int64, c_void_p, c_void_p]),
    "rk_bn_fold": (
        ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int32, c_void_p, c_void_p, c_void_p]),
    # include/rankops_io.h (host input path)
    "rk_vocab_load": (c_void_p, [c_char_p, c_int32]),
    "rk_vocab_parse": (c_void_p, [c_char_p, c_int64, c_int32]),
    "rk_vocab_size": (c_int64, [c_void_p]),
    "rk_vocab_free": (None, [c_void_p]),
    "rk_bucketize": (
        ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int32]),
    "rk_label_encode": (
        ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int64, c_void_p, POINTER(c_int64),
                       c_int32]),
    "rk_sequence_lengths": (
        ctypes.c_int,
        [c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int64, ctypes.c_char, c_void_p, POINTER(c_int64), c_int32]),
    "rk_bucketize_sequences": (
        ctypes.c_int,
        [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int64, ctypes.c_char, c_int64, c_void_p, c_int64,
         c_void_p, c_int32]),
    "rk_vocab_export_size": (ctypes.c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(ctypes.c_uint64)]),
    "rk_vocab_export": (ctypes.c_int, [c_void_p, c_void_p, c_void_p]),
    "rk_bucketize_device": (
        ctypes.c_int,
        [c_void_p, ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int64, c_void_p,
         c_int64, c_void_p]),
    "rk_bucketize_sequences_device": (
        ctypes.c_int,
        [c_void_p, ctypes.c_uint64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int64, ctypes.c_char,
         c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
}

_lib = None
_load_error = None
_initialised = set()


class RankOpsError(RuntimeError):
    pass


def _hip_runtimes_mapped():
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return paths


def load():
    """Loads librankops.so (once) and declares every C-ABI prototype."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise RankOpsError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"rankops: native library not found at {LIB_PATH}; build it with "
                       f"`make -C csrc` or __graft_entry__.build()")
        raise RankOpsError(_load_error)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rk_abi_version() != ABI_VERSION:
        raise RankOpsError(f"rankops: ABI mismatch ({lib.rk_abi_version()} != {ABI_VERSION})")
    runtimes = _hip_runtimes_mapped()
    if len(runtimes) > 1:
        raise RankOpsError(f"rankops: two HIP runtimes mapped in one process: {sorted(runtimes)}")
    _lib = lib
    return lib


def build_info() -> dict:
    """The loaded library's provenance (rk_build_info): {"src": hash of the sources it was built
    from, "arch", "extra": extra compile flags (timing builds)}, plus "path" and "tree_src" (the
    same hash over the csrc/ and include/ files next to this package; None without them)."""
    d = dict(kv.split("=", 1) for kv in load().rk_build_info().decode().split())
    d["path"] = LIB_PATH
    d["tree_src"] = tree_source_hash()
    return d


def tree_source_hash():
    """sha256[:16] over csrc/{*.hip,*.h,*.cpp} (name order) + include/rankops.h + rankops_io.h,
    as the Makefile computes SRC_HASH."""
    import hashlib
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(os.path.dirname(here), "csrc")
    inc = os.path.join(os.path.dirname(os.path.dirname(here)), "include")
    if not os.path.isdir(csrc) or not os.path.isdir(inc):
        return None
    h = hashlib.sha256()
    names = sorted(n for n in os.listdir(csrc) if os.path.splitext(n)[1] in (".hip", ".h", ".cpp"))
    for path in [os.path.join(csrc, n) for n in names] + [os.path.join(inc, n) for n in ("rankops.h", "rankops_io.h")]:
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def last_error() -> str:
    return load().rk_last_error().decode(errors="replace")


def check(rc: int, what: str):
    if rc != RK_OK:
        err = RankOpsError(f"{what} failed (code {rc}): {last_error()}")
        err.code = rc
        raise err


def ensure_device(device: torch.device):
    """Initialises the library's per-device state (flag word) once per device."""
    lib = load()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _initialised:
        check(lib.rk_init(idx), "rk_init")
        _initialised.add(idx)
    return idx


def error_flags(device=None, reset=True) -> int:
    """Reads the device flag word (synchronises).  Bit 0: an embedding index was out of range."""
    lib = load()
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    idx = ensure_device(dev)
    out = c_uint32(0)
    check(lib.rk_error_flags(idx, ctypes.byref(out), 1 if reset else 0), "rk_error_flags")
    return int(out.value)


_RAW_STREAM = torch._C._cuda_getCurrentRawStream  # the current stream's handle, without a Stream object


def raw_stream(device) -> int:
    """The current HIP stream of `device` (torch.device or index) as an integer handle: the value
    torch.cuda.current_stream(device).cuda_stream returns, at a fraction of its host cost."""
    if isinstance(device, str):
        device = torch.device(device)
    if isinstance(device, torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
    else:
        idx = torch.cuda.current_device() if device is None else int(device)
    return _RAW_STREAM(idx)


def stream_of(t: torch.Tensor) -> int:
    return _RAW_STREAM(t.get_device())


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def fptr(t: torch.Tensor, offset_elems: int = 0):
    return t.data_ptr() + offset_elems * t.element_size()
