"""ctypes binding of the C-ABI library ``libmolclr_hip.so`` (include/molclr.h).

This is the only way the Python side reaches the GPU kernels.  Loading fails
loudly if the library has not been built (``python -m molclr_amd.build``);
there is no CPU or eager-PyTorch fallback for any op.

``torch`` is imported first on purpose: torch ships its own HIP runtime
(SONAME ``libamdhip64.so.7``) and the dynamic loader then resolves the
library's HIP dependency to that same runtime, so streams and device pointers
handed over from torch are valid in the kernels.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int64, c_size_t, c_uint64, c_void_p
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = Path(os.environ.get("MOLCLR_LIB", Path(__file__).resolve().parent / "libmolclr_hip.so"))

_P = c_void_p
_I64 = c_int64

# name -> (restype, argtypes); mirrors include/molclr.h exactly
SIGNATURES = {
    "molclr_version": (c_char_p, []),
    "molclr_last_error": (c_char_p, []),
    "molclr_graph_build_workspace_bytes": (c_size_t, [_I64, _I64]),
    "molclr_graph_build": (c_int, [_P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _P, _P, _P, c_size_t, _P]),
    "molclr_graph_build_multi": (c_int, [c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                         c_size_t, _P]),
    "molclr_stage_segments": (c_int, [c_int, _P, _P, _P, _I64, _I64, _P, _P]),
    "molclr_graph_build_dev": (c_int, [c_int, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P,
                                       _P, _P, _P, c_size_t, _P]),
    "molclr_mask_views_workspace_bytes": (c_size_t, [_I64]),
    "molclr_mask_views": (c_int, [_P, _P, _P, _P, _P, _I64, _I64, _P, _I64, c_uint64, c_int, _P, _P,
                                  _P, _P, _P, _I64, _I64, _P, _P, c_size_t, _P]),
    "molclr_atom_embed_fwd": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _P, _P]),
    "molclr_atom_embed_bwd_workspace_bytes": (c_size_t, [_I64, _I64, _I64, _I64]),
    "molclr_atom_embed_bwd": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, c_int, _P, c_size_t,
                                      _P]),
    "molclr_edge_tables_combine": (c_int, [c_int, _P, _P, _P, _I64, _P]),
    "molclr_gine_aggregate_fwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P]),
    "molclr_rowmax_layout": (_I64, [_I64]),
    "molclr_rowmax_bytes": (c_size_t, [_I64, _I64]),
    "molclr_gine_aggregate_fwd_rowmax": (c_int, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P, _P,
                                                 _P]),
    "molclr_gine_aggregate_bwd_workspace_bytes": (c_size_t, [_I64, _I64]),
    "molclr_gine_aggregate_bwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, c_int, _P,
                                          c_size_t, _P]),
    "molclr_gcn_aggregate_fwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P]),
    "molclr_gcn_aggregate_bwd_workspace_bytes": (c_size_t, [_I64, _I64]),
    "molclr_gcn_aggregate_bwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, c_int,
                                         _P, c_size_t, _P]),
    "molclr_gemm_f32_workspace_bytes": (c_size_t, [_I64, _I64, _I64]),
    "molclr_gemm_f32": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, c_int, c_int, c_int,
                                _P, _P, _I64, _P, c_size_t, _P]),
    "molclr_gemm_f32_impl": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, c_int, c_int,
                                     c_int, _P, _P, _I64, _P, c_size_t, _P, c_int]),
    "molclr_bplanes_bytes": (c_size_t, [_I64, _I64]),
    "molclr_bplanes_make": (c_int, [_P, _I64, _I64, _I64, c_int, _P, _P]),
    "molclr_bplanes_make_batch": (c_int, [c_int, _P, _P, _P, _P, _P, _P, _P]),
    "molclr_gemm_f32_bplanes": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, c_int, _P,
                                        _P, _I64, _P, c_size_t, _P]),
    "molclr_gemm_f32_bplanes_tile": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int,
                                             c_int, _P, _P, _I64, _P, c_size_t, _P, c_int]),
    "molclr_linear_wgrad_workspace_bytes": (c_size_t, [_I64, _I64, _I64]),
    "molclr_linear_wgrad": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P, c_size_t,
                                    _P]),
    "molclr_linear_wgrad_groups": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P,
                                           c_size_t, _P, c_int]),
    "molclr_absmax_f32": (c_int, [_P, _I64, _I64, _I64, _P, c_int, _P]),
    "molclr_hplanes_bytes": (c_size_t, [_I64, _I64]),
    "molclr_hplanes_make_batch": (c_int, [c_int, _P, _P, _P, _P, _P, _P, _P]),
    "molclr_absmax_rows_f32": (c_int, [_P, _I64, _I64, _I64, _P, _P, c_int, _P]),
    "molclr_bn_row_parts": (c_int, [_I64]),
    "molclr_batchnorm_seg_bwd_max": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P, _I64,
                                             c_int, c_int, _P, _P, _P, c_size_t, _P]),
    "molclr_gemm_row_parts": (_I64, [_I64]),
    "molclr_gemm_f32_bplanes_max": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P,
                                            _P, _I64, _P, _P, _P, _P, _P, c_size_t, _P]),
    "molclr_gemm_f32_h3": (c_int, [_P, _P, c_int, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P,
                                   _P, _I64, _P, _P, _P, _P, _P]),
    "molclr_gemm_f32_h3_bits": (c_int, [_P, _P, c_int, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int,
                                        _P, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "molclr_gemm_f32_h3_impl": (c_int, [_P, _P, c_int, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int,
                                        _P, _P, _I64, _P, _P, _P, _P, _P, _P, c_int]),
    "molclr_linear_wgrad_h3_groups": (c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64,
                                              c_int, _P, c_size_t, _P, c_int]),
    "molclr_linear_wgrad_h3": (c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int,
                                       _P, c_size_t, _P]),
    "molclr_colsum_f32_workspace_bytes": (c_size_t, [_I64, _I64]),
    "molclr_colsum_f32": (c_int, [_P, _P, _I64, _I64, _I64, c_int, _P, c_size_t, _P]),
    "molclr_batchnorm_workspace_bytes": (c_size_t, [_I64, _I64]),
    "molclr_batchnorm_fwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, c_double,
                                     c_double, c_int, c_int, _P, c_size_t, _P]),
    "molclr_batchnorm_bwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, c_int, c_int,
                                     _P, c_size_t, _P]),
    "molclr_batchnorm_seg_workspace_bytes": (c_size_t, [c_int, _P, _I64]),
    "molclr_batchnorm_seg_fwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P, _I64, c_int,
                                         c_double, c_double, c_int, c_int, _P, c_size_t, _P]),
    "molclr_batchnorm_seg_bwd": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P, _I64, c_int,
                                         c_int, c_int, _P, c_size_t, _P]),
    "molclr_batchnorm_seg_dev_workspace_bytes": (c_size_t, [c_int, _I64, _I64]),
    "molclr_batchnorm_seg_fwd_dev": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P, _I64,
                                             _I64, c_int, c_double, c_double, c_int, c_int, _P,
                                             c_size_t, _P]),
    "molclr_batchnorm_seg_bwd_dev": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, c_int, _P, _I64,
                                             _I64, c_int, c_int, c_int, _P, _P, _P, c_size_t, _P]),
    "molclr_segment_pool_fwd": (c_int, [_P, _P, _P, _I64, _I64, c_int, _P]),
    "molclr_segment_pool_bwd": (c_int, [_P, _P, _P, _I64, _I64, _I64, c_int, _P]),
    "molclr_l2norm_fwd": (c_int, [_P, _P, _P, _I64, _I64, c_double, _P]),
    "molclr_l2norm_bwd": (c_int, [_P, _P, _P, _P, _I64, _I64, c_double, _P]),
    "molclr_ntxent_prep": (c_int, [_P, _P, _P, _I64, _I64, c_int, _P]),
    "molclr_ntxent_prep_bwd": (c_int, [_P, _P, _P, _P, _I64, _I64, c_int, _P]),
    "molclr_ntxent_prep_pair": (c_int, [_P, _P, _P, _P, _P, _I64, _I64, c_double, c_int, _P]),
    "molclr_ntxent_prep_pair_bwd": (c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, c_double, c_int,
                                            _P]),
    "molclr_ntxent_workspace_bytes": (c_size_t, [_I64, _I64, _I64]),
    "molclr_ntxent_fwd": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, c_double, _P, _P, _P,
                                  c_size_t, _P]),
    "molclr_ntxent_bwd": (c_int, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, c_double, _P, _P,
                                  c_size_t, _P]),
    "molclr_ntxent_sim_bytes": (c_size_t, [_I64, _I64, _I64, c_int]),
    "molclr_ntxent_fwd_impl": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, c_double, _P, _P,
                                       _P, _P, c_size_t, _P, c_int]),
    "molclr_ntxent_bwd_impl": (c_int, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, c_double, _P,
                                       _P, _P, c_size_t, _P, c_int]),
    "molclr_sum_f32": (c_int, [_P, _P, _I64, _P]),
    "molclr_linear_wgrad_h3_pair_workspace_bytes": (c_size_t, [_I64, _I64, _I64, _I64, _I64]),
    "molclr_linear_wgrad_h3_pair": (c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64,
                                            _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64,
                                            _I64, c_int, _P, c_size_t, _P]),
    "molclr_adam_step": (c_int, [_P, _P, _P, _P, _I64, _P, _P, c_double, c_double, c_double,
                                 c_double, _P]),
    "molclr_adam_step_ex": (c_int, [_P, _P, _P, _P, _I64, _P, _P, c_double, c_double, c_double,
                                    c_double, c_int, _P]),
    "molclr_step_tail": (c_int, [_P, _P, _P, _P, _P, _P]),
    "molclr_gin_encoder_arena_bytes": (c_size_t, [c_int, _I64, _I64, c_int]),
    "molclr_gin_encoder_workspace_bytes": (c_size_t, [c_int, _I64, _I64, c_int]),
    "molclr_gin_encoder_fwd": (c_int, [_P, _P, _P, _P, _P, c_size_t, _P, c_size_t, _P]),
    "molclr_gin_encoder_bwd": (c_int, [_P, _P, _P, _P, _P, _P, c_size_t, _P, c_size_t, _P]),
    "molclr_gcn_encoder_arena_bytes": (c_size_t, [c_int, _I64, _I64]),
    "molclr_gcn_encoder_workspace_bytes": (c_size_t, [c_int, _I64, _I64]),
    "molclr_gcn_encoder_fwd": (c_int, [_P, _P, _P, _P, _P, c_size_t, _P, c_size_t, _P]),
    "molclr_gcn_encoder_bwd": (c_int, [_P, _P, _P, _P, _P, _P, c_size_t, _P, c_size_t, _P]),
    "molclr_aug_views_workspace_bytes": (c_size_t, [_I64, _I64, _I64]),
    "molclr_aug_views_plan": (c_int, [_P, _P, _P, _I64, _I64, _P, _I64, ctypes.c_uint64, c_int,
                                      c_int, _I64, _I64, _P, _P, _P, _P, c_size_t, _P]),
    "molclr_aug_views_big_workspace_bytes": (c_size_t, [_I64, _I64, _I64]),
    "molclr_aug_views_plan_big": (c_int, [_P, _P, _P, _I64, _I64, _P, _I64, ctypes.c_uint64,
                                          c_int, c_int, _I64, _I64, _P, _P, _P, _P, c_size_t,
                                          _I64, _I64, _I64, _P, c_size_t, _P]),
    "molclr_aug_views_write": (c_int, [_P, _P, _P, _P, _P, _I64, _I64, _P, _I64, _P, _I64, _I64,
                                       _I64, _P, _P, _P, _P, _P, c_size_t, _P]),
    "molclr_atom_embed_fwd_bf16": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _P, _P]),
    "molclr_atom_embed_bwd_bf16": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, c_int, _P,
                                           c_size_t, _P]),
    "molclr_gine_aggregate_fwd_bf16": (c_int, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P]),
    "molclr_gine_aggregate_bwd_bf16": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, c_int,
                                               _P, c_size_t, _P]),
    "molclr_segment_max_fwd": (c_int, [_P, _P, _P, _P, _I64, _I64, c_int, _P]),
    "molclr_segment_max_bwd": (c_int, [_P, _P, _P, _I64, _I64, _I64, c_int, _P]),
    "molclr_segment_pool_fwd_bf16": (c_int, [_P, _P, _P, _I64, _I64, c_int, _P]),
    "molclr_segment_pool_bwd_bf16": (c_int, [_P, _P, _P, _I64, _I64, _I64, c_int, _P]),
    "molclr_gemm_bf16": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P, _P, _I64,
                                 _P]),
    "molclr_gemm_bf16_bits": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P, _P, _P,
                                      _P]),
    "molclr_gemm_bf16_impl": (c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P, _P,
                                      _I64, _P, c_int]),
    "molclr_linear_wgrad_bf16_workspace_bytes": (c_size_t, [_I64, _I64, _I64]),
    "molclr_linear_wgrad_bf16_impl": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int,
                                              _P, c_size_t, _P, c_int]),
    "molclr_linear_wgrad_bf16": (c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, c_int, _P,
                                         c_size_t, _P]),
    "molclr_ktimer_start": (c_int, [c_int]),
    "molclr_ktimer_read": (c_int, [c_int, _P, _P]),
    "molclr_ktimer_stop": (c_int, []),
}

EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_MASK = 0, 1, 2, 3
EPI_ACCUMULATE = 16
NUM_ECOMB = 15  # combined edge-table rows (bond type * 3 + bond dir)
MAX_LAYERS = 16
MAX_SEGMENTS = 8
DTYPE_F32, DTYPE_BF16 = 0, 1
STATUS_ATOM_RANGE = 8  # MOLCLR_STATUS_ATOM_RANGE
KTIMER_GINE_AGG = 1
KTIMER_GEMM = 2
KTIMER_NTXENT = 4
KTIMER_GCN_AGG = 8
AUG_SUBGRAPH, AUG_MIX = 0, 1


_L16 = c_void_p * 16


class GinEncoder(ctypes.Structure):
    """struct molclr_gin_encoder (include/molclr.h)."""
    _fields_ = [("num_layer", ctypes.c_int32), ("training", ctypes.c_int32), ("dim", c_int64),
                ("n_atom", c_int64), ("n_chiral", c_int64), ("momentum", c_double),
                ("eps", c_double), ("x_embedding1", c_void_p), ("x_embedding2", c_void_p)] + [
        (f, _L16) for f in ("mlp0_weight", "mlp0_bias", "mlp2_weight", "mlp2_bias",
                            "edge_embedding1", "edge_embedding2", "bn_weight", "bn_bias",
                            "bn_running_mean", "bn_running_var", "bn_num_batches_tracked",
                            "mlp0_planes", "mlp0_planes_t", "mlp2_planes", "mlp2_planes_t")] + [
        ("dtype", ctypes.c_int32), ("fp32_gemm", ctypes.c_int32), ("status", c_void_p)]


class GinEncoderGrads(ctypes.Structure):
    """struct molclr_gin_encoder_grads."""
    _fields_ = [("x_embedding1", c_void_p), ("x_embedding2", c_void_p)] + [
        (f, _L16) for f in ("mlp0_weight", "mlp0_bias", "mlp2_weight", "mlp2_bias",
                            "edge_embedding1", "edge_embedding2", "bn_weight", "bn_bias")] + [
        ("layer_done", _L16), ("embed_done", c_void_p)]


class GcnEncoder(ctypes.Structure):
    """struct molclr_gcn_encoder (include/molclr.h)."""
    _fields_ = [("num_layer", ctypes.c_int32), ("training", ctypes.c_int32), ("dim", c_int64),
                ("n_atom", c_int64), ("n_chiral", c_int64), ("momentum", c_double),
                ("eps", c_double), ("x_embedding1", c_void_p), ("x_embedding2", c_void_p)] + [
        (f, _L16) for f in ("weight", "bias", "edge_embedding1", "edge_embedding2", "bn_weight",
                            "bn_bias", "bn_running_mean", "bn_running_var",
                            "bn_num_batches_tracked", "weight_planes", "weight_planes_t")] + [
        ("fp32_gemm", ctypes.c_int32), ("status", c_void_p)]


class GcnEncoderGrads(ctypes.Structure):
    """struct molclr_gcn_encoder_grads."""
    _fields_ = [("x_embedding1", c_void_p), ("x_embedding2", c_void_p)] + [
        (f, _L16) for f in ("weight", "bias", "edge_embedding1", "edge_embedding2", "bn_weight",
                            "bn_bias")] + [("layer_done", _L16), ("embed_done", c_void_p)]


class DeviceGraphC(ctypes.Structure):
    """struct molclr_device_graph."""
    _fields_ = [("num_nodes", c_int64), ("num_edges", c_int64), ("num_graphs", c_int64)] + [
        (f, c_void_p) for f in ("rowptr", "col", "rowptr_t", "col_t", "ecount", "graph_ptr",
                                "ecode", "nbr", "nbr_t")] + [
        ("num_segments", ctypes.c_int32), ("segment_nodes", c_int64 * 8),
        ("segment_nodes_dev", c_void_p)]


class GraphSegmentC(ctypes.Structure):
    """struct molclr_graph_segment."""
    _fields_ = [("edge_index", c_void_p), ("edge_attr", c_void_p), ("batch", c_void_p),
                ("num_nodes", c_int64), ("num_edges", c_int64), ("num_graphs", c_int64)]


class StageSourceC(ctypes.Structure):
    """struct molclr_stage_source."""
    _fields_ = [("x", c_void_p), ("edge_index", c_void_p), ("edge_attr", c_void_p),
                ("batch", c_void_p), ("num_nodes", c_int64), ("num_edges", c_int64)]


class StagedSegmentC(ctypes.Structure):
    """struct molclr_graph_staged_segment."""
    _fields_ = [("edge_index", c_void_p), ("edge_attr", c_void_p), ("batch", c_void_p),
                ("node_cap", c_int64), ("edge_cap", c_int64), ("num_graphs", c_int64)]


class MolclrError(RuntimeError):
    pass


_lib = None


def load() -> ctypes.CDLL:
    """Load and type the library (once).  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not found: the MolCLR HIP kernels are not built. "
            "Run `python -m molclr_amd.build` (hipcc, gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    return (load().molclr_last_error() or b"").decode()


# Dry run (graph_step.CapturedTrainStep, before a capture): every call is
# skipped, so a pass through the Python layer only allocates what it would
# use (notably the cached weight images) and launches nothing.
DRY_RUN = [False]


class dry_run:
    def __enter__(self):
        DRY_RUN[0] = True

    def __exit__(self, *exc):
        DRY_RUN[0] = False


def call(name: str, *args) -> None:
    """Call an int-returning entry point and raise on a non-zero status."""
    if DRY_RUN[0]:
        return
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise MolclrError(f"{name} failed (status {rc}): {last_error()}")


def query(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_of(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream
