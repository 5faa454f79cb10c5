"""ctypes binding of ``libsrml_ops.so`` (the hand-written gfx950 kernels).

Every kernel entry point is ``extern "C"`` and takes raw device pointers plus the HIP stream
torch is currently using, so launches are ordered with torch's own work and can be captured
into a HIP graph by ``torch.cuda.graph``. A non-zero return is a launch error and raises.

Policy: when a tensor lives on a GPU the native kernel MUST run — if the library is missing
or fails to load the op raises (no silent fallback to a PyTorch implementation). CPU tensors
(GPU-less CI) use the reference PyTorch implementations in ``ops/__init__.py``.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Any, Dict, Optional, Tuple

import torch

from . import build as _build

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_D = ctypes.c_double
_F = ctypes.c_float

# name -> argtypes (restype: int status, except the size queries in _LONG_RESULT)
_LONG_RESULT = ("srml_rf_bootstrap_ws", "srml_logreg_fold_ws", "srml_qn_mb_scratch", "srml_qn_fused_scratch",
                "srml_qn_fused_barrier_offset",
                "srml_logreg_fold_parts", "srml_qn_args_size", "srml_logit_residual_ws", "srml_xtv_mfma_ws",
                "srml_rf_partition_ws", "srml_dbscan_labels_ws", "srml_umap_categorical_ws",
                "srml_label_sort_ws", "srml_radix_sort_ws", "srml_lloyd_moved_ws", "srml_sum_f32_ws", "srml_sum_sq_ws")
SIGNATURES: Dict[str, Tuple[Any, ...]] = {
    "srml_col_moments_f32": (_P, _L, _I, _L, _P, _P, _P),
    "srml_col_moments_f64": (_P, _L, _I, _L, _P, _P, _P),
    "srml_standardize_f32": (_P, _L, _I, _L, _P, _P, _P),
    "srml_gram_f32": (_P, _L, _I, _L, _P, _P, _P),
    "srml_gram_f32_ex": (_P, _L, _I, _L, _P, _P, _P, _I, _P),
    "srml_mirror_upper_f64": (_P, _I, _P),
    "srml_xw_f32": (_P, _L, _I, _L, _P, _I, _P, _P, _L, _P),
    "srml_dgemm": (_I, _I, _I, _I, _I, _D, _P, _L, _P, _L, _D, _P, _L, _P),
    "srml_dgemm_splitk": (_I, _I, _I, _I, _I, _D, _P, _L, _P, _L, _D, _P, _L, _I, _P, _P),
    "srml_sign_flip_f64": (_P, _I, _I, _L, _P),
    "srml_xtv_f32": (_P, _L, _I, _L, _P, _I, _L, _P, _P),
    "srml_row_sqnorm_f32": (_P, _L, _I, _L, _P, _P),
    "srml_logreg_binary_f32": (_P, _L, _I, _L, _P, _P, _D, _P, _P),
    "srml_logreg_binary2_f32": (_P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P),
    "srml_logreg_binary3_f32": (_P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P, _I, _P),
    "srml_logreg_binary4_f32": (_P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P, _I, _P, _P, _P, _P),
    "srml_logreg_fold_parts": (_L,),
    "srml_logreg_fold_ws": (_L, _I, _L, _P),
    "srml_logreg_zcache_ok": (_L, _I, _L, _P),
    "srml_logreg_binary_lds_f32": (_P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P),
    "srml_logreg_binary_lds_f64": (_P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P),
    "srml_xtv2_f32": (_P, _L, _I, _L, _P, _I, _L, _P, _L, _L, _P, _P),
    "srml_xtv_mfma_f32": (_P, _L, _I, _L, _P, _I, _L, _P, _L, _L, _P, _P),
    "srml_xtv_mfma_det_f32": (_P, _L, _I, _L, _P, _I, _L, _P, _L, _L, _P, _P, _P),
    "srml_fold_partials_f64": (_P, _L, _L, _L, _L, _P, _L, _L, _P, _P),
    "srml_xw_t_f32": (_P, _L, _I, _L, _P, _I, _L, _P, _P, _L, _P),
    "srml_xw_t_f32_skip": (_P, _L, _I, _L, _P, _I, _L, _P, _P, _L, _P, _P),
    "srml_xw_t_f32_variant": (_P, _L, _I, _L, _P, _I, _L, _P, _P, _L, _I, _P),
    "srml_logit_residual_f32": (_P, _L, _I, _L, _P, _P, _L, _I, _P, _L, _P, _L, _P, _L, _P, _P),
    "srml_logit_residual_zc_f32": (_P, _L, _I, _L, _P, _P, _L, _I, _P, _L, _P, _L, _P, _L, _P, _P, _P, _P, _P),
    "srml_logit_residual_f64": (_P, _L, _I, _L, _P, _P, _L, _I, _P, _L, _P, _L, _P, _L, _P, _P),
    "srml_logit_residual_det_f32": (_P, _L, _I, _L, _P, _P, _L, _I, _P, _L, _P, _L, _P, _L, _P, _P, _P),
    "srml_logit_residual_ws": (_L, _I),
    "srml_xtv_mfma_ws": (_L, _I, _I),
    "srml_mbin_f32": (_P, _L, _I, _L, _P, _P, _L, _I, _P, _L, _P),
    "srml_qn_step_batch": (_P, _I, _P),
    "srml_mlogit_f32": (_P, _L, _I, _L, _P, _P, _P, _P, _I, _P, _P),
    "srml_mlogit_supported": (_I, _I),
    "srml_qn_step": (_P, _P),
    "srml_qn_step_mb": (_P, _P, _P),
    "srml_qn_step_fused": (_P, _P, _P, _I, _L, _P),
    "srml_qn_step_mbf": (_P, _P, _P, _I, _L, _P),
    "srml_kmeans_lloyd_small": (_P, _L, _I, _L, _P, _I, _P, _P, _P, _P, _P, _P, _P),
    "srml_kmeans_lloyd_mfma": (_P, _L, _I, _L, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P),
    "srml_kmeans_small_update": (_P, _I, _I, _P, _P, _P, _D, _P, _P, _P, _P),
    "srml_qn_fused_scratch": (),
    "srml_qn_fused_barrier_offset": (),
    "srml_qn_fused_resident": (_L,),
    "srml_qn_mb_scratch": (),
    "srml_kmeanspp_gram": (_P, _I, _L, _P, _I, _I, ctypes.c_ulonglong, _P, _P),
    "srml_qn_max_history": (),
    "srml_qn_args_size": (),
    "srml_nearest_centroid_f32": (_P, _L, _I, _L, _P, _I, _L, _P, _P, _P),
    "srml_nn_finalize": (_P, _L, _P, _P, _P, _P),
    "srml_split_bf16x3": (_P, _L, _I, _L, _I, _L, _P, _P),
    "srml_nearest_centroid_split": (_P, _L, _L, _I, _P, _I, _L, _P, _P, _P),
    "srml_split_bf16x3_tiled": (_P, _L, _I, _L, _I, _L, _P, _P),
    "srml_nearest_centroid_split_tiled": (_P, _L, _L, _I, _P, _I, _L, _P, _P, _P),
    "srml_nearest_centroid_split_tiled_np": (_P, _L, _L, _I, _P, _I, _L, _P, _P, _I, _P),
    "srml_nearest_centroid_split_top2": (_P, _L, _L, _I, _P, _I, _L, _P, _P, _P, _P, _P, _P),
    "srml_split_bf16x3_tiled_centered": (_P, _L, _I, _L, _P, _I, _L, _P, _P),
    "srml_split_bf16x3_tiled_centered_rows": (_P, _L, _P, _L, _I, _P, _I, _L, _P, _P),
    "srml_row_sqnorm_centered_f32": (_P, _L, _I, _L, _P, _P, _P),
    "srml_row_sqnorm_centered_amax_f32": (_P, _L, _I, _L, _P, _P, _P, _P),
    "srml_rf_sample_features_floyd": (_I, _I),
    "srml_rf_bootstrap_ws": (_I, _L),
    "srml_rf_bootstrap": (_I, _L, _D, ctypes.c_ulonglong, _P, _P, _P, _P, _P),
    "srml_split_f16_tiled_centered": (_P, _L, _I, _L, _P, _I, _L, _F, _P, _P, _P),
    "srml_nearest_centroid_f16_top2": (_P, _L, _L, _I, _P, _I, _L, _P, _P, _P, _F, _F, _P, _P, _P),
    "srml_nearest_centroid_f16_top2_nslot": (_I,),
    "srml_split_top2_select_f16": (_P, _P, _L, _I, _P, _P, _F, _F, _F, _P, _P, _P, _P, _P, _P),
    "srml_split_f16_tiled_centered_rows": (_P, _L, _P, _L, _I, _P, _I, _L, _F, _P, _P, _P),
    "srml_f16_plane_gather_rows": (_P, _L, _I, _P, _L, _L, _P, _P),
    "srml_nearest_f16_rowloop": (_P, _L, _L, _I, _P, _I, _L, _P, _F, _P, _P),
    "srml_f16_plane_gather_rows_ex": (_P, _L, _I, _P, _L, _L, _P, _P, _P, _P, _P),
    "srml_split_top2_select_f16_thr": (_P, _P, _L, _I, _P, _P, _F, _F, _F, _P, _P, _P, _P, _P, _P, _P),
    "srml_nearest_centroid_f16_cand": (_P, _L, _L, _I, _P, _I, _L, _P, _P, _P, _F, _F, _P, _P, _P, _I, _P),
    "srml_kmeans_cand_exact": (_P, _L, _P, _P, _L, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P),
    "srml_nearest_centroid_split_top2_nslot": (_I,),
    "srml_split_top2_select": (_P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P),
    "srml_split_scatter_refined": (_P, _P, _I, _P, _P, _P, _P),
    "srml_kmeans_accumulate_f32": (_P, _L, _I, _L, _P, _I, _P, _P, _P, _P),
    "srml_kmeans_accumulate_sorted_f32": (_P, _L, _I, _L, _P, _P, _P, _P),
    "srml_kmeans_accumulate_sorted_rows_f32": (_P, _L, _I, _L, _P, _P, _P, _P, _P),
    "srml_lloyd_moved_ws": (_L,),
    "srml_lloyd_moved_count": (_P, _P, _L, _P, _P, _P),
    "srml_lloyd_moved_compact": (_P, _P, _L, _P, _L, _P, _P, _P, _P),
    "srml_counts_from_offsets": (_P, _I, _P, _P),
    "srml_sum_f32_ws": (),
    "srml_sum_f32_f64": (_P, _L, _P, _P, _P),
    "srml_lloyd_centre_update": (_P, _I, _I, _P, _P, _P, _P),
    "srml_kmeans_segment_sums_f32": (_P, _L, _I, _L, _P, _P, _I, _P, _I, _P, _P),
    "srml_kmeans_segment_sums_f64": (_P, _L, _I, _L, _P, _P, _I, _P, _I, _P, _P),
    "srml_nearest_centroid_f64": (_P, _L, _I, _L, _P, _I, _L, _P, _P, _P, _P, _P, _P),
    "srml_row_sqnorm_f64": (_P, _L, _I, _L, _P, _P),
    "srml_knn_dist_f32": (_P, _L, _I, _L, _P, _L, _L, _P, _P, _L, _P),
    "srml_topk_rows_f32": (_P, _L, _L, _L, _I, _P, _L, ctypes.c_longlong, _I, _P, _P, _L, _L, _P),
    "srml_knn_f32": (_P, _L, _I, _L, _P, _L, _L, _P, _I, _I, _P, _P, ctypes.c_longlong, _P),
    "srml_ivf_search_f32": (_P, _L, _I, _L, _P, _I, _P, _P, _L, _P, _P, _I, _P, _P, _P),
    "srml_knn_lists_f32": (_P, _I, _L, _P, _P, _P, _I, _P, _P, _I, _I, _P, _P, _P),
    "srml_f16_centre_prep": (_P, _I, _I, _I, _P, _F, _I, _P, _P, _P, _P, _P),
    "srml_knn_lists_f16c": (_P, _I, _L, _P, _P, _P, _I, _P, _P, _I, _I, _P, _P, _P),
    "srml_knn_pairs_f16c": (_P, _I, _L, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P),
    "srml_center_rows_f16": (_P, _I, _L, _P, _P, _I, _L, _P, _P, _P),
    "srml_dbscan_degree_f32": (_P, _L, _I, _L, _P, _F, _L, _L, _P, _P),
    "srml_dbscan_link_f32": (_P, _L, _I, _L, _P, _F, _L, _L, _P, _P, _P, _P),
    "srml_uf_unite_pairs": (_P, _L, _P, _P),
    "srml_uf_compress": (_P, _L, _P),
    "srml_dbscan_labels_ws": (_L,),
    "srml_umap_categorical_ws": (_L, _L),
    "srml_umap_categorical": (_P, _P, _P, _L, _P, _L, _D, _D, _D, _P, _P, _P),
    "srml_dbscan_labels": (_P, _P, _P, _L, _P, _P, _P),
    "srml_oneshot_alloc": (_L, _P, _P),
    "srml_oneshot_open": (_P, _P),
    "srml_oneshot_close": (_P,),
    "srml_oneshot_free": (_P,),
    "srml_oneshot_allreduce": (_P, _P, _L, _I, _P, _I, _I, ctypes.c_ulonglong, _L, ctypes.c_longlong, _P, _P),
    "srml_umap_smooth_knn": (_P, _P, _L, _I, _L, _D, _D, _I, _P, _I, _P, _P, _P, _P),
    "srml_umap_fuzzy_union_knn": (_P, _P, _L, _I, _L, ctypes.c_float, _P, _P, _P, _P),
    "srml_umap_epoch": (_P, _P, _L, _P, _P, _P, _P, _P, _P, _I, _I, _F, _F, _F, _F, _F, _I, _I, ctypes.c_uint, _P, _P,
                        _I, _P),
    "srml_umap_neg_table": (_P, _P, _L, _I, _P, _P),
    "srml_syevj_f64": (_P, _I, _P, _P, _I, _D, _P),
    "srml_potrf_f64": (_P, _I, _L, _P, _P),
    "srml_potrs_f64": (_P, _I, _L, _P, _P),
    "srml_potrs_backward_f64": (_P, _I, _L, _P, _P),
    "srml_cd_gram_f64": (_P, _I, _L, _P, _P, _P, _P, _I, _D, _P, _P),
    "srml_rf_quantize_u8": (_P, _L, _I, _L, _P, _I, _P, _P),
    "srml_rf_quantize_u8_ld": (_P, _L, _I, _L, _P, _I, _P, _L, _P),
    "srml_rf_pack_wy": (_P, _P, _P, _L, _P, _P),
    "srml_rf_quantiles_f32": (_P, _I, _I, _I, _P, _P),
    "srml_rf_hist": (_P, _L, _P, _P, _P, _I, _P, _I, _I, _I, _I, _D, _I, _P, _P, _I, _P),
    "srml_rf_interleave_u8": (_P, _L, _I, _I, _P, _P),
    "srml_rf_hist_fb": (_I, _I, _I),
    "srml_rf_hist_fb_max": (),
    "srml_rf_best_split": (_P, _P, _I, _I, _I, _I, _I, _I, _D, _D, _P, _P, _P),
    "srml_rf_node_split_ok": (_I, _I, _I),
    "srml_rf_transpose_u8": (_P, _L, _I, _P, _P),
    "srml_rf_node_split": (_P, _L, _P, _P, _P, _I, _P, _I, _I, _I, _I, _D, _D, _P, _P, _P),
    "srml_rf_route": (_P, _L, _P, _P, _L, _P, _P, _P, _P, _P),
    "srml_rf_route_segments": (_P, _L, _P, _L, _P, _I, _P, _P, _P, _P, _P),
    "srml_rf_node_stats": (_P, _P, _P, _L, _P, _I, _I, _I, _P, _P),
    "srml_rf_node_stats_det": (_P, _P, _P, _P, _I, _I, _I, _P, _P),
    "srml_label_sort": (_P, _L, _I, _P, _P, _P, _P, _P),
    "srml_label_sort_ws": (_L, _I),
    "srml_label_sort_kmax": (),
    "srml_radix_sort_ws": (_L,),
    "srml_knn_refine_sort_f32": (_P, _L, _I, _L, _P, _L, _P, _I, _L, _I, _P, _P, _P),
    "srml_radix_sort_u64": (_P, _P, _P, _P, _L, _I, _P, _P),
    "srml_label_counts": (_P, _L, _I, _P, _P),
    "srml_rf_hist_wide": (_P, _L, _P, _P, _P, _I, _P, _I, _I, _I, _I, _D, _I, _I, _I, _P, _P, _P),
    "srml_rf_hist_wide_fb": (_I, _I, _I),
    "srml_rf_hist_fixed": (_P, _L, _P, _P, _P, _I, _P, _I, _I, _D, _I, _P, _I, _P),
    "srml_rf_hist_fixed_finish": (_P, _L, _D, _P),
    "srml_csr_logreg_binary_f32": (_P, _P, _P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P),
    "srml_csr_logreg_binary_f64": (_P, _P, _P, _L, _I, _L, _P, _P, _D, _P, _P, _P, _P),
    "srml_csr_spmm_f32": (_P, _P, _P, _L, _L, _P, _I, _P, _P, _P),
    "srml_csr_spmm_f64": (_P, _P, _P, _L, _L, _P, _I, _P, _P, _P),
    "srml_csr_spmtm_f32": (_P, _P, _P, _L, _L, _P, _I, _P, _P),
    "srml_csr_spmtm_f64": (_P, _P, _P, _L, _L, _P, _I, _P, _P),
    "srml_csr_spmm_ld_f32": (_P, _P, _P, _L, _L, _P, _I, _L, _P, _P, _L, _P),
    "srml_csr_spmm_ld_f64": (_P, _P, _P, _L, _L, _P, _I, _L, _P, _P, _L, _P),
    "srml_csr_spmtm_ld_f32": (_P, _P, _P, _L, _L, _P, _I, _L, _P, _L, _P),
    "srml_csr_spmtm_ld_f64": (_P, _P, _P, _L, _L, _P, _I, _L, _P, _L, _P),
    "srml_csr_row_sums_f32": (_P, _P, _L, _P, _P),
    "srml_confusion_counts": (_P, _I, _P, _I, _L, _I, _P, _P),
    "srml_logloss_sum": (_P, _I, _L, _I, _L, _P, _I, _D, _P, _P),
    "srml_reg_moments": (_P, _I, _P, _I, _L, _P, _P),
    "srml_csr_col_moments_f32": (_P, _P, _L, _P, _P, _P),
    "srml_csr_col_moments_f64": (_P, _P, _L, _P, _P, _P),
    "srml_memcpy_h2d_async": (_P, _P, _L, _P),
    "srml_memcpy_d2h_sync": (_P, _P, _L, _P),
    "srml_memset_async": (_P, _I, _L, _P),
    "srml_rf_predict_nodes2": (_P, _L, _L, _I, _P, _P, _I, _P, _I, _P, _P, _P),
    "srml_rf_predict": (_P, _L, _L, _P, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P),
    "srml_rf_left_totals": (_P, _I, _L, _I, _I, _I, _P, _P, _P),
    "srml_rf_gather_feature": (_P, _L, _P, _L, _P, _P),
    "srml_rf_decide": (_P, _P, _P, _L, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P),
    "srml_rf_level_pack": (_P, _L, _P, _I, _I, _I, _P, _P, _P, _P),
    "srml_seg_lower_bound": (_P, _P, _P, _L, _P, _I, _P, _P),
    "srml_scatter_shift": (_P, _I, _P, _P, _P, _D, _P),
    "srml_sum_sq_ws": (),
    "srml_sum_sq": (_P, _I, _L, _P, _P, _P),
    "srml_lsq_prepare": (_P, _I, _P, _P, _P, _D, _D, _D, _D, _D, _I, _I, _I, _P, _P, _P),
    "srml_lsq_finish": (_P, _I, _P, _P, _D, _D, _I, _P, _P),
    "srml_rf_sample_features": (_I, _I, _I, ctypes.c_ulonglong, _P, _P),
    "srml_rf_partition": (_P, _L, _P, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P),
    "srml_rf_partition_ws": (_L, _I),
    "srml_ivf_candidate_max": (_P, _I, _P, _L, _P, _P, _P),
    "srml_ivf_candidates_f32": (_P, _L, _L, _I, _L, _P, _I, _P, _P, _P, _L, _P, _P, _P, _P, _L, _P),
    "srml_row_list": (_P, _I, _L, _P, _P),
    "srml_cd_sweep_global_f64": (_P, _I, _L, _P, _P, _P, _P, _P, _P, _P, _I, _P),
    "srml_logit_residual_wide_f32": (_P, _L, _I, _L, _P, _P, _L, _P, _L, _P, _P, _P),
    "srml_logit_residual_wide_f64": (_P, _L, _I, _L, _P, _P, _L, _P, _L, _P, _P, _P),
}

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None


def _load() -> ctypes.CDLL:
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.lib_path()
        if (not os.path.exists(path) or _build.needs_build()) and os.environ.get("SRML_NO_AUTOBUILD", "0") != "1":
            try:
                _build.build()
            except Exception as e:  # noqa: BLE001
                if not os.path.exists(path):
                    _load_error = "build failed: %s" % e
                    raise RuntimeError(_load_error)
        # make sure torch's HIP runtime is the one our library binds to
        import torch.cuda  # noqa: F401

        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        for name, argt in SIGNATURES.items():
            try:
                fn = getattr(lib, name)
            except AttributeError:
                continue
            fn.argtypes = list(argt)
            fn.restype = ctypes.c_long if name in _LONG_RESULT else ctypes.c_int
        _lib = lib
        return lib


def lib() -> ctypes.CDLL:
    """The loaded native library; raises RuntimeError if it cannot be built/loaded."""
    return _load()


def available() -> bool:
    try:
        _load()
        return True
    except Exception:  # noqa: BLE001
        return False


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args: Any) -> None:
    """Launch ``name`` with its declared ctypes signature. An entry point without one would get
    ctypes' default int conversion (64-bit pointers and sizes truncated), so it is refused."""
    if name not in SIGNATURES:
        raise KeyError("native.call: %s has no entry in ops/native.py SIGNATURES" % name)
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError("%s launch failed with HIP status %d" % (name, rc))
