"""Random forest (classification + regression) grown level-wise on the device.

Reference: cuML ``RandomForestClassifier/Regressor`` (quantile bins, bootstrap, per-node feature
sampling, level-wise histogram splits) driven from ``tree.py:254-434``, FIL inference
(``tree.py:571-613``) and the ensemble-per-rank distribution with the forests gathered through
the Spark driver as base64 treelite JSON (``tree.py:337-378``).

MI355X pipeline per tree (one rank):

1. once per fit: quantile bin edges from a row sample (device sort), the shard quantised to a
   feature-major uint8 matrix (``srml_rf_quantize_u8``);
2. Poisson(subsamplingRate) bootstrap multiplicities (Spark's bagging) on the device; the row
   index array holds the in-bag rows, node segments stay contiguous and row-ordered;
3. per level: device feature subsets per node, ``srml_rf_hist`` (LDS-privatised histograms over
   (node, 8-feature, row-chunk) work items), ``srml_rf_best_split`` (Gini / entropy / variance
   gain sweep + block arg-max), ``srml_rf_route`` + a stable device sort to re-partition rows
   into child segments. Only per-node split records (a few doubles per node) come to the host;
4. leaves store Spark's per-tree prediction (normalised class distribution / mean).

Distribution: ``ensemble`` (reference parity: each rank grows its share of trees on its local
rows, forests exchanged with ONE device all-gather) or ``data_parallel`` (every rank grows the
same trees over ALL rows: identical seeds, per-level histogram + node-total all-reduce over
RCCL — the north-star mode for datasets larger than one GPU's share).
"""
from __future__ import annotations

import os

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext
from ..utils.determinism import deterministic

ROWS_PER_ITEM = 4096
CHUNK_MAJOR_ITEMS = os.environ.get("SRML_RF_ITEM_ORDER", "chunk") == "chunk"
# The histogram gathers from the 32-byte record layout of the bins (when a node's feature chunks
# are dense enough, ops.rf_il_useful) at levels whose nodes hold on average less than IL_DENSITY
# of the rows: there one record load per row beats one cache line per (row, feature), while
# denser nodes share the lines of the feature-major columns (1M x 3000 regression trace: levels
# 5-6 37 / 31 ms vs 63 / 53 ms, levels 2-3 23 / 39 ms feature-major vs 56 / 63 ms).
# SRML_RF_IL_DENSITY=0 turns the record layout off.
IL_DENSITY = float(os.environ.get("SRML_RF_IL_DENSITY", "0.3"))
# Record-layout kernel: "wide" = one 1024-thread block per (row chunk, ~100-400 features), each
# row's records fetched once per block (ops.rf_hist_fb_wide); "narrow" = 8-feature items.
IL_KERNEL = os.environ.get("SRML_RF_IL_KERNEL", "wide")
# record bytes of the wide kernel's layout: 64-B records use half of each 128-B line a sparse
# row gather touches where 32-B records used a quarter
WIDE_REC_BYTES = int(os.environ.get("SRML_RF_REC_BYTES", "64"))
WIDE_ROWS_PER_ITEM = 8192
WIDE_ROWS_MAX = 65536
# packed regression cells in the wide kernel (one u64 LDS atomic per row and feature instead of a
# u32 count + u64 sum; sums quantised to 2^-22 max|y| per row): SRML_RF_PACK=0 keeps the exact
# fixed point; deterministic mode always does
RF_PACK = os.environ.get("SRML_RF_PACK", "1") != "0"
INT_MAX = 2**31 - 1
# data-parallel forests: each level's histograms are REDUCE-SCATTERED by node (every rank gets the
# summed histograms of 1/W of the candidate nodes), each rank searches its nodes' splits and only
# the per-node split records + left-child totals are all-gathered — half the wire bytes of
# all-reducing every histogram, identical splits. SRML_RF_DP_SCATTER=0: all-reduce every histogram.
RF_DP_SCATTER = os.environ.get("SRML_RF_DP_SCATTER", "1") != "0"
# sibling subtraction (nodes that see every feature, featureSubsetStrategy="all"): from depth 1 only
# the smaller child of each split is histogrammed (and, data-parallel, all-reduced); the larger is
# its parent's histogram minus the smaller's. Per-node feature sampling draws a fresh subset per
# node, so there the parent's histogram does not cover the children's features and every node is
# built. SRML_RF_SIBLING_SUB=0 turns it off.
RF_SIBLING_SUB = os.environ.get("SRML_RF_SIBLING_SUB", "1") != "0"
# SRML_RF_LEVEL_LOG=1: per-level host timing of the last grow_forest call in LAST_LEVELS (segments,
# candidates, seconds of host work vs waits on the device per section)
LEVEL_LOG = os.environ.get("SRML_RF_LEVEL_LOG", "0") == "1"
# one blocking device->host copy per level: the split decisions (which candidates split, their child
# slots) are taken on the device, the route / partition / child totals run on the candidate count as
# an upper bound, and ONE copy brings the split records, child bounds and child stats back
# (SRML_RF_ONE_SYNC=0: the two-copy loop; max_leaves > 0 always takes it — its per-tree budget is
# decided on the host)
RF_ONE_SYNC = os.environ.get("SRML_RF_ONE_SYNC", "1") != "0"
# the one-sync level bookkeeping in native kernels (ops.rf_decide / rf_level_pack); 0: torch ops
RF_LEVEL_NATIVE = os.environ.get("SRML_RF_LEVEL_NATIVE", "1") != "0"
# levels whose nodes average fewer in-bag positions than this gather from a row-major copy of the
# bins (built once, at the first such level): a row's sampled features share cache lines there,
# where the feature-major matrix costs one line per (row, feature) (0 = off)
RM_ROWS = float(os.environ.get("SRML_RF_ROWMAJOR_ROWS", "10000"))
# classification levels on the row-major copy whose nodes average fewer positions than this build
# each node's histogram and split search in one block (ops.rf_node_split: the histograms stay in
# LDS) instead of rf_hist + rf_best_split (0 = off); nodes above FUSED_MAX_ROWS keep the unfused path
FUSED_ROWS = float(os.environ.get("SRML_RF_FUSED_ROWS", "10000"))
FUSED_MAX_ROWS = 1 << 20
FUSED_MIN_NODES = 256  # one block per node: fewer nodes leave most CUs idle
# narrow feature samples (several rows per wave instruction) measured slower than the unfused
# record-layout kernels: north-star 50M x 64 (8 sampled features) levels 12-15 51 / 47 / 47 / 55 ms
# fused vs 32 / 36 / 42 / 57 ms (profiles/rf_levels_northstar_50M_r5_fused_narrow.txt)
FUSED_MIN_NF = 33
LAST_LEVELS: List[Dict[str, Any]] = []


class _LevelClock:
    """Accumulates wall time between marks into named sections (no-op unless LEVEL_LOG)."""

    def __init__(self) -> None:
        import time

        self._now = time.perf_counter
        self.t = self._now()
        self.rec: Dict[str, Any] = {}

    def mark(self, name: str) -> None:
        if not LEVEL_LOG:
            return
        t = self._now()
        self.rec[name] = round(self.rec.get(name, 0.0) + (t - self.t), 6)
        self.t = t


def _left_totals(hist: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """(C, S) fp64 class totals of each node's left child under its best split (zeros for nodes
    without one): the winning feature's histogram summed up to the split bin."""
    return ops.rf_left_totals(hist, out)


def feature_subset_size(strategy: Any, n: int, n_trees: int, classification: bool) -> int:
    if isinstance(strategy, str):
        s = strategy.lower()
        if s == "auto":
            s = "all" if n_trees == 1 else ("sqrt" if classification else "onethird")
        if s == "all":
            return n
        if s == "sqrt":
            return max(1, int(math.ceil(math.sqrt(n))))
        if s == "log2":
            return max(1, int(math.ceil(math.log2(n)))) if n > 1 else 1
        if s == "onethird":
            return max(1, int(math.ceil(n / 3.0)))
        try:
            strategy = float(s)
        except ValueError:
            raise ValueError("unsupported featureSubsetStrategy %r" % strategy)
    v = float(strategy)
    if v > 1.0 or (v == 1.0 and isinstance(strategy, int) and strategy > 1):
        return max(1, min(n, int(v)))
    return max(1, min(n, int(math.ceil(v * n))))


def bin_edges(X: torch.Tensor, n_bins: int, ctx: WorkerContext, m_total: int, seed: int,
              sample_rows: Optional[int] = None, host: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(n, n_bins-1) fp32 quantile edges, identical on every rank (sampled rows all-gathered).

    Sample size follows Spark's ``findSplits`` (max(maxBins^2, 10000) rows over the whole dataset,
    capped at the 32768 the per-feature LDS sort holds). ``host``: the page-locked source of a
    streamed ingest — the same sampled rows are gathered on the host and sent ahead of the shard,
    so the edges exist before the shard has landed."""
    m, n = X.shape
    if sample_rows is None:
        sample_rows = min(32768, max(n_bins * n_bins, 10000))
    g = torch.Generator(device="cpu")
    g.manual_seed(int(seed) * 7919 + ctx.rank)
    want = max(1, int(sample_rows * m // max(m_total, 1)))
    if m > want and host is not None:
        sel = torch.randperm(m, generator=g)[:want].sort().values
        Sh = torch.empty((want, n), dtype=host.dtype, pin_memory=True)
        torch.index_select(host, 0, sel, out=Sh)
        S = Sh.to(X.device, non_blocking=True).float()
    elif m > want:
        sel = torch.randperm(m, generator=g)[:want].sort().values.to(X.device)
        S = X.index_select(0, sel).float()
    elif host is not None:
        S = host.to(X.device, non_blocking=True).float()
    else:
        S = X.float()
    if ctx.world_size > 1:
        S = torch.cat([p.to(X.device) for p in ctx.comm.allgatherv(S.contiguous())], 0)
    return ops.rf_quantiles(S, n_bins - 1)  # (n, B-1), non-decreasing per feature


@dataclass
class Tree:
    feature: List[int] = field(default_factory=list)
    threshold: List[float] = field(default_factory=list)
    left: List[int] = field(default_factory=list)
    right: List[int] = field(default_factory=list)
    value: List[List[float]] = field(default_factory=list)
    impurity: List[float] = field(default_factory=list)
    gain: List[float] = field(default_factory=list)
    count: List[float] = field(default_factory=list)
    depth: int = 0

    def to_dict(self) -> Dict[str, Any]:
        return {"feature": self.feature, "threshold": self.threshold, "left": self.left, "right": self.right,
                "value": self.value, "impurity": self.impurity, "gain": self.gain, "count": self.count,
                "depth": self.depth}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Tree":
        t = cls()
        for k in ("feature", "threshold", "left", "right", "value", "impurity", "gain", "count"):
            setattr(t, k, list(d[k]))
        t.depth = int(d.get("depth", 0))
        return t

    @property
    def num_nodes(self) -> int:
        return len(self.feature)


def _leaf_values_np(tot: np.ndarray, regression: bool) -> np.ndarray:
    """Leaf values of all segments: (L, 1) weighted means or (L, S) class probabilities."""
    if regression:
        n = tot[:, 0]
        return np.where(n > 0, tot[:, 1] / np.where(n > 0, n, 1.0), 0.0)[:, None]
    s = tot.sum(1, keepdims=True)
    return np.where(s > 0, tot / np.where(s > 0, s, 1.0), 0.0)


def _impurities_np(tot: np.ndarray, crit: int) -> np.ndarray:
    """Impurity of all segments: variance (crit 2), Gini (0) or entropy (1)."""
    if crit == 2:
        n = tot[:, 0]
        safe = np.where(n > 0, n, 1.0)
        mu = tot[:, 1] / safe
        return np.where(n > 0, np.maximum(tot[:, 2] / safe - mu * mu, 0.0), 0.0)
    n = tot.sum(1)
    safe = np.where(n > 0, n, 1.0)[:, None]
    pr = tot / safe
    if crit == 0:
        v = 1.0 - (pr * pr).sum(1)
    else:
        with np.errstate(divide="ignore", invalid="ignore"):
            v = -np.where(pr > 0, pr * np.log2(np.where(pr > 0, pr, 1.0)), 0.0).sum(1)
    return np.where(n > 0, v, 0.0)


def _seg_stats(tot: torch.Tensor, regression: bool, crit: int) -> torch.Tensor:
    """Per segment [leaf value(s) (1 | S) | weight sum | impurity] (L, V + 2) fp64, computed where
    the totals live (the device: ~25 ms of numpy per 200k-segment level on the host) with the
    formulas of ``_leaf_values_np`` / ``_impurities_np``."""
    tot = tot.double()
    if regression:
        n = tot[:, 0]
        safe = torch.where(n > 0, n, torch.ones_like(n))
        mu = tot[:, 1] / safe
        val = torch.where(n > 0, mu, torch.zeros_like(mu))[:, None]
        imp = torch.where(n > 0, torch.clamp_min(tot[:, 2] / safe - mu * mu, 0.0), torch.zeros_like(n))
        return torch.cat([val, n[:, None], imp[:, None]], 1)
    n = tot.sum(1)
    safe = torch.where(n > 0, n, torch.ones_like(n))[:, None]
    pr = tot / safe
    val = torch.where(n[:, None] > 0, pr, torch.zeros_like(pr))
    if crit == 0:
        v = 1.0 - (pr * pr).sum(1)
    else:
        v = -torch.where(pr > 0, pr * torch.log2(torch.where(pr > 0, pr, torch.ones_like(pr))),
                         torch.zeros_like(pr)).sum(1)
    imp = torch.where(n > 0, v, torch.zeros_like(v))
    return torch.cat([val, n[:, None], imp[:, None]], 1)


class _ForestRecords:
    """Level-wise node records of a forest grown level-synchronously, assembled into ``Tree``s
    once at the end (per-node Python bookkeeping cost ~10 us/node: 0.25 s for a 50-tree,
    depth-13 forest)."""

    def __init__(self, n_trees: int) -> None:
        self.nn = np.ones(n_trees, dtype=np.int64)  # nodes per tree (roots = node 0)
        self.seg: List[Tuple[np.ndarray, ...]] = []    # (tree, nid, value (L, V), count, impurity)
        self.split: List[Tuple[np.ndarray, ...]] = []  # (tree, nid, feature, threshold, gain, left, right)
        self.depth = 0

    def add_children(self, t_i: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """Left/right ids for splits of trees ``t_i`` (in order): per tree, consecutive ids in
        order of appearance."""
        order_t = np.argsort(t_i, kind="stable")
        ts = t_i[order_t]
        starts = np.r_[0, np.nonzero(np.diff(ts))[0] + 1]
        lens = np.diff(np.r_[starts, len(ts)])
        rank_sorted = np.arange(len(ts)) - np.repeat(starts, lens)
        rank = np.empty_like(rank_sorted)
        rank[order_t] = rank_sorted
        left = self.nn[t_i] + 2 * rank
        np.add.at(self.nn, t_i, 2)
        return left, left + 1

    def build(self) -> List[Tree]:
        T = len(self.nn)
        V = self.seg[0][2].shape[1] if self.seg else 1
        trees = []
        seg = [np.concatenate([r[i] for r in self.seg]) for i in range(5)] if self.seg else None
        spl = [np.concatenate([r[i] for r in self.split]) for i in range(7)] if self.split else None
        seg_by = np.argsort(seg[0], kind="stable") if seg is not None else None
        seg_bounds = np.searchsorted(seg[0][seg_by], np.arange(T + 1)) if seg is not None else None
        spl_by = np.argsort(spl[0], kind="stable") if spl is not None else None
        spl_bounds = np.searchsorted(spl[0][spl_by], np.arange(T + 1)) if spl is not None else None
        for t in range(T):
            nn = int(self.nn[t])
            feature = np.full(nn, -1, dtype=np.int64)
            threshold = np.zeros(nn)
            left = np.full(nn, -1, dtype=np.int64)
            right = np.full(nn, -1, dtype=np.int64)
            value = np.zeros((nn, V))
            impurity = np.zeros(nn)
            gain = np.zeros(nn)
            count = np.zeros(nn)
            if seg is not None:
                sel = seg_by[seg_bounds[t]: seg_bounds[t + 1]]
                nid = seg[1][sel]
                value[nid] = seg[2][sel]
                count[nid] = seg[3][sel]
                impurity[nid] = seg[4][sel]
            if spl is not None:
                sel = spl_by[spl_bounds[t]: spl_bounds[t + 1]]
                nid = spl[1][sel]
                feature[nid] = spl[2][sel]
                threshold[nid] = spl[3][sel]
                gain[nid] = spl[4][sel]
                left[nid] = spl[5][sel]
                right[nid] = spl[6][sel]
            # numpy node arrays (JSON conversion happens only when a model is persisted)
            tr = Tree(feature=feature, threshold=threshold, left=left, right=right, value=value, impurity=impurity,
                      gain=gain, count=count, depth=self.depth)
            trees.append(tr)
        return trees


def _node_stats(yv: torch.Tensor, idx: torch.Tensor, wpos: torch.Tensor, bounds: torch.Tensor, S: int,
                regression: bool) -> torch.Tensor:
    return ops.rf_node_stats(idx, wpos, yv, bounds, S, regression)


HIST_BUDGET_BYTES = 1 << 30


def _root_hist_streamed(pending: PendingBins, bins: torch.Tensor, idx: torch.Tensor, wpos: torch.Tensor,
                        yv: torch.Tensor, c_start: np.ndarray, c_cnt: np.ndarray, feats: torch.Tensor, C: int, B: int,
                        SH: int, regression: bool, fb: int, yscale: Optional[float]) -> torch.Tensor:
    """Root-level histograms of C segments (rows ascending inside each) built chunk by chunk as the
    streamed shard lands: every chunk is binned, then the items over that chunk's positions of every
    segment add into one zeroed histogram. The item lists of all chunks are built and uploaded
    before the first chunk is queued (no host read waits for the transfer)."""
    dev = bins.device
    m = bins.shape[1]
    nf = feats.shape[1]
    nfc = (nf + fb - 1) // fb
    Ch = feats.shape[0]  # histogram rows: C, or C padded for the node-partitioned reduce-scatter
    assert C == len(c_start) and Ch >= C
    hist = ops.zeros((Ch, nf, B, SH), dtype=torch.float64 if regression else torch.int32, device=dev)
    wy = ops.rf_hist_wy(idx, yv, None, wpos)
    rows_at = torch.tensor([r0 for r0, _ in pending.bounds] + [m], dtype=idx.dtype, device=dev)
    # P[j, c]: first position of segment j whose row is >= the start of chunk c
    P = ops.seg_lower_bound(idx, c_start, c_cnt, rows_at)
    per_chunk = []
    for ci in range(len(pending.bounds)):
        lo, hi = P[:, ci], P[:, ci + 1]
        cnt = hi - lo
        rpi = int(min(WIDE_ROWS_MAX, max(ROWS_PER_ITEM, (int(cnt.sum()) * nfc) // 8192)))
        rpi = (rpi + 511) // 512 * 512
        nch = (cnt + rpi - 1) // rpi
        tot_ch = int(nch.sum())
        node_rep = np.repeat(np.arange(C), nch)
        chunk = np.arange(tot_ch) - np.repeat(np.cumsum(nch) - nch, nch)
        rb = lo[node_rep] + chunk * rpi
        re = np.minimum(rb + rpi, hi[node_rep])
        it = np.empty((tot_ch * nfc, 4), dtype=np.int32)  # feature-chunk-major, atomics only
        it[:, 0] = np.tile(node_rep, nfc)
        it[:, 1] = np.tile(rb, nfc)
        it[:, 2] = np.tile(re, nfc)
        it[:, 3] = np.repeat(np.arange(nfc, dtype=np.int32), tot_ch)
        per_chunk.append(it)
    off = np.cumsum([0] + [a.shape[0] for a in per_chunk])
    items_all = _h2d(np.concatenate(per_chunk, 0), dev)
    for ci, _rows in enumerate(pending.chunks()):
        if off[ci + 1] > off[ci]:
            ops.rf_hist(bins, idx, yv, None, items_all[off[ci]: off[ci + 1]], feats, Ch, B, SH, regression,
                        pos_weight=wpos, fb=fb, yscale=yscale, out=hist, wy=wy)
    return hist


def _expand_siblings(built: torch.Tensor, derive: np.ndarray, sib_pos: np.ndarray, prev_hist: torch.Tensor,
                     parent_row: np.ndarray) -> torch.Tensor:
    """Histograms of every candidate (cand order) from the built ones (cand[~derive] order): a
    derived node's histogram is its parent's minus its (built) sibling's."""
    dev = built.device
    C = derive.size
    full = torch.empty((C,) + tuple(built.shape[1:]), dtype=built.dtype, device=dev)
    bpos = _h2d(np.nonzero(~derive)[0], dev)
    full.index_copy_(0, bpos, built)
    d = np.nonzero(derive)[0]
    if d.size:
        dpos = _h2d(d, dev)
        par = prev_hist.index_select(0, _h2d(parent_row[d], dev))
        full.index_copy_(0, dpos, par - full.index_select(0, _h2d(sib_pos[d], dev)))
    return full


def _h2d(a: np.ndarray, dev: torch.device) -> torch.Tensor:
    """Host array -> device without a blocking copy: staged through page-locked memory and queued
    on the stream (the caching host allocator keeps the staging buffer until the copy ran)."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dev.type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def _pad_rows(t: torch.Tensor, rows: int) -> torch.Tensor:
    """``t`` with zero rows appended up to ``rows``."""
    return torch.cat([t, ops.zeros((rows - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)], 0)


def _level_one_sync_device(bins: torch.Tensor, idx: torch.Tensor, wpos: torch.Tensor, bounds: torch.Tensor,
                           tot: torch.Tensor, yv: torch.Tensor, cand: np.ndarray, L: int, out_d: torch.Tensor,
                           fsel_d: torch.Tensor, res_left: List[torch.Tensor], S: int, regression: bool, crit: int,
                           data_parallel: bool, ctx: WorkerContext, dev: torch.device, clk: "_LevelClock"
                           ) -> Optional[tuple]:
    """``_level_one_sync`` with its bookkeeping in native kernels (ops.rf_decide / rf_level_pack:
    split ranks, routing arrays, children totals, segment stats and the read-back buffer) — the
    torch version launched ~55 library kernels per level. Same results and return value."""
    C = int(cand.size)
    cand_d = _h2d(cand.astype(np.int64), dev)
    left = None
    if not regression:
        left = torch.cat(res_left, 0) if len(res_left) > 1 else res_left[0]
    node_feature, node_bin, child_base, tot_n = ops.rf_decide(out_d, fsel_d, cand_d, L, left,
                                                              None if regression else tot)
    clk.mark("decide_host")
    keys = ops.rf_route_segments(bins, idx, bounds, node_feature, node_bin, child_base)
    idx_n, wpos_n, bounds_n = ops.rf_partition(keys, bounds, node_feature, child_base, C, idx, wpos, trim=False)
    if regression:
        tot_n = _node_stats(yv, idx_n, wpos_n, bounds_n, S, regression)
        if data_parallel:
            ctx.comm.allreduce(tot_n)
    clk.mark("route_launch")
    V2 = 3 if regression else int(tot_n.shape[1]) + 2
    hb = ops.rf_level_pack(bounds_n, tot_n, regression, crit, out_d, fsel_d).cpu().numpy()
    clk.mark("end_sync")
    nb = 2 * C + 1
    off = nb + 2 * C * V2
    out_all = hb[off: off + 6 * C].reshape(C, 6)
    feat_all = hb[off + 6 * C:]
    ci_sel = np.nonzero(out_all[:, 1] >= 0)[0]
    k = int(ci_sel.size)
    if LEVEL_LOG:
        clk.rec["candidates"] = C
        clk.rec["splits"] = k
    if k == 0:
        return None
    bounds_h = hb[: 2 * k + 1].astype(np.int64)
    stats_h = hb[nb: nb + 2 * k * V2].reshape(2 * k, V2)
    kept = int(bounds_h[-1])
    return (idx_n[:kept], wpos_n[:kept], bounds_n[: 2 * k + 1], tot_n[: 2 * k], bounds_h, stats_h, out_all,
            feat_all, ci_sel)


def _level_one_sync(bins: torch.Tensor, idx: torch.Tensor, wpos: torch.Tensor, bounds: torch.Tensor,
                    tot: torch.Tensor, yv: torch.Tensor, cand: np.ndarray, L: int, res_out_d: List[torch.Tensor],
                    res_fsel_d: List[torch.Tensor], res_left: List[torch.Tensor], S: int, regression: bool,
                    crit: int, data_parallel: bool, ctx: WorkerContext, dev: torch.device, clk: "_LevelClock"
                    ) -> Optional[tuple]:
    """The split decisions, routing, re-partition and child totals of one level with ONE blocking
    copy (RF_ONE_SYNC): candidate j splits iff its record has a feature (out[j, 1] >= 0); its children
    take slots 2 r, 2 r + 1 with r its rank among the splitting candidates (an exclusive scan on the
    device), so route / partition / node stats run with the candidate count C as the bound on the
    splits (children past the real ones are empty segments). Returns None when nothing splits, else
    (idx, wpos, bounds, tot, bounds_h, stats_h, out_all, feat_all, ci_sel) trimmed to the k splits."""
    out_d = torch.cat(res_out_d, 0) if len(res_out_d) > 1 else res_out_d[0]
    fsel_d = (torch.cat(res_fsel_d, 0) if len(res_fsel_d) > 1 else res_fsel_d[0]).view(-1)
    C = int(cand.size)
    if RF_LEVEL_NATIVE and dev.type == "cuda" and out_d.dtype == torch.float64 and fsel_d.dtype == torch.float64:
        return _level_one_sync_device(bins, idx, wpos, bounds, tot, yv, cand, L, out_d, fsel_d, res_left, S,
                                      regression, crit, data_parallel, ctx, dev, clk)
    ok_d = out_d[:, 1] >= 0
    oki = ok_d.to(torch.int32)
    pos_d = torch.cumsum(oki, 0, dtype=torch.int32) - oki
    cand_d = _h2d(cand.astype(np.int64), dev)
    node_feature = torch.full((L,), -1, dtype=torch.int32, device=dev)
    node_bin = ops.zeros(L, dtype=torch.int32, device=dev)
    child_base = ops.zeros(L, dtype=torch.int32, device=dev)
    node_feature[cand_d] = torch.where(ok_d, fsel_d.to(torch.int32), torch.full_like(oki, -1))
    node_bin[cand_d] = torch.where(ok_d, out_d[:, 2].to(torch.int32), torch.zeros_like(oki))
    child_base[cand_d] = torch.where(ok_d, 2 * pos_d, torch.zeros_like(oki))
    clk.mark("decide_host")
    keys = ops.rf_route_segments(bins, idx, bounds, node_feature, node_bin, child_base)
    idx_n, wpos_n, bounds_n = ops.rf_partition(keys, bounds, node_feature, child_base, C, idx, wpos, trim=False)
    if regression:
        tot_n = _node_stats(yv, idx_n, wpos_n, bounds_n, S, regression)
    else:
        # children totals: the winning histogram's prefix (left) and the parent's rest (right), moved to
        # the split's child slots; candidates that do not split go to a discarded row
        left = torch.cat(res_left, 0) if len(res_left) > 1 else res_left[0]
        pair = torch.stack([left, tot.index_select(0, cand_d) - left], 1)
        dest = torch.where(ok_d, pos_d.long(), torch.full_like(pos_d, C, dtype=torch.int64))
        tot_n = ops.zeros((C + 1, 2, S), dtype=pair.dtype, device=dev)
        tot_n.index_copy_(0, dest, pair)
        tot_n = tot_n[:C].reshape(2 * C, S)
    if data_parallel and regression:
        ctx.comm.allreduce(tot_n)
    clk.mark("route_launch")
    stats = _seg_stats(tot_n, regression, crit)
    V2 = int(stats.shape[1])
    hb = torch.cat([bounds_n.double(), stats.reshape(-1), out_d.double().reshape(-1), fsel_d.double()]).cpu().numpy()
    clk.mark("end_sync")
    nb = 2 * C + 1
    off = nb + 2 * C * V2
    out_all = hb[off: off + 6 * C].reshape(C, 6)
    feat_all = hb[off + 6 * C:]
    ci_sel = np.nonzero(out_all[:, 1] >= 0)[0]
    k = int(ci_sel.size)
    if LEVEL_LOG:
        clk.rec["candidates"] = C
        clk.rec["splits"] = k
    if k == 0:
        return None
    bounds_h = hb[: 2 * k + 1].astype(np.int64)
    stats_h = hb[nb: nb + 2 * k * V2].reshape(2 * k, V2)
    kept = int(bounds_h[-1])
    return (idx_n[:kept], wpos_n[:kept], bounds_n[: 2 * k + 1], tot_n[: 2 * k], bounds_h, stats_h, out_all,
            feat_all, ci_sel)


def grow_forest(bins: torch.Tensor, edges_h: np.ndarray, y: torch.Tensor, ctx: WorkerContext,
                gen: torch.Generator, p: Dict[str, Any], S: int, regression: bool, data_parallel: bool,
                gen_boot: Optional[torch.Generator], n_trees: int, pending: Optional[PendingBins] = None) -> List[Tree]:
    """Grow ``n_trees`` trees level-synchronously: every level of every tree is ONE histogram /
    split / route / partition pass over the concatenated (tree, node) segments, so the per-level
    launches and host round trips are amortised over the whole forest (cuML grows trees
    concurrently on streams for the same reason; here they share one batched launch).

    ``pending``: a streamed shard's chunks not binned yet — the root level's histograms are then
    built chunk by chunk right behind each chunk's binning, under the PCIe transfer (every item
    accumulates with atomics into one zeroed histogram: the same sums, in another order)."""
    dev = bins.device
    n, m = bins.shape
    B = edges_h.shape[1] + 1
    SH = 2 if regression else S  # regression histograms carry (count, sum) only
    crit = {"gini": 0, "entropy": 1, "variance": 2, "mse": 2}[p["split_criterion"]]
    max_depth = int(p["max_depth"])
    min_leaf = float(p["min_samples_leaf"])
    min_split = float(p["min_samples_split"])
    min_gain = float(p.get("min_impurity_decrease", 0.0))
    nf = int(p["_nf"])
    max_leaves = int(p.get("max_leaves", -1))
    yv = y.float().contiguous()
    rec = _ForestRecords(n_trees)
    # bootstrap multiplicities per tree (Spark: Poisson(subsamplingRate) bagging); positions of
    # all trees are concatenated: segment = (tree, node), rows stay ascending inside a segment
    if p["bootstrap"]:
        # one native pass draws every tree's Poisson multiplicities and compacts the in-bag rows
        # (tree-major, ascending); the seed is one draw of the bootstrap generator per call
        boot_seed = int(torch.randint(0, 1 << 62, (1,), generator=gen_boot or gen,
                                      device=(gen_boot or gen).device).item())
        idx, wpos, bounds_h = ops.rf_bootstrap(n_trees, m, float(p.get("max_samples", 1.0)), boot_seed, dev)
        idx, wpos = idx.to(dev).contiguous(), wpos.to(dev).contiguous()
    else:
        idx = torch.arange(m, dtype=torch.int32, device=dev).repeat(n_trees)
        wpos = torch.ones(n_trees * m, dtype=torch.float32, device=dev)
        bounds_h = np.arange(n_trees + 1, dtype=np.int64) * m
    seg_tree = np.arange(n_trees, dtype=np.int64)
    seg_nid = np.zeros(n_trees, dtype=np.int64)  # every tree's root is node 0
    bounds_h = np.asarray(bounds_h, dtype=np.int64)
    counts = np.diff(bounds_h)
    bounds = torch.from_numpy(bounds_h).to(dev)
    tot = _node_stats(yv, idx, wpos, bounds, S, regression)
    if data_parallel:
        ctx.comm.allreduce(tot)
    n_leaves = np.ones(n_trees, dtype=np.int64)
    fb = ops.rf_hist_fb(B, SH, regression)  # features per histogram work item (fits the LDS slab)
    nfc = (nf + fb - 1) // fb
    # one draw of the fit's generator per call seeds every level's feature subsets (identical on
    # the ranks of a data-parallel fit, whose generators share the seed)
    call_seed = int(torch.randint(0, 1 << 62, (1,), generator=gen, device=dev).item())
    bins_il = None
    bins_rm: Optional[torch.Tensor] = None
    # packed cells need every item's weights <= 2^20: rows per item (<= WIDE_ROWS_MAX) x max weight
    pack_scale = None
    if (regression and RF_PACK and dev.type == "cuda" and IL_KERNEL == "wide" and not deterministic()
            and float(wpos.max().item()) * WIDE_ROWS_MAX <= ops.RF_PACK_MAX_WEIGHT):
        pack_scale = ops.rf_pack_scale(yv)
    wide_fb = (ops.rf_hist_fb_wide(B, SH, regression, packed=pack_scale is not None)
               if dev.type == "cuda" and IL_KERNEL == "wide" else 0)
    wide_fb = wide_fb if wide_fb > fb and ops.rf_il_useful(n, nf, min(wide_fb, nf)) else 0
    use_il = (dev.type == "cuda" and IL_DENSITY > 0 and max_depth >= 4
              and (wide_fb > 0 or ops.rf_il_useful(n, nf, fb))
              and 3 * bins.numel() < torch.cuda.mem_get_info(dev)[0])
    # i64 fixed-point scale bounded by the heaviest tree's total bootstrap weight (no cell overflows)
    yscale = ops.rf_yscale(yv, float(tot[:, 0].max().item())) if regression and dev.type == "cuda" else None
    hist_cell = (8 if regression else 4) * nf * B * SH
    group = max(1, HIST_BUDGET_BYTES // max(hist_cell, 1))
    W = ctx.world_size
    sib_sub = RF_SIBLING_SUB and nf >= n
    scatter = data_parallel and W > 1 and RF_DP_SCATTER and not sib_sub
    prev_hist: Optional[torch.Tensor] = None  # last level's candidate histograms (cand order), summed
    prev_parent = None  # per segment: its parent's row of prev_hist
    depth = 0
    # host copies per level: ONE at the end of a level (child bounds + child totals together) and
    # ONE after the split search (split records with the winning feature ids gathered on the device)
    # per segment [leaf value(s) | weight sum | impurity], formed on the device
    stats_h = _seg_stats(tot, regression, crit).cpu().numpy()
    if LEVEL_LOG:
        LAST_LEVELS.clear()
    while len(seg_tree):
        L = len(seg_tree)
        clk = _LevelClock()
        if LEVEL_LOG:
            LAST_LEVELS.append(clk.rec)
            clk.rec.update(depth=depth, segments=int(L))
        wsum = stats_h[:, -2].copy()
        imps = stats_h[:, -1].copy()
        rec.seg.append((seg_tree.copy(), seg_nid.copy(), stats_h[:, :-2].copy(), wsum.copy(), imps))
        rec.depth = depth
        if depth >= max_depth:
            break
        cand = np.nonzero((wsum >= max(min_split, 2 * min_leaf)) & (imps > 0.0))[0]
        if cand.size == 0:
            break
        total = int(bounds_h[-1])
        # ---- histograms + split search, in groups of candidate segments bounded by memory ----
        res_out: List[np.ndarray] = []
        res_feat: List[np.ndarray] = []
        one_sync = RF_ONE_SYNC and max_leaves <= 0
        wy_lvl: Optional[torch.Tensor] = None  # (weight, class) pairs of this level's positions (fused split)
        res_out_d: List[torch.Tensor] = []  # one_sync: the groups' split records / feature ids, on the device
        res_fsel_d: List[torch.Tensor] = []
        res_left: List[torch.Tensor] = []  # classification: left-child totals of every candidate
        streamed_root = (pending is not None and depth == 0 and cand.size <= group and dev.type == "cuda"
                         and not deterministic())
        if pending is not None and not streamed_root:
            pending.finish()
            pending = None
        derive = None
        if sib_sub and prev_hist is not None and cand.size <= group and not streamed_root:
            # sibling pairs that are both candidates: histogram the one with less (global, weighted)
            # rows, derive the other (ties: derive the right child); children of split p are
            # segments 2i, 2i + 1. The totals are the all-reduced ones: every rank picks the same.
            pos = np.full(L, -1, dtype=np.int64)
            pos[cand] = np.arange(cand.size)
            sib_pos = pos[cand ^ 1]
            mine, theirs = wsum[cand], wsum[cand ^ 1]
            derive = (sib_pos >= 0) & ((mine > theirs) | ((mine == theirs) & ((cand & 1) == 1)))
        keep_hist = sib_sub and cand.size <= group
        for g0 in range(0, cand.size, group):
            cg = cand[g0: g0 + group] if derive is None else cand[~derive]
            C = int(cg.size)
            # node-partitioned reduce-scatter needs the node count padded to a multiple of W (the
            # padding nodes get no items: zero histograms, no split)
            Cp = -(-C // W) * W if scatter else C
            if nf >= n:
                feats = torch.arange(n, device=dev, dtype=torch.int32).repeat(C, 1)
            else:
                # each node's feature sample in ascending feature order (selection sampling on the
                # device): chunk c of every node then covers nearby columns of the bin matrix (see
                # the item order below) and few 32-feature records (the record-layout gathers)
                feats = ops.rf_sample_features(C, n, nf, call_seed ^ (depth * 1000003 + g0 * 7919 + 1), dev)
            c_start, c_cnt = bounds_h[cg], counts[cg]
            if streamed_root:
                hist = _root_hist_streamed(pending, bins, idx, wpos, yv, c_start, c_cnt,
                                           feats if Cp == C else _pad_rows(feats, Cp), C, B, SH, regression, fb, yscale)
                pending = None
            il = None
            rm = None
            fb_l, nfc_l, rpi_min, blocks = fb, nfc, ROWS_PER_ITEM, 8192
            # (a data-parallel level sums its histograms over the ranks: fused only on one rank)
            fused = (not regression and (not data_parallel or W == 1) and derive is None and not streamed_root
                     and dev.type == "cuda" and not deterministic() and FUSED_ROWS > 0
                     and float(c_cnt.mean()) < FUSED_ROWS and C >= FUSED_MIN_NODES and nf >= FUSED_MIN_NF
                     and ops.rf_node_split_ok(nf, B, SH))
            # nodes above FUSED_MAX_ROWS (one block each would straggle) take the unfused kernels;
            # their records are merged back by node below
            big = np.nonzero(c_cnt > FUSED_MAX_ROWS)[0] if fused else np.zeros(0, dtype=np.int64)
            if LEVEL_LOG:
                clk.rec["fused"] = bool(fused)
                clk.rec["fused_big_nodes"] = int(big.size)
            if use_il and not fused and float(c_cnt.mean()) < IL_DENSITY * m:
                if bins_il is None:
                    # built once, at the first sparse level
                    bins_il = ops.rf_interleave(bins, WIDE_REC_BYTES if wide_fb else 32)
                il = bins_il
                if wide_fb:
                    # 1024-thread blocks over ~100-400 features: fewer, longer work items
                    fb_l, rpi_min, blocks = wide_fb, WIDE_ROWS_PER_ITEM, 2048
                    nfc_l = (nf + fb_l - 1) // fb_l
            if fused or (il is None and RM_ROWS > 0 and dev.type == "cuda" and not deterministic()
                         and float(c_cnt.mean()) < RM_ROWS):
                if bins_rm is None:
                    bins_rm = ops.rf_row_major(bins)  # (m, n) row-major, built once
                rm = bins_rm
            merge = None
            if fused:
                # small nodes: histogram + split search per node in one block, nothing to HBM between
                if wy_lvl is None:
                    wy_lvl = ops.rf_hist_wy(idx, yv, None, wpos)
                se_h = np.stack([c_start, c_start + c_cnt], 1).astype(np.int32)
                se_h[big] = 0  # big nodes: empty here (records replaced below)
                se = _h2d(se_h, dev)
                clk.mark("items_host")
                out, left_c = ops.rf_node_split(rm, idx, wy_lvl, se, feats, B, SH, crit, min_leaf, min_gain)
                prev_hist = None
                if big.size:
                    # the big nodes run the unfused path below on their own (node slots 0 .. len(big))
                    big_t = _h2d(big, dev)
                    merge = (out, left_c, big_t, C, feats)
                    c_start, c_cnt, feats = c_start[big], c_cnt[big], feats.index_select(0, big_t)
                    C = Cp = int(big.size)
                else:
                    res_left.append(left_c)
            if not fused or merge is not None:
                # rows per work item: enough blocks to fill the chip, few per (node, feature chunk)
                rpi = int(min(WIDE_ROWS_MAX, max(rpi_min, (int(c_cnt.sum()) * nfc_l) // blocks)))
                rpi = (rpi + 511) // 512 * 512
                nch = (c_cnt + rpi - 1) // rpi
                tot_ch = int(nch.sum())
                node_rep = np.repeat(np.arange(C), nch)
                first = np.repeat(np.cumsum(nch) - nch, nch)
                chunk = np.arange(tot_ch) - first
                rb = c_start[node_rep] + chunk * rpi
                re = np.minimum(rb + rpi, c_start[node_rep] + c_cnt[node_rep])
                it = np.empty((tot_ch * nfc_l, 4), dtype=np.int32)
                # single-chunk nodes own their histogram cells: plain stores, no zeroing, no atomics
                single = np.where(nch[node_rep] == 1, 1 << 30, 0).astype(np.int32)
                if CHUNK_MAJOR_ITEMS:
                    # feature-chunk-major launch order: the blocks in flight at any time all read
                    # feature chunk c of their nodes — a few dozen adjacent bin columns, so every column
                    # comes from HBM about once per level and the other nodes' gathers hit L2 / MALL
                    # (node-major order streamed each node's own sample: deep levels re-read the whole
                    # matrix once per node)
                    it[:, 0] = np.tile(node_rep, nfc_l)
                    it[:, 1] = np.tile(rb, nfc_l)
                    it[:, 2] = np.tile(re, nfc_l)
                    it[:, 3] = np.repeat(np.arange(nfc_l, dtype=np.int32), tot_ch) | np.tile(single, nfc_l)
                else:
                    it[:, 0] = np.repeat(node_rep, nfc_l)
                    it[:, 1] = np.repeat(rb, nfc_l)
                    it[:, 2] = np.repeat(re, nfc_l)
                    it[:, 3] = np.tile(np.arange(nfc_l), tot_ch) | np.repeat(single, nfc_l)
                clk.mark("items_host")
                if not streamed_root:
                    items_t = _h2d(it, dev)
                    excl = ({"multi_nodes": _h2d(np.nonzero(nch != 1)[0], dev)}
                            if dev.type == "cuda" else None)
                    hist = ops.rf_hist(bins, idx, yv, None, items_t, feats if Cp == C else _pad_rows(feats, Cp),
                                       Cp, B, SH, regression, pos_weight=wpos, fb=fb_l, yscale=yscale,
                                       exclusive=excl, bins_il=il, wide=il is not None and fb_l == wide_fb,
                                       rec_bytes=WIDE_REC_BYTES if wide_fb else 32, bins_rm=rm,
                                       packed_scale=pack_scale if fb_l == wide_fb else None)
                if Cp > C:
                    hist[C:].zero_()  # padding nodes (no items; an `exclusive` histogram is not pre-zeroed)
                if scatter:
                    own = ctx.comm.reduce_scatter(hist)  # summed histograms of this rank's Cp / W nodes
                    del hist
                    out_o, _ = ops.rf_best_split(own, B, SH, regression, crit, min_leaf, min_gain)
                    recs = [out_o] if regression else [out_o, _left_totals(own, out_o)]
                    del own
                    # every rank's split records (+ left totals): a few doubles per node
                    allr = ctx.comm.allgather(torch.cat(recs, 1).contiguous())[:C]
                    out = allr[:, :6]
                    if not regression:
                        res_left.append(allr[:, 6:])
                else:
                    if data_parallel:
                        ctx.comm.allreduce(hist)  # (sibling subtraction: the built half only)
                    if derive is not None:
                        hist = _expand_siblings(hist, derive, sib_pos, prev_hist, prev_parent[cand])
                        C = int(cand.size)
                        feats = torch.arange(n, device=dev, dtype=torch.int32).repeat(C, 1)
                    out, _ = ops.rf_best_split(hist, B, SH, regression, crit, min_leaf, min_gain)
                    if not regression:
                        res_left.append(_left_totals(hist, out))
                    # (a fused level's big nodes: this histogram covers only them, not the level's
                    # candidate list that the next level's parent rows index, so nothing is kept and
                    # the next level histograms every node)
                    prev_hist = hist if keep_hist and merge is None else None
                    del hist
            if merge is not None:
                out_f, left_f, big_t, C, feats = merge
                out_f[big_t] = out
                left_f[big_t] = res_left.pop()
                out = out_f
                res_left.append(left_f)
            # the winning feature ids gathered on the device: one copy of (records | feature id)
            fsel = ops.rf_gather_feature(feats[:C], out)
            clk.mark("hist_split_launch")
            if one_sync:
                res_out_d.append(out[:C])
                res_fsel_d.append(fsel)
                continue
            rec_h = torch.cat([out, fsel], 1).cpu().numpy()
            clk.mark("split_sync")
            out_h = rec_h[:, :-1]
            res_out.append(out_h)
            ok = out_h[:, 1] >= 0
            res_feat.append(np.where(ok, rec_h[:, -1].astype(np.int64), -1))
        if one_sync:
            step = _level_one_sync(bins, idx, wpos, bounds, tot, yv, cand, L, res_out_d, res_fsel_d, res_left, S,
                                   regression, crit, data_parallel, ctx, dev, clk)
            if step is None:
                break
            idx, wpos, bounds, tot, bounds_h, stats_h, out_all, feat_all, ci_sel = step
            counts = np.diff(bounds_h)
            k = int(ci_sel.size)
            j_sel = cand[ci_sel]
            t_sel = seg_tree[j_sel]
            b_sel = out_all[ci_sel, 2].astype(np.int64)
            f_sel = feat_all[ci_sel].astype(np.int64)
            lnode, rnode = rec.add_children(t_sel)
            rec.split.append((t_sel, seg_nid[j_sel], f_sel, edges_h[f_sel, b_sel], out_all[ci_sel, 0].astype(np.float64),
                              lnode, rnode))
            np.add.at(n_leaves, t_sel, 1)
            prev_parent = np.repeat(ci_sel, 2)
            if not keep_hist:
                prev_hist = None
            seg_tree = np.repeat(t_sel, 2).astype(np.int64)
            seg_nid = np.stack([lnode, rnode], 1).reshape(-1).astype(np.int64)
            depth += 1
            continue
        out_all = np.concatenate(res_out, 0)
        feat_all = np.concatenate(res_feat, 0)
        # ---- decide splits (honour max_leaves per tree) ----
        ok = out_all[:, 1] >= 0
        order = np.nonzero(ok)[0]
        if max_leaves > 0 and order.size:
            keep = []
            by_tree: Dict[int, List[int]] = {}
            for ci in order:
                by_tree.setdefault(int(seg_tree[cand[ci]]), []).append(int(ci))
            for t_i, cis in by_tree.items():
                cis.sort(key=lambda ci: -out_all[ci, 0])
                keep += cis[: max(0, max_leaves - int(n_leaves[t_i]))]
            keep_set = set(keep)
        else:
            keep_set = None
        node_feature = np.full(L, -1, dtype=np.int32)
        node_bin = np.zeros(L, dtype=np.int32)
        child_base = np.zeros(L, dtype=np.int32)
        sel_mask = np.ones(order.size, dtype=bool) if keep_set is None else \
            np.fromiter((int(ci) in keep_set for ci in order), dtype=bool, count=order.size)
        ci_sel = order[sel_mask]
        k = int(ci_sel.size)
        if k:
            j_sel = cand[ci_sel]
            t_sel = seg_tree[j_sel]
            b_sel = out_all[ci_sel, 2].astype(np.int64)
            f_sel = feat_all[ci_sel].astype(np.int64)
            lnode, rnode = rec.add_children(t_sel)
            rec.split.append((t_sel, seg_nid[j_sel], f_sel, edges_h[f_sel, b_sel], out_all[ci_sel, 0].astype(np.float64),
                              lnode, rnode))
            node_feature[j_sel] = f_sel
            node_bin[j_sel] = b_sel
            child_base[j_sel] = 2 * np.arange(k, dtype=np.int32)
            np.add.at(n_leaves, t_sel, 1)
            new_tree = np.repeat(t_sel, 2)
            new_nid = np.stack([lnode, rnode], 1).reshape(-1)
        if k == 0:
            break
        # ---- route + stable partition into child segments ----
        clk.mark("decide_host")
        if LEVEL_LOG:
            clk.rec["candidates"] = int(cand.size)
            clk.rec["splits"] = int(k)
        meta = _h2d(np.stack([node_feature, node_bin, child_base]), dev)
        keys = ops.rf_route_segments(bins, idx, bounds, meta[0].contiguous(), meta[1].contiguous(),
                                     meta[2].contiguous())
        idx, wpos, bounds = ops.rf_partition(keys, bounds, meta[0].contiguous(), meta[2].contiguous(), k, idx, wpos,
                                             kept=int(counts[j_sel].sum()))
        if regression:
            tot = _node_stats(yv, idx, wpos, bounds, S, regression)
        else:
            # children totals: each split node's left-child totals (prefix of its winning histogram up
            # to the split bin); node_feature >= 0 segments are in cand order == split order
            left = torch.cat(res_left, 0)[_h2d(ci_sel, dev)]
            split_seg = _h2d(np.nonzero(node_feature >= 0)[0], dev)
            right = tot[split_seg] - left
            tot = torch.stack([left, right], 1).reshape(2 * k, S)
        if data_parallel and regression:
            ctx.comm.allreduce(tot)
        # one copy: child bounds (exact in fp64 below 2^53 rows) and the children's segment stats
        clk.mark("route_launch")
        hb = torch.cat([bounds.double(), _seg_stats(tot, regression, crit).reshape(-1)]).cpu().numpy()
        clk.mark("end_sync")
        bounds_h = hb[: 2 * k + 1].astype(np.int64)
        stats_h = hb[2 * k + 1:].reshape(2 * k, -1)
        counts = np.diff(bounds_h)
        prev_parent = np.repeat(ci_sel, 2)  # new segments 2i, 2i + 1 come from candidate ci_sel[i]
        if not keep_hist:
            prev_hist = None
        seg_tree = np.asarray(new_tree, dtype=np.int64)
        seg_nid = np.asarray(new_nid, dtype=np.int64)
        depth += 1
    return rec.build()


def grow_tree(bins: torch.Tensor, edges_h: np.ndarray, y: torch.Tensor, ctx: WorkerContext, gen: torch.Generator,
              p: Dict[str, Any], S: int, regression: bool, data_parallel: bool,
              gen_boot: Optional[torch.Generator] = None) -> Tree:
    return grow_forest(bins, edges_h, y, ctx, gen, p, S, regression, data_parallel, gen_boot, 1)[0]


class PendingBins:
    """Row chunks of a streamed shard whose bins are not computed yet. ``chunks()`` queues each
    chunk's quantise pass behind its DMA and yields the chunk's row range, so per-chunk consumers
    (the root-level histograms) interleave with the transfer; ``finish()`` bins whatever is left.
    Nothing is queued before the first ``chunks()`` step, so host reads issued until then do not
    wait for the transfer."""

    def __init__(self, stream: Any, edges: torch.Tensor, bins: torch.Tensor) -> None:
        self.bounds = list(stream.bounds)
        self._it = stream.chunks()
        self._edges = edges
        self._bins = bins
        self.done = False

    def chunks(self) -> Any:
        for r0, r1, Xc in self._it:
            ops.rf_quantize(Xc, self._edges, out=self._bins, col0=r0)
            yield r0, r1
        self.done = True

    def finish(self) -> None:
        if not self.done:
            for _ in self.chunks():
                pass


def quantize_features(X: torch.Tensor, n_bins: int, ctx: WorkerContext, m_total: int, seed: int,
                      stream: Any = None, defer: bool = False) -> Tuple[Any, ...]:
    """(feature-major uint8 bins, host fp64 edges) of the shard: the quantile binning every tree
    of a fit shares (and every param map of a fitMultiple with the same maxBins / seed).

    ``stream`` (``ops.ingest.StreamedRows`` of a pinned shard still in flight): the edges come from
    host-gathered sample rows and every row chunk is binned as soon as its DMA lands, so the
    binning pass runs under the PCIe transfer instead of after it (same rows, same edges, same
    bins as the in-memory path). ``defer`` (streamed only): return (bins, edges, PendingBins) with
    the chunks not yet binned — the caller consumes them (or calls ``finish()``) before reading
    the bins."""
    if n_bins > 256:
        raise ValueError("maxBins > 256 is not supported (uint8 bins)")
    host = getattr(stream, "host", None) if stream is not None else None
    if host is not None and X.is_cuda and X.dtype == torch.float32 and host.dtype == torch.float32:
        edges = bin_edges(X, n_bins, ctx, m_total, seed, host=host)
        edges_h = edges.double().cpu().numpy()  # waits for the sample only: no chunk work is queued yet
        m, n = X.shape
        bins = torch.empty((n, m), dtype=torch.uint8, device=X.device)
        pending = PendingBins(stream, edges, bins)
        if defer:
            return bins, edges_h, pending
        pending.finish()
        return bins, edges_h
    if stream is not None:
        stream.wait_all()
    edges = bin_edges(X, n_bins, ctx, m_total, seed)
    bins = ops.rf_quantize(X, edges)
    return bins, edges.double().cpu().numpy()


def fit_forest(X: torch.Tensor, y: torch.Tensor, ctx: WorkerContext, m_total: int, p: Dict[str, Any],
               n_trees_local: int, classification: bool, num_classes: int, data_parallel: bool,
               rank_seed: int, binned: Optional[Tuple[torch.Tensor, np.ndarray]] = None) -> List[Dict[str, Any]]:
    m, n = X.shape
    n_bins = int(p["n_bins"])
    seed = int(p["random_state"]) if p.get("random_state") is not None else 0
    bins, edges_h, *rest = binned if binned is not None else quantize_features(X, n_bins, ctx, m_total, seed)
    pending = rest[0] if rest else None  # streamed chunks not binned yet: the first batch's root level bins them
    S = num_classes if classification else 3
    # feature-subset RNG: shared by all ranks in data-parallel mode (same trees everywhere);
    # bootstrap RNG: always rank-specific (each rank bags its own rows)
    gen = torch.Generator(device=X.device)
    gen.manual_seed((int(seed) if data_parallel else int(rank_seed)) & 0x7FFFFFFFFFFF)
    gen_boot = torch.Generator(device=X.device)
    gen_boot.manual_seed((int(rank_seed) * 31 + 17) & 0x7FFFFFFFFFFF)
    trees: List[Dict[str, Any]] = []
    # trees per batch: positions + weights cost ~8 B per in-bag row and tree
    per_batch = max(1, int((4 << 30) // max(8 * m, 1)))
    try:
        for t0 in range(0, n_trees_local, per_batch):
            nt = min(per_batch, n_trees_local - t0)
            for t in grow_forest(bins, edges_h, y, ctx, gen, p, S, not classification, data_parallel, gen_boot, nt,
                                 pending=pending):
                trees.append(t.to_dict())
            if pending is not None:
                pending.finish()
                pending = None
    finally:
        # a rank with no trees of its own (numTrees < world size) never enters the loop: the shared
        # bins (reused by later param maps with the same maxBins / seed) must still be complete;
        # finishing also makes the current stream wait on every chunk's copy event, so later
        # readers of X (another quantisation key, a transform) never race the DMA
        if pending is not None:
            pending.finish()
    return trees


def pack_forest(trees: List[Dict[str, Any]], S: int, device: torch.device) -> Dict[str, torch.Tensor]:
    """Flatten trees (node lists or arrays) into the breadth-first device arrays of ``rf_predict``."""
    feats, thr, left, right, voff, vals, roots = [], [], [], [], [], [], []
    base = 0
    for t in trees:
        f = np.asarray(t["feature"], dtype=np.int64).reshape(-1)
        nn_ = f.shape[0]
        roots.append(base)
        feats.append(f)
        thr.append(np.asarray(t["threshold"], dtype=np.float64).reshape(-1))
        lt = np.asarray(t["left"], dtype=np.int64).reshape(-1)
        rt = np.asarray(t["right"], dtype=np.int64).reshape(-1)
        left.append(np.where(lt >= 0, lt + base, -1))
        right.append(np.where(rt >= 0, rt + base, -1))
        v = np.zeros((nn_, S))
        if nn_:
            tv = np.asarray(t["value"], dtype=np.float64).reshape(nn_, -1)[:, :S]
            v[:, : tv.shape[1]] = tv
        vals.append(v.reshape(-1))
        base += nn_
    cat = lambda parts, dt: np.concatenate(parts).astype(dt) if parts else np.zeros(0, dt)  # noqa: E731
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(device)  # noqa: E731
    f_all, thr_all = cat(feats, np.int32), cat(thr, np.float32)
    l_all, r_all = cat(left, np.int32), cat(right, np.int32)
    voff = (np.arange(base, dtype=np.int64) * S).astype(np.int32)
    # 16-B node records for the wave-per-row kernel: splits {feature, left, right, thr bits},
    # leaves {-1, value offset, leaf id within its tree, 0}
    local = np.concatenate([np.arange(len(f), dtype=np.int32) for f in feats]) if feats else np.zeros(0, np.int32)
    leaf = f_all < 0
    nodes = np.zeros((base, 4), dtype=np.int32)
    nodes[:, 0] = np.where(leaf, -1, f_all)
    nodes[:, 1] = np.where(leaf, voff, l_all)
    nodes[:, 2] = np.where(leaf, local, r_all)
    nodes[:, 3] = np.where(leaf, 0, thr_all.view(np.int32))
    return {
        "roots": i32(np.asarray(roots, dtype=np.int32)), "feature": i32(f_all),
        "threshold": torch.from_numpy(thr_all).to(device),
        "left": i32(l_all), "right": i32(r_all),
        "value_off": i32(voff),
        "values": torch.from_numpy(cat(vals, np.float32)).to(device),
        "nodes": i32(nodes),
    }


def forest_predict(X: torch.Tensor, packed: Dict[str, torch.Tensor], S: int, want_leaves: bool = False
                   ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    return ops.rf_predict(X.float(), packed["roots"], packed["feature"], packed["threshold"], packed["left"],
                          packed["right"], packed["value_off"], packed["values"], S, want_leaves,
                          nodes=packed.get("nodes"))


def feature_importances(trees: List[Dict[str, Any]], n: int) -> np.ndarray:
    """Spark's definition: per tree, sum over split nodes of gain * count, normalised; averaged and
    renormalised over the forest."""
    total = np.zeros(n)
    for t in trees:
        imp = np.zeros(n)
        f = np.asarray(t["feature"], dtype=np.int64)
        split = f >= 0
        np.add.at(imp, f[split], (np.asarray(t["gain"], dtype=np.float64) * np.asarray(t["count"], dtype=np.float64))[split])
        s = imp.sum()
        if s > 0:
            total += imp / s
    s = total.sum()
    return total / s if s > 0 else total
