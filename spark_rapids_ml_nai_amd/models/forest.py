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

import json
import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext

ROWS_PER_ITEM = 4096
INT_MAX = 2**31 - 1


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
              sample_rows: int = 1 << 16) -> torch.Tensor:
    """(n, n_bins-1) fp32 quantile edges, identical on every rank (sampled rows all-gathered)."""
    m, n = X.shape
    g = torch.Generator(device="cpu")
    g.manual_seed(int(seed) * 7919 + ctx.rank)
    want = max(1, int(round(sample_rows * m / max(m_total, 1))))
    if m > want:
        sel = torch.randperm(m, generator=g)[:want].sort().values.to(X.device)
        S = X.index_select(0, sel).float()
    else:
        S = X.float()
    if ctx.world_size > 1:
        S = torch.cat([p.to(X.device) for p in ctx.comm.allgatherv(S.contiguous())], 0)
    Ss, _ = torch.sort(S, 0)
    k = Ss.shape[0]
    q = torch.arange(1, n_bins, device=X.device, dtype=torch.float64) / n_bins
    pos = (q * k).long().clamp(0, k - 1)
    E = Ss.index_select(0, pos).T.contiguous()  # (n, B-1), non-decreasing per feature
    return E


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

    def add_node(self) -> int:
        self.feature.append(-1)
        self.threshold.append(0.0)
        self.left.append(-1)
        self.right.append(-1)
        self.value.append([])
        self.impurity.append(0.0)
        self.gain.append(0.0)
        self.count.append(0.0)
        return len(self.feature) - 1

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


def _leaf_value(tot: np.ndarray, regression: bool) -> List[float]:
    if regression:
        return [float(tot[1] / tot[0]) if tot[0] > 0 else 0.0]
    s = tot.sum()
    return [float(v / s) if s > 0 else 0.0 for v in tot]


def _impurity_np(tot: np.ndarray, crit: int) -> float:
    if crit == 2:
        n = tot[0]
        if n <= 0:
            return 0.0
        mu = tot[1] / n
        return float(max(tot[2] / n - mu * mu, 0.0))
    n = tot.sum()
    if n <= 0:
        return 0.0
    p = tot / n
    if crit == 0:
        return float(1.0 - (p * p).sum())
    nz = p[p > 0]
    return float(-(nz * np.log2(nz)).sum())


def grow_tree(bins: torch.Tensor, edges_h: np.ndarray, y: torch.Tensor, ctx: WorkerContext, gen: torch.Generator,
              p: Dict[str, Any], S: int, regression: bool, data_parallel: bool,
              gen_boot: Optional[torch.Generator] = None) -> Tree:
    dev = bins.device
    n, m = bins.shape
    B = edges_h.shape[1] + 1
    crit = {"gini": 0, "entropy": 1, "variance": 2, "mse": 2}[p["split_criterion"]]
    max_depth = int(p["max_depth"])
    min_leaf = float(p["min_samples_leaf"])
    min_split = float(p["min_samples_split"])
    min_gain = float(p.get("min_impurity_decrease", 0.0))
    nf = int(p["_nf"])
    max_leaves = int(p.get("max_leaves", -1))
    # bootstrap multiplicities (Spark: Poisson(subsamplingRate) bagging)
    if p["bootstrap"]:
        rate = float(p.get("max_samples", 1.0))
        w = torch.poisson(torch.full((m,), rate, device=dev), generator=gen_boot or gen).clamp_max(255).to(torch.uint8)
    else:
        w = torch.ones(m, dtype=torch.uint8, device=dev)
    idx = torch.nonzero(w, as_tuple=False).view(-1).to(torch.int32)
    yv = y.float()
    tree = Tree()
    root = tree.add_node()
    # level state: tree node ids, segment starts/counts (host)
    level_nodes = [root]
    starts = np.array([0], dtype=np.int64)
    counts = np.array([int(idx.shape[0])], dtype=np.int64)
    depth = 0
    n_leaves = 1
    # root totals (weighted class counts / regression moments); deeper levels inherit their
    # totals from the parent's winning split (prefix of its histogram), no pass over the rows
    wr = w[idx.long()].double()
    if regression:
        yr = yv[idx.long()].double()
        tot = torch.stack([wr.sum(), (wr * yr).sum(), (wr * yr * yr).sum()]).view(1, 3)
    else:
        tot = torch.bincount(yv[idx.long()].long(), weights=wr, minlength=S)[:S].double().view(1, S)
    if data_parallel:
        ctx.comm.allreduce(tot)
    nfc = (nf + 7) // 8
    while level_nodes:
        L = len(level_nodes)
        total = int(counts.sum())
        seg_node = torch.repeat_interleave(torch.arange(L, device=dev, dtype=torch.int32),
                                           torch.from_numpy(counts).to(dev))
        tot_h = tot.cpu().numpy()
        wsum = tot_h[:, 0] if regression else tot_h.sum(1)
        for j, nid in enumerate(level_nodes):
            tree.value[nid] = _leaf_value(tot_h[j], regression)
            tree.count[nid] = float(wsum[j])
            tree.impurity[nid] = _impurity_np(tot_h[j], crit)
        tree.depth = depth
        if depth >= max_depth:
            break
        cand = [j for j in range(L) if wsum[j] >= max(min_split, 2 * min_leaf) and tree.impurity[level_nodes[j]] > 0.0]
        if not cand:
            break
        # feature subsets (device RNG; identical on all ranks in data-parallel mode)
        C = len(cand)
        if nf >= n:
            feats = torch.arange(n, device=dev, dtype=torch.int32).repeat(C, 1)
        else:
            feats = torch.rand((C, n), generator=gen, device=dev).argsort(1)[:, :nf].to(torch.int32).contiguous()
        # work items (node slot, row begin, row end, feature chunk), built vectorised
        cand_a = np.asarray(cand, dtype=np.int64)
        c_start, c_cnt = starts[cand_a], counts[cand_a]
        # rows per work item: enough blocks to fill the chip (~8K) but as few per (node, feature
        # chunk) as possible — every block flushes its LDS histogram with global fp64 atomics
        rpi = int(min(65536, max(ROWS_PER_ITEM, (int(c_cnt.sum()) * nfc) // 8192)))
        rpi = (rpi + 511) // 512 * 512
        nch = (c_cnt + rpi - 1) // rpi
        tot_ch = int(nch.sum())
        if tot_ch:
            node_rep = np.repeat(np.arange(C), nch)
            first = np.repeat(np.cumsum(nch) - nch, nch)
            chunk = np.arange(tot_ch) - first
            rb = c_start[node_rep] + chunk * rpi
            re = np.minimum(rb + rpi, c_start[node_rep] + c_cnt[node_rep])
            it = np.empty((tot_ch * nfc, 4), dtype=np.int32)
            it[:, 0] = np.repeat(node_rep, nfc)
            it[:, 1] = np.repeat(rb, nfc)
            it[:, 2] = np.repeat(re, nfc)
            it[:, 3] = np.tile(np.arange(nfc), tot_ch)
            items_t = torch.from_numpy(it).to(dev)
        else:
            items_t = torch.zeros((0, 4), dtype=torch.int32, device=dev)
        SH = 2 if regression else S  # regression histograms carry (count, sum) only
        hist = ops.rf_hist(bins, idx, yv, w, items_t, feats, C, B, SH, regression)
        if data_parallel:
            ctx.comm.allreduce(hist)
        out, _ = ops.rf_best_split(hist, B, SH, regression, crit, min_leaf, min_gain)
        out_h = out.cpu().numpy()
        feats_h = feats.cpu().numpy()
        # honour max_leaves: keep the best-gain splits that fit
        order = [ci for ci in range(C) if out_h[ci, 1] >= 0]
        if max_leaves > 0:
            order.sort(key=lambda ci: -out_h[ci, 0])
            order = order[: max(0, max_leaves - n_leaves)]
        split_set = set(order)
        node_feature = np.full(L, -1, dtype=np.int32)
        node_bin = np.zeros(L, dtype=np.int32)
        child_base = np.zeros(L, dtype=np.int32)
        next_nodes: List[int] = []
        k = 0
        split_ci: List[int] = []
        split_slot: List[int] = []
        split_bin: List[int] = []
        split_j: List[int] = []
        for ci, j in enumerate(cand):
            if ci not in split_set:
                continue
            split_ci.append(ci)
            split_slot.append(int(out_h[ci, 1]))
            split_bin.append(int(out_h[ci, 2]))
            split_j.append(j)
            nid = level_nodes[j]
            slot = int(out_h[ci, 1])
            b = int(out_h[ci, 2])
            f = int(feats_h[ci, slot])
            tree.feature[nid] = f
            tree.threshold[nid] = float(edges_h[f, b])
            tree.gain[nid] = float(out_h[ci, 0])
            lnode, rnode = tree.add_node(), tree.add_node()
            tree.left[nid], tree.right[nid] = lnode, rnode
            next_nodes += [lnode, rnode]
            node_feature[j] = f
            node_bin[j] = b
            child_base[j] = 2 * k
            k += 1
            n_leaves += 1
        if k == 0:
            break
        if not regression:
            # children totals = prefix of the winning feature's histogram up to the split bin
            ci_t = torch.tensor(split_ci, device=dev)
            sel = hist[ci_t, torch.tensor(split_slot, device=dev)].double()  # (k, B, S)
            left = sel.cumsum(1)[torch.arange(k, device=dev), torch.tensor(split_bin, device=dev)]
            right = tot[torch.tensor(split_j, device=dev)] - left
            tot = torch.stack([left, right], 1).reshape(2 * k, S)
        keys = ops.rf_route(bins, idx[:total].contiguous(), seg_node.contiguous(),
                            torch.from_numpy(node_feature).to(dev), torch.from_numpy(node_bin).to(dev),
                            torch.from_numpy(child_base).to(dev))
        keys_sorted, perm = torch.sort(keys, stable=True)
        kept = int((keys_sorted != INT_MAX).sum().item())
        idx = idx[:total][perm[:kept]].contiguous()
        # child segment boundaries in the sorted key order (no atomics: keys are sorted)
        bounds = torch.searchsorted(keys_sorted[:kept].contiguous(),
                                    torch.arange(2 * k + 1, device=dev, dtype=keys_sorted.dtype))
        if regression:
            # children (count, sum, sumsq) as segment sums over the routed rows (histograms hold no
            # sum of squares): one cumsum + boundary gathers
            rows = idx.long()
            wr = w[rows].double()
            yr = yv[rows].double()
            # (3, N) row-contiguous scans: torch's outer-dim scan of an (N, 3) tensor is ~100x slower
            v = torch.stack([wr, wr * yr, wr * yr * yr], 0)
            cs = torch.cat([torch.zeros((3, 1), dtype=torch.float64, device=dev), v.cumsum(1)], 1)
            tot = (cs[:, bounds[1:]] - cs[:, bounds[:-1]]).T.contiguous()
            if data_parallel:
                ctx.comm.allreduce(tot)
        cnt = (bounds[1:] - bounds[:-1]).cpu().numpy().astype(np.int64)
        counts = cnt
        starts = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
        level_nodes = next_nodes
        depth += 1
    return tree


def fit_forest(X: torch.Tensor, y: torch.Tensor, ctx: WorkerContext, m_total: int, p: Dict[str, Any],
               n_trees_local: int, classification: bool, num_classes: int, data_parallel: bool,
               rank_seed: int) -> List[Dict[str, Any]]:
    m, n = X.shape
    n_bins = int(p["n_bins"])
    if n_bins > 256:
        raise ValueError("maxBins > 256 is not supported (uint8 bins)")
    seed = int(p["random_state"]) if p.get("random_state") is not None else 0
    edges = bin_edges(X, n_bins, ctx, m_total, seed)
    bins = ops.rf_quantize(X, edges)
    edges_h = edges.double().cpu().numpy()
    S = num_classes if classification else 3
    # feature-subset RNG: shared by all ranks in data-parallel mode (same trees everywhere);
    # bootstrap RNG: always rank-specific (each rank bags its own rows)
    gen = torch.Generator(device=X.device)
    gen.manual_seed((int(seed) if data_parallel else int(rank_seed)) & 0x7FFFFFFFFFFF)
    gen_boot = torch.Generator(device=X.device)
    gen_boot.manual_seed((int(rank_seed) * 31 + 17) & 0x7FFFFFFFFFFF)
    trees = []
    for _ in range(n_trees_local):
        t = grow_tree(bins, edges_h, y, ctx, gen, p, S, not classification, data_parallel, gen_boot)
        trees.append(t.to_dict())
    del bins
    return trees


def pack_forest(trees: List[Dict[str, Any]], S: int, device: torch.device) -> Dict[str, torch.Tensor]:
    feats, thr, left, right, voff, vals, roots = [], [], [], [], [], [], []
    base = 0
    vbase = 0
    for t in trees:
        nn_ = len(t["feature"])
        roots.append(base)
        feats.extend(t["feature"])
        thr.extend(t["threshold"])
        left.extend([(l + base) if l >= 0 else -1 for l in t["left"]])
        right.extend([(r + base) if r >= 0 else -1 for r in t["right"]])
        for v in t["value"]:
            vv = list(v) + [0.0] * (S - len(v))
            voff.append(vbase)
            vals.extend(vv[:S])
            vbase += S
        base += nn_
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=device)
    return {
        "roots": i32(roots), "feature": i32(feats), "threshold": torch.tensor(thr, dtype=torch.float32, device=device),
        "left": i32(left), "right": i32(right), "value_off": i32(voff),
        "values": torch.tensor(vals, dtype=torch.float32, device=device),
    }


def forest_predict(X: torch.Tensor, packed: Dict[str, torch.Tensor], S: int, want_leaves: bool = False
                   ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    return ops.rf_predict(X.float(), packed["roots"], packed["feature"], packed["threshold"], packed["left"],
                          packed["right"], packed["value_off"], packed["values"], S, want_leaves)


def feature_importances(trees: List[Dict[str, Any]], n: int) -> np.ndarray:
    """Spark's definition: per tree, sum over split nodes of gain * count, normalised; averaged and
    renormalised over the forest."""
    total = np.zeros(n)
    for t in trees:
        imp = np.zeros(n)
        for f, g, c in zip(t["feature"], t["gain"], t["count"]):
            if f >= 0:
                imp[f] += g * c
        s = imp.sum()
        if s > 0:
            total += imp / s
    s = total.sum()
    return total / s if s > 0 else total
