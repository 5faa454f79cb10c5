"""Synthetic benchmark data generated directly on the device (one shard per rank).

Same distribution families as the reference generators (``python/benchmark/gen_data.py``,
``gen_data_distributed.py`` — SURVEY Appendix D): ``low_rank_matrix`` (bell + tail singular
profile, effective_rank 10, tail_strength 0.5), ``regression`` (N(0,1) features, sparse
informative ground truth ~100·U(0,1), Gaussian noise), ``classification`` (hypercube-vertex
class clusters over informative features + linear redundant features + noise), ``uniform``
(``RandomRDDs.uniformVectorRDD``) and ``blobs``. Generating on the GPU keeps 1M x 3000 shards
to a second instead of minutes of host RNG; the result is copied once into pinned host memory
(``to_pinned_numpy``) so that the timed fit starts from host-resident "Arrow" data like a
Spark executor's batches.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch


def _gen(device: torch.device, seed: int) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def low_rank_matrix(m: int, n: int, device: torch.device, seed: int = 0, effective_rank: int = 10,
                    tail_strength: float = 0.5, rank_cap: int = 256, m_total: Optional[int] = None) -> torch.Tensor:
    g = _gen(device, seed)
    r = min(n, rank_cap)
    i = torch.arange(r, device=device, dtype=torch.float32)
    low = (1 - tail_strength) * torch.exp(-1.0 * (i / effective_rank) ** 2)
    tail = tail_strength * torch.exp(-0.1 * i / effective_rank)
    s = low + tail
    # V: orthonormal rows shared by every rank (seeded identically)
    gv = _gen(device, 12345)
    V, _ = torch.linalg.qr(torch.randn(n, r, device=device, generator=gv, dtype=torch.float32))
    U = torch.randn(m, r, device=device, generator=g, dtype=torch.float32) / float(np.sqrt(m_total or m))
    return (U * s) @ V.T


def regression(m: int, n: int, device: torch.device, seed: int = 0, n_informative: int = 10,
               noise: float = 0.0, bias: float = 0.0, n_targets: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """sklearn ``make_regression`` semantics with its defaults, as the reference's generators use
    them (``gen_data.py:339-392`` passes no ``n_informative`` -> 10; ``gen_data_distributed.py:364``
    defaults it to 10; noise 0 and bias 0 unless the workload's script sets them, e.g. ``--noise 10``
    for the linear-regression data, ``run_benchmark.sh:251-260``): N(0, 1) features, ground truth
    100 U(0, 1) on ``n_informative`` random columns (shared by every partition; the random column
    choice is sklearn's column shuffle), ``y = X w + bias + N(0, noise^2)``. Rows are i.i.d., so
    sklearn's row shuffle changes nothing. ``n_targets > 1`` gives an (m, T) target (the
    multinomial-logistic ground truth of ``gen_data_distributed.py:445-455``)."""
    g = _gen(device, seed)
    X = torch.randn(m, n, device=device, generator=g, dtype=torch.float32)
    gw = _gen(device, 777)
    k = max(1, min(int(n_informative), n))
    w = torch.zeros(n, n_targets, device=device)
    idx = torch.randperm(n, device=device, generator=gw)[:k]
    w[idx] = 100.0 * torch.rand(k, n_targets, device=device, generator=gw)
    y = X @ w + bias
    if noise > 0.0:
        y = y + noise * torch.randn(y.shape, device=device, generator=g)
    return X, (y[:, 0] if n_targets == 1 else y)


def logistic_labels(y: torch.Tensor, seed: int) -> torch.Tensor:
    """The reference's ``--logistic_regression`` labels (``gen_data_distributed.py:513-537``):
    binary ``Bernoulli(sigmoid(y))`` of the UNSCALED linear target, or for an (m, C) target a
    class sampled from ``softmax(y)`` (uniform anchor against the cumulative probabilities)."""
    g = _gen(y.device, seed + 7919)
    if y.dim() == 1:
        return torch.bernoulli(torch.sigmoid(y.double()), generator=g).float()
    cdf = torch.softmax(y.double(), dim=1).cumsum(1)
    anchor = torch.rand(y.shape[0], 1, device=y.device, generator=g, dtype=torch.float64)
    return (anchor > cdf).sum(1).clamp_max(y.shape[1] - 1).float()


_CLS_SHARED: Dict[Tuple[Any, ...], Tuple[np.ndarray, List[np.ndarray], Optional[np.ndarray], Optional[np.ndarray]]] = {}


def classification_shared(n: int, n_informative: int, n_redundant: int, n_classes: int = 2,
                          n_clusters_per_class: int = 2, class_sep: float = 1.0, random_state: int = 1,
                          shuffle: bool = True
                          ) -> Tuple[np.ndarray, List[np.ndarray], Optional[np.ndarray], Optional[np.ndarray]]:
    """What every partition of the reference's distributed ``make_classification`` shares, drawn
    from ONE ``RandomState(random_state)`` in the reference's order
    (``gen_data_distributed.py:1047-1075``): hypercube-vertex centroids (scaled to +-class_sep),
    one random covariance ``A_k = 2 U(n_inf, n_inf) - 1`` per cluster, the redundant mix
    ``B = 2 U(n_inf, n_red) - 1`` (no rescaling) and the column shuffle. Shift 0 / scale 1 (the
    reference's defaults) draw nothing. Cached: the bench draws its train and holdout shards from
    the same parameters."""
    key = (n, n_informative, n_redundant, n_classes, n_clusters_per_class, float(class_sep), int(random_state),
           bool(shuffle))
    hit = _CLS_SHARED.get(key)
    if hit is not None:
        return hit
    from sklearn.datasets._samples_generator import _generate_hypercube

    if n_informative + n_redundant > n:
        raise ValueError("Number of informative and redundant features must sum to less than the number of features")
    n_clusters = n_classes * n_clusters_per_class
    if n_informative < np.log2(n_clusters):
        raise ValueError("n_classes * n_clusters_per_class must be smaller or equal 2**n_informative")
    gen = np.random.RandomState(int(random_state))
    centroids = _generate_hypercube(n_clusters, n_informative, gen).astype(np.float64, copy=False)
    centroids = centroids * (2 * class_sep) - class_sep
    A = [2 * gen.uniform(size=(n_informative, n_informative)) - 1 for _ in range(n_clusters)]
    B = 2 * gen.uniform(size=(n_informative, n_redundant)) - 1 if n_redundant > 0 else None
    cols = None
    if shuffle:
        cols = np.arange(n)
        gen.shuffle(cols)
    _CLS_SHARED.clear()  # one parameter set at a time (4 x n_inf^2 doubles at the headline shape)
    _CLS_SHARED[key] = (centroids, A, B, cols)
    return _CLS_SHARED[key]


def classification(m: int, n: int, device: torch.device, seed: int = 0, n_classes: int = 2,
                   n_informative: Optional[int] = None, n_redundant: Optional[int] = None,
                   class_sep: float = 1.0, flip_y: float = 0.01, n_clusters_per_class: int = 2,
                   random_state: int = 1, shuffle: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """One partition (``m`` rows, partition seed ``seed``) of the reference's distributed
    ``make_classification`` (``gen_data_distributed.py:1088-1151``), generated on the device:
    balanced clusters (labels ``k % n_classes``), informative features ``z A_k + centroid_k`` with
    ``z ~ N(0, I)``, redundant features ``X_inf B``, N(0, 1) useless features, ``flip_y`` label
    noise, then the partition's rows and the shared columns shuffled. Defaults follow the
    reference benchmark (``run_benchmark.sh``: n_informative = n_redundant = n / 3)."""
    g = _gen(device, seed)
    ni = n_informative if n_informative is not None else max(1, n // 3)
    nr = n_redundant if n_redundant is not None else max(0, n // 3)
    ni = min(ni, n)
    nr = min(nr, n - ni)
    centroids, A, B, cols = classification_shared(n, ni, nr, n_classes, n_clusters_per_class, class_sep,
                                                  random_state, shuffle)
    n_clusters = len(A)
    per = [m // n_clusters] * n_clusters
    for i in range(m - sum(per)):
        per[i % n_clusters] += 1
    X = torch.empty(m, n, device=device, dtype=torch.float32)
    y = torch.empty(m, device=device, dtype=torch.int64)
    Xi = torch.randn(m, ni, device=device, generator=g, dtype=torch.float32)
    stop = 0
    for k in range(n_clusters):
        start, stop = stop, stop + per[k]
        y[start:stop] = k % n_classes
        Ak = torch.from_numpy(A[k]).to(device=device, dtype=torch.float32)
        ck = torch.from_numpy(centroids[k]).to(device=device, dtype=torch.float32)
        X[start:stop, :ni] = torch.addmm(ck, Xi[start:stop], Ak)
    del Xi
    if nr > 0:
        X[:, ni: ni + nr] = X[:, :ni] @ torch.from_numpy(B).to(device=device, dtype=torch.float32)
    if ni + nr < n:
        X[:, ni + nr:] = torch.randn(m, n - ni - nr, device=device, generator=g)
    if flip_y >= 0.0:
        flip = torch.rand(m, device=device, generator=g) < flip_y
        y = torch.where(flip, torch.randint(0, n_classes, (m,), device=device, generator=g), y)
    if shuffle:
        perm = torch.randperm(m, device=device, generator=g)
        X = X.index_select(0, perm).index_select(1, torch.from_numpy(cols).to(device))
        y = y[perm]
    return X, y.float()


def uniform(m: int, n: int, device: torch.device, seed: int = 0) -> torch.Tensor:
    return torch.rand(m, n, device=device, generator=_gen(device, seed), dtype=torch.float32)


def blobs(m: int, n: int, device: torch.device, seed: int = 0, centers: int = 20,
          cluster_std: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
    g = _gen(device, seed)
    gc = _gen(device, 4242)
    C = (torch.rand(centers, n, device=device, generator=gc) * 20 - 10)
    lab = torch.randint(0, centers, (m,), device=device, generator=g)
    X = C[lab] + cluster_std * torch.randn(m, n, device=device, generator=g)
    return X, lab.float()


def to_pinned_numpy(t: torch.Tensor) -> np.ndarray:
    """Device tensor -> numpy array backed by pinned host memory (fast H2D path in ingest)."""
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=torch.cuda.is_available())
    h.copy_(t)
    return h.numpy()


def sparse_density_values(density: Any, density_curve: str, n_chunks: int, cols: int, rows: int,
                          num_partitions: int) -> np.ndarray:
    """Per-column-chunk target densities (reference gen_data_distributed.py:672-723): a scalar or
    list of densities, or a Linear / Exponential curve from ~1 nnz per partition up to ``density``,
    rescaled so the average stays ``density``; values above 1 are cropped."""
    if density_curve not in ("None", None, ""):
        d = float(density[0] if isinstance(density, (list, tuple)) else density)
        n_chunks = min(int(n_chunks), cols)
        lo = num_partitions / float(rows)
        if density_curve == "Linear":
            vals = np.linspace(lo, d, n_chunks)
        elif density_curve == "Exponential":
            vals = np.logspace(np.log10(lo), np.log10(d), n_chunks)
        else:
            raise ValueError("Unsupported density curve %r (None | Linear | Exponential)" % density_curve)
        vals = vals * (n_chunks * d / vals.sum())
    else:
        vals = np.asarray(density if isinstance(density, (list, tuple)) else [density], dtype=np.float64)
    return np.minimum(vals, 1.0)


def sparse_regression(rows: int, cols: int, seed: int = 1, partition_seed: int = 1, density: Any = 0.1,
                      density_curve: str = "None", n_chunk: int = 10, redundant_cols: int = 0,
                      n_informative: int = 10, noise: float = 0.0, bias: Any = 0.0, shuffle: bool = True,
                      logistic_regression: bool = False, n_classes: int = 2, num_partitions: int = 1,
                      dtype=np.float64) -> Tuple[Any, np.ndarray, np.ndarray]:
    """One partition of the reference's ``SparseRegressionDataGen`` (gen_data_distributed.py:581-944)
    generated directly in CSR (no dense m x n intermediate): per column chunk a scipy random sparse
    block at that chunk's density, optional redundant columns = informative columns x U(0,1)
    mixing, the shared column shuffle, y = X w + bias (+ noise), logistic / multinomial sampling.

    ``seed`` fixes what every partition shares (ground truth, column order); ``partition_seed`` the
    rows of this partition. Returns (X csr_matrix (rows, cols), y ndarray, ground_truth)."""
    import scipy.sparse as sp

    gen = np.random.RandomState(seed)
    multinomial = logistic_regression and n_classes > 2
    orig_cols = cols - int(redundant_cols)
    dens = sparse_density_values(density, density_curve, n_chunk, orig_cols, rows, num_partitions)
    if (redundant_cols > 0 and density_curve in ("None", None, "")
            and redundant_cols / cols > float(np.mean(dens))):
        redundant_cols, orig_cols = 0, cols  # the reference drops them: they would break the density
    nt = n_classes if multinomial else 1
    n_informative = min(int(n_informative), orig_cols)
    truth = np.zeros((cols, nt))
    truth[:n_informative, :] = 100 * gen.uniform(size=(n_informative, nt))
    col_idx = np.arange(cols)
    if shuffle:
        gen.shuffle(col_idx)
        truth = truth[col_idx]
    pg = np.random.RandomState(partition_seed)
    nch = len(dens)
    per = np.full(nch, orig_cols // nch)
    per[: orig_cols % nch] += 1
    blocks = []
    if redundant_cols > 0 and density_curve in ("None", None, ""):
        d0 = float(dens[0])
        blocks.append(sp.random(rows, orig_cols, density=(d0 - redundant_cols / cols) / (1 - redundant_cols / cols),
                                random_state=pg, format="csr", dtype=dtype, data_rvs=pg.standard_normal))
    else:
        for c, d in zip(per, dens):
            blocks.append(sp.random(rows, int(c), density=float(d), random_state=pg, format="csr", dtype=dtype,
                                    data_rvs=pg.standard_normal))
    X = sp.hstack(blocks, format="csr") if len(blocks) > 1 else blocks[0]
    if redundant_cols > 0:
        mix = pg.random_sample((n_informative, int(redundant_cols)))
        red = sp.csr_matrix(X[:, :n_informative] @ mix)
        X = sp.hstack([X, red], format="csr")
    if shuffle:
        X = X[:, col_idx]
    X.sum_duplicates()
    X.sort_indices()
    y = np.asarray(X @ truth) + (np.asarray(bias, dtype=np.float64) if multinomial else float(np.ravel(bias)[0]
                                                                                              if np.ndim(bias) else bias))
    if noise > 0.0:
        y = y + pg.normal(scale=noise, size=y.shape)
    if logistic_regression:
        if multinomial:
            z = y - y.max(1, keepdims=True)
            p = np.exp(z)
            p /= p.sum(1, keepdims=True)
            y = (pg.random_sample((rows, 1)) > np.cumsum(p, 1)).sum(1).astype(np.float64)
        else:
            y = pg.binomial(1, 1.0 / (1.0 + np.exp(-y[:, 0]))).astype(np.float64)
    else:
        y = y[:, 0]
    return X.astype(dtype), y, np.squeeze(truth)
