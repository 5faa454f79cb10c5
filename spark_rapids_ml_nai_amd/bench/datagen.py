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

from typing import Any, Optional, Tuple

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


def regression(m: int, n: int, device: torch.device, seed: int = 0, n_informative: Optional[int] = None,
               noise: float = 1.0, bias: float = 0.0) -> Tuple[torch.Tensor, torch.Tensor]:
    g = _gen(device, seed)
    X = torch.randn(m, n, device=device, generator=g, dtype=torch.float32)
    gw = _gen(device, 777)
    k = n_informative or max(1, n // 10)
    w = torch.zeros(n, device=device)
    idx = torch.randperm(n, device=device, generator=gw)[:k]
    w[idx] = 100.0 * torch.rand(k, device=device, generator=gw)
    y = X @ w + bias + noise * torch.randn(m, device=device, generator=g)
    return X, y


def classification(m: int, n: int, device: torch.device, seed: int = 0, n_classes: int = 2,
                   n_informative: Optional[int] = None, n_redundant: Optional[int] = None,
                   class_sep: float = 1.0, flip_y: float = 0.01) -> Tuple[torch.Tensor, torch.Tensor]:
    g = _gen(device, seed)
    ni = n_informative if n_informative is not None else max(1, n // 3)
    nr = n_redundant if n_redundant is not None else max(0, n // 3)
    ni = min(ni, n)
    nr = min(nr, n - ni)
    y = torch.randint(0, n_classes, (m,), device=device, generator=g)
    gc = _gen(device, 999)
    centroids = (torch.randint(0, 2, (n_classes, ni), device=device, generator=gc).float() * 2 - 1) * class_sep
    X = torch.empty(m, n, device=device, dtype=torch.float32)
    X[:, :ni] = torch.randn(m, ni, device=device, generator=g) + centroids[y]
    if nr > 0:
        B = 2 * torch.rand(ni, nr, device=device, generator=gc) - 1
        X[:, ni: ni + nr] = (X[:, :ni] @ B) / float(np.sqrt(ni))
    if ni + nr < n:
        X[:, ni + nr:] = torch.randn(m, n - ni - nr, device=device, generator=g)
    flip = torch.rand(m, device=device, generator=g) < flip_y
    y = torch.where(flip, torch.randint(0, n_classes, (m,), device=device, generator=g), y)
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
