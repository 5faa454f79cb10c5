"""Synthetic dataset generator CLI (reference ``python/benchmark/gen_data.py`` and
``gen_data_distributed.py``), writing partitioned Parquet without Spark.

    python -m spark_rapids_ml_nai_amd.bench.gen_data <type> --num_rows 1000000 --num_cols 3000 \
        --feature_type array --output_num_files 50 --output_dir /data/1m_3k.parquet [--overwrite]

Types: default (uniform), blobs, regression, classification, low_rank_matrix, sparse_regression.
Each output file is one partition generated from its own seed (``seed + file index``) — the
distributed generator's scheme — on the GPU when one is visible, else on the CPU, with the same
distribution families as the reference (``bench/datagen.py``). Columns: ``feature_array``
(array<dtype> or VectorUDT) or ``c0..c{n-1}`` (multi_cols), plus ``label`` where the type has one.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
from typing import Dict, List, Optional, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import torch

from ..core.dataframe import VECTOR_STRUCT, dense_to_list_array, dense_to_vector_array, vector_field
from . import datagen

TYPES = ("default", "blobs", "regression", "classification", "low_rank_matrix", "sparse_regression")


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Generate a random dataset as partitioned Parquet.")
    p.add_argument("type", choices=TYPES)
    p.add_argument("--num_rows", type=int, default=100)
    p.add_argument("--num_cols", type=int, default=30)
    p.add_argument("--dtype", choices=["float32", "float64"], default="float32")
    p.add_argument("--feature_type", choices=["array", "vector", "multi_cols"], default="multi_cols")
    p.add_argument("--output_dir", required=True)
    p.add_argument("--output_num_files", type=int, default=None)
    p.add_argument("--overwrite", action="store_true")
    p.add_argument("--train_fraction", type=float, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", default=None, help="cpu | cuda (default: cuda when visible)")
    # type specific
    p.add_argument("--n_clusters", "--centers", dest="centers", type=int, default=20)
    p.add_argument("--cluster_std", type=float, default=1.0)
    p.add_argument("--n_informative", type=int, default=None)
    p.add_argument("--n_redundant", type=int, default=None)
    p.add_argument("--n_classes", type=int, default=2)
    p.add_argument("--noise", type=float, default=0.0)  # make_regression's default
    p.add_argument("--bias", type=float, default=0.0)
    p.add_argument("--logistic_regression", action="store_true", help="regression: emit 0/1 labels")
    p.add_argument("--effective_rank", type=int, default=10)
    p.add_argument("--tail_strength", type=float, default=0.5)
    p.add_argument("--density", type=str, default="0.1",
                   help="sparse_regression: fraction of non-zeros, or a comma list (one per column chunk)")
    p.add_argument("--density_curve", choices=["None", "Linear", "Exponential"], default="None",
                   help="sparse_regression: density ramp over --n_chunk column chunks, averaging --density")
    p.add_argument("--n_chunk", type=int, default=10)
    p.add_argument("--redundant_cols", type=int, default=0,
                   help="sparse_regression: columns that are random mixes of the informative ones")
    p.add_argument("--no_shuffle", action="store_true")
    return p


def gen_partition(args: argparse.Namespace, rows: int, seed: int, device: torch.device
                  ) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    n = args.num_cols
    y = None
    if args.type == "default":
        X = datagen.uniform(rows, n, device, seed)
    elif args.type == "blobs":
        X, y = datagen.blobs(rows, n, device, seed, centers=args.centers, cluster_std=args.cluster_std)
    elif args.type == "sparse_regression":
        dens = [float(v) for v in str(args.density).split(",")]
        X, y, _ = datagen.sparse_regression(
            rows, n, seed=args.seed + 1, partition_seed=seed + 1000003, density=dens if len(dens) > 1 else dens[0],
            density_curve=args.density_curve, n_chunk=args.n_chunk, redundant_cols=args.redundant_cols,
            n_informative=args.n_informative or 10, noise=args.noise, bias=args.bias, shuffle=not args.no_shuffle,
            logistic_regression=args.logistic_regression, n_classes=args.n_classes,
            num_partitions=args.output_num_files or 1)
        return X, y  # CSR (float64, as the reference's sparse VectorUDT) + labels
    elif args.type == "regression":
        multi = args.logistic_regression and args.n_classes > 2
        X, y = datagen.regression(rows, n, device, seed, n_informative=args.n_informative or 10, noise=args.noise,
                                  bias=args.bias, n_targets=args.n_classes if multi else 1)
        if args.logistic_regression:  # Bernoulli / softmax-sampled labels of the unscaled target
            y = datagen.logistic_labels(y, seed)
    elif args.type == "classification":
        X, y = datagen.classification(rows, n, device, seed, n_classes=args.n_classes,
                                      n_informative=args.n_informative, n_redundant=args.n_redundant)
    elif args.type == "low_rank_matrix":
        X = datagen.low_rank_matrix(rows, n, device, seed, effective_rank=args.effective_rank,
                                    tail_strength=args.tail_strength, m_total=args.num_rows)
    else:
        raise ValueError(args.type)
    dt = np.float32 if args.dtype == "float32" else np.float64
    Xh = X.cpu().numpy().astype(dt, copy=False)
    yh = y.cpu().numpy().astype(dt, copy=False) if y is not None else None
    return Xh, yh


def _sparse_vector_array(X) -> pa.Array:
    import scipy.sparse as sp

    csr = X if sp.issparse(X) else sp.csr_matrix(X)
    csr = csr.tocsr()
    m, n = csr.shape
    return pa.StructArray.from_arrays(
        [pa.array(np.zeros(m, dtype=np.int8)), pa.array(np.full(m, n, dtype=np.int32)),
         pa.ListArray.from_arrays(pa.array(csr.indptr.astype(np.int32)), pa.array(csr.indices.astype(np.int32))),
         pa.ListArray.from_arrays(pa.array(csr.indptr.astype(np.int32)), pa.array(csr.data.astype(np.float64)))],
        fields=list(VECTOR_STRUCT))


def to_table(args: argparse.Namespace, X: np.ndarray, y: Optional[np.ndarray]) -> pa.Table:
    arrays: List[pa.Array] = []
    fields: List[pa.Field] = []
    if args.type == "sparse_regression":
        arrays.append(_sparse_vector_array(X))
        fields.append(vector_field("feature_array"))
    elif args.feature_type == "array":
        a = dense_to_list_array(X)
        arrays.append(a)
        fields.append(pa.field("feature_array", a.type))
    elif args.feature_type == "vector":
        arrays.append(dense_to_vector_array(X))
        fields.append(vector_field("feature_array"))
    else:
        for j in range(X.shape[1]):
            a = pa.array(np.ascontiguousarray(X[:, j]))
            arrays.append(a)
            fields.append(pa.field("c%d" % j, a.type))
    if y is not None:
        arrays.append(pa.array(y))
        fields.append(pa.field("label", arrays[-1].type))
    return pa.Table.from_arrays(arrays, schema=pa.schema(fields))


def generate(argv: Optional[List[str]] = None) -> Dict[str, int]:
    args = _parser().parse_args(argv)
    device = torch.device(args.device) if args.device else torch.device(
        "cuda" if torch.cuda.is_available() else "cpu")
    out = args.output_dir
    if os.path.exists(out):
        if not args.overwrite:
            raise FileExistsError("%s exists (use --overwrite)" % out)
        shutil.rmtree(out)
    nfiles = args.output_num_files or max(1, min(64, args.num_rows // 100000 or 1))
    bounds = np.linspace(0, args.num_rows, nfiles + 1).astype(np.int64)
    dirs = [out] if args.train_fraction is None else [os.path.join(out, "train"), os.path.join(out, "eval")]
    for d in dirs:
        os.makedirs(d, exist_ok=True)
    counts = {d: 0 for d in dirs}
    for i in range(nfiles):
        rows = int(bounds[i + 1] - bounds[i])
        if rows == 0:
            continue
        X, y = gen_partition(args, rows, args.seed + i, device)
        if y is not None:
            y = np.asarray(y, dtype=np.float64 if args.type == "sparse_regression" else y.dtype)
        if args.train_fraction is None:
            pq.write_table(to_table(args, X, y), os.path.join(out, "part-%05d.parquet" % i))
            counts[out] += rows
        else:
            u = np.random.default_rng(args.seed + 10007 * (i + 1)).random(rows) < args.train_fraction
            for d, mask in zip(dirs, (u, ~u)):
                if mask.any():
                    pq.write_table(to_table(args, X[mask], None if y is None else y[mask]),
                                   os.path.join(d, "part-%05d.parquet" % i))
                    counts[d] += int(mask.sum())
    return counts


def main() -> int:
    counts = generate(sys.argv[1:])
    for d, c in counts.items():
        print("%s: %d rows" % (d, c))
    print("gen_data finished")
    return 0


if __name__ == "__main__":
    sys.exit(main())
