"""Does the approximate kNN graph's recall move UMAP's embedding quality? Fits UMAP on the same
N rows with the exact graph (brute force) and with the IVF graph at several nprobe, and scores
every embedding by trustworthiness on one fixed row sample (exact ranks in the input space).
Prints one JSON line per (family, graph): fit seconds, trustworthiness, graph recall@15 on a
query sample vs the exact graph."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--families", default="classification,low_rank")
    ap.add_argument("--graphs", default="brute,list16,query16,query32",
                    help="brute | list<N> (probe by the list centre) | query<N> (per-query probes) | ivf<N>")
    ap.add_argument("--sample", type=int, default=20_000)
    a = ap.parse_args()
    from northstar import trustworthiness

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.umap import UMAP

    dev = torch.device("cuda", 0)
    n = 128
    N = a.rows
    for fam in a.families.split(","):
        if fam == "classification":
            X, _ = datagen.classification(N, n, dev, seed=7, n_informative=n // 2, n_redundant=n // 4)
        elif fam == "blobs":
            X, _ = datagen.blobs(N, n, dev, seed=7, centers=20)
        else:
            X = datagen.low_rank_matrix(N, n, dev, seed=7)
        Xh = datagen.to_pinned_numpy(X.float())
        del X
        torch.cuda.empty_cache()
        idx = np.sort(np.random.default_rng(0).choice(N, size=a.sample, replace=False))
        Xs = torch.from_numpy(np.ascontiguousarray(Xh[idx])).to(dev)
        df = DataFrame.from_numpy(Xh)
        for gname in a.graphs.split(","):
            if gname == "brute":
                kw = dict(build_algo="brute_force_knn")
            elif gname.startswith("list") or gname.startswith("query"):  # probe mode + count
                mode = "list" if gname.startswith("list") else "query"
                kw = dict(build_algo="ivf", build_kwds={"nprobe": int(gname[len(mode):]), "probe": mode})
            else:
                kw = dict(build_algo="ivf", build_kwds={"nprobe": int(gname[3:])})
            est = UMAP(n_neighbors=15, n_components=2, random_state=1, featuresCol="features", **kw)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model = est.fit(df)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            E = torch.from_numpy(np.asarray(model.embedding_)[idx]).to(dev)
            tw = trustworthiness(Xs, E)
            print(json.dumps({"family": fam, "rows": N, "graph": gname, "fit_s": round(dt, 3),
                              "trustworthiness": round(tw, 5)}), flush=True)
            del model, E
            torch.cuda.empty_cache()
        del df, Xh, Xs


if __name__ == "__main__":
    main()
