"""IVF all-points graph: recall@k against exact neighbours vs nprobe, per data family and size.

Queries are a random sample of the graph's own rows; their exact neighbours are searched over
ALL N rows (brute force, ``knn_graph``), so the recall is the fitted graph's, not a subsample's.
Prints one JSON line per (family, N, nprobe): recall, graph build seconds."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="100000,2000000")
    ap.add_argument("--families", default="blobs,classification,low_rank")
    ap.add_argument("--nprobe", default="16,32,64")
    ap.add_argument("--queries", type=int, default=2000)
    ap.add_argument("--k", type=int, default=15)
    ap.add_argument("--cols", type=int, default=128)
    ap.add_argument("--probe", default="list,query", help="list: probe the list centre's nearest lists; "
                    "query: each row's own nearest lists (per-query probing)")
    ap.add_argument("--nnd", default="0", help="NN-descent refinement rounds (comma list)")
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models.knn_graph import knn_graph, knn_graph_ivf

    dev = torch.device("cuda", 0)
    n = a.cols
    for fam in a.families.split(","):
        for N in [int(x) for x in a.rows.split(",")]:
            if fam == "blobs":
                X, _ = datagen.blobs(N, n, dev, seed=7, centers=20)
            elif fam == "classification":
                X, _ = datagen.classification(N, n, dev, seed=7, n_informative=n // 2, n_redundant=n // 4)
            else:
                X = datagen.low_rank_matrix(N, n, dev, seed=7)
            X = X.float().contiguous()
            g = torch.Generator(device=dev).manual_seed(3)
            q = torch.randperm(N, device=dev, generator=g)[: a.queries]
            _, ei = knn_graph(X.index_select(0, q), X, a.k + 1)
            ei = ei.cpu()
            for probe, npb, nnd in [(pm, int(x), int(r)) for pm in a.probe.split(",") for x in a.nprobe.split(",")
                                    for r in a.nnd.split(",")]:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                phases = {}
                _, gi = knn_graph_ivf(X, a.k, nprobe=npb, seed=1, probe=probe, phases=phases, nnd_iters=nnd)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                gq = gi.index_select(0, q).cpu()
                hit = 0.0
                for r in range(q.shape[0]):
                    # the exact list includes the row itself (distance 0): compare the k nearest,
                    # self included, as the IVF graph also returns the row itself first
                    hit += len(set(gq[r].tolist()) & set(ei[r, : a.k].tolist())) / float(a.k)
                print(json.dumps({"family": fam, "rows": N, "cols": n, "probe": probe, "nprobe": npb, "nnd": nnd, "k": a.k,
                                  "recall": round(hit / q.shape[0], 4), "graph_s": round(dt, 3),
                                  "phases": {k: v["s"] for k, v in phases.items()}}), flush=True)
                del gi
                torch.cuda.empty_cache()
            del X
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
