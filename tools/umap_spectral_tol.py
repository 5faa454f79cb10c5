"""UMAP 20M x 128 fit time and embedding trustworthiness vs the spectral-init stopping tolerance
(SRML_UMAP_SPECTRAL_TOL) and the Chebyshev degree, on one data family."""
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
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--family", default="blobs")
    ap.add_argument("--settings", default="1e-6:1,1e-5:1,1e-4:1,1e-6:4")
    a = ap.parse_args()
    from northstar import trustworthiness

    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import umap as U

    dev = torch.device("cuda", 0)
    n = 128
    if a.family == "blobs":
        X, _ = datagen.blobs(a.rows, n, dev, seed=7000, centers=20)
    elif a.family == "low_rank":
        X = datagen.low_rank_matrix(a.rows, n, dev, seed=7000)
    else:
        X, _ = datagen.classification(a.rows, n, dev, seed=7000, n_informative=n // 2, n_redundant=n // 4)
    idx = torch.from_numpy(np.sort(np.random.default_rng(0).choice(a.rows, size=20000, replace=False))).to(dev)
    Xs = X.index_select(0, idx)
    params = {"n_neighbors": 15, "n_components": 2, "random_state": 1}
    U.umap_fit(X[:20000].contiguous(), params)
    for st in a.settings.split(","):
        tol, deg = st.split(":")
        U.SPECTRAL_TOL, U.CHEB_DEGREE = float(tol), int(deg)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        E = U.umap_fit(X, params)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ph = U.LAST_PHASES.get("spectral", {})
        tw = trustworthiness(Xs, torch.from_numpy(np.asarray(E)[idx.cpu().numpy()]).to(dev))
        print(json.dumps({"family": a.family, "rows": a.rows, "tol": float(tol), "cheb": int(deg), "fit_s": round(dt, 3),
                          "spectral_s": ph.get("s"), "products": ph.get("products"),
                          "trustworthiness": round(tw, 5)}), flush=True)
        del E
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
