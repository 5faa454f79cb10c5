"""How much Lloyd work could distance bounds skip on the bench's KMeans shapes (1M x 3000, k=1000,
random init)? Runs a plain fp32 torch Lloyd, records per iteration the best/second-best distances
and the Hamerly test (u + shift[a] < l - max shift) of the PREVIOUS iteration's bounds, and times
the library's fit on the same data. One JSON line per dataset family."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from spark_rapids_ml_nai_amd.bench import datagen  # noqa: E402


def probe(family: str, m: int, n: int, k: int, iters: int) -> dict:
    dev = torch.device("cuda", 0)
    X = datagen.low_rank_matrix(m, n, dev, seed=1000, m_total=m) if family == "low_rank_matrix" else \
        datagen.uniform(m, n, dev, seed=1000)
    g = torch.Generator(device="cpu").manual_seed(1)
    C = X[torch.randperm(m, generator=g)[:k].to(dev)].double()
    xn = (X * X).sum(1)
    u = l = a = None
    skip = []
    changed = []
    for it in range(iters):
        Cf = C.float()
        cn = (Cf * Cf).sum(1)
        d1 = torch.empty(m, device=dev)
        d2 = torch.empty(m, device=dev)
        lab = torch.empty(m, dtype=torch.long, device=dev)
        for r0 in range(0, m, 65536):
            D = (xn[r0:r0 + 65536, None] + cn[None, :] - 2.0 * X[r0:r0 + 65536] @ Cf.T).clamp_min(0).sqrt()
            v, i = D.topk(2, dim=1, largest=False)
            d1[r0:r0 + 65536], d2[r0:r0 + 65536], lab[r0:r0 + 65536] = v[:, 0], v[:, 1], i[:, 0]
        if a is not None:
            skip.append(float((u < l).float().mean()))
            changed.append(float((lab != a).float().mean()))
        sums = torch.zeros_like(C).index_add_(0, lab, X.double())
        cnt = torch.bincount(lab, minlength=k).double()
        newC = torch.where(cnt[:, None] > 0, sums / cnt.clamp_min(1)[:, None], C)
        shift = (newC - C).norm(dim=1).float()
        C = newC
        a = lab
        u = d1 + shift[lab]
        l = d2 - shift.max()
    out = {"family": family, "m": m, "n": n, "k": k, "hamerly_skip_frac": [round(s, 4) for s in skip],
           "label_changed_frac": [round(c, 4) for c in changed]}
    # the library fit on the same data (pinned host copy, like the bench)
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.clustering import KMeans

    df = DataFrame.from_numpy(datagen.to_pinned_numpy(X))
    del X
    torch.cuda.empty_cache()
    est = KMeans(k=k, maxIter=iters, tol=1e-20, initMode="random", seed=1)
    est.fit(df)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model = est.fit(df)
    torch.cuda.synchronize()
    out["fit_s"] = round(time.perf_counter() - t0, 4)
    out["refined_frac"] = model._model_attributes.get("refined_frac")
    return out


if __name__ == "__main__":
    fams = sys.argv[1].split(",") if len(sys.argv) > 1 else ["low_rank_matrix", "uniform"]
    for f in fams:
        print(json.dumps(probe(f, 1_000_000, 3000, 1000, 30)), flush=True)
        torch.cuda.empty_cache()
