"""torch.bincount vs index_add_ on the device (labels -> counts), the shapes UMAP / KMeans use."""
import time

import torch

dev = torch.device("cuda")
for n, k in [(10_000_000, 10_000), (10_000_000, 20), (100_000_000, 20), (10_000_000, 10_000_000)]:
    lab = torch.randint(0, k, (n,), device=dev)
    res = {}
    for name, fn in [("bincount", lambda: torch.bincount(lab, minlength=k)),
                     ("index_add", lambda: torch.zeros(k, dtype=torch.int64, device=dev).index_add_(
                         0, lab, torch.ones(1, dtype=torch.int64, device=dev).expand(n))),
                     ("scatter_add", lambda: torch.zeros(k, dtype=torch.int64, device=dev).scatter_add_(
                         0, lab, torch.ones(1, dtype=torch.int64, device=dev).expand(n)))]:
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            out = fn()
        torch.cuda.synchronize()
        res[name] = round((time.perf_counter() - t0) / 3 * 1e3, 3)
        if name != "bincount":
            assert torch.equal(out, torch.bincount(lab, minlength=k))
    print(n, k, res, flush=True)
