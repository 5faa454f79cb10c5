"""Per-evaluation time of the fused multi-class / multi-model logistic passes at 1M x 3000 fp32.

    python tools/mlogit_bench.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main() -> None:
    from spark_rapids_ml_nai_amd import ops

    dev = torch.device("cuda", 0)
    m, n = 1_000_000, 3000
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.rand((m, n), device=dev, generator=g)
    res = {}
    for K in (4, 10):
        y = torch.randint(0, K, (m,), device=dev, generator=g).float()
        w = torch.zeros(K * n, dtype=torch.float64, device=dev)
        b = torch.zeros(K, dtype=torch.float64, device=dev)
        out = torch.zeros(K * n + K + 1, dtype=torch.float64, device=dev)
        t = _time(lambda: ops.logistic_loss_grad(X, y, w, b, K, out.zero_()))
        res["multinomial_K%d_ms" % K] = round(t * 1e3, 3)
    yb = (torch.rand(m, device=dev, generator=g) > 0.5).float()
    for M in (1, 4, 8):
        WB = torch.zeros((M, n + 1), dtype=torch.float64, device=dev)
        OUT = torch.zeros((M, n + 2), dtype=torch.float64, device=dev)
        t = _time(lambda: ops.logistic_loss_grad_multi(X, yb, WB, OUT.zero_()))
        res["multi_binary_M%d_ms" % M] = round(t * 1e3, 3)
    w1 = torch.zeros(n, dtype=torch.float64, device=dev)
    b1 = torch.zeros(1, dtype=torch.float64, device=dev)
    o1 = torch.zeros(n + 2, dtype=torch.float64, device=dev)
    res["binary_fused_ms"] = round(_time(lambda: ops.logistic_loss_grad(X, yb, w1, b1, 1, o1.zero_())) * 1e3, 3)
    res["hbm_floor_ms"] = round(m * n * 4 / 5.8e12 * 1e3, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
