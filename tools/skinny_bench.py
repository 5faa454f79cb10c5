"""Skinny-GEMM kernels at 1M x 3000 fp32: X W (Z = X Wt^T, srml_xw_f32 VALU vs srml_xw_t_f32 MFMA)
and X^T V (srml_xtv2_f32 VALU vs srml_xtv_mfma_f32 MFMA) per K, with max relative error vs fp64.

    python tools/skinny_bench.py [--rows 1000000 --cols 3000]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=3000)
    ap.add_argument("--variants", action="store_true", help="also time the xw_t tuning variants")
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd.ops import native

    dev = torch.device("cuda", 0)
    m, n = a.rows, a.cols
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.rand((m, n), device=dev, generator=g) - 0.5
    st = native.stream(dev)
    chk = slice(0, 4096)
    Xc = X[chk].double()
    res = {"rows": m, "cols": n, "hbm_floor_ms": round(m * n * 4 / 5.8e12 * 1e3, 3)}
    for K in (1, 4, 8, 10, 16, 32):
        Wt = torch.rand((K, n), device=dev, generator=g) - 0.5
        kk = next(w for w in (1, 2, 3, 4, 8, 16, 32) if w >= K)
        Wp = torch.zeros((n, kk), device=dev)
        Wp[:, :K] = Wt.t()
        Zo = torch.empty((m, kk), device=dev)
        Zn = torch.empty((m, K), device=dev)
        old = lambda: native.call("srml_xw_f32", X.data_ptr(), m, n, n, Wp.data_ptr(), kk, None, Zo.data_ptr(), kk, st)
        new = lambda: native.call("srml_xw_t_f32", X.data_ptr(), m, n, n, Wt.data_ptr(), K, n, None, Zn.data_ptr(), K,
                                  st)
        res["xw_valu_K%d_ms" % K] = round(_time(old) * 1e3, 3)
        res["xw_mfma_K%d_ms" % K] = round(_time(new) * 1e3, 3)
        if a.variants:
            for v in (1, 2, 3):
                fn = lambda: native.call("srml_xw_t_f32_variant", X.data_ptr(), m, n, n, Wt.data_ptr(), K, n, None,
                                         Zn.data_ptr(), K, v, st)
                res["xw_mfma_K%d_v%d_ms" % (K, v)] = round(_time(fn) * 1e3, 3)
            new()
        ref = Xc @ Wt.double().t()
        scale = (Xc.abs() @ Wt.double().abs().t()).max().item()
        res["xw_mfma_K%d_err" % K] = float((Zn[chk].double() - ref).abs().max().item() / scale)
        res["xw_valu_K%d_err" % K] = float((Zo[chk, :K].double() - ref).abs().max().item() / scale)
        if K > 16:
            continue
        V = torch.rand((m, K), device=dev, generator=g) - 0.5
        o1 = torch.zeros((n, K), dtype=torch.float64, device=dev)
        o2 = torch.zeros((n, K), dtype=torch.float64, device=dev)
        v1 = lambda: native.call("srml_xtv2_f32", X.data_ptr(), m, n, n, V.data_ptr(), K, K, o1.data_ptr(), K, 1, None,
                                 st)
        v2 = lambda: native.call("srml_xtv_mfma_f32", X.data_ptr(), m, n, n, V.data_ptr(), K, K, o2.data_ptr(), K, 1,
                                 None, st)
        res["xtv_valu_K%d_ms" % K] = round(_time(v1) * 1e3, 3)
        res["xtv_mfma_K%d_ms" % K] = round(_time(v2) * 1e3, 3)
        o1.zero_()
        o2.zero_()
        v1()
        v2()
        ref = X[:200000].double().t() @ V[:200000].double()
        o3 = torch.zeros((n, K), dtype=torch.float64, device=dev)
        native.call("srml_xtv_mfma_f32", X.data_ptr(), 200000, n, n, V.data_ptr(), K, K, o3.data_ptr(), K, 1, None, st)
        sc = (X[:200000].abs().double().t() @ V[:200000].abs().double()).max().item()
        res["xtv_mfma_K%d_err" % K] = float((o3 - ref).abs().max().item() / sc)
        res["xtv_mfma_vs_valu_K%d" % K] = float((o1 - o2).abs().max().item() / (o1.abs().max().item() + 1e-30))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
