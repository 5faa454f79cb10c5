"""IVF all-points kNN probe at the UMAP north-star shape: list-size balance, candidate pairs
and the knn_lists kernel's achieved rate.

    python tools/ivf_probe.py [--rows 20000000] [--cols 128]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20_000_000)
    ap.add_argument("--cols", type=int, default=128)
    ap.add_argument("--k", type=int, default=15)
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import knn_graph as KG

    dev = torch.device("cuda", 0)
    X, _ = datagen.blobs(a.rows, a.cols, dev, seed=7000, centers=20)
    N = X.shape[0]
    nlist = max(1, int(round(N / KG.IVF_LIST_ROWS)))
    nprobe = KG.IVF_NPROBE
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    C = KG.train_quantizer(X, nlist, 0)
    lab = ops.nearest_list(X, C, ops.quantizer_planes(X) if nlist > 256 else None)
    order, off, _ = ops.label_sort(lab, nlist)
    order = order.long()
    counts = off[1:] - off[:-1]
    Xs = X.index_select(0, order).contiguous()
    xn = ops.row_sqnorm(Xs)
    cn = torch.where(counts > 0, ops.row_sqnorm(C), torch.full((nlist,), float("inf"), device=dev))
    _, probes = ops.knn(C, C, nprobe, inorm=cn, qnorm=torch.zeros(nlist, device=dev))
    ok = (probes >= 0) & torch.isfinite(cn[probes.clamp_min(0)])
    probes = torch.where(ok, probes, torch.full_like(probes, -1))
    tile_q0, tile_list = KG.ivf_tiles(counts, off)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    cand = torch.where(probes >= 0, counts[probes.clamp_min(0)], torch.zeros_like(probes)).sum(1)
    rows = torch.minimum(off[tile_list + 1] - tile_q0, torch.full_like(tile_q0, 128))
    pairs = float((rows * cand[tile_list]).double().sum())
    padded = float((128 * ((cand[tile_list] + 127) // 128)).double().sum() * 128)
    res = {"rows": N, "nlist": nlist, "nprobe": nprobe, "tiles": int(tile_list.shape[0]), "prep_s": round(t1 - t0, 3),
           "list_rows": {q: int(torch.quantile(counts.double(), q).item()) for q in (0.0, 0.5, 0.9, 0.99, 1.0)},
           "pairs": pairs, "pairs_per_row": pairs / N, "padded_tile_pairs": padded}
    for mode in ("f32", "f16"):
        for rep in range(2):
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            od, oi = ops.knn_lists(Xs, xn, off, probes.int(), tile_q0, tile_list, a.k,
                                   centroids=C if mode == "f16" else None)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t2
        res["knn_lists_%s_s" % mode] = round(dt, 3)
        res["tflops_padded_%s" % mode] = round(2.0 * a.cols * padded / dt / 1e12, 2)
        res["_idx_" + mode] = oi[::997].clone()
    i32, i16 = res.pop("_idx_f32"), res.pop("_idx_f16")
    hit = (i16.unsqueeze(2) == i32.unsqueeze(1)).any(2) & (i16 >= 0)
    res["f16_vs_f32_set_recall"] = round(hit.sum().item() / max(1, (i32 >= 0).sum().item()), 5)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
