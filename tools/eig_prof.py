"""Time the PCA top-k eigensolver on a 3000 x 3000 covariance of the bench's low-rank data."""
import os, sys, time, cProfile, pstats, io
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spark_rapids_ml_nai_amd.bench import datagen
from spark_rapids_ml_nai_amd.models.eig import topk_eigh
dev = torch.device("cuda")
X = datagen.low_rank_matrix(200000, 3000, dev, seed=1, m_total=200000).double()
Xc = X - X.mean(0)
C = (Xc.T @ Xc) / (X.shape[0] - 1)
del X, Xc
topk_eigh(C, 3); torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter()
    w, V = topk_eigh(C, 3)
    torch.cuda.synchronize()
    print("eig s", round(time.perf_counter() - t0, 4), w)
pr = cProfile.Profile(); pr.enable(); topk_eigh(C, 3); torch.cuda.synchronize(); pr.disable()
out = io.StringIO(); pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(12); print(out.getvalue()[:3000])
