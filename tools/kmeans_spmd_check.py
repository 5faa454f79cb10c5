"""One KMeans fit per torchrun rank on its shard of a fixed blob dataset (the small-k MFMA Lloyd
loop: k = 20, 64 columns), run by tests/test_multirank_gpu.py with and without delta steps; rank 0
prints the model (centres, iterations) as one JSON line."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ROWS, COLS, K = 400_000, 64, 20


def main() -> None:
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo")
    rng = np.random.default_rng(7)
    C = rng.uniform(-4, 4, (K, COLS))
    X = (C[rng.integers(0, K, ROWS)] + 1.5 * rng.standard_normal((ROWS, COLS))).astype(np.float32)
    b = np.linspace(0, ROWS, world + 1).astype(np.int64)
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.clustering import KMeans

    # random rows as the start: several blobs share a start centre, so the fit takes several steps
    est = KMeans(k=K, maxIter=20, tol=0.0, seed=3, initMode="random", featuresCol="features")
    est.num_workers = world
    model = est.fit(DataFrame.from_numpy(X[b[rank]:b[rank + 1]]))
    if rank == 0:
        ma = getattr(model, "_model_attributes", {}) or {}
        print(json.dumps({"iters": int(ma.get("n_iter", -1)), "world": world,
                          "delta": os.environ.get("SRML_LLOYD_SMALL_DELTA"),
                          "centres": np.asarray(model.cluster_centers_, dtype=np.float64).tolist()}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
