"""torchrun driver (ranks sharing the GPU over gloo): an ensemble-mode RandomForest fitMultiple on
each rank's page-locked shard whose FIRST param map has fewer trees than ranks (a rank grows no
tree for it, so its streamed chunks are binned only by the finish-after-the-loop path), then a map
that every rank grows trees for. The second model must equal a standalone fit of that map on the
same ranks (garbage bins reused from the first map would change it). Rank 0 prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> None:
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier

    g = np.random.default_rng(100 + rank)
    m, n = 20000, 16
    X = torch.empty((m, n), dtype=torch.float32).pin_memory()
    X.copy_(torch.from_numpy(g.standard_normal((m, n)).astype(np.float32)))
    Xh = X.numpy()
    y = (Xh[:, 0] + 0.5 * Xh[:, 1] > 0).astype(np.float64)
    df = DataFrame.from_numpy(Xh, y)
    est = RandomForestClassifier(numTrees=1, maxDepth=6, seed=3, split_mode="ensemble", num_workers=world)
    models = dict(est.fitMultiple(df, [{est.numTrees: 1}, {est.numTrees: 2 * world}]))
    solo = RandomForestClassifier(numTrees=2 * world, maxDepth=6, seed=3, split_mode="ensemble",
                                  num_workers=world).fit(df)
    a = models[1].transform(df).to_numpy("probability")
    b = solo.transform(df).to_numpy("probability")
    if rank == 0:
        print(json.dumps({"world": world, "equal": bool(np.array_equal(a, b)),
                          "trees": [models[0].getNumTrees, models[1].getNumTrees]}))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
