"""Section timing of the device L-BFGS step (``qn_step_kernel``): runs a binary LogReg fit with
``SRML_QN_PROBE=1`` (the kernel stamps wall_clock64 at 8 points of its last launch) and prints
the per-section durations in microseconds (wall_clock64 ticks at 100 MHz on CDNA)."""
import os
import sys

os.environ["SRML_QN_PROBE"] = "1"
os.environ["SRML_QN_GRAPH"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spark_rapids_ml_nai_amd.models import qn  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    m, n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000, 3000
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(m, n, device=dev, generator=g)
    y = (X[:, 0] + 0.5 * torch.randn(m, device=dev, generator=g) > 0).float()
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    seen = []
    orig = qn.DeviceQN.step

    def step(self):
        orig(self)
        seen.append(self)

    qn.DeviceQN.step = step
    logistic_fit(X, y, m, WorkerContext.single(dev), 1e-5, 0.0, True, False, 20, 1e-30)
    torch.cuda.synchronize()
    p = seen[-1].probe.cpu().numpy().astype(np.int64)
    d = np.diff(p[:8]) / 100.0  # 100 MHz -> us
    for nm, v in zip(["pass0 (+reduce)", "accept: pass1a", "pass1b (S/Y dots)", "tid0 + compact solve",
                      "pass2 (direction)", "reduce p2v", "pass3 (trial)"], d):
        print("%-24s %8.2f us" % (nm, v))
    print("total %.2f us" % ((p[7] - p[0]) / 100.0))


if __name__ == "__main__":
    main()
