"""Section timing of the on-device QN step kernel (SRML_QN_PROBE=1): runs a LogisticRegression fit on
a synthetic shard and prints the wall-clock split of one step (10 ns ticks)."""
import os
import sys

os.environ["SRML_QN_PROBE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spark_rapids_ml_nai_amd.models import qn  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
m = 20000
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(m, n, device=dev, generator=g)
y = (X[:, 0] > 0).float()
from spark_rapids_ml_nai_amd import ops  # noqa: E402

P = qn.QNProblem(n=n, K=1, fit_intercept=True, m_total=float(m), l2=np.r_[np.full(n, 1e-3), 0.0],
                 l1=np.zeros(n + 1), inv_sigma=np.ones(n), max_iter=30, tol=1e-30)
st = qn.DeviceQN(P, np.zeros(n + 1), dev)
stamps = []
for it in range(40):
    ops.logistic_loss_grad(X, y, st.w_dev, st.b_dev, 1, st.out, None)
    st.step()
    torch.cuda.synchronize()
    p = st.probe.cpu().numpy().copy()
    if p[7] > 0:
        stamps.append(np.diff(p[:8]))
    st.probe.zero_()
a = np.array(stamps)
print("sections (10ns ticks): pass0 | 1a | 1b | solve | pass2 | red | trial  (median over %d accepted steps)" % len(a))
print(np.median(a, 0), "total us", np.median(a.sum(1)) / 100)
