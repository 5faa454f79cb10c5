"""On-device quasi-Newton (models/qn.py, ops/csrc/qn.hip) and LogisticRegression numerics.

Oracles: scikit-learn's LogisticRegression under Spark's objective mapping
(mean loss + reg * ((1 - a)/2 ||w||^2 + a ||w||_1)  <=>  sklearn C = 1 / (m * reg)), the reference's
own test matrix (python/tests/test_logistic_regression.py: binomial / multinomial x L2 / L1 /
elastic-net), and, for the kernels, the numpy state machine ``HostQN`` and a plain PyTorch fp64
loss/gradient.
"""
import warnings

import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import DataFrame, ops
from spark_rapids_ml_nai_amd.models.qn import HostQN, QNProblem, minimize

warnings.filterwarnings("ignore")

DEVICES = ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.fixture(params=DEVICES)
def device(request, monkeypatch):
    if request.param == "cpu":
        monkeypatch.setenv("SRML_FORCE_CPU", "1")
    else:
        monkeypatch.delenv("SRML_FORCE_CPU", raising=False)
    return request.param


def _data(m, n, classes, seed=0, dtype=np.float32):
    from sklearn.datasets import make_classification

    X, y = make_classification(n_samples=m, n_features=n, n_informative=max(2, n // 2), n_redundant=0,
                               n_classes=classes, n_clusters_per_class=1, random_state=seed, class_sep=0.8)
    return X.astype(dtype), y.astype(np.float64)


def _sk(X, y, reg, a, multi):
    from sklearn.linear_model import LogisticRegression as SK

    m = X.shape[0]
    C = 1.0 / (m * reg)
    if a == 0.0:
        sk = SK(C=C, penalty="l2", solver="lbfgs", tol=1e-12, max_iter=20000)
    else:
        sk = SK(C=C, penalty="elasticnet", l1_ratio=a, solver="saga", tol=1e-12, max_iter=200000)
    sk.fit(X.astype(np.float64), y)
    return sk.coef_, sk.intercept_


def _spark_objective(X, y, W, b, reg, a):
    """Spark's (unstandardised) objective evaluated in fp64."""
    X = X.astype(np.float64)
    Z = X @ W.T + b
    if W.shape[0] == 1:
        z = Z[:, 0]
        loss = np.mean(np.logaddexp(0, z) - y * z)
    else:
        lse = np.logaddexp.reduce(Z, axis=1)
        loss = np.mean(lse - Z[np.arange(len(y)), y.astype(int)])
    return loss + reg * ((1 - a) / 2 * np.sum(W * W) + a * np.sum(np.abs(W)))


@pytest.mark.parametrize("classes,reg,a", [(2, 1e-2, 0.0), (2, 3e-3, 1.0), (2, 1e-2, 0.5), (4, 1e-2, 0.0),
                                           (3, 5e-3, 0.5)])
def test_logistic_vs_sklearn(device, classes, reg, a):
    """Binomial / multinomial x L2 / L1 / elastic-net against sklearn (Spark objective mapping)."""
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X, y = _data(600, 12, classes, seed=classes)
    model = LogisticRegression(regParam=reg, elasticNetParam=a, standardization=False, maxIter=2000,
                               tol=1e-12).fit(DataFrame.from_numpy(X, y))
    W = np.asarray(model.coef_)
    b = np.asarray(model.intercept_)
    Wsk, bsk = _sk(X, y, reg, a, classes > 2)
    if classes > 2:
        bsk = bsk - bsk.mean()
    f_ours = _spark_objective(X, y, W, b, reg, a)
    f_sk = _spark_objective(X, y, Wsk, bsk, reg, a)
    # same optimum: objective within 1e-7 relative, coefficients within 2e-3
    assert f_ours <= f_sk * (1 + 1e-7) + 1e-12, (f_ours, f_sk)
    np.testing.assert_allclose(W, Wsk, atol=2e-3, rtol=2e-3)
    np.testing.assert_allclose(b, bsk, atol=2e-3, rtol=2e-3)
    if a > 0:  # OWL-QN produces exact zeros where sklearn's saga does
        assert np.all((np.abs(Wsk) < 1e-6) <= (np.abs(W) < 1e-5))


def test_logistic_standardization_matches_scaled_problem(device):
    """standardization=True == the unstandardised fit of X / sigma (Spark's definition)."""
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X, y = _data(500, 6, 2, seed=7)
    X[:, 1] *= 25.0
    sig = X.astype(np.float64).std(0, ddof=1)
    m1 = LogisticRegression(regParam=0.02, standardization=True, maxIter=1000, tol=1e-12).fit(DataFrame.from_numpy(X, y))
    m2 = LogisticRegression(regParam=0.02, standardization=False, maxIter=1000, tol=1e-12).fit(
        DataFrame.from_numpy((X / sig).astype(np.float32), y))
    np.testing.assert_allclose(np.asarray(m1.coef_)[0] * sig, np.asarray(m2.coef_)[0], rtol=2e-3, atol=2e-4)


def test_host_qn_quadratic():
    """L-BFGS on a convex quadratic reaches the exact minimiser (compact-form direction)."""
    rng = np.random.default_rng(0)
    n = 30
    A = rng.standard_normal((n, n))
    H = A @ A.T + n * np.eye(n)
    c = rng.standard_normal(n)
    P = QNProblem(n=n, K=1, fit_intercept=False, m_total=1.0, l2=np.zeros(n), l1=np.zeros(n),
                  inv_sigma=np.ones(n), max_iter=500, tol=1e-14)
    st = HostQN(P, np.zeros(n))
    while not st.done:
        w = st.wb()[:n]
        out = np.concatenate([H @ w - c, [0.0], [0.5 * w @ H @ w - c @ w]])
        st.step(out)
    np.testing.assert_allclose(st.x, np.linalg.solve(H, c), rtol=1e-8, atol=1e-10)
    assert st.iter < 100


def test_host_qn_l1_sparsity():
    """OWL-QN on a lasso problem: the known soft-threshold solution of a diagonal quadratic."""
    n = 8
    h = np.arange(1, n + 1, dtype=np.float64)
    c = np.linspace(-2, 2, n)
    lam = 0.7
    P = QNProblem(n=n, K=1, fit_intercept=False, m_total=1.0, l2=np.zeros(n), l1=np.full(n, lam),
                  inv_sigma=np.ones(n), max_iter=500, tol=1e-14)
    st = HostQN(P, np.zeros(n))
    while not st.done:
        w = st.wb()[:n]
        st.step(np.concatenate([h * w - c, [0.0], [0.5 * np.sum(h * w * w) - c @ w]]))
    expect = np.sign(c) * np.maximum(np.abs(c) - lam, 0) / h
    np.testing.assert_allclose(st.x, expect, atol=1e-8)
    assert np.all(st.x[np.abs(c) <= lam] == 0.0)


def test_logistic_reports_solver_path(device):
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X, y = _data(300, 8, 3, seed=3)
    model = LogisticRegression(regParam=1e-2, maxIter=50).fit(DataFrame.from_numpy(X, y))
    info = model._solver_info
    assert info["n_evals"] >= model.num_iters >= 1
    if device == "gpu":
        assert info["path"] == "two_pass_multinomial_f32"
    else:
        assert info["path"] == "torch-cpu"


# ---------------------------------------------------------------------------------- GPU kernels
def _ref_loss_grad(X, y, W, b, K):
    Xd = X.double().cpu()
    yd = y.double().cpu()
    Wd = W.double().cpu().view(K, -1)
    Z = Xd @ Wd.T + b.double().cpu().view(1, K)
    if K == 1:
        z = Z.view(-1)
        r = (torch.sigmoid(z) - yd).view(-1, 1)
        loss = (torch.nn.functional.softplus(z) - yd * z).sum()
    else:
        lse = torch.logsumexp(Z, 1)
        Y = torch.nn.functional.one_hot(yd.long(), K).double()
        r = torch.exp(Z - lse.view(-1, 1)) - Y
        loss = (lse - (Z * Y).sum(1)).sum()
    return torch.cat([(r.T @ Xd).reshape(-1), r.sum(0), loss.view(1)])


@pytest.mark.gpu
@pytest.mark.parametrize("m,n,K,dtype,path", [
    (5000, 3000, 1, torch.float32, "fused_binary_f32"),
    (3001, 130, 1, torch.float32, "fused_binary_f32"),
    (2000, 5000, 1, torch.float32, "lds_binary_f32"),
    (3000, 257, 1, torch.float64, "lds_binary_f64"),
    (4000, 3000, 10, torch.float32, "two_pass_multinomial_f32"),
    (3000, 129, 3, torch.float32, "two_pass_multinomial_f32"),
    (2500, 1001, 16, torch.float32, "two_pass_multinomial_f32"),
    (2000, 4096, 5, torch.float32, "two_pass_multinomial_f32"),
    (4000, 3000, 10, torch.float32, "fused_multinomial_f32"),
    (3000, 129, 3, torch.float32, "fused_multinomial_f32"),
    (1500, 300, 20, torch.float32, "two_pass_wide_f32"),
    (1200, 257, 70, torch.float32, "two_pass_wide_f32"),
    (600, 20000, 1, torch.float32, "two_pass_binary_f32"),
    (1500, 300, 20, torch.float64, "two_pass_multinomial_f64"),
    (2000, 77, 3, torch.float64, "two_pass_multinomial_f64"),
    (5000, 3000, 1, torch.float32, "two_pass_deterministic_f32"),
    (3001, 130, 1, torch.float32, "two_pass_deterministic_f32"),
    (4000, 3000, 10, torch.float32, "two_pass_deterministic_f32"),
    (3000, 129, 3, torch.float32, "two_pass_deterministic_f32"),
])
def test_logistic_loss_grad_kernels(gpu_device, m, n, K, dtype, path, monkeypatch):
    if path == "fused_multinomial_f32":
        monkeypatch.setenv("SRML_LOGREG_FUSED", "1")
    if path == "two_pass_deterministic_f32":
        monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(m + n + K)
    X = torch.randn(m, n, generator=g, dtype=torch.float64).to(dtype).to(gpu_device)
    if K == 1:
        y = (torch.rand(m, generator=g) < 0.4).float().to(gpu_device)
    else:
        y = torch.randint(0, K, (m,), generator=g).float().to(gpu_device)
    Kk = K
    W = (0.05 * torch.randn(Kk * n, generator=g, dtype=torch.float64)).to(gpu_device)
    b = (0.3 * torch.randn(Kk, generator=g, dtype=torch.float64)).to(gpu_device)
    assert ops.logistic_path(X, Kk) == path
    out = torch.zeros(Kk * n + Kk + 1, dtype=torch.float64, device=gpu_device)
    ops.logistic_loss_grad(X, y, W, b, Kk, out)
    ops.logistic_loss_grad(X, y, W, b, Kk, out)  # accumulates
    ref = 2 * _ref_loss_grad(X, y, W, b, Kk)
    got = out.cpu()
    scale = ref[:-1].abs().max().item()
    assert (got[:-1] - ref[:-1]).abs().max().item() <= 2e-5 * scale + 1e-6
    assert abs(got[-1].item() - ref[-1].item()) <= 1e-5 * abs(ref[-1].item())
    # the done flag short-circuits the pass
    flag = torch.ones(1, dtype=torch.int32, device=gpu_device)
    out2 = torch.zeros_like(out)
    ops.logistic_loss_grad(X, y, W, b, Kk, out2, flag)
    if not path.startswith("torch"):
        assert out2.abs().max().item() == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("K,l1", [(1, 0.0), (1, 0.01), (4, 0.0), (3, 0.02)])
def test_qn_kernel_matches_host(gpu_device, K, l1):
    """The device state machine takes the same path as HostQN on a logistic problem."""
    m, n = 2000, 40
    g = torch.Generator().manual_seed(11 + K)
    Xc = torch.randn(m, n, generator=g, dtype=torch.float64)
    if K == 1:
        y = (Xc[:, 0] + 0.5 * torch.randn(m, generator=g, dtype=torch.float64) > 0).double()
    else:
        y = torch.argmax(Xc[:, :K] + 0.5 * torch.randn(m, K, generator=g, dtype=torch.float64), 1).double()
    N = K * n + K
    P = QNProblem(n=n, K=K, fit_intercept=True, m_total=float(m),
                  l2=np.concatenate([np.full(K * n, 0.01), np.zeros(K)]),
                  l1=np.concatenate([np.full(K * n, l1), np.zeros(K)]),
                  inv_sigma=np.linspace(0.5, 1.5, n), max_iter=60 if l1 == 0.0 else 300, tol=1e-12)

    def ev_cpu(w, b, flag, out):
        out += _ref_loss_grad(Xc, y, w, b, K)

    host = minimize(P, np.zeros(N), ev_cpu, None, torch.device("cpu"))
    Xg, yg = Xc.to(gpu_device), y.to(gpu_device)

    def ev_gpu(w, b, flag, out):
        out += _ref_loss_grad(Xg, yg, w, b, K).to(gpu_device)

    dev = minimize(P, np.zeros(N), ev_gpu, None, gpu_device, batch=4)
    info = {k: (host[k], dev[k]) for k in ("iter", "n_evals", "status", "f")}
    if l1 == 0.0:
        # smooth problem: identical decisions, states equal to rounding
        assert dev["iter"] == host["iter"] and dev["status"] == host["status"], info
        assert abs(dev["f"] - host["f"]) <= 1e-10 * abs(host["f"]), info
        np.testing.assert_allclose(dev["theta"], host["theta"], rtol=1e-6, atol=1e-8)
    else:
        # OWL-QN's orthant projections make the path sensitive to the last bit of the reductions:
        # require the same optimum instead of the same trajectory
        assert abs(dev["f"] - host["f"]) <= 1e-7 * abs(host["f"]), info
        np.testing.assert_allclose(dev["theta"], host["theta"], atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("K,l1,n", [(1, 0.0, 3000), (4, 0.0, 700), (1, 0.01, 1500)])
def test_qn_multiblock_step_matches_single_block(gpu_device, K, l1, n, monkeypatch):
    """srml_qn_step_mb (four G-block launches) advances the same state machine as the single-block
    step: same decisions and iterations on smooth problems, same optimum with OWL-QN."""
    from spark_rapids_ml_nai_amd.models import qn as qnm

    m = 3000
    g = torch.Generator().manual_seed(21 + K)
    Xc = torch.randn(m, n, generator=g, dtype=torch.float64)
    if K == 1:
        y = (Xc[:, 0] + 0.5 * torch.randn(m, generator=g, dtype=torch.float64) > 0).double()
    else:
        y = torch.argmax(Xc[:, :K] + 0.5 * torch.randn(m, K, generator=g, dtype=torch.float64), 1).double()
    N = K * n + K
    P = QNProblem(n=n, K=K, fit_intercept=True, m_total=float(m),
                  l2=np.concatenate([np.full(K * n, 0.01), np.zeros(K)]),
                  l1=np.concatenate([np.full(K * n, l1), np.zeros(K)]),
                  inv_sigma=np.linspace(0.5, 1.5, n), max_iter=40 if l1 == 0.0 else 150, tol=1e-12)
    Xg, yg = Xc.to(gpu_device), y.to(gpu_device)

    def ev_gpu(w, b, flag, out):
        out += _ref_loss_grad(Xg, yg, w, b, K).to(gpu_device)

    res = {}
    for mode in ("single", "mb", "fused"):  # srml_qn_step / srml_qn_step_mb / srml_qn_step_fused
        monkeypatch.setattr(qnm, "QN_MB", mode != "single")
        monkeypatch.setattr(qnm, "QN_STEP", mode)
        res[mode] = minimize(P, np.zeros(N), ev_gpu, None, gpu_device, batch=4)
    a = res["single"]
    for mode in ("mb", "fused"):
        b = res[mode]
        info = {k: (a[k], b[k]) for k in ("iter", "n_evals", "status", "f")}
        info["mode"] = mode
        if l1 == 0.0:
            assert a["iter"] == b["iter"] and a["status"] == b["status"] and a["n_evals"] == b["n_evals"], info
            assert abs(a["f"] - b["f"]) <= 1e-10 * abs(a["f"]), info
            np.testing.assert_allclose(b["theta"], a["theta"], rtol=1e-6, atol=1e-8)
        else:
            assert abs(a["f"] - b["f"]) <= 1e-7 * abs(a["f"]), info
            np.testing.assert_allclose(b["theta"], a["theta"], atol=2e-3)


@pytest.mark.gpu
def test_logistic_fit_fused_fold_matches_unfused(gpu_device, monkeypatch):
    """One-rank binary LogReg with the fold moved into the optimiser step (the evaluation leaves
    its partial rows; srml_qn_step_mbf / srml_qn_step_fused fold them) reproduces the fit whose
    evaluation folds them itself."""
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.models import qn as qnm
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    rng = np.random.default_rng(11)
    m, n = 20000, 1500  # a fold-workspace shape (1024 < n <= 4096)
    X = rng.standard_normal((m, n)).astype(np.float32)
    y = (X[:, :8].sum(1) + 0.5 * rng.standard_normal(m) > 0).astype(np.float32)
    Xt, yt = torch.from_numpy(X).to(gpu_device), torch.from_numpy(y).to(gpu_device)
    assert ops.logreg_workspace(Xt) is not None and ops.logistic_path(Xt, 1) == "fused_binary_f32"
    ctx = WorkerContext.single(gpu_device)
    out = {}
    for mode in ("single", "mb", "fused"):  # unfolded single-block step / srml_qn_step_mbf / fused
        monkeypatch.setattr(qnm, "QN_MB", mode != "single")
        monkeypatch.setattr(qnm, "QN_STEP", mode)
        out[mode] = logistic_fit(Xt, yt, m, ctx, reg=1e-3, l1_ratio=0.0, fit_intercept=True,
                                 standardization=True, max_iter=60, tol=1e-10)
    a = out["single"]
    for mode in ("mb", "fused"):
        b = out[mode]
        # the fp32 evaluation's partials are summed in another order, so a convergence test at
        # tol 1e-10 (below fp32 noise) may stop at another iteration: compare the optimum
        assert abs(a["objective"] - b["objective"]) <= 1e-6 * abs(a["objective"]), (mode, a["objective"],
                                                                                    b["objective"])
        np.testing.assert_allclose(np.asarray(b["coef_"]), np.asarray(a["coef_"]), rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1100, 256])  # prefetching column-split kernel / narrow kernel
def test_logreg_margin_only_evaluation_matches_full(gpu_device, n):
    """The line-search margin cache: full evaluations store the row margins; a margins-only
    evaluation at beta between two stored points gives the loss / bias gradient of a full pass at
    w0 + beta (w1 - w0) (margins are linear along a search direction) and no gradient columns."""
    from spark_rapids_ml_nai_amd import ops

    rng = np.random.default_rng(21)
    m = 9000
    X = torch.from_numpy(rng.standard_normal((m, n)).astype(np.float32)).to(gpu_device)
    y = torch.from_numpy((rng.random(m) > 0.4).astype(np.float32)).to(gpu_device)
    assert ops.logreg_zcache_ok(X)
    w0 = torch.from_numpy(rng.standard_normal(n) * 0.05).to(gpu_device)
    w1 = torch.from_numpy(rng.standard_normal(n) * 0.05).to(gpu_device)
    b0 = torch.tensor([0.3], dtype=torch.float64, device=gpu_device)
    b1 = torch.tensor([-0.2], dtype=torch.float64, device=gpu_device)
    fl = torch.zeros(16, dtype=torch.int32, device=gpu_device)
    zb = torch.zeros(2 * m, dtype=torch.float64, device=gpu_device)
    sc = torch.zeros(8, dtype=torch.float64, device=gpu_device)
    outs = []
    for w, b, zsel in ((w0, b0, 1), (w1, b1, 0)):  # margins of w0 -> zb[0:m] (z0), w1 -> zb[m:] (z1)
        fl[10] = zsel
        o = torch.zeros(n + 2, dtype=torch.float64, device=gpu_device)
        ops.logistic_loss_grad(X, y, w, b, 1, o, zcache=(fl, zb, sc))
        outs.append(o)
    fl[10] = 0
    fl[9] = 1
    beta = 0.37
    sc[6] = beta
    oc = torch.zeros(n + 2, dtype=torch.float64, device=gpu_device)
    ops.logistic_loss_grad(X, y, w0, b0, 1, oc, zcache=(fl, zb, sc))
    of = torch.zeros(n + 2, dtype=torch.float64, device=gpu_device)
    ops.logistic_loss_grad(X, y, w0 + beta * (w1 - w0), b0 + beta * (b1 - b0), 1, of)
    assert torch.count_nonzero(oc[:n]) == 0
    torch.testing.assert_close(oc[n:], of[n:], rtol=1e-9, atol=1e-9)
    # the stored margins themselves: z = X w + b in fp64 from fp32 rows
    zref = X.double() @ w0 + b0
    torch.testing.assert_close(zb[:m], zref, rtol=1e-9, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("n,classes", [(1200, 2), (256, 2), (300, 4), (200, 11), (2000, 9)])  # last: N > 16384
def test_logistic_fit_margin_cache_matches_full_evaluations(gpu_device, monkeypatch, n, classes):
    """A fit whose rejected line-search trials are margins-only evaluations (binary: narrow /
    prefetching kernels; multinomial: the two-pass margin / residual / X^T R passes) reaches the
    optimum of the all-full-evaluation fit, with fewer passes over X."""
    from spark_rapids_ml_nai_amd.models import qn as qnm
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    rng = np.random.default_rng(12)
    m = 30000
    X = rng.standard_normal((m, n)).astype(np.float32)
    score = X[:, :10].sum(1) + 2.0 * rng.standard_normal(m)
    if classes == 2:
        y = (score > 0).astype(np.float32)
    else:
        y = np.clip(np.floor((score + 8.0) * classes / 16.0), 0, classes - 1).astype(np.float32)
    Xt, yt = torch.from_numpy(X).to(gpu_device), torch.from_numpy(y).to(gpu_device)
    ctx = WorkerContext.single(gpu_device)
    out = {}
    for zc in (False, True):
        monkeypatch.setattr(qnm, "QN_ZCACHE", zc)
        out[zc] = logistic_fit(Xt, yt, m, ctx, reg=1e-5, l1_ratio=0.0, fit_intercept=True,
                               standardization=False, max_iter=200, tol=1e-30)
    a, b = out[False], out[True]
    assert abs(a["objective"] - b["objective"]) <= 1e-7 * abs(a["objective"]), (a["objective"], b["objective"])
    np.testing.assert_allclose(np.asarray(b["coef_"]), np.asarray(a["coef_"]), rtol=2e-2, atol=2e-3)
    sb = b["_solver"]
    assert sb.get("n_margin_only", 0) > 0, sb
    if classes == 2:
        # full passes per L-BFGS iteration: the cache serves the rejected trials. (Total pass counts
        # are not compared: at tol 1e-30 both fits end when the search runs on fp noise, and the
        # atomics' summation order makes that tail's length differ run to run.)
        full_b = (sb["n_evals"] - sb["n_margin_only"]) / max(1, b["num_iters"])
        full_a = a["_solver"]["n_evals"] / max(1, a["num_iters"])
        assert full_b <= full_a, (a["_solver"], a["num_iters"], sb, b["num_iters"])


@pytest.mark.gpu
@pytest.mark.parametrize("fit_intercept,standardization", [(False, False), (True, True), (False, True)])
def test_logistic_fit_margin_cache_intercept_and_scaling(gpu_device, monkeypatch, fit_intercept, standardization):
    """The margins stay linear in the step with or without an intercept and with the
    standardisation folded into the coefficients: same optimum as the all-full-evaluation fit."""
    from spark_rapids_ml_nai_amd.models import qn as qnm
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    rng = np.random.default_rng(31)
    m, n = 20000, 1100
    X = (rng.standard_normal((m, n)) * rng.uniform(0.2, 5.0, n) + rng.uniform(-1, 1, n)).astype(np.float32)
    y = (X[:, :6].sum(1) + rng.standard_normal(m) > 0).astype(np.float32)
    Xt, yt = torch.from_numpy(X).to(gpu_device), torch.from_numpy(y).to(gpu_device)
    ctx = WorkerContext.single(gpu_device)
    out = {}
    for zc in (False, True):
        monkeypatch.setattr(qnm, "QN_ZCACHE", zc)
        out[zc] = logistic_fit(Xt, yt, m, ctx, reg=1e-4, l1_ratio=0.0, fit_intercept=fit_intercept,
                               standardization=standardization, max_iter=100, tol=1e-30)
    a, b = out[False], out[True]
    assert abs(a["objective"] - b["objective"]) <= 1e-7 * abs(a["objective"]), (a["objective"], b["objective"])
    assert b["_solver"].get("n_margin_only", 0) > 0, b["_solver"]
    np.testing.assert_allclose(np.asarray(b["coef_"]), np.asarray(a["coef_"]), rtol=2e-2, atol=2e-3)
    np.testing.assert_allclose(np.asarray(b["intercept_"]), np.asarray(a["intercept_"]), rtol=2e-3, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1501, 3001])
def test_logistic_fit_unaligned_width_has_no_fold(gpu_device, monkeypatch, n):
    """A width the prefetching kernel rejects (n % 4 != 0) gets no partial-row workspace, so the
    default (mb) step cannot fold rows nobody wrote: the fit equals the unfolded single step."""
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.models import qn as qnm
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    rng = np.random.default_rng(5)
    m = 6000
    X = rng.standard_normal((m, n)).astype(np.float32)
    y = (X[:, :8].sum(1) + 0.5 * rng.standard_normal(m) > 0).astype(np.float32)
    Xt, yt = torch.from_numpy(X).to(gpu_device), torch.from_numpy(y).to(gpu_device)
    assert ops.logreg_workspace(Xt) is None
    ctx = WorkerContext.single(gpu_device)
    out = {}
    for mode in ("single", "mb"):
        monkeypatch.setattr(qnm, "QN_MB", mode != "single")
        monkeypatch.setattr(qnm, "QN_STEP", mode)
        out[mode] = logistic_fit(Xt, yt, m, ctx, reg=1e-2, l1_ratio=0.0, fit_intercept=True,
                                 standardization=True, max_iter=40, tol=1e-10)
    a, b = out["single"], out["mb"]
    assert np.isfinite(np.asarray(b["coef_"])).all()
    assert abs(a["objective"] - b["objective"]) <= 1e-6 * abs(a["objective"])
    np.testing.assert_allclose(np.asarray(b["coef_"]), np.asarray(a["coef_"]), rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
def test_logistic_fit_multi_batched_matches_single(gpu_device):
    """Hyper-parameter batching: a grid of binary fits sharing every pass over X (srml_mbin_f32 +
    srml_qn_step_batch) reproduces the one-at-a-time fits."""
    import torch

    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit, logistic_fit_multi, logistic_stats
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    rng = np.random.default_rng(3)
    m, n = 6000, 40
    X = (rng.standard_normal((m, n)) * rng.uniform(0.5, 2.0, n)).astype(np.float32)
    w = rng.standard_normal(n)
    y = (X @ w + 0.3 * rng.standard_normal(m) > 0).astype(np.float32)
    Xt = torch.from_numpy(X).to(gpu_device)
    yt = torch.from_numpy(y).to(gpu_device)
    ctx = WorkerContext.single(gpu_device)
    stats = logistic_stats(Xt, yt, m, ctx, False)
    settings = [dict(reg=r, l1_ratio=a, fit_intercept=fi, standardization=sd, max_iter=100, tol=1e-10)
                for r, a, fi, sd in [(1e-3, 0.0, True, True), (1e-2, 0.0, True, False), (1e-3, 0.5, True, True),
                                     (1e-2, 1.0, False, True), (0.1, 0.0, True, True)]]
    assert ops.mbin_supported(Xt, len(settings))
    batched = logistic_fit_multi(Xt, yt, m, ctx, settings, stats=stats)
    for s, b in zip(settings, batched):
        assert b["_solver"]["path"] == "batched_binary_f32"
        one = logistic_fit(Xt, yt, m, ctx, s["reg"], s["l1_ratio"], s["fit_intercept"], s["standardization"],
                           s["max_iter"], s["tol"], stats=stats)
        assert abs(b["objective"] - one["objective"]) <= 1e-6 * max(1.0, abs(one["objective"]))
        np.testing.assert_allclose(np.asarray(b["coef_"]), np.asarray(one["coef_"]), rtol=2e-3, atol=2e-3)
        np.testing.assert_allclose(b["intercept_"], one["intercept_"], rtol=2e-3, atol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["0", "1"])
def test_mbin_kernel_matches_torch(gpu_device, fused, monkeypatch):
    monkeypatch.setenv("SRML_LOGREG_FUSED", fused)
    import torch

    from spark_rapids_ml_nai_amd import ops

    rng = np.random.default_rng(4)
    m, n, M = 5000, 300, 7
    X = torch.from_numpy(rng.standard_normal((m, n)).astype(np.float32))
    y = torch.from_numpy((rng.random(m) > 0.4).astype(np.float32))
    WB = torch.from_numpy(rng.standard_normal((M, n + 1)) * 0.05)
    ref = ops.logistic_loss_grad_multi(X, y, WB, torch.zeros((M, n + 2), dtype=torch.float64))
    got = ops.logistic_loss_grad_multi(X.to(gpu_device), y.to(gpu_device), WB.to(gpu_device),
                                       torch.zeros((M, n + 2), dtype=torch.float64, device=gpu_device))
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("classes", [2, 4])
def test_logistic_deterministic_mode_bit_identical(gpu_device, classes, monkeypatch):
    """SRML_DETERMINISTIC=1: two fits give bit-identical coefficients (ordered folds, no atomics)
    and agree with the default (atomic) path to solver tolerance."""
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X, y = _data(20000, 300, classes, seed=3)
    df = DataFrame.from_numpy(X, y)
    est = LogisticRegression(regParam=1e-3, maxIter=60, tol=1e-10, standardization=False)
    ref = est.fit(df)
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    a = est.fit(df)
    b = est.fit(df)
    assert np.array_equal(np.asarray(a.coef_), np.asarray(b.coef_))
    assert np.array_equal(np.asarray(a.intercept_), np.asarray(b.intercept_))
    np.testing.assert_allclose(np.asarray(a.coef_), np.asarray(ref.coef_), atol=2e-3, rtol=2e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("classes", [2, 4])
def test_logistic_graph_replay_matches_eager(gpu_device, classes, monkeypatch):
    """One-rank fits replay the QN batch (evaluation + optimiser step, x8) from a HIP graph; the
    fit matches the eager launches to solver tolerance (the fp64 atomic folds reorder between any
    two runs) and the graph was really replayed."""
    from spark_rapids_ml_nai_amd.classification import LogisticRegression
    from spark_rapids_ml_nai_amd.models import qn

    X, y = _data(20000, 300, classes, seed=5)
    df = DataFrame.from_numpy(X, y)
    est = LogisticRegression(regParam=1e-3, maxIter=80, tol=1e-10)
    monkeypatch.setattr(qn, "QN_GRAPH", False)
    r0 = dict(qn.GRAPH_STATS)
    eager = est.fit(df)
    assert qn.GRAPH_STATS == r0
    monkeypatch.setattr(qn, "QN_GRAPH", True)
    graph = est.fit(df)
    assert qn.GRAPH_STATS["captures"] == r0["captures"] + 1 and qn.GRAPH_STATS["replays"] > r0["replays"]
    np.testing.assert_allclose(np.asarray(graph.coef_), np.asarray(eager.coef_), atol=2e-3, rtol=2e-3)
    np.testing.assert_allclose(graph.intercept_, eager.intercept_, atol=2e-3, rtol=2e-3)
    assert abs(graph.objective - eager.objective) <= 1e-7 * abs(eager.objective)
