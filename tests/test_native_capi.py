"""C ABI / JNI-parity layer (reference jvm/native/src/rapidsml_jni.cu) and the
device Jacobi eigensolver. Oracle: numpy fp64."""
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_capi_program():
    from spark_rapids_ml_nai_amd.native import build_capi

    exe = build_capi.build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


def test_jni_shim_program():
    """native/jni/srml_jni.cpp executed through the test JNIEnv (no JVM): dgemm layout, cov,
    calSVD conventions, accumulateCov, argument checks, pin balance."""
    from spark_rapids_ml_nai_amd.native import build_capi

    build_capi.build()
    r = subprocess.run([build_capi.shim_test_path()], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "jni shim: ok" in r.stdout


def test_capi_python_bindings():
    from spark_rapids_ml_nai_amd import native

    rng = np.random.default_rng(0)
    X = rng.standard_normal((2000, 40))
    np.testing.assert_allclose(native.dgemm_cov(X), X.T @ X, rtol=1e-12, atol=1e-9)
    A = rng.standard_normal((33, 17))
    B = rng.standard_normal((33, 21))
    np.testing.assert_allclose(native.dgemm(A, B, transa=True), A.T @ B, rtol=1e-12, atol=1e-12)
    C = X.T @ X
    U, S = native.cal_svd(C)
    w = np.linalg.eigvalsh(C)[::-1]
    np.testing.assert_allclose(S, np.sqrt(w), rtol=1e-10)
    np.testing.assert_allclose(C @ U, U * (S ** 2), rtol=1e-8, atol=1e-8 * w[0])
    # deterministic signs: max-|x| entry of every column positive
    idx = np.abs(U).argmax(0)
    assert np.all(U[idx, np.arange(U.shape[1])] > 0)
    acc = np.ones(5)
    native.accumulate_cov(acc, np.full(5, 2.0))
    assert np.all(acc == 3.0)


@pytest.mark.parametrize("n", [2, 3, 17, 128, 301])
def test_syevj(gpu_device, n):
    from spark_rapids_ml_nai_amd import ops

    g = torch.Generator().manual_seed(n)
    M = torch.randn(n, n, generator=g, dtype=torch.float64)
    A = M @ M.T + torch.diag(torch.linspace(0, 1, n, dtype=torch.float64))
    w, V = ops.syevj(A.to(gpu_device))
    wr = torch.linalg.eigvalsh(A).flip(0)
    torch.testing.assert_close(w.cpu(), wr, rtol=1e-10, atol=1e-10 * wr[0].item())
    Vc = V.cpu()
    torch.testing.assert_close(Vc.T @ Vc, torch.eye(n, dtype=torch.float64), rtol=0, atol=1e-10)
    torch.testing.assert_close(A @ Vc, Vc * w.cpu(), rtol=0, atol=1e-9 * wr[0].item())
