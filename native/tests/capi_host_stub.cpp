// Host-only stand-in for the srml_capi_* entry points of libsrml_ops.so, for the ASan/UBSan build
// of the JNI shim (ci/run_tests.sh sanitize; tests/test_native_sanitize.py). It runs the SAME
// argument validation as the device library (ops/csrc/capi_check.h) and computes the results with
// plain loops (cyclic Jacobi for the eigendecomposition), so the sanitizers see every byte the
// shim and the checks touch on the host. No GPU, no HIP runtime.
#include <algorithm>
#include <cmath>
#include <vector>

#include "capi_check.h"
#include "srml/srml.h"

extern "C" {

int srml_capi_dgemm(int transa, int transb, int m, int n, int k, double alpha, const double* A, int lda,
                    const double* B, int ldb, double beta, double* C, int ldc, int /*device*/) {
  size_t na = 0, nb = 0, nc = 0;
  const int chk = srml_check_gemm(transa, transb, m, n, k, lda, ldb, ldc, &na, &nb, &nc);
  if (chk) return chk;
  if (m == 0 || n == 0) return 0;
  if ((na && !A) || (nb && !B) || !C) return SRML_EARG;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < m; ++i) {
      double acc = 0.0;
      for (int l = 0; l < k; ++l) {
        const double a = transa ? A[(size_t)i * lda + l] : A[(size_t)l * lda + i];
        const double b = transb ? B[(size_t)l * ldb + j] : B[(size_t)j * ldb + l];
        acc += a * b;
      }
      double& c = C[(size_t)j * ldc + i];
      c = alpha * acc + (beta != 0.0 ? beta * c : 0.0);
    }
  return 0;
}

int srml_capi_dgemm_device(const double* X, long rows, int n, const double* P, int k, int /*p_on_host*/, double* C,
                           void* /*stream*/) {
  size_t nx = 0, np = 0, nc = 0;
  const int chk = srml_check_xp(rows, n, k, &nx, &np, &nc);
  if (chk) return chk;
  if (rows == 0 || k == 0) return 0;
  if ((nx && !X) || (np && !P) || !C) return SRML_EARG;
  for (long r = 0; r < rows; ++r)
    for (int j = 0; j < k; ++j) {
      double acc = 0.0;
      for (int i = 0; i < n; ++i) acc += X[(size_t)r * n + i] * P[(size_t)i * k + j];
      C[(size_t)r * k + j] = acc;
    }
  return 0;
}

int srml_capi_dgemm_cov(const double* X, long rows, int cols, double* C, int /*device*/) {
  size_t nx = 0, ncov = 0;
  const int chk = srml_check_cov(rows, cols, &nx, &ncov);
  if (chk) return chk;
  if (cols == 0) return 0;
  if ((nx && !X) || !C) return SRML_EARG;
  std::fill(C, C + ncov, 0.0);
  for (long r = 0; r < rows; ++r)
    for (int i = 0; i < cols; ++i)
      for (int j = 0; j < cols; ++j) C[(size_t)i * cols + j] += X[(size_t)r * cols + i] * X[(size_t)r * cols + j];
  return 0;
}

int srml_capi_cal_svd(const double* A, int m, double* U, double* S, int /*device*/) {
  size_t nm = 0;
  const int chk = srml_check_svd(m, &nm);
  if (chk) return chk;
  if (m == 0) return 0;
  if (!A || !U || !S) return SRML_EARG;
  std::vector<double> a(A, A + nm), v(nm, 0.0);
  for (int i = 0; i < m; ++i) v[(size_t)i * m + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {  // cyclic Jacobi rotations
    double off = 0.0;
    for (int p = 0; p < m; ++p)
      for (int q = p + 1; q < m; ++q) off += a[(size_t)p * m + q] * a[(size_t)p * m + q];
    if (off < 1e-30) break;
    for (int p = 0; p < m; ++p)
      for (int q = p + 1; q < m; ++q) {
        const double apq = a[(size_t)p * m + q];
        if (std::fabs(apq) < 1e-300) continue;
        const double th = (a[(size_t)q * m + q] - a[(size_t)p * m + p]) / (2.0 * apq);
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int r = 0; r < m; ++r) {  // A <- J^T A J, V <- V J
          const double arp = a[(size_t)r * m + p], arq = a[(size_t)r * m + q];
          a[(size_t)r * m + p] = c * arp - s * arq;
          a[(size_t)r * m + q] = s * arp + c * arq;
        }
        for (int r = 0; r < m; ++r) {
          const double apr = a[(size_t)p * m + r], aqr = a[(size_t)q * m + r];
          a[(size_t)p * m + r] = c * apr - s * aqr;
          a[(size_t)q * m + r] = s * apr + c * aqr;
        }
        for (int r = 0; r < m; ++r) {
          const double vrp = v[(size_t)r * m + p], vrq = v[(size_t)r * m + q];
          v[(size_t)r * m + p] = c * vrp - s * vrq;
          v[(size_t)r * m + q] = s * vrp + c * vrq;
        }
      }
  }
  std::vector<int> order(m);
  for (int i = 0; i < m; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int x, int y) { return a[(size_t)x * m + x] > a[(size_t)y * m + y]; });
  for (int j = 0; j < m; ++j) {
    const int src = order[j];
    S[j] = std::sqrt(std::max(a[(size_t)src * m + src], 0.0));
    int big = 0;
    for (int i = 0; i < m; ++i)
      if (std::fabs(v[(size_t)i * m + src]) > std::fabs(v[(size_t)big * m + src])) big = i;
    const double sgn = v[(size_t)big * m + src] < 0 ? -1.0 : 1.0;  // N1 signFlip convention
    for (int i = 0; i < m; ++i) U[(size_t)j * m + i] = sgn * v[(size_t)i * m + src];  // column-major
  }
  return 0;
}

int srml_capi_accumulate_cov(double* acc, const double* c, long len) {
  if (len < 0 || (len && (!acc || !c))) return SRML_EARG;
  for (long i = 0; i < len; ++i) acc[i] += c[i];
  return 0;
}

const char* srml_capi_version(void) { return "spark-rapids-ml-nai-amd 24.06.0 (host stub)"; }
}
