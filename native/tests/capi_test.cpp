// Stand-alone C++ check of the C ABI against naive host references (runs on the GPU box:
// `python -m spark_rapids_ml_nai_amd.native.build_capi --test`).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "srml/srml.h"

static double rnd(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) & 0xffffff) / double(0x1000000) - 0.5;
}

static int check(const char* what, double err, double tol) {
  std::printf("%-28s max err %.3e (tol %.1e) %s\n", what, err, tol, err <= tol ? "ok" : "FAIL");
  return err <= tol ? 0 : 1;
}

int main() {
  int fails = 0;
  unsigned seed = 7;
  // ---- dgemm (column-major, op(A) = A^T) ----
  const int m = 37, n = 29, k = 53;
  std::vector<double> A(k * m), B(k * n), C(m * n, 1.0), R(m * n);
  for (auto& v : A) v = rnd(seed);
  for (auto& v : B) v = rnd(seed);
  // A stored k x m (lda = k) used transposed, B k x n (ldb = k)
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0;
      for (int l = 0; l < k; ++l) s += A[i * k + l] * B[j * k + l];
      R[j * m + i] = 2.0 * s + 0.5 * 1.0;
    }
  int rc = srml_capi_dgemm(1, 0, m, n, k, 2.0, A.data(), k, B.data(), k, 0.5, C.data(), m, 0);
  double e = 0;
  for (int i = 0; i < m * n; ++i) e = std::fmax(e, std::fabs(C[i] - R[i]));
  fails += rc != 0 || check("srml_capi_dgemm", e, 1e-12);
  // ---- cov ----
  const long rows = 1000;
  const int cols = 24;
  std::vector<double> X(rows * cols), G(cols * cols);
  for (auto& v : X) v = rnd(seed);
  rc = srml_capi_dgemm_cov(X.data(), rows, cols, G.data(), 0);
  e = 0;
  for (int i = 0; i < cols; ++i)
    for (int j = 0; j < cols; ++j) {
      double s = 0;
      for (long r = 0; r < rows; ++r) s += X[r * cols + i] * X[r * cols + j];
      e = std::fmax(e, std::fabs(G[i * cols + j] - s));
    }
  fails += rc != 0 || check("srml_capi_dgemm_cov", e, 1e-10);
  // ---- cal_svd: A = G (SPD); check A u = s^2 u and orthonormality ----
  std::vector<double> U(cols * cols), S(cols);
  rc = srml_capi_cal_svd(G.data(), cols, U.data(), S.data(), 0);
  e = 0;
  for (int c = 0; c < cols; ++c) {
    const double lam = S[c] * S[c];
    for (int i = 0; i < cols; ++i) {
      double s = 0;
      for (int j = 0; j < cols; ++j) s += G[i * cols + j] * U[c * cols + j];
      e = std::fmax(e, std::fabs(s - lam * U[c * cols + i]) / (S[0] * S[0]));
    }
    if (c > 0 && S[c] > S[c - 1] + 1e-12) e = 1.0;
  }
  double o = 0;
  for (int a = 0; a < cols; ++a)
    for (int b = 0; b < cols; ++b) {
      double s = 0;
      for (int i = 0; i < cols; ++i) s += U[a * cols + i] * U[b * cols + i];
      o = std::fmax(o, std::fabs(s - (a == b ? 1.0 : 0.0)));
    }
  fails += rc != 0 || check("srml_capi_cal_svd residual", e, 1e-10);
  fails += check("srml_capi_cal_svd orthonorm", o, 1e-10);
  std::vector<double> acc(10, 1.0), add(10, 2.0);
  srml_capi_accumulate_cov(acc.data(), add.data(), 10);
  fails += check("srml_capi_accumulate_cov", std::fabs(acc[9] - 3.0), 0.0);
  std::printf("%s: %d failure(s)\n", srml_capi_version(), fails);
  return fails ? 1 : 0;
}
