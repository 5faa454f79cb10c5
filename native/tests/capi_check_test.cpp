// Argument validation of the C ABI (ops/csrc/capi_check.h) at its edges: negative and zero
// dimensions, leading dimensions below the stored rows, size_t overflow of the buffer sizes,
// null pointers, zero-length accumulate. Linked against the host stub for the sanitizer tier
// (the GPU library runs the same checks before touching caller memory).
#include <cstdint>
#include <cstdio>
#include <vector>

#include "capi_check.h"
#include "srml/srml.h"

static int failures = 0;
#define EXPECT(cond)                                             \
  do {                                                           \
    if (!(cond)) {                                               \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                \
    }                                                            \
  } while (0)

int main() {
  size_t na, nb, nc;
  // column-major 3x2 = op(A) 3x4 . op(B) 4x2
  EXPECT(srml_check_gemm(0, 0, 3, 2, 4, 3, 4, 3, &na, &nb, &nc) == 0 && na == 12 && nb == 8 && nc == 6);
  EXPECT(srml_check_gemm(1, 1, 3, 2, 4, 4, 2, 3, &na, &nb, &nc) == 0 && na == 12 && nb == 8);
  EXPECT(srml_check_gemm(0, 0, 3, 2, 4, 2, 4, 3, &na, &nb, &nc) == SRML_EARG);  // lda < m
  EXPECT(srml_check_gemm(1, 0, 3, 2, 4, 3, 4, 3, &na, &nb, &nc) == SRML_EARG);  // transposed A: lda < k
  EXPECT(srml_check_gemm(0, 0, 3, 2, 4, 3, 4, 2, &na, &nb, &nc) == SRML_EARG);  // ldc < m
  EXPECT(srml_check_gemm(0, 0, -1, 2, 4, 3, 4, 3, &na, &nb, &nc) == SRML_EARG);
  EXPECT(srml_check_gemm(0, 0, 0, 0, 0, 1, 1, 1, &na, &nb, &nc) == 0);
  size_t nx, ncov;
  EXPECT(srml_check_cov(-5, 3, &nx, &ncov) == SRML_EARG);
  EXPECT(srml_check_cov(INT64_MAX / 2, 1 << 30, &nx, &ncov) == SRML_ESIZE);  // rows * cols wraps size_t
  size_t nm;
  EXPECT(srml_check_svd(-1, &nm) == SRML_EARG);
  EXPECT(srml_check_svd(70000, &nm) == 0 && nm == (size_t)70000 * 70000);
  size_t np;
  EXPECT(srml_check_xp(10, -1, 3, &nx, &np, &nc) == SRML_EARG);

  // entry points reject bad arguments before reading any buffer
  std::vector<double> a(12, 1.0), b(8, 1.0), c(6, 0.0);
  EXPECT(srml_capi_dgemm(0, 0, 3, 2, 4, 1.0, a.data(), 2, b.data(), 4, 0.0, c.data(), 3, 0) == SRML_EARG);
  EXPECT(srml_capi_dgemm(0, 0, 3, 2, 4, 1.0, nullptr, 3, b.data(), 4, 0.0, c.data(), 3, 0) == SRML_EARG);
  EXPECT(srml_capi_dgemm(0, 0, 3, 2, 4, 1.0, a.data(), 3, b.data(), 4, 0.0, c.data(), 3, 0) == 0 && c[5] == 4.0);
  // lda larger than m: only the leading m entries of each stored column are read
  std::vector<double> a2(5 * 4, 1.0);
  EXPECT(srml_capi_dgemm(0, 0, 3, 2, 4, 1.0, a2.data(), 5, b.data(), 4, 0.0, c.data(), 3, 0) == 0 && c[0] == 4.0);
  EXPECT(srml_capi_dgemm_cov(nullptr, 4, 3, c.data(), 0) == SRML_EARG);
  std::vector<double> u(4), s(2);
  EXPECT(srml_capi_cal_svd(a.data(), -2, u.data(), s.data(), 0) == SRML_EARG);
  EXPECT(srml_capi_accumulate_cov(nullptr, nullptr, 0) == 0);
  EXPECT(srml_capi_accumulate_cov(c.data(), nullptr, 3) == SRML_EARG);
  std::printf("capi checks: %s\n", failures ? "FAILED" : "ok");
  return failures ? 1 : 0;
}
