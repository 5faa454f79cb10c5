/* Host-side argument validation of the srml_capi_* host-array API (header-only, no HIP).
 *
 * Shared by the device implementation (spark_rapids_ml_nai_amd/ops/csrc/capi.hip) and the
 * host-only stub used by the ASan/UBSan build of the JNI shim (native/tests/capi_host_stub.cpp),
 * so the sanitizer tier exercises exactly the checks the GPU library runs before it touches
 * caller memory. Status codes: 0 ok, SRML_EARG invalid argument, SRML_ESIZE size overflow.
 */
#ifndef SRML_CAPI_CHECK_H_
#define SRML_CAPI_CHECK_H_

#include <stddef.h>
#include <stdint.h>

#define SRML_EARG (-3)
#define SRML_ESIZE (-4)

#ifdef __cplusplus
extern "C" {
#endif

/* a * b into *out without size_t wrap-around (1 = ok). */
static inline int srml_mul_ok(size_t a, size_t b, size_t* out) {
  if (a != 0 && b > SIZE_MAX / a) return 0;
  *out = a * b;
  return 1;
}

/* Column-major GEMM C(m x n) = op(A) op(B), cuBLAS convention: op(A) is m x k, op(B) is k x n.
 * Checks the dimensions and leading dimensions and returns the element count of each buffer
 * (ld * number of stored columns). */
static inline int srml_check_gemm(int transa, int transb, int m, int n, int k, int lda, int ldb, int ldc,
                                  size_t* na, size_t* nb, size_t* nc) {
  if (m < 0 || n < 0 || k < 0) return SRML_EARG;
  const int a_rows = transa ? k : m, a_cols = transa ? m : k;
  const int b_rows = transb ? n : k, b_cols = transb ? k : n;
  if (lda < (a_rows > 1 ? a_rows : 1) || ldb < (b_rows > 1 ? b_rows : 1) || ldc < (m > 1 ? m : 1)) return SRML_EARG;
  if (!srml_mul_ok((size_t)lda, (size_t)a_cols, na) || !srml_mul_ok((size_t)ldb, (size_t)b_cols, nb) ||
      !srml_mul_ok((size_t)ldc, (size_t)n, nc))
    return SRML_ESIZE;
  if (*na > SIZE_MAX / sizeof(double) || *nb > SIZE_MAX / sizeof(double) || *nc > SIZE_MAX / sizeof(double))
    return SRML_ESIZE;
  return 0;
}

/* X^T X of a rows x cols row-major matrix: element counts of X and C. */
static inline int srml_check_cov(long rows, int cols, size_t* nx, size_t* nc) {
  if (rows < 0 || cols < 0) return SRML_EARG;
  if (!srml_mul_ok((size_t)rows, (size_t)cols, nx) || !srml_mul_ok((size_t)cols, (size_t)cols, nc)) return SRML_ESIZE;
  if (*nx > SIZE_MAX / sizeof(double)) return SRML_ESIZE;
  return 0;
}

/* m x m symmetric eigendecomposition. */
static inline int srml_check_svd(int m, size_t* nm) {
  if (m < 0) return SRML_EARG;
  if (!srml_mul_ok((size_t)m, (size_t)m, nm) || *nm > SIZE_MAX / sizeof(double)) return SRML_ESIZE;
  return 0;
}

/* X (rows x n) . P (n x k): element counts of X, P and C. */
static inline int srml_check_xp(long rows, int n, int k, size_t* nx, size_t* np, size_t* nc) {
  if (rows < 0 || n < 0 || k < 0) return SRML_EARG;
  if (!srml_mul_ok((size_t)rows, (size_t)n, nx) || !srml_mul_ok((size_t)n, (size_t)k, np) ||
      !srml_mul_ok((size_t)rows, (size_t)k, nc))
    return SRML_ESIZE;
  return 0;
}

#ifdef __cplusplus
}
#endif
#endif /* SRML_CAPI_CHECK_H_ */
