/* Public C ABI of libsrml_ops.so (MI355X / gfx950).
 *
 * Kernel entry points take device pointers and a hipStream_t (passed as void*) and launch
 * asynchronously; the srml_capi_* host-array API mirrors the reference JNI library
 * (jvm/native/src/rapidsml_jni.{cu,cpp,hpp}) and synchronises before returning.
 * All functions return 0 (or a positive count where documented) on success, < 0 on error.
 */
#ifndef SRML_SRML_H_
#define SRML_SRML_H_

#ifdef __cplusplus
extern "C" {
#endif

/* ---- host-array API (reference JNI parity) ---------------------------------------------- */
/* C = alpha op(A) op(B) + beta C, column-major, cuBLAS argument convention (N4 dgemm). */
int srml_capi_dgemm(int transa, int transb, int m, int n, int k, double alpha, const double* A, int lda,
                    const double* B, int ldb, double beta, double* C, int ldc, int device);
/* C (rows x k, row-major, device) = X (rows x n, row-major, device) . P (n x k) (N2 dgemmWithColumnViewPtr). */
int srml_capi_dgemm_device(const double* X, long rows, int n, const double* P, int k, int p_on_host, double* C,
                           void* stream);
/* C (cols x cols) = X^T X for a host rows x cols row-major matrix (N3 dgemmCov). */
int srml_capi_dgemm_cov(const double* X, long rows, int cols, double* C, int device);
/* Symmetric eigendecomposition: U column-major (descending), S = sqrt(eigenvalues), sign-flipped (N5 calSVD). */
int srml_capi_cal_svd(const double* A, int m, double* U, double* S, int device);
/* acc += c (N8 accumulateCov). */
int srml_capi_accumulate_cov(double* acc, const double* c, long len);
const char* srml_capi_version(void);

/* ---- device kernels (selection) ---------------------------------------------------------- */
int srml_dgemm(int ta, int tb, int M, int N, int K, double alpha, const double* A, long lda, const double* B,
               long ldb, double beta, double* C, long ldc, void* stream);
int srml_syevj_f64(const double* A, int n, double* W, double* V, int max_sweeps, double tol, void* stream);
int srml_sign_flip_f64(double* U, int rows, int cols, long ld, void* stream);
int srml_gram_f32(const float* X, long m, int n, long ld, const float* mean, double* G, void* stream);
int srml_col_moments_f32(const float* X, long m, int n, long ld, double* sum, double* sumsq, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SRML_SRML_H_ */
