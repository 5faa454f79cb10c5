// Host-array C ABI with the reference JNI library's capabilities (jvm/native/src/rapidsml_jni.cu,
// SURVEY N2-N9), built on this library's kernels:
//   srml_capi_dgemm           N4  full host GEMM (column-major, cuBLAS argument convention)
//   srml_capi_dgemm_device    N2/N6  device GEMM on a row-major rows x n list-column child buffer
//   srml_capi_dgemm_cov       N3/N7  C = X^T X of a rows x cols row-major fp64 matrix (returns status)
//   srml_capi_cal_svd         N5  eigendecomposition of a symmetric matrix -> U (column-major,
//                                 descending), S = sqrt(eigenvalues), deterministic column signs
//   srml_capi_accumulate_cov  N8  acc += c (declared but never implemented in the reference)
// Every entry point returns 0 on success or a negative status; it synchronises its own stream,
// so callers (JNI shim, Python, C++) never see partially written outputs.
#include <cstring>

#include "capi_check.h"
#include "common.h"

extern "C" int srml_dgemm(int ta, int tb, int M, int N, int K, double alpha, const double* A, long lda,
                          const double* B, long ldb, double beta, double* C, long ldc, hipStream_t stream);
extern "C" int srml_syevj_f64(const double* A, int n, double* W, double* V, int max_sweeps, double tol,
                              hipStream_t stream);
extern "C" int srml_sign_flip_f64(double* U, int rows, int cols, long ld, hipStream_t stream);

namespace {

struct DeviceGuard {
  int prev = 0;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = 0;
    if (dev >= 0) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

template <typename T>
struct DevBuf {
  T* p = nullptr;
  explicit DevBuf(size_t n) {
    if (n && hipMalloc((void**)&p, n * sizeof(T)) != hipSuccess) p = nullptr;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

__global__ void seq_root_kernel(double* __restrict__ s, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s[i] = sqrt(fmax(s[i], 0.0));
}

__global__ void transpose_kernel(const double* __restrict__ in, double* __restrict__ out, int n) {
  __shared__ double tile[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  for (int j = threadIdx.y; j < 32; j += 8) {
    const int r = by + j, c = bx + threadIdx.x;
    if (r < n && c < n) tile[j][threadIdx.x] = in[(long)r * n + c];
  }
  __syncthreads();
  for (int j = threadIdx.y; j < 32; j += 8) {
    const int r = bx + j, c = by + threadIdx.x;
    if (r < n && c < n) out[(long)r * n + c] = tile[threadIdx.x][j];
  }
}
}  // namespace

SRML_API int srml_capi_dgemm(int transa, int transb, int m, int n, int k, double alpha, const double* A, int lda,
                             const double* B, int ldb, double beta, double* C, int ldc, int device) {
  // column-major r x c with leading dimension ld == row-major (c x ld) buffer
  size_t na = 0, nb = 0, nc = 0;
  const int chk = srml_check_gemm(transa, transb, m, n, k, lda, ldb, ldc, &na, &nb, &nc);
  if (chk) return chk;
  if (m == 0 || n == 0) return 0;
  if ((na && !A) || (nb && !B) || !C) return SRML_EARG;
  DeviceGuard g(device);
  if (!g.ok) return -1;
  DevBuf<double> a(na), b(nb), c(nc);
  if ((na && !a.p) || (nb && !b.p) || !c.p) return -2;
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return -1;
  hipError_t err = hipSuccess;
  if (na) SRML_TRY(err, hipMemcpyAsync(a.p, A, na * sizeof(double), hipMemcpyHostToDevice, s));
  if (nb) SRML_TRY(err, hipMemcpyAsync(b.p, B, nb * sizeof(double), hipMemcpyHostToDevice, s));
  if (beta != 0.0) SRML_TRY(err, hipMemcpyAsync(c.p, C, nc * sizeof(double), hipMemcpyHostToDevice, s));
  // C_colmajor = op(A) op(B)  <=>  row-major C^T (n x m) = op(B)^T op(A)^T with the same flags
  int rc = srml_dgemm(transb, transa, n, m, k, alpha, b.p, ldb, a.p, lda, beta, c.p, ldc, s);
  SRML_TRY(err, hipMemcpyAsync(C, c.p, nc * sizeof(double), hipMemcpyDeviceToHost, s));
  SRML_TRY(err, hipStreamSynchronize(s));
  SRML_TRY(err, hipStreamDestroy(s));
  if (rc) return rc < 0 ? rc : -rc;
  return err == hipSuccess ? 0 : -(int)err;
}

// C (rows x k, row-major, device) = X (rows x n, row-major, device) . P (n x k row-major, host or device)
SRML_API int srml_capi_dgemm_device(const double* X, long rows, int n, const double* P, int k, int p_on_host,
                                    double* C, hipStream_t stream) {
  size_t nx = 0, np = 0, nc = 0;
  const int chk = srml_check_xp(rows, n, k, &nx, &np, &nc);
  if (chk) return chk;
  if (rows == 0 || k == 0) return 0;
  if ((nx && !X) || (np && !P) || !C) return SRML_EARG;
  const double* pd = P;
  DevBuf<double> tmp(p_on_host ? (size_t)n * k : 0);
  hipError_t err = hipSuccess;
  if (p_on_host) {
    if (!tmp.p) return -2;
    SRML_TRY(err, hipMemcpyAsync(tmp.p, P, (size_t)n * k * sizeof(double), hipMemcpyHostToDevice, stream));
    pd = tmp.p;
  }
  const int rc = srml_dgemm(0, 0, (int)rows, k, n, 1.0, X, n, pd, k, 0.0, C, k, stream);
  SRML_TRY(err, hipStreamSynchronize(stream));
  if (rc) return rc < 0 ? rc : -rc;
  return err == hipSuccess ? 0 : -(int)err;
}

SRML_API int srml_capi_dgemm_cov(const double* X, long rows, int cols, double* C, int device) {
  size_t nx = 0, ncov = 0;
  const int chk = srml_check_cov(rows, cols, &nx, &ncov);
  if (chk) return chk;
  if (cols == 0) return 0;
  if ((nx && !X) || !C) return SRML_EARG;
  DeviceGuard g(device);
  if (!g.ok) return -1;
  DevBuf<double> x((size_t)rows * cols), c((size_t)cols * cols);
  if ((rows && !x.p) || !c.p) return -2;
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return -1;
  hipError_t err = hipSuccess;
  if (rows) SRML_TRY(err, hipMemcpyAsync(x.p, X, (size_t)rows * cols * sizeof(double), hipMemcpyHostToDevice, s));
  int rc = 0;
  if (rows)
    rc = srml_dgemm(1, 0, cols, cols, (int)rows, 1.0, x.p, cols, x.p, cols, 0.0, c.p, cols, s);
  else
    SRML_TRY(err, hipMemsetAsync(c.p, 0, (size_t)cols * cols * sizeof(double), s));
  SRML_TRY(err, hipMemcpyAsync(C, c.p, (size_t)cols * cols * sizeof(double), hipMemcpyDeviceToHost, s));
  SRML_TRY(err, hipStreamSynchronize(s));
  SRML_TRY(err, hipStreamDestroy(s));
  if (rc) return rc < 0 ? rc : -rc;
  return err == hipSuccess ? 0 : -(int)err;
}

SRML_API int srml_capi_cal_svd(const double* A, int m, double* U, double* S, int device) {
  size_t nm = 0;
  const int chk = srml_check_svd(m, &nm);
  if (chk) return chk;
  if (m == 0) return 0;
  if (!A || !U || !S) return SRML_EARG;
  DeviceGuard g(device);
  if (!g.ok) return -1;
  DevBuf<double> a((size_t)m * m), v((size_t)m * m), w(m), ut((size_t)m * m);
  if (!a.p || !v.p || !w.p || !ut.p) return -2;
  hipStream_t s;
  if (hipStreamCreate(&s) != hipSuccess) return -1;
  hipError_t err = hipSuccess;
  SRML_TRY(err, hipMemcpyAsync(a.p, A, (size_t)m * m * sizeof(double), hipMemcpyHostToDevice, s));
  const int sweeps = srml_syevj_f64(a.p, m, w.p, v.p, 30, 1e-15, s);
  int rc = sweeps < 0 ? sweeps : 0;
  if (rc == 0) {
    rc = srml_sign_flip_f64(v.p, m, m, m, s);  // columns are eigenvectors (row-major)
    hipLaunchKernelGGL(seq_root_kernel, dim3((m + 255) / 256), dim3(256), 0, s, w.p, m);
    // U column-major == row-major transpose of V
    hipLaunchKernelGGL(transpose_kernel, dim3((m + 31) / 32, (m + 31) / 32), dim3(32, 8), 0, s, v.p, ut.p, m);
    SRML_TRY(err, hipMemcpyAsync(U, ut.p, (size_t)m * m * sizeof(double), hipMemcpyDeviceToHost, s));
    SRML_TRY(err, hipMemcpyAsync(S, w.p, (size_t)m * sizeof(double), hipMemcpyDeviceToHost, s));
  }
  SRML_TRY(err, hipStreamSynchronize(s));
  SRML_TRY(err, hipStreamDestroy(s));
  if (rc) return rc < 0 ? rc : -rc;
  return err == hipSuccess ? 0 : -(int)err;
}

SRML_API int srml_capi_accumulate_cov(double* acc, const double* c, long len) {
  if (len < 0 || (len && (!acc || !c))) return SRML_EARG;
  for (long i = 0; i < len; ++i) acc[i] += c[i];
  return 0;
}

SRML_API const char* srml_capi_version() { return "spark-rapids-ml-nai-amd 24.06.0 (gfx950)"; }
