// Symmetric eigensolver: parallel two-sided (cyclic round-robin) Jacobi in fp64, fully on device.
//
// Reference N5 (`calSVD`, rapidsml_jni.cu:215-269) calls cuSOLVER syevd through RAFT eigDC and then
// reverses, square-roots and sign-flips. Here: each sweep is n-1 rounds of n/2 disjoint (p, q)
// rotations (circle-method tournament, so every pair meets once per sweep). A round is two
// kernels over ping-pong buffers, which keeps every read race-free:
//   rows:    A2[p,:], A2[q,:] = rotate(A[p,:], A[q,:])  (+ the pair's (c, s) from A's 2x2 block)
//   columns: A[:,p],  A[:,q]  = rotate(A2[:,p], A2[:,q]);  V[:,p], V[:,q] likewise
// One sweep (2(n-1) launches) is captured once into a hipGraph and replayed; the off-diagonal
// Frobenius norm is checked after every sweep (one 8-byte D2H). Convergence is quadratic, so
// ~6-10 sweeps reach fp64 round-off. Output: eigenvalues descending + eigenvectors as columns
// (row-major V[i * n + k] = k-th eigenvector's i-th entry).
#include <algorithm>

#include "common.h"

namespace {

__device__ __forceinline__ int rr_index(int k, int r, int N) {
  // circle method: position 0 fixed, the others rotate by r
  return k == 0 ? 0 : 1 + (k - 1 + r) % (N - 1);
}

__global__ __launch_bounds__(256) void jacobi_rows_kernel(const double* __restrict__ A, double* __restrict__ A2,
                                                          double* __restrict__ cs, int n, int N, int r) {
  const int k = blockIdx.y;  // pair
  int p = rr_index(k, r, N), q = rr_index(N - 1 - k, r, N);
  if (p > q) {
    const int t = p;
    p = q;
    q = t;
  }
  const bool pad = q >= n;  // odd n: the padding index pairs with someone each round
  double c = 1.0, s = 0.0;
  if (!pad) {
    const double apq = A[(long)p * n + q];
    if (fabs(apq) > 1e-300) {
      const double app = A[(long)p * n + p], aqq = A[(long)q * n + q];
      const double theta = (aqq - app) / (2.0 * apq);
      const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      c = 1.0 / sqrt(t * t + 1.0);
      s = t * c;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    cs[2 * k] = c;
    cs[2 * k + 1] = s;
  }
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    if (pad) {
      if (p < n) A2[(long)p * n + j] = A[(long)p * n + j];
      continue;
    }
    const double ap = A[(long)p * n + j], aq = A[(long)q * n + j];
    A2[(long)p * n + j] = c * ap - s * aq;
    A2[(long)q * n + j] = s * ap + c * aq;
  }
}

__global__ __launch_bounds__(256) void jacobi_cols_kernel(const double* __restrict__ A2, double* __restrict__ A,
                                                          double* __restrict__ V, const double* __restrict__ cs,
                                                          int n, int N, int r) {
  const int half = N / 2;
  const long total = (long)n * half;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int k = (int)(t % half);
    const long i = t / half;
    int p = rr_index(k, r, N), q = rr_index(N - 1 - k, r, N);
    if (p > q) {
      const int tt = p;
      p = q;
      q = tt;
    }
    if (q >= n) {
      if (p < n) A[i * n + p] = A2[i * n + p];
      continue;
    }
    const double c = cs[2 * k], s = cs[2 * k + 1];
    const double ap = A2[i * n + p], aq = A2[i * n + q];
    A[i * n + p] = c * ap - s * aq;
    A[i * n + q] = s * ap + c * aq;
    const double vp = V[i * n + p], vq = V[i * n + q];
    V[i * n + p] = c * vp - s * vq;
    V[i * n + q] = s * vp + c * vq;
  }
}

__global__ __launch_bounds__(256) void offdiag_kernel(const double* __restrict__ A, int n, double* __restrict__ out) {
  double acc = 0.0, dg = 0.0;
  const long nn = (long)n * n;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < nn; t += (long)gridDim.x * blockDim.x) {
    const long i = t / n, j = t % n;
    const double v = A[t];
    if (i != j) acc += v * v; else dg += v * v;
  }
  acc = wave_sum(acc);
  dg = wave_sum(dg);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&out[0], acc);
    atomicAdd(&out[1], dg);
  }
}

__global__ void eye_kernel(double* __restrict__ V, int n) {
  const long nn = (long)n * n;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < nn; t += (long)gridDim.x * blockDim.x)
    V[t] = (t / n == t % n) ? 1.0 : 0.0;
}

__global__ void diag_kernel(const double* __restrict__ A, int n, double* __restrict__ w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w[i] = A[(long)i * n + i];
}

// out[i, k] = V[i, order[k]]
__global__ void gather_cols_kernel(const double* __restrict__ V, const int* __restrict__ order, int n,
                                   double* __restrict__ out) {
  const long nn = (long)n * n;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < nn; t += (long)gridDim.x * blockDim.x) {
    const long i = t / n;
    const int k = (int)(t % n);
    out[t] = V[i * n + order[k]];
  }
}

inline unsigned blocks_for(long work) {
  long b = (work + 255) / 256;
  if (b > 4096) b = 4096;
  return (unsigned)(b < 1 ? 1 : b);
}
}  // namespace

// Jacobi eigendecomposition of the symmetric n x n matrix A (device, row-major; not modified).
// W: n eigenvalues, descending. V: n x n row-major, column k = eigenvector of W[k] (unnormalised
// sign). Returns the number of sweeps (> 0) or a negative error.
SRML_API int srml_syevj_f64(const double* A, int n, double* W, double* V, int max_sweeps, double tol,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  if (n == 1) {
    hipError_t err = hipSuccess;
    SRML_TRY(err, hipMemcpyAsync(W, A, sizeof(double), hipMemcpyDeviceToDevice, stream));
    const double one = 1.0;
    SRML_TRY(err, hipMemcpyAsync(V, &one, sizeof(double), hipMemcpyHostToDevice, stream));
    SRML_TRY(err, hipStreamSynchronize(stream));
    return err == hipSuccess ? 1 : -(int)err;
  }
  hipError_t err = hipSuccess;
  const int N = n + (n & 1);
  const size_t mat = (size_t)n * n * sizeof(double);
  double *a = nullptr, *a2 = nullptr, *vv = nullptr, *cs = nullptr, *red = nullptr;
  int* ord = nullptr;
  if (hipMallocAsync((void**)&a, mat, stream) != hipSuccess) return -2;
  SRML_TRY(err, hipMallocAsync((void**)&a2, mat, stream));
  SRML_TRY(err, hipMallocAsync((void**)&vv, mat, stream));
  SRML_TRY(err, hipMallocAsync((void**)&cs, sizeof(double) * N, stream));
  SRML_TRY(err, hipMallocAsync((void**)&red, sizeof(double) * 2, stream));
  SRML_TRY(err, hipMallocAsync((void**)&ord, sizeof(int) * n, stream));
  SRML_TRY(err, hipMemcpyAsync(a, A, mat, hipMemcpyDeviceToDevice, stream));
  hipLaunchKernelGGL(eye_kernel, dim3(blocks_for((long)n * n)), dim3(256), 0, stream, vv, n);

  // capture one sweep
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipStream_t cap = nullptr;
  SRML_TRY(err, hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  SRML_TRY(err, hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
  const dim3 rgrid((unsigned)((n + 255) / 256 < 64 ? (n + 255) / 256 : 64), (unsigned)(N / 2));
  const unsigned cgrid = blocks_for((long)n * (N / 2));
  for (int r = 0; r < N - 1; ++r) {
    hipLaunchKernelGGL(jacobi_rows_kernel, rgrid, dim3(256), 0, cap, a, a2, cs, n, N, r);
    hipLaunchKernelGGL(jacobi_cols_kernel, dim3(cgrid), dim3(256), 0, cap, a2, a, vv, cs, n, N, r);
  }
  SRML_TRY(err, hipStreamEndCapture(cap, &graph));
  int rc = 0;
  if (!graph || hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) rc = -3;
  int sweeps = 0;
  double host[2] = {0.0, 0.0};
  if (rc == 0) {
    hipEvent_t ev;
    SRML_TRY(err, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    SRML_TRY(err, hipEventRecord(ev, stream));
    SRML_TRY(err, hipStreamWaitEvent(cap, ev, 0));  // workspace init on `stream` precedes the first sweep
    for (sweeps = 1; sweeps <= max_sweeps; ++sweeps) {
      SRML_TRY(err, hipGraphLaunch(exec, cap));
      SRML_TRY(err, hipMemsetAsync(red, 0, sizeof(double) * 2, cap));
      hipLaunchKernelGGL(offdiag_kernel, dim3(blocks_for((long)n * n)), dim3(256), 0, cap, a, n, red);
      SRML_TRY(err, hipMemcpyAsync(host, red, sizeof(host), hipMemcpyDeviceToHost, cap));
      SRML_TRY(err, hipStreamSynchronize(cap));
      if (host[0] <= tol * tol * (host[0] + host[1])) break;
    }
    if (sweeps > max_sweeps) sweeps = max_sweeps;
    SRML_TRY(err, hipEventRecord(ev, cap));
    SRML_TRY(err, hipStreamWaitEvent(stream, ev, 0));
    SRML_TRY(err, hipEventDestroy(ev));
  }
  if (exec) SRML_TRY(err, hipGraphExecDestroy(exec));
  if (graph) SRML_TRY(err, hipGraphDestroy(graph));
  SRML_TRY(err, hipStreamDestroy(cap));
  if (rc == 0) {
    // eigenvalues -> host, sort descending, reorder columns
    double* wd = a2;  // reuse workspace
    hipLaunchKernelGGL(diag_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, a, n, wd);
    double* wh = (double*)malloc(sizeof(double) * n);
    int* oh = (int*)malloc(sizeof(int) * n);
    SRML_TRY(err, hipMemcpyAsync(wh, wd, sizeof(double) * n, hipMemcpyDeviceToHost, stream));
    SRML_TRY(err, hipStreamSynchronize(stream));
    for (int i = 0; i < n; ++i) oh[i] = i;
    std::stable_sort(oh, oh + n, [wh](int x, int y) { return wh[x] > wh[y]; });
    double* ws = (double*)malloc(sizeof(double) * n);
    for (int i = 0; i < n; ++i) ws[i] = wh[oh[i]];
    SRML_TRY(err, hipMemcpyAsync(W, ws, sizeof(double) * n, hipMemcpyHostToDevice, stream));
    SRML_TRY(err, hipMemcpyAsync(ord, oh, sizeof(int) * n, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(gather_cols_kernel, dim3(blocks_for((long)n * n)), dim3(256), 0, stream, vv, ord, n, V);
    SRML_TRY(err, hipStreamSynchronize(stream));
    free(wh);
    free(oh);
    free(ws);
  }
  SRML_TRY(err, hipFreeAsync(a, stream));
  SRML_TRY(err, hipFreeAsync(a2, stream));
  SRML_TRY(err, hipFreeAsync(vv, stream));
  SRML_TRY(err, hipFreeAsync(cs, stream));
  SRML_TRY(err, hipFreeAsync(red, stream));
  SRML_TRY(err, hipFreeAsync(ord, stream));
  const int st = srml_status();
  if (rc != 0) return rc;
  if (err != hipSuccess) return -(int)err;
  return st != 0 ? -st : sweeps;
}
