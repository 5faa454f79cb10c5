// Fixed-point glue of the one-pass second-order statistics and the least-squares solve
// (models/stats.py `scatter_stats`, models/linear.py `lsq_solve`) in three kernels instead of ~60
// torch launches and a dozen n x n temporaries per fit:
//
//   * scatter_shift: the local scatter accumulated about a shift mu0 moved to the GLOBAL mean in
//     one pass: G += m_r (e e^T - d d^T), d = mean_r - mu0, e = mean_r - mean (both rank-one
//     corrections of stats.py's numerics note at once);
//   * sum_sq: fp64 sum and sum of squares of the label vector (fixed-order fold);
//   * lsq_prepare: the standardised normal equations of Spark's objective — per feature the std,
//     its keep flag (constant columns drop out), the scaled right-hand side and the L1 / L2 weights;
//     per (i, j) A = (scatter / m [+ mean_i mean_j without intercept]) / (s_i s_j) keep_i keep_j,
//     plus, for the direct solvers, diag(l2 + 1 - keep) (identity rows for dropped columns);
//   * lsq_finish: w = wt keep ystd / s and the intercept ybar - mean . w (one block, fixed order).
// Reference behaviour: python/src/spark_rapids_ml/regression.py:508-560 (cuML LinearRegression /
// Ridge / CD solvers on standardised data, Spark's regParam / elasticNetParam objective).
#include <hip/hip_runtime.h>

#include "common.h"

namespace {

constexpr int LQ_THREADS = 256;
constexpr int LQ_SUM_BLOCKS = 256;

__global__ __launch_bounds__(LQ_THREADS) void scatter_shift_kernel(double* __restrict__ G, int n,
                                                                   const double* __restrict__ mean_r,
                                                                   const double* __restrict__ mu0,
                                                                   const double* __restrict__ mean, double m_r) {
  const long total = (long)n * n;
  for (long i = (long)blockIdx.x * LQ_THREADS + threadIdx.x; i < total; i += (long)gridDim.x * LQ_THREADS) {
    const int r = (int)(i / n), c = (int)(i - (long)r * n);
    const double dr = mean_r[r] - mu0[r], dc = mean_r[c] - mu0[c];
    const double er = mean_r[r] - mean[r], ec = mean_r[c] - mean[c];
    G[i] += m_r * (er * ec - dr * dc);
  }
}

template <typename T>
__global__ __launch_bounds__(LQ_THREADS) void sum_sq_part_kernel(const T* __restrict__ y, long m,
                                                                 double* __restrict__ part) {
  __shared__ double ws[2][LQ_THREADS / 64];
  double a = 0.0, b = 0.0;
  for (long i = (long)blockIdx.x * LQ_THREADS + threadIdx.x; i < m; i += (long)gridDim.x * LQ_THREADS) {
    const double v = (double)y[i];
    a += v;
    b += v * v;
  }
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    ws[0][wid] = a;
    ws[1][wid] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0, q = 0.0;
    for (int w = 0; w < LQ_THREADS / 64; ++w) {
      s += ws[0][w];
      q += ws[1][w];
    }
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = q;
  }
}

__global__ __launch_bounds__(64) void sum_sq_fold_kernel(const double* __restrict__ part, int np,
                                                         double* __restrict__ out) {
  if (threadIdx.x == 0) {
    double s = 0.0, q = 0.0;
    for (int i = 0; i < np; ++i) {
      s += part[2 * i];
      q += part[2 * i + 1];
    }
    out[0] = s;
    out[1] = q;
  }
}

struct LsqScalars {
  double m, ybar, ystd, reg, l1_ratio;
  int fit_intercept, standardization, add_diag;
};

__device__ __forceinline__ double lsq_std(const double* sumsq, const double* mean, double m, int i) {
  const double v = sumsq[i] / m - mean[i] * mean[i];
  return v > 0.0 ? sqrt(v) : 0.0;
}

// vectors: xstd / safe / keep / b / l1 / l2 (n each), then the matrix
__global__ __launch_bounds__(LQ_THREADS) void lsq_prepare_kernel(const double* __restrict__ S, int n,
                                                                 const double* __restrict__ mean,
                                                                 const double* __restrict__ sumsq,
                                                                 const double* __restrict__ xty, LsqScalars p,
                                                                 double* __restrict__ A, double* __restrict__ vec) {
  const long total = (long)n * n;
  const double lam = p.reg / p.ystd;
  for (long i = (long)blockIdx.x * LQ_THREADS + threadIdx.x; i < total + n; i += (long)gridDim.x * LQ_THREADS) {
    if (i < total) {
      const int r = (int)(i / n), c = (int)(i - (long)r * n);
      const double sr = lsq_std(sumsq, mean, p.m, r), sc = lsq_std(sumsq, mean, p.m, c);
      double a = 0.0;
      if (sr > 0.0 && sc > 0.0) {
        a = S[i] / p.m;
        if (!p.fit_intercept) a += mean[r] * mean[c];
        a /= sr * sc;
      }
      if (p.add_diag && r == c) {
        const double l2 = p.reg * (1.0 - p.l1_ratio) * (p.standardization || sr == 0.0 ? 1.0 : 1.0 / (sr * sr));
        a += sr > 0.0 ? l2 : l2 + 1.0;
      }
      A[i] = a;
    } else {
      const int r = (int)(i - total);
      const double s = lsq_std(sumsq, mean, p.m, r);
      const bool keep = s > 0.0;
      const double safe = keep ? s : 1.0;
      const double xy = xty[r] / p.m;
      const double rhs = p.fit_intercept ? xy - mean[r] * p.ybar : xy;
      vec[r] = safe;                                         // safe std
      vec[n + r] = keep ? 1.0 : 0.0;                         // keep
      vec[2 * n + r] = keep ? rhs / (safe * p.ystd) : 0.0;   // b
      vec[3 * n + r] = lam * p.l1_ratio * (p.standardization ? 1.0 : 1.0 / safe);
      vec[4 * n + r] = p.reg * (1.0 - p.l1_ratio) * (p.standardization ? 1.0 : 1.0 / (safe * safe));
    }
  }
}

// one block: w = wt keep ystd / safe (n), out[n] = intercept (ybar - mean . w, fixed order)
__global__ __launch_bounds__(LQ_THREADS) void lsq_finish_kernel(const double* __restrict__ wt, int n,
                                                                const double* __restrict__ vec,
                                                                const double* __restrict__ mean, double ystd,
                                                                double ybar, int fit_intercept,
                                                                double* __restrict__ out) {
  __shared__ double ws[LQ_THREADS / 64];
  double a = 0.0;
  for (int i = threadIdx.x; i < n; i += LQ_THREADS) {
    const double w = wt[i] * vec[n + i] * ystd / vec[i];
    out[i] = w;
    a += mean[i] * w;
  }
  a = wave_sum(a);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) ws[wid] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < LQ_THREADS / 64; ++w) s += ws[w];
    out[n] = fit_intercept ? ybar - s : 0.0;
  }
}

}  // namespace

// G (n x n fp64, full) += m_r ((mean_r - mean)(mean_r - mean)^T - (mean_r - mu0)(mean_r - mu0)^T)
SRML_API int srml_scatter_shift(double* G, int n, const double* mean_r, const double* mu0, const double* mean,
                                double m_r, hipStream_t stream) {
  if (n <= 0) return 0;
  long blocks = ((long)n * n + LQ_THREADS - 1) / LQ_THREADS;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(scatter_shift_kernel, dim3((unsigned)blocks), dim3(LQ_THREADS), 0, stream, G, n, mean_r, mu0,
                     mean, m_r);
  return srml_status();
}

SRML_API long srml_sum_sq_ws() { return 2 * LQ_SUM_BLOCKS; }

// out[0] = sum y, out[1] = sum y^2 in fp64 (y fp32 or fp64; part: srml_sum_sq_ws() doubles)
SRML_API int srml_sum_sq(const void* y, int is_f64, long m, double* part, double* out, hipStream_t stream) {
  if (m < 0) return -2;
  if (is_f64)
    hipLaunchKernelGGL(sum_sq_part_kernel<double>, dim3(LQ_SUM_BLOCKS), dim3(LQ_THREADS), 0, stream,
                       reinterpret_cast<const double*>(y), m, part);
  else
    hipLaunchKernelGGL(sum_sq_part_kernel<float>, dim3(LQ_SUM_BLOCKS), dim3(LQ_THREADS), 0, stream,
                       reinterpret_cast<const float*>(y), m, part);
  hipLaunchKernelGGL(sum_sq_fold_kernel, dim3(1), dim3(64), 0, stream, part, LQ_SUM_BLOCKS, out);
  return srml_status();
}

// Standardised normal equations (see lsq_prepare_kernel): A (n x n), vec = [safe | keep | b | l1 |
// l2] (5n). S: the global centred scatter; mean / sumsq / xty: global column means, sums of
// squares, raw X^T y; m the global row count.
SRML_API int srml_lsq_prepare(const double* S, int n, const double* mean, const double* sumsq, const double* xty,
                              double m, double ybar, double ystd, double reg, double l1_ratio, int fit_intercept,
                              int standardization, int add_diag, double* A, double* vec, hipStream_t stream) {
  if (n <= 0 || m <= 0.0 || ystd <= 0.0) return -2;
  LsqScalars p{m, ybar, ystd, reg, l1_ratio, fit_intercept, standardization, add_diag};
  long blocks = ((long)n * n + n + LQ_THREADS - 1) / LQ_THREADS;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(lsq_prepare_kernel, dim3((unsigned)blocks), dim3(LQ_THREADS), 0, stream, S, n, mean, sumsq, xty,
                     p, A, vec);
  return srml_status();
}

// out (n + 1): raw-unit coefficients and the intercept from the standardised solution wt
SRML_API int srml_lsq_finish(const double* wt, int n, const double* vec, const double* mean, double ystd,
                             double ybar, int fit_intercept, double* out, hipStream_t stream) {
  if (n <= 0) return -2;
  hipLaunchKernelGGL(lsq_finish_kernel, dim3(1), dim3(LQ_THREADS), 0, stream, wt, n, vec, mean, ystd, ybar,
                     fit_intercept, out);
  return srml_status();
}
