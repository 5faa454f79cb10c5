// Column moments and fused standardisation.
//
// col_moments: one streaming pass over a row-major (m x n) fp32/fp64 block producing per-column
// sum and sum of squares (and optionally sum of |x| and a weighted label cross term) in fp64.
// Work decomposition: blockIdx.x covers 4*256 consecutive columns (each lane owns 4 adjacent
// columns -> 16-byte vector loads, a wave64 instruction moves 1 KiB), blockIdx.y strides over
// row chunks; per-thread partials are accumulated in fp32/fp64 registers over the chunk then
// folded with one fp64 atomic per column per block. Used by PCA/LinReg centering, LogReg
// standardisation (reference classification.py:998-1033 did this with cupy + JSON allGather)
// and the regression metrics pass.
#include "common.h"

template <typename T>
__global__ __launch_bounds__(256) void col_moments_kernel(const T* __restrict__ X, long m, int n, long ld,
                                                          double* __restrict__ sum, double* __restrict__ sumsq,
                                                          long rows_per_block) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  if (c0 >= n) return;
  double s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
  const bool full = (c0 + 3 < n) && ((ld & 3) == 0) && (sizeof(T) == 4);
  if (full) {
    // 4 independent fp32 partial chains per column, folded to fp64 every 256 rows
    float fs[4] = {0, 0, 0, 0}, fq[4] = {0, 0, 0, 0};
    int cnt = 0;
    for (long r = r0; r < r1; ++r) {
      floatx4 v = *reinterpret_cast<const floatx4*>(reinterpret_cast<const float*>(X) + r * ld + c0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fs[j] += v[j];
        fq[j] = fmaf(v[j], v[j], fq[j]);
      }
      if (++cnt == 256) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { s[j] += fs[j]; q[j] += fq[j]; fs[j] = 0.f; fq[j] = 0.f; }
        cnt = 0;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { s[j] += fs[j]; q[j] += fq[j]; }
  } else {
    for (long r = r0; r < r1; ++r) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (c0 + j < n) {
          double v = (double)X[r * ld + c0 + j];
          s[j] += v;
          q[j] += v * v;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c0 + j < n) {
      atomicAdd(&sum[c0 + j], s[j]);
      if (sumsq) atomicAdd(&sumsq[c0 + j], q[j]);
    }
  }
}

static void moments_grid(long m, int n, dim3& grid, long& rpb) {
  unsigned gx = ceil_div(n, 1024);
  // aim for ~2048 blocks total so the 256 CUs stream with enough waves in flight
  long gy = (2048 + gx - 1) / gx;
  rpb = (m + gy - 1) / gy;
  if (rpb < 64) rpb = 64;
  gy = (m + rpb - 1) / rpb;
  if (gy < 1) gy = 1;
  grid = dim3(gx, (unsigned)gy);
}

SRML_API int srml_col_moments_f32(const float* X, long m, int n, long ld, double* sum, double* sumsq,
                                  hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  dim3 grid; long rpb;
  moments_grid(m, n, grid, rpb);
  hipLaunchKernelGGL(col_moments_kernel<float>, grid, dim3(256), 0, stream, X, m, n, ld, sum, sumsq, rpb);
  return srml_status();
}

SRML_API int srml_col_moments_f64(const double* X, long m, int n, long ld, double* sum, double* sumsq,
                                  hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  dim3 grid; long rpb;
  moments_grid(m, n, grid, rpb);
  hipLaunchKernelGGL(col_moments_kernel<double>, grid, dim3(256), 0, stream, X, m, n, ld, sum, sumsq, rpb);
  return srml_status();
}

// X[r, c] = (X[r, c] - mean[c]) * scale[c]   (in place; mean or scale may be null)
template <typename T>
__global__ __launch_bounds__(256) void standardize_kernel(T* __restrict__ X, long m, int n, long ld,
                                                          const T* __restrict__ mean, const T* __restrict__ scale) {
  long total = m * (long)n;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long r = i / n;
    int c = (int)(i - r * n);
    T v = X[r * ld + c];
    if (mean) v -= mean[c];
    if (scale) v *= scale[c];
    X[r * ld + c] = v;
  }
}

SRML_API int srml_standardize_f32(float* X, long m, int n, long ld, const float* mean, const float* scale,
                                  hipStream_t stream) {
  long total = m * (long)n;
  if (total <= 0) return 0;
  long g = (total + 255) / 256; if (g > 4096) g = 4096; unsigned grid = (unsigned)g;
  hipLaunchKernelGGL(standardize_kernel<float>, dim3(grid), dim3(256), 0, stream, X, m, n, ld, mean, scale);
  return srml_status();
}
