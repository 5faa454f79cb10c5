// Evaluation partials computed where the predictions are (CrossValidator transform-evaluate pass).
//
// Reference: the per-batch evaluate functions of the classification / regression models run cudf
// group-bys and cuML log_loss on the worker GPU (classification.py:113-155, regression.py:144-173)
// and ship only the small partial results. Here:
//  * srml_confusion_counts — C x C (label, prediction) counts, LDS-privatised per block (C <= 64),
//    global atomics beyond; labels / predictions that are not integers in [0, C) land in one
//    "invalid" counter (the caller then falls back to the host path);
//  * srml_logloss_sum     — sum_r -log(max(prob[r, y_r], eps)), fp64 block reduction + one atomic;
//  * srml_reg_moments      — moments of [label, label - prediction, prediction]: sums, sums of
//    squares and |x| in one pass, then the squared deviations about the exact means in a second
//    pass (the means are read on the device: no host round trip).
// Predictions / probabilities may be fp64, fp32, int64 or int32 (kind 0 / 1 / 2 / 3).
#include "common.h"

namespace {

__device__ __forceinline__ double load_kind(const void* p, int kind, long i) {
  switch (kind) {
    case 1: return (double)reinterpret_cast<const float*>(p)[i];
    case 2: return (double)reinterpret_cast<const long long*>(p)[i];
    case 3: return (double)reinterpret_cast<const int*>(p)[i];
    default: return reinterpret_cast<const double*>(p)[i];
  }
}

__device__ __forceinline__ int class_of(double v, int C) {
  if (!(v >= 0.0) || v >= (double)C) return -1;
  const int c = (int)v;
  return (double)c == v ? c : -1;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;  // valid in thread 0
}

template <bool LDS>
__global__ __launch_bounds__(256) void confusion_kernel(const void* __restrict__ y, int ykind,
                                                        const void* __restrict__ p, int pkind, long m, int C,
                                                        unsigned long long* __restrict__ counts) {
  __shared__ unsigned int h[LDS ? 64 * 64 : 1];
  __shared__ unsigned int bad;
  if (LDS) {
    for (int i = threadIdx.x; i < C * C; i += 256) h[i] = 0u;
  }
  if (threadIdx.x == 0) bad = 0u;
  __syncthreads();
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < m; r += (long)gridDim.x * 256) {
    const int a = class_of(load_kind(y, ykind, r), C), b = class_of(load_kind(p, pkind, r), C);
    if (a < 0 || b < 0) {
      atomicAdd(&bad, 1u);
    } else if (LDS) {
      atomicAdd(&h[a * C + b], 1u);
    } else {
      atomicAdd(&counts[(long)a * C + b], 1ull);
    }
  }
  __syncthreads();
  if (LDS) {
    for (int i = threadIdx.x; i < C * C; i += 256)
      if (h[i]) atomicAdd(&counts[i], (unsigned long long)h[i]);
  }
  if (threadIdx.x == 0 && bad) atomicAdd(&counts[(long)C * C], (unsigned long long)bad);
}

__global__ __launch_bounds__(256) void logloss_kernel(const void* __restrict__ prob, int kind, long m, int C, long ld,
                                                      const void* __restrict__ y, int ykind, double eps,
                                                      double* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < m; r += (long)gridDim.x * 256) {
    int c = (int)load_kind(y, ykind, r);
    c = c < 0 ? 0 : (c >= C ? C - 1 : c);  // host path: clip(label, 0, C - 1)
    const double pl = load_kind(prob, kind, r * ld + c);
    s += -log(pl > eps ? pl : eps);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

// out[0..2] sums, [3..5] sums of squares, [6..8] sums of |x| of (y, y - p, p)
__global__ __launch_bounds__(256) void reg_sums_kernel(const void* __restrict__ y, int ykind,
                                                       const void* __restrict__ p, int pkind, long m,
                                                       double* __restrict__ out) {
  __shared__ double red[4];
  double v[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) v[i] = 0.0;
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < m; r += (long)gridDim.x * 256) {
    const double a = load_kind(y, ykind, r), c = load_kind(p, pkind, r);
    const double x[3] = {a, a - c, c};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      v[j] += x[j];
      v[3 + j] += x[j] * x[j];
      v[6 + j] += fabs(x[j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const double t = block_sum(v[i], red);
    if (threadIdx.x == 0) atomicAdd(&out[i], t);
  }
}

// out[9..11] += sum (x - mean)^2, mean = out[0..2] / m (written by reg_sums_kernel before)
__global__ __launch_bounds__(256) void reg_dev_kernel(const void* __restrict__ y, int ykind,
                                                      const void* __restrict__ p, int pkind, long m,
                                                      double* __restrict__ out) {
  __shared__ double red[4];
  const double mu[3] = {out[0] / (double)m, out[1] / (double)m, out[2] / (double)m};
  double v[3] = {0.0, 0.0, 0.0};
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < m; r += (long)gridDim.x * 256) {
    const double a = load_kind(y, ykind, r), c = load_kind(p, pkind, r);
    const double x[3] = {a - mu[0], (a - c) - mu[1], c - mu[2]};
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] += x[j] * x[j];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double t = block_sum(v[j], red);
    if (threadIdx.x == 0) atomicAdd(&out[9 + j], t);
  }
}

unsigned grid_rows(long m) {
  long b = (m + 255) / 256;
  if (b > 2048) b = 2048;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace

// counts: C * C + 1 zeroed uint64 (row = label, column = prediction; the last one counts rows whose
// label or prediction is not an integer in [0, C))
SRML_API int srml_confusion_counts(const void* y, int ykind, const void* p, int pkind, long m, int C,
                                   unsigned long long* counts, hipStream_t stream) {
  if (m <= 0) return 0;
  if (C < 1 || C > 4096) return -2;
  if (C <= 64)
    hipLaunchKernelGGL(confusion_kernel<true>, dim3(grid_rows(m)), dim3(256), 0, stream, y, ykind, p, pkind, m, C,
                       counts);
  else
    hipLaunchKernelGGL(confusion_kernel<false>, dim3(grid_rows(m)), dim3(256), 0, stream, y, ykind, p, pkind, m, C,
                       counts);
  return srml_status();
}

// out: one zeroed double
SRML_API int srml_logloss_sum(const void* prob, int kind, long m, int C, long ld, const void* y, int ykind,
                              double eps, double* out, hipStream_t stream) {
  if (m <= 0) return 0;
  if (C < 1 || ld < C) return -2;
  hipLaunchKernelGGL(logloss_kernel, dim3(grid_rows(m)), dim3(256), 0, stream, prob, kind, m, C, ld, y, ykind, eps,
                     out);
  return srml_status();
}

// out: 12 zeroed doubles [sum(3) | sum sq(3) | sum abs(3) | sum sq dev(3)] of (y, y - p, p)
SRML_API int srml_reg_moments(const void* y, int ykind, const void* p, int pkind, long m, double* out,
                              hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(reg_sums_kernel, dim3(grid_rows(m)), dim3(256), 0, stream, y, ykind, p, pkind, m, out);
  hipLaunchKernelGGL(reg_dev_kernel, dim3(grid_rows(m)), dim3(256), 0, stream, y, ykind, p, pkind, m, out);
  return srml_status();
}
