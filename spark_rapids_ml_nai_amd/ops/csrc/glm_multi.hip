// GLM loss/gradient passes beyond the fp32 binary fast path (glm.hip):
//
//  * srml_mlogit_f32 — multinomial (softmax) logistic loss + gradient for K <= 16 classes in ONE
//    pass over X (the reference's cuML QN reads X twice per evaluation: a GEMM for the margins, a
//    transposed GEMM for the gradient; the previous path here ran xw + torch softmax + xtv, i.e.
//    four passes for K = 10). Column-split rows: each of the 4 waves of a block owns a 256*V-column
//    slice of every row; a lane keeps its 4*V columns of all K class-weight rows (fp32) and of the
//    K gradient rows in registers, the row slice streams through a register prefetch ring. Per row:
//    K partial margins per lane -> wave64 DPP reductions -> LDS exchange between the 4 waves ->
//    every lane evaluates the (max-shifted) softmax, the residuals p_k - [y == k] and the loss,
//    then updates its K gradient slices from the row still in registers.
//    out layout (fp64): [grad W (K x n, class-major) | grad b (K) | loss sum].
//  * srml_logreg_binary_lds_{f32,f64} — binary loss + gradient for fp64 inputs and for fp32 rows
//    wider than the register-resident fast path (n <= 16384): one wave per row, the gradient of
//    the block accumulates in LDS (fp64 ds_add), one fp64 atomic per column per block.
// Both take the intercept(s) and an optional `done` flag from device memory so they chain with the
// on-device quasi-Newton step (qn.hip) without host round trips.
#include "common.h"

template <int KB, int V, int D>
__global__ __launch_bounds__(256, 1) void mlogit_pf_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                           const float* __restrict__ y,
                                                           const double* __restrict__ W,
                                                           const double* __restrict__ bvec,
                                                           const int* __restrict__ flag, int K,
                                                           double* __restrict__ out, long rows_per_block,
                                                           int vec) {
  if (flag && *flag) return;
  __shared__ float part[2][KB][4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int cbase = wid * 256 * V;
  float wreg[KB][V][4];
  float g[KB][V][4];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int c = cbase + (v * 64 + lane) * 4;
#pragma unroll
    for (int k = 0; k < KB; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        wreg[k][v][q] = (k < K && c + q < n) ? (float)W[(long)k * n + c + q] : 0.f;
        g[k][v][q] = 0.f;
      }
  }
  double bb[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) bb[k] = (k < K && bvec) ? bvec[k] : 0.0;
  double gb[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) gb[k] = 0.0;
  double loss = 0.0;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  if (r0 >= r1) return;

  auto load = [&](long r, floatx4 (&x)[V]) {
    const float* row = X + r * ld;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = cbase + (v * 64 + lane) * 4;
      if (vec && c + 3 < n) {
        x[v] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(row + c));
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[v][q] = (c + q < n) ? row[c + q] : 0.f;
      }
    }
  };
  int buf = 0;
  auto process = [&](long r, const floatx4 (&x)[V]) {
    float pk[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      float a = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int q = 0; q < 4; ++q) a = fmaf(x[v][q], wreg[k][v][q], a);
      pk[k] = wave_sum(a);
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < KB; ++k) part[buf][k][wid] = pk[k];
    }
    __syncthreads();
    double z[KB];
    double zmax = -1e300;
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      z[k] = (double)part[buf][k][0] + (double)part[buf][k][1] + (double)part[buf][k][2] + (double)part[buf][k][3] + bb[k];
      if (k < K) zmax = fmax(zmax, z[k]);
    }
    float e[KB];
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      e[k] = k < K ? __expf((float)(z[k] - zmax)) : 0.f;
      se += e[k];
    }
    const int yi = (int)y[r];
    const float inv = 1.f / se;
    double zy = 0.0;
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const float res = e[k] * inv - (k == yi ? 1.f : 0.f);
      if (k == yi) zy = z[k];
      if (wid == 0 && lane == 0) gb[k] += (double)res;
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int q = 0; q < 4; ++q) g[k][v][q] = fmaf(res, x[v][q], g[k][v][q]);
    }
    if (wid == 0 && lane == 0) loss += zmax + (double)__logf(se) - zy;
    buf ^= 1;
  };
  floatx4 x[D + 1][V];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (r0 + d < r1) load(r0 + d, x[d]);
  for (long rb = r0; rb < r1; rb += D + 1) {
#pragma unroll
    for (int ph = 0; ph <= D; ++ph) {
      const long cur = rb + ph;
      if (cur < r1) {
        const long nxt = cur + D;
        if (nxt < r1) load(nxt, x[(ph + D) % (D + 1)]);
        process(cur, x[ph]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    if (k >= K) break;
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = cbase + (v * 64 + lane) * 4 + q;
        if (c < n) atomicAdd(&out[(long)k * n + c], (double)g[k][v][q]);
      }
  }
  if (wid == 0 && lane == 0) {
    const long base = (long)K * n;
    for (int k = 0; k < K; ++k) atomicAdd(&out[base + k], gb[k]);
    atomicAdd(&out[base + K], loss);
  }
}

SRML_API int srml_mlogit_supported(int n, int K) {
  if (K < 2 || K > 16 || n <= 0 || n > 4096) return 0;
  const int V = (n + 1023) / 1024;
  const int KB = K <= 4 ? 4 : K <= 8 ? 8 : K <= 12 ? 12 : 16;
  return KB * V <= 36 ? 1 : 0;
}

SRML_API int srml_mlogit_f32(const float* X, long m, int n, long ld, const float* y, const double* W, const double* b,
                             const int* flag, int K, double* out, hipStream_t stream) {
  if (m <= 0) return 0;
  if (!srml_mlogit_supported(n, K)) return -2;
  const int V = (n + 1023) / 1024;
  const int KB = K <= 4 ? 4 : K <= 8 ? 8 : K <= 12 ? 12 : 16;
  // one 4-wave block per CU is resident (register-heavy); a few blocks per CU amortise the
  // per-block K*n-wide atomic flush against tail imbalance
  long blocks = m / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  long rpb = (m + blocks - 1) / blocks;
  blocks = (m + rpb - 1) / rpb;
  const int vec = ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  dim3 grid((unsigned)blocks), blk(256);
#define SRML_ML(KK, VV) \
  hipLaunchKernelGGL((mlogit_pf_kernel<KK, VV, 2>), grid, blk, 0, stream, X, m, n, ld, y, W, b, flag, K, out, rpb, vec)
  if (KB == 4) {
    if (V == 1) SRML_ML(4, 1); else if (V == 2) SRML_ML(4, 2); else if (V == 3) SRML_ML(4, 3); else SRML_ML(4, 4);
  } else if (KB == 8) {
    if (V == 1) SRML_ML(8, 1); else if (V == 2) SRML_ML(8, 2); else if (V == 3) SRML_ML(8, 3); else SRML_ML(8, 4);
  } else if (KB == 12) {
    if (V == 1) SRML_ML(12, 1); else if (V == 2) SRML_ML(12, 2); else SRML_ML(12, 3);
  } else {
    if (V == 1) SRML_ML(16, 1); else SRML_ML(16, 2);
  }
#undef SRML_ML
  return srml_status();
}

// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void logreg_binary_lds_kernel(const T* __restrict__ X, long m, int n, long ld,
                                                                const float* __restrict__ y,
                                                                const double* __restrict__ w, double b_in,
                                                                const double* __restrict__ bptr,
                                                                const int* __restrict__ flag,
                                                                double* __restrict__ out, long rows_per_block) {
  if (flag && *flag) return;
  extern __shared__ double gl[];  // [n]
  const double b = bptr ? *bptr : b_in;
  for (int i = threadIdx.x; i < n; i += 256) gl[i] = 0.0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  double gb = 0.0, loss = 0.0;
  for (long r = r0 + wid; r < r1; r += 4) {
    const T* row = X + r * ld;
    double dot = 0.0;
    for (int c = lane; c < n; c += 64) dot = fma((double)row[c], w[c], dot);
    dot = wave_sum(dot);
    double res, lt;
    logistic_terms(dot + b, (double)y[r], res, lt);
    if (lane == 0) {
      gb += res;
      loss += lt;
    }
    for (int c = lane; c < n; c += 64) atomicAdd(&gl[c], res * (double)row[c]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) atomicAdd(&out[i], gl[i]);
  if (lane == 0) {
    atomicAdd(&out[n], gb);
    atomicAdd(&out[n + 1], loss);
  }
}

template <typename T>
static int binary_lds_launch(const T* X, long m, int n, long ld, const float* y, const double* w, double b,
                             const double* bptr, const int* flag, double* out, hipStream_t stream) {
  if (m <= 0) return 0;
  if (n <= 0 || n > 16384) return -2;
  long blocks = m / 64;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  long rpb = (m + blocks - 1) / blocks;
  blocks = (m + rpb - 1) / rpb;
  const size_t lds = (size_t)n * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)logreg_binary_lds_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL((logreg_binary_lds_kernel<T>), dim3((unsigned)blocks), dim3(256), lds, stream, X, m, n, ld, y, w, b,
                     bptr, flag, out, rpb);
  return srml_status();
}

SRML_API int srml_logreg_binary_lds_f32(const float* X, long m, int n, long ld, const float* y, const double* w,
                                        double b, const double* bptr, const int* flag, double* out,
                                        hipStream_t stream) {
  return binary_lds_launch<float>(X, m, n, ld, y, w, b, bptr, flag, out, stream);
}

SRML_API int srml_logreg_binary_lds_f64(const double* X, long m, int n, long ld, const float* y, const double* w,
                                        double b, const double* bptr, const int* flag, double* out,
                                        hipStream_t stream) {
  return binary_lds_launch<double>(X, m, n, ld, y, w, b, bptr, flag, out, stream);
}
