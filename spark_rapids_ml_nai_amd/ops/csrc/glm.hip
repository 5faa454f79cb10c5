// GLM primitives: transposed skinny products and the fused logistic loss/gradient.
//
//  * srml_xtv_f32    — out (n x k, fp64) += X^T V  with V (m x k), k <= 4. One streaming pass over
//                      X: lanes own 4 adjacent columns (16-B loads), V rows are broadcast, fp32
//                      partial chains folded to fp64 every 256 rows, one fp64 atomic per column
//                      per block. Normal-equation right-hand side X^T y (LinearRegression),
//                      multinomial LogReg gradient X^T (P - Y).
//  * srml_row_sqnorm_f32 — ||x_r||^2 per row (KMeans inertia, kNN/DBSCAN distances).
//  * srml_logreg_binary_f32 — ONE pass over X per L-BFGS function evaluation:
//        z_r = x_r · w + b ;  loss += softplus(z_r) - y_r z_r ;  g += (sigmoid(z_r) - y_r) x_r
//    wave-per-row: the row (up to 256*V floats) is held in registers while its dot product is
//    reduced with wave64 shuffles, then reused for the gradient update, so X is read exactly
//    once (the reference's cuML QN path reads it twice: forward GEMV then X^T residual).
//    w lives in LDS, each wave keeps a private gradient accumulator in registers, waves fold
//    into LDS and blocks fold into the fp64 output with atomics.
#include "common.h"
#include <stdlib.h>

// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void xtv_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                  const float* __restrict__ V, long ldv, double* __restrict__ out,
                                                  long rows_per_block) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  if (c0 >= n) return;
  double acc[K][4];
  float facc[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[k][j] = 0.0; facc[k][j] = 0.f; }
  const bool full = (c0 + 3 < n) && ((ld & 3) == 0);
  int cnt = 0;
  for (long r = r0; r < r1; ++r) {
    floatx4 x;
    if (full) {
      x = *reinterpret_cast<const floatx4*>(X + r * ld + c0);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = (c0 + j < n) ? X[r * ld + c0 + j] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float v = V[r * ldv + k];
#pragma unroll
      for (int j = 0; j < 4; ++j) facc[k][j] = fmaf(x[j], v, facc[k][j]);
    }
    if (++cnt == 256) {
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[k][j] += facc[k][j]; facc[k][j] = 0.f; }
      cnt = 0;
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[k][j] += facc[k][j];
      if (c0 + j < n) atomicAdd(&out[(long)(c0 + j) * K + k], acc[k][j]);
    }
}

SRML_API int srml_xtv_f32(const float* X, long m, int n, long ld, const float* V, int k, long ldv, double* out,
                          hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  unsigned gx = ceil_div(n, 1024);
  long gy = (2048 + gx - 1) / gx;
  long rpb = (m + gy - 1) / gy;
  if (rpb < 64) rpb = 64;
  gy = (m + rpb - 1) / rpb;
  dim3 grid(gx, (unsigned)gy);
  switch (k) {
    case 1: hipLaunchKernelGGL(xtv_kernel<1>, grid, dim3(256), 0, stream, X, m, n, ld, V, ldv, out, rpb); break;
    case 2: hipLaunchKernelGGL(xtv_kernel<2>, grid, dim3(256), 0, stream, X, m, n, ld, V, ldv, out, rpb); break;
    case 3: hipLaunchKernelGGL(xtv_kernel<3>, grid, dim3(256), 0, stream, X, m, n, ld, V, ldv, out, rpb); break;
    case 4: hipLaunchKernelGGL(xtv_kernel<4>, grid, dim3(256), 0, stream, X, m, n, ld, V, ldv, out, rpb); break;
    default: return -1;
  }
  return srml_status();
}

// Wider / strided variant for the two-pass multi-class and multi-model GLM gradients:
// out[c * so_c + k * so_k] += sum_r X[r][c] V[r][k], k < K <= 16, skipped once *flag != 0.
template <int K>
__global__ __launch_bounds__(256) void xtv2_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                   const float* __restrict__ V, long ldv, double* __restrict__ out,
                                                   long so_c, long so_k, long rows_per_block, int kk,
                                                   const int* __restrict__ flag) {
  if (flag && *flag) return;
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  if (c0 >= n) return;
  double acc[K][4];
  float facc[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[k][j] = 0.0; facc[k][j] = 0.f; }
  const bool full = (c0 + 3 < n) && ((ld & 3) == 0);
  int cnt = 0;
  for (long r = r0; r < r1; ++r) {
    floatx4 x;
    if (full) {
      x = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(X + r * ld + c0));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = (c0 + j < n) ? X[r * ld + c0 + j] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float v = k < kk ? V[r * ldv + k] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) facc[k][j] = fmaf(x[j], v, facc[k][j]);
    }
    if (++cnt == 256) {
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[k][j] += facc[k][j]; facc[k][j] = 0.f; }
      cnt = 0;
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[k][j] += facc[k][j];
      if (k < kk && c0 + j < n) atomicAdd(&out[(long)(c0 + j) * so_c + (long)k * so_k], acc[k][j]);
    }
}

SRML_API int srml_xtv2_f32(const float* X, long m, int n, long ld, const float* V, int k, long ldv, double* out,
                           long so_c, long so_k, const int* flag, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  unsigned gx = ceil_div(n, 1024);
  long gy = (2048 + gx - 1) / gx;
  long rpb = (m + gy - 1) / gy;
  if (rpb < 64) rpb = 64;
  gy = (m + rpb - 1) / rpb;
  dim3 grid(gx, (unsigned)gy);
#define SRML_XTV2(KK)                                                                                            \
  hipLaunchKernelGGL(xtv2_kernel<KK>, grid, dim3(256), 0, stream, X, m, n, ld, V, ldv, out, so_c, so_k, rpb, k, flag)
  if (k <= 1) SRML_XTV2(1);
  else if (k <= 2) SRML_XTV2(2);
  else if (k <= 4) SRML_XTV2(4);
  else if (k <= 8) SRML_XTV2(8);
  else if (k <= 12) SRML_XTV2(12);
  else if (k <= 16) SRML_XTV2(16);
  else return -1;
#undef SRML_XTV2
  return srml_status();
}

// MFMA variant of the same product for K <= 16: out^T (K x n) = V^T X accumulated on
// v_mfma_f32_16x16x4_f32 with the reduction running over rows. A = V^T (lane: V[r + (l>>4)][l&15]);
// B = 4 rows x 16 columns of X where lane l loads ONE 16-B vector X[r + (l>>4)][c0 + 4(l&15) .. +3]
// and component q feeds column tile q (columns c0 + 4j + q), so every X load is a full 256-B row
// segment. fp32 partials fold into fp64 registers every 256 rows (the VALU kernel's precision
// contract); a wave owns 64 columns, a block 256 columns x rows_per_block rows.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void xtv_mfma_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                       const float* __restrict__ V, int K, long ldv,
                                                       double* __restrict__ out, long so_c, long so_k,
                                                       long rows_per_block, int vec, const int* __restrict__ flag,
                                                       double* __restrict__ ws) {
  if (flag && *flag) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int c0 = (blockIdx.x * WPB + (threadIdx.x >> 6)) * 64;
  if (c0 >= n) return;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  const int cl = c0 + 4 * li;
  const bool cfull = vec && (c0 + 63 < n);  // wave-uniform: MFMAs ignore EXEC, so no lane may diverge
  const bool kok = li < K;
  double accd[4][4];
  floatx4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) accd[q][e] = 0.0;
  }
  const int kl = kok ? li : 0;
  long rc = r0;
  if (cfull) {
    // branch-free body over whole 256-row chunks: 16 rows (4 MFMA steps) per group, the next
    // group's 16-B X loads and V words issued before this group's MFMAs
    const float* xp = X + (rc + g) * ld + cl;
    const float* vp = V + (rc + g) * ldv + kl;
    for (; rc + 256 <= r1; rc += 256) {
      floatx4 x[4];
      float a[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        x[s] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(xp + 4 * s * ld));
        a[s] = vp[4 * s * ldv];
      }
#pragma unroll 1
      for (int grp = 0; grp < 16; ++grp) {
        xp += 16 * ld;
        vp += 16 * ldv;
        floatx4 xn[4];
        float an[4];
        if (grp < 15) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            xn[s] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(xp + 4 * s * ld));
            an[s] = vp[4 * s * ldv];
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float av = kok ? a[s] : 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, x[s][q], acc[q], 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          x[s] = xn[s];
          a[s] = an[s];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int e = 0; e < 4; ++e) accd[q][e] += (double)acc[q][e];
        acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  for (; rc < r1; rc += 256) {  // ragged chunk / partial column group: guarded loads
#pragma unroll 4
    for (int s = 0; s < 64; ++s) {
      const long r = rc + 4 * s + g;
      const bool ok = r < r1;
      floatx4 x;
#pragma unroll
      for (int q = 0; q < 4; ++q) x[q] = (ok && cl + q < n) ? X[r * ld + cl + q] : 0.f;
      const float a = (ok && kok) ? V[r * ldv + li] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, x[q], acc[q], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 4; ++e) accd[q][e] += (double)acc[q][e];
      acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
  // lane holds D[i = 4g + e][j = l & 15] of tile q: class k = 4g + e, column c0 + 4j + q
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int col = cl + q;
    if (col >= n) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * g + e;
      if (k >= K) continue;
      if (ws)  // deterministic mode: this block-row's partial, folded in order by the launcher
        ws[((long)blockIdx.y * n + col) * K + k] = accd[q][e];
      else
        atomicAdd(&out[(long)col * so_c + (long)k * so_k], accd[q][e]);
    }
  }
}

namespace {
struct XtvGrid {
  int wpb;
  unsigned gx;
  long gy, rpb;
};
XtvGrid xtv_mfma_grid(long m, int n) {
  // 16 waves (1024 columns = 4 KB of every row) per block when n is wide enough: one block streams
  // long contiguous row segments; narrow n keeps 4-wave blocks so the grid still fills the chip.
  XtvGrid gr;
  gr.wpb = n >= 2048 ? 16 : 4;
  gr.gx = ceil_div(n, 64 * gr.wpb);
  const long target = gr.wpb == 16 ? 512 : 2048;
  long gy = (target + gr.gx - 1) / gr.gx;
  long rpb = (m + gy - 1) / gy;
  rpb = ((rpb + 255) / 256) * 256;
  gr.gy = (m + rpb - 1) / rpb;
  gr.rpb = rpb;
  return gr;
}
}  // namespace

// Workspace (doubles) the deterministic variant needs: one n x K partial per block row.
SRML_API long srml_xtv_mfma_ws(long m, int n, int k) {
  if (m <= 0 || n <= 0) return 0;
  return xtv_mfma_grid(m, n).gy * (long)n * k;
}

static int xtv_mfma_launch(const float* X, long m, int n, long ld, const float* V, int k, long ldv, double* out,
                           long so_c, long so_k, const int* flag, double* ws, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  if (k < 1 || k > 16) return -2;
  const int vec = ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  const XtvGrid gr = xtv_mfma_grid(m, n);
  if (gr.wpb == 16)
    hipLaunchKernelGGL(xtv_mfma_kernel<16>, dim3(gr.gx, (unsigned)gr.gy), dim3(1024), 0, stream, X, m, n, ld, V, k,
                       ldv, out, so_c, so_k, gr.rpb, vec, flag, ws);
  else
    hipLaunchKernelGGL(xtv_mfma_kernel<4>, dim3(gr.gx, (unsigned)gr.gy), dim3(256), 0, stream, X, m, n, ld, V, k, ldv,
                       out, so_c, so_k, gr.rpb, vec, flag, ws);
  int st = srml_status();
  if (st || !ws) return st;
  return srml_fold_partials_f64(ws, gr.gy, (long)n * k, (long)n * k, k, out, so_c, so_k, flag, stream);
}

SRML_API int srml_xtv_mfma_f32(const float* X, long m, int n, long ld, const float* V, int k, long ldv, double* out,
                               long so_c, long so_k, const int* flag, hipStream_t stream) {
  return xtv_mfma_launch(X, m, n, ld, V, k, ldv, out, so_c, so_k, flag, nullptr, stream);
}

// Deterministic variant: block-row partials to ws (srml_xtv_mfma_ws doubles), then an ordered fold.
SRML_API int srml_xtv_mfma_det_f32(const float* X, long m, int n, long ld, const float* V, int k, long ldv,
                                   double* out, long so_c, long so_k, const int* flag, double* ws,
                                   hipStream_t stream) {
  if (!ws) return -2;
  return xtv_mfma_launch(X, m, n, ld, V, k, ldv, out, so_c, so_k, flag, ws, stream);
}

__global__ __launch_bounds__(256) void fold_partials_kernel(const double* __restrict__ ws, long parts, long pstride,
                                                            long width, long inner, double* __restrict__ out,
                                                            long so_outer, long so_inner,
                                                            const int* __restrict__ flag) {
  if (flag && *flag) return;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= width) return;
  double s = 0.0;
  for (long p = 0; p < parts; ++p) s += ws[p * pstride + i];
  out[(i / inner) * so_outer + (i % inner) * so_inner] += s;
}

SRML_API int srml_fold_partials_f64(const double* ws, long parts, long pstride, long width, long inner, double* out,
                                    long so_outer, long so_inner, const int* flag, hipStream_t stream) {
  if (width <= 0 || parts <= 0) return 0;
  if (inner < 1) return -2;
  hipLaunchKernelGGL(fold_partials_kernel, dim3(ceil_div(width, 256)), dim3(256), 0, stream, ws, parts, pstride, width,
                     inner, out, so_outer, so_inner, flag);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void row_sqnorm_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                         float* __restrict__ out, const float* __restrict__ mu,
                                                         unsigned* __restrict__ amax = nullptr) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  const bool vec = ((ld & 3) == 0) && ((n & 3) == 0);
  float mx = 0.f;  // max |x - mu| seen by this lane (amax: the fp16 KMeans filter's plane scale)
  for (long r = wave; r < m; r += nw) {
    const float* row = X + r * ld;
    float s = 0.f;
    if (vec) {
      for (int d = lane * 4; d < n; d += 256) {
        floatx4 v = *reinterpret_cast<const floatx4*>(row + d);
        if (mu) {
          const floatx4 c = *reinterpret_cast<const floatx4*>(mu + d);
          v[0] -= c[0]; v[1] -= c[1]; v[2] -= c[2]; v[3] -= c[3];
        }
        s = fmaf(v[0], v[0], fmaf(v[1], v[1], fmaf(v[2], v[2], fmaf(v[3], v[3], s))));
        if (amax) mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
    } else {
      for (int d = lane; d < n; d += 64) {
        const float v = mu ? row[d] - mu[d] : row[d];
        s = fmaf(v, v, s);
        mx = fmaxf(mx, fabsf(v));
      }
    }
    s = wave_sum(s);
    if (lane == 0) out[r] = s;
  }
  if (amax) {
    mx = wave_max(mx);  // non-negative floats order like their bit patterns
    if (lane == 0) atomicMax(amax, __float_as_uint(mx));
  }
}

SRML_API int srml_row_sqnorm_f32(const float* X, long m, int n, long ld, float* out, hipStream_t stream) {
  if (m <= 0) return 0;
  long blocks = (m + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(row_sqnorm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, out,
                     (const float*)nullptr);
  return srml_status();
}

// ||x_r - mu||^2 per row (mu: n floats, 16-B aligned): the centred norms of the KMeans search
SRML_API int srml_row_sqnorm_centered_f32(const float* X, long m, int n, long ld, const float* mu, float* out,
                                          hipStream_t stream) {
  if (m <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(mu) & 15) return -5;
  long blocks = (m + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(row_sqnorm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, out, mu);
  return srml_status();
}

// ||x_r - mu||^2 per row plus max |x - mu| over the whole matrix into *amax (float bits, caller
// zeroes it): one pass over X for both the centred norms and the fp16 filter plane's scale
SRML_API int srml_row_sqnorm_centered_amax_f32(const float* X, long m, int n, long ld, const float* mu, float* out,
                                               unsigned* amax, hipStream_t stream) {
  if (m <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(mu) & 15) return -5;
  long blocks = (m + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(row_sqnorm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, out, mu, amax);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// fused binary logistic loss + gradient
// out layout (fp64): [0..n) gradient wrt w, [n] gradient wrt b, [n+1] loss sum
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float softplus_f(float z) {
  // log(1 + exp(z)) without overflow
  return z > 0.f ? z + log1pf(__expf(-z)) : log1pf(__expf(z));
}


template <int V, bool REREAD>
__global__ __launch_bounds__(256) void logreg_binary_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                            const float* __restrict__ y, const double* __restrict__ w,
                                                            double b_in, const double* __restrict__ bptr,
                                                            const int* __restrict__ flag, double* __restrict__ out,
                                                            long rows_per_block) {
  if (flag && *flag) return;  // the on-device quasi-Newton driver has converged
  const double b = bptr ? *bptr : b_in;
  // w is kept in fp64 (LDS) and margins / losses are evaluated in fp64 so that the objective the
  // quasi-Newton line search sees is smooth to ~1e-15; X stays fp32 and the kernel stays
  // HBM-bound (fp64 FMA rate is far above the 1 FMA per 4 streamed bytes needed here).
  extern __shared__ __attribute__((aligned(16))) double ldsd[];  // w[256*V] (fp64) then gsum[256*V] (fp32)
  double* ws = ldsd;
  float* gs = reinterpret_cast<float*>(ldsd + 256 * V);
  const int NV = 256 * V;
  for (int i = threadIdx.x; i < NV; i += 256) {
    ws[i] = (i < n) ? w[i] : 0.0;
    gs[i] = 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);

  floatx4 g[V];
#pragma unroll
  for (int v = 0; v < V; ++v) g[v] = floatx4{0.f, 0.f, 0.f, 0.f};
  double gb = 0.0, loss = 0.0;
  const bool vec = ((ld & 3) == 0);
  for (long r = r0 + wid; r < r1; r += 4) {
    const float* row = X + r * ld;
    floatx4 x[REREAD ? 1 : V];
    double dot = 0.0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = (v * 64 + lane) * 4;
      floatx4& xv = x[REREAD ? 0 : v];
      if (vec && c + 3 < n) {
        xv = *reinterpret_cast<const floatx4*>(row + c);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) xv[q] = (c + q < n) ? row[c + q] : 0.f;
      }
      const double2 w01 = *reinterpret_cast<const double2*>(&ws[c]);
      const double2 w23 = *reinterpret_cast<const double2*>(&ws[c + 2]);
      dot = fma((double)xv[0], w01.x, fma((double)xv[1], w01.y, fma((double)xv[2], w23.x,
                fma((double)xv[3], w23.y, dot))));
    }
    dot = wave_sum(dot);
    const double z = dot + b;
    const double yr = (double)y[r];
    double res, lt;
    logistic_terms(z, yr, res, lt);
    if (lane == 0) {
      loss += lt;
      gb += res;
    }
    const float rf = (float)res;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      floatx4 xv;
      if (REREAD) {  // second touch of the row hits L1/L2; HBM traffic is unchanged
        const int c = (v * 64 + lane) * 4;
        if (vec && c + 3 < n) {
          xv = *reinterpret_cast<const floatx4*>(row + c);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) xv[q] = (c + q < n) ? row[c + q] : 0.f;
        }
      } else {
        xv = x[v];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) g[v][q] = fmaf(rf, xv[q], g[v][q]);
    }
  }
  // fold the 4 waves' gradients in LDS, then one fp64 atomic per column per block
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int q = 0; q < 4; ++q) atomicAdd(&gs[(v * 64 + lane) * 4 + q], g[v][q]);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) atomicAdd(&out[i], (double)gs[i]);
  if (lane == 0) {
    atomicAdd(&out[n], gb);
    atomicAdd(&out[n + 1], loss);
  }
}


// Column-split variant for 1024 < n <= 4096: each of the 4 waves owns a 256*V-column slice of
// every row (x and its gradient slice stay in registers), the block processes R rows per step;
// per-row partial margins are exchanged through LDS (double-buffered, one barrier per step).
template <int V, int R>
__global__ __launch_bounds__(256, 2) void logreg_binary_split_kernel(const float* __restrict__ X, long m, int n,
                                                                     long ld, const float* __restrict__ y,
                                                                     const double* __restrict__ w, double b_in,
                                                                     const double* __restrict__ bptr,
                                                                     const int* __restrict__ flag,
                                                                     double* __restrict__ out, long rows_per_block) {
  if (flag && *flag) return;
  const double b = bptr ? *bptr : b_in;
  __shared__ double part[2][R][4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int cbase = wid * 256 * V;
  double wreg[V][4];
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = cbase + (v * 64 + lane) * 4 + q;
      wreg[v][q] = c < n ? w[c] : 0.0;
    }
  floatx4 g[V];
#pragma unroll
  for (int v = 0; v < V; ++v) g[v] = floatx4{0.f, 0.f, 0.f, 0.f};
  double gb = 0.0, loss = 0.0;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  const bool vec = ((ld & 3) == 0);
  int buf = 0;
  for (long rb = r0; rb < r1; rb += R) {
    floatx4 x[R][V];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long r = rb + i;
      double dot = 0.0;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int c = cbase + (v * 64 + lane) * 4;
        // branch-free: clamped row / column, out-of-range lanes multiply by zero weights
        // (wreg is 0 beyond n) and rows past r1 are dropped after the reduction
        const float* row = X + (r < r1 ? r : r1 - 1) * ld;
        floatx4 xv;
        if (vec) {
          xv = *reinterpret_cast<const floatx4*>(row + (c + 3 < n ? c : 0));
          if (c + 3 >= n) xv = floatx4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) xv[q] = row[c + q < n ? c + q : 0] * (c + q < n ? 1.f : 0.f);
        }
        x[i][v] = xv;
        dot = fma((double)xv[0], wreg[v][0], fma((double)xv[1], wreg[v][1],
              fma((double)xv[2], wreg[v][2], fma((double)xv[3], wreg[v][3], dot))));
      }
      dot = wave_sum(dot);
      if (lane == 0) part[buf][i][wid] = dot;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long r = rb + i;
      if (r >= r1) break;
      const double z = part[buf][i][0] + part[buf][i][1] + part[buf][i][2] + part[buf][i][3] + b;
      const double yr = (double)y[r];
      double res, lt;
      logistic_terms(z, yr, res, lt);
      if (wid == 0 && lane == 0) {
        loss += lt;
        gb += res;
      }
      const float rf = (float)res;
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int q = 0; q < 4; ++q) g[v][q] = fmaf(rf, x[i][v][q], g[v][q]);
    }
    buf ^= 1;
  }
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = cbase + (v * 64 + lane) * 4 + q;
      if (c < n) atomicAdd(&out[c], (double)g[v][q]);
    }
  if (wid == 0 && lane == 0) {
    atomicAdd(&out[n], gb);
    atomicAdd(&out[n + 1], loss);
  }
}

// Column-split + prefetch variant: like logreg_binary_split_kernel, but the next R-row batch is
// loaded into a second register set while the current batch's margins are reduced / exchanged
// through LDS and its gradient is accumulated, so each wave keeps 2 * R * V * 1 KiB of X in flight
// across the per-batch barrier (the kernel is HBM-latency bound, not VALU bound).
// Line-search margin cache (zfl != null; the optimiser's flag block, see qn.hip F_ZMODE): along a
// search direction the margins are linear in the step, z(a) = z0 + (a / a1) (z(a1) - z0), so once
// a full evaluation at a1 is rejected, the backtracking trials need only the loss from the two
// stored margin vectors (16 B per row instead of the row's n floats):
//   mode 0 / 2  full pass; the row margins (intercept included) go to zb[(1 - zsel) m + r];
//   mode 1      loss / bias gradient from z0 = zb[zsel m ..], z1 = zb[(1 - zsel) m ..] and
//               beta = zsc[SC_BETA]; the gradient columns of the partial row are zero.
constexpr int LR_F_ZMODE = 9, LR_F_ZSEL = 10, LR_SC_BETA = 6;

// margins-only evaluation of one block's rows (zmode 1, see logreg_binary_pf_kernel): loss and
// bias gradient from z0 + beta (z1 - z0); the partial row's gradient columns (ws) are zero
__device__ __forceinline__ void lr_margin_only(long m, int n, const float* __restrict__ y, double* __restrict__ out,
                                               float* __restrict__ ws, const double* __restrict__ zb,
                                               const double* __restrict__ zsc, int zsel, long q0, long rows) {
  __shared__ double mred[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const double beta = zsc[LR_SC_BETA];
  const double* z0 = zb + (long)zsel * m;
  const double* z1 = zb + (long)(1 - zsel) * m;
  const long q1 = min(m, q0 + rows);
  double gbc = 0.0, lossc = 0.0;
  for (long r = q0 + threadIdx.x; r < q1; r += blockDim.x) {
    const double a = z0[r];
    double res, lt;
    logistic_terms(a + beta * (z1[r] - a), (double)y[r], res, lt);
    gbc += res;
    lossc += lt;
  }
  gbc = wave_sum(gbc);
  lossc = wave_sum(lossc);
  if (lane == 0) {
    mred[0][wid] = gbc;
    mred[1][wid] = lossc;
  }
  __syncthreads();
  gbc = (mred[0][0] + mred[0][1]) + (mred[0][2] + mred[0][3]);
  lossc = (mred[1][0] + mred[1][1]) + (mred[1][2] + mred[1][3]);
  if (ws == nullptr) {
    if (threadIdx.x == 0) {
      if (gbc != 0.0) atomicAdd(&out[n], gbc);
      if (lossc != 0.0) atomicAdd(&out[n + 1], lossc);
    }
    return;
  }
  const long wsc = (long)((n + 3) & ~3) + 4;
  float* mine = ws + (long)blockIdx.x * wsc;
  for (int c = 4 * threadIdx.x; c < n; c += 4 * blockDim.x)
    *reinterpret_cast<floatx4*>(mine + c) = floatx4{0.f, 0.f, 0.f, 0.f};
  if (threadIdx.x == 0) {
    double* md = reinterpret_cast<double*>(mine + wsc - 4);
    md[0] = gbc;
    md[1] = lossc;
  }
}

template <int V, int R, int D, bool NT = false>
__global__ __launch_bounds__(256, 2) void logreg_binary_pf_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                                  const float* __restrict__ y,
                                                                  const double* __restrict__ w, double b_in,
                                                                  const double* __restrict__ bptr,
                                                                  const int* __restrict__ flag,
                                                                  double* __restrict__ out, long rows_per_block,
                                                                  float* __restrict__ ws, const int* __restrict__ zfl,
                                                                  double* __restrict__ zb,
                                                                  const double* __restrict__ zsc) {
  if (flag && *flag) return;
  const double b = bptr ? *bptr : b_in;
  __shared__ double part[2][R][4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int zmode = zfl ? zfl[LR_F_ZMODE] : 0;
  const int zsel = zfl ? zfl[LR_F_ZSEL] : 0;
  if (zmode == 1) {
    lr_margin_only(m, n, y, out, ws, zb, zsc, zsel, (long)blockIdx.x * rows_per_block, rows_per_block);
    return;
  }
  double* zw = zfl ? zb + (long)(1 - zsel) * m : nullptr;
  const int cbase = wid * 256 * V;
  double wreg[V][4];
  int coff[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int c = cbase + (v * 64 + lane) * 4;
    coff[v] = (c + 3 < n) ? c : 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) wreg[v][q] = (c + 3 < n) ? w[c + q] : 0.0;
  }
  // tail columns (n % 4 != 0 or ld unaligned) are handled by the generic kernel; see launcher
  floatx4 g[V];
#pragma unroll
  for (int v = 0; v < V; ++v) g[v] = floatx4{0.f, 0.f, 0.f, 0.f};
  double gb = 0.0, loss = 0.0;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  if (r0 >= r1 && ws == nullptr) return;  // (partial rows: an empty block still stores its zero row)

  auto load = [&](long rb, floatx4 (&x)[R][V]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long r = rb + i < r1 ? rb + i : r1 - 1;
      const float* row = X + r * ld;
#pragma unroll
      for (int v = 0; v < V; ++v)
        x[i][v] = NT ? __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(row + coff[v]))
                     : *reinterpret_cast<const floatx4*>(row + coff[v]);
    }
  };
  int buf = 0;
  auto process = [&](long rb, const floatx4 (&x)[R][V]) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double dot = 0.0;
#pragma unroll
      for (int v = 0; v < V; ++v)
        dot = fma((double)x[i][v][0], wreg[v][0], fma((double)x[i][v][1], wreg[v][1],
              fma((double)x[i][v][2], wreg[v][2], fma((double)x[i][v][3], wreg[v][3], dot))));
      dot = wave_sum(dot);
      if (lane == 0) part[buf][i][wid] = dot;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const long r = rb + i;
      if (r < r1) {
        const double z = part[buf][i][0] + part[buf][i][1] + part[buf][i][2] + part[buf][i][3] + b;
        double res, lt;
        logistic_terms(z, (double)y[r], res, lt);
        if (wid == 0 && lane == 0) {
          loss += lt;
          gb += res;
          if (zw) zw[r] = z;
        }
        const float rf = (float)res;
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
          for (int q = 0; q < 4; ++q) g[v][q] = fmaf(rf, x[i][v][q], g[v][q]);
      }
    }
    buf ^= 1;
  };
  // ring of D + 1 register batches: batch j is loaded D batches ahead of its use
  floatx4 x[D + 1][R][V];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (r0 + d * R < r1) load(r0 + d * R, x[d]);
  for (long rb = r0; rb < r1; rb += (D + 1) * R) {
#pragma unroll
    for (int ph = 0; ph <= D; ++ph) {
      const long cur = rb + ph * R;
      if (cur < r1) {
        const long nxt = cur + D * R;
        if (nxt < r1) load(nxt, x[(ph + D) % (D + 1)]);
        process(cur, x[ph]);
      }
    }
  }
  if (ws == nullptr) {
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = cbase + (v * 64 + lane) * 4 + q;
        if (cbase + (v * 64 + lane) * 4 + 3 < n) atomicAdd(&out[c], (double)g[v][q]);
      }
    if (wid == 0 && lane == 0) {
      atomicAdd(&out[n], gb);
      atomicAdd(&out[n + 1], loss);
    }
    return;
  }
  // Partial-row epilogue: when every block of a chip-filling grid ends at the same moment (all
  // 768 blocks of a 125k-row shard are resident at once), n fp64 atomics per block arrive as one
  // burst on the same n addresses (2.3M atomics: ~40 us of a 0.29 ms evaluation). Instead each
  // block stores its fp32 partial row with plain vector stores and fold_rows_kernel sums them
  // right after (same stream; the kernel boundary orders the stores).
  const long wst = (long)((n + 3) & ~3) + 4;  // floats per partial row: columns, then gb, loss (fp64)
  float* mine = ws + (long)blockIdx.x * wst;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int c = cbase + (v * 64 + lane) * 4;
    if (c + 3 < n) *reinterpret_cast<floatx4*>(mine + c) = g[v];
  }
  if (wid == 0 && lane == 0) {
    double* md = reinterpret_cast<double*>(mine + wst - 4);
    md[0] = gb;
    md[1] = loss;
  }
}

// Narrow rows (n <= 512, the BASELINE north-star LogisticRegression is 200M x 256): a 64-lane wave
// per row leaves 3/4 of the lanes idle below n = 256 and keeps one 1 KiB row in flight per wave
// behind its dependent reduce -> exp/log chain. Here 16 lanes own a row (G float4 of it per lane),
// a wave works on 4 rows at once, the row dot product is a 16-lane DPP reduction (the DPP row
// size) and D row batches are loaded ahead into a register ring, so each wave keeps up to
// 4 (D + 1) rows of X in flight.
template <int G, int D>
__global__ __launch_bounds__(256) void logreg_binary_narrow_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                                   const float* __restrict__ y,
                                                                   const double* __restrict__ w, double b_in,
                                                                   const double* __restrict__ bptr,
                                                                   const int* __restrict__ flag,
                                                                   double* __restrict__ out, long rows_per_block,
                                                                   const int* __restrict__ zfl,
                                                                   double* __restrict__ zb,
                                                                   const double* __restrict__ zsc) {
  if (flag && *flag) return;
  const int zmode = zfl ? zfl[LR_F_ZMODE] : 0;
  const int zsel = zfl ? zfl[LR_F_ZSEL] : 0;
  if (zmode == 1) {  // line-search margin cache: see logreg_binary_pf_kernel
    lr_margin_only(m, n, y, out, nullptr, zb, zsc, zsel, (long)blockIdx.x * rows_per_block, rows_per_block);
    return;
  }
  double* zw = zfl ? zb + (long)(1 - zsel) * m : nullptr;
  __shared__ float gsum[4][64 * G];
  __shared__ double red[2][4];
  const double b = bptr ? *bptr : b_in;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int sub = lane & 15, grp = lane >> 4;
  double wr[G][4];
  bool cok[G];
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const int c = (k * 16 + sub) * 4;
    cok[k] = c + 3 < n;
#pragma unroll
    for (int q = 0; q < 4; ++q) wr[k][q] = cok[k] ? w[c + q] : 0.0;
  }
  floatx4 g[G];
#pragma unroll
  for (int k = 0; k < G; ++k) g[k] = floatx4{0.f, 0.f, 0.f, 0.f};
  double gb = 0.0, loss = 0.0;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  const int roff = wid * 4 + grp;  // this lane group's row within a 16-row step of the block
  auto load = [&](long base, floatx4 (&x)[G]) {
    long r = base + roff;
    if (r >= r1) r = r1 - 1;  // clamped rows are loaded but never accumulated
    const float* row = X + r * ld;
#pragma unroll
    for (int k = 0; k < G; ++k)
      x[k] = cok[k] ? __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(row + (k * 16 + sub) * 4))
                    : floatx4{0.f, 0.f, 0.f, 0.f};
  };
  auto process = [&](long base, const floatx4 (&x)[G]) {
    const long r = base + roff;
    double dot = 0.0;
#pragma unroll
    for (int k = 0; k < G; ++k)
      dot = fma((double)x[k][0], wr[k][0], fma((double)x[k][1], wr[k][1],
            fma((double)x[k][2], wr[k][2], fma((double)x[k][3], wr[k][3], dot))));
    dot += dpp_d<0xb1>(dot);   // quad_perm [1,0,3,2]
    dot += dpp_d<0x4e>(dot);   // quad_perm [2,3,0,1]
    dot += dpp_d<0x141>(dot);  // row_half_mirror
    dot += dpp_d<0x140>(dot);  // row_mirror: every lane of the 16-lane row holds the row's dot
    if (r < r1) {
      double res, lt;
      logistic_terms(dot + b, (double)y[r], res, lt);
      if (sub == 0) {
        loss += lt;
        gb += res;
        if (zw) zw[r] = dot + b;
      }
      const float rf = (float)res;
#pragma unroll
      for (int k = 0; k < G; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) g[k][q] = fmaf(rf, x[k][q], g[k][q]);
    }
  };
  floatx4 xs[D + 1][G];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (r0 + d * 16 < r1) load(r0 + d * 16, xs[d]);
  for (long rb = r0; rb < r1; rb += (D + 1) * 16) {
#pragma unroll
    for (int ph = 0; ph <= D; ++ph) {
      const long cur = rb + ph * 16;
      if (cur < r1) {
        const long nxt = cur + D * 16;
        if (nxt < r1) load(nxt, xs[(ph + D) % (D + 1)]);
        process(cur, xs[ph]);
      }
    }
  }
  // fold the 4 row groups of the wave (lanes sub, sub + 16, sub + 32, sub + 48 share columns),
  // then the 4 waves through LDS, then one fp64 atomic per column per block
#pragma unroll
  for (int k = 0; k < G; ++k)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = g[k][q];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (grp == 0) gsum[wid][(k * 16 + sub) * 4 + q] = v;
    }
  loss = wave_sum(loss);
  gb = wave_sum(gb);
  if (lane == 0) {
    red[0][wid] = gb;
    red[1][wid] = loss;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < n; c += 256) {
    const float v = (gsum[0][c] + gsum[1][c]) + (gsum[2][c] + gsum[3][c]);
    if (v != 0.f) atomicAdd(&out[c], (double)v);
  }
  if (threadIdx.x == 0) {
    atomicAdd(&out[n], (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]));
    atomicAdd(&out[n + 1], (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
  }
}

// Sum of `parts` partial rows (fp32 columns + 2 trailing fp64 [gb, loss]) into out (fp64), no
// atomics: block b owns columns [64 b, 64 b + 64) — 16 lanes x float4 per row, 16 row groups
// striding the rows (independent 16-B loads, fp64 sums), folded through LDS and added into its
// own columns with plain read-modify-writes; the extra last block folds gb / loss. (A per-slice
// fp64 atomic fold took 12 us at 768 partial rows: 48-way contention on every column.)
__global__ __launch_bounds__(256) void fold_rows_kernel(const float* __restrict__ ws, int parts, long wst, int n,
                                                        double* __restrict__ out, const int* __restrict__ flag) {
  if (flag && *flag) return;
  __shared__ double red[16][65];
  const int t = threadIdx.x;
  const int q = t & 15, rg = t >> 4;
  const int ncb = (n + 63) / 64;
  if ((int)blockIdx.x < ncb) {
    const int c = (int)blockIdx.x * 64 + 4 * q;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (c < n) {
      int p = rg;
      for (; p + 48 < parts; p += 64) {  // 4 rows in flight per thread
        floatx4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[j] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(ws + (long)(p + 16 * j) * wst + c));
#pragma unroll
        for (int j = 0; j < 4; ++j) { a0 += v[j][0]; a1 += v[j][1]; a2 += v[j][2]; a3 += v[j][3]; }
      }
      for (; p < parts; p += 16) {
        const floatx4 v = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(ws + (long)p * wst + c));
        a0 += v[0]; a1 += v[1]; a2 += v[2]; a3 += v[3];
      }
    }
    red[rg][4 * q] = a0;
    red[rg][4 * q + 1] = a1;
    red[rg][4 * q + 2] = a2;
    red[rg][4 * q + 3] = a3;
    __syncthreads();
    if (t < 64) {
      const int cc = (int)blockIdx.x * 64 + t;
      double sum = 0.0;
#pragma unroll
      for (int g = 0; g < 16; ++g) sum += red[g][t];
      if (cc < n) out[cc] += sum;
    }
    return;
  }
  // last block: gb and loss
  double gb = 0.0, loss = 0.0;
  for (int p = t; p < parts; p += 256) {
    const double* pd = reinterpret_cast<const double*>(ws + (long)p * wst + wst - 4);
    gb += pd[0];
    loss += pd[1];
  }
  gb = wave_sum(gb);
  loss = wave_sum(loss);
  if ((t & 63) == 0) {
    red[0][t >> 6] = gb;
    red[1][t >> 6] = loss;
  }
  __syncthreads();
  if (t == 0) {
    out[n] += (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    out[n + 1] += (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

static long logreg_grid(long m) {
  // ~>= 160 rows per block: each block pays a w load and an n-wide flush, so small shards (the
  // per-rank rows of a multi-GPU fit) want fewer blocks (125k rows: 768 blocks = 3 per CU, all
  // resident at once (149 VGPRs); 1M rows: 2048)
  static const long blocks_env = getenv("SRML_LOGREG_BLOCKS") ? atol(getenv("SRML_LOGREG_BLOCKS")) : 0;
  long blocks = blocks_env;
  if (blocks <= 0) {
    blocks = m / 163;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 512) blocks = 512;
  }
  long rpb = (m + blocks - 1) / blocks;
  if (rpb < 16) rpb = 16;
  return (m + rpb - 1) / rpb;
}

// The prefetching column-split kernel (the only one with a partial-row epilogue) runs for this
// shape / layout: 1024 < n <= 4096, 16-B aligned rows, n % 4 == 0, SRML_LOGREG_SPLIT == 2.
static bool logreg_pf_eligible(int n, long ld, const void* X) {
  static const int split = getenv("SRML_LOGREG_SPLIT") ? atoi(getenv("SRML_LOGREG_SPLIT")) : 2;
  return split == 2 && n > 1024 && n <= 4096 && (n & 3) == 0 && (ld & 3) == 0 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

static bool logreg_fold_enabled() {
  // SRML_LOGREG_FOLD=0: one fp64 atomic flush per block instead of partial rows + a fold
  static const int fold = getenv("SRML_LOGREG_FOLD") ? atoi(getenv("SRML_LOGREG_FOLD")) : 1;
  return fold != 0;
}

// Floats of the partial-row workspace srml_logreg_binary3_f32 needs for X (m x n, row stride ld)
// — 0 unless the evaluation of exactly this operand writes partial rows (the consumer may then
// fold them; any other kernel flushes into `out` and would leave a workspace unwritten).
SRML_API long srml_logreg_fold_ws(long m, int n, long ld, const void* X) {
  if (m <= 0 || !logreg_fold_enabled() || !logreg_pf_eligible(n, ld, X)) return 0;
  return logreg_grid(m) * (((n + 3) & ~3) + 4);
}

// Partial rows (= blocks) the workspace holds for m rows; row stride ((n + 3) & ~3) + 4 floats.
SRML_API long srml_logreg_fold_parts(long m) { return m <= 0 ? 0 : logreg_grid(m); }

static int logreg_binary_launch(const float* X, long m, int n, long ld, const float* y, const double* w, double b,
                                const double* bptr, const int* flag, double* out, float* fold_ws, int leave,
                                hipStream_t stream, const int* zfl = nullptr, double* zb = nullptr,
                                const double* zsc = nullptr);

// b: intercept by value, or (bptr != null) read on the device; flag (optional): skip when *flag != 0
SRML_API int srml_logreg_binary2_f32(const float* X, long m, int n, long ld, const float* y, const double* w, double b,
                                     const double* bptr, const int* flag, double* out, hipStream_t stream) {
  return logreg_binary_launch(X, m, n, ld, y, w, b, bptr, flag, out, nullptr, 0, stream);
}

// Same with the caller's partial-row workspace (srml_logreg_fold_ws floats, owned by ONE fit: the
// block partials and their fold are two launches, so interleaved fits need separate workspaces).
// leave != 0: the rows are NOT folded into `out` here — the consumer (the fused optimiser step,
// srml_qn_step_fused) folds them itself.
SRML_API int srml_logreg_binary3_f32(const float* X, long m, int n, long ld, const float* y, const double* w, double b,
                                     const double* bptr, const int* flag, double* out, float* fold_ws, int leave,
                                     hipStream_t stream) {
  return logreg_binary_launch(X, m, n, ld, y, w, b, bptr, flag, out, fold_ws, leave, stream);
}

// Same with the optimiser's line-search margin cache (see logreg_binary_pf_kernel): zfl = the QN
// flag block, zb = 2 m doubles of margins, zsc = the QN scalars. Only the prefetching column-split
// kernel implements it: -2 for any other shape (the caller checks srml_logreg_fold_ws > 0 first).
static bool logreg_narrow_eligible(int n, long ld, const void* X) {
  static const int narrow = getenv("SRML_LOGREG_NARROW") ? atoi(getenv("SRML_LOGREG_NARROW")) : 1;
  return narrow && n <= 512 && (n & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}

// Whether the evaluation of X (m x n, row stride ld) runs a kernel with the line-search margin
// cache (the narrow n <= 512 or the prefetching 1024 < n <= 4096 kernel).
SRML_API int srml_logreg_zcache_ok(long m, int n, long ld, const void* X) {
  return m > 0 && (logreg_narrow_eligible(n, ld, X) || logreg_pf_eligible(n, ld, X)) ? 1 : 0;
}

SRML_API int srml_logreg_binary4_f32(const float* X, long m, int n, long ld, const float* y, const double* w, double b,
                                     const double* bptr, const int* flag, double* out, float* fold_ws, int leave,
                                     const int* zfl, double* zb, const double* zsc, hipStream_t stream) {
  if (m > 0 && !srml_logreg_zcache_ok(m, n, ld, X)) return -2;
  return logreg_binary_launch(X, m, n, ld, y, w, b, bptr, flag, out, fold_ws, leave, stream, zfl, zb, zsc);
}

static int logreg_binary_launch(const float* X, long m, int n, long ld, const float* y, const double* w, double b,
                                const double* bptr, const int* flag, double* out, float* fold_ws, int leave,
                                hipStream_t stream, const int* zfl, double* zb, const double* zsc) {
  if (m <= 0) return 0;
  if (zfl && !logreg_pf_eligible(n, ld, X) && !logreg_narrow_eligible(n, ld, X)) return -2;
  if (logreg_narrow_eligible(n, ld, X)) {
    long nb = m / 256;  // ~256 rows (16 steps of 16) per block, 512 .. 4096 blocks
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    long rpb = (m + nb - 1) / nb;
    rpb = (rpb + 15) / 16 * 16;
    const long blocks = (m + rpb - 1) / rpb;
    const int G = (n + 63) / 64;
#define SRML_LR_NARROW(GG, DD)                                                                                       \
  hipLaunchKernelGGL((logreg_binary_narrow_kernel<GG, DD>), dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, \
                     y, w, b, bptr, flag, out, rpb, zfl, zb, zsc)
    if (G <= 1) SRML_LR_NARROW(1, 3);
    else if (G <= 2) SRML_LR_NARROW(2, 3);
    else if (G <= 4) SRML_LR_NARROW(4, 3);
    else SRML_LR_NARROW(8, 2);
#undef SRML_LR_NARROW
    return srml_status();
  }
  // grid sweep (tools/lr_small_sweep.sh): 125k rows 768 blocks 0.310 ms, 1024 0.331, 1536 0.345,
  // 512 0.328; 1M rows: 2048 best
  const long blocks = logreg_grid(m);
  long rpb = (m + blocks - 1) / blocks;
  if (rpb < 16) rpb = 16;
  int V = (n + 255) / 256;
  const size_t vpad = V <= 1 ? 1 : V <= 2 ? 2 : V <= 4 ? 4 : V <= 8 ? 8 : V <= 12 ? 12 : 16;
  size_t lds = 256 * vpad * (sizeof(double) + sizeof(float));
  dim3 grid((unsigned)blocks), blk(256);
  static const int split = getenv("SRML_LOGREG_SPLIT") ? atoi(getenv("SRML_LOGREG_SPLIT")) : 2;
  // prefetching column-split kernel: needs 16-B aligned rows and n % 4 == 0 (no tail columns)
  if (logreg_pf_eligible(n, ld, X)) {
    static const int rsel = getenv("SRML_LOGREG_R") ? atoi(getenv("SRML_LOGREG_R")) : 1;
    static const int dsel = getenv("SRML_LOGREG_D") ? atoi(getenv("SRML_LOGREG_D")) : 3;
    static const int nt = getenv("SRML_LOGREG_NT") ? atoi(getenv("SRML_LOGREG_NT")) : 1;  // nontemporal X stream: +2%
    const int VS = (n + 1023) / 1024;
    // partial-row epilogue + fold kernel when the caller passed a workspace
    const long wst = ((n + 3) & ~3) + 4;
    float* fws = logreg_fold_enabled() ? fold_ws : nullptr;
#define SRML_LR_PF(VV, RR, DD)                                                                              \
    hipLaunchKernelGGL((logreg_binary_pf_kernel<VV, RR, DD>), grid, blk, 0, stream, X, m, n, ld, y, w, b, bptr, \
                       flag, out, rpb, fws, zfl, zb, zsc)
#define SRML_LR_PF_V(RR, DD) \
    do { if (VS == 2) SRML_LR_PF(2, RR, DD); else if (VS == 3) SRML_LR_PF(3, RR, DD); else SRML_LR_PF(4, RR, DD); } while (0)
    if (rsel == 2 && dsel == 1) SRML_LR_PF_V(2, 1);
    else if (rsel == 2) SRML_LR_PF_V(2, 2);
    else if (dsel == 1) SRML_LR_PF_V(1, 1);
    else if (dsel == 3 && nt) {
#define SRML_LR_PF_NT(VV)                                                                                        \
  hipLaunchKernelGGL((logreg_binary_pf_kernel<VV, 1, 3, true>), grid, blk, 0, stream, X, m, n, ld, y, w, b, bptr, \
                     flag, out, rpb, fws, zfl, zb, zsc)
      if (VS == 2) SRML_LR_PF_NT(2);
      else if (VS == 3) SRML_LR_PF_NT(3);
      else SRML_LR_PF_NT(4);
#undef SRML_LR_PF_NT
    }
    else if (dsel == 3) SRML_LR_PF_V(1, 3);
    else SRML_LR_PF_V(1, 2);
    if (fws && !leave)
      hipLaunchKernelGGL(fold_rows_kernel, dim3(ceil_div(n, 64) + 1), dim3(256), 0, stream, fws, (int)blocks, wst, n,
                         out, flag);
    return srml_status();
  }
  if (split == 1 && n > 1024 && n <= 4096) {
    static const int rsel = getenv("SRML_LOGREG_R") ? atoi(getenv("SRML_LOGREG_R")) : 4;
    const int VS = (n + 1023) / 1024;
#define SRML_LR_SPLIT(VV, RR) \
    hipLaunchKernelGGL((logreg_binary_split_kernel<VV, RR>), grid, blk, 0, stream, X, m, n, ld, y, w, b, bptr, flag, out, rpb)
    if (rsel == 8) {
      if (VS == 1) SRML_LR_SPLIT(1, 8); else if (VS == 2) SRML_LR_SPLIT(2, 8);
      else if (VS == 3) SRML_LR_SPLIT(3, 8); else SRML_LR_SPLIT(4, 8);
    } else if (rsel == 2) {
      if (VS == 1) SRML_LR_SPLIT(1, 2); else if (VS == 2) SRML_LR_SPLIT(2, 2);
      else if (VS == 3) SRML_LR_SPLIT(3, 2); else SRML_LR_SPLIT(4, 2);
    } else {
      if (VS == 1) SRML_LR_SPLIT(1, 4); else if (VS == 2) SRML_LR_SPLIT(2, 4);
      else if (VS == 3) SRML_LR_SPLIT(3, 4); else SRML_LR_SPLIT(4, 4);
    }
    return srml_status();
  }
  const int reread = 0;
#define SRML_LR_LAUNCH(VV)                                                                                       \
  do {                                                                                                           \
    if (reread)                                                                                                  \
      hipLaunchKernelGGL((logreg_binary_kernel<VV, true>), grid, blk, lds, stream, X, m, n, ld, y, w, b, bptr, flag, out, rpb);  \
    else                                                                                                         \
      hipLaunchKernelGGL((logreg_binary_kernel<VV, false>), grid, blk, lds, stream, X, m, n, ld, y, w, b, bptr, flag, out, rpb); \
  } while (0)
  if (V <= 1) SRML_LR_LAUNCH(1);
  else if (V <= 2) SRML_LR_LAUNCH(2);
  else if (V <= 4) SRML_LR_LAUNCH(4);
  else if (V <= 8) SRML_LR_LAUNCH(8);
  else if (V <= 12) SRML_LR_LAUNCH(12);
  else if (V <= 16) SRML_LR_LAUNCH(16);
  else return -2;  // n > 4096: caller uses the two-pass GEMV path
  return srml_status();
}

SRML_API int srml_logreg_binary_f32(const float* X, long m, int n, long ld, const float* y, const double* w, double b,
                                    double* out, hipStream_t stream) {
  return srml_logreg_binary2_f32(X, m, n, ld, y, w, b, nullptr, nullptr, out, stream);
}
