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
//  * srml_mbin_f32 — the same pass for M INDEPENDENT binary models (hyper-parameter batching:
//    fitMultiple / CrossValidator grids share every read of X): model k's margin x.w_k + b_k,
//    sigmoid residual and softplus loss, gradients [grad w_k | grad b_k | loss_k] per model row.
//  * srml_logreg_binary_lds_{f32,f64} — binary loss + gradient for fp64 inputs and for fp32 rows
//    wider than the register-resident fast path (n <= 16384): one wave per row, the gradient of
//    the block accumulates in LDS (fp64 ds_add), one fp64 atomic per column per block.
// Both take the intercept(s) and an optional `done` flag from device memory so they chain with the
// on-device quasi-Newton step (qn.hip) without host round trips.
#include "common.h"

// SIG = false: softmax over K classes, W (K x n, ldw = n), bvec[k], out = [grad W | grad b | loss].
// SIG = true : K independent binary models, W rows of stride ldw with the intercept at W[k*ldw + n]
//              (bvec = W + n, ldb = ldw), out rows of stride ldo = [grad w_k (n) | grad b_k | loss_k].
template <int KB, int V, int G, bool SIG>
__global__ __launch_bounds__(256, 1) void mlogit_pf_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                           const float* __restrict__ y,
                                                           const double* __restrict__ W, long ldw,
                                                           const double* __restrict__ bvec, long ldb,
                                                           const int* __restrict__ flag, int K,
                                                           double* __restrict__ out, long ldo,
                                                           long rows_per_block, int vec) {
  if (flag && *flag) return;
  // G rows per LDS exchange / barrier (the 4 waves' column-slice margins of a row must meet);
  // the next G rows stream into the other register buffer meanwhile
  __shared__ float part[2][G][KB][4];
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
        wreg[k][v][q] = (k < K && c + q < n) ? (float)W[(long)k * ldw + c + q] : 0.f;
        g[k][v][q] = 0.f;
      }
  }
  // per-class intercepts and the intercept-gradient / loss accumulators live in LDS: only one lane
  // updates them, and per-lane fp64 copies (3 KB doubles) would push the register-resident weight
  // and gradient slices into scratch
  __shared__ double s_bb[KB], s_gb[KB], s_lk[KB];
  if (threadIdx.x < KB) {
    const int k = threadIdx.x;
    s_bb[k] = (k < K && bvec) ? bvec[(long)k * ldb] : 0.0;
    s_gb[k] = 0.0;
    s_lk[k] = 0.0;
  }
  __syncthreads();
  double loss = 0.0;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  if (r0 >= r1) return;

  auto load = [&](long rg, floatx4 (&x)[G][V]) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const long r = rg + gi < r1 ? rg + gi : r1 - 1;  // clamped: the tail rows are never processed
      const float* row = X + r * ld;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int c = cbase + (v * 64 + lane) * 4;
        if (vec && c + 3 < n) {
          x[gi][v] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(row + c));
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) x[gi][v][q] = (c + q < n) ? row[c + q] : 0.f;
        }
      }
    }
  };
  int buf = 0;
  auto process = [&](long rg, const floatx4 (&x)[G][V]) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        float a = 0.f;
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
          for (int q = 0; q < 4; ++q) a = fmaf(x[gi][v][q], wreg[k][v][q], a);
        a = wave_sum(a);
        if (lane == 0) part[buf][gi][k][wid] = a;
      }
    __syncthreads();
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const long r = rg + gi;
      if (r >= r1) break;
      double z[KB];
      double zmax = -1e300;
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        z[k] = (double)part[buf][gi][k][0] + (double)part[buf][gi][k][1] + (double)part[buf][gi][k][2] +
               (double)part[buf][gi][k][3] + s_bb[k];
        if (k < K) zmax = fmax(zmax, z[k]);
      }
      if constexpr (SIG) {
        const double yr = (double)y[r];
#pragma unroll
        for (int k = 0; k < KB; ++k) {
          double res = 0.0, l = 0.0;
          if (k < K) logistic_terms(z[k], yr, res, l);
          const float rf = (float)res;
          if (wid == 0 && lane == 0) { s_gb[k] += res; s_lk[k] += l; }
#pragma unroll
          for (int v = 0; v < V; ++v)
#pragma unroll
            for (int q = 0; q < 4; ++q) g[k][v][q] = fmaf(rf, x[gi][v][q], g[k][v][q]);
        }
      } else {
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
          if (wid == 0 && lane == 0) s_gb[k] += (double)res;
#pragma unroll
          for (int v = 0; v < V; ++v)
#pragma unroll
            for (int q = 0; q < 4; ++q) g[k][v][q] = fmaf(res, x[gi][v][q], g[k][v][q]);
        }
        if (wid == 0 && lane == 0) loss += zmax + (double)__logf(se) - zy;
      }
    }
    buf ^= 1;
  };
  floatx4 xa[G][V], xb[G][V];
  load(r0, xa);
  for (long rg = r0; rg < r1; rg += 2 * G) {
    if (rg + G < r1) load(rg + G, xb);
    process(rg, xa);
    if (rg + G < r1) {
      if (rg + 2 * G < r1) load(rg + 2 * G, xa);
      process(rg + G, xb);
    }
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    if (k < K) {  // a guard, not a break: the loop stays unrolled and g[k] static (no scratch)
#pragma unroll
      for (int v = 0; v < V; ++v)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = cbase + (v * 64 + lane) * 4 + q;
          if (c < n) atomicAdd(&out[(long)k * ldo + c], (double)g[k][v][q]);
        }
    }
  }
  if (wid == 0 && lane == 0) {
    // static indices (k < KB, guarded by K): the per-class accumulators stay in registers
    if constexpr (SIG) {
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        if (k < K) {
          atomicAdd(&out[(long)k * ldo + n], s_gb[k]);
          atomicAdd(&out[(long)k * ldo + n + 1], s_lk[k]);
        }
      }
    } else {
      const long base = (long)K * n;
#pragma unroll
      for (int k = 0; k < KB; ++k)
        if (k < K) atomicAdd(&out[base + k], s_gb[k]);
      atomicAdd(&out[base + K], loss);
    }
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
#define SRML_ML(KK, VV)                                                                                          \
  hipLaunchKernelGGL((mlogit_pf_kernel<KK, VV, (KK <= 4 ? 4 : KK <= 8 ? 2 : 1), false>), grid, blk, 0, stream, X, m, \
                     n, ld, y, W, (long)n, b, 1L, flag, K, out, (long)n, rpb, vec)
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

// M independent binary models in one pass: WB (M rows of stride ldw: w (n) then b), out (M rows of
// stride ldo: grad w (n), grad b, loss), both fp64; same support rule as the multinomial pass.
SRML_API int srml_mbin_f32(const float* X, long m, int n, long ld, const float* y, const double* WB, long ldw, int M,
                           double* out, long ldo, hipStream_t stream) {
  if (m <= 0) return 0;
  if (M < 1 || ldw < n + 1 || ldo < n + 2) return -2;
  if (M == 1 ? !srml_mlogit_supported(n, 2) : !srml_mlogit_supported(n, M)) return -2;
  const int V = (n + 1023) / 1024;
  const int KB = M <= 4 ? 4 : M <= 8 ? 8 : M <= 12 ? 12 : 16;
  long blocks = m / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  long rpb = (m + blocks - 1) / blocks;
  blocks = (m + rpb - 1) / rpb;
  const int vec = ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  dim3 grid((unsigned)blocks), blk(256);
#define SRML_MB(KK, VV)                                                                                             \
  hipLaunchKernelGGL((mlogit_pf_kernel<KK, VV, (KK <= 4 ? 4 : KK <= 8 ? 2 : 1), true>), grid, blk, 0, stream, X, m, n, \
                     ld, y, WB, ldw, WB + n, ldw, (const int*)nullptr, M, out, ldo, rpb, vec)
  if (KB == 4) {
    if (V == 1) SRML_MB(4, 1); else if (V == 2) SRML_MB(4, 2); else if (V == 3) SRML_MB(4, 3); else SRML_MB(4, 4);
  } else if (KB == 8) {
    if (V == 1) SRML_MB(8, 1); else if (V == 2) SRML_MB(8, 2); else if (V == 3) SRML_MB(8, 3); else SRML_MB(8, 4);
  } else if (KB == 12) {
    if (V == 1) SRML_MB(12, 1); else if (V == 2) SRML_MB(12, 2); else SRML_MB(12, 3);
  } else {
    if (V == 1) SRML_MB(16, 1); else SRML_MB(16, 2);
  }
#undef SRML_MB
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Residual stage of the two-pass GLM gradients (margins Z = X W^T from srml_xw_f32, then
// X^T R from srml_xtv2_f32): per row, z_k = Z[r][k] + b_k (fp64 bias from device memory);
//   mode 0 (softmax over K classes): R[r][k] = p_k - [y == k], loss += logsumexp(z) - z_y;
//   mode 1 (K independent binary models): R[r][k] = sigmoid(z_k) - y, loss_k += softplus(z_k) - y z_k.
// Bias gradients (column sums of R) and the loss(es) are block-reduced and added into out:
// gb_k at gb[k * sgb], loss at loss[0] (mode 0) or loss[k * sl] (mode 1).
// zfl (optional): the optimiser's line-search margin cache (qn.hip F_ZMODE / F_ZSEL / SC_BETA), m x K
// fp64 margins (bias included) per buffer in zb: a full evaluation stores its margins in buffer
// 1 - zsel; a margins-only evaluation (F_ZMODE == 1) takes z = z0 + beta (z1 - z0) instead of Z + b
// and writes no R (the X^T R pass is skipped then).
template <typename TZ, int KB>
__global__ __launch_bounds__(256) void logit_residual_kernel(const TZ* __restrict__ Z, long m, int K, long ldz,
                                                             const float* __restrict__ y,
                                                             const double* __restrict__ b, long sb, int mode,
                                                             TZ* __restrict__ R, long ldr,
                                                             double* __restrict__ gb, long sgb,
                                                             double* __restrict__ loss, long sl,
                                                             const int* __restrict__ flag, double* __restrict__ ws,
                                                             const int* __restrict__ zfl = nullptr,
                                                             double* __restrict__ zb = nullptr,
                                                             const double* __restrict__ zsc = nullptr) {
  if (flag && *flag) return;
  const int zmode = zfl ? zfl[9] : 0, zsel = zfl ? zfl[10] : 0;
  const double beta = (zfl && zmode == 1) ? zsc[6] : 0.0;
  const double* z0c = zfl ? zb + (long)zsel * m * K : nullptr;
  double* z1c = zfl ? zb + (long)(1 - zsel) * m * K : nullptr;
  __shared__ double red[4][2 * KB + 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double bk[KB], sg[KB], sls[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    bk[k] = (k < K && b) ? b[(long)k * sb] : 0.0;
    sg[k] = 0.0;
    sls[k] = 0.0;
  }
  double lsum = 0.0;
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < m; r += (long)gridDim.x * 256) {
    double z[KB];
    const float yr = y[r];
    if (zmode == 1) {
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        const double a = k < K ? z0c[r * K + k] : 0.0;
        z[k] = k < K ? a + beta * (z1c[r * K + k] - a) : 0.0;
      }
    } else {
#pragma unroll
      for (int k = 0; k < KB; ++k) z[k] = k < K ? (double)Z[r * ldz + k] + bk[k] : 0.0;
      if (zfl) {
#pragma unroll
        for (int k = 0; k < KB; ++k)
          if (k < K) z1c[r * K + k] = z[k];
      }
    }
    if (mode == 0) {
      double zmax = -1e300;
#pragma unroll
      for (int k = 0; k < KB; ++k)
        if (k < K) zmax = fmax(zmax, z[k]);
      // fp64 softmax: the loss feeds the line search, whose sufficient-decrease test must resolve
      // changes far below fp32's log/exp error
      double e[KB];
      double se = 0.0;
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        e[k] = k < K ? exp(z[k] - zmax) : 0.0;
        se += e[k];
      }
      const int yi = (int)yr;
      const double inv = 1.0 / se;
      double zy = 0.0;
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        if (k < K) {
          const double res = e[k] * inv - (k == yi ? 1.0 : 0.0);
          if (k == yi) zy = z[k];
          if (zmode != 1) R[r * ldr + k] = (TZ)res;
          sg[k] += res;
        }
      }
      lsum += zmax + log(se) - zy;
    } else {
#pragma unroll
      for (int k = 0; k < KB; ++k) {
        if (k < K) {
          double res, l;
          logistic_terms(z[k], (double)yr, res, l);
          if (zmode != 1) R[r * ldr + k] = (TZ)res;
          sg[k] += res;
          sls[k] += l;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    const double a = wave_sum(sg[k]);
    const double c = wave_sum(sls[k]);
    if (lane == 0) { red[wid][k] = a; red[wid][KB + k] = c; }
  }
  const double lw = wave_sum(lsum);
  if (lane == 0) red[wid][2 * KB] = lw;
  __syncthreads();
  if (ws) {  // deterministic mode: [gb (K) | per-model loss (K) | loss] of this block, folded in order
    double* wb = ws + (long)blockIdx.x * (2 * K + 1);
    if (threadIdx.x < K) {
      const int k = threadIdx.x;
      wb[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
      wb[K + k] = red[0][KB + k] + red[1][KB + k] + red[2][KB + k] + red[3][KB + k];
    }
    if (threadIdx.x == 0) wb[2 * K] = red[0][2 * KB] + red[1][2 * KB] + red[2][2 * KB] + red[3][2 * KB];
    return;
  }
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    atomicAdd(&gb[(long)k * sgb], red[0][k] + red[1][k] + red[2][k] + red[3][k]);
    if (mode == 1)
      atomicAdd(&loss[(long)k * sl], red[0][KB + k] + red[1][KB + k] + red[2][KB + k] + red[3][KB + k]);
  }
  if (threadIdx.x == 0 && mode == 0)
    atomicAdd(&loss[0], red[0][2 * KB] + red[1][2 * KB] + red[2][2 * KB] + red[3][2 * KB]);
}

static long logit_residual_blocks(long m) {
  long blocks = (m + 255) / 256;
  return blocks > 2048 ? 2048 : blocks;
}

// Workspace (doubles) of the deterministic residual stage.
SRML_API long srml_logit_residual_ws(long m, int K) { return m <= 0 ? 0 : logit_residual_blocks(m) * (2L * K + 1); }

template <typename TZ>
static int logit_residual_launch(const TZ* Z, long m, int K, long ldz, const float* y, const double* b, long sb,
                                 int mode, TZ* R, long ldr, double* gb, long sgb, double* loss, long sl,
                                 const int* flag, double* ws, hipStream_t stream, const int* zfl = nullptr,
                                 double* zb = nullptr, const double* zsc = nullptr) {
  if (m <= 0) return 0;
  if (K < 1 || K > 16) return -2;
  const long blocks = logit_residual_blocks(m);
#define SRML_RES(KK)                                                                                             \
  hipLaunchKernelGGL((logit_residual_kernel<TZ, KK>), dim3((unsigned)blocks), dim3(256), 0, stream, Z, m, K, ldz, y, b, sb, \
                     mode, R, ldr, gb, sgb, loss, sl, flag, ws, zfl, zb, zsc)
  if (K <= 4) SRML_RES(4);
  else if (K <= 8) SRML_RES(8);
  else SRML_RES(16);
#undef SRML_RES
  int st = srml_status();
  if (st || !ws) return st;
  const long pst = 2L * K + 1;
  st = srml_fold_partials_f64(ws, blocks, pst, K, K, gb, 0, sgb, flag, stream);
  if (st) return st;
  if (mode == 1) return srml_fold_partials_f64(ws + K, blocks, pst, K, K, loss, 0, sl, flag, stream);
  return srml_fold_partials_f64(ws + 2 * K, blocks, pst, 1, 1, loss, 0, 0, flag, stream);
}

SRML_API int srml_logit_residual_f32(const float* Z, long m, int K, long ldz, const float* y, const double* b, long sb,
                                     int mode, float* R, long ldr, double* gb, long sgb, double* loss, long sl,
                                     const int* flag, hipStream_t stream) {
  return logit_residual_launch(Z, m, K, ldz, y, b, sb, mode, R, ldr, gb, sgb, loss, sl, flag, nullptr, stream);
}

// With the optimiser's line-search margin cache (see logit_residual_kernel): zfl = QN flags, zb =
// 2 m K fp64 margins, zsc = QN scalars.
SRML_API int srml_logit_residual_zc_f32(const float* Z, long m, int K, long ldz, const float* y, const double* b,
                                        long sb, int mode, float* R, long ldr, double* gb, long sgb, double* loss,
                                        long sl, const int* flag, const int* zfl, double* zb, const double* zsc,
                                        hipStream_t stream) {
  return logit_residual_launch(Z, m, K, ldz, y, b, sb, mode, R, ldr, gb, sgb, loss, sl, flag, nullptr, stream, zfl, zb,
                               zsc);
}

// fp64 margins / residuals (float32_inputs=False two-pass GLM: margins and X^T R on the fp64 MFMA GEMM)
SRML_API int srml_logit_residual_f64(const double* Z, long m, int K, long ldz, const float* y, const double* b, long sb,
                                     int mode, double* R, long ldr, double* gb, long sgb, double* loss, long sl,
                                     const int* flag, hipStream_t stream) {
  return logit_residual_launch(Z, m, K, ldz, y, b, sb, mode, R, ldr, gb, sgb, loss, sl, flag, nullptr, stream);
}

// Deterministic variant: per-block partials to ws (srml_logit_residual_ws doubles), ordered folds.
SRML_API int srml_logit_residual_det_f32(const float* Z, long m, int K, long ldz, const float* y, const double* b,
                                         long sb, int mode, float* R, long ldr, double* gb, long sgb, double* loss,
                                         long sl, const int* flag, double* ws, hipStream_t stream) {
  if (!ws) return -2;
  return logit_residual_launch(Z, m, K, ldz, y, b, sb, mode, R, ldr, gb, sgb, loss, sl, flag, ws, stream);
}

// ------------------------------------------------------------------------------------------
// Softmax residual for many classes (K > 16, where the register-array kernel above stops): one
// wave per row, the lanes stride over the K margins (max, sum of exponentials and the residual
// row by wave reductions); R = softmax(Z + b) - onehot(y) is written for the X^T R pass and the
// per-row losses lse - z_y are block-reduced into ONE fp64 atomic per block. The bias gradient
// (column sums of R) is formed by the caller's column-sum pass over R.
// T = double (float32_inputs=False): the softmax runs in fp64 (exp/log), matching the K <= 16 path.
template <typename T>
__global__ __launch_bounds__(256) void logit_residual_wide_kernel(const T* __restrict__ Z, long m, int K, long ldz,
                                                                  const float* __restrict__ y,
                                                                  const double* __restrict__ b, long sb,
                                                                  T* __restrict__ R, long ldr,
                                                                  double* __restrict__ loss, const int* __restrict__ flag) {
  if (flag && *flag) return;
  __shared__ double part[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double lsum = 0.0;
  for (long r = (long)blockIdx.x * 4 + wid; r < m; r += (long)gridDim.x * 4) {
    const T* z = Z + r * ldz;
    T mx = -(T)__builtin_huge_val();
    for (int c = lane; c < K; c += 64) mx = fmax(mx, z[c] + (T)b[(long)c * sb]);
    mx = wave_max(mx);
    T se = 0;
    for (int c = lane; c < K; c += 64) se += fexp(z[c] + (T)b[(long)c * sb] - mx);
    se = wave_sum(se);
    const T lse = mx + flog(se);
    const int yi = (int)y[r];
    T* rr = R + r * ldr;
    for (int c = lane; c < K; c += 64) rr[c] = fexp(z[c] + (T)b[(long)c * sb] - lse) - (c == yi ? (T)1 : (T)0);
    if (lane == 0) lsum += (double)lse - ((double)z[yi] + b[(long)yi * sb]);
  }
  if (lane == 0) part[wid] = lsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = (part[0] + part[1]) + (part[2] + part[3]);
    if (t != 0.0) atomicAdd(loss, t);
  }
}

template <typename T>
static int logit_residual_wide_launch(const T* Z, long m, int K, long ldz, const float* y, const double* b, long sb,
                                      T* R, long ldr, double* loss, const int* flag, hipStream_t stream) {
  if (m <= 0) return 0;
  if (K < 2) return -2;
  long blocks = (m + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(logit_residual_wide_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, stream, Z, m, K, ldz, y, b,
                     sb, R, ldr, loss, flag);
  return srml_status();
}

// R (m x K, leading dim ldr) and loss += sum_r (lse_r - z_{r,y_r}) for K classes (any K >= 2).
SRML_API int srml_logit_residual_wide_f32(const float* Z, long m, int K, long ldz, const float* y, const double* b,
                                          long sb, float* R, long ldr, double* loss, const int* flag,
                                          hipStream_t stream) {
  return logit_residual_wide_launch(Z, m, K, ldz, y, b, sb, R, ldr, loss, flag, stream);
}

SRML_API int srml_logit_residual_wide_f64(const double* Z, long m, int K, long ldz, const float* y, const double* b,
                                          long sb, double* R, long ldr, double* loss, const int* flag,
                                          hipStream_t stream) {
  return logit_residual_wide_launch(Z, m, K, ldz, y, b, sb, R, ldr, loss, flag, stream);
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
