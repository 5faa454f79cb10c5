// On-device quasi-Newton driver (L-BFGS, and OWL-QN for L1 / elastic-net) for the GLM solvers.
//
// Reference: cuML's QN solver behind LogisticRegressionMG (classification.py:957-1151,
// lbfgs_memory=10, penalty_normalized=False): it runs its L-BFGS / OWL-QN iteration on the host
// and pays a device round trip per function evaluation. Here the whole optimiser state lives in
// device memory and ONE single-block kernel advances it after every (all-reduced) loss+gradient
// evaluation, so a fit is a stream of   [fused loss/grad pass] -> [RCCL all-reduce] -> [qn step]
// launches with no host synchronisation; the host only polls a `done` flag every few evaluations
// (and the evaluation kernels early-exit once it is set).
//
// State machine per call (one evaluation at the trial point xt has just been summed into `out`):
//   pass 0  smooth gradient at xt in the optimiser's (standardised) coordinates, penalty terms,
//           directional derivatives; `out` is re-zeroed for the next evaluation.
//   line search (backtracking Armijo — cuML's default LBFGS_LS_BT_ARMIJO — with a safeguarded quadratic
//           interpolation step in [0.1, 0.5] instead of plain halving; optional weak
//           Wolfe with inc = 2.1 until bracketed; OWL-QN: Armijo on the projected step).
//   accept  pass 1 computes, in ONE fused multi-value block reduction, every dot product the
//           compact L-BFGS representation needs (Byrd-Nocedal-Schnabel: H = gI + [S gY] M [S gY]^T)
//           — new-pair products with the history and S^T pg, Y^T pg — instead of the 2m dependent
//           reductions of the two-loop recursion; thread 0 solves the small triangular systems;
//           pass 2 stores the pair, forms the direction (orthant-constrained for OWL-QN) and
//           moves x; pass 3 writes the next trial point (orthant-projected) and the evaluation
//           parameters w = xt[:Kn] * inv_sigma, b = xt[Kn:].
// Convergence (cuML qn semantics): max|pg| <= tol * max(|f|, tol); |f_{k-past} - f_k| <= delta *
// max(|f|, tol); k >= max_iter; or a failed line search (the last accepted point is kept).
#include "common.h"

namespace {

constexpr int QN_T = 512;      // one block, 8 waves: the passes are latency-bound (204 VGPRs, no spills)
constexpr int QN_NW = QN_T / 64;
constexpr int QN_MMAX = 12;    // history capacity (runtime M <= 12; the reference uses 10)
constexpr int QN_NV = 6 + 5 * QN_MMAX;

// F_ZC .. F_NCHEAP / SC_ALPHA1, SC_BETA: the line-search margin cache of the multi-block step
// (binary LogisticRegression, Armijo, no L1; glm.hip logreg_binary_pf_kernel reads F_ZMODE /
// F_ZSEL / SC_BETA): F_ZMODE is the mode of the NEXT evaluation — 0 full, 1 margins-only (a
// backtracking trial: loss from z0 + beta (z1 - z0)), 2 full at a point a margins-only trial
// already accepted; F_ZSEL selects which of the two margin buffers holds z0 (the accepted point).
// F_SKIPX: 1 while the next evaluation must not read X (margins-only, or the fit is done) — the
// skip word of the multinomial margin pass / X^T R pass (two-pass GLM)
enum { F_DONE = 0, F_STATUS, F_ITER, F_NEVAL, F_LS, F_COUNT, F_HEAD, F_STARTED, F_BRACKET, F_ZMODE, F_ZSEL,
       F_NCHEAP, F_ZC, F_SKIPX };
enum { ST_RUNNING = 0, ST_CONV_GRAD = 1, ST_CONV_F = 2, ST_MAXITER = 3, ST_LS_FAIL = 4 };
enum { SC_F = 0, SC_ALPHA, SC_DGINIT, SC_GAMMA, SC_GINF, SC_ALPHA1, SC_BETA };

}  // namespace

// Host-visible argument block (mirrored by a ctypes.Structure in ops/__init__.py)
struct QnArgs {
  long N;        // parameters: Kn + (K if fit_intercept else 0)
  long Kn;       // coefficients K * n
  int n, K, M, past, max_iter, max_ls, l1, wolfe;
  double tol, delta, inv_m, c1, c2;
  double *x, *g, *pg, *d, *xt, *gt;  // [N] each
  double *S, *Y;                     // [M][N]
  double *SY, *YY;                   // [M][M] slot-indexed s_i.y_j, y_i.y_j
  double *fh;                        // [past] objective history
  double *sc;                        // scalars
  const double *l2, *l1c;            // [N] penalty coefficients in optimiser coordinates
  const double *isg;                 // [n] 1 / sigma (0 for constant columns)
  int *fl;                           // int flags
  double *wb;                        // evaluation parameters [Kn | K] in the original space
  double *out;                       // summed evaluation [grad_w (Kn) | grad_b (K) | loss]
  long long *probe;                  // optional: wall-clock stamps of the kernel's sections (tuning)
};

// Block-wide sum of NV per-thread values; every thread receives the totals. `red` holds
// NV * QN_NW wave partials followed by NV totals (the totals are folded by NV threads, so no thread
// holds NV * QN_NW LDS loads in registers).
template <int NV>
__device__ __forceinline__ void qn_block_sum(double (&v)[NV], double* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const double t = wave_sum(v[i]);
    if (lane == 0) red[i * QN_NW + wid] = t;
    __builtin_amdgcn_sched_barrier(0);  // one reduction at a time: no NV-wide live DPP temporaries
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < QN_NW; ++w) s += red[threadIdx.x * QN_NW + w];
    red[NV * QN_NW + threadIdx.x] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[NV * QN_NW + i];
}

__device__ __forceinline__ double qn_block_max(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int w = 1; w < QN_NW; ++w) r = fmax(r, red[w]);
  __syncthreads();
  return r;
}

// OWL-QN pseudo-gradient of f + sum c_i |x_i|
__device__ __forceinline__ double pseudo_grad(double x, double g, double c) {
  if (c <= 0.0) return g;
  if (x > 0.0) return g + c;
  if (x < 0.0) return g - c;
  if (g + c < 0.0) return g + c;
  if (g - c > 0.0) return g - c;
  return 0.0;
}

// Element loops: every thread owns i = tid + k * QN_T and handles QN_U of its elements per batch,
// issuing all of a batch's loads before any store (the state vectors are separate allocations, but
// the compiler cannot prove it, so without batching each element's loads would wait for the
// previous element's stores: one full memory latency per element).
constexpr int QN_U = 4;
#define QN_BATCH(i0) for (long i0 = threadIdx.x; i0 < A.N; i0 += (long)QN_T * QN_U)
#define QN_LANE(u, i0) const long i_##u = (i0) + (long)(u) * QN_T

// next trial point xt = x + alpha d (orthant-projected on L1 coordinates) and its evaluation params
__device__ void qn_set_trial(const QnArgs& A, double alpha) {
  QN_BATCH(i0) {
    double xv[QN_U], dv[QN_U], pv[QN_U], cv[QN_U], sv[QN_U];
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      const bool ok = i < A.N;
      xv[u] = ok ? A.x[i] : 0.0;
      dv[u] = ok ? A.d[i] : 0.0;
      pv[u] = (ok && A.l1) ? A.pg[i] : 0.0;
      cv[u] = (ok && A.l1) ? A.l1c[i] : 0.0;
      sv[u] = (ok && i < A.Kn) ? A.isg[i % A.n] : 1.0;
    }
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      if (i < A.N) {
        double t = xv[u] + alpha * dv[u];
        if (cv[u] > 0.0) {
          const double orth = xv[u] != 0.0 ? (xv[u] > 0.0 ? 1.0 : -1.0) : (pv[u] < 0.0 ? 1.0 : (pv[u] > 0.0 ? -1.0 : 0.0));
          if (t * orth <= 0.0) t = 0.0;
        }
        A.xt[i] = t;
        A.wb[i] = t * sv[u];
      }
    }
  }
}

#define QN_PROBE(k) \
  do { if (A.probe && threadIdx.x == 0) A.probe[k] = wall_clock64(); } while (0)

__device__ __forceinline__ void qn_step_body(const QnArgs& A) {
  __shared__ double red[QN_NV * (QN_NW + 1)];
  __shared__ double cf_a[QN_MMAX], cf_t[QN_MMAX];
  __shared__ double s_sy[QN_MMAX * QN_MMAX], s_yy[QN_MMAX * QN_MMAX];
  __shared__ double s_p1[QN_MMAX], s_p2[QN_MMAX], s_t[QN_MMAX], s_a[QN_MMAX];
  __shared__ int s_sl[QN_MMAX];
  __shared__ double s_v[QN_NV];
  __shared__ double s_misc[4];
  __shared__ int s_ctl[4];
  int* fl = A.fl;
  if (fl[F_DONE]) return;
  QN_PROBE(0);
  const int tid = threadIdx.x;
  const long N = A.N, Kn = A.Kn;
  const int M = A.M;
  const double lossv = A.out[Kn + A.K];
  // optimiser scalars, loaded up front so their latency hides under pass 0
  const bool started = fl[F_STARTED] != 0;
  const int pre_iter = fl[F_ITER];
  const int count = fl[F_COUNT];
  const int head = fl[F_HEAD];
  const int pre_ls = fl[F_LS];
  const int pre_neval = fl[F_NEVAL];
  const bool bracket = fl[F_BRACKET] != 0;
  const double f = A.sc[SC_F];
  double alpha = A.sc[SC_ALPHA];
  const double dginit = A.sc[SC_DGINIT];
  const double pre_gamma = A.sc[SC_GAMMA];
  const double pre_fh_next = (A.past > 0 && started) ? A.fh[(pre_iter + 1) % A.past] : 0.0;
  // line-search margin cache (see the multi-block step K2): the mode of the evaluation just summed
  const bool zc = fl[F_ZC] != 0;
  const int zmode = zc ? fl[F_ZMODE] : 0;
  const double alpha1 = A.sc[SC_ALPHA1];

  // ---- pass 0: smooth gradient at xt (optimiser coordinates), penalties, directional terms
  double p0[4] = {0.0, 0.0, 0.0, 0.0};
  QN_BATCH(i0) {
    double xv[QN_U], ov[QN_U], sv[QN_U], l2v[QN_U], l1v[QN_U], dv[QN_U], pv[QN_U], xo[QN_U];
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      const bool ok = i < N;
      xv[u] = ok ? A.xt[i] : 0.0;
      ov[u] = ok ? A.out[i] : 0.0;
      sv[u] = (ok && i < Kn) ? A.isg[i % A.n] : 1.0;
      l2v[u] = ok ? A.l2[i] : 0.0;
      l1v[u] = ok ? A.l1c[i] : 0.0;
      dv[u] = ok ? A.d[i] : 0.0;
      pv[u] = ok ? A.pg[i] : 0.0;
      xo[u] = ok ? A.x[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      if (i < N) {
        const double gi = ov[u] * A.inv_m * sv[u] + l2v[u] * xv[u];
        A.gt[i] = gi;
        p0[0] += l2v[u] * xv[u] * xv[u];
        p0[1] += l1v[u] * fabs(xv[u]);
        p0[2] += gi * dv[u];
        p0[3] += pv[u] * (xv[u] - xo[u]);
      }
    }
  }
  qn_block_sum<4>(p0, red);  // every read of `out` precedes this barrier
  QN_PROBE(1);
  for (long i = tid; i < Kn + A.K + 1; i += QN_T) A.out[i] = 0.0;
  const double ft = lossv * A.inv_m + 0.5 * p0[0] + p0[1];

  // ---- line search decision (uniform: every thread sees the same reduced values)
  if (tid == 0 && zc && zmode == 1) fl[F_NCHEAP] += 1;
  if (started) {
    bool accept = true;
    double width = 1.0;
    if (zc && zmode == 2 && isfinite(ft)) {
      // a margins-only trial passed at this point: this full evaluation supplies its gradient
    } else if (!isfinite(ft)) {
      accept = false;
      width = 0.5;
    } else {
      const double dgtest = A.l1 ? p0[3] : alpha * dginit;
      if (ft > f + A.c1 * dgtest) {
        // safeguarded quadratic interpolation through phi(0), phi'(0) alpha, phi(alpha)
        accept = false;
        const double den = 2.0 * (ft - f - dgtest);
        width = den > 0.0 ? -dgtest / den : 0.5;
        width = isfinite(width) ? fmin(0.5, fmax(0.1, width)) : 0.5;
      } else if (A.wolfe && !A.l1 && !bracket && p0[2] < A.c2 * dginit) {
        accept = false;
        width = 2.1;
      }
    }
    if (!accept) {
      const int ls = pre_ls + 1;
      __syncthreads();
      if (ls >= A.max_ls) {
        if (tid == 0) {
          fl[F_LS] = ls;
          fl[F_NEVAL] = pre_neval + 1;
          fl[F_STATUS] = ST_LS_FAIL;
          fl[F_DONE] = 1;
          fl[F_SKIPX] = 1;
        }
        return;
      }
      const double alpha_tried = alpha;
      alpha *= width;
      qn_set_trial(A, alpha);
      if (tid == 0) {
        fl[F_LS] = ls;
        fl[F_NEVAL] = pre_neval + 1;
        if (width < 1.0) fl[F_BRACKET] = 1;
        A.sc[SC_ALPHA] = alpha;
        if (zc && isfinite(ft)) {
          const double a1 = zmode == 0 ? alpha_tried : alpha1;
          A.sc[SC_ALPHA1] = a1;
          A.sc[SC_BETA] = alpha / a1;
          fl[F_ZMODE] = 1;
          fl[F_SKIPX] = 1;
        } else if (zc) {
          fl[F_ZMODE] = 0;
          fl[F_SKIPX] = 0;
        }
      }
      return;
    }
    if (zc && zmode == 1) {  // accepted on margins only: evaluate the same point in full next
      if (tid == 0) {
        fl[F_NEVAL] = pre_neval + 1;
        fl[F_ZMODE] = 2;
        fl[F_SKIPX] = 0;
      }
      return;
    }
  }
  if (tid == 0 && zc) {  // this full evaluation's margins are the accepted point's
    fl[F_ZSEL] ^= 1;
    fl[F_ZMODE] = 0;
    fl[F_SKIPX] = 0;
  }

  // ---- accepted: pass 1 — pseudo-gradient at xt and every dot product of the compact form
  // 1a: pseudo-gradient at xt, new pair s = xt - x, y = gt - g (kept in the free d / wb buffers for
  //     the next passes), and s.y, y.y, s.pg, y.pg, pg.pg, max |pg|
  double v5[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double ginf = 0.0;
  QN_BATCH(i0) {
    double xv[QN_U], gv[QN_U], xo[QN_U], go[QN_U], cv[QN_U];
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      const bool ok = i < N;
      xv[u] = ok ? A.xt[i] : 0.0;
      gv[u] = ok ? A.gt[i] : 0.0;
      xo[u] = ok ? A.x[i] : 0.0;
      go[u] = ok ? A.g[i] : 0.0;
      cv[u] = (ok && A.l1) ? A.l1c[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      if (i < N) {
        const double sx = started ? xv[u] - xo[u] : 0.0;
        const double yx = started ? gv[u] - go[u] : 0.0;
        const double pgi = pseudo_grad(xv[u], gv[u], cv[u]);
        A.pg[i] = pgi;
        A.d[i] = sx;
        A.wb[i] = yx;
        ginf = fmax(ginf, fabs(pgi));
        v5[0] += sx * yx;
        v5[1] += yx * yx;
        v5[2] += sx * pgi;
        v5[3] += yx * pgi;
        v5[4] += pgi * pgi;
      }
    }
  }
  // stage the history Gram blocks in LDS: the serial small solve below must not chase global loads
  for (int i = tid; i < M * M; i += QN_T) {
    s_sy[i] = A.SY[i];
    s_yy[i] = A.YY[i];
  }
  qn_block_sum<6>(v5, red);
  QN_PROBE(2);
  ginf = qn_block_max(ginf, red);
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < 6; ++j) s_v[j] = v5[j];
  }
  // 1b: products with the stored pairs, QN_JB history slots per sweep (bounded register set)
  constexpr int QN_JB = 5;
  constexpr int QN_UB = 2;
  for (int j0 = 0; j0 < M; j0 += QN_JB) {
    double w[5 * QN_JB];
#pragma unroll
    for (int q = 0; q < 5 * QN_JB; ++q) w[q] = 0.0;
    for (long i0 = tid; i0 < N; i0 += (long)QN_T * QN_UB) {
      double sv[QN_UB], yv[QN_UB], pv[QN_UB], Sv[QN_UB][QN_JB], Yv[QN_UB][QN_JB];
#pragma unroll
      for (int u = 0; u < QN_UB; ++u) {
        const long i = i0 + (long)u * QN_T;
        const bool ok = i < N;
        sv[u] = ok ? A.d[i] : 0.0;
        yv[u] = ok ? A.wb[i] : 0.0;
        pv[u] = ok ? A.pg[i] : 0.0;
#pragma unroll
        for (int jj = 0; jj < QN_JB; ++jj) {
          const bool okj = ok && (j0 + jj < M);
          Sv[u][jj] = okj ? A.S[(long)(j0 + jj) * N + i] : 0.0;
          Yv[u][jj] = okj ? A.Y[(long)(j0 + jj) * N + i] : 0.0;
        }
      }
#pragma unroll
      for (int u = 0; u < QN_UB; ++u)
#pragma unroll
        for (int jj = 0; jj < QN_JB; ++jj) {
          w[5 * jj + 0] += sv[u] * Yv[u][jj];
          w[5 * jj + 1] += Sv[u][jj] * yv[u];
          w[5 * jj + 2] += yv[u] * Yv[u][jj];
          w[5 * jj + 3] += Sv[u][jj] * pv[u];
          w[5 * jj + 4] += Yv[u][jj] * pv[u];
        }
    }
    qn_block_sum<5 * QN_JB>(w, red);
    if (tid == 0) {
#pragma unroll
      for (int jj = 0; jj < QN_JB; ++jj) {
        const int j = j0 + jj;
        if (j < M) {
          s_v[6 + j] = w[5 * jj + 0];
          s_v[6 + QN_MMAX + j] = w[5 * jj + 1];
          s_v[6 + 2 * QN_MMAX + j] = w[5 * jj + 2];
          s_v[6 + 3 * QN_MMAX + j] = w[5 * jj + 3];
          s_v[6 + 4 * QN_MMAX + j] = w[5 * jj + 4];
        }
      }
    }
  }

  QN_PROBE(3);
  // ---- lane 0: history bookkeeping and convergence (LDS + prefetched scalars only)
  if (tid == 0) {
    int cnt = count, hd = head, status = ST_RUNNING;
    double gamma = started ? pre_gamma : 1.0;
    for (int j = 0; j < M; ++j) {
      s_p1[j] = s_v[6 + 3 * QN_MMAX + j];
      s_p2[j] = s_v[6 + 4 * QN_MMAX + j];
    }
    const double ys = s_v[0], yy = s_v[1];
    const bool newp = started && yy > 0.0 && ys > 1e-10 * yy;
    if (newp) {
      const int h = hd;
      for (int j = 0; j < M; ++j) {
        if (j == h) continue;
        s_sy[h * M + j] = s_v[6 + j];
        s_sy[j * M + h] = s_v[6 + QN_MMAX + j];
        s_yy[h * M + j] = s_v[6 + 2 * QN_MMAX + j];
        s_yy[j * M + h] = s_v[6 + 2 * QN_MMAX + j];
      }
      s_sy[h * M + h] = ys;
      s_yy[h * M + h] = yy;
      s_p1[h] = s_v[2];
      s_p2[h] = s_v[3];
      hd = (h + 1) % M;
      cnt = cnt < M ? cnt + 1 : M;
      gamma = ys / yy;
    }
    const double fn = ft;
    const int iter = pre_iter + (started ? 1 : 0);
    const double fmag = fmax(fabs(fn), A.tol);
    if (ginf <= A.tol * fmag) status = ST_CONV_GRAD;
    if (A.past > 0) {
      const double fold = started ? pre_fh_next : 0.0;
      if (status == ST_RUNNING && started && iter >= A.past && fabs(fold - fn) <= A.delta * fmag) status = ST_CONV_F;
      A.fh[iter % A.past] = fn;
    }
    if (status == ST_RUNNING && iter >= A.max_iter) status = ST_MAXITER;
    for (int c = 0; c < cnt; ++c) s_sl[c] = (hd - cnt + c + 2 * M) % M;
    s_ctl[0] = status;
    s_ctl[1] = newp ? 1 : 0;
    s_ctl[2] = cnt;
    s_misc[0] = gamma;
    fl[F_ITER] = iter;
    fl[F_HEAD] = hd;
    fl[F_COUNT] = cnt;
    fl[F_NEVAL] = pre_neval + 1;
    fl[F_LS] = 0;
    fl[F_BRACKET] = 0;
    fl[F_STARTED] = 1;
    A.sc[SC_F] = fn;
    A.sc[SC_GAMMA] = gamma;
    A.sc[SC_GINF] = ginf;
  }
  __syncthreads();
  // ---- wave 0: compact-form coefficients, lane c = chronological pair c:
  //      t = R^-1 p1 (back substitution), a = R^-T ((D + gamma YtY) t - gamma p2) (forward),
  //      R_ce = s_c.y_e (c <= e); one broadcast + one FMA per lane per step
  if (tid < 64) {
    const int cnt = s_ctl[2];
    const double gamma = s_misc[0];
    const int c = tid;
    const bool act = c < cnt;
    const int slc = act ? s_sl[c] : 0;
    double Rrow[QN_MMAX], Rcol[QN_MMAX], Yrow[QN_MMAX], tv[QN_MMAX];
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) {
      const bool ok = act && e < cnt;
      const int sle = ok ? s_sl[e] : 0;
      Rrow[e] = ok ? s_sy[slc * M + sle] : 0.0;
      Rcol[e] = ok ? s_sy[sle * M + slc] : 0.0;
      Yrow[e] = ok ? s_yy[slc * M + sle] : 0.0;
      tv[e] = 0.0;
    }
    const double diag = act ? s_sy[slc * M + slc] : 1.0;
    double acc = act ? s_p1[slc] : 0.0;
    double tmine = 0.0;
#pragma unroll
    for (int e = QN_MMAX - 1; e >= 0; --e) {
      if (e < cnt) {
        const double te = __shfl(acc / diag, e, 64);
        tv[e] = te;
        if (c == e) tmine = te;
        if (c < e) acc -= Rrow[e] * te;
      }
    }
    acc = diag * tmine - gamma * (act ? s_p2[slc] : 0.0);
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) acc += gamma * Yrow[e] * tv[e];
    double amine = 0.0;
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) {
      if (e < cnt) {
        const double ae = __shfl(acc / diag, e, 64);
        if (c == e) amine = ae;
        if (c > e) acc -= Rcol[e] * ae;
      }
    }
    if (c < QN_MMAX) {
      cf_a[c] = 0.0;
      cf_t[c] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    if (act) {
      cf_a[slc] = amine;
      cf_t[slc] = gamma * tmine;
    }
  }
  __syncthreads();
  if (s_ctl[1]) {
    for (int i = tid; i < M * M; i += QN_T) {
      A.SY[i] = s_sy[i];
      A.YY[i] = s_yy[i];
    }
  }
  __syncthreads();
  const int status = s_ctl[0];
  const bool newp = s_ctl[1] != 0;
  const int cnt = s_ctl[2];
  const double gamma = s_misc[0];
  QN_PROBE(4);

  // ---- pass 2: store the pair, x <- xt, g <- gt, direction d = -H pg
  double p2v[2] = {0.0, 0.0};
  QN_BATCH(i0) {
    double xv[QN_U], gv[QN_U], sv[QN_U], yv[QN_U], pv[QN_U], cv[QN_U];
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      const bool ok = i < N;
      xv[u] = ok ? A.xt[i] : 0.0;
      gv[u] = ok ? A.gt[i] : 0.0;
      sv[u] = ok ? A.d[i] : 0.0;
      yv[u] = ok ? A.wb[i] : 0.0;
      pv[u] = ok ? A.pg[i] : 0.0;
      cv[u] = (ok && A.l1) ? A.l1c[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < QN_U; ++u) {
      const long i = i0 + (long)u * QN_T;
      if (i < N) {
        if (newp) {
          A.S[(long)head * N + i] = sv[u];
          A.Y[(long)head * N + i] = yv[u];
        }
        A.x[i] = xv[u];
        A.g[i] = gv[u];
      }
    }
    if (status == ST_RUNNING) {
      double hg[QN_U];
#pragma unroll
      for (int u = 0; u < QN_U; ++u) hg[u] = gamma * pv[u];
      constexpr int QN_G = 4;  // history slots whose loads are in flight together
      for (int c0 = 0; c0 < cnt; c0 += QN_G) {
        double Sv[QN_G][QN_U], Yv[QN_G][QN_U], ca[QN_G], ct[QN_G];
#pragma unroll
        for (int q = 0; q < QN_G; ++q) {
          const bool okq = c0 + q < cnt;
          const int j = okq ? s_sl[c0 + q] : 0;
          ca[q] = okq ? cf_a[j] : 0.0;
          ct[q] = okq ? cf_t[j] : 0.0;
#pragma unroll
          for (int u = 0; u < QN_U; ++u) {
            const long i = i0 + (long)u * QN_T;
            const bool ok = okq && i < N;
            Sv[q][u] = ok ? A.S[(long)j * N + i] : 0.0;
            Yv[q][u] = ok ? A.Y[(long)j * N + i] : 0.0;
          }
        }
#pragma unroll
        for (int q = 0; q < QN_G; ++q)
#pragma unroll
          for (int u = 0; u < QN_U; ++u) hg[u] += ca[q] * Sv[q][u] - ct[q] * Yv[q][u];
      }
#pragma unroll
      for (int u = 0; u < QN_U; ++u) {
        const long i = i0 + (long)u * QN_T;
        if (i < N) {
          double di = -hg[u];
          if (cv[u] > 0.0 && di * pv[u] >= 0.0) di = 0.0;
          A.d[i] = di;
          p2v[0] += pv[u] * di;
          p2v[1] += di * di;
        }
      }
    }
  }
  if (status != ST_RUNNING) {
    if (tid == 0) {
      fl[F_STATUS] = status;
      fl[F_DONE] = 1;
      fl[F_SKIPX] = 1;
    }
    return;
  }
  QN_PROBE(5);
  qn_block_sum<2>(p2v, red);
  double dg = p2v[0], dd = p2v[1];
  int cnt2 = cnt;
  if (!(dg < 0.0)) {  // not a descent direction: drop the history, steepest descent
    for (long i = tid; i < N; i += QN_T) A.d[i] = -A.pg[i];  // rare
    dg = -s_v[4];
    dd = s_v[4];
    cnt2 = 0;
    __syncthreads();
  }
  // ---- pass 3: next trial point (first iteration / after a reset: alpha = 1 / ||d||)
  alpha = cnt2 == 0 ? 1.0 / fmax(sqrt(dd), 1e-300) : 1.0;
  QN_PROBE(6);
  qn_set_trial(A, alpha);
  QN_PROBE(7);
  if (tid == 0) {
    if (cnt2 == 0) {
      fl[F_COUNT] = 0;
      A.sc[SC_GAMMA] = 1.0;
    }
    A.sc[SC_ALPHA] = alpha;
    A.sc[SC_DGINIT] = dg;
  }
}

__global__ __launch_bounds__(QN_T) void qn_step_kernel(QnArgs A) { qn_step_body(A); }

// hyper-parameter batching: one block per independent problem, args array in device memory
__global__ __launch_bounds__(QN_T) void qn_step_batch_kernel(const QnArgs* __restrict__ args) {
  const QnArgs A = args[blockIdx.x];
  qn_step_body(A);
}

SRML_API int srml_qn_step_batch(const QnArgs* args_dev, int count, hipStream_t stream) {
  if (count <= 0) return 0;
  hipLaunchKernelGGL(qn_step_batch_kernel, dim3((unsigned)count), dim3(QN_T), 0, stream, args_dev);
  return srml_status();
}

SRML_API int srml_qn_step(const QnArgs* a, hipStream_t stream) {
  if (a->M < 1 || a->M > QN_MMAX || a->N <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(qn_step_kernel, dim3(1), dim3(QN_T), 0, stream, *a);
  return srml_status();
}

SRML_API int srml_qn_max_history() { return QN_MMAX; }
SRML_API long srml_qn_args_size() { return (long)sizeof(QnArgs); }

// ------------------------------------------------------------------------------------------
// Multi-block step (one problem): the single-block step above spends ~40 us walking ~1.7 MB of
// optimiser state (x, g, pg, d, xt, gt and the S / Y history) through ONE CU. Here the same state
// machine runs as four launches over G blocks of 256 threads (element i belongs to one thread of
// one block), the kernel boundaries standing in for grid barriers:
//   K1  pass 0 (gt, penalty / directional partials); pre-step scalars snapshotted to scratch;
//   K2  every block reduces K1's partials (block order: all blocks see the same bits) and takes the
//       same line-search decision; reject -> its share of the next trial point (block 0 updates
//       the flags); accept -> pass 1 (pg, s, y and every compact-form dot product) partials;
//   K3  every block reduces them, repeats the bookkeeping / convergence test / compact-form solve
//       redundantly (identical inputs, identical results), stores its share of the new pair,
//       x <- xt, g <- gt and the direction, and leaves the p.d / d.d partials;
//   K4  reduce, descent check, its share of the next trial point; block 0 commits the optimiser
//       scalars, flags and history Gram blocks (deferred so no block of K3 reads state another
//       block of K3 already advanced).
// Same arithmetic as the single-block step except the summation order of the reductions.
// ------------------------------------------------------------------------------------------
namespace {

constexpr int MB_T = 256;
constexpr int MB_NW = MB_T / 64;
constexpr int MB_GMAX = 64;
constexpr int MB_GAMAX = 512;  // K1 partial rows: the folding K1 runs ceil(N / 32) blocks
constexpr int MB_PW = 6 + 5 * QN_MMAX + 1;  // pass-1 partials: 6 dots, 5 history products per slot, max |pg|
enum {
  S_STARTED = 0, S_ITER, S_COUNT, S_HEAD, S_LS, S_NEVAL, S_BRACKET, S_F, S_ALPHA, S_DGINIT, S_GAMMA, S_FHN, S_LOSS,
  S_ZMODE, S_ZC, S_ALPHA1,
  S_PHASE = 16, S_STATUS, S_NEWP, S_CNT, S_HD, S_GAM, S_FT, S_GINF, S_ITERN, S_FN,
  S_CF = 32,                              // cf_a[QN_MMAX] | cf_t[QN_MMAX]
  S_SL = S_CF + 2 * QN_MMAX,              // chronological slots [QN_MMAX]
  S_SY = S_SL + QN_MMAX,                  // updated SY [QN_MMAX^2] | YY [QN_MMAX^2] (committed by K4)
  S_PA = S_SY + 2 * QN_MMAX * QN_MMAX,    // K1 partials [G1][4]
  S_PB = S_PA + 4 * MB_GAMAX,             // K2 partials [G][MB_PW]
  S_PC = S_PB + MB_PW * MB_GMAX,          // K3 partials [G][2]
  S_END = S_PC + 2 * MB_GMAX
};

// block-wide sums of NV values (256 threads): thread j < NV gets total j in `out` (LDS)
template <int NV>
__device__ __forceinline__ void mb_block_sum(const double (&v)[NV], double* red, double* out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const double t = wave_sum(v[i]);
    if (lane == 0) red[i * MB_NW + wid] = t;
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < MB_NW; ++w) s += red[threadIdx.x * MB_NW + w];
    out[threadIdx.x] = s;
  }
  __syncthreads();
}

// grid totals of a [G][width] partial table (width <= MB_T) into LDS `tot` (all threads). Every
// thread of the block loads: slice s = tid / width of the blocks, eight independent loads in flight
// per thread, then an LDS combine of the slices in fixed order — the partials come from other CUs
// (L2 / fabric latency ~1 us each), so a one-thread-per-column serial loop over G blocks costs
// ~G us; this costs ~ceil(G / (8 * slices)) round trips.
__device__ __forceinline__ void mb_grid_sum(const double* part, int G, int width, double* tot, bool max_last) {
  __shared__ double gs[MB_T];
  const int t = threadIdx.x, S = MB_T / width;
  const int j = t % width, sl = t / width;
  const bool mx = max_last && j == width - 1;
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (sl < S) {
    int b = sl;
    for (; b + 7 * S < G; b += 8 * S) {
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = part[(long)(b + k * S) * width + j];
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] = mx ? fmax(a[k], v[k]) : a[k] + v[k];
    }
    for (; b < G; b += S) {
      const double v = part[(long)b * width + j];
      a[0] = mx ? fmax(a[0], v) : a[0] + v;
    }
  }
  gs[t] = mx ? fmax(fmax(fmax(a[0], a[1]), fmax(a[2], a[3])), fmax(fmax(a[4], a[5]), fmax(a[6], a[7])))
             : ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (t < width) {
    double x = gs[t];
    for (int q = 1; q < S; ++q) x = mx ? fmax(x, gs[q * width + t]) : x + gs[q * width + t];
    tot[t] = x;
  }
  __syncthreads();
}

}  // namespace

// Each kernel issues EVERY load it may need at entry (element data, history columns, grid
// partials, snapshot scalars), before its early exits and decisions: what the previous launch wrote
// comes from beyond this CU's caches (~1 us per round trip), so the kernel's time is its count of
// DEPENDENT round trips — one here, plus the boundary.

// pre-step snapshot of the flags / scalars (block 0, thread 0 of K1): later kernels read these,
// K2 / K4 rewrite the flags
struct MbSnap {
  int started, iter, count, head, ls, neval, bracket, zmode, zc;
  double f, alpha, dginit, gamma, alpha1;
};

__device__ __forceinline__ MbSnap mb_snap_load(const QnArgs& A) {
  const int* fl = A.fl;
  MbSnap q;
  q.started = fl[F_STARTED];
  q.iter = fl[F_ITER];
  q.count = fl[F_COUNT];
  q.head = fl[F_HEAD];
  q.ls = fl[F_LS];
  q.neval = fl[F_NEVAL];
  q.bracket = fl[F_BRACKET];
  q.f = A.sc[SC_F];
  q.alpha = A.sc[SC_ALPHA];
  q.dginit = A.sc[SC_DGINIT];
  q.gamma = A.sc[SC_GAMMA];
  q.zc = fl[F_ZC];
  q.zmode = q.zc ? fl[F_ZMODE] : 0;
  q.alpha1 = A.sc[SC_ALPHA1];
  return q;
}

__device__ __forceinline__ void mb_snap_store(const QnArgs& A, const MbSnap& q, double* scr) {
  scr[S_STARTED] = q.started ? 1.0 : 0.0;
  scr[S_ITER] = q.iter;
  scr[S_COUNT] = q.count;
  scr[S_HEAD] = q.head;
  scr[S_LS] = q.ls;
  scr[S_NEVAL] = q.neval;
  scr[S_BRACKET] = q.bracket;
  scr[S_F] = q.f;
  scr[S_ALPHA] = q.alpha;
  scr[S_DGINIT] = q.dginit;
  scr[S_GAMMA] = q.gamma;
  scr[S_FHN] = (A.past > 0 && q.started) ? A.fh[(q.iter + 1) % A.past] : 0.0;
  scr[S_ZMODE] = q.zmode;
  scr[S_ZC] = q.zc;
  scr[S_ALPHA1] = q.alpha1;
  scr[S_PHASE] = 0.0;
}

// pass 0 of element i from its summed evaluation value `ov`
struct MbP0In {
  double xv, l2v, l1v, dv, pgv, xo, isg;
};

__device__ __forceinline__ MbP0In mb_p0_load(const QnArgs& A, long i, bool own) {
  MbP0In e{0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0};
  if (own) {
    e.xv = A.xt[i];
    e.l2v = A.l2[i];
    e.l1v = A.l1c[i];
    e.dv = A.d[i];
    e.pgv = A.pg[i];
    e.xo = A.x[i];
    if (i < A.Kn) e.isg = A.isg[i % A.n];
  }
  return e;
}

__device__ __forceinline__ void mb_p0(const QnArgs& A, long i, bool own, const MbP0In& e, double ov, double (&p0)[4]) {
  if (!own) return;
  const double gi = ov * A.inv_m * e.isg + e.l2v * e.xv;
  A.gt[i] = gi;
  p0[0] = e.l2v * e.xv * e.xv;
  p0[1] = e.l1v * fabs(e.xv);
  p0[2] = gi * e.dv;
  p0[3] = e.pgv * (e.xv - e.xo);
}

__global__ __launch_bounds__(MB_T) void qn_mb1_kernel(QnArgs A, double* __restrict__ scr) {
  __shared__ double red[4 * MB_NW], tot[4];
  const bool first = blockIdx.x == 0 && threadIdx.x == 0;
  const long i = (long)blockIdx.x * MB_T + threadIdx.x;
  const bool own = i < A.N;
  const int done = A.fl[F_DONE];
  MbSnap q{};
  double loss = 0.0;
  if (first) {
    q = mb_snap_load(A);
    loss = A.out[A.Kn + A.K];
  }
  const MbP0In e = mb_p0_load(A, i, own);
  const double ov = own ? A.out[i] : 0.0;
  if (done) {
    if (first) scr[S_PHASE] = 0.0;  // K3 / K4 must not act on a stale phase
    return;
  }
  if (first) {
    mb_snap_store(A, q, scr);
    scr[S_LOSS] = loss;
  }
  double p0[4] = {0.0, 0.0, 0.0, 0.0};
  mb_p0(A, i, own, e, ov, p0);
  if (own && i < A.Kn + A.K) A.out[i] = 0.0;  // this element's evaluation sum is consumed
  mb_block_sum<4>(p0, red, tot);
  if (threadIdx.x < 4) scr[S_PA + blockIdx.x * 4 + threadIdx.x] = tot[threadIdx.x];
}

// trial point of element i: t = x + alpha d, projected onto x's orthant for L1 coordinates
__device__ __forceinline__ void mb_trial(const QnArgs& A, long i, double xv, double dv, double pv, double cv,
                                         double isg, double alpha) {
  double t = xv + alpha * dv;
  if (A.l1 && cv > 0.0) {
    const double orth = xv != 0.0 ? (xv > 0.0 ? 1.0 : -1.0) : (pv < 0.0 ? 1.0 : (pv > 0.0 ? -1.0 : 0.0));
    if (t * orth <= 0.0) t = 0.0;
  }
  A.xt[i] = t;
  A.wb[i] = t * isg;
}

__global__ __launch_bounds__(MB_T) void qn_mb2_kernel(QnArgs A, double* __restrict__ scr, int ga) {
  __shared__ double red[MB_PW * MB_NW], p0[4];
  int* fl = A.fl;
  const int M = A.M;
  const long N = A.N;
  const long i = (long)blockIdx.x * MB_T + threadIdx.x;
  const bool own = i < N;
  const bool first = blockIdx.x == 0 && threadIdx.x == 0;
  // ---- every load up front
  const int done = fl[F_DONE];
  const bool started = scr[S_STARTED] != 0.0;
  const double f = scr[S_F], dginit = scr[S_DGINIT], alpha0 = scr[S_ALPHA], loss = scr[S_LOSS];
  const bool bracket = scr[S_BRACKET] != 0.0;
  const int pre_ls = (int)scr[S_LS], pre_neval = (int)scr[S_NEVAL];
  const bool zc = scr[S_ZC] != 0.0;
  const int zmode = (int)scr[S_ZMODE];
  const double alpha1 = scr[S_ALPHA1];
  double xt = 0.0, gt = 0.0, xo = 0.0, go = 0.0, cv = 0.0, dv = 0.0, pv = 0.0, isg = 1.0;
  double Sv[QN_MMAX], Yv[QN_MMAX];
  if (own) {
    xt = A.xt[i];
    gt = A.gt[i];
    xo = A.x[i];
    go = A.g[i];
    cv = A.l1c[i];
    dv = A.d[i];
    pv = A.pg[i];
    if (i < A.Kn) isg = A.isg[i % A.n];
  }
#pragma unroll
  for (int j = 0; j < QN_MMAX; ++j) {
    Sv[j] = (own && j < M) ? A.S[(long)j * N + i] : 0.0;
    Yv[j] = (own && j < M) ? A.Y[(long)j * N + i] : 0.0;
  }
  if (done) return;
  mb_grid_sum(scr + S_PA, ga, 4, p0, false);  // ga: K1's block count
  double alpha = alpha0;
  const double ft = loss * A.inv_m + 0.5 * p0[0] + p0[1];
  if (first)  // the loss sum (read from the snapshot) and bias sums without a parameter (no intercept)
    for (long j = N; j < A.Kn + A.K + 1; ++j) A.out[j] = 0.0;
  if (first && zc && zmode == 1) fl[F_NCHEAP] += 1;
  if (started) {
    bool accept = true;
    double width = 1.0;
    if (zc && zmode == 2 && isfinite(ft)) {
      // a margins-only trial passed the test at this point: this full evaluation supplies its
      // gradient (and the exact loss), nothing is re-tested
    } else if (!isfinite(ft)) {
      accept = false;
      width = 0.5;
    } else {
      const double dgtest = A.l1 ? p0[3] : alpha * dginit;
      if (ft > f + A.c1 * dgtest) {
        accept = false;
        const double den = 2.0 * (ft - f - dgtest);
        width = den > 0.0 ? -dgtest / den : 0.5;
        width = isfinite(width) ? fmin(0.5, fmax(0.1, width)) : 0.5;
      } else if (A.wolfe && !A.l1 && !bracket && p0[2] < A.c2 * dginit) {
        accept = false;
        width = 2.1;
      }
    }
    if (!accept) {
      const int ls = pre_ls + 1;
      if (ls >= A.max_ls) {
        if (first) {
          fl[F_LS] = ls;
          fl[F_NEVAL] = pre_neval + 1;
          fl[F_STATUS] = ST_LS_FAIL;
          fl[F_DONE] = 1;
          fl[F_SKIPX] = 1;
        }
        return;
      }
      alpha *= width;
      if (own) mb_trial(A, i, xo, dv, pv, cv, isg, alpha);
      if (first) {
        fl[F_LS] = ls;
        fl[F_NEVAL] = pre_neval + 1;
        if (width < 1.0) fl[F_BRACKET] = 1;
        A.sc[SC_ALPHA] = alpha;
        if (zc && isfinite(ft)) {
          // the rejected full evaluation's margins (at step alpha0) become z1; later trials of this
          // search are margins-only evaluations at beta = alpha / alpha1
          const double a1 = zmode == 0 ? alpha0 : alpha1;
          A.sc[SC_ALPHA1] = a1;
          A.sc[SC_BETA] = alpha / a1;
          fl[F_ZMODE] = 1;
          fl[F_SKIPX] = 1;
        } else if (zc) {
          fl[F_ZMODE] = 0;  // a non-finite loss: no trusted margins, the next trial runs in full
          fl[F_SKIPX] = 0;
        }
      }
      return;
    }
    if (zc && zmode == 1) {  // accepted on margins only: evaluate the same point in full next
      if (first) {
        fl[F_NEVAL] = pre_neval + 1;
        fl[F_ZMODE] = 2;
        fl[F_SKIPX] = 0;
      }
      return;
    }
  }
  if (first) {
    scr[S_PHASE] = 1.0;
    scr[S_FT] = ft;
    if (zc) {  // this full evaluation's margins (the other buffer) are the new accepted point's
      fl[F_ZSEL] ^= 1;
      fl[F_ZMODE] = 0;
      fl[F_SKIPX] = 0;
    }
  }
  // accepted: pass 1 partials of this block's elements
  double v[MB_PW];
#pragma unroll
  for (int j = 0; j < MB_PW; ++j) v[j] = 0.0;
  if (own) {
    const double sx = started ? xt - xo : 0.0;
    const double yx = started ? gt - go : 0.0;
    const double pgi = pseudo_grad(xt, gt, A.l1 ? cv : 0.0);
    A.pg[i] = pgi;
    A.d[i] = sx;
    A.wb[i] = yx;
    v[0] = sx * yx;
    v[1] = yx * yx;
    v[2] = sx * pgi;
    v[3] = yx * pgi;
    v[4] = pgi * pgi;
    v[MB_PW - 1] = fabs(pgi);
#pragma unroll
    for (int j = 0; j < QN_MMAX; ++j) {
      v[6 + j] = sx * Yv[j];
      v[6 + QN_MMAX + j] = Sv[j] * yx;
      v[6 + 2 * QN_MMAX + j] = yx * Yv[j];
      v[6 + 3 * QN_MMAX + j] = Sv[j] * pgi;
      v[6 + 4 * QN_MMAX + j] = Yv[j] * pgi;
    }
  }
  // block sums (the last entry is a max); history slots >= M are zero and skipped
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < MB_PW - 1; ++j) {
    const bool live = j < 6 || ((j - 6) % QN_MMAX) < M;
    const double t = live ? wave_sum(v[j]) : 0.0;
    if (lane == 0) red[j * MB_NW + wid] = t;
    __builtin_amdgcn_sched_barrier(0);
  }
  {
    double mx = v[MB_PW - 1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) red[(MB_PW - 1) * MB_NW + wid] = mx;
  }
  __syncthreads();
  if (threadIdx.x < MB_PW) {
    const int j = threadIdx.x;
    double s = 0.0;
    for (int w = 0; w < MB_NW; ++w)
      s = j == MB_PW - 1 ? fmax(s, red[j * MB_NW + w]) : s + red[j * MB_NW + w];
    scr[S_PB + (long)blockIdx.x * MB_PW + j] = s;
  }
}

__global__ __launch_bounds__(MB_T) void qn_mb3_kernel(QnArgs A, double* __restrict__ scr) {
  __shared__ double tot[MB_PW], red[2 * MB_NW], t2[2];
  __shared__ double s_sy[QN_MMAX * QN_MMAX], s_yy[QN_MMAX * QN_MMAX], s_p1[QN_MMAX], s_p2[QN_MMAX];
  __shared__ double cf_a[QN_MMAX], cf_t[QN_MMAX], s_misc[2];
  __shared__ int s_sl[QN_MMAX], s_ctl[4];
  const int G = gridDim.x, M = A.M, tid = threadIdx.x;
  const long N = A.N;
  const long i = (long)blockIdx.x * MB_T + tid;
  const bool own = i < N;
  // ---- every load up front
  const double phase = scr[S_PHASE];
  const bool started = scr[S_STARTED] != 0.0;
  const int pre_count = (int)scr[S_COUNT], head = (int)scr[S_HEAD], pre_iter = (int)scr[S_ITER];
  const double pre_gamma = scr[S_GAMMA], fn = scr[S_FT], fhn = scr[S_FHN];
  // K4's block 0 commits the updated blocks: every block reads the old ones here
  const double sy0 = tid < M * M ? A.SY[tid] : 0.0, yy0 = tid < M * M ? A.YY[tid] : 0.0;
  double xt = 0.0, gt = 0.0, sv = 0.0, yv = 0.0, pv = 0.0, cv = 0.0;
  double Sv[QN_MMAX], Yv[QN_MMAX];
  if (own) {
    xt = A.xt[i];
    gt = A.gt[i];
    sv = A.d[i];
    yv = A.wb[i];
    pv = A.pg[i];
    cv = A.l1c[i];
  }
#pragma unroll
  for (int j = 0; j < QN_MMAX; ++j) {
    Sv[j] = (own && j < M) ? A.S[(long)j * N + i] : 0.0;
    Yv[j] = (own && j < M) ? A.Y[(long)j * N + i] : 0.0;
  }
  if (phase != 1.0) return;
  if (tid < M * M) {
    s_sy[tid] = sy0;
    s_yy[tid] = yy0;
  }
  mb_grid_sum(scr + S_PB, G, MB_PW, tot, true);  // (its barriers also publish s_sy / s_yy)
  if (tid == 0) {
    int cnt = pre_count, hd = head, status = ST_RUNNING;
    double gamma = started ? pre_gamma : 1.0;
    for (int j = 0; j < M; ++j) {
      s_p1[j] = tot[6 + 3 * QN_MMAX + j];
      s_p2[j] = tot[6 + 4 * QN_MMAX + j];
    }
    const double ys = tot[0], yy = tot[1];
    const bool newp = started && yy > 0.0 && ys > 1e-10 * yy;
    if (newp) {
      const int h = hd;
      for (int j = 0; j < M; ++j) {
        if (j == h) continue;
        s_sy[h * M + j] = tot[6 + j];
        s_sy[j * M + h] = tot[6 + QN_MMAX + j];
        s_yy[h * M + j] = tot[6 + 2 * QN_MMAX + j];
        s_yy[j * M + h] = tot[6 + 2 * QN_MMAX + j];
      }
      s_sy[h * M + h] = ys;
      s_yy[h * M + h] = yy;
      s_p1[h] = tot[2];
      s_p2[h] = tot[3];
      hd = (h + 1) % M;
      cnt = cnt < M ? cnt + 1 : M;
      gamma = ys / yy;
    }
    const double ginf = tot[MB_PW - 1];
    const int iter = pre_iter + (started ? 1 : 0);
    const double fmag = fmax(fabs(fn), A.tol);
    if (ginf <= A.tol * fmag) status = ST_CONV_GRAD;
    if (A.past > 0 && status == ST_RUNNING && started && iter >= A.past && fabs(fhn - fn) <= A.delta * fmag)
      status = ST_CONV_F;
    if (status == ST_RUNNING && iter >= A.max_iter) status = ST_MAXITER;
    for (int c = 0; c < cnt; ++c) s_sl[c] = (hd - cnt + c + 2 * M) % M;
    s_ctl[0] = status;
    s_ctl[1] = newp ? 1 : 0;
    s_ctl[2] = cnt;
    s_ctl[3] = hd;
    s_misc[0] = gamma;
    s_misc[1] = ginf;
    if (blockIdx.x == 0) {  // the commit record for K4
      scr[S_STATUS] = status;
      scr[S_NEWP] = newp ? 1.0 : 0.0;
      scr[S_CNT] = cnt;
      scr[S_HD] = hd;
      scr[S_GAM] = gamma;
      scr[S_GINF] = ginf;
      scr[S_ITERN] = iter;
      scr[S_FN] = fn;
    }
  }
  __syncthreads();
  // compact-form coefficients (wave 0, as the single-block step)
  if (tid < 64) {
    const int cnt = s_ctl[2];
    const double gamma = s_misc[0];
    const int c = tid;
    const bool act = c < cnt;
    const int slc = act ? s_sl[c] : 0;
    double Rrow[QN_MMAX], Rcol[QN_MMAX], Yrow[QN_MMAX], tv[QN_MMAX];
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) {
      const bool ok = act && e < cnt;
      const int sle = ok ? s_sl[e] : 0;
      Rrow[e] = ok ? s_sy[slc * M + sle] : 0.0;
      Rcol[e] = ok ? s_sy[sle * M + slc] : 0.0;
      Yrow[e] = ok ? s_yy[slc * M + sle] : 0.0;
      tv[e] = 0.0;
    }
    const double diag = act ? s_sy[slc * M + slc] : 1.0;
    double acc = act ? s_p1[slc] : 0.0;
    double tmine = 0.0;
#pragma unroll
    for (int e = QN_MMAX - 1; e >= 0; --e) {
      if (e < cnt) {
        const double te = __shfl(acc / diag, e, 64);
        tv[e] = te;
        if (c == e) tmine = te;
        if (c < e) acc -= Rrow[e] * te;
      }
    }
    acc = diag * tmine - gamma * (act ? s_p2[slc] : 0.0);
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) acc += gamma * Yrow[e] * tv[e];
    double amine = 0.0;
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) {
      if (e < cnt) {
        const double ae = __shfl(acc / diag, e, 64);
        if (c == e) amine = ae;
        if (c > e) acc -= Rcol[e] * ae;
      }
    }
    if (c < QN_MMAX) {
      cf_a[c] = 0.0;
      cf_t[c] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    if (act) {
      cf_a[slc] = amine;
      cf_t[slc] = gamma * tmine;
    }
  }
  __syncthreads();
  const int status = s_ctl[0];
  const bool newp = s_ctl[1] != 0;
  const double gamma = s_misc[0];
  if (blockIdx.x == 0 && newp)  // staged for K4 (other blocks of this launch still read A.SY / A.YY)
    for (int k = tid; k < M * M; k += MB_T) {
      scr[S_SY + k] = s_sy[k];
      scr[S_SY + QN_MMAX * QN_MMAX + k] = s_yy[k];
    }
  // pass 2: store the pair, x <- xt, g <- gt, direction (inactive slots have zero coefficients)
  double p2v[2] = {0.0, 0.0};
  if (own) {
    if (newp) {
      A.S[(long)head * N + i] = sv;
      A.Y[(long)head * N + i] = yv;
    }
    A.x[i] = xt;
    A.g[i] = gt;
    if (status == ST_RUNNING) {
      double hg = gamma * pv;
#pragma unroll
      for (int j = 0; j < QN_MMAX; ++j) {
        if (j < M) {
          const bool fresh = newp && j == head;  // the pair stored just above
          hg += cf_a[j] * (fresh ? sv : Sv[j]) - cf_t[j] * (fresh ? yv : Yv[j]);
        }
      }
      double di = -hg;
      if (A.l1 && cv > 0.0 && di * pv >= 0.0) di = 0.0;
      A.d[i] = di;
      p2v[0] = pv * di;
      p2v[1] = di * di;
    }
  }
  mb_block_sum<2>(p2v, red, t2);
  if (tid < 2) scr[S_PC + blockIdx.x * 2 + tid] = t2[tid];
}

__global__ __launch_bounds__(MB_T) void qn_mb4_kernel(QnArgs A, double* __restrict__ scr) {
  __shared__ double p2[2], pbt[MB_PW];
  const int G = gridDim.x, M = A.M, tid = threadIdx.x;
  const bool first = blockIdx.x == 0 && tid == 0;
  const long i = (long)blockIdx.x * MB_T + tid;
  const bool own = i < A.N;
  int* fl = A.fl;
  // ---- every load up front
  const double phase = scr[S_PHASE];
  const int status = (int)scr[S_STATUS];
  const bool newp = scr[S_NEWP] != 0.0;
  const int cnt0 = (int)scr[S_CNT];
  double sy = 0.0, yy = 0.0;
  if (blockIdx.x == 0 && tid < M * M) {
    sy = scr[S_SY + tid];
    yy = scr[S_SY + QN_MMAX * QN_MMAX + tid];
  }
  double xv = 0.0, dv = 0.0, pv = 0.0, cv = 0.0, isg = 1.0;
  if (own) {
    xv = A.x[i];
    dv = A.d[i];
    pv = A.pg[i];
    cv = A.l1c[i];
    if (i < A.Kn) isg = A.isg[i % A.n];
  }
  if (phase != 1.0) return;
  if (blockIdx.x == 0) {  // commit the step's history blocks and scalars
    if (newp && tid < M * M) {
      A.SY[tid] = sy;
      A.YY[tid] = yy;
    }
    if (tid == 0) {
      const int iter = (int)scr[S_ITERN];
      if (A.past > 0) A.fh[iter % A.past] = scr[S_FN];
      fl[F_ITER] = iter;
      fl[F_HEAD] = (int)scr[S_HD];
      fl[F_COUNT] = cnt0;
      fl[F_NEVAL] = (int)scr[S_NEVAL] + 1;
      fl[F_LS] = 0;
      fl[F_BRACKET] = 0;
      fl[F_STARTED] = 1;
      A.sc[SC_F] = scr[S_FN];
      A.sc[SC_GAMMA] = scr[S_GAM];
      A.sc[SC_GINF] = scr[S_GINF];
    }
  }
  if (status != ST_RUNNING) {
    if (first) {
      fl[F_STATUS] = status;
      fl[F_DONE] = 1;
      fl[F_SKIPX] = 1;
    }
    return;
  }
  mb_grid_sum(scr + S_PC, G, 2, p2, false);
  double dg = p2[0], dd = p2[1];
  int cnt2 = cnt0;
  if (!(dg < 0.0)) {  // not a descent direction: drop the history, steepest descent (rare)
    mb_grid_sum(scr + S_PB, G, MB_PW, pbt, true);  // pg.pg is in the K2 partials
    const double pp = pbt[4];
    dv = -pv;
    if (own) A.d[i] = dv;
    dg = -pp;
    dd = pp;
    cnt2 = 0;
  }
  const double alpha = cnt2 == 0 ? 1.0 / fmax(sqrt(dd), 1e-300) : 1.0;
  if (own) mb_trial(A, i, xv, dv, pv, cv, isg, alpha);
  if (first) {
    if (cnt2 == 0) {
      fl[F_COUNT] = 0;
      A.sc[SC_GAMMA] = 1.0;
    }
    A.sc[SC_ALPHA] = alpha;
    A.sc[SC_DGINIT] = dg;
  }
}

// doubles of scratch the multi-block step needs (independent of N)
SRML_API long srml_qn_mb_scratch() { return (long)S_END; }

// One optimiser step as four G-block launches (G = ceil(N / 256) <= 64; larger problems use the
// single-block step). `scratch`: srml_qn_mb_scratch() doubles owned by this problem.
SRML_API int srml_qn_step_mb(const QnArgs* a, double* scratch, hipStream_t stream) {
  if (a->M < 1 || a->M > QN_MMAX || a->N <= 0 || !scratch) return (int)hipErrorInvalidValue;
  const long G = (a->N + MB_T - 1) / MB_T;
  if (G > MB_GMAX) return srml_qn_step(a, stream);
  const dim3 grid((unsigned)G), blk(MB_T);
  hipLaunchKernelGGL(qn_mb1_kernel, grid, blk, 0, stream, *a, scratch);
  hipLaunchKernelGGL(qn_mb2_kernel, grid, blk, 0, stream, *a, scratch, (int)G);
  hipLaunchKernelGGL(qn_mb3_kernel, grid, blk, 0, stream, *a, scratch);
  hipLaunchKernelGGL(qn_mb4_kernel, grid, blk, 0, stream, *a, scratch);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Fused step: the whole optimiser step as ONE launch of G blocks (32 elements each) with three
// software grid barriers (arrive counter + generation word in the scratch, agent-scope release /
// acquire; G <= 512 blocks of 256 threads are co-resident on 256 CUs, and the wait is bounded by
// wall-clock: a barrier that does not complete in ~1 s marks the step failed instead of hanging).
// In front of pass 0 it can FOLD the binary evaluation's fp32 partial gradient rows itself
// (`fws`: the fused binary kernel's per-block rows, single-rank fits), so an evaluation + step is
// two launches: every kernel costs ~5 us of dispatch / ramp on its own, which the four-launch
// step and a separate fold kernel paid six times per evaluation.
// ------------------------------------------------------------------------------------------
namespace {

constexpr int FU_E = 32;       // elements per block
constexpr int FU_GMAX = 512;   // N <= 16384
constexpr int ST_BARRIER = 5;  // status: a grid barrier timed out (never expected)
enum {
  F_PA = S_END,                        // [G][6] pass-0 partials (+ folded loss, + folded bias grad)
  F_PB = F_PA + 6 * FU_GMAX,           // [G][MB_PW] pass-1 partials
  F_PC = F_PB + MB_PW * FU_GMAX,       // [G][2]
  F_BAR = F_PC + 2 * FU_GMAX,          // 2 x u32 (arrive, generation) in one double slot
  F_END = F_BAR + 2
};

__device__ __forceinline__ bool fu_barrier(double* scr, unsigned G) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* arrive = reinterpret_cast<unsigned*>(scr + F_BAR);
    unsigned* gen = arrive + 1;
    const unsigned my = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();  // release this block's partials
    int ok = 1;
    if (atomicAdd(arrive, 1u) == G - 1) {
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == my) {
        if (wall_clock64() - t0 > 100000000LL) {  // ~1 s at the 100 MHz constant clock
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __threadfence();  // acquire the other blocks' partials
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

}  // namespace

// Fold of the binary evaluation's fp32 partial gradient rows for this block's FU_E elements
// (columns blockIdx.x * FU_E ...): 8 lanes x float4 per row, 32 row groups, 8 rows in flight per
// thread; the bias element and the loss are the trailing doubles of every row (summed by the
// block owning element Kn / the last block). Returns the element's sum in `oval` and the block's
// loss contribution in `lpart`.
__device__ __forceinline__ void fu_fold_block(const QnArgs& A, const float* __restrict__ fws, int parts, long wst,
                                              double (*fold)[33], double* red, bool own, long i, unsigned G,
                                              double& oval, double& lpart) {
  const int tid = threadIdx.x;
  const int q = tid & 7, rg = tid >> 3;  // 8 lanes x float4 = 32 columns, 32 row groups
  const long c = (long)blockIdx.x * FU_E + 4 * q;
  // the bias gradient (element Kn, owned by one block) and the loss (block G - 1): trailing
  // doubles of every row, summed over the block's 256 threads; issued first, all in flight
  const bool has_bias = A.K == 1 && A.Kn < A.N && (long)blockIdx.x == A.Kn / FU_E;
  const bool has_loss = blockIdx.x == G - 1;
  double gb = 0.0, ls = 0.0;
  if (has_bias || has_loss)
    for (int p = tid; p < parts; p += 4 * MB_T) {
      double t0[4], t1[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int pk = p + k * MB_T;
        const double* pd = reinterpret_cast<const double*>(fws + (long)(pk < parts ? pk : 0) * wst + wst - 4);
        t0[k] = pk < parts ? pd[0] : 0.0;
        t1[k] = pk < parts ? pd[1] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        gb += t0[k];
        ls += t1[k];
      }
    }
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (c < A.Kn) {
    int p = rg;
    for (; p + 32 * 11 < parts; p += 32 * 12) {  // 12 rows in flight per thread
      floatx4 v[12];
#pragma unroll
      for (int j = 0; j < 12; ++j)
        v[j] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(fws + (long)(p + 32 * j) * wst + c));
#pragma unroll
      for (int j = 0; j < 12; ++j) { a0 += v[j][0]; a1 += v[j][1]; a2 += v[j][2]; a3 += v[j][3]; }
    }
    for (; p < parts; p += 32) {
      const floatx4 v = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(fws + (long)p * wst + c));
      a0 += v[0]; a1 += v[1]; a2 += v[2]; a3 += v[3];
    }
  }
  fold[rg][4 * q] = a0;
  fold[rg][4 * q + 1] = a1;
  fold[rg][4 * q + 2] = a2;
  fold[rg][4 * q + 3] = a3;
  const double sums[2] = {has_bias ? gb : 0.0, has_loss ? ls : 0.0};
  double tv2[2];
  {
    const int lane = tid & 63, wid = tid >> 6;
    for (int k = 0; k < 2; ++k) {
      const double t = wave_sum(sums[k]);
      if (lane == 0) red[k * MB_NW + wid] = t;
    }
  }
  __syncthreads();
  tv2[0] = (red[0] + red[1]) + (red[2] + red[3]);
  tv2[1] = (red[MB_NW] + red[MB_NW + 1]) + (red[MB_NW + 2] + red[MB_NW + 3]);
  if (own) {
    if (i < A.Kn) {
      double s = 0.0;
#pragma unroll
      for (int g2 = 0; g2 < 32; ++g2) s += fold[g2][tid];
      oval = s;
    } else {
      oval = tv2[0];  // the bias element
    }
  }
  lpart = tv2[1];
  __syncthreads();
}

__global__ __launch_bounds__(MB_T) void qn_fused_kernel(QnArgs A, double* __restrict__ scr,
                                                        const float* __restrict__ fws, int parts, long wst) {
  __shared__ double red[MB_PW * MB_NW], tot[MB_PW], fold[32][33];
  __shared__ double s_sy[QN_MMAX * QN_MMAX], s_yy[QN_MMAX * QN_MMAX], s_p1[QN_MMAX], s_p2[QN_MMAX];
  __shared__ double cf_a[QN_MMAX], cf_t[QN_MMAX], s_misc[2];
  __shared__ int s_sl[QN_MMAX], s_ctl[4];
  int* fl = A.fl;
  if (fl[F_DONE]) return;  // uniform: no block reaches a barrier
  const unsigned G = gridDim.x;
  const int tid = threadIdx.x, M = A.M;
  const long N = A.N;
  const long i = (long)blockIdx.x * FU_E + tid;  // this thread's element (tid < FU_E)
  const bool own = tid < FU_E && i < N;
  const bool first = blockIdx.x == 0 && tid == 0;
  // ---- pre-step scalars (every block reads them here; only block 0 rewrites them, after the
  //      last barrier it takes)
  const bool started = fl[F_STARTED] != 0;
  const int pre_iter = fl[F_ITER], count = fl[F_COUNT], head = fl[F_HEAD], pre_ls = fl[F_LS];
  const int pre_neval = fl[F_NEVAL];
  const bool bracket = fl[F_BRACKET] != 0;
  const double f = A.sc[SC_F], dginit = A.sc[SC_DGINIT], pre_gamma = A.sc[SC_GAMMA];
  double alpha = A.sc[SC_ALPHA];
  const double pre_fh_next = (A.past > 0 && started) ? A.fh[(pre_iter + 1) % A.past] : 0.0;
  // ---- this block's gradient sums: folded from the evaluation's partial rows, or from `out`
  double oval = 0.0, lpart = 0.0;
  if (fws) {
    fu_fold_block(A, fws, parts, wst, fold, red, own, i, G, oval, lpart);
  } else {
    if (own) {
      oval = A.out[i];
      A.out[i] = 0.0;  // consumed
    }
    if (first) lpart = A.out[A.Kn + A.K];  // the loss sum; zeroed by block 0 after the barrier
  }
  // ---- pass 0
  double p0[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  if (own) {
    const double xv = A.xt[i];
    const double gi = oval * A.inv_m * (i < A.Kn ? A.isg[i % A.n] : 1.0) + A.l2[i] * xv;
    A.gt[i] = gi;
    p0[0] = A.l2[i] * xv * xv;
    p0[1] = A.l1c[i] * fabs(xv);
    p0[2] = gi * A.d[i];
    p0[3] = A.pg[i] * (xv - A.x[i]);
  }
  if (tid == 0) p0[4] = lpart;
  mb_block_sum<5>(p0, red, tot);
  if (tid < 5) scr[F_PA + blockIdx.x * 6 + tid] = tot[tid];
  if (!fu_barrier(scr, G)) {
    if (first) { fl[F_STATUS] = ST_BARRIER; fl[F_DONE] = 1; }
    return;
  }
  mb_grid_sum(scr + F_PA, (int)G, 6, red, false);
  const double q0 = red[0], q1 = red[1], q2 = red[2], q3 = red[3], lossv = red[4];
  __syncthreads();
  const double ft = lossv * A.inv_m + 0.5 * q0 + q1;
  if (first && !fws)  // the loss sum (read before the barrier) and bias sums without a parameter
    for (long j = N; j < A.Kn + A.K + 1; ++j) A.out[j] = 0.0;
  if (started) {
    bool accept = true;
    double width = 1.0;
    if (!isfinite(ft)) {
      accept = false;
      width = 0.5;
    } else {
      const double dgtest = A.l1 ? q3 : alpha * dginit;
      if (ft > f + A.c1 * dgtest) {
        accept = false;
        const double den = 2.0 * (ft - f - dgtest);
        width = den > 0.0 ? -dgtest / den : 0.5;
        width = isfinite(width) ? fmin(0.5, fmax(0.1, width)) : 0.5;
      } else if (A.wolfe && !A.l1 && !bracket && q2 < A.c2 * dginit) {
        accept = false;
        width = 2.1;
      }
    }
    if (!accept) {
      const int ls = pre_ls + 1;
      if (ls >= A.max_ls) {
        if (first) {
          fl[F_LS] = ls;
          fl[F_NEVAL] = pre_neval + 1;
          fl[F_STATUS] = ST_LS_FAIL;
          fl[F_DONE] = 1;
        }
        return;
      }
      alpha *= width;
      if (own) {  // next trial point
        const double xv = A.x[i], dv = A.d[i];
        double t = xv + alpha * dv;
        if (A.l1 && A.l1c[i] > 0.0) {
          const double pv = A.pg[i];
          const double orth = xv != 0.0 ? (xv > 0.0 ? 1.0 : -1.0) : (pv < 0.0 ? 1.0 : (pv > 0.0 ? -1.0 : 0.0));
          if (t * orth <= 0.0) t = 0.0;
        }
        A.xt[i] = t;
        A.wb[i] = t * (i < A.Kn ? A.isg[i % A.n] : 1.0);
      }
      if (first) {
        fl[F_LS] = ls;
        fl[F_NEVAL] = pre_neval + 1;
        if (width < 1.0) fl[F_BRACKET] = 1;
        A.sc[SC_ALPHA] = alpha;
      }
      return;
    }
  }
  // ---- accepted: pass 1 partials (own elements)
  {
    double v[MB_PW];
#pragma unroll
    for (int j = 0; j < MB_PW; ++j) v[j] = 0.0;
    if (own) {
      const double xv = A.xt[i], gv = A.gt[i];
      const double sx = started ? xv - A.x[i] : 0.0;
      const double yx = started ? gv - A.g[i] : 0.0;
      const double pgi = pseudo_grad(xv, gv, A.l1 ? A.l1c[i] : 0.0);
      A.pg[i] = pgi;
      A.d[i] = sx;
      A.wb[i] = yx;
      v[0] = sx * yx;
      v[1] = yx * yx;
      v[2] = sx * pgi;
      v[3] = yx * pgi;
      v[4] = pgi * pgi;
      v[MB_PW - 1] = fabs(pgi);
#pragma unroll
      for (int j = 0; j < QN_MMAX; ++j) {
        if (j < M) {
          const double Sj = A.S[(long)j * N + i], Yj = A.Y[(long)j * N + i];
          v[6 + j] = sx * Yj;
          v[6 + QN_MMAX + j] = Sj * yx;
          v[6 + 2 * QN_MMAX + j] = yx * Yj;
          v[6 + 3 * QN_MMAX + j] = Sj * pgi;
          v[6 + 4 * QN_MMAX + j] = Yj * pgi;
        }
      }
    }
    // only wave 0 holds elements (FU_E = 32 < 64): the wave sum is the block sum
    const int lane = tid & 63;
    if (tid < 64) {
#pragma unroll
      for (int j = 0; j < MB_PW - 1; ++j) {
        const double t = wave_sum(v[j]);
        if (lane == 0) scr[F_PB + (long)blockIdx.x * MB_PW + j] = t;
        __builtin_amdgcn_sched_barrier(0);
      }
      double mx = v[MB_PW - 1];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
      if (lane == 0) scr[F_PB + (long)blockIdx.x * MB_PW + MB_PW - 1] = mx;
    }
  }
  for (int k = tid; k < M * M; k += MB_T) {  // old history blocks, before anyone commits new ones
    s_sy[k] = A.SY[k];
    s_yy[k] = A.YY[k];
  }
  if (!fu_barrier(scr, G)) {
    if (first) { fl[F_STATUS] = ST_BARRIER; fl[F_DONE] = 1; }
    return;
  }
  mb_grid_sum(scr + F_PB, G, MB_PW, tot, true);
  if (tid == 0) {
    int cnt = count, hd = head, status = ST_RUNNING;
    double gamma = started ? pre_gamma : 1.0;
    for (int j = 0; j < M; ++j) {
      s_p1[j] = tot[6 + 3 * QN_MMAX + j];
      s_p2[j] = tot[6 + 4 * QN_MMAX + j];
    }
    const double ys = tot[0], yy = tot[1];
    const bool newp = started && yy > 0.0 && ys > 1e-10 * yy;
    if (newp) {
      const int h = hd;
      for (int j = 0; j < M; ++j) {
        if (j == h) continue;
        s_sy[h * M + j] = tot[6 + j];
        s_sy[j * M + h] = tot[6 + QN_MMAX + j];
        s_yy[h * M + j] = tot[6 + 2 * QN_MMAX + j];
        s_yy[j * M + h] = tot[6 + 2 * QN_MMAX + j];
      }
      s_sy[h * M + h] = ys;
      s_yy[h * M + h] = yy;
      s_p1[h] = tot[2];
      s_p2[h] = tot[3];
      hd = (h + 1) % M;
      cnt = cnt < M ? cnt + 1 : M;
      gamma = ys / yy;
    }
    const double ginf = tot[MB_PW - 1];
    const int iter = pre_iter + (started ? 1 : 0);
    const double fmag = fmax(fabs(ft), A.tol);
    if (ginf <= A.tol * fmag) status = ST_CONV_GRAD;
    if (A.past > 0 && status == ST_RUNNING && started && iter >= A.past && fabs(pre_fh_next - ft) <= A.delta * fmag)
      status = ST_CONV_F;
    if (status == ST_RUNNING && iter >= A.max_iter) status = ST_MAXITER;
    for (int c = 0; c < cnt; ++c) s_sl[c] = (hd - cnt + c + 2 * M) % M;
    s_ctl[0] = status;
    s_ctl[1] = newp ? 1 : 0;
    s_ctl[2] = cnt;
    s_ctl[3] = hd;
    s_misc[0] = gamma;
    s_misc[1] = ginf;
  }
  __syncthreads();
  if (tid < 64) {  // compact-form coefficients (wave 0)
    const int cnt = s_ctl[2];
    const double gamma = s_misc[0];
    const int c = tid;
    const bool act = c < cnt;
    const int slc = act ? s_sl[c] : 0;
    double Rrow[QN_MMAX], Rcol[QN_MMAX], Yrow[QN_MMAX], tv[QN_MMAX];
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) {
      const bool ok = act && e < cnt;
      const int sle = ok ? s_sl[e] : 0;
      Rrow[e] = ok ? s_sy[slc * M + sle] : 0.0;
      Rcol[e] = ok ? s_sy[sle * M + slc] : 0.0;
      Yrow[e] = ok ? s_yy[slc * M + sle] : 0.0;
      tv[e] = 0.0;
    }
    const double diag = act ? s_sy[slc * M + slc] : 1.0;
    double acc = act ? s_p1[slc] : 0.0;
    double tmine = 0.0;
#pragma unroll
    for (int e = QN_MMAX - 1; e >= 0; --e) {
      if (e < cnt) {
        const double te = __shfl(acc / diag, e, 64);
        tv[e] = te;
        if (c == e) tmine = te;
        if (c < e) acc -= Rrow[e] * te;
      }
    }
    acc = diag * tmine - gamma * (act ? s_p2[slc] : 0.0);
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) acc += gamma * Yrow[e] * tv[e];
    double amine = 0.0;
#pragma unroll
    for (int e = 0; e < QN_MMAX; ++e) {
      if (e < cnt) {
        const double ae = __shfl(acc / diag, e, 64);
        if (c == e) amine = ae;
        if (c > e) acc -= Rcol[e] * ae;
      }
    }
    if (c < QN_MMAX) {
      cf_a[c] = 0.0;
      cf_t[c] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    if (act) {
      cf_a[slc] = amine;
      cf_t[slc] = gamma * tmine;
    }
  }
  __syncthreads();
  const int status = s_ctl[0];
  const bool newp = s_ctl[1] != 0;
  const int cnt = s_ctl[2];
  const double gamma = s_misc[0];
  // ---- pass 2 (own elements): store the pair, x <- xt, g <- gt, direction
  double p2v[2] = {0.0, 0.0};
  if (own) {
    const double xv = A.xt[i], gv = A.gt[i], sv = A.d[i], yv = A.wb[i], pv = A.pg[i];
    if (newp) {
      A.S[(long)head * N + i] = sv;
      A.Y[(long)head * N + i] = yv;
    }
    A.x[i] = xv;
    A.g[i] = gv;
    if (status == ST_RUNNING) {
      double hg = gamma * pv;
      for (int c = 0; c < cnt; ++c) {
        const int j = s_sl[c];
        hg += cf_a[j] * A.S[(long)j * N + i] - cf_t[j] * A.Y[(long)j * N + i];
      }
      double di = -hg;
      if (A.l1 && A.l1c[i] > 0.0 && di * pv >= 0.0) di = 0.0;
      A.d[i] = di;
      p2v[0] = pv * di;
      p2v[1] = di * di;
    }
  }
  if (tid < 64) {
    const double a = wave_sum(p2v[0]), b = wave_sum(p2v[1]);
    if (tid == 0) {
      scr[F_PC + blockIdx.x * 2] = a;
      scr[F_PC + blockIdx.x * 2 + 1] = b;
    }
  }
  // every block is past its reads of the pre-step state and the old history blocks beyond this
  // barrier: block 0 commits after it
  if (!fu_barrier(scr, G)) {
    if (first) { fl[F_STATUS] = ST_BARRIER; fl[F_DONE] = 1; }
    return;
  }
  if (blockIdx.x == 0) {
    if (newp)
      for (int k = tid; k < M * M; k += MB_T) {
        A.SY[k] = s_sy[k];
        A.YY[k] = s_yy[k];
      }
    if (tid == 0) {
      const int iter = pre_iter + (started ? 1 : 0);
      if (A.past > 0) A.fh[iter % A.past] = ft;
      fl[F_ITER] = iter;
      fl[F_HEAD] = s_ctl[3];
      fl[F_COUNT] = cnt;
      fl[F_NEVAL] = pre_neval + 1;
      fl[F_LS] = 0;
      fl[F_BRACKET] = 0;
      fl[F_STARTED] = 1;
      A.sc[SC_F] = ft;
      A.sc[SC_GAMMA] = gamma;
      A.sc[SC_GINF] = s_misc[1];
      if (status != ST_RUNNING) {
        fl[F_STATUS] = status;
        fl[F_DONE] = 1;
      }
    }
  }
  if (status != ST_RUNNING) return;
  mb_grid_sum(scr + F_PC, (int)G, 2, red, false);
  double dg = red[0], dd = red[1];
  int cnt2 = cnt;
  if (!(dg < 0.0)) {  // not a descent direction: drop the history, steepest descent (rare)
    if (own) A.d[i] = -A.pg[i];
    dg = -tot[4];
    dd = tot[4];
    cnt2 = 0;
  }
  const double alpha2 = cnt2 == 0 ? 1.0 / fmax(sqrt(dd), 1e-300) : 1.0;
  if (own) {
    const double xv = A.x[i], dv = A.d[i];
    double t = xv + alpha2 * dv;
    if (A.l1 && A.l1c[i] > 0.0) {
      const double pv = A.pg[i];
      const double orth = xv != 0.0 ? (xv > 0.0 ? 1.0 : -1.0) : (pv < 0.0 ? 1.0 : (pv > 0.0 ? -1.0 : 0.0));
      if (t * orth <= 0.0) t = 0.0;
    }
    A.xt[i] = t;
    A.wb[i] = t * (i < A.Kn ? A.isg[i % A.n] : 1.0);
  }
  if (first) {
    if (cnt2 == 0) {
      fl[F_COUNT] = 0;
      A.sc[SC_GAMMA] = 1.0;
    }
    A.sc[SC_ALPHA] = alpha2;
    A.sc[SC_DGINIT] = dg;
  }
}

SRML_API long srml_qn_fused_scratch() { return (long)F_END; }

// Offset (in doubles) of the fused step's barrier words in its scratch: a caller that abandons a
// step whose barrier timed out zeroes them before the scratch is used again.
SRML_API long srml_qn_fused_barrier_offset() { return (long)F_BAR; }

// 1 when the fused step's G = ceil(N / 32) blocks are guaranteed co-resident on the current
// device (occupancy x CUs >= G), so its software grid barriers cannot wait on an unscheduled
// block; 0 otherwise (the caller takes the multi-launch step instead).
SRML_API int srml_qn_fused_resident(long N) {
  const long G = (N + FU_E - 1) / FU_E;
  if (N <= 0 || G > FU_GMAX) return 0;
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(qn_fused_kernel), MB_T,
                                                   0) != hipSuccess)
    return 0;
  return (long)per_cu * cus >= G ? 1 : 0;
}

// One optimiser step as ONE launch (G = ceil(N / 32) <= 512 blocks; larger N: the single-block
// step). fws (optional): the fused binary evaluation's partial rows (parts rows of wst floats,
// srml_logreg_binary3_f32's workspace) folded in place of `out` — single-rank fits only (a
// multi-rank fit all-reduces `out` between the evaluation and the step). The scratch's barrier
// words must start at zero (a zeroed allocation) and every launch leaves them so.
SRML_API int srml_qn_step_fused(const QnArgs* a, double* scratch, const float* fws, int parts, long wst,
                                hipStream_t stream) {
  if (a->M < 1 || a->M > QN_MMAX || a->N <= 0 || !scratch) return (int)hipErrorInvalidValue;
  const long G = (a->N + FU_E - 1) / FU_E;
  if (G > FU_GMAX) return srml_qn_step(a, stream);
  if (fws && (a->K != 1 || (wst & 3) || parts <= 0)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(qn_fused_kernel, dim3((unsigned)G), dim3(MB_T), 0, stream, *a, scratch, fws, parts, wst);
  return srml_status();
}

// K1 of the multi-block step with the fold of the binary evaluation's partial rows in front
// (one-rank fits): ceil(N / 32) blocks, each folds its 32 elements' columns (fu_fold_block) and
// writes the pass-0 partials; K2..K4 as in srml_qn_step_mb. Replaces fold_rows_kernel + K1.
__global__ __launch_bounds__(MB_T) void qn_mb1f_kernel(QnArgs A, double* __restrict__ scr,
                                                       const float* __restrict__ fws, int parts, long wst) {
  __shared__ double red[4 * MB_NW], tot[4], fold[32][33];
  const bool first = blockIdx.x == 0 && threadIdx.x == 0;
  const unsigned G = gridDim.x;
  const long i = (long)blockIdx.x * FU_E + threadIdx.x;
  const bool own = threadIdx.x < FU_E && i < A.N;
  // every load up front (the fold's rows are read even when the fit is done: a finished fit's
  // remaining graph replays cost one wasted read each, against a round trip on every step)
  const int done = A.fl[F_DONE];
  MbSnap q{};
  if (first) q = mb_snap_load(A);
  const MbP0In e = mb_p0_load(A, i, own);
  double oval = 0.0, lpart = 0.0;
  fu_fold_block(A, fws, parts, wst, fold, red, own, i, G, oval, lpart);
  if (done) {
    if (first) scr[S_PHASE] = 0.0;
    return;
  }
  if (first) mb_snap_store(A, q, scr);
  if (blockIdx.x == G - 1 && threadIdx.x == 0) scr[S_LOSS] = lpart;
  double p0[4] = {0.0, 0.0, 0.0, 0.0};
  mb_p0(A, i, own, e, oval, p0);
  mb_block_sum<4>(p0, red, tot);
  if (threadIdx.x < 4) scr[S_PA + blockIdx.x * 4 + threadIdx.x] = tot[threadIdx.x];
}

// One optimiser step of a one-rank binary fit as four launches with the evaluation's fold in K1:
// fws = srml_logreg_binary3_f32's workspace left unfolded (leave = 1), parts rows of wst floats.
SRML_API int srml_qn_step_mbf(const QnArgs* a, double* scratch, const float* fws, int parts, long wst,
                              hipStream_t stream) {
  if (a->M < 1 || a->M > QN_MMAX || a->N <= 0 || !scratch || !fws) return (int)hipErrorInvalidValue;
  if (a->K != 1 || (wst & 3) || parts <= 0) return (int)hipErrorInvalidValue;
  const long G = (a->N + MB_T - 1) / MB_T, G1 = (a->N + FU_E - 1) / FU_E;
  if (G > MB_GMAX || G1 > MB_GAMAX) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)G), blk(MB_T);
  hipLaunchKernelGGL(qn_mb1f_kernel, dim3((unsigned)G1), blk, 0, stream, *a, scratch, fws, parts, wst);
  hipLaunchKernelGGL(qn_mb2_kernel, grid, blk, 0, stream, *a, scratch, (int)G1);
  hipLaunchKernelGGL(qn_mb3_kernel, grid, blk, 0, stream, *a, scratch);
  hipLaunchKernelGGL(qn_mb4_kernel, grid, blk, 0, stream, *a, scratch);
  return srml_status();
}
