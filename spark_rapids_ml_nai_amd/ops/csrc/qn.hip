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

enum { F_DONE = 0, F_STATUS, F_ITER, F_NEVAL, F_LS, F_COUNT, F_HEAD, F_STARTED, F_BRACKET };
enum { ST_RUNNING = 0, ST_CONV_GRAD = 1, ST_CONV_F = 2, ST_MAXITER = 3, ST_LS_FAIL = 4 };
enum { SC_F = 0, SC_ALPHA, SC_DGINIT, SC_GAMMA, SC_GINF };

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
  if (started) {
    bool accept = true;
    double width = 1.0;
    if (!isfinite(ft)) {
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
        }
        return;
      }
      alpha *= width;
      qn_set_trial(A, alpha);
      if (tid == 0) {
        fl[F_LS] = ls;
        fl[F_NEVAL] = pre_neval + 1;
        if (width < 1.0) fl[F_BRACKET] = 1;
        A.sc[SC_ALPHA] = alpha;
      }
      return;
    }
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
