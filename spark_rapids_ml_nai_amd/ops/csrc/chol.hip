// Dense SPD solves and Gram-matrix coordinate descent for the linear models, on device.
//
//  * srml_potrf_f64: blocked right-looking Cholesky (lower, row-major), 32-wide panels (64: env):
//      diag block factored in LDS by one workgroup -> panel TRSM (thread per row, L11 in LDS)
//      -> trailing update A22 -= A21 A21^T on the f64 MFMA GEMM (srml_dgemm).
//    A non-positive pivot sets *info = column + 1 (the caller falls back to an eigen solve).
//  * srml_potrs_f64: L L^T x = b for one right-hand side (two single-workgroup sweeps with
//    block-wide dot products; O(n^2), latency-bound but ~ms at n = 3000).
//  * srml_cd_gram_f64: cyclic coordinate descent for 1/2 w'Aw - b'w + sum l1|w| + 1/2 sum l2 w^2
//    (Spark/cuML elastic-net objective on the standardised Gram matrix, "covariance updates"):
//    one 1024-thread workgroup keeps w and A·w in LDS, each coordinate update streams one row
//    of A (L2-resident) — the whole solve is one kernel launch instead of a host loop.
// Reference: cuML LinearRegressionMG / RidgeMG / CDMG solves (regression.py:498-613).
#include "common.h"

#include <stdlib.h>

extern "C" int srml_dgemm(int ta, int tb, int M, int N, int K, double alpha, const double* A, long lda,
                          const double* B, long ldb, double beta, double* C, long ldc, hipStream_t stream);
extern "C" int srml_dgemm_syrk_lower(int M, int K, double alpha, const double* A, long lda, double beta, double* C,
                                     long ldc, hipStream_t stream);

namespace {
// panel width: 64 (SRML_POTRF_NB=64) or 32 (default): the panel chain (diagonal factor -> TRSM ->
// next panel) is latency-bound, and a 32-wide panel shortens both kernels' dependent chains ~4x
// for twice the panels
constexpr int NB_MAX = 64;

template <int NB>
__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ A, long lda, int k0, int nb,
                                                         int* __restrict__ info) {
  __shared__ double S[NB][NB + 1];
  const int t = threadIdx.x;
  for (int idx = t; idx < nb * nb; idx += 256) {
    const int i = idx / nb, j = idx % nb;
    S[i][j] = A[(long)(k0 + i) * lda + k0 + j];
  }
  __syncthreads();
  for (int j = 0; j < nb; ++j) {
    if (t == 0) {
      const double d = S[j][j];
      if (!(d > 0.0)) {
        if (*info == 0) *info = k0 + j + 1;
        S[j][j] = 1.0;
      } else {
        S[j][j] = sqrt(d);
      }
    }
    __syncthreads();
    const double djj = S[j][j];
    for (int i = j + 1 + t; i < nb; i += 256) S[i][j] /= djj;
    __syncthreads();
    const int r = nb - j - 1;
    for (int idx = t; idx < r * r; idx += 256) {
      const int i = j + 1 + idx / r, l = j + 1 + idx % r;
      if (l <= i) S[i][l] -= S[i][j] * S[l][j];
    }
    __syncthreads();
  }
  for (int idx = t; idx < nb * nb; idx += 256) {
    const int i = idx / nb, j = idx % nb;
    A[(long)(k0 + i) * lda + k0 + j] = j <= i ? S[i][j] : 0.0;
  }
}

// Register-resident variant of the diagonal-block factorisation (one wave, lane i = row i, the
// row in 64 VGPR pairs with compile-time indices): per pivot column j the pivot and every S[l][j]
// reach all lanes by scalar readlane broadcasts, and the right-looking update is one FMA per
// (l, lane). Entries above the diagonal are updated too but never read, so no masking is needed;
// padded rows (i >= nb) hold identity rows. No LDS and no barriers inside the 64-step chain.
__device__ __forceinline__ double bcast_f64(double v, int src) {
  const long long bits = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), src);
  const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int NB>
__global__ __launch_bounds__(64) void potrf_diag_reg_kernel(double* __restrict__ A, long lda, int k0, int nb,
                                                            int* __restrict__ info) {
  const int i = threadIdx.x;
  double c[NB];
  const double* row = A + (long)(k0 + (i < nb ? i : 0)) * lda + k0;
#pragma unroll
  for (int l = 0; l < NB; ++l) c[l] = (i < nb && l < nb) ? row[l] : (i == l ? 1.0 : 0.0);
  int bad = 0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double d = bcast_f64(c[j], j);
    if (!(d > 0.0)) {
      if (!bad && j < nb) bad = k0 + j + 1;
      d = 1.0;
    } else {
      d = sqrt(d);
    }
    const double rd = 1.0 / d;  // one division per column, the scaling is a multiply
    if (i == j) c[j] = d;
    else if (i > j) c[j] *= rd;
#pragma unroll
    for (int l = j + 1; l < NB; ++l) c[l] = fma(-c[j], bcast_f64(c[j], l), c[l]);
  }
  if (i == 0 && bad && *info == 0) *info = bad;
  if (i < nb) {
    double* out = A + (long)(k0 + i) * lda + k0;
#pragma unroll
    for (int l = 0; l < NB; ++l)
      if (l < nb) out[l] = l <= i ? c[l] : 0.0;
  }
}

// rows r >= k1: x (1 x NB) solves x L11^T = A[r, k0:k0+NB] (only full panels reach the TRSM: the
// last, possibly narrower, diagonal block has no rows below it)
template <int NB>
__global__ __launch_bounds__(256) void potrf_trsm_kernel(double* __restrict__ A, long lda, int k0, int k1, int n) {
  __shared__ double L[NB][NB + 1];
  __shared__ double rd[NB];  // 1 / L[j][j]: a multiply, not a division, on each row's chain
  const int t = threadIdx.x;
  for (int idx = t; idx < NB * NB; idx += 256) {
    const int i = idx / NB, j = idx % NB;
    L[i][j] = A[(long)(k0 + i) * lda + k0 + j];
  }
  __syncthreads();
  if (t < NB) rd[t] = 1.0 / L[t][t];
  __syncthreads();
  const int r = k1 + blockIdx.x * 256 + t;
  if (r >= n) return;
  double x[NB];
  double* row = A + (long)r * lda + k0;
#pragma unroll
  for (int j = 0; j < NB; ++j) x[j] = row[j];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double s = x[j];
#pragma unroll
    for (int l = 0; l < j; ++l) s -= x[l] * L[j][l];
    x[j] = s * rd[j];
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) row[j] = x[j];
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < nw; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(1024) void potrs_kernel(const double* __restrict__ L, int n, long lda,
                                                     double* __restrict__ b) {
  extern __shared__ double x[];  // the right-hand side lives in LDS: no cross-wave global RAW
  __shared__ double red[16];
  for (int i = threadIdx.x; i < n; i += blockDim.x) x[i] = b[i];
  __syncthreads();
  // forward: L z = b
  for (int i = 0; i < n; ++i) {
    double s = 0.0;
    for (int j = threadIdx.x; j < i; j += blockDim.x) s += L[(long)i * lda + j] * x[j];
    s = block_sum(s, red);
    if (threadIdx.x == 0) x[i] = (x[i] - s) / L[(long)i * lda + i];
    __syncthreads();
  }
  // backward: L^T x = z
  for (int i = n - 1; i >= 0; --i) {
    double s = 0.0;
    for (int j = i + 1 + threadIdx.x; j < n; j += blockDim.x) s += L[(long)j * lda + i] * x[j];
    s = block_sum(s, red);
    if (threadIdx.x == 0) x[i] = (x[i] - s) / L[(long)i * lda + i];
    __syncthreads();
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) b[i] = x[i];
}

// Blocked triangular solves (L L^T x = b) in one workgroup: 64-row blocks; the off-diagonal part
// of each block is a coalesced GEMV by all 16 waves, the 64 x 64 diagonal block is staged in LDS
// and solved by ONE wave with scalar broadcasts (no barrier per row). Replaces a row-at-a-time
// loop with two barriers per row (~9 ms at n = 3000).
constexpr int TS_B = 64;

__global__ __launch_bounds__(1024) void potrs_blocked_kernel(const double* __restrict__ L, int n, long lda,
                                                             double* __restrict__ b, int backward_only) {
  extern __shared__ double x[];               // n
  __shared__ double blk[TS_B][TS_B + 1];      // diagonal block
  __shared__ double part[16][TS_B];           // partial sums of the backward GEMV
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  for (int i = t; i < n; i += blockDim.x) x[i] = b[i];
  __syncthreads();
  auto bcast = [](double v, int src) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), src);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  };
  // forward: L z = b (skipped when b already holds z: the augmented factorisation computed it)
  for (int j0 = 0; j0 < (backward_only ? 0 : n); j0 += TS_B) {
    const int nb = n - j0 < TS_B ? n - j0 : TS_B;
    // x[j0 + r] -= L[j0 + r, 0:j0] . x[0:j0]: wave w takes rows r = w, w + 16, ...; 8 loads in
    // flight per lane (a dependent load per 64 columns left the sweep latency-bound)
    for (int r = wid; r < nb; r += 16) {
      const double* row = L + (long)(j0 + r) * lda;
      double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      int c = lane;
      for (; c + 7 * 64 < j0; c += 8 * 64) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = row[c + 64 * u];
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] = fma(v[u], x[c + 64 * u], s[u]);
      }
      for (; c < j0; c += 64) s[0] = fma(row[c], x[c], s[0]);
      double t8 = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
      t8 = wave_sum(t8);
      if (lane == 0) x[j0 + r] -= t8;
    }
    for (int e = t; e < nb * nb; e += blockDim.x) {
      const int r = e / nb, c = e - r * nb;
      blk[r][c] = L[(long)(j0 + r) * lda + j0 + c];
    }
    __syncthreads();
    if (wid == 0) {
      double xr = lane < nb ? x[j0 + lane] : 0.0;
      for (int c = 0; c < nb; ++c) {
        const double xc = bcast(xr, c) / blk[c][c];
        if (lane == c) xr = xc;
        if (lane > c && lane < nb) xr = fma(-blk[lane][c], xc, xr);
      }
      if (lane < nb) x[j0 + lane] = xr;
    }
    __syncthreads();
  }
  // backward: L^T x = z
  const int last0 = ((n - 1) / TS_B) * TS_B;
  for (int j0 = last0; j0 >= 0; j0 -= TS_B) {
    const int nb = n - j0 < TS_B ? n - j0 : TS_B;
    // x[j0 + i] -= sum_{j >= j0 + nb} L[j][j0 + i] x[j]: lane = column i, waves split the rows j
    {
      // 8 rows in flight per lane: one dependent 512-B row load per iteration ran the backward
      // sweep at ~23 GB/s (1.55 ms at n = 3000)
      double s[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      if (lane < nb) {
        int j = j0 + nb + wid;
        for (; j + 7 * 16 < n; j += 8 * 16) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = L[(long)(j + 16 * u) * lda + j0 + lane];
#pragma unroll
          for (int u = 0; u < 8; ++u) s[u] = fma(v[u], x[j + 16 * u], s[u]);
        }
        for (; j < n; j += 16) s[0] = fma(L[(long)j * lda + j0 + lane], x[j], s[0]);
      }
      part[wid][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    }
    for (int e = t; e < nb * nb; e += blockDim.x) {
      const int r = e / nb, c = e - r * nb;
      blk[r][c] = L[(long)(j0 + r) * lda + j0 + c];
    }
    __syncthreads();
    if (wid == 0) {
      double xr = 0.0;
      if (lane < nb) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < 16; ++w) s += part[w][lane];
        xr = x[j0 + lane] - s;
      }
      for (int c = nb - 1; c >= 0; --c) {
        const double xc = bcast(xr, c) / blk[c][c];
        if (lane == c) xr = xc;
        if (lane < c) xr = fma(-blk[c][lane], xc, xr);
      }
      if (lane < nb) x[j0 + lane] = xr;
    }
    __syncthreads();
  }
  for (int i = t; i < n; i += blockDim.x) b[i] = x[i];
}

// A: n x n (row-major, symmetric), b, l1, l2: n. w: in/out (initial guess). Result iterations in *iters.
__global__ __launch_bounds__(1024) void cd_gram_kernel(const double* __restrict__ A, int n, long lda,
                                                       const double* __restrict__ b, const double* __restrict__ l1,
                                                       const double* __restrict__ l2, double* __restrict__ w_out,
                                                       int max_iter, double tol, int* __restrict__ iters) {
  extern __shared__ double sm[];  // w[n], g[n] (= A w)
  double* w = sm;
  double* g = sm + n;
  __shared__ double bc[4];
  const int t = threadIdx.x;
  for (int i = t; i < n; i += blockDim.x) w[i] = w_out[i];
  __syncthreads();
  // g = A w
  for (int i = t; i < n; i += blockDim.x) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += A[(long)i * lda + j] * w[j];
    g[i] = s;
  }
  __syncthreads();
  int it = 0;
  for (; it < max_iter; ++it) {
    double max_delta = 0.0, max_w = 0.0;  // meaningful on thread 0
    for (int j = 0; j < n; ++j) {
      if (t == 0) {
        const double ajj = A[(long)j * lda + j];
        const double diag = ajj + l2[j];
        double d = 0.0;
        if (diag > 0.0) {
          const double rho = b[j] - g[j] + ajj * w[j];
          double nw = 0.0;
          if (rho > l1[j]) nw = (rho - l1[j]) / diag;
          else if (rho < -l1[j]) nw = (rho + l1[j]) / diag;
          d = nw - w[j];
          w[j] = nw;
          max_w = fmax(max_w, fabs(nw));
          max_delta = fmax(max_delta, fabs(d));
        }
        bc[0] = d;
      }
      __syncthreads();
      const double d = bc[0];
      if (d != 0.0) {
        const double* row = A + (long)j * lda;  // symmetric: column j == row j
        for (int i = t; i < n; i += blockDim.x) g[i] += d * row[i];
      }
      __syncthreads();
    }
    if (t == 0) bc[1] = (max_delta <= tol * fmax(max_w, 1e-300)) ? 1.0 : 0.0;
    __syncthreads();
    if (bc[1] != 0.0) {
      ++it;
      break;
    }
  }
  for (int i = t; i < n; i += blockDim.x) w_out[i] = w[i];
  if (t == 0) *iters = it;
}

// Block-cyclic form of the same Gauss-Seidel sweep (identical coordinate order and updates):
// the CB x CB diagonal block of A is staged in LDS and ONE wave runs the CB sequential
// coordinate updates on it — its lanes own g / w of the block's coordinates, the coordinate's
// delta is broadcast with a lane shuffle, so there is no workgroup barrier and no global load
// inside the sequential chain. The rest of g is then brought up to date with one coalesced
// rank-CB update g += A[blk, :]^T d (A symmetric) by all 1024 threads. Per sweep A is streamed
// once; the per-coordinate cost drops from two barriers plus a dependent 24 KB row fetch to
// ~20 fp64 VALU instructions.
constexpr int CD_CB = 64;

__global__ __launch_bounds__(1024) void cd_gram_block_kernel(const double* __restrict__ A, int n, long lda,
                                                             const double* __restrict__ b, const double* __restrict__ l1,
                                                             const double* __restrict__ l2, double* __restrict__ w_out,
                                                             int max_iter, double tol, int* __restrict__ iters) {
  extern __shared__ double sm[];  // w[n], g[n], blk[CB][CB + 1], dv[CB]
  double* w = sm;
  double* g = sm + n;
  double* blk = g + n;
  double* dv = blk + CD_CB * (CD_CB + 1);
  __shared__ int done;
  const int t = threadIdx.x;
  const int lane = t & 63;
  for (int i = t; i < n; i += blockDim.x) w[i] = w_out[i];
  __syncthreads();
  for (int i = t; i < n; i += blockDim.x) {  // g = A w, column reads (A symmetric) -> coalesced
    double s = 0.0;
#pragma unroll 8
    for (int j = 0; j < n; ++j) s = fma(A[(long)j * lda + i], w[j], s);
    g[i] = s;
  }
  __syncthreads();
  int it = 0;
  double max_delta = 0.0, max_w = 0.0;  // wave 0 (lane-partial, reduced at the sweep end)
  for (; it < max_iter; ++it) {
    max_delta = 0.0;
    max_w = 0.0;
    for (int j0 = 0; j0 < n; j0 += CD_CB) {
      const int nb = n - j0 < CD_CB ? n - j0 : CD_CB;
      for (int e = t; e < nb * nb; e += blockDim.x) {
        const int r = e / nb, c = e - r * nb;
        blk[r * (CD_CB + 1) + c] = A[(long)(j0 + r) * lda + j0 + c];
      }
      __syncthreads();
      if (t < 64) {
        const bool own = lane < nb;
        const int jj = j0 + (own ? lane : 0);
        double gl = own ? g[jj] : 0.0;
        double wl = own ? w[jj] : 0.0;
        const double w0 = wl;
        const double ajj = own ? blk[lane * (CD_CB + 1) + lane] : 0.0;
        const double diag = own ? ajj + l2[jj] : 0.0;
        const double inv_diag = diag > 0.0 ? 1.0 / diag : 0.0;
        const double bj = own ? b[jj] : 0.0;
        const double l1j = own ? l1[jj] : 0.0;
        for (int c = 0; c < nb; ++c) {
          // every lane evaluates its own coordinate's update; lane c's is the one applied
          double d = 0.0, nw = wl;
          if (diag > 0.0) {
            const double rho = bj - gl + ajj * wl;
            nw = rho > l1j ? (rho - l1j) * inv_diag : (rho < -l1j ? (rho + l1j) * inv_diag : 0.0);
            d = nw - wl;
          }
          {  // c is wave-uniform: broadcast through scalar readlanes instead of ds_bpermute
            const long long bits = __double_as_longlong(d);
            const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), c);
            const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), c);
            d = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
          }
          if (lane == c) {
            if (diag > 0.0) {
              wl = nw;
              max_w = fmax(max_w, fabs(nw));
              max_delta = fmax(max_delta, fabs(d));
            }
          }
          if (d != 0.0 && own) gl = fma(blk[c * (CD_CB + 1) + lane], d, gl);
        }
        if (own) {
          g[jj] = gl;
          w[jj] = wl;
          dv[lane] = wl - w0;
        }
      }
      __syncthreads();
      // unconditional, unrolled loads: 16 independent row reads in flight per thread (a
      // data-dependent skip here serialised one HBM round trip per coordinate)
      for (int i = t; i < n; i += blockDim.x) {
        if (i >= j0 && i < j0 + nb) continue;
        const double* col = A + (long)j0 * lda + i;
        double s0 = 0.0, s1 = 0.0;
        int c = 0;
        for (; c + 16 <= nb; c += 16) {
          double v[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) v[u] = col[(long)(c + u) * lda];
#pragma unroll
          for (int u = 0; u < 16; u += 2) {
            s0 = fma(v[u], dv[c + u], s0);
            s1 = fma(v[u + 1], dv[c + u + 1], s1);
          }
        }
        for (; c < nb; ++c) s0 = fma(col[(long)c * lda], dv[c], s0);
        g[i] += s0 + s1;
      }
      __syncthreads();
    }
    if (t < 64) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        max_delta = fmax(max_delta, __shfl_xor(max_delta, o, 64));
        max_w = fmax(max_w, __shfl_xor(max_w, o, 64));
      }
      if (t == 0) done = (max_delta <= tol * fmax(max_w, 1e-300)) ? 1 : 0;
    }
    __syncthreads();
    if (done) {
      ++it;
      break;
    }
  }
  for (int i = t; i < n; i += blockDim.x) w_out[i] = w[i];
  if (t == 0) *iters = it;
}

// Pipelined block-cyclic sweep (same coordinate order and updates as cd_gram_block_kernel). The
// rank-CB update of g by block b's delta no longer sits between two chains: while wave 0 runs
// the sequential chain of block b, waves 1..15 apply the PREVIOUS block's delta to every other
// row of g (the 64 x n panel stream, the bandwidth-heavy part), and only the 64 x 64 piece that
// block b itself needs is applied before its chain. One barrier per block; the chain (latency)
// and the panel stream (one CU's L2 bandwidth) overlap instead of adding up.
__global__ __launch_bounds__(1024) void cd_gram_pipe_kernel(const double* __restrict__ A, int n, long lda,
                                                            const double* __restrict__ b, const double* __restrict__ l1,
                                                            const double* __restrict__ l2, double* __restrict__ w_out,
                                                            int max_iter, double tol, int* __restrict__ iters,
                                                            int w0_zero) {
  extern __shared__ double sm[];  // w[n], g[n], blk[CB][CB + 1], dv[2][CB], part[16][CB]
  double* w = sm;
  double* g = sm + n;
  double* blk = g + n;
  double* dvb = blk + CD_CB * (CD_CB + 1);
  double* part = dvb + 2 * CD_CB;
  __shared__ int done;
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  for (int i = t; i < n; i += blockDim.x) w[i] = w0_zero ? 0.0 : w_out[i];
  __syncthreads();
  for (int i = t; i < n; i += blockDim.x) {  // g = A w (skipped for a zero start)
    double s = 0.0;
    if (!w0_zero) {
#pragma unroll 8
      for (int j = 0; j < n; ++j) s = fma(A[(long)j * lda + i], w[j], s);
    }
    g[i] = s;
  }
  for (int i = t; i < 2 * CD_CB; i += blockDim.x) dvb[i] = 0.0;
  __syncthreads();
  const int nblk = (n + CD_CB - 1) / CD_CB;
  int it = 0, step = 0;
  int p0 = -1, pnb = 0;  // previous block (cyclic across sweeps): start row, size
  double max_delta = 0.0, max_w = 0.0;
  for (; it < max_iter; ++it) {
    max_delta = 0.0;
    max_w = 0.0;
    for (int bi = 0; bi < nblk; ++bi, ++step) {
      const int j0 = bi * CD_CB;
      const int nb = n - j0 < CD_CB ? n - j0 : CD_CB;
      double* dprev = dvb + ((step + 1) & 1) * CD_CB;  // delta of the previous block
      double* dcur = dvb + (step & 1) * CD_CB;
      // phase A (all waves): stage block b's diagonal tile; partial sums of the previous block's
      // delta onto block b's rows (wave w takes previous-block columns 4w .. 4w + 3)
      for (int e = t; e < nb * nb; e += blockDim.x) {
        const int r = e / nb, c = e - r * nb;
        blk[r * (CD_CB + 1) + c] = A[(long)(j0 + r) * lda + j0 + c];
      }
      {
        double s = 0.0;
        if (p0 >= 0 && p0 != j0 && lane < nb) {  // (one block only: its chain already updated g)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int c = 4 * wid + u;
            if (c < pnb) s = fma(A[(long)(p0 + c) * lda + j0 + lane], dprev[c], s);
          }
        }
        part[wid * CD_CB + lane] = s;
      }
      __syncthreads();
      if (wid == 0) {  // sequential chain of block b
        const bool own = lane < nb;
        const int jj = j0 + (own ? lane : 0);
        double gl = 0.0;
        if (own) {
          gl = g[jj];
#pragma unroll
          for (int q = 0; q < 16; ++q) gl += part[q * CD_CB + lane];
        }
        double wl = own ? w[jj] : 0.0;
        const double w0 = wl;
        const double ajj = own ? blk[lane * (CD_CB + 1) + lane] : 0.0;
        const double diag = own ? ajj + l2[jj] : 0.0;
        const double inv_diag = diag > 0.0 ? 1.0 / diag : 0.0;
        const double bj = own ? b[jj] : 0.0;
        const double l1j = own ? l1[jj] : 0.0;
        for (int c = 0; c < nb; ++c) {
          double d = 0.0, nw = wl;
          if (diag > 0.0) {
            const double rho = bj - gl + ajj * wl;
            nw = rho > l1j ? (rho - l1j) * inv_diag : (rho < -l1j ? (rho + l1j) * inv_diag : 0.0);
            d = nw - wl;
          }
          {
            const long long bits = __double_as_longlong(d);
            const int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffLL), c);
            const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), c);
            d = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
          }
          if (lane == c && diag > 0.0) {
            wl = nw;
            max_w = fmax(max_w, fabs(nw));
            max_delta = fmax(max_delta, fabs(d));
          }
          if (d != 0.0 && own) gl = fma(blk[c * (CD_CB + 1) + lane], d, gl);
        }
        if (own) {
          g[jj] = gl;
          w[jj] = wl;
        }
        dcur[lane] = own ? wl - w0 : 0.0;
      } else if (p0 >= 0) {
        // waves 1..15: previous block's delta onto every row outside blocks (b-1, b)
        for (int i = t - 64; i < n; i += blockDim.x - 64) {
          if ((i >= p0 && i < p0 + pnb) || (i >= j0 && i < j0 + nb)) continue;
          const double* col = A + (long)p0 * lda + i;
          double s0 = 0.0, s1 = 0.0;
          int c = 0;
          for (; c + 16 <= pnb; c += 16) {
            double v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = col[(long)(c + u) * lda];
#pragma unroll
            for (int u = 0; u < 16; u += 2) {
              s0 = fma(v[u], dprev[c + u], s0);
              s1 = fma(v[u + 1], dprev[c + u + 1], s1);
            }
          }
          for (; c < pnb; ++c) s0 = fma(col[(long)c * lda], dprev[c], s0);
          g[i] += s0 + s1;
        }
      }
      __syncthreads();
      p0 = j0;
      pnb = nb;
    }
    if (t < 64) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        max_delta = fmax(max_delta, __shfl_xor(max_delta, o, 64));
        max_w = fmax(max_w, __shfl_xor(max_w, o, 64));
      }
      if (t == 0) done = (max_delta <= tol * fmax(max_w, 1e-300)) ? 1 : 0;
    }
    __syncthreads();
    if (done) {
      ++it;
      break;
    }
  }
  for (int i = t; i < n; i += blockDim.x) w_out[i] = w[i];
  if (t == 0) *iters = it;
}
}  // namespace

SRML_API int srml_potrf_f64(double* A, int n, long lda, int* info, hipStream_t stream) {
  if (n <= 0) return 0;
  // diagonal-block kernel: 1 = one wave, readlane broadcasts (64 us per 64 x 64 block); 0 = 256
  // threads in LDS with two barriers per column. (One wave with the scaled pivot column shared
  // through LDS broadcast reads measured 115 us: the chain is latency-bound, not readlane-bound.)
  static const int diag_reg = getenv("SRML_POTRF_REG") ? atoi(getenv("SRML_POTRF_REG")) : 1;
  static const int nbw = (getenv("SRML_POTRF_NB") && atoi(getenv("SRML_POTRF_NB")) == NB_MAX) ? NB_MAX : 32;
  hipError_t err = hipSuccess;
  SRML_TRY(err, hipMemsetAsync(info, 0, sizeof(int), stream));
  for (int k0 = 0; k0 < n; k0 += nbw) {
    const int nb = n - k0 < nbw ? n - k0 : nbw;
    const int k1 = k0 + nb;
    if (nbw == NB_MAX) {
      if (diag_reg)
        hipLaunchKernelGGL(potrf_diag_reg_kernel<NB_MAX>, dim3(1), dim3(64), 0, stream, A, lda, k0, nb, info);
      else
        hipLaunchKernelGGL(potrf_diag_kernel<NB_MAX>, dim3(1), dim3(256), 0, stream, A, lda, k0, nb, info);
    } else {
      if (diag_reg)
        hipLaunchKernelGGL(potrf_diag_reg_kernel<32>, dim3(1), dim3(64), 0, stream, A, lda, k0, nb, info);
      else
        hipLaunchKernelGGL(potrf_diag_kernel<32>, dim3(1), dim3(256), 0, stream, A, lda, k0, nb, info);
    }
    if (k1 < n) {
      const int m2 = n - k1;
      if (nbw == NB_MAX)
        hipLaunchKernelGGL(potrf_trsm_kernel<NB_MAX>, dim3((m2 + 255) / 256), dim3(256), 0, stream, A, lda, k0, k1, n);
      else
        hipLaunchKernelGGL(potrf_trsm_kernel<32>, dim3((m2 + 255) / 256), dim3(256), 0, stream, A, lda, k0, k1, n);
      // trailing update A22 -= A21 A21^T on the lower-triangle tiles only (SRML_POTRF_SYRK=0: full)
      static const int syrk = getenv("SRML_POTRF_SYRK") ? atoi(getenv("SRML_POTRF_SYRK")) : 1;
      const int rc = syrk ? srml_dgemm_syrk_lower(m2, nb, -1.0, A + (long)k1 * lda + k0, lda, 1.0,
                                                  A + (long)k1 * lda + k1, lda, stream)
                          : srml_dgemm(0, 1, m2, m2, nb, -1.0, A + (long)k1 * lda + k0, lda, A + (long)k1 * lda + k0,
                                       lda, 1.0, A + (long)k1 * lda + k1, lda, stream);
      if (rc) return rc;
    }
  }
  const int st = srml_status();
  return err != hipSuccess ? (int)err : st;
}

SRML_API int srml_potrs_f64(const double* L, int n, long lda, double* b, hipStream_t stream) {
  if (n <= 0) return 0;
  const size_t lds = (size_t)n * sizeof(double);
  if (lds > 150 * 1024) return -9;
  if (lds <= 110 * 1024) {  // + 41 KB static (diagonal block, partial sums)
    (void)hipFuncSetAttribute((const void*)potrs_blocked_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL(potrs_blocked_kernel, dim3(1), dim3(1024), lds, stream, L, n, lda, b, 0);
    return srml_status();
  }
  (void)hipFuncSetAttribute((const void*)potrs_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(potrs_kernel, dim3(1), dim3(1024), lds, stream, L, n, lda, b);
  return srml_status();
}

// L^T x = z only (z = L^-1 b from the augmented factorisation of [A b; b^T c], whose last row
// is z^T: the forward sweep rides along with the Cholesky's panel updates for free)
SRML_API int srml_potrs_backward_f64(const double* L, int n, long lda, double* z, hipStream_t stream) {
  if (n <= 0) return 0;
  const size_t lds = (size_t)n * sizeof(double);
  if (lds > 110 * 1024) return -9;
  (void)hipFuncSetAttribute((const void*)potrs_blocked_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(potrs_blocked_kernel, dim3(1), dim3(1024), lds, stream, L, n, lda, z, 1);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Global-memory block-cyclic coordinate descent for Gram matrices too wide for the LDS-resident
// kernels (n > ~9600 — w and g no longer fit 150 KiB). Same coordinate order and updates as the
// cyclic sweep: per block of CD_CB coordinates, `cd_chain_kernel` (one wave) runs the sequential
// soft-threshold chain against a block-local copy of g (A_bb staged in LDS) and emits the deltas;
// `cd_panel_kernel` (a grid over all n rows, coalesced row reads of the symmetric A) then applies
// the block's rank-CB update g += A[:, block] dv before the next block's chain. w and g live in
// device memory (L2-resident); the host launches one sweep at a time and reads the convergence
// word once per sweep.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void cd_chain_kernel(const double* __restrict__ A, int n, long lda,
                                                      const double* __restrict__ b, const double* __restrict__ l1,
                                                      const double* __restrict__ l2, double* __restrict__ w,
                                                      const double* __restrict__ g, int c0, double* __restrict__ dv,
                                                      double* __restrict__ stats) {
  __shared__ double ab[CD_CB][CD_CB + 1];
  const int lane = threadIdx.x;
  const int cb = min(CD_CB, n - c0);
  for (int r = 0; r < cb; ++r)
    if (lane < cb) ab[r][lane] = A[(long)(c0 + r) * lda + c0 + lane];
  double gl = lane < cb ? g[c0 + lane] : 0.0;
  double wl = lane < cb ? w[c0 + lane] : 0.0;
  double mx_d = 0.0, mx_w = 0.0, dl = 0.0;
  __syncthreads();
  for (int c = 0; c < cb; ++c) {
    const double gc = __shfl(gl, c, 64), wc = __shfl(wl, c, 64);
    const double ajj = ab[c][c];
    const double diag = ajj + l2[c0 + c];
    double d = 0.0, nw = wc;
    if (diag > 0.0) {
      const double rho = b[c0 + c] - gc + ajj * wc;
      const double lc = l1[c0 + c];
      nw = rho > lc ? (rho - lc) / diag : (rho < -lc ? (rho + lc) / diag : 0.0);
      d = nw - wc;
      mx_w = fmax(mx_w, fabs(nw));  // coordinates with a non-positive diagonal are skipped entirely
    }
    if (d != 0.0) {
      if (lane < cb) gl = fma(d, ab[c][lane], gl);  // A symmetric: row c of the block = column c
      if (lane == c) wl = nw;
      mx_d = fmax(mx_d, fabs(d));
    }
    if (lane == c) dl = d;
  }
  if (lane < cb) {
    w[c0 + lane] = wl;
    dv[lane] = dl;
  }
  if (lane == 0) {  // non-negative doubles order like their bit patterns
    atomicMax(reinterpret_cast<unsigned long long*>(stats), __double_as_longlong(mx_d));
    atomicMax(reinterpret_cast<unsigned long long*>(stats) + 1, __double_as_longlong(mx_w));
  }
}

__global__ __launch_bounds__(256) void cd_panel_kernel(const double* __restrict__ A, int n, long lda, int c0,
                                                       const double* __restrict__ dv, double* __restrict__ g) {
  __shared__ double d[CD_CB];
  const int cb = min(CD_CB, n - c0);
  if (threadIdx.x < CD_CB) d[threadIdx.x] = threadIdx.x < cb ? dv[threadIdx.x] : 0.0;
  __syncthreads();
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int c = 0; c < cb; ++c)
    if (d[c] != 0.0) acc = fma(A[(long)(c0 + c) * lda + i], d[c], acc);
  g[i] += acc;
}

__global__ __launch_bounds__(256) void cd_gemv_kernel(const double* __restrict__ A, int n, long lda,
                                                      const double* __restrict__ w, double* __restrict__ g) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double acc = 0.0;
  for (int j = 0; j < n; ++j) acc = fma(A[(long)j * lda + i], w[j], acc);
  g[i] = acc;
}

// One sweep of the global-memory CD (g = A w maintained in `g`; stats[0..1] = max |delta|, max |w|
// of the sweep, zeroed by the caller). init != 0: g = A w first.
SRML_API int srml_cd_sweep_global_f64(const double* A, int n, long lda, const double* b, const double* l1,
                                      const double* l2, double* w, double* g, double* dv, double* stats, int init,
                                      hipStream_t stream) {
  if (n <= 0) return 0;
  const unsigned gb = (unsigned)((n + 255) / 256);
  if (init) hipLaunchKernelGGL(cd_gemv_kernel, dim3(gb), dim3(256), 0, stream, A, n, lda, w, g);
  for (int c0 = 0; c0 < n; c0 += CD_CB) {
    hipLaunchKernelGGL(cd_chain_kernel, dim3(1), dim3(64), 0, stream, A, n, lda, b, l1, l2, w, g, c0, dv, stats);
    hipLaunchKernelGGL(cd_panel_kernel, dim3(gb), dim3(256), 0, stream, A, n, lda, c0, dv, g);
  }
  return srml_status();
}

SRML_API int srml_cd_gram_f64(const double* A, int n, long lda, const double* b, const double* l1, const double* l2,
                              double* w, int max_iter, double tol, int* iters, hipStream_t stream) {
  if (n <= 0) return 0;
  static const int pipe = getenv("SRML_CD_PIPE") ? atoi(getenv("SRML_CD_PIPE")) : 1;
  const size_t lds_pipe = ((size_t)2 * n + CD_CB * (CD_CB + 1) + 18 * CD_CB) * sizeof(double);
  if (pipe && lds_pipe <= 150 * 1024) {  // n <= ~6900
    (void)hipFuncSetAttribute((const void*)cd_gram_pipe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_pipe);
    hipLaunchKernelGGL(cd_gram_pipe_kernel, dim3(1), dim3(1024), lds_pipe, stream, A, n, lda, b, l1, l2, w, max_iter,
                       tol, iters, 0);
    return srml_status();
  }
  const size_t lds_blk = ((size_t)2 * n + CD_CB * (CD_CB + 1) + CD_CB) * sizeof(double);
  if (lds_blk <= 150 * 1024) {  // n <= ~7500
    (void)hipFuncSetAttribute((const void*)cd_gram_block_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds_blk);
    hipLaunchKernelGGL(cd_gram_block_kernel, dim3(1), dim3(1024), lds_blk, stream, A, n, lda, b, l1, l2, w, max_iter,
                       tol, iters);
    return srml_status();
  }
  const size_t lds = (size_t)2 * n * sizeof(double);
  if (lds > 150 * 1024) return -9;  // n <= 9600
  (void)hipFuncSetAttribute((const void*)cd_gram_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(cd_gram_kernel, dim3(1), dim3(1024), lds, stream, A, n, lda, b, l1, l2, w, max_iter, tol, iters);
  return srml_status();
}
