// Dense linear-algebra building blocks for the solvers.
//
//  * srml_xw_f32     — skinny GEMM  out = X W + bias  (X: m x n row-major, W: n x k, k <= 32).
//                      Bandwidth-bound: ONE pass over X, W staged in LDS, each wave owns a row
//                      at a time with 16-B vector loads, per-lane k partial sums reduced with
//                      wave64 shuffles. PCA transform (X·pcᵀ), GLM / linear predictions, and the
//                      reference's JNI `dgemm` on a cudf list column (rapidsml_jni.cu:75-107).
//  * srml_dgemm      — fp64 C = alpha op(A) op(B) + beta C on the f64 MFMA
//                      (`v_mfma_f64_16x16x4_f64`), LDS-tiled 64x64 per 256-thread block.
//                      Krylov products with the fp64 covariance (PCA eigensolver), normal-
//                      equation solves, and the C-ABI `srml_dgemm` (reference JNI dgemm,
//                      rapidsml_jni.cu:131-212).
//                      Tall-skinny / long-K shapes (X^T V, C·Q with few output tiles) split K over
//                      grid.z: every split writes its partial tile to a workspace with plain stores
//                      and one ordered pass folds the splits (alpha, beta applied there), so the
//                      result is bit-reproducible (no atomics) and the grid still fills the chip.
//  * srml_sign_flip_f64 — deterministic eigenvector signs: one wave per column finds the
//                      max-|x| entry with a wave64 arg-max and negates the column if that entry
//                      is negative (reference N1 `signFlip`, rapidsml_jni.cu:35-61, which used
//                      one thread per column).
#include "common.h"

// ------------------------------------------------------------------------------------------
// skinny GEMM
// ------------------------------------------------------------------------------------------
// Two-row-per-wave variant for n <= 256*V: every lane issues all of its 16-B loads for two rows
// before the first FMA (2*V loads in flight per lane, no per-iteration vmcnt(0) round trip),
// then reduces the K partial sums of each row with wave64 shuffles.
template <int K, int V>
__global__ __launch_bounds__(256) void xw_rows_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                      const float* __restrict__ W, const float* __restrict__ bias,
                                                      float* __restrict__ out, long ldo) {
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // [256*V][K], zero-padded
  for (int i = threadIdx.x; i < 256 * V * K; i += blockDim.x) Ws[i] = (i / K < n) ? W[i] : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * 4;
  for (long r0 = 2 * wave; r0 < m; r0 += 2 * nwaves) {
    const long ra = r0, rb = (r0 + 1 < m) ? r0 + 1 : r0;
    float acca[K], accb[K];
#pragma unroll
    for (int c = 0; c < K; ++c) { acca[c] = 0.f; accb[c] = 0.f; }
    // the two rows stream through in chunks of VC float4 per lane: all V chunks at once when the
    // row slices and the 2K accumulators fit the register budget, else VC = 2 per step (wide K x
    // long rows would otherwise spill the row slices to scratch)
    constexpr int VC = (2 * K + 8 * V <= 112) ? V : 2;
#pragma unroll 1
    for (int v0 = 0; v0 < V; v0 += VC) {
      floatx4 xa[VC], xb[VC];
#pragma unroll
      for (int u = 0; u < VC; ++u) {
        const int c = ((v0 + u) * 64 + lane) * 4;
        const int cc = (v0 + u < V && c < n) ? c : 0;  // n % 4 == 0 on this path; padded W rows are zero
        xa[u] = *reinterpret_cast<const floatx4*>(X + ra * ld + cc);
        xb[u] = *reinterpret_cast<const floatx4*>(X + rb * ld + cc);
      }
#pragma unroll
      for (int u = 0; u < VC; ++u) {
        const int c = ((v0 + u) * 64 + lane) * 4;
        const float sel = (v0 + u < V && c < n) ? 1.f : 0.f;
        const int cw = v0 + u < V ? c : 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float* w = &Ws[(cw + q) * K];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            acca[j] = fmaf(xa[u][q] * sel, w[j], acca[j]);
            accb[j] = fmaf(xb[u][q] * sel, w[j], accb[j]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j) { acca[j] = wave_sum(acca[j]); accb[j] = wave_sum(accb[j]); }
    if (lane < K) {
      float va = 0.f, vb = 0.f;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j == lane) { va = acca[j]; vb = accb[j]; }
      const float bb = bias ? bias[lane] : 0.f;
      out[ra * ldo + lane] = va + bb;
      if (rb != ra) out[rb * ldo + lane] = vb + bb;
    }
  }
}

template <int K, bool VEC>
__global__ __launch_bounds__(256) void xw_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                 const float* __restrict__ W, const float* __restrict__ bias,
                                                 float* __restrict__ out, long ldo, int wlds_rows) {
  extern __shared__ __attribute__((aligned(16))) float Ws[];  // [wlds_rows][K]
  for (int i = threadIdx.x; i < wlds_rows * K; i += blockDim.x) Ws[i] = W[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * 4;
  for (long r = wave; r < m; r += nwaves) {
    const float* row = X + r * ld;
    float acc[K];
#pragma unroll
    for (int c = 0; c < K; ++c) acc[c] = 0.f;
    if (VEC) {
      for (int d = lane * 4; d < n; d += 256) {
        floatx4 v = *reinterpret_cast<const floatx4*>(row + d);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float* w = (d + q < wlds_rows) ? &Ws[(d + q) * K] : &W[(long)(d + q) * K];
#pragma unroll
          for (int c = 0; c < K; ++c) acc[c] = fmaf(v[q], w[c], acc[c]);
        }
      }
    } else {
      for (int d = lane; d < n; d += 64) {
        const float v = row[d];
        const float* w = (d < wlds_rows) ? &Ws[d * K] : &W[(long)d * K];
#pragma unroll
        for (int c = 0; c < K; ++c) acc[c] = fmaf(v, w[c], acc[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < K; ++c) acc[c] = wave_sum(acc[c]);
    if (lane < K) {
      float v = 0.f;
#pragma unroll
      for (int c = 0; c < K; ++c)
        if (c == lane) v = acc[c];
      out[r * ldo + lane] = v + (bias ? bias[lane] : 0.f);
    }
  }
}

template <int K>
static int launch_xw(const float* X, long m, int n, long ld, const float* W, const float* bias, float* out, long ldo,
                     hipStream_t stream) {
  const int max_rows = (48 * 1024) / (4 * K);
  const int wrows = n < max_rows ? n : max_rows;
  const bool vec = ((ld & 3) == 0) && ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  long blocks = (m + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (vec && K <= 4 && n <= 4096) {
    const int V = (n + 255) / 256;
    long b2 = (m + 7) / 8;
    if (b2 > 8192) b2 = 8192;
    if (b2 < 1) b2 = 1;
#define SRML_XW_ROWS(VV)                                                                                          \
    hipLaunchKernelGGL((xw_rows_kernel<K, VV>), dim3((unsigned)b2), dim3(256), (size_t)256 * VV * K * sizeof(float), \
                       stream, X, m, n, ld, W, bias, out, ldo)
    if (V <= 1) SRML_XW_ROWS(1);
    else if (V <= 2) SRML_XW_ROWS(2);
    else if (V <= 4) SRML_XW_ROWS(4);
    else if (V <= 8) SRML_XW_ROWS(8);
    else if (V <= 12) SRML_XW_ROWS(12);
    else SRML_XW_ROWS(16);
    return srml_status();
  }
  size_t lds = (size_t)wrows * K * sizeof(float);
  if (vec)
    hipLaunchKernelGGL((xw_kernel<K, true>), dim3((unsigned)blocks), dim3(256), lds, stream, X, m, n, ld, W, bias, out,
                       ldo, wrows);
  else
    hipLaunchKernelGGL((xw_kernel<K, false>), dim3((unsigned)blocks), dim3(256), lds, stream, X, m, n, ld, W, bias, out,
                       ldo, wrows);
  return srml_status();
}

SRML_API int srml_xw_f32(const float* X, long m, int n, long ld, const float* W, int k, const float* bias, float* out,
                         long ldo, hipStream_t stream) {
  if (m <= 0) return 0;
  switch (k) {
    case 1: return launch_xw<1>(X, m, n, ld, W, bias, out, ldo, stream);
    case 2: return launch_xw<2>(X, m, n, ld, W, bias, out, ldo, stream);
    case 3: return launch_xw<3>(X, m, n, ld, W, bias, out, ldo, stream);
    case 4: return launch_xw<4>(X, m, n, ld, W, bias, out, ldo, stream);
    case 8: return launch_xw<8>(X, m, n, ld, W, bias, out, ldo, stream);
    case 16: return launch_xw<16>(X, m, n, ld, W, bias, out, ldo, stream);
    case 32: return launch_xw<32>(X, m, n, ld, W, bias, out, ldo, stream);
    default: return -1;  // caller pads k up to a supported width
  }
}

// ------------------------------------------------------------------------------------------
// Skinny GEMM on the exact-fp32 MFMA: Z (m x K) = X (m x n) Wt^T (+ bias), Wt (K x n) row-major,
// K <= 16 * NT. A wave owns 64 rows (4 row tiles of 16) and all K columns; per 16-deep k step each
// lane issues one 16-B load per row tile (row l&15, columns k0 + 4(l>>4) .. +3) and one per column
// tile of Wt, then 4 x v_mfma_f32_16x16x4_f32 per tile pair, component q of the loaded vectors
// feeding MFMA q: the reduction index is permuted identically for A and B, so the sum is exact.
// The VALU variant above re-reads W from LDS per element (K LDS words per X element) and spills
// to global W once n*K outgrows the LDS slice; here the W bytes per wave are 1/4 of the X bytes
// (L1/L2 hits shared by the 4 waves of a block) and the math is on the matrix cores, so the pass
// runs at the HBM rate for every K <= 32.
template <int NT, int RT, bool PIPE>
__global__ __launch_bounds__(256) void xw_mfma_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                      const float* __restrict__ Wt, int K, long ldw,
                                                      const float* __restrict__ bias, float* __restrict__ out,
                                                      long ldo, int vec, const int* __restrict__ skip) {
  if (skip && *skip) return;  // the optimiser's margins-only evaluation: no pass over X
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * (16 * RT);
  if (row0 >= m) return;
  floatx4 acc[RT][NT];
  const float* xr[RT];
  const float* wr[NT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const long r = row0 + t * 16 + li;
    xr[t] = X + (r < m ? r : m - 1) * ld;
#pragma unroll
    for (int c = 0; c < NT; ++c) acc[t][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    const int j = c * 16 + li;
    wr[c] = Wt + (long)(j < K ? j : K - 1) * ldw;
  }
  // Main loop: 64 columns per step, four 16-B loads per row tile = 256 contiguous bytes of each of
  // the wave's 64 rows in flight (DRAM page locality); the fp32 chain is folded into `tot` every
  // 256 columns so the rounding error grows with 256 + n/256 terms rather than n.
  floatx4 tot[RT][NT];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int c = 0; c < NT; ++c) tot[t][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int n64 = vec ? (n & ~63) : 0;
  int k0 = 0;
  if (n64 > 0) {
    floatx4 a[RT][4], b[NT][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int t = 0; t < RT; ++t) a[t][u] = *reinterpret_cast<const floatx4*>(xr[t] + 16 * u + 4 * g);
#pragma unroll
      for (int c = 0; c < NT; ++c) b[c][u] = *reinterpret_cast<const floatx4*>(wr[c] + 16 * u + 4 * g);
    }
    for (int step = 0; k0 < n64; ++step) {
      const int kn = k0 + 64;
      floatx4 an[RT][4], bn[NT][4];
      if (PIPE && kn < n64) {  // next step's loads in flight under this step's MFMAs
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int t = 0; t < RT; ++t) an[t][u] = *reinterpret_cast<const floatx4*>(xr[t] + kn + 16 * u + 4 * g);
#pragma unroll
          for (int c = 0; c < NT; ++c) bn[c][u] = *reinterpret_cast<const floatx4*>(wr[c] + kn + 16 * u + 4 * g);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int c = 0; c < NT; ++c)
              acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][u][q], b[c][u][q], acc[t][c], 0, 0, 0);
      if ((step & 3) == 3) {
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int c = 0; c < NT; ++c) {
            tot[t][c] += acc[t][c];
            acc[t][c] = floatx4{0.f, 0.f, 0.f, 0.f};
          }
      }
      k0 = kn;
      if (k0 >= n64) break;
      if (PIPE) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int t = 0; t < RT; ++t) a[t][u] = an[t][u];
#pragma unroll
          for (int c = 0; c < NT; ++c) b[c][u] = bn[c][u];
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int t = 0; t < RT; ++t) a[t][u] = *reinterpret_cast<const floatx4*>(xr[t] + k0 + 16 * u + 4 * g);
#pragma unroll
          for (int c = 0; c < NT; ++c) b[c][u] = *reinterpret_cast<const floatx4*>(wr[c] + k0 + 16 * u + 4 * g);
        }
      }
    }
  }
  const int nfull = vec ? (n & ~15) : 0;
  for (; k0 < nfull; k0 += 16) {
    const int kk = k0 + 4 * g;
    floatx4 a[RT], b[NT];
#pragma unroll
    for (int t = 0; t < RT; ++t) a[t] = *reinterpret_cast<const floatx4*>(xr[t] + kk);
#pragma unroll
    for (int c = 0; c < NT; ++c) b[c] = *reinterpret_cast<const floatx4*>(wr[c] + kk);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int c = 0; c < NT; ++c) acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][q], b[c][q], acc[t][c], 0, 0, 0);
  }
  for (; k0 < n; k0 += 16) {  // tail / unaligned rows: guarded scalar loads
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = k0 + 4 * g + q;
      const bool ok = kk < n;
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        const float av = ok ? xr[t][kk] : 0.f;
#pragma unroll
        for (int c = 0; c < NT; ++c) {
          const float bv = ok ? wr[c][kk] : 0.f;
          acc[t][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t][c], 0, 0, 0);
        }
      }
    }
  }
  // D layout: lane holds D[i = 4g + e][j = l & 15], e = 0..3
#pragma unroll
  for (int c = 0; c < NT; ++c) {
    const int col = c * 16 + li;
    if (col >= K) continue;
    const float bb = bias ? bias[col] : 0.f;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long r = row0 + t * 16 + 4 * g + e;
        if (r < m) out[r * ldo + col] = (tot[t][c][e] + acc[t][c][e]) + bb;
      }
  }
}

static int xw_t_launch(const float* X, long m, int n, long ld, const float* Wt, int K, long ldw, const float* bias,
                       float* out, long ldo, int variant, hipStream_t stream, const int* skip = nullptr) {
  if (m <= 0) return 0;
  if (n <= 0 || K < 1 || K > 32) return -2;
  const int vec = ((ld & 3) == 0) && ((ldw & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                  ((reinterpret_cast<uintptr_t>(Wt) & 15) == 0);
  const int rt = (variant & 1) ? 2 : 4;
  const bool pipe = (variant & 2) != 0;
  const long blocks = (m + 64 * rt - 1) / (64 * rt);
  if (blocks > 0x7fffffffL) return -2;
#define SRML_XWT(NT_, RT_, P_)                                                                                    \
  hipLaunchKernelGGL((xw_mfma_kernel<NT_, RT_, P_>), dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, Wt, K, \
                     ldw, bias, out, ldo, vec, skip)
  if (K <= 16) {
    if (rt == 4) { if (pipe) SRML_XWT(1, 4, true); else SRML_XWT(1, 4, false); }
    else { if (pipe) SRML_XWT(1, 2, true); else SRML_XWT(1, 2, false); }
  } else {
    if (rt == 4) { if (pipe) SRML_XWT(2, 4, true); else SRML_XWT(2, 4, false); }
    else { if (pipe) SRML_XWT(2, 2, true); else SRML_XWT(2, 2, false); }
  }
#undef SRML_XWT
  return srml_status();
}

SRML_API int srml_xw_t_f32(const float* X, long m, int n, long ld, const float* Wt, int K, long ldw, const float* bias,
                           float* out, long ldo, hipStream_t stream) {
  // measured at 1M x 3000 (tools/skinny_bench.py --variants): double-buffered loads win everywhere;
  // 2 row tiles per wave (more waves in flight) up to K = 12, 4 (half the Wt re-reads) above
  return xw_t_launch(X, m, n, ld, Wt, K, ldw, bias, out, ldo, K <= 12 ? 3 : 2, stream);
}

// Same, skipped on the device when *skip != 0 (the QN step's F_SKIPX word: a margins-only
// evaluation or a finished fit).
SRML_API int srml_xw_t_f32_skip(const float* X, long m, int n, long ld, const float* Wt, int K, long ldw,
                                const float* bias, float* out, long ldo, const int* skip, hipStream_t stream) {
  return xw_t_launch(X, m, n, ld, Wt, K, ldw, bias, out, ldo, K <= 12 ? 3 : 2, stream, skip);
}

// Tuning entry (tools/skinny_bench.py): variant bit 0 = 2 row tiles per wave (else 4), bit 1 =
// double-buffered loads.
SRML_API int srml_xw_t_f32_variant(const float* X, long m, int n, long ld, const float* Wt, int K, long ldw,
                                   const float* bias, float* out, long ldo, int variant, hipStream_t stream) {
  return xw_t_launch(X, m, n, ld, Wt, K, ldw, bias, out, ldo, variant, stream);
}

// ------------------------------------------------------------------------------------------
// fp64 GEMM on f64 MFMA (16x16x4): block tile 64x64, 4 waves each 32x32 (2x2 MFMA tiles), BK=16
// ------------------------------------------------------------------------------------------
namespace {
constexpr int DT = 64;
constexpr int DK = 16;
}

// v_mfma_f64_16x16x4_f64: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]; D: col=l&15, row=(l>>4)+4*r
__global__ __launch_bounds__(256) void dgemm_kernel(int M, int N, int K, double alpha, const double* __restrict__ A,
                                                    long lda, int ta, const double* __restrict__ B, long ldb, int tb,
                                                    double beta, double* __restrict__ C, long ldc, int kchunk,
                                                    double* __restrict__ ws, int lower) {
  __shared__ double As[DK][DT + 1];  // As[k][i]
  __shared__ double Bs[DK][DT + 1];  // Bs[k][j]
  const int i0 = blockIdx.y * DT, j0 = blockIdx.x * DT;
  if (lower && j0 >= i0 + DT) return;  // lower: tiles wholly above the diagonal are not computed
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wi = wid >> 1, wj = wid & 1;
  doublex4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = doublex4{0, 0, 0, 0};

  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  for (int k0 = kbeg; k0 < kend; k0 += DK) {
    // stage 64x16 of op(A) and 16x64 of op(B): 1024 elements each, 4 per thread
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      int e = t + 256 * p;
      int kk = e / DT, ii = e % DT;  // natural for ta (A^T: row k contiguous in i)
      int gi = i0 + ii, gk = k0 + kk;
      double va = 0.0;
      if (ta) {
        if (gi < M && gk < kend) va = A[(long)gk * lda + gi];
      } else {
        int kk2 = e % DK, ii2 = e / DK;  // A row-major: k contiguous
        gi = i0 + ii2; gk = k0 + kk2;
        if (gi < M && gk < kend) va = A[(long)gi * lda + gk];
        kk = kk2; ii = ii2;
      }
      As[kk][ii] = va;
      int jj = e % DT, kb = e / DT;
      int gj = j0 + jj, gkb = k0 + kb;
      double vb = 0.0;
      if (!tb) {
        if (gj < N && gkb < kend) vb = B[(long)gkb * ldb + gj];
      } else {
        int kb2 = e % DK, jj2 = e / DK;  // B^T: B stored N x K row-major
        gj = j0 + jj2; gkb = k0 + kb2;
        if (gj < N && gkb < kend) vb = B[(long)gj * ldb + gkb];
        kb = kb2; jj = jj2;
      }
      Bs[kb][jj] = vb;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < DK / 4; ++ks) {
      const int k = ks * 4 + (lane >> 4);
      double a0 = As[k][wi * 32 + (lane & 15)];
      double a1 = As[k][wi * 32 + 16 + (lane & 15)];
      double b0 = Bs[k][wj * 32 + (lane & 15)];
      double b1 = Bs[k][wj * 32 + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int gi = i0 + wi * 32 + mt * 16 + (lane >> 4) + 4 * r;
        int gj = j0 + wj * 32 + nt * 16 + (lane & 15);
        if (gi < M && gj < N) {
          if (ws) {
            ws[((long)blockIdx.z * M + gi) * N + gj] = acc[mt][nt][r];
          } else {
            double* c = &C[(long)gi * ldc + gj];
            *c = alpha * acc[mt][nt][r] + (beta != 0.0 ? beta * *c : 0.0);
          }
        }
      }
}

// C = alpha * sum_z ws[z] + beta C, splits folded in index order (deterministic)
__global__ __launch_bounds__(256) void dgemm_fold_kernel(int M, int N, int splits, double alpha,
                                                         const double* __restrict__ ws, double beta,
                                                         double* __restrict__ C, long ldc) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)M * N) return;
  const long MN = (long)M * N;
  double s = 0.0;
  for (int z = 0; z < splits; ++z) s += ws[z * MN + idx];
  const int i = (int)(idx / N), j = (int)(idx % N);
  double* c = &C[(long)i * ldc + j];
  *c = alpha * s + (beta != 0.0 ? beta * *c : 0.0);
}

SRML_API int srml_dgemm(int ta, int tb, int M, int N, int K, double alpha, const double* A, long lda, const double* B,
                        long ldb, double beta, double* C, long ldc, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  dim3 grid(ceil_div(N, DT), ceil_div(M, DT), 1);
  hipLaunchKernelGGL(dgemm_kernel, grid, dim3(256), 0, stream, M, N, K, alpha, A, lda, ta, B, ldb, tb, beta, C, ldc,
                     K > 0 ? K : 1, (double*)nullptr, 0);
  return srml_status();
}

// C = alpha A A^T + beta C (A: M x K row-major) on the 64 x 64 tiles that touch the lower
// triangle only (the entries above the diagonal of diagonal tiles are computed too): the
// Cholesky trailing update, whose upper triangle is never read.
SRML_API int srml_dgemm_syrk_lower(int M, int K, double alpha, const double* A, long lda, double beta, double* C,
                                   long ldc, hipStream_t stream) {
  if (M <= 0) return 0;
  dim3 grid(ceil_div(M, DT), ceil_div(M, DT), 1);
  hipLaunchKernelGGL(dgemm_kernel, grid, dim3(256), 0, stream, M, M, K, alpha, A, lda, 0, A, lda, 1, beta, C, ldc,
                     K > 0 ? K : 1, (double*)nullptr, 1);
  return srml_status();
}

// Split-K variant: `splits` slices of K (multiples of the 16-deep k-step) into `ws`
// (splits * M * N doubles), then the ordered fold.
SRML_API int srml_dgemm_splitk(int ta, int tb, int M, int N, int K, double alpha, const double* A, long lda,
                               const double* B, long ldb, double beta, double* C, long ldc, int splits, double* ws,
                               hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (splits <= 1 || ws == nullptr) return srml_dgemm(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, stream);
  int kchunk = (K + splits - 1) / splits;
  kchunk = ((kchunk + DK - 1) / DK) * DK;
  splits = (K + kchunk - 1) / kchunk;
  dim3 grid(ceil_div(N, DT), ceil_div(M, DT), (unsigned)splits);
  hipLaunchKernelGGL(dgemm_kernel, grid, dim3(256), 0, stream, M, N, K, alpha, A, lda, ta, B, ldb, tb, beta, C, ldc,
                     kchunk, ws, 0);
  int st = srml_status();
  if (st) return st;
  const long MN = (long)M * N;
  hipLaunchKernelGGL(dgemm_fold_kernel, dim3(ceil_div(MN, 256)), dim3(256), 0, stream, M, N, splits, alpha, ws, beta,
                     C, ldc);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// sign flip (one wave per column)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sign_flip_kernel(double* __restrict__ U, int rows, int cols, long ld) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= cols) return;
  double best = -1.0, bval = 0.0;
  int bidx = 0x7fffffff;
  for (int r = lane; r < rows; r += 64) {
    double v = U[(long)r * ld + c];
    double a = fabs(v);
    if (a > best) { best = a; bval = v; bidx = r; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ob = __shfl_xor(best, o, 64);
    double ov = __shfl_xor(bval, o, 64);
    int oi = __shfl_xor(bidx, o, 64);
    if (ob > best || (ob == best && oi < bidx)) { best = ob; bval = ov; bidx = oi; }
  }
  if (bval < 0.0) {
    for (int r = lane; r < rows; r += 64) U[(long)r * ld + c] = -U[(long)r * ld + c];
  }
}

SRML_API int srml_sign_flip_f64(double* U, int rows, int cols, long ld, hipStream_t stream) {
  if (cols <= 0) return 0;
  hipLaunchKernelGGL(sign_flip_kernel, dim3(ceil_div(cols, 4)), dim3(256), 0, stream, U, rows, cols, ld);
  return srml_status();
}
