// Gram / covariance SYRK on the MFMA matrix cores:  C += (X - mu)^T (X - mu)
//
// The hot primitive of PCA, LinearRegression (normal equations) and Ridge (reference: cuML
// PCAMG / LinearRegressionMG covariance, and the JNI `dgemmCov` cuBLAS call,
// jvm/native/src/rapidsml_jni.cu:109-127). MI355X design:
//  * exact-fp32 MFMA `v_mfma_f32_32x32x2_f32` (gfx950 has no xf32; f32-in MFMA runs at the
//    f32 vector peak, 64 FLOP/clk/SIMD, with one VGPR per operand and the VALU left free);
//  * only upper-triangle 128x128 output tiles are computed (SYRK halves the FLOPs), mirrored by
//    a tiny kernel afterwards;
//  * split-K over rows for parallelism (tiles x row-chunks >> 256 CUs); partial tiles are folded
//    into an fp64 C with global fp64 atomics (two 256-B row segments per wave instruction, the
//    full-rate atomic shape), so the across-chunk / across-rank sum is fp64;
//  * mean centring fused into the LDS staging pass (no centred copy of X is ever written);
//  * register-staged double-buffered LDS: tile t+1's global loads are in flight while the MFMAs
//    of tile t run; one barrier per k-tile;
//  * XCD-aware block remap so concurrently running tiles of one row-chunk share the XCD L2.
#include "common.h"

namespace {
constexpr int BT = 128;  // output tile edge
constexpr int BK = 32;   // rows per k-step
constexpr int NTHREADS = 256;

struct TileStage {
  floatx4 a[4];
  floatx4 b[4];
  floatx4 mua, mub;
  unsigned okmask;  // bits 0..15: A elements valid, 16..31: B elements valid
};

// Branch-free staging: every lane always issues its loads from a clamped, valid address; masking
// and mean-centring are applied in store_stage() (after the MFMAs of the current tile), so hipcc
// emits no per-load branch or early vmcnt wait and the next tile's loads stay in flight.
template <bool CENTER, bool VEC>
__device__ __forceinline__ void load_stage(const float* __restrict__ X, long ld, int n, long r_base, long r_end,
                                           int i0, int j0, const float* __restrict__ mu, TileStage& st) {
  const int t = threadIdx.x;
  const int c4 = (t & 31) * 4;
  const int ca = i0 + c4, cb = j0 + c4;
  const bool oka = ca < n, okb = cb < n;  // n % 4 == 0 on the VEC path
  const int cac = oka ? ca : 0, cbc = okb ? cb : 0;
  unsigned mask = 0u;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int rr = (t >> 5) + 8 * p;
    const long r = r_base + rr;
    const bool okr = r < r_end;
    const float* row = X + (okr ? r : r_end - 1) * ld;
    if (VEC) {
      st.a[p] = *reinterpret_cast<const floatx4*>(row + cac);
      st.b[p] = *reinterpret_cast<const floatx4*>(row + cbc);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        st.a[p][q] = row[min(ca + q, n - 1)];
        st.b[p][q] = row[min(cb + q, n - 1)];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ina = okr && (VEC ? oka : (ca + q < n));
      const bool inb = okr && (VEC ? okb : (cb + q < n));
      mask |= (ina ? 1u : 0u) << (4 * p + q);
      mask |= (inb ? 1u : 0u) << (16 + 4 * p + q);
    }
  }
  st.okmask = mask;
}

template <bool CENTER>
__device__ __forceinline__ void load_mean(const float* __restrict__ mu, int n, int i0, int j0, TileStage& st) {
  const int c4 = (threadIdx.x & 31) * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    st.mua[q] = CENTER ? mu[min(i0 + c4 + q, n - 1)] : 0.f;
    st.mub[q] = CENTER ? mu[min(j0 + c4 + q, n - 1)] : 0.f;
  }
}

template <bool CENTER>
__device__ __forceinline__ void store_stage(float (*As)[BT], float (*Bs)[BT], bool diag, const TileStage& st) {
  const int t = threadIdx.x;
  const int c4 = (t & 31) * 4;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int rr = (t >> 5) + 8 * p;
    floatx4 a, b;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = ((st.okmask >> (4 * p + q)) & 1u) ? (CENTER ? st.a[p][q] - st.mua[q] : st.a[p][q]) : 0.f;
      b[q] = ((st.okmask >> (16 + 4 * p + q)) & 1u) ? (CENTER ? st.b[p][q] - st.mub[q] : st.b[p][q]) : 0.f;
    }
    *reinterpret_cast<floatx4*>(&As[rr][c4]) = a;
    if (!diag) *reinterpret_cast<floatx4*>(&Bs[rr][c4]) = b;
  }
}

template <bool CENTER, bool VEC>
__global__ __launch_bounds__(NTHREADS, 2) void gram_f32_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                               const float* __restrict__ mu, double* __restrict__ C,
                                                               int T, int ntiles, long rows_per_chunk,
                                                               double* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) float As[2][BK][BT];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BT];

  const int nblocks = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nblocks);
  const int tile = bid % ntiles;
  const int chunk = bid / ntiles;
  // tile -> (ti, tj), ti <= tj, row-major over the upper triangle (scalar loop, T <= ~100)
  int ti = 0, rem = tile;
  while (rem >= T - ti) { rem -= T - ti; ++ti; }
  const int tj = ti + rem;
  const int i0 = ti * BT, j0 = tj * BT;
  const bool diag = (ti == tj);

  const long r_begin = (long)chunk * rows_per_chunk;
  const long r_end = min(m, r_begin + rows_per_chunk);
  if (r_begin >= r_end) return;
  const int nk = (int)((r_end - r_begin + BK - 1) / BK);

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;   // 4 waves: 2 x 2 over the 128x128 tile
  const int wi = wid >> 1, wj = wid & 1;
  const int li = lane & 31, lk = lane >> 5;

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  TileStage st;
  load_mean<CENTER>(mu, n, i0, j0, st);
  load_stage<CENTER, VEC>(X, ld, n, r_begin, r_end, i0, j0, mu, st);
  store_stage<CENTER>(As[0], Bs[0], diag, st);
  __syncthreads();

  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = (kt + 1 < nk);
    if (more) load_stage<CENTER, VEC>(X, ld, n, r_begin + (long)(kt + 1) * BK, r_end, i0, j0, mu, st);

    const float(*A)[BT] = As[cur];
    const float(*B)[BT] = diag ? As[cur] : Bs[cur];
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int k = 2 * kk + lk;
      float a0 = A[k][wi * 64 + li];
      float a1 = A[k][wi * 64 + 32 + li];
      float b0 = B[k][wj * 64 + li];
      float b1 = B[k][wj * 64 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) store_stage<CENTER>(As[cur ^ 1], Bs[cur ^ 1], diag, st);
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: C/D map of the 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int gj = j0 + wj * 64 + nt * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gi = i0 + wi * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (gi < n && gj < n && gi <= gj) {
          if (ws)
            ws[((long)chunk * n + gi) * n + gj] = (double)acc[mt][nt][r];
          else
            atomicAdd(&C[(long)gi * n + gj], (double)acc[mt][nt][r]);
        }
      }
    }
  }
}

// C[i][j] (i <= j) += sum over chunks in index order (deterministic mode)
__global__ void gram_fold_kernel(const double* __restrict__ ws, int chunks, int n, double* __restrict__ C) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nn = (long)n * n;
  if (idx >= nn) return;
  const int i = (int)(idx / n), j = (int)(idx % n);
  if (i > j) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += ws[c * nn + idx];
  C[idx] += s;
}

__global__ void mirror_upper_kernel(double* __restrict__ C, int n) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)n * n;
  if (idx >= total) return;
  int i = (int)(idx / n), j = (int)(idx % n);
  if (i > j) C[idx] = C[(long)j * n + i];
}
}  // namespace

// C (n x n fp64, zeroed by the caller or holding a running sum) += (X-mu)^T (X-mu), upper triangle.
// ws != null (deterministic mode): at most ws_chunks row chunks, each storing its partial tiles
// into ws[chunk] (ws_chunks * n * n fp64) with plain stores, folded into C in chunk order — the
// same fp32-per-chunk / fp64-across-chunk precision as the atomic path, bit-reproducible.
SRML_API int srml_gram_f32_ex(const float* X, long m, int n, long ld, const float* mu, double* C, double* ws,
                              int ws_chunks, hipStream_t stream) {
  const int max_chunks = ws ? ws_chunks : 0;
  if (n <= 0) return 0;
  if (m > 0) {
    const int T = (n + BT - 1) / BT;
    const int ntiles = T * (T + 1) / 2;
    // split rows so that tiles*chunks ~ 2-4 blocks per CU, chunks >= 1 k-step each
    long want_blocks = 2048;
    long chunks = (want_blocks + ntiles - 1) / ntiles;
    long ksteps = (m + BK - 1) / BK;
    if (chunks > ksteps) chunks = ksteps;
    if (max_chunks > 0 && chunks > max_chunks) chunks = max_chunks;
    if (chunks < 1) chunks = 1;
    long rows_per_chunk = (m + chunks - 1) / chunks;
    rows_per_chunk = ((rows_per_chunk + BK - 1) / BK) * BK;
    chunks = (m + rows_per_chunk - 1) / rows_per_chunk;
    const unsigned nblocks = (unsigned)(ntiles * chunks);
    const bool vec = ((ld & 3) == 0) && ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
    if (mu) {
      if (vec)
        hipLaunchKernelGGL((gram_f32_kernel<true, true>), dim3(nblocks), dim3(NTHREADS), 0, stream, X, m, n, ld, mu, C, T,
                           ntiles, rows_per_chunk, ws);
      else
        hipLaunchKernelGGL((gram_f32_kernel<true, false>), dim3(nblocks), dim3(NTHREADS), 0, stream, X, m, n, ld, mu, C,
                           T, ntiles, rows_per_chunk, ws);
    } else {
      if (vec)
        hipLaunchKernelGGL((gram_f32_kernel<false, true>), dim3(nblocks), dim3(NTHREADS), 0, stream, X, m, n, ld, mu, C,
                           T, ntiles, rows_per_chunk, ws);
      else
        hipLaunchKernelGGL((gram_f32_kernel<false, false>), dim3(nblocks), dim3(NTHREADS), 0, stream, X, m, n, ld, mu, C,
                           T, ntiles, rows_per_chunk, ws);
    }
    int st = srml_status();
    if (st) return st;
    if (ws) {
      const long nn = (long)n * n;
      hipLaunchKernelGGL(gram_fold_kernel, dim3(ceil_div(nn, 256)), dim3(256), 0, stream, ws, (int)chunks, n, C);
      st = srml_status();
      if (st) return st;
    }
  }
  return 0;
}

SRML_API int srml_gram_f32(const float* X, long m, int n, long ld, const float* mu, double* C, hipStream_t stream) {
  return srml_gram_f32_ex(X, m, n, ld, mu, C, nullptr, 0, stream);
}

SRML_API int srml_mirror_upper_f64(double* C, int n, hipStream_t stream) {
  long total = (long)n * n;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(mirror_upper_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, C, n);
  return srml_status();
}
