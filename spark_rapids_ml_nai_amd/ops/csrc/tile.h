// Shared MFMA operand staging for the distance-GEMM kernels (KMeans, kNN, DBSCAN).
#pragma once
#include "common.h"

namespace srml_tile {
constexpr int BK = 32;
constexpr int PADK = BK + 1;

__device__ __forceinline__ unsigned orderable(float f) {
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unorderable(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// ROWS x 32 tile of a row-major matrix, staged through registers. load(): branch-free (clamped
// addresses + select after the load) so the next k-tile's loads stay in flight under the MFMAs;
// store(): scalar ds_writes into the padded [row][33] LDS image (conflict-free operand reads).
template <int ROWS, bool VEC>
struct RowTile {
  static constexpr int PER = (ROWS * 8 + 255) / 256;
  floatx4 v[PER];
  unsigned okmask;  // bit 4p+q: element valid (row and column in range)

  // issue the loads only; masking happens in store() so no wait is emitted before the MFMAs
  __device__ __forceinline__ void load(const float* __restrict__ A, long lda, long nrows, int ncols, long row0,
                                       int k0) {
    const int t = threadIdx.x;
    okmask = 0u;
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int idx = t + 256 * p;
      const int rr = (idx >> 3) % ROWS;
      const int c4 = (idx & 7) * 4;
      const long r = row0 + rr;
      const bool okr = (idx < ROWS * 8) && (r < nrows);
      const float* row = A + (okr ? r : 0) * lda;
      const int kc = k0 + c4;
      if (VEC) {
        const bool okk = kc < ncols;  // ncols % 4 == 0 on the VEC path
        v[p] = *reinterpret_cast<const floatx4*>(row + (okk ? kc : 0));
        okmask |= (okr && okk) ? (0xFu << (4 * p)) : 0u;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool okk = kc + q < ncols;
          v[p][q] = row[okk ? kc + q : 0];
          okmask |= (okr && okk) ? (1u << (4 * p + q)) : 0u;
        }
      }
    }
  }

  __device__ __forceinline__ void store(float (*dst)[PADK]) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int idx = t + 256 * p;
      if (PER * 256 == ROWS * 8 || idx < ROWS * 8) {
        const int rr = idx >> 3;
        const int c4 = (idx & 7) * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[rr][c4 + q] = ((okmask >> (4 * p + q)) & 1u) ? v[p][q] : 0.f;
      }
    }
  }
};

}  // namespace srml_tile

namespace srml_tile {
// Double-buffered LDS staging for one 128 x 128 distance tile.
struct Stage128 {
  float Xs[2][128][PADK];
  float Cs[2][128][PADK];
};

// acc[mt][nt] (wave (wm, wn) of a 2 x 2 wave grid, 2 x 2 32x32 MFMA tiles each) += A[a0:a0+128] . B[b0:b0+128]^T
// over the full feature dimension n. Rows beyond na / nb read as zeros. Ends with a __syncthreads so
// the caller may reuse the staging LDS immediately.
template <bool VEC>
__device__ __forceinline__ void gemm_tile_128(const float* __restrict__ A, long lda, long na, long a0,
                                              const float* __restrict__ B, long ldb, long nb, long b0, int n,
                                              Stage128& st, floatx16 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int nk = (n + BK - 1) / BK;
  RowTile<128, VEC> xt;
  RowTile<128, VEC> ct;
  xt.load(A, lda, na, n, a0, 0);
  ct.load(B, ldb, nb, n, b0, 0);
  xt.store(st.Xs[0]);
  ct.store(st.Cs[0]);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      xt.load(A, lda, na, n, a0, (kt + 1) * BK);
      ct.load(B, ldb, nb, n, b0, (kt + 1) * BK);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int kx = 2 * kk + lk;
      float a[2], b[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) a[mt] = st.Xs[cur][wm * 64 + mt * 32 + li][kx];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) b[nt] = st.Cs[cur][wn * 64 + nt * 32 + li][kx];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
    if (more) {
      xt.store(st.Xs[cur ^ 1]);
      ct.store(st.Cs[cur ^ 1]);
    }
    __syncthreads();
    cur ^= 1;
  }
}

// C/D layout of the 32x32x2 f32 MFMA for wave (wm, wn): local row / column of accumulator element r.
__device__ __forceinline__ int acc_row(int mt, int r) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  return (wid >> 1) * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int acc_col(int nt) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  return (wid & 1) * 64 + nt * 32 + (lane & 31);
}
}  // namespace srml_tile
