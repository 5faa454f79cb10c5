// fp64-input kernels (``float32_inputs=False``): the paths that used to drop to library GEMMs.
//
//  * srml_nearest_centroid_f64 — fused fp64 distance GEMM + arg-min on the f64 matrix cores
//      (`v_mfma_f64_16x16x4_f64`). Block = 64 rows x ALL centroids: the block walks the centroid
//      tiles (64 per tile) itself and keeps each row's running (min, arg-min) in registers, so
//      the comparison is exact in fp64 (no packed 32-bit key, no cross-block atomics) and
//      labels / distances are written once. The X panel is re-read per centroid tile from L2 /
//      the 256 MB MALL; grid = ceil(m/64) blocks (>> 256 CUs at the sizes that matter).
//      Reference: cuML KMeans fp64 path (fusedL2NN<double>).
//  * srml_row_sqnorm_f64 — ||x_r||^2 in fp64 (wave per row, DPP wave reduction).
#include "common.h"

namespace {
constexpr int NB = 64;   // rows per block
constexpr int NC = 64;   // centroids per tile
constexpr int NK = 16;   // k-step

// MFMA f64 16x16x4: A[i = l&15][k = l>>4], B[k = l>>4][j = l&15]; D: col = l&15, row = (l>>4) + 4r
__global__ __launch_bounds__(256) void nearest_centroid_f64_kernel(const double* __restrict__ X, long m, int n, long ldx,
                                                                   const double* __restrict__ C, int k, long ldc,
                                                                   const double* __restrict__ cnorm,
                                                                   const double* __restrict__ xnorm,
                                                                   int* __restrict__ labels, float* __restrict__ dist,
                                                                   double* __restrict__ dist64) {
  __shared__ double Xs[NK][NB + 1];
  __shared__ double Cs[NK][NC + 1];
  __shared__ double red_v[2][NB];
  __shared__ int red_i[2][NB];
  const long row0 = (long)xcd_remap(blockIdx.x, gridDim.x) * NB;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wi = wid >> 1, wj = wid & 1;

  double bv[2][4];
  int bi[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) { bv[a][r] = __builtin_huge_val(); bi[a][r] = 0x7fffffff; }

  for (int j0 = 0; j0 < k; j0 += NC) {
    doublex4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = doublex4{0, 0, 0, 0};
    for (int k0 = 0; k0 < n; k0 += NK) {
      // 64 x 16 panels of X and C: thread t loads 4 elements of each, k fastest (coalesced rows)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int e = t + 256 * p;
        const int kk = e % NK, ii = e / NK;
        const long gr = row0 + ii;
        const int gk = k0 + kk;
        Xs[kk][ii] = (gr < m && gk < n) ? X[gr * ldx + gk] : 0.0;
        const int gc = j0 + ii;
        Cs[kk][ii] = (gc < k && gk < n) ? C[(long)gc * ldc + gk] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < NK / 4; ++ks) {
        const int kq = ks * 4 + (lane >> 4);
        const double a0 = Xs[kq][wi * 32 + (lane & 15)];
        const double a1 = Xs[kq][wi * 32 + 16 + (lane & 15)];
        const double b0 = Cs[kq][wj * 32 + (lane & 15)];
        const double b1 = Cs[kq][wj * 32 + 16 + (lane & 15)];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
      }
      __syncthreads();
    }
    // epilogue: partial distance ||c||^2 - 2 x.c, running arg-min per owned row (ties -> lower index)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int j = j0 + wj * 32 + nt * 16 + (lane & 15);
      if (j < k) {
        const double cn = cnorm[j];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double d = cn - 2.0 * acc[mt][nt][r];
            if (d < bv[mt][r] || (d == bv[mt][r] && j < bi[mt][r])) { bv[mt][r] = d; bi[mt][r] = j; }
          }
      }
    }
  }
  // reduce over the 16 lanes holding one row (same lane>>4), then over the two column waves
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double v = bv[mt][r];
      int i = bi[mt][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const double ov = __shfl_xor(v, o, 64);
        const int oi = __shfl_xor(i, o, 64);
        if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }
      }
      if ((lane & 15) == 0) {
        const int lr = wi * 32 + mt * 16 + (lane >> 4) + 4 * r;
        red_v[wj][lr] = v;
        red_i[wj][lr] = i;
      }
    }
  __syncthreads();
  if (t < NB) {
    const long gr = row0 + t;
    if (gr < m) {
      double v = red_v[0][t];
      int i = red_i[0][t];
      if (red_v[1][t] < v || (red_v[1][t] == v && red_i[1][t] < i)) { v = red_v[1][t]; i = red_i[1][t]; }
      const double d = v + xnorm[gr];
      const double dc = d > 0.0 ? d : 0.0;
      labels[gr] = i;
      dist[gr] = (float)dc;
      if (dist64) dist64[gr] = dc;
    }
  }
}

__global__ __launch_bounds__(256) void row_sqnorm_f64_kernel(const double* __restrict__ X, long m, int n, long ld,
                                                             double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  for (long r = wave; r < m; r += nw) {
    const double* row = X + r * ld;
    double s = 0.0;
    for (int d = lane; d < n; d += 64) s = fma(row[d], row[d], s);
    s = wave_sum(s);
    if (lane == 0) out[r] = s;
  }
}
}  // namespace

SRML_API int srml_row_sqnorm_f64(const double* X, long m, int n, long ld, double* out, hipStream_t stream) {
  if (m <= 0) return 0;
  long blocks = (m + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(row_sqnorm_f64_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, out);
  return srml_status();
}

// labels (int32 [m]), dist (fp32 [m], ||x - c||^2 >= 0), optional dist64 (fp64 [m]).
SRML_API int srml_nearest_centroid_f64(const double* X, long m, int n, long ldx, const double* C, int k, long ldc,
                                       const double* cnorm, const double* xnorm, int* labels, float* dist,
                                       double* dist64, hipStream_t stream) {
  if (m <= 0) return 0;
  if (k <= 0 || n <= 0 || !xnorm || !cnorm) return -1;
  const long blocks = (m + NB - 1) / NB;
  if (blocks > 0x7fffffffL) return -1;
  hipLaunchKernelGGL(nearest_centroid_f64_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ldx, C, k, ldc,
                     cnorm, xnorm, labels, dist, dist64);
  return srml_status();
}
