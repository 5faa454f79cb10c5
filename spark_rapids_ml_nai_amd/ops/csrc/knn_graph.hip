// All-points approximate k-nearest-neighbour graph over IVF lists (UMAP / kNN graph at scale).
//
// The rows are k-means-bucketed into contiguous inverted lists (items sorted by list). A block
// owns one tile of <= 128 query rows that all belong to list c, and sweeps the items of the
// nprobe lists nearest to c's centroid (probes[c]) in 128-row tiles: MFMA distance tile
// (exact fp32 `v_mfma_f32_32x32x2_f32`, double-buffered LDS staging shared with the exact kNN
// kernel) -> partial distances ||i||^2 - 2 q.i through LDS -> per-row sorted top-k insertion.
// Because every query of a tile probes the same lists, the whole search is dense GEMM-shaped
// work on the matrix cores (the per-query IVF scan kernel is SIMT dot products); the price is
// probing by the query's *list* instead of by the query itself, which the caller compensates
// with a few extra probes. Replaces cuML UMAP's brute-force / NN-descent graph build for the
// north-star 20M x 128 configuration (BASELINE.json config 5; reference umap.py:924-958 calls
// cuML UMAP's own kNN on one GPU).
//
// Tiles are XCD-remapped so consecutive tiles of one list (same probe set, same item rows) run
// on one XCD and share its L2. Output positions are row indices in the sorted (list) order.
#include "common.h"

#include "tile.h"

namespace {
using namespace srml_tile;
constexpr int KG_KMAX = 64;

template <bool VEC>
__global__ __launch_bounds__(256, 1) void knn_lists_kernel(const float* __restrict__ X, int n, long ld,
                                                           const float* __restrict__ xnorm,
                                                           const long long* __restrict__ list_off,
                                                           const int* __restrict__ probes, int nprobe,
                                                           const long long* __restrict__ tile_q0,
                                                           const int* __restrict__ tile_list, int ntiles, int k,
                                                           float* __restrict__ out_d, int* __restrict__ out_i) {
  constexpr int BM = 128, BN = 128, MT = 2, NT = 2;
  union Smem {
    struct {
      float Xs[2][BM][PADK];
      float Cs[2][BN][PADK];
    } st;
    float D[BM][BN + 1];
  };
  __shared__ Smem sm;
  __shared__ float topd[BM][KG_KMAX + 1];
  __shared__ int topi[BM][KG_KMAX + 1];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  if (b >= ntiles) return;  // block-uniform
  const int c = tile_list[b];
  const long q0 = tile_q0[b];
  const long q1 = min(q0 + (long)BM, (long)list_off[c + 1]);
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lk = lane >> 5, li = lane & 31;
  for (int i = t; i < BM * (KG_KMAX + 1); i += 256) {
    (&topd[0][0])[i] = __builtin_huge_valf();
    (&topi[0][0])[i] = -1;
  }
  const int nk = (n + BK - 1) / BK;
  for (int p = 0; p < nprobe; ++p) {
    const int l = probes[(long)c * nprobe + p];
    if (l < 0) continue;
    const long s = list_off[l], e = list_off[l + 1];
    for (long c0 = s; c0 < e; c0 += BN) {
      floatx16 acc[MT][NT];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int bb = 0; bb < NT; ++bb)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[a][bb][r] = 0.f;
      RowTile<BM, VEC> xt;
      RowTile<BN, VEC> ct;
      xt.load(X, ld, q1, n, q0, 0);
      ct.load(X, ld, e, n, c0, 0);
      __syncthreads();  // the previous tile's top-k scan is done with sm.D
      xt.store(sm.st.Xs[0]);
      ct.store(sm.st.Cs[0]);
      __syncthreads();
      int cur = 0;
      for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + 1 < nk;
        if (more) {
          xt.load(X, ld, q1, n, q0, (kt + 1) * BK);
          ct.load(X, ld, e, n, c0, (kt + 1) * BK);
        }
#pragma unroll
        for (int kk = 0; kk < BK / 2; ++kk) {
          const int kx = 2 * kk + lk;
          float av[MT], bv[NT];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) av[mt] = sm.st.Xs[cur][wm * MT * 32 + mt * 32 + li][kx];
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) bv[nt] = sm.st.Cs[cur][wn * NT * 32 + nt * 32 + li][kx];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mt], bv[nt], acc[mt][nt], 0, 0, 0);
        }
        if (more) {
          xt.store(sm.st.Xs[cur ^ 1]);
          ct.store(sm.st.Cs[cur ^ 1]);
        }
        __syncthreads();
        cur ^= 1;
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int cl = wn * NT * 32 + nt * 32 + li;
        const long cg = c0 + cl;
        const float in = cg < e ? xnorm[cg] : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = wm * MT * 32 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
            sm.D[rl][cl] = cg < e ? fmaf(-2.f, acc[mt][nt][r], in) : __builtin_huge_valf();
          }
      }
      __syncthreads();
      if (t < BM) {
        float thr = topd[t][k - 1];
        const int ncol = (int)min((long)BN, e - c0);
        for (int cc = 0; cc < ncol; ++cc) {
          const float d = sm.D[t][cc];
          if (d < thr) {
            int q = k - 1;
            while (q > 0 && topd[t][q - 1] > d) {
              topd[t][q] = topd[t][q - 1];
              topi[t][q] = topi[t][q - 1];
              --q;
            }
            topd[t][q] = d;
            topi[t][q] = (int)(c0 + cc);
            thr = topd[t][k - 1];
          }
        }
      }
    }
  }
  __syncthreads();
  if (t < BM && q0 + t < q1) {
    const long base = (q0 + t) * (long)k;
    for (int j = 0; j < k; ++j) {
      out_d[base + j] = topd[t][j];
      out_i[base + j] = topi[t][j];
    }
  }
}
}  // namespace

// X: N x n rows sorted by list (row-major, leading dimension ld); xnorm: ||x||^2 of those rows;
// list_off: nlist + 1 offsets (int64); probes: nlist x nprobe list ids (int32, -1 = none);
// tiles: (tile_q0[i], tile_list[i]) = first sorted row of a <= 128-row query tile and its list.
// out_d / out_i: N x k (only the rows of the given tiles are written): ||i||^2 - 2 q.i (without
// the ||q||^2 term) and item positions in the sorted order, ascending.
SRML_API int srml_knn_lists_f32(const float* X, int n, long ld, const float* xnorm, const long long* list_off,
                                const int* probes, int nprobe, const long long* tile_q0, const int* tile_list,
                                int ntiles, int k, float* out_d, int* out_i, hipStream_t stream) {
  if (ntiles <= 0) return 0;
  if (k < 1 || k > KG_KMAX) return -8;
  const bool vec = ((ld & 3) == 0) && ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(knn_lists_kernel<true>, dim3((unsigned)ntiles), dim3(256), 0, stream, X, n, ld, xnorm, list_off,
                       probes, nprobe, tile_q0, tile_list, ntiles, k, out_d, out_i);
  else
    hipLaunchKernelGGL(knn_lists_kernel<false>, dim3((unsigned)ntiles), dim3(256), 0, stream, X, n, ld, xnorm,
                       list_off, probes, nprobe, tile_q0, tile_list, ntiles, k, out_d, out_i);
  return srml_status();
}
