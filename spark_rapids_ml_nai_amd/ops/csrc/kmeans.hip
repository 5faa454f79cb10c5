// KMeans (and nearest-centroid) kernels.
//
// srml_nearest_centroid_f32: fused distance GEMM + arg-min. For every row x and centroid c the
//   MFMA tile computes x·c (exact f32 `v_mfma_f32_32x32x2_f32`); the epilogue turns it into the
//   partial squared distance ||c||^2 - 2 x·c and reduces the arg-min over the tile's columns with
//   wave64 shuffles; per-row results from different centroid tiles are merged with ONE 64-bit
//   atomicMin on a packed (orderable-dist << 32 | index) key. The m x k distance matrix is never
//   materialised (reference: cuML KMeansMG / RAFT fusedL2NN).
//   Grid: (row tiles) x (centroid tiles), centroid tile fastest and XCD-remapped, so the blocks
//   that share one X row tile run on the same XCD and read it from that L2 (HBM traffic for X
//   ~1x instead of k/BN x). Two tile shapes: 128x128 (large k) and 256x32 (small k, e.g. the
//   k=20 north-star config, where a 128-wide centroid tile would idle 84% of the MFMAs).
// srml_nn_finalize: unpack keys -> int32 labels and full squared distances (+||x||^2, >= 0).
// srml_kmeans_accumulate_f32: per-cluster sums / counts for the Lloyd update.
//   small k*n: block-private sums in LDS (ds_add_f32), flushed with fp64 global atomics;
//   large k*n: wave-per-row fp32 global atomics, 256 contiguous bytes per atomic instruction
//   (the full-rate atomic shape on MI355X).
#include <cstdlib>
#include <cstring>

#include "common.h"

#include "tile.h"

namespace {
using namespace srml_tile;

// BM x BN block tile, WM x WN waves (WM*WN = 4), each wave MT x NT tiles of 32x32
template <int BM, int BN, int WM, int MT, int NT, bool VEC>
__global__ __launch_bounds__(256, 2) void nearest_centroid_kernel(const float* __restrict__ X, long m, int n, long ldx,
                                                                  const float* __restrict__ C, int k, long ldc,
                                                                  const float* __restrict__ cnorm,
                                                                  unsigned long long* __restrict__ best,
                                                                  int n_ctiles) {
  constexpr int WN = 4 / WM;
  __shared__ float Xs[2][BM][PADK];
  __shared__ float Cs[2][BN][PADK];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const long rtile = bid / n_ctiles;
  const int ctile = bid % n_ctiles;
  const long row0 = rtile * BM;
  const int col0 = ctile * BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int li = lane & 31, lk = lane >> 5;

  floatx16 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = (n + BK - 1) / BK;
  RowTile<BM, VEC> xt;
  RowTile<BN, VEC> ct;
  xt.load(X, ldx, m, n, row0, 0);
  ct.load(C, ldc, k, n, col0, 0);
  xt.store(Xs[0]);
  ct.store(Cs[0]);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {  // issue next tile's global loads; they land while this tile's MFMAs run
      xt.load(X, ldx, m, n, row0, (kt + 1) * BK);
      ct.load(C, ldc, k, n, col0, (kt + 1) * BK);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int kx = 2 * kk + lk;
      float a[MT], b[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = Xs[cur][wm * MT * 32 + mt * 32 + li][kx];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) b[nt] = Cs[cur][wn * NT * 32 + nt * 32 + li][kx];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          if (col0 + wn * NT * 32 + nt * 32 < k)  // wave-uniform: a tile of padding centres is skipped
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
    if (more) {
      xt.store(Xs[cur ^ 1]);
      ct.store(Cs[cur ^ 1]);
    }
    __syncthreads();
    cur ^= 1;
  }

  // epilogue: per-row arg-min over this wave's columns, then one packed atomicMin per row
  float cn[NT];
  int cj[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    cj[nt] = col0 + wn * NT * 32 + nt * 32 + li;
    cn[nt] = (cj[nt] < k) ? cnorm[cj[nt]] : 0.f;
  }
  // one centre tile, all of it in this wave's columns (small k): the row minima are final here, so
  // lane li < 16 keeps row r = li of each half and ONE plain store per 32-row tile writes them
  // (per-row atomicMin from one lane each cost more than the distance GEMM at k = 20)
  const bool final_here = n_ctiles == 1 && WN == 1;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    unsigned long long keep = ~0ull;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float bv = __builtin_huge_valf();
      int bi = 0x7fffffff;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if (cj[nt] < k) {
          const float d = fmaf(-2.f, acc[mt][nt][r], cn[nt]);
          if (d < bv) { bv = d; bi = cj[nt]; }
        }
      }
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) {
        const float ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      const unsigned long long key =
          bi == 0x7fffffff ? ~0ull : (((unsigned long long)orderable(bv) << 32) | (unsigned)bi);
      if (final_here) {
        if (li == r) keep = key;
      } else if (li == 0 && bi != 0x7fffffff) {
        const long row = row0 + wm * MT * 32 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < m) atomicMin(&best[row], key);
      }
    }
    if (final_here && li < 16) {
      const long row = row0 + wm * MT * 32 + mt * 32 + (li & 3) + 8 * (li >> 2) + 4 * lk;
      if (row < m) best[row] = keep;
    }
  }
}

__global__ void nn_finalize_kernel(const unsigned long long* __restrict__ best, long m, const float* __restrict__ xnorm,
                                   int* __restrict__ labels, float* __restrict__ dist) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const unsigned long long key = best[i];
  labels[i] = (int)(key & 0xffffffffu);
  float d = unorderable((unsigned)(key >> 32)) + (xnorm ? xnorm[i] : 0.f);
  dist[i] = d > 0.f ? d : 0.f;
}

template <bool VEC>
__global__ __launch_bounds__(256) void accumulate_lds_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                             const int* __restrict__ labels, int k,
                                                             double* __restrict__ sums, int* __restrict__ counts,
                                                             long rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float s_sum[];  // k*n floats then k ints
  int* s_cnt = reinterpret_cast<int*>(s_sum + (long)k * n);
  for (int i = threadIdx.x; i < k * n; i += 256) s_sum[i] = 0.f;
  for (int i = threadIdx.x; i < k; i += 256) s_cnt[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(m, r0 + rows_per_block);
  // U rows per wave step: their labels and values are loaded together (one dependent global
  // round trip per U rows instead of per row), then added into the block's LDS sums
  constexpr int U = 8;
  long r = r0 + wid;
  for (; r + 4 * (U - 1) < r1; r += 4 * U) {
    int l[U];
#pragma unroll
    for (int u = 0; u < U; ++u) l[u] = labels[r + 4 * u];
    if (lane < U) atomicAdd(&s_cnt[labels[r + 4 * lane]], 1);
    for (int d0 = 0; d0 < n; d0 += 64) {
      const int d = d0 + lane;
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = d < n ? X[(r + 4 * u) * ld + d] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (d < n) atomicAdd(&s_sum[(long)l[u] * n + d], v[u]);
    }
  }
  for (; r < r1; r += 4) {
    const int l = labels[r];
    if (lane == 0) atomicAdd(&s_cnt[l], 1);
    float* dst = s_sum + (long)l * n;
    const float* row = X + r * ld;
    for (int d = lane; d < n; d += 64) atomicAdd(&dst[d], row[d]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k * n; i += 256) {
    const float v = s_sum[i];
    if (v != 0.f) atomicAdd(&sums[i], (double)v);
  }
  for (int i = threadIdx.x; i < k; i += 256)
    if (s_cnt[i]) atomicAdd(&counts[i], s_cnt[i]);
}

__global__ __launch_bounds__(256) void accumulate_global_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                                const int* __restrict__ labels,
                                                                float* __restrict__ sums, int* __restrict__ counts) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  for (long r = wave; r < m; r += nw) {
    const int l = labels[r];
    if (lane == 0) atomicAdd(&counts[l], 1);
    float* dst = sums + (long)l * n;
    const float* row = X + r * ld;
    for (int d = lane; d < n; d += 64) atomicAdd(&dst[d], row[d]);
  }
}
// Sorted-segment cluster sums: rows visited in label-sorted order (perm / slab from a device
// sort), so a chunk of RPB consecutive rows spans few clusters. Each thread owns VW consecutive
// columns and accumulates in fp32 registers while the (block-uniform) label stays the same; at a
// label change or the chunk end the partial goes out as fp64 atomics. Atomics per iteration:
// ~(m / RPB + k) * n instead of the m * n of per-row scattering (accumulate_global_kernel).
template <int VW>
__global__ __launch_bounds__(256) void accumulate_sorted_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                                const int* __restrict__ perm,
                                                                const int* __restrict__ slab,
                                                                double* __restrict__ sums, int rpb,
                                                                const int* __restrict__ rows = nullptr) {
  __shared__ int s_row[256];
  __shared__ int s_lab[256];
  const long r0 = (long)blockIdx.x * rpb;
  const int cnt = (int)min((long)rpb, m - r0);
  for (int i = threadIdx.x; i < cnt; i += 256) {
    s_row[i] = rows ? rows[perm[r0 + i]] : perm[r0 + i];  // rows: perm indexes a row list
    s_lab[i] = slab[r0 + i];
  }
  __syncthreads();
  const int c = (blockIdx.y * 256 + threadIdx.x) * VW;
  if (c >= n) return;
  float acc[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) acc[j] = 0.f;
  int cur = s_lab[0];
  auto flush = [&](int lab) {
    double* dst = sums + (long)lab * n + c;
#pragma unroll
    for (int j = 0; j < VW; ++j)
      if (VW == 1 || c + j < n) atomicAdd(dst + j, (double)acc[j]);
  };
  constexpr int U = 8;
  for (int i0 = 0; i0 < cnt; i0 += U) {
    float v[U][VW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u;
      if (i < cnt) {
        // a negative entry ~r SUBTRACTS row r (the Lloyd delta update: moved rows enter their new
        // cluster and leave their old one in ONE label-sorted list)
        const int rr = s_row[i];
        const float sg = rr < 0 ? -1.f : 1.f;
        const float* row = X + (long)(rr < 0 ? ~rr : rr) * ld + c;
        if constexpr (VW == 4) {
          const float4 q = *reinterpret_cast<const float4*>(row);
          v[u][0] = sg * q.x; v[u][1] = sg * q.y; v[u][2] = sg * q.z; v[u][3] = sg * q.w;
        } else {
#pragma unroll
          for (int j = 0; j < VW; ++j) v[u][j] = sg * row[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u;
      if (i < cnt) {
        const int l = s_lab[i];
        if (l != cur) {
          flush(cur);
#pragma unroll
          for (int j = 0; j < VW; ++j) acc[j] = 0.f;
          cur = l;
        }
#pragma unroll
        for (int j = 0; j < VW; ++j) acc[j] += v[u][j];
      }
    }
  }
  flush(cur);
}

// ------------------------------------------------------------------------------------------
// Exact k-nearest-neighbours: fused MFMA distance tiles + per-query top-k in LDS.
// Block = 128 queries x one slice of the item range; the query tile's top-k list lives in LDS
// for the whole item sweep, so the q x items distance matrix is never materialised (reference:
// cuML NearestNeighborsMG brute force, knn.py:638-749). After each 128x128 MFMA tile the
// partial distances (||i||^2 - 2 q.i) go through the (reused) staging LDS and 128 threads each
// merge one query row with a threshold test + insertion into a sorted list (most candidates are
// rejected by the threshold after the first tiles). Item-range slices (grid.y) keep >= 512
// blocks in flight for small query sets; slices are merged by the caller.
// ------------------------------------------------------------------------------------------
constexpr int KNN_KMAX = 64;

template <bool VEC>
__global__ __launch_bounds__(256, 1) void knn_kernel(const float* __restrict__ Q, long mq, int n, long ldq,
                                                     const float* __restrict__ I, long mi, long ldi,
                                                     const float* __restrict__ inorm, int k, long items_per_slice,
                                                     float* __restrict__ out_d, long long* __restrict__ out_i,
                                                     long long id_offset) {
  constexpr int BM = 128, BN = 128, MT = 2, NT = 2;
  union Smem {
    struct {
      float Xs[2][BM][PADK];
      float Cs[2][BN][PADK];
    } st;
    float D[BM][BN + 1];
  };
  __shared__ Smem sm;
  // +1 pad: thread t walks row t, so an unpadded 64-word stride would put every thread on one bank
  __shared__ float topd[BM][KNN_KMAX + 1];
  __shared__ int topi[BM][KNN_KMAX + 1];
  const long q0 = (long)blockIdx.x * BM;
  const long slice = blockIdx.y;
  const long ibeg = slice * items_per_slice;
  const long iend = min(mi, ibeg + items_per_slice);
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int li = lane & 31, lk = lane >> 5;
  for (int i = t; i < BM * (KNN_KMAX + 1); i += 256) {
    (&topd[0][0])[i] = __builtin_huge_valf();
    (&topi[0][0])[i] = -1;
  }
  const int nk = (n + BK - 1) / BK;
  for (long c0 = ibeg; c0 < iend; c0 += BN) {
    floatx16 acc[MT][NT];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    RowTile<BM, VEC> xt;
    RowTile<BN, VEC> ct;
    xt.load(Q, ldq, mq, n, q0, 0);
    ct.load(I, ldi, iend, n, c0, 0);
    __syncthreads();  // previous tile's top-k scan has finished with sm.D
    xt.store(sm.st.Xs[0]);
    ct.store(sm.st.Cs[0]);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) {
        xt.load(Q, ldq, mq, n, q0, (kt + 1) * BK);
        ct.load(I, ldi, iend, n, c0, (kt + 1) * BK);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        const int kx = 2 * kk + lk;
        float a[MT], b[NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[mt] = sm.st.Xs[cur][wm * MT * 32 + mt * 32 + li][kx];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) b[nt] = sm.st.Cs[cur][wn * NT * 32 + nt * 32 + li][kx];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
      }
      if (more) {
        xt.store(sm.st.Xs[cur ^ 1]);
        ct.store(sm.st.Cs[cur ^ 1]);
      }
      __syncthreads();
      cur ^= 1;
    }
    // partial distances -> LDS tile (staging buffers are dead now)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int cl = wn * NT * 32 + nt * 32 + li;
      const long cg = c0 + cl;
      const float in = cg < iend ? inorm[cg] : 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * MT * 32 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
          sm.D[rl][cl] = cg < iend ? fmaf(-2.f, acc[mt][nt][r], in) : __builtin_huge_valf();
        }
    }
    __syncthreads();
    if (t < BM) {
      float thr = topd[t][k - 1];
      const int ncol = (int)min((long)BN, iend - c0);
      for (int c = 0; c < ncol; ++c) {
        const float d = sm.D[t][c];
        if (d < thr) {
          int p = k - 1;
          while (p > 0 && topd[t][p - 1] > d) {
            topd[t][p] = topd[t][p - 1];
            topi[t][p] = topi[t][p - 1];
            --p;
          }
          topd[t][p] = d;
          topi[t][p] = (int)(c0 + c - ibeg);
          thr = topd[t][k - 1];
        }
      }
    }
  }
  __syncthreads();
  if (t < BM && q0 + t < mq) {
    const long base = ((q0 + t) * gridDim.y + slice) * (long)k;
    for (int j = 0; j < k; ++j) {
      out_d[base + j] = topd[t][j];
      out_i[base + j] = topi[t][j] >= 0 ? (long long)topi[t][j] + ibeg + id_offset : -1;
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// IVF-Flat search: one block per query; the query's nprobe inverted lists (items pre-sorted by
// list, contiguous) are swept by the 4 waves, one item per wave step: lanes split the feature
// dimension (16-B loads), the dot product is a DPP wave reduction, and a wave-private sorted
// top-k list in LDS takes the candidate when it beats the list's threshold. The four lists are
// merged at the end (reference: cuML NearestNeighbors(algorithm="ivfflat"), knn.py:1295-1380).
// ------------------------------------------------------------------------------------------
namespace {
// G lanes per item (G = pow2 >= n/4, <= 64): a wave scores 64/G items per step, each group
// reduces its dot product with in-group shuffles; candidates are inserted in item order with
// wave-uniform threshold tests (a 128-wide item used only 32 lanes of a 64-lane wave per step).
template <int G>
__global__ __launch_bounds__(256) void ivf_search_kernel(const float* __restrict__ Q, long nq, int n, long ldq,
                                                         const int* __restrict__ probes, int nprobe,
                                                         const long long* __restrict__ list_off,
                                                         const float* __restrict__ items, long ldi,
                                                         const float* __restrict__ inorm,
                                                         const long long* __restrict__ ids, int k,
                                                         float* __restrict__ out_d, long long* __restrict__ out_i) {
  constexpr int IPW = 64 / G;  // items per wave step
  extern __shared__ __attribute__((aligned(16))) float qs[];  // n floats (padded to 4)
  __shared__ float wd[4][KNN_KMAX];
  __shared__ long long wi[4][KNN_KMAX];
  const long q = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int gi = lane / G, gl = lane % G;
  for (int d = t; d < n; d += 256) qs[d] = Q[q * ldq + d];
  for (int j = t; j < 4 * KNN_KMAX; j += 256) {
    (&wd[0][0])[j] = __builtin_huge_valf();
    (&wi[0][0])[j] = -1;
  }
  __syncthreads();
  float thr = __builtin_huge_valf();
  const bool vec = ((n & 3) == 0) && ((ldi & 3) == 0);
  for (int p = 0; p < nprobe; ++p) {
    const int l = probes[q * nprobe + p];
    if (l < 0) continue;
    const long s = list_off[l], e = list_off[l + 1];
    for (long j0 = s + (long)wid * IPW; j0 < e; j0 += 4 * IPW) {
      const long j = j0 + gi;
      float acc = 0.f;
      if (j < e) {
        const float* row = items + j * ldi;
        if (vec) {
          for (int d = gl * 4; d < n; d += 4 * G) {
            const floatx4 x = *reinterpret_cast<const floatx4*>(row + d);
            acc = fmaf(x[0], qs[d], fmaf(x[1], qs[d + 1], fmaf(x[2], qs[d + 2], fmaf(x[3], qs[d + 3], acc))));
          }
        } else {
          for (int d = gl; d < n; d += G) acc = fmaf(row[d], qs[d], acc);
        }
      }
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
      const float dist = j < e ? fmaf(-2.f, acc, inorm[j]) : __builtin_huge_valf();
#pragma unroll
      for (int g = 0; g < IPW; ++g) {
        const float dg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dist), g * G));
        if (dg < thr) {  // wave-uniform
          if (lane == 0) {
            int pos = k - 1;
            while (pos > 0 && wd[wid][pos - 1] > dg) {
              wd[wid][pos] = wd[wid][pos - 1];
              wi[wid][pos] = wi[wid][pos - 1];
              --pos;
            }
            wd[wid][pos] = dg;
            wi[wid][pos] = ids[j0 + g];
          }
          __builtin_amdgcn_wave_barrier();
          thr = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wd[wid][k - 1])));
        }
      }
    }
  }
  __syncthreads();
  if (t == 0) {  // 4-way merge of the wave lists
    int h[4] = {0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      int bw = 0;
      float bd = wd[0][h[0]];
      for (int w = 1; w < 4; ++w)
        if (wd[w][h[w]] < bd) { bd = wd[w][h[w]]; bw = w; }
      out_d[q * k + j] = bd;
      out_i[q * k + j] = wi[bw][h[bw]];
      if (h[bw] < k - 1) ++h[bw]; else wd[bw][h[bw]] = __builtin_huge_valf();
    }
  }
}
}  // namespace

SRML_API int srml_ivf_search_f32(const float* Q, long nq, int n, long ldq, const int* probes, int nprobe,
                                 const long long* list_off, const float* items, long ldi, const float* inorm,
                                 const long long* ids, int k, float* out_d, long long* out_i, hipStream_t stream) {
  if (nq <= 0) return 0;
  if (k < 1 || k > KNN_KMAX) return -8;
  const size_t lds = (size_t)((n + 3) / 4) * 4 * sizeof(float);
  const int need = (n + 3) / 4;  // lanes that a 16-B-per-lane pass over one item occupies
#define SRML_IVF(GG)                                                                                        \
  hipLaunchKernelGGL((ivf_search_kernel<GG>), dim3((unsigned)nq), dim3(256), lds, stream, Q, nq, n, ldq, probes, \
                     nprobe, list_off, items, ldi, inorm, ids, k, out_d, out_i)
  if (need <= 8) SRML_IVF(8);
  else if (need <= 16) SRML_IVF(16);
  else if (need <= 32) SRML_IVF(32);
  else SRML_IVF(64);
#undef SRML_IVF
  return srml_status();
}

// out_d / out_i: (mq, slices, k) partial top-k (distance WITHOUT the ||q||^2 term)
SRML_API int srml_knn_f32(const float* Q, long mq, int n, long ldq, const float* I, long mi, long ldi,
                          const float* inorm, int k, int slices, float* out_d, long long* out_i, long long id_offset,
                          hipStream_t stream) {
  if (mq <= 0) return 0;
  if (k < 1 || k > KNN_KMAX) return -8;
  const bool vec = ((ldq & 3) == 0) && ((ldi & 3) == 0) && ((n & 3) == 0) &&
                   ((reinterpret_cast<uintptr_t>(Q) & 15) == 0) && ((reinterpret_cast<uintptr_t>(I) & 15) == 0);
  if (slices < 1) slices = 1;
  long per = (mi + slices - 1) / slices;
  per = ((per + 127) / 128) * 128;
  if (per < 128) per = 128;
  dim3 grid(ceil_div(mq, 128), (unsigned)slices);
  if (vec)
    hipLaunchKernelGGL(knn_kernel<true>, grid, dim3(256), 0, stream, Q, mq, n, ldq, I, mi, ldi, inorm, k, per, out_d,
                       out_i, id_offset);
  else
    hipLaunchKernelGGL(knn_kernel<false>, grid, dim3(256), 0, stream, Q, mq, n, ldq, I, mi, ldi, inorm, k, per,
                       out_d, out_i, id_offset);
  return srml_status();
}

SRML_API int srml_nearest_centroid_f32(const float* X, long m, int n, long ldx, const float* C, int k, long ldc,
                                       const float* cnorm, unsigned long long* best, hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  const bool vec = ((ldx & 3) == 0) && ((ldc & 3) == 0) && ((n & 3) == 0) &&
                   ((reinterpret_cast<uintptr_t>(X) & 15) == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0);
  // rows are independent: launches of at most srml_max_blocks(256) row x centroid tiles each
  // (e.g. 20M rows x 19531 IVF lists is 23.9M tiles of 128 x 128, past the 2^32 work-item grid)
  if (k > 64) {
    constexpr int BM = 128, BN = 128;
    const int ct = (k + BN - 1) / BN;
    const long rows_per = (srml_max_blocks(256) / ct) * BM;
    if (rows_per < BM) return -3;
    for (long r0 = 0; r0 < m; r0 += rows_per) {
      const long mc = m - r0 < rows_per ? m - r0 : rows_per;
      const long nb = (mc + BM - 1) / BM * ct;
      if (vec)
        hipLaunchKernelGGL((nearest_centroid_kernel<BM, BN, 2, 2, 2, true>), dim3((unsigned)nb), dim3(256), 0, stream,
                           X + r0 * ldx, mc, n, ldx, C, k, ldc, cnorm, best + r0, ct);
      else
        hipLaunchKernelGGL((nearest_centroid_kernel<BM, BN, 2, 2, 2, false>), dim3((unsigned)nb), dim3(256), 0, stream,
                           X + r0 * ldx, mc, n, ldx, C, k, ldc, cnorm, best + r0, ct);
    }
  } else {
    // k <= 64: 128-row x 64-centre tiles, 4 waves of 32 rows x 64 centres (the 256-row tile's
    // 85 KB of LDS admitted one block per CU: the small-k search ran latency-bound at ~0.6 TB/s)
    constexpr int BM = 128, BN = 64;
    const int ct = (k + BN - 1) / BN;
    const long rows_per = (srml_max_blocks(256) / ct) * BM;
    for (long r0 = 0; r0 < m; r0 += rows_per) {
      const long mc = m - r0 < rows_per ? m - r0 : rows_per;
      const long nb = (mc + BM - 1) / BM * ct;
      if (vec)
        hipLaunchKernelGGL((nearest_centroid_kernel<BM, BN, 4, 1, 2, true>), dim3((unsigned)nb), dim3(256), 0, stream,
                           X + r0 * ldx, mc, n, ldx, C, k, ldc, cnorm, best + r0, ct);
      else
        hipLaunchKernelGGL((nearest_centroid_kernel<BM, BN, 4, 1, 2, false>), dim3((unsigned)nb), dim3(256), 0, stream,
                           X + r0 * ldx, mc, n, ldx, C, k, ldc, cnorm, best + r0, ct);
    }
  }
  return srml_status();
}

SRML_API int srml_nn_finalize(const unsigned long long* best, long m, const float* xnorm, int* labels, float* dist,
                              hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(nn_finalize_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, best, m, xnorm, labels,
                     dist);
  return srml_status();
}

// sums: fp64 (k*n) when use_lds, fp32 otherwise (sums_f32); counts int32 (k)
SRML_API int srml_kmeans_accumulate_f32(const float* X, long m, int n, long ld, const int* labels, int k,
                                        double* sums_f64, float* sums_f32, int* counts, hipStream_t stream) {
  if (m <= 0) return 0;
  const size_t lds = (size_t)k * n * sizeof(float) + (size_t)k * sizeof(int);
  if (sums_f64 && lds <= 64 * 1024) {
    long blocks = 1024;
    long rpb = (m + blocks - 1) / blocks;
    if (rpb < 256) rpb = 256;
    blocks = (m + rpb - 1) / rpb;
    hipLaunchKernelGGL(accumulate_lds_kernel<true>, dim3((unsigned)blocks), dim3(256), lds, stream, X, m, n, ld, labels, k,
                       sums_f64, counts, rpb);
  } else {
    if (!sums_f32) return -4;
    long blocks = (m + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(accumulate_global_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, labels,
                       sums_f32, counts);
  }
  return srml_status();
}

// sums (k*n fp64) += rows of X grouped by label, rows visited in label-sorted order. rows
// (nullable): perm indexes this list of (possibly ~negated) row ids instead of X directly (the
// Lloyd delta update's moved-row list, sorted by label without a gathered copy).
SRML_API int srml_kmeans_accumulate_sorted_rows_f32(const float* X, long m, int n, long ld, const int* perm,
                                                    const int* rows, const int* sorted_labels, double* sums,
                                                    hipStream_t stream) {
  if (m <= 0) return 0;
  const bool vec = ((ld & 3) == 0) && ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  // rows per block: 256, or fewer so a short list (the Lloyd delta update: ~1 % of the rows move)
  // still spreads over ~1024 blocks — 256-row blocks gave a few dozen blocks each walking 256
  // rows in dependent 8-row steps (0.33 ms for ~2500 rows at n = 3000)
  const long gy = vec ? (n / 4 + 255) / 256 : (n + 255) / 256;
  long want = (m * gy + 1023) / 1024;
  want = (want + 7) / 8 * 8;
  const int rpb = (int)(want < 8 ? 8 : (want > 256 ? 256 : want));
  const long gx = (m + rpb - 1) / rpb;
  if (vec) {
    dim3 grid((unsigned)gx, (unsigned)((n / 4 + 255) / 256));
    hipLaunchKernelGGL(accumulate_sorted_kernel<4>, grid, dim3(256), 0, stream, X, m, n, ld, perm, sorted_labels,
                       sums, rpb, rows);
  } else {
    dim3 grid((unsigned)gx, (unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(accumulate_sorted_kernel<1>, grid, dim3(256), 0, stream, X, m, n, ld, perm, sorted_labels,
                       sums, rpb, rows);
  }
  return srml_status();
}

SRML_API int srml_kmeans_accumulate_sorted_f32(const float* X, long m, int n, long ld, const int* perm,
                                               const int* sorted_labels, double* sums, hipStream_t stream) {
  return srml_kmeans_accumulate_sorted_rows_f32(X, m, n, ld, perm, nullptr, sorted_labels, sums, stream);
}

// Deterministic / fp64 cluster sums: rows visited in label-sorted order (perm), cluster l owns
// the segment [off[l], off[l+1]), cut into S equal splits. One block per (cluster, 256-column
// chunk, split) sums its rows in order into fp64 registers and stores the partial into ws[split];
// a second pass folds the S partials in split order. No atomics: bit-reproducible run to run
// (SRML_DETERMINISTIC=1), and the fp64-input path (T = double) of the Lloyd update.
template <typename T>
__global__ __launch_bounds__(256) void segment_sums_kernel(const T* __restrict__ X, int n, long ld,
                                                           const int* __restrict__ perm,
                                                           const long* __restrict__ off, int k,
                                                           double* __restrict__ ws) {
  const int l = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  const int sp = blockIdx.z, S = gridDim.z;
  if (c >= n) return;
  const long a = off[l], len = off[l + 1] - a;
  const long s0 = a + len * sp / S, s1 = a + len * (sp + 1) / S;
  constexpr int U = 8;
  double acc = 0.0;
  long i = s0;
  for (; i + U <= s1; i += U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = X[(long)perm[i + u] * ld + c];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (double)v[u];
  }
  for (; i < s1; ++i) acc += (double)X[(long)perm[i] * ld + c];
  ws[((long)sp * k + l) * n + c] = acc;
}

__global__ __launch_bounds__(256) void segment_fold_kernel(const double* __restrict__ ws, int S, long kn,
                                                           double* __restrict__ sums) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= kn) return;
  double s = 0.0;
  for (int z = 0; z < S; ++z) s += ws[z * kn + i];
  sums[i] = s;
}

template <typename T>
static int launch_segment_sums(const T* X, long m, int n, long ld, const int* perm, const long* off, int k,
                               double* sums, int splits, double* ws, hipStream_t stream) {
  if (k <= 0 || n <= 0) return 0;
  (void)m;
  if (splits < 1 || !ws) { splits = 1; ws = sums; }
  dim3 grid((unsigned)k, ceil_div(n, 256), (unsigned)splits);
  hipLaunchKernelGGL(segment_sums_kernel<T>, grid, dim3(256), 0, stream, X, n, ld, perm, off, k, ws);
  int st = srml_status();
  if (st || ws == sums) return st;
  const long kn = (long)k * n;
  hipLaunchKernelGGL(segment_fold_kernel, dim3(ceil_div(kn, 256)), dim3(256), 0, stream, ws, splits, kn, sums);
  return srml_status();
}

// sums (k*n fp64, fully written) of the rows perm[off[l]:off[l+1]] per cluster l; each segment is
// cut into `splits` parts summed into ws (splits * k * n fp64; null / splits = 1: direct).
SRML_API int srml_kmeans_segment_sums_f32(const float* X, long m, int n, long ld, const int* perm, const long* off,
                                          int k, double* sums, int splits, double* ws, hipStream_t stream) {
  return launch_segment_sums<float>(X, m, n, ld, perm, off, k, sums, splits, ws, stream);
}
SRML_API int srml_kmeans_segment_sums_f64(const double* X, long m, int n, long ld, const int* perm, const long* off,
                                          int k, double* sums, int splits, double* ws, hipStream_t stream) {
  return launch_segment_sums<double>(X, m, n, ld, perm, off, k, sums, splits, ws, stream);
}

// ------------------------------------------------------------------------------------------
// Weighted k-means++ seeding of a small candidate set entirely on the device (the reduction step
// of k-means||, Spark's LocalKMeans): ONE block runs the k sequential picks with no host round
// trip (the previous path did two .item() syncs per centre: ~10k for k=1000 and 5 trials).
// Distances come from the candidates' Gram matrix G = C C^T (MFMA SYRK), so a pick costs one
// pass over nc values: d2[i] = min(d2[i], G_ii + G_cc - 2 G_ic); the next centre is drawn with
// probability w_i d2_i / sum (block-wide inclusive scan + a counter-based uniform).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ double uniform01(unsigned long long seed, unsigned long long ctr) {
  return (double)(splitmix64(seed * 0x2545F4914F6CDD1Dull + ctr) >> 11) * (1.0 / 9007199254740992.0);
}

constexpr int KPP_T = 1024;
constexpr int KPP_PER = 8;     // candidates per thread (nc <= 8192)
constexpr int KPP_TRIALS = 16; // max greedy trials per centre
constexpr int KPP_CHUNK = 4;   // greedy trials whose G-row loads are issued together

// block-wide inverse-CDF draws of L targets u[j] * total over p >= 0 (candidate base + q of the
// thread that owns the target's half-open prefix range); picks[j] = -1 if total == 0
__device__ void kpp_sample(const double (*wv)[KPP_T], const double (&d2)[KPP_PER], int base, int cnt,
                           const double* u, int L, double* lds, int* picks) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double loc = 0.0;
#pragma unroll
  for (int q = 0; q < KPP_PER; ++q) loc += q < cnt ? wv[q][threadIdx.x] * d2[q] : 0.0;
  // inclusive scan of the per-thread sums within the wave, then across the 16 waves
  double x = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  if (threadIdx.x < L) picks[threadIdx.x] = -1;
  __syncthreads();
  double wave_off = 0.0, total = 0.0;
  for (int w = 0; w < KPP_T / 64; ++w) {
    const double v = lds[w];
    if (w < wid) wave_off += v;
    total += v;
  }
  const double excl = wave_off + x - loc;  // sum of all candidates before this thread's
  for (int j = 0; j < L; ++j) {
    const double target = u[j] * total;
    if (total > 0.0 && excl <= target && target < excl + loc) {
      double run = excl;
      int hit = -1;
#pragma unroll
      for (int q = 0; q < KPP_PER; ++q) {  // static indices: the candidate arrays stay in VGPRs
        if (q < cnt) {
          run += wv[q][threadIdx.x] * d2[q];
          if (hit < 0 && target < run) hit = q;
        }
      }
      picks[j] = base + (hit < 0 ? cnt - 1 : hit);  // exactly one thread owns the target (half-open ranges)
    }
  }
  __syncthreads();
  for (int j = 0; j < L; ++j) {  // rounding at the very top of the range: last positive candidate
    if (total > 0.0 && picks[j] < 0) {
      __syncthreads();
      if (loc > 0.0) atomicMax(&picks[j], base + cnt - 1);
      __syncthreads();
    }
  }
  __syncthreads();
}

// Greedy weighted k-means++ (the reduction step of k-means||, as cuML / scikit-learn run it):
// centre 0 ~ w; every later centre draws L candidates ~ w_i d2_i and keeps the one that lowers
// the potential sum_i w_i min(d2_i, ||c_i - cand||^2) the most (single-draw k-means++ merged two
// of eight separated blobs in ~1 of 4 seeds). Distances from the Gram matrix G = C C^T.
__global__ __launch_bounds__(KPP_T) void kmeanspp_gram_kernel(const double* __restrict__ G, int nc, long ldg,
                                                              const double* __restrict__ w, int k, int L,
                                                              unsigned long long seed, int* __restrict__ out) {
  __shared__ double lds[KPP_T / 64];
  __shared__ double pot[KPP_T / 64][KPP_TRIALS];
  __shared__ double u[KPP_TRIALS];
  __shared__ int picks[KPP_TRIALS];
  // ||c_i||^2 and w_i of this thread's candidates live in LDS (128 KB), so the 128-VGPR budget of
  // a 1024-thread block holds d2 plus the in-flight G-row loads without scratch spills
  __shared__ double s_gii[KPP_PER][KPP_T];
  __shared__ double s_w[KPP_PER][KPP_T];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int base = threadIdx.x * KPP_PER;
  const int cnt = max(0, min(KPP_PER, nc - base));
  double d2[KPP_PER];  // p_q = w_q d2_q is formed where it is used
#pragma unroll
  for (int q = 0; q < KPP_PER; ++q) {
    const int i = base + q;
    const bool ok = q < cnt;
    s_w[q][threadIdx.x] = ok ? w[i] : 0.0;
    s_gii[q][threadIdx.x] = ok ? G[(long)i * ldg + i] : 0.0;
    d2[q] = 1.0;  // the first draw is ~ w alone
  }
  if (threadIdx.x == 0) u[0] = uniform01(seed, 0);
  __syncthreads();
  kpp_sample(s_w, d2, base, cnt, u, 1, lds, picks);
#pragma unroll
  for (int q = 0; q < KPP_PER; ++q) d2[q] = INFINITY;
  int c = picks[0] < 0 ? 0 : picks[0];
  if (threadIdx.x == 0) out[0] = c;
  for (int t = 1; t < k; ++t) {
    const double gcc = G[(long)c * ldg + c];
    const double* gc = G + (long)c * ldg;
#pragma unroll
    for (int q = 0; q < KPP_PER; ++q) {
      const double dd = fmax(s_gii[q][threadIdx.x] + gcc - 2.0 * gc[min(base + q, nc - 1)], 0.0);
      if (q < cnt) d2[q] = fmin(d2[q], dd);
    }
    __syncthreads();  // picks / u of the previous step fully consumed
    if (threadIdx.x < L) u[threadIdx.x] = uniform01(seed, (unsigned long long)t * KPP_TRIALS + threadIdx.x);
    __syncthreads();
    kpp_sample(s_w, d2, base, cnt, u, L, lds, picks);
    if (picks[0] < 0) {  // all mass on chosen points: any candidate
      c = (int)(splitmix64(seed + 77 * t) % (unsigned long long)nc);
    } else {
      // potential of each trial: one pass over this thread's candidates per trial, block-reduced.
      // KPP_CHUNK trials at a time with branch-free (clamped) loads, so their G-row reads are in
      // flight together instead of one latency per trial; a candidate past nc has wv = 0 and adds
      // +0.0, so every trial's sum is bit-identical to the one-trial-at-a-time order.
      for (int j0 = 0; j0 < L; j0 += KPP_CHUNK) {
        double s[KPP_CHUNK];
#pragma unroll
        for (int jj = 0; jj < KPP_CHUNK; ++jj) {
          const int tj = picks[min(j0 + jj, L - 1)];
          const double* gt = G + (long)tj * ldg;
          const double gtt = gt[tj];
          double a = 0.0;
#pragma unroll
          for (int q = 0; q < KPP_PER; ++q) {
            const double g = gt[min(base + q, nc - 1)];
            if (q < cnt) a += s_w[q][threadIdx.x] * fmin(d2[q], fmax(s_gii[q][threadIdx.x] + gtt - 2.0 * g, 0.0));
          }
          s[jj] = a;
        }
#pragma unroll
        for (int jj = 0; jj < KPP_CHUNK; ++jj) {
          if (j0 + jj < L) {  // block-uniform
            const double r = wave_sum(s[jj]);
            if (lane == 0) pot[wid][j0 + jj] = r;
          }
        }
      }
      __syncthreads();
      int best = 0;
      double bv = INFINITY;
      for (int j = 0; j < L; ++j) {
        double tot = 0.0;
        for (int v = 0; v < KPP_T / 64; ++v) tot += pot[v][j];
        if (tot < bv) { bv = tot; best = j; }
      }
      c = picks[best];
    }
    if (threadIdx.x == 0) out[t] = c;
  }
}

// Register-resident variant for nc <= 4096 candidates and <= 8 trials (k <= 1096): every thread
// owns 4 candidates, issues the G-row loads of ALL trials of a pick at once (one memory latency
// instead of one per chunk) and keeps them in VGPRs, so the winner's row updates d2 without being
// read again; trial potentials are reduced by a transposing butterfly (10 double shuffles instead
// of 8 full wave sums) and each wave finds the winner itself (no extra barrier); the draw's
// uniforms are computed per lane and broadcast with readlane. Three block barriers per pick.
constexpr int KPR_PER = 4;
constexpr int KPR_LT = 8;

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__global__ __launch_bounds__(KPP_T) void kmeanspp_gram_reg_kernel(const double* __restrict__ G, int nc, long ldg,
                                                                  const double* __restrict__ w, int k, int L,
                                                                  unsigned long long seed, int* __restrict__ out) {
  __shared__ double s_wave[KPP_T / 64];
  __shared__ double s_pot[KPP_T / 64][KPR_LT];
  __shared__ int s_pick[2][KPR_LT];  // double-buffered by pick parity: read after the last barrier of a pick
  __shared__ double s_w[KPR_PER][KPP_T];
  __shared__ double s_gii[KPR_PER][KPP_T];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int base = tid * KPR_PER;
  const int cnt = max(0, min(KPR_PER, nc - base));
  double d2[KPR_PER];
#pragma unroll
  for (int q = 0; q < KPR_PER; ++q) {
    const int i = min(base + q, nc - 1);
    s_w[q][tid] = q < cnt ? w[i] : 0.0;
    s_gii[q][tid] = q < cnt ? G[(long)i * ldg + i] : 0.0;
    d2[q] = 1.0;  // the first draw is ~ w alone
  }
  // inverse-CDF draws of nd targets (uniforms seed/ctr0 + j) over p_q = w_q d2_q -> s_pick[pb][0..nd);
  // returns the first pick (-1: no mass)
  auto draw = [&](int nd, unsigned long long ctr0, int pb) -> int {
    int* pick = s_pick[pb];
    double loc = 0.0;
#pragma unroll
    for (int q = 0; q < KPR_PER; ++q) loc += q < cnt ? s_w[q][tid] * d2[q] : 0.0;
    double x = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wid] = x;
    if (tid < KPR_LT) pick[tid] = -1;
    const double uj = uniform01(seed, ctr0 + (unsigned long long)(lane & (KPR_LT - 1)));
    __syncthreads();
    double wave_off = 0.0, total = 0.0;
#pragma unroll
    for (int v = 0; v < KPP_T / 64; ++v) {
      const double s = s_wave[v];
      if (v < wid) wave_off += s;
      total += s;
    }
    const double excl = wave_off + x - loc;
#pragma unroll
    for (int j = 0; j < KPR_LT; ++j) {
      if (j < nd) {
        const double target = readlane_d(uj, j) * total;
        if (total > 0.0 && excl <= target && target < excl + loc) {
          double run = excl;
          int hit = -1;
#pragma unroll
          for (int q = 0; q < KPR_PER; ++q) {
            if (q < cnt) {
              run += s_w[q][tid] * d2[q];
              if (hit < 0 && target < run) hit = q;
            }
          }
          pick[j] = base + (hit < 0 ? cnt - 1 : hit);  // exactly one owner (half-open ranges)
        }
      }
    }
    __syncthreads();
    bool miss = false;
#pragma unroll
    for (int j = 0; j < KPR_LT; ++j) miss |= j < nd && pick[j] < 0;
    if (total > 0.0 && miss) {  // block-uniform; rounding at the very top: last positive candidate
      __syncthreads();
#pragma unroll
      for (int j = 0; j < KPR_LT; ++j)
        if (j < nd && pick[j] < 0 && loc > 0.0) atomicMax(&pick[j], base + cnt - 1);
      __syncthreads();
    }
    return pick[0];
  };
  const int p0 = draw(1, 0, 0);
#pragma unroll
  for (int q = 0; q < KPR_PER; ++q) d2[q] = INFINITY;
  int c = p0 < 0 ? 0 : p0;
  if (tid == 0) out[0] = c;
  // this thread's 4 candidates of row r (32-B aligned: ldg % 4 == 0; threads past nc read column 0..3)
  const int rb = cnt > 0 ? base : 0;
  auto row4 = [&](const double* r, double (&v)[KPR_PER]) {
    const double2* r2 = reinterpret_cast<const double2*>(r + rb);
    const double2 lo = r2[0], hi = r2[1];
    v[0] = lo.x;
    v[1] = lo.y;
    v[2] = hi.x;
    v[3] = hi.y;
  };
  auto update_d2 = [&](int cc) {  // d2 = min(d2, ||c_i - c_cc||^2) from row cc (cc block-uniform)
    const double* gc = G + (long)cc * ldg;
    const double gcc = gc[cc];
    double v[KPR_PER];
    row4(gc, v);
#pragma unroll
    for (int q = 0; q < KPR_PER; ++q) {
      const double dd = fmax(s_gii[q][tid] + gcc - 2.0 * v[q], 0.0);
      if (q < cnt) d2[q] = fmin(d2[q], dd);
    }
  };
  update_d2(c);
  for (int t = 1; t < k; ++t) {
    const int pb = t & 1;
    if (draw(L, (unsigned long long)t * KPP_TRIALS, pb) < 0) {  // all mass on chosen points: any candidate (block-uniform)
      c = (int)(splitmix64(seed + 77 * t) % (unsigned long long)nc);
      update_d2(c);
      if (tid == 0) out[t] = c;
      __syncthreads();  // s_wave reads of this pick done before the next draw writes them
      continue;
    }
    const int* pick = s_pick[pb];
    double g[KPR_LT][KPR_PER], gtt[KPR_LT];
#pragma unroll
    for (int j = 0; j < KPR_LT; ++j) {  // all trials' row reads in flight together
      const int tj = __builtin_amdgcn_readfirstlane(pick[j < L ? j : 0]);  // uniform: scalar row base
      const double* r = G + (long)tj * ldg;
      gtt[j] = r[tj];
      row4(r, g[j]);
    }
    // g becomes the trial distances in place (gtt dies here)
#pragma unroll
    for (int q = 0; q < KPR_PER; ++q) {
      const double gq = s_gii[q][tid];
#pragma unroll
      for (int j = 0; j < KPR_LT; ++j) g[j][q] = fmax(gq + gtt[j] - 2.0 * g[j][q], 0.0);
    }
    double pot[KPR_LT];
#pragma unroll
    for (int j = 0; j < KPR_LT; ++j) pot[j] = 0.0;
#pragma unroll
    for (int q = 0; q < KPR_PER; ++q) {
      const double wq = s_w[q][tid];
#pragma unroll
      for (int j = 0; j < KPR_LT; ++j)
        if (q < cnt) pot[j] += wq * fmin(d2[q], g[j][q]);
    }
    // transposing butterfly: after xor 32 / 16 / 8 a lane holds trial j = (lane >> 3) & 7's partial
    const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
    double h4[4], h2[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double send = b5 ? pot[i] : pot[i + 4];
      h4[i] = (b5 ? pot[i + 4] : pot[i]) + __shfl_xor(send, 32, 64);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double send = b4 ? h4[i] : h4[i + 2];
      h2[i] = (b4 ? h4[i + 2] : h4[i]) + __shfl_xor(send, 16, 64);
    }
    double h1 = (b3 ? h2[1] : h2[0]) + __shfl_xor(b3 ? h2[0] : h2[1], 8, 64);
    h1 += __shfl_xor(h1, 4, 64);
    h1 += __shfl_xor(h1, 2, 64);
    h1 += __shfl_xor(h1, 1, 64);
    if ((lane & 7) == 0) s_pot[wid][lane >> 3] = h1;
    __syncthreads();
    // every wave: lane = 8 v + j sums waves v and v + 8 of trial j, then over v, then arg-min over j
    const int jj = lane & 7, vv = lane >> 3;
    double tot = s_pot[vv][jj] + s_pot[vv + 8][jj];
    tot += __shfl_xor(tot, 8, 64);
    tot += __shfl_xor(tot, 16, 64);
    tot += __shfl_xor(tot, 32, 64);
    if (jj >= L) tot = INFINITY;
    int bj = jj;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      const double ot = __shfl_xor(tot, o, 64);
      const int oj = __shfl_xor(bj, o, 64);
      if (ot < tot || (ot == tot && oj < bj)) { tot = ot; bj = oj; }
    }
    const int best = __builtin_amdgcn_readfirstlane(bj);
#pragma unroll
    for (int j = 0; j < KPR_LT; ++j) {
      if (j == best) {
#pragma unroll
        for (int q = 0; q < KPR_PER; ++q)
          if (q < cnt) d2[q] = fmin(d2[q], g[j][q]);
      }
    }
    c = __builtin_amdgcn_readfirstlane(pick[best]);
    if (tid == 0) out[t] = c;
  }
}

// G: nc x nc, row stride ldg >= nc; the register kernel needs ldg % 4 == 0 and a 32-B aligned G
SRML_API int srml_kmeanspp_gram(const double* G, int nc, long ldg, const double* w, int k, int trials,
                                unsigned long long seed, int* out, hipStream_t stream) {
  if (nc <= 0 || k <= 0) return 0;
  if (nc > KPP_T * KPP_PER || trials < 1 || trials > KPP_TRIALS || ldg < nc) return (int)hipErrorInvalidValue;
  const char* e = getenv("SRML_KPP_KERNEL");  // =block forces the chunked kernel (A/B; read per call)
  const int mode = e && !strcmp(e, "block") ? 1 : 0;
  if (mode == 0 && nc <= KPP_T * KPR_PER && trials <= KPR_LT && ldg % KPR_PER == 0 && ((uintptr_t)G & 31) == 0)
    hipLaunchKernelGGL(kmeanspp_gram_reg_kernel, dim3(1), dim3(KPP_T), 0, stream, G, nc, ldg, w, k, trials, seed,
                       out);
  else
    hipLaunchKernelGGL(kmeanspp_gram_kernel, dim3(1), dim3(KPP_T), 0, stream, G, nc, ldg, w, k, trials, seed, out);
  return srml_status();
}

namespace {

// ------------------------------------------------------------------------------------------
// Small-k Lloyd step, fused (k <= 32, n <= 64, the BASELINE KMeans k = 20 on 100M x 64): ONE
// pass over X per iteration computes every row's nearest centre AND the per-cluster sums / counts
// by those labels (and the inertia), where the generic path read X twice (distance GEMM, then
// cluster sums) with short-lived blocks that ran latency-bound (~0.6 TB/s at n = 64).
//   * a thread owns one row (NV float4 in registers, the wave's 64 rows = 64 x 16 KB in flight);
//   * distances on the VALU against the centres held transposed in LDS (cT[d][KP]: the KP values
//     of column d are one broadcast ds_read per 4 centres), packed fp32 FMAs, arg-min with the
//     lowest index on ties (the MFMA search's tie rule);
//   * cluster sums as a one-hot GEMM on the fp32 matrix cores: the wave stages its 64 rows in LDS,
//     A = one-hot(label) (32 clusters x 2 rows), B = the rows (2 x 32 columns) per
//     v_mfma_f32_32x32x2f32, accumulators = sums[cluster][column] across all the wave's row groups;
//   * persistent blocks (grid <= 2 per CU) loop over 256-row groups; at the end the 4 waves'
//     accumulators are summed in LDS and each block adds its k x n partial with fp64 atomics
//     (sums / counts / inertia must start at zero).
// sums == nullptr: search only (labels / dist), e.g. the k-means|| passes.
template <int NV, int KP>
__global__ __launch_bounds__(256, 2) void lloyd_small_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                             const float* __restrict__ C, int k,
                                                             const float* __restrict__ cnorm,
                                                             int* __restrict__ labels, float* __restrict__ dist,
                                                             double* __restrict__ sums, int* __restrict__ counts,
                                                             double* __restrict__ inertia) {
  constexpr int NT = (4 * NV + 31) / 32;  // 32-column tiles of the sums
  constexpr int XST = 4 * NV + 4;          // staged row stride (floats): 16-B aligned, rotates banks
  __shared__ __attribute__((aligned(16))) float cT[4 * NV][KP];
  __shared__ float s_cn[KP];
  __shared__ __attribute__((aligned(16))) float xs[4][64 * XST];
  __shared__ int s_lab[4][64];
  __shared__ int s_cnt[32];
  __shared__ double s_in[4];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int li = lane & 31, lk = lane >> 5;
  const bool acc_sums = sums != nullptr;
  for (int i = t; i < 4 * NV * KP; i += 256) {
    const int d = i / KP, j = i % KP;
    cT[d][j] = (j < k && d < n) ? C[(long)j * n + d] : 0.f;
  }
  if (t < KP) s_cn[t] = t < k ? cnorm[t] : __builtin_huge_valf();
  if (t < 32) s_cnt[t] = 0;
  __syncthreads();
  floatx16 acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  double in_sum = 0.0;
  const long groups = (m + 255) / 256;
  float* xw = xs[wid];
  // the wave's 64 rows are read lane-linearly (float4 f = lane + 64 i of the 64 x NV float4 chunk:
  // consecutive lanes, consecutive 16 B when ld == n) one group AHEAD: the loads of group g + 1 are
  // in flight while group g's distances and one-hot MFMAs run; staged rows then go to LDS, where
  // each lane reads its own row back (XST = 4 NV + 4 keeps a 16-lane phase of ds_read_b128 on
  // distinct banks) and the MFMA loop reads its B fragments
  floatx4 pre[NV];
  auto fetch = [&](long g) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = lane + 64 * i, rr = f / NV, comp = f % NV;
      const long r = g * 256 + wid * 64 + rr;
      pre[i] = (g < groups && r < m && 4 * comp < n) ? *reinterpret_cast<const floatx4*>(X + r * ld + 4 * comp)
                                                    : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  fetch(blockIdx.x);
  for (long gi = blockIdx.x; gi < groups; gi += gridDim.x) {
    const long row = gi * 256 + t;
    const bool live = row < m;
    __builtin_amdgcn_wave_barrier();  // every lane is done with the previous group's staged rows
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = lane + 64 * i;
      *reinterpret_cast<floatx4*>(&xw[(f / NV) * XST + 4 * (f % NV)]) = pre[i];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    floatx4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) x[v] = *reinterpret_cast<const floatx4*>(&xw[lane * XST + 4 * v]);
    fetch(gi + gridDim.x);  // next group's rows: in flight under this group's work
    // distances: dp[j / 2] = (x.c_j, x.c_{j+1})
    typedef float float2v __attribute__((ext_vector_type(2)));
    float2v dp[KP / 2];
#pragma unroll
    for (int j = 0; j < KP / 2; ++j) dp[j] = float2v{0.f, 0.f};
    float xn = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float xv = x[v][q];
        xn = fmaf(xv, xv, xn);
        const float2v xx = float2v{xv, xv};
        const floatx4* cp = reinterpret_cast<const floatx4*>(&cT[4 * v + q][0]);
#pragma unroll
        for (int j4 = 0; j4 < KP / 4; ++j4) {
          const floatx4 c4 = cp[j4];
          dp[2 * j4] = __builtin_elementwise_fma(xx, float2v{c4[0], c4[1]}, dp[2 * j4]);
          dp[2 * j4 + 1] = __builtin_elementwise_fma(xx, float2v{c4[2], c4[3]}, dp[2 * j4 + 1]);
        }
      }
    }
    float bv = __builtin_huge_valf();
    int bi = 0;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      const float d = fmaf(-2.f, dp[j / 2][j & 1], s_cn[j]);  // +inf for j >= k
      if (d < bv) { bv = d; bi = j; }
    }
    float dd = bv + xn;
    dd = dd > 0.f ? dd : 0.f;
    if (live) {
      labels[row] = bi;
      dist[row] = dd;
      in_sum += (double)dd;
    }
    if (!acc_sums) continue;
    // one-hot GEMM over the wave's 64 staged rows
    s_lab[wid][lane] = live ? bi : -1;
    if (live) atomicAdd(&s_cnt[bi], 1);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll 4
    for (int s2 = 0; s2 < 32; ++s2) {
      const int rr = 2 * s2 + lk;
      const float a = s_lab[wid][rr] == li ? 1.f : 0.f;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        const int col = q * 32 + li;
        const float b = col < 4 * NV ? xw[rr * XST + col] : 0.f;
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[q], 0, 0, 0);
      }
    }
  }
  // block totals: inertia, counts, sums (4 waves' accumulators through LDS, one wave flushes)
  {
    double v = in_sum;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_in[wid] = v;
  }
  __syncthreads();
  if (t == 0 && inertia) atomicAdd(inertia, (s_in[0] + s_in[1]) + (s_in[2] + s_in[3]));
  if (!acc_sums) return;
  if (t < k && s_cnt[t]) atomicAdd(&counts[t], s_cnt[t]);
  // acc[q][r] = sums[cluster (r&3) + 8(r>>2) + 4 lk][column q * 32 + li]; reuse xs as [4][32][NT*32]
  float* red = &xs[0][0];
  constexpr int RW = NT * 32;
#pragma unroll
  for (int q = 0; q < NT; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cl = (r & 3) + 8 * (r >> 2) + 4 * lk;
      red[(wid * 32 + cl) * RW + q * 32 + li] = acc[q][r];
    }
  __syncthreads();
  for (int i = t; i < k * n; i += 256) {
    const int cl = i / n, col = i % n;
    const float v = (red[(0 * 32 + cl) * RW + col] + red[(1 * 32 + cl) * RW + col]) +
                    (red[(2 * 32 + cl) * RW + col] + red[(3 * 32 + cl) * RW + col]);
    if (v != 0.f) atomicAdd(&sums[(long)cl * n + col], (double)v);
  }
}

}  // namespace

// Fused small-k Lloyd step (see lloyd_small_kernel): labels / squared distances of every row, and
// when sums != null the per-cluster fp64 sums, int32 counts and the fp64 inertia (all three must be
// zeroed by the caller). Needs k <= 32 (the VALU search of k = 41 measured 4.1 ms at 10M x 64,
// no faster than the MFMA search), n <= 64,
// n % 4 == 0, ld % 4 == 0, 16-B aligned X. (Centres through the scalar path instead of LDS
// broadcast reads measured 3.7x slower.)
SRML_API int srml_kmeans_lloyd_small(const float* X, long m, int n, long ld, const float* C, int k,
                                     const float* cnorm, int* labels, float* dist, double* sums, int* counts,
                                     double* inertia, hipStream_t stream) {
  if (m <= 0) return 0;
  if (k < 1 || k > 32 || n < 1 || n > 64 || (n & 3) || (ld & 3) ||
      (reinterpret_cast<uintptr_t>(X) & 15))
    return (int)hipErrorInvalidValue;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const long groups = (m + 255) / 256;
  const unsigned grid = (unsigned)(groups < 2L * cus ? groups : 2L * cus);
#define SRML_LLOYD(NV, KP)                                                                                         \
  hipLaunchKernelGGL((lloyd_small_kernel<NV, KP>), dim3(grid), dim3(256), 0, stream, X, m, n, ld, C, k, cnorm, labels, \
                     dist, sums, counts, inertia)
#define SRML_LLOYD_K(NV)                  \
  do {                                    \
    if (k <= 8) SRML_LLOYD(NV, 8);        \
    else if (k <= 16) SRML_LLOYD(NV, 16); \
    else if (k <= 24) SRML_LLOYD(NV, 24); \
    else SRML_LLOYD(NV, 32);              \
  } while (0)
  if (n <= 16) SRML_LLOYD_K(4);
  else if (n <= 32) SRML_LLOYD_K(8);
  else SRML_LLOYD_K(16);
#undef SRML_LLOYD_K
#undef SRML_LLOYD
  return srml_status();
}

