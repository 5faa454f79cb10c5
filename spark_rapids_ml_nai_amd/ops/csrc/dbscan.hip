// DBSCAN kernels (reference: cuML DBSCANMG brute force, clustering.py:940-998).
//
// The N x N eps-adjacency is never materialised. Both passes sweep the lower triangle of 128 x 128
// tile pairs (bj <= bi, a rank owns a contiguous range of that linear tile index) and recompute the
// tile's distances on MFMA (||a||^2 + ||b||^2 - 2 a.b, fp32):
//   srml_dbscan_degree_f32: eps-degree of every row (self included); each tile counts its rows
//     and, off the diagonal, its columns (symmetry) -> one global atomicAdd per row / column.
//   srml_dbscan_link_f32: connected components of the core points. Inside a tile the core-core
//     eps edges are merged with a 256-slot union-find in LDS (rows = slots 0..127, columns =
//     128..255); only the resulting local spanning edges (<= 255 per tile instead of up to 16K)
//     are applied to the global lock-free union-find (hook larger root under smaller with CAS,
//     path halving — the ECL-CC scheme), so the root of every component is its smallest index.
//     Border points keep the nearest core neighbour as a packed (orderable dist << 32 | index)
//     64-bit atomicMin key.
//   srml_uf_unite_pairs / srml_uf_compress: merge another rank's forest, flatten to roots.
#include "common.h"
#include "tile.h"

namespace {
using namespace srml_tile;

__device__ __forceinline__ void tri_decode(long t, long& bi, long& bj) {
  double d = sqrt(8.0 * (double)t + 1.0);
  long i = (long)((d - 1.0) * 0.5);
  while (i > 0 && i * (i + 1) / 2 > t) --i;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  bi = i;
  bj = t - i * (i + 1) / 2;
}

union DbSmem {
  Stage128 st;
  float D[128][129];
};

template <bool VEC>
__device__ __forceinline__ void distance_tile(const float* __restrict__ X, long N, int n, long ld,
                                              const float* __restrict__ xnorm, float eps2, long r0, long c0,
                                              DbSmem& sm) {
  floatx16 acc[2][2];
  gemm_tile_128<VEC>(X, ld, N, r0, X, ld, N, c0, n, sm.st, acc);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const int cl = acc_col(nt);
    const long gc = c0 + cl;
    const float cn = gc < N ? xnorm[gc] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = acc_row(mt, r);
        const long gr = r0 + rl;
        const float rn = gr < N ? xnorm[gr] : 0.f;
        const float d = fmaxf(fmaf(-2.f, acc[mt][nt][r], rn + cn), 0.f);
        sm.D[rl][cl] = (gr < N && gc < N && d <= eps2) ? d : __builtin_huge_valf();
      }
  }
  __syncthreads();
}

template <bool VEC>
__global__ __launch_bounds__(256, 2) void dbscan_degree_kernel(const float* __restrict__ X, long N, int n, long ld,
                                                               const float* __restrict__ xnorm, float eps2, long t0,
                                                               long t1, int* __restrict__ counts) {
  __shared__ DbSmem sm;
  const int t = threadIdx.x;
  for (long tile = t0 + blockIdx.x; tile < t1; tile += gridDim.x) {
    long bi, bj;
    tri_decode(tile, bi, bj);
    const long r0 = bi * 128, c0 = bj * 128;
    distance_tile<VEC>(X, N, n, ld, xnorm, eps2, r0, c0, sm);
    if (t < 128) {
      int cnt = 0;
      for (int c = 0; c < 128; ++c) cnt += sm.D[t][c] != __builtin_huge_valf();
      if (cnt) atomicAdd(&counts[r0 + t], cnt);
    } else if (bi != bj) {
      const int c = t - 128;
      int cnt = 0;
      for (int r = 0; r < 128; ++r) cnt += sm.D[r][c] != __builtin_huge_valf();
      if (cnt) atomicAdd(&counts[c0 + c], cnt);
    }
    __syncthreads();
  }
}

// ---- union-find -------------------------------------------------------------------------------
__device__ __forceinline__ int uf_find(volatile int* p, int x) {
  int y = p[x];
  while (y != x) {
    const int z = p[y];
    if (z != y) p[x] = z;  // path halving; parents only ever point to smaller indices
    x = y;
    y = z;
  }
  return x;
}

__device__ __forceinline__ void uf_unite(int* p, int a, int b) {
  volatile int* vp = p;
  a = uf_find(vp, a);
  b = uf_find(vp, b);
  while (a != b) {
    if (a < b) {
      const int s = a;
      a = b;
      b = s;
    }
    const int old = atomicCAS(&p[a], a, b);  // hook the larger root under the smaller
    if (old == a) return;
    a = uf_find(vp, old);
    b = uf_find(vp, b);
  }
}

__device__ __forceinline__ unsigned long long nn_key(float d, long idx) {
  return ((unsigned long long)orderable(d) << 32) | (unsigned long long)(unsigned)idx;
}

template <bool VEC>
__global__ __launch_bounds__(256, 2) void dbscan_link_kernel(const float* __restrict__ X, long N, int n, long ld,
                                                             const float* __restrict__ xnorm, float eps2, long t0,
                                                             long t1, const unsigned char* __restrict__ core,
                                                             int* __restrict__ parent,
                                                             unsigned long long* __restrict__ best) {
  __shared__ DbSmem sm;
  __shared__ int lp[256];
  __shared__ unsigned char lcore[256];
  __shared__ unsigned long long cbest[128];
  const int t = threadIdx.x;
  for (long tile = t0 + blockIdx.x; tile < t1; tile += gridDim.x) {
    long bi, bj;
    tri_decode(tile, bi, bj);
    const long r0 = bi * 128, c0 = bj * 128;
    const long gid = t < 128 ? r0 + t : c0 + (t - 128);
    lcore[t] = gid < N ? core[gid] : 0;
    lp[t] = (bi == bj && t >= 128) ? t - 128 : t;  // diagonal tile: column slot c is row slot c
    if (t < 128) cbest[t] = ~0ull;
    distance_tile<VEC>(X, N, n, ld, xnorm, eps2, r0, c0, sm);  // ends with __syncthreads
    if (t < 128 && r0 + t < N) {
      const bool rc = lcore[t];
      unsigned long long rb = ~0ull;
      for (int c = 0; c < 128; ++c) {
        const float d = sm.D[t][c];
        if (d == __builtin_huge_valf()) continue;
        const bool cc = lcore[128 + c];
        if (rc && cc) {
          // local union in LDS (same CAS scheme on slot indices)
          volatile int* vp = lp;
          int a = uf_find(vp, t), b = uf_find(vp, 128 + c);
          while (a != b) {
            if (a < b) {
              const int s = a;
              a = b;
              b = s;
            }
            const int old = atomicCAS(&lp[a], a, b);
            if (old == a) break;
            a = uf_find(vp, old);
            b = uf_find(vp, b);
          }
        } else if (!rc && cc) {
          const unsigned long long key = nn_key(d, c0 + c);
          rb = key < rb ? key : rb;
        } else if (rc && !cc) {
          atomicMin(&cbest[c], nn_key(d, r0 + t));
        }
      }
      if (rb != ~0ull) atomicMin(&best[r0 + t], rb);
    }
    __syncthreads();
    if (t < 128 && cbest[t] != ~0ull) atomicMin(&best[c0 + t], cbest[t]);
    if (gid < N && lcore[t]) {
      const int r = uf_find((volatile int*)lp, t);
      if (r != t) {
        const long g2 = r < 128 ? r0 + r : c0 + (r - 128);
        if (g2 != gid) uf_unite(parent, (int)gid, (int)g2);
      }
    }
    __syncthreads();
  }
}

__global__ void uf_unite_pairs_kernel(int* __restrict__ parent, long N, const int* __restrict__ other) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long)gridDim.x * blockDim.x) {
    const int o = other[i];
    if (o != (int)i) uf_unite(parent, (int)i, o);
  }
}

__global__ void uf_compress_kernel(int* __restrict__ parent, long N) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long)gridDim.x * blockDim.x)
    parent[i] = uf_find((volatile int*)parent, (int)i);
}

inline bool vec_ok(const float* X, long ld, int n) {
  return ((ld & 3) == 0) && ((n & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
}

inline unsigned grid_for(long tiles) {
  long g = tiles < 8192 ? tiles : 8192;
  return (unsigned)(g < 1 ? 1 : g);
}
}  // namespace

// number of lower-triangle tile pairs for N rows
SRML_API long srml_dbscan_num_tiles(long N) {
  const long nt = (N + 127) / 128;
  return nt * (nt + 1) / 2;
}

SRML_API int srml_dbscan_degree_f32(const float* X, long N, int n, long ld, const float* xnorm, float eps2, long t0,
                                    long t1, int* counts, hipStream_t stream) {
  if (N <= 0 || t1 <= t0) return 0;
  if (N > 0x7fffffffL) return -3;
  if (vec_ok(X, ld, n))
    hipLaunchKernelGGL(dbscan_degree_kernel<true>, dim3(grid_for(t1 - t0)), dim3(256), 0, stream, X, N, n, ld, xnorm,
                       eps2, t0, t1, counts);
  else
    hipLaunchKernelGGL(dbscan_degree_kernel<false>, dim3(grid_for(t1 - t0)), dim3(256), 0, stream, X, N, n, ld, xnorm,
                       eps2, t0, t1, counts);
  return srml_status();
}

SRML_API int srml_dbscan_link_f32(const float* X, long N, int n, long ld, const float* xnorm, float eps2, long t0,
                                  long t1, const unsigned char* core, int* parent, unsigned long long* best,
                                  hipStream_t stream) {
  if (N <= 0 || t1 <= t0) return 0;
  if (N > 0x7fffffffL) return -3;
  if (vec_ok(X, ld, n))
    hipLaunchKernelGGL(dbscan_link_kernel<true>, dim3(grid_for(t1 - t0)), dim3(256), 0, stream, X, N, n, ld, xnorm,
                       eps2, t0, t1, core, parent, best);
  else
    hipLaunchKernelGGL(dbscan_link_kernel<false>, dim3(grid_for(t1 - t0)), dim3(256), 0, stream, X, N, n, ld, xnorm,
                       eps2, t0, t1, core, parent, best);
  return srml_status();
}

SRML_API int srml_uf_unite_pairs(int* parent, long N, const int* other, hipStream_t stream) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(uf_unite_pairs_kernel, dim3(grid_for((N + 255) / 256)), dim3(256), 0, stream, parent, N, other);
  return srml_status();
}

SRML_API int srml_uf_compress(int* parent, long N, hipStream_t stream) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(uf_compress_kernel, dim3(grid_for((N + 255) / 256)), dim3(256), 0, stream, parent, N);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Cluster labels from the compressed union-find forest (replaces a library unique + searchsorted):
// the components' roots are the core points that are their own parent (the smallest core index
// of each component), so cluster ids are the exclusive prefix count of those flags, read at each
// point's root: ids follow the roots' order, i.e. sklearn's first-core-point numbering.
//   K1: per 1024-element block the flags' exclusive prefix (wave scans) + the block total;
//   K2: one block scans the block totals;
//   K3: label = id of the root (core points), of the nearest core neighbour's root (border
//       points with one), -1 otherwise (noise).
// ------------------------------------------------------------------------------------------
namespace {
constexpr int DL_T = 1024;

__global__ __launch_bounds__(DL_T) void dbscan_root_prefix_kernel(const int* __restrict__ parent,
                                                                  const unsigned char* __restrict__ core, long N,
                                                                  int* __restrict__ local, int* __restrict__ btot) {
  __shared__ int ws[DL_T / 64];
  const long i = (long)blockIdx.x * DL_T + threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int f = (i < N && core[i] && parent[i] == (int)i) ? 1 : 0;
  int x = f;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) ws[wid] = x;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wid; ++w) base += ws[w];
  if (i < N) local[i] = base + x - f;
  if (threadIdx.x == DL_T - 1) btot[blockIdx.x] = base + x;
}

__global__ __launch_bounds__(DL_T) void dbscan_block_scan_kernel(int* __restrict__ btot, long nb) {
  __shared__ int carry;
  __shared__ int ws[DL_T / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (long c0 = 0; c0 < nb; c0 += DL_T) {
    const long i = c0 + threadIdx.x;
    const int v = i < nb ? btot[i] : 0;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) ws[wid] = x;
    __syncthreads();
    int base = carry;
    int tot = 0;
    for (int w = 0; w < DL_T / 64; ++w) {
      if (w < wid) base += ws[w];
      tot += ws[w];
    }
    if (i < nb) btot[i] = base + x - v;  // exclusive
    __syncthreads();
    if (threadIdx.x == 0) carry += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void dbscan_assign_labels_kernel(const int* __restrict__ parent,
                                                                   const unsigned char* __restrict__ core,
                                                                   const long long* __restrict__ best, long N,
                                                                   const int* __restrict__ local,
                                                                   const int* __restrict__ boff,
                                                                   long long* __restrict__ labels) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long)gridDim.x * 256) {
    long r = -1;
    if (core[i]) {
      r = parent[i];
    } else if (best[i] != -1) {
      const long nb = (long)(best[i] & 0xFFFFFFFFll);
      r = parent[nb < N ? nb : N - 1];
    }
    labels[i] = r < 0 ? -1 : (long long)(local[r] + boff[r / DL_T]);
  }
}
}  // namespace

// labels (int64, N) of DBSCAN points from the compressed forest `parent` (int32, roots = smallest
// core index), the core flags and `best` (nearest core neighbour in the low 32 bits, -1 = none).
// ws: 2 N + N / 1024 + 1 int32 of workspace.
SRML_API long srml_dbscan_labels_ws(long N) { return 2 * N + N / DL_T + 2; }

SRML_API int srml_dbscan_labels(const int* parent, const unsigned char* core, const long long* best, long N,
                                long long* labels, int* ws, hipStream_t stream) {
  if (N <= 0) return 0;
  const long nb = (N + DL_T - 1) / DL_T;
  int* local = ws;
  int* btot = ws + N;
  hipLaunchKernelGGL(dbscan_root_prefix_kernel, dim3((unsigned)nb), dim3(DL_T), 0, stream, parent, core, N, local,
                     btot);
  hipLaunchKernelGGL(dbscan_block_scan_kernel, dim3(1), dim3(DL_T), 0, stream, btot, nb);
  const long g = (N + 255) / 256;
  hipLaunchKernelGGL(dbscan_assign_labels_kernel, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, stream, parent,
                     core, best, N, local, btot, labels);
  return srml_status();
}
