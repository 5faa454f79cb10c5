// Large-k exact kNN (64 < k <= 1024) and the row-wise top-k selection shared with the k <= 64
// slice merge.
//
//  * srml_knn_dist_f32 — D[q][i] = ||i||^2 - 2 q.i for a (query chunk x item chunk) on the fp32
//      matrices cores (the 128x128 `gemm_tile_128` MFMA tile shared with KMeans/DBSCAN), XCD-
//      remapped so the item tiles of one query panel share an L2. The register/LDS-resident
//      insertion lists of `srml_knn_f32` stop paying past k = 64 (the list no longer fits and every
//      candidate pays an O(k) insertion), so for large k the distances of a bounded chunk are
//      materialised (<= 1 GB, sized by the caller) and selected by:
//  * srml_topk_rows_f32 — one block per (row, column slice): exact k-smallest by a three-pass
//      radix select on orderable 32-bit keys (11/11/10-bit digits, LDS histograms, block scan to
//      find the digit holding the k-th key), then ONE ordered collection pass (block scans in
//      index order, so ties at the threshold keep the lowest columns and the result is
//      deterministic) and a bitonic sort of (key, column) pairs in LDS. Optional input ids turn
//      the same kernel into the merge of per-slice / per-chunk partial lists.
// Reference: cuML NearestNeighborsMG brute force + RAFT select_k (knn.py:638-749).
#include "common.h"

#include "tile.h"

namespace {
using namespace srml_tile;

constexpr int TK_T = 256;
// k <= TK_KMAX: the selected (key, column) pairs are bitonic-sorted in dynamic LDS sized to the
// next power of two of k (8 B per pair: 128 KiB at k = 16384)
constexpr int TK_KMAX = 16384;

template <bool VEC>
__global__ __launch_bounds__(256, 2) void knn_dist_kernel(const float* __restrict__ Q, long mq, int n, long ldq,
                                                          const float* __restrict__ I, long mi, long ldi,
                                                          const float* __restrict__ inorm, float* __restrict__ D,
                                                          long ldd, int n_itiles) {
  __shared__ Stage128 st;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const long qt = bid / n_itiles;
  const int it = bid % n_itiles;
  floatx16 acc[2][2];
  gemm_tile_128<VEC>(Q, ldq, mq, qt * 128, I, ldi, mi, (long)it * 128, n, st, acc);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    const long i = (long)it * 128 + acc_col(nt);
    const float in = i < mi ? inorm[i] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long q = qt * 128 + acc_row(mt, r);
        if (q < mq && i < mi) D[q * ldd + i] = fmaf(-2.f, acc[mt][nt][r], in);
      }
  }
}

// exclusive block scan of one int per thread (256 threads); `total` = block sum
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  int base = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int tw = s_w[w];
    if (w < wid) base += tw;
    total += tw;
  }
  __syncthreads();
  return base + x - v;
}

__global__ __launch_bounds__(TK_T) void topk_rows_kernel(const float* __restrict__ vals, long ldv, long slice_len,
                                                         int L_total, const long long* __restrict__ ids, long ldid,
                                                         long long id_base, int k, float* __restrict__ out_v,
                                                         long long* __restrict__ out_i, long ldo, long slice_ldo) {
  __shared__ int hist[2048];
  extern __shared__ unsigned tk_dyn[];  // skey[kpad] | spos[kpad]
  int kp2 = 1;
  while (kp2 < k) kp2 <<= 1;
  unsigned* skey = tk_dyn;
  int* spos = reinterpret_cast<int*>(tk_dyn + kp2);
  __shared__ int s_w[4];
  __shared__ int s_digit, s_below;
  const long row = blockIdx.x;
  const long c0 = (long)blockIdx.y * slice_len;
  const int L = (int)min(slice_len, (long)L_total - c0);
  const float* v = vals + row * ldv + c0;
  const int t = threadIdx.x;
  const int kk = L < k ? (L > 0 ? L : 0) : k;
  const bool take_all = kk == L;
  unsigned prefix = 0u, mask = 0u;
  int need = kk;
  if (!take_all) {
    for (int pass = 0; pass < 3; ++pass) {
      const int shift = pass == 0 ? 21 : (pass == 1 ? 10 : 0);
      const unsigned nb = pass == 2 ? 1024u : 2048u;
      for (int i = t; i < 2048; i += TK_T) hist[i] = 0;
      __syncthreads();
      for (int i = t; i < L; i += TK_T) {
        const unsigned key = orderable(v[i]);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & (nb - 1u)], 1);
      }
      __syncthreads();
      int loc[8];
      int s = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) { loc[b] = hist[8 * t + b]; s += loc[b]; }
      int total;
      const int base = block_excl_scan(s, s_w, total);
      if (base < need && need <= base + s) {
        int cum = base;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          if (cum + loc[b] >= need) { s_digit = 8 * t + b; s_below = cum; break; }
          cum += loc[b];
        }
      }
      __syncthreads();
      prefix |= (unsigned)s_digit << shift;
      mask |= (nb - 1u) << shift;
      need -= s_below;
      __syncthreads();
    }
  }
  // ordered collection: keys < T in column order, then the first `need` keys == T
  const unsigned T = prefix;
  const int nless = kk - need;
  int run_lt = 0, run_eq = 0;
  for (int b0 = 0; b0 < L; b0 += TK_T) {
    const int i = b0 + t;
    const unsigned key = i < L ? orderable(v[i]) : 0xffffffffu;
    const bool lt = i < L && (take_all || key < T);
    const bool eq = i < L && !take_all && key == T;
    int total;
    const int ex = block_excl_scan((lt ? 1 : 0) | (eq ? (1 << 16) : 0), s_w, total);
    if (lt) {
      const int p = run_lt + (ex & 0xffff);
      skey[p] = key;
      spos[p] = i;
    }
    if (eq) {
      const int r = run_eq + (ex >> 16);
      if (r < need) {
        skey[nless + r] = key;
        spos[nless + r] = i;
      }
    }
    run_lt += total & 0xffff;
    run_eq += total >> 16;
  }
  int kpad = 1;
  while (kpad < kk) kpad <<= 1;
  for (int p = kk + t; p < kpad; p += TK_T) { skey[p] = 0xffffffffu; spos[p] = 0x7fffffff; }
  __syncthreads();
  for (int size = 2; size <= kpad; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < kpad; i += TK_T) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const unsigned ki = skey[i], kj = skey[j];
          const int pi = spos[i], pj = spos[j];
          const bool gt = ki > kj || (ki == kj && pi > pj);
          if (gt == up) { skey[i] = kj; skey[j] = ki; spos[i] = pj; spos[j] = pi; }
        }
      }
      __syncthreads();
    }
  }
  float* ov = out_v + row * ldo + (long)blockIdx.y * slice_ldo;
  long long* oi = out_i + row * ldo + (long)blockIdx.y * slice_ldo;
  for (int p = t; p < k; p += TK_T) {
    if (p < kk) {
      const int c = spos[p];
      ov[p] = unorderable(skey[p]);
      oi[p] = ids ? ids[row * ldid + c0 + c] : id_base + c0 + c;
    } else {
      ov[p] = __builtin_huge_valf();
      oi[p] = -1;
    }
  }
}

// Exact re-scoring + sort of a query's <= 64 selected candidates (the kNN refine step: direct
// q - x distances instead of ||x||^2 - 2 q.x, so near-duplicates keep their digits). One wave per
// query: the query sits in registers (lanes over dimensions), every candidate row is read once
// coalesced and wave-reduced on DPP, then the (distance, position) pairs are bitonic-sorted across
// the 64 lanes (ties keep the candidate order). Replaces index_select of the candidate rows +
// elementwise + reduction + torch.sort (the gathered rows never touch HBM).
// metric 0: squared euclidean; 1: -2 q.x (inner product, ascending = most similar first).
// TAIL: dimensions past the 64*QT held in registers are streamed (the query row stays L2-hot
// across the k candidates), so any n is served.
template <int QT, bool TAIL>
__global__ __launch_bounds__(256) void knn_refine_sort_kernel(const float* __restrict__ Q, long mq, int n, long ldq,
                                                              const float* __restrict__ X, long ldx,
                                                              const long long* __restrict__ pos, int k, long ldp,
                                                              int metric, float* __restrict__ dout,
                                                              long long* __restrict__ pout) {
  const long q = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= mq) return;  // wave-uniform
  float qv[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int d = lane + 64 * t;
    qv[t] = d < n ? Q[q * ldq + d] : 0.f;
  }
  const long long mine = lane < k ? pos[q * ldp + lane] : -1;
  float my = __builtin_huge_valf();
  for (int j = 0; j < k; ++j) {
    const long long c = __shfl(mine, j, 64);  // wave-uniform candidate
    if (c < 0) continue;
    const float* xr = X + c * ldx;
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int d = lane + 64 * t;
      if (d < n) {
        const float x = xr[d];
        if (metric == 0) {
          const float df = qv[t] - x;
          acc = fmaf(df, df, acc);
        } else {
          acc = fmaf(qv[t], x, acc);
        }
      }
    }
    if (TAIL) {
      for (int d = 64 * QT + lane; d < n; d += 64) {
        const float qd = Q[q * ldq + d], x = xr[d];
        if (metric == 0) {
          const float df = qd - x;
          acc = fmaf(df, df, acc);
        } else {
          acc = fmaf(qd, x, acc);
        }
      }
    }
    const float tot = wave_sum(acc);
    if (lane == j) my = metric == 0 ? tot : -2.f * tot;
  }
  // bitonic sort of (my, lane) ascending across the wave. A NaN distance (NaN features) sorts as
  // +inf: `<` / `==` give no order for NaN, which could let padding lanes (>= k) into the first k;
  // +inf ties break by lane id, so every candidate lane (< k) still precedes the padding
  if (my != my) my = __builtin_huge_valf();
  float v = my;
  int id = lane;
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float ov = __shfl_xor(v, stride, 64);
      const int oid = __shfl_xor(id, stride, 64);
      const bool up = ((lane & size) == 0);
      const bool lower = (lane & stride) == 0;
      const bool o_less = ov < v || (ov == v && oid < id);
      // the lower lane of an ascending pair keeps the smaller element
      const bool take = (lower == up) ? o_less : !o_less;
      if (take) {
        v = ov;
        id = oid;
      }
    }
  }
  const long long src = __shfl(mine, id, 64);
  if (lane < k) {
    dout[q * k + lane] = v;
    pout[q * k + lane] = src < 0 ? -1 : src;
  }
}
}  // namespace

// D (mq x mi, leading dim ldd) = inorm[i] - 2 Q I^T for one (query chunk, item chunk).
SRML_API int srml_knn_dist_f32(const float* Q, long mq, int n, long ldq, const float* I, long mi, long ldi,
                               const float* inorm, float* D, long ldd, hipStream_t stream) {
  if (mq <= 0 || mi <= 0) return 0;
  const long nq = (mq + 127) / 128, ni = (mi + 127) / 128;
  if (nq * ni > 0x7fffffffL || ni > 0x7fffffffL) return -1;
  const bool vec = ((ldq & 3) == 0) && ((ldi & 3) == 0) && ((n & 3) == 0) &&
                   ((reinterpret_cast<uintptr_t>(Q) & 15) == 0) && ((reinterpret_cast<uintptr_t>(I) & 15) == 0);
  if (vec)
    hipLaunchKernelGGL(knn_dist_kernel<true>, dim3((unsigned)(nq * ni)), dim3(256), 0, stream, Q, mq, n, ldq, I, mi, ldi,
                       inorm, D, ldd, (int)ni);
  else
    hipLaunchKernelGGL(knn_dist_kernel<false>, dim3((unsigned)(nq * ni)), dim3(256), 0, stream, Q, mq, n, ldq, I, mi,
                       ldi, inorm, D, ldd, (int)ni);
  return srml_status();
}

// Row-wise k smallest (ascending, ties by column) of `rows` rows of L_total values (leading dim
// ldv), split into column slices of `slice_len` (grid.y); slice s of row r writes k results at
// out[r * ldo + s * slice_ldo]. ids: optional int64 ids of the input values (leading dim ldid);
// without them the id of column c is id_base + c. k <= 16384.
SRML_API int srml_topk_rows_f32(const float* vals, long rows, long ldv, long slice_len, int L_total,
                                const long long* ids, long ldid, long long id_base, int k, float* out_v,
                                long long* out_i, long ldo, long slice_ldo, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (k <= 0 || k > TK_KMAX || slice_len <= 0 || L_total <= 0) return -1;
  const long slices = (L_total + slice_len - 1) / slice_len;
  if (rows > 0x7fffffffL || slices > 65535) return -1;
  int kp2 = 1;
  while (kp2 < k) kp2 <<= 1;
  const size_t shm = (size_t)kp2 * (sizeof(unsigned) + sizeof(int));
  if (shm > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)topk_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(topk_rows_kernel, dim3((unsigned)rows, (unsigned)slices), dim3(TK_T), shm, stream, vals, ldv,
                     slice_len, L_total, ids, ldid, id_base, k, out_v, out_i, ldo, slice_ldo);
  return srml_status();
}

SRML_API int srml_topk_kmax() { return TK_KMAX; }

// ------------------------------------------------------------------------------------------
// IVF large-k candidates (64 < k <= 1024; the k <= 64 paths keep LDS insertion lists): for every
// (query, probe) the distances ||i||^2 - 2 q.i to each item of the probed list are written, with
// the item's id (or list position), into the query's row of a candidate matrix at the prefix
// offset of its earlier probes; columns past the query's candidate count are +inf / -1. One block
// per (query, probe): the query vector is staged in LDS once, the list's items stream through
// 64-row LDS tiles (coalesced 16-B row loads, row stride n + 1 words: conflict-free column reads)
// and each thread forms one item's dot product. srml_topk_rows_f32 (with ids) then selects k per
// query. qlist: optional query -> list map (all-points kNN over IVF lists: a row probes the lists
// of its own list's probe set); without it probes are per query.
// ------------------------------------------------------------------------------------------
constexpr int IVC_T = 256;
constexpr int IVC_ROWS = 64;
constexpr int IVC_NC = 512;  // feature chunk staged in LDS (133 KiB with the 64-row tile)

__global__ __launch_bounds__(IVC_T) void ivf_candidates_kernel(const float* __restrict__ Q, long q0, int n, long ldq,
                                                               const int* __restrict__ probes, int nprobe,
                                                               const int* __restrict__ qlist,
                                                               const long long* __restrict__ list_off,
                                                               const float* __restrict__ items, long ldi,
                                                               const float* __restrict__ inorm,
                                                               const long long* __restrict__ ids, float* __restrict__ D,
                                                               long long* __restrict__ DI, long ldd, int nc) {
  // features are staged in chunks of nc (= min(n, IVC_NC)) columns, so any width fits the LDS:
  // each row's dot product accumulates in its thread's register across the chunks
  extern __shared__ float ivc_s[];  // q chunk [nc] | tile[IVC_ROWS][nc + 1]
  float* qs = ivc_s;
  float* tile = ivc_s + nc;
  const int tn = nc + 1;
  const long qi = q0 + blockIdx.x;  // global query (row) index
  const int p = blockIdx.y;
  const int* pr = probes + (long)(qlist ? qlist[qi] : qi) * nprobe;
  const int l = pr[p];
  // this probe's offset in the query's candidate row
  long off = 0;
  for (int j = 0; j < p; ++j)
    if (pr[j] >= 0) off += list_off[pr[j] + 1] - list_off[pr[j]];
  if (l < 0) return;
  const long b0 = list_off[l], b1 = list_off[l + 1];
  float* drow = D + (long)blockIdx.x * ldd + off;
  long long* irow = DI + (long)blockIdx.x * ldd + off;
  for (long r0 = b0; r0 < b1; r0 += IVC_ROWS) {
    const int rows = (int)min((long)IVC_ROWS, b1 - r0);
    float acc = 0.f;
    for (int c0 = 0; c0 < n; c0 += nc) {
      const int w = min(nc, n - c0);
      __syncthreads();  // previous chunk / tile consumed
      for (int c = threadIdx.x; c < w; c += IVC_T) qs[c] = Q[qi * ldq + c0 + c];
      for (int e = threadIdx.x; e < rows * w; e += IVC_T) {
        const int rr = e / w, cc = e - rr * w;
        tile[rr * tn + cc] = items[(r0 + rr) * ldi + c0 + cc];
      }
      __syncthreads();
      if (threadIdx.x < rows) {
        const float* row = tile + threadIdx.x * tn;
        for (int c = 0; c < w; ++c) acc = fmaf(qs[c], row[c], acc);
      }
    }
    if (threadIdx.x < rows) {
      const long it = r0 + threadIdx.x;
      drow[it - b0] = inorm[it] - 2.f * acc;
      irow[it - b0] = ids ? ids[it] : it;
    }
  }
}

__global__ void ivf_count_kernel(const int* __restrict__ probes, int nprobe, const int* __restrict__ qlist, long nq,
                                 const long long* __restrict__ list_off, unsigned long long* __restrict__ cmax) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const int* pr = probes + (long)(qlist ? qlist[q] : q) * nprobe;
  unsigned long long c = 0;
  for (int j = 0; j < nprobe; ++j)
    if (pr[j] >= 0) c += (unsigned long long)(list_off[pr[j] + 1] - list_off[pr[j]]);
  atomicMax(cmax, c);
}

// Largest candidate count over nq queries (-> *cmax, which the caller zeroes): sizes the matrix.
SRML_API int srml_ivf_candidate_max(const int* probes, int nprobe, const int* qlist, long nq, const long long* list_off,
                                    unsigned long long* cmax, hipStream_t stream) {
  if (nq <= 0) return 0;
  hipLaunchKernelGGL(ivf_count_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, stream, probes, nprobe, qlist,
                     nq, list_off, cmax);
  return srml_status();
}

__global__ void row_list_kernel(const long long* __restrict__ list_off, int nlist, long N, int* __restrict__ qlist) {
  const long r = (long)blockIdx.x * 256 + threadIdx.x;
  if (r >= N) return;
  int lo = 0, hi = nlist - 1;  // largest l with list_off[l] <= r
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (list_off[mid] <= r) lo = mid; else hi = mid - 1;
  }
  qlist[r] = lo;
}

// List of every row of a list-sorted matrix (list_off: nlist + 1 offsets covering the N rows).
SRML_API int srml_row_list(const long long* list_off, int nlist, long N, int* qlist, hipStream_t stream) {
  if (N <= 0 || nlist <= 0) return 0;
  hipLaunchKernelGGL(row_list_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, stream, list_off, nlist, N, qlist);
  return srml_status();
}

__global__ void ivf_fill_kernel(float* __restrict__ D, long long* __restrict__ DI, long total) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  D[i] = __builtin_huge_valf();
  DI[i] = -1;
}

// Candidate matrix rows for queries [q0, q0 + nq) (row r of D / DI = query q0 + r, ldd columns,
// ldd >= the largest candidate count of these queries; the caller sizes it).
SRML_API int srml_ivf_candidates_f32(const float* Q, long q0, long nq, int n, long ldq, const int* probes, int nprobe,
                                     const int* qlist, const long long* list_off, const float* items, long ldi,
                                     const float* inorm, const long long* ids, float* D, long long* DI, long ldd,
                                     hipStream_t stream) {
  if (nq <= 0) return 0;
  if (n <= 0 || nprobe <= 0 || nprobe > 65535 || nq > 0x7fffffffL || ldd <= 0) return -1;
  const int nc = n < IVC_NC ? n : IVC_NC;
  const size_t shm = (size_t)(nc + IVC_ROWS * (nc + 1)) * sizeof(float);
  const long total = nq * ldd;
  hipLaunchKernelGGL(ivf_fill_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, D, DI, total);
  if (shm > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)ivf_candidates_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipLaunchKernelGGL(ivf_candidates_kernel, dim3((unsigned)nq, (unsigned)nprobe), dim3(IVC_T), shm, stream, Q, q0, n,
                     ldq, probes, nprobe, qlist, list_off, items, ldi, inorm, ids, D, DI, ldd, nc);
  return srml_status();
}

// Q (mq x n, ld ldq) fp32, X (items x n, ld ldx) fp32, pos (mq x k, ld ldp) int64 candidate rows
// of X (-1 = none, sorts last at +inf); k <= 64, n <= 1024. Outputs dout / pout (mq x k, dense).
SRML_API int srml_knn_refine_sort_f32(const float* Q, long mq, int n, long ldq, const float* X, long ldx,
                                      const long long* pos, int k, long ldp, int metric, float* dout, long long* pout,
                                      hipStream_t stream) {
  if (mq <= 0) return 0;
  if (k < 1 || k > 64 || n < 1 || ldq < n || ldx < n || ldp < k || (metric != 0 && metric != 1)) return -2;
  const dim3 grid(ceil_div(mq, 4)), blk(256);
#define SRML_KRS(QQ) \
  hipLaunchKernelGGL(QQ, grid, blk, 0, stream, Q, mq, n, ldq, X, ldx, pos, k, ldp, metric, dout, pout)
  if (n <= 64) SRML_KRS((knn_refine_sort_kernel<1, false>));
  else if (n <= 128) SRML_KRS((knn_refine_sort_kernel<2, false>));
  else if (n <= 256) SRML_KRS((knn_refine_sort_kernel<4, false>));
  else if (n <= 512) SRML_KRS((knn_refine_sort_kernel<8, false>));
  else if (n <= 1024) SRML_KRS((knn_refine_sort_kernel<16, false>));
  else SRML_KRS((knn_refine_sort_kernel<16, true>));
#undef SRML_KRS
  return srml_status();
}
