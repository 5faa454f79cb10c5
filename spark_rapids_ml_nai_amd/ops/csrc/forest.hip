// Random-forest kernels: quantisation, level-wise histogram build, split search, row routing
// and forest inference (reference: cuML RandomForest{Classifier,Regressor} / FIL called from
// tree.py:309-414 and 571-613; SURVEY §2.4(c) RF rows).
//
// Data layout: the fp32 row-major feature block is quantised ONCE per fit into a FEATURE-MAJOR
// uint8 matrix (n x m): a histogram pass for feature f streams bins[f][row] for the node's rows,
// which are kept in ascending row order inside each node's segment of a row-index array (stable
// partitions), so reads are monotone and mostly coalesced at the top of the tree.
//
//  * srml_rf_quantize_u8 — 256-row x 32-feature tiles: coalesced fp32 row reads, per-feature
//    binary search in the (L1/L2-resident) edge table, LDS transpose, 256-byte feature rows out.
//  * srml_rf_hist — one block per work item (node, 8-feature chunk, row chunk): histograms are
//    privatised in LDS (ds_add) and flushed with one global atomic per non-empty cell.
//    Classification cells are per-class weighted counts (uint32); regression cells are
//    (count, sum y, sum y^2) in fp32 (fp64 fold on flush).
//  * srml_rf_best_split — one block per node: every thread sweeps the bins of one candidate
//    feature with running left statistics (Gini / entropy / variance gain, min-instances per
//    child), then a block arg-max (ties -> lowest feature slot, lowest bin).
//  * srml_rf_route — child key per row (2*slot + goes_right; dropped rows -> sentinel) for the
//    stable re-partition of the row-index array.
//  * srml_rf_predict_nodes2 — FIL-equivalent inference on raw fp32 rows, wave per row with the
//    trees spread over the 64 lanes. n <= 4096: the wave first streams its row into its own LDS
//    slice with coalesced 16-B loads, so the ~depth x trees feature gathers hit LDS and HBM sees X
//    exactly once; wider rows gather from global (all lanes on one row's lines at once, L1/L2
//    hits after the first touch). Nodes are one 16-B load each ({feature, left, right,
//    threshold}, breadth-first, L2-resident); per-lane class sums folded with DPP wave
//    reductions (fixed order: deterministic). srml_rf_predict (thread per row) stays for the
//    C ABI.
#include "common.h"

namespace {
constexpr int FB = 8;   // max features per histogram work item (runtime fb <= FB; ops.rf_hist_fb)
}

// ------------------------------------------------------------------------------------------
// Quantile bin edges: one block per feature sorts that feature's (transposed, contiguous) sample
// column in LDS with a bitonic network (k <= 32768, padded to a power of two with +inf; NaN sorts
// as +inf) and writes the order statistics floor(q_j * k), q_j = (j + 1) / (nq + 1). Replaces a
// segmented device sort of the whole (k x n) sample plus its index permutations (~15 ms / fit).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void rf_quantiles_kernel(const float* __restrict__ ST, int k, int kpad, int nq,
                                                            float* __restrict__ out) {
  extern __shared__ float key[];  // [kpad]
  const int f = blockIdx.x;
  const float* col = ST + (long)f * k;
  for (int i = threadIdx.x; i < kpad; i += 1024) {
    float v = i < k ? col[i] : INFINITY;
    key[i] = (v != v) ? INFINITY : v;
  }
  __syncthreads();
  for (int size = 2; size <= kpad; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < (kpad >> 1); i += 1024) {
        const int pos = 2 * i - (i & (stride - 1));
        const int q = pos + stride;
        const float a = key[pos], b = key[q];
        const bool asc = (pos & size) == 0;
        if ((a > b) == asc) {
          key[pos] = b;
          key[q] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int j = threadIdx.x; j < nq; j += 1024) {
    long p = (long)((double)(j + 1) / (double)(nq + 1) * (double)k);
    if (p > k - 1) p = k - 1;
    if (p < 0) p = 0;
    out[(long)f * nq + j] = key[p];
  }
}

SRML_API int srml_rf_quantiles_f32(const float* ST, int k, int n, int nq, float* out, hipStream_t stream) {
  if (n <= 0 || nq <= 0) return 0;
  if (k <= 0 || k > 32768) return (int)hipErrorInvalidValue;
  int kpad = 2;
  while (kpad < k) kpad <<= 1;
  const size_t lds = (size_t)kpad * sizeof(float);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)rf_quantiles_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(rf_quantiles_kernel, dim3((unsigned)n), dim3(1024), lds, stream, ST, k, kpad, nq, out);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Quantisation: a block owns 32 features x QROWS rows. The 32 edge tables are staged in LDS
// (row stride NE2 + 1 floats: table f starts in bank f, so the first search step of the 32 lanes
// reading one row is conflict-free), and bin(x) = #edges strictly below x is a branchless
// lower_bound over the +inf-padded power-of-two table (log2 NE2 LDS reads, no divergence).
// Rows are processed 256 at a time: coalesced fp32 reads (32 features = 128 B per row), the
// byte tile is transposed in LDS and written as 256-byte feature rows.
// ------------------------------------------------------------------------------------------
constexpr int QROWS = 1024;

__global__ __launch_bounds__(256) void rf_quantize_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                          const float* __restrict__ edges, int nedges, int ne2,
                                                          unsigned char* __restrict__ out, long ldo) {
  // edge table transposed, [ne2][32]: lane fl (feature f0 + fl) reads e[j * 32] of its own column, so
  // the 32 lanes of a ds_read_b32 group always sit in 32 distinct banks whatever their search
  // positions (the [32][ne2 + 1] layout met random bank conflicts from the second step on)
  extern __shared__ float etab[];
  __shared__ unsigned char tile[32][256 + 4];
  const int f0 = blockIdx.y * 32;
  const int t = threadIdx.x;
  for (int i = t; i < 32 * ne2; i += 256) {
    const int fl = i / ne2, j = i - fl * ne2;
    const int f = f0 + fl;
    etab[j * 32 + fl] = (f < n && j < nedges) ? edges[(long)f * nedges + j] : INFINITY;
  }
  __syncthreads();
  const int fl = t & 31;
  const int f = f0 + fl;
  const float* e = etab + fl;
  for (long r0 = (long)blockIdx.x * QROWS; r0 < min(m, (long)(blockIdx.x + 1) * QROWS); r0 += 256) {
    // QU rows per thread at a time: their loads are issued together and their binary searches
    // advance in lockstep (QU independent LDS-read chains instead of one dependent chain)
    constexpr int QU = 8;
    for (int p0 = 0; p0 < 32; p0 += QU) {
      float x[QU];
      int lo[QU];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const long r = r0 + (t >> 5) + 8 * (p0 + u);
        x[u] = (r < m && f < n) ? X[r * ld + f] : 0.f;
        lo[u] = 0;
      }
      for (int step = ne2 >> 1; step > 0; step >>= 1) {
#pragma unroll
        for (int u = 0; u < QU; ++u) lo[u] = (e[(lo[u] + step - 1) * 32] < x[u]) ? lo[u] + step : lo[u];
      }
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int rl = (t >> 5) + 8 * (p0 + u);
        const long r = r0 + rl;
        tile[fl][rl] = (r < m && f < n) ? (unsigned char)lo[u] : (unsigned char)0;
      }
    }
    __syncthreads();
    // 32 features x 256 rows: each thread writes 4 consecutive bytes of one feature row
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int idx = t + 256 * p;  // 0..2047
      const int fl2 = idx >> 6;     // 64 x 4-byte words per feature row
      const int w = idx & 63;
      const int ff = f0 + fl2;
      const long rr = r0 + w * 4;
      if (ff < n) {
        unsigned char* dst = out + (long)ff * ldo + rr;
        if (rr + 3 < m && ((reinterpret_cast<uintptr_t>(dst) & 3) == 0)) {
          *reinterpret_cast<unsigned*>(dst) = *reinterpret_cast<const unsigned*>(&tile[fl2][w * 4]);
        } else {
          for (int q = 0; q < 4; ++q)
            if (rr + q < m) dst[q] = tile[fl2][w * 4 + q];
        }
      }
    }
    __syncthreads();
  }
}

// out: feature-major bins, row stride ldo >= m (a row chunk of a larger matrix: out + chunk start)
SRML_API int srml_rf_quantize_u8_ld(const float* X, long m, int n, long ld, const float* edges, int nedges,
                                    unsigned char* out, long ldo, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  if (nedges < 0 || nedges > 255 || ldo < m) return (int)hipErrorInvalidValue;
  int ne2 = 1;
  while (ne2 < nedges + 1) ne2 <<= 1;
  const size_t lds = (size_t)32 * ne2 * sizeof(float);
  dim3 grid(ceil_div(m, QROWS), ceil_div(n, 32));
  hipLaunchKernelGGL(rf_quantize_kernel, grid, dim3(256), lds, stream, X, m, n, ld, edges, nedges, ne2, out, ldo);
  return srml_status();
}

SRML_API int srml_rf_quantize_u8(const float* X, long m, int n, long ld, const float* edges, int nedges,
                                 unsigned char* out, hipStream_t stream) {
  return srml_rf_quantize_u8_ld(X, m, n, ld, edges, nedges, out, m, stream);
}

// ------------------------------------------------------------------------------------------
// histogram build. items: int4 {node_slot, row_begin, row_end, feature_chunk}
// node_feats: [nodes][nf] global feature ids. wy: (weight, label) per position of idx (compacted
// once per level, so the row stream is two contiguous loads + 8 byte-gathers per row). hist
// layout: [node][nf][B][S] with S = C (class counts, uint32) or 2 (regression weighted count and
// sum, fp32 in LDS folded into the fp64 output). Two rows per thread per step: all 16 bin gathers are
// issued before the first LDS atomic (ILP instead of a load->atomic chain per row).
// ------------------------------------------------------------------------------------------
// 32-byte record layout of the bins ("interleaved"): record (g, r) = the bins of features 32g ..
// 32g + 31 of row r, at byte (g * m + r) * 32 (srml_rf_interleave_u8). A node's feature chunk
// (ascending sampled features) usually falls into one or two groups, so a row costs one or two
// 32-byte loads instead of one scattered byte gather per feature — the deep levels, where a
// node's rows are sparse, stop paying a full cache line per (row, feature).
__device__ __forceinline__ unsigned rec_word(const uint4& lo, const uint4& hi, int q) {
  switch (q) {  // q is wave-uniform: scalar branches, no register indexing
    case 0: return lo.x;
    case 1: return lo.y;
    case 2: return lo.z;
    case 3: return lo.w;
    case 4: return hi.x;
    case 5: return hi.y;
    case 6: return hi.z;
    default: return hi.w;
  }
}

// RM: `bins` is row-major (m x n bytes; the kernel's `m` argument carries the row stride n): a row's
// sampled features sit within its n bytes, so the deep levels' per-row gathers share cache lines
// instead of touching one line per (row, feature) of the feature-major matrix.
template <bool REG, bool FIXED = false, bool IL = false, bool RM = false>
__global__ __launch_bounds__(256) void rf_hist_kernel(const unsigned char* __restrict__ bins, long m,
                                                      const int* __restrict__ idx, const float2* __restrict__ wy,
                                                      const int4* __restrict__ items, const int* __restrict__ node_feats,
                                                      int nf, int B, int S, int fb, double yscale,
                                                      unsigned* __restrict__ hist_u, double* __restrict__ hist_d) {
  // LDS (classification): u32 counts [feature][class][bin].
  // LDS (regression): u32 weighted counts [feature][bin] then i64 fixed-point sums of w*y
  //   [feature][bin]. Integer LDS atomics: ds_add_f32 issues ~50x slower than ds_add_u32 on
  //   gfx950 (SQ_WAIT_INST_LDS), and the 2^-38·max|y| fixed-point step is finer than fp32.
  extern __shared__ __attribute__((aligned(16))) unsigned lh_u[];
  unsigned long long* lh_s = reinterpret_cast<unsigned long long*>(lh_u + ((fb * B + 1) & ~1));  // 8-B aligned
  const int4 it = items[blockIdx.x];
  // item.w = feature chunk | RF_ITEM_EXCLUSIVE: this item is its node's only row chunk, so it owns
  // its histogram cells outright (plain stores of every cell, zeros included; the caller does not
  // pre-zero such nodes) instead of atomics into a zeroed buffer
  const bool excl = (it.w >> 30) & 1;
  const int node = it.x, rb = it.y, re = it.z, fc = it.w & 0x3fffffff;
  const int f_begin = fc * fb;
  const int nfb = min(fb, nf - f_begin);
  const int words = REG ? ((fb * B + 1) & ~1) + 2 * fb * B : fb * B * S;
  for (int i = threadIdx.x; i < words; i += 256) lh_u[i] = 0u;
  const unsigned char* col[FB];
  int grp[FB], byo[FB];
#pragma unroll
  for (int j = 0; j < FB; ++j) {
    const int f = (j < nfb) ? node_feats[(long)node * nf + f_begin + j] : 0;
    col[j] = RM ? bins + f : bins + (long)f * m;
    grp[j] = f >> 5;
    byo[j] = f & 31;
  }
  __syncthreads();
  for (int i = rb + threadIdx.x; i < re; i += 512) {
    const int i2 = i + 256;
    const bool has2 = i2 < re;
    const int r1 = idx[i];
    const int r2 = has2 ? idx[i2] : r1;
    const float2 a1 = wy[i];
    const float2 a2 = has2 ? wy[i2] : make_float2(0.f, 0.f);
    int b1[FB], b2[FB];
    if (IL) {
      uint4 lo1 = make_uint4(0, 0, 0, 0), hi1 = lo1, lo2 = lo1, hi2 = lo1;
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        if (j < nfb) {
          if (j == 0 || grp[j] != grp[j - 1]) {  // sorted features: each record loaded once per row
            const uint4* p1 = reinterpret_cast<const uint4*>(bins + ((long)grp[j] * m + r1) * 32);
            const uint4* p2 = reinterpret_cast<const uint4*>(bins + ((long)grp[j] * m + r2) * 32);
            lo1 = p1[0];
            hi1 = p1[1];
            lo2 = p2[0];
            hi2 = p2[1];
          }
          const int sh = 8 * (byo[j] & 3);
          b1[j] = (rec_word(lo1, hi1, byo[j] >> 2) >> sh) & 0xff;
          b2[j] = (rec_word(lo2, hi2, byo[j] >> 2) >> sh) & 0xff;
        } else {
          b1[j] = b2[j] = 0;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        b1[j] = RM ? col[j][(long)r1 * m] : col[j][r1];
        b2[j] = RM ? col[j][(long)r2 * m] : col[j][r2];
      }
    }
    const unsigned w1 = (unsigned)a1.x, w2 = (unsigned)a2.x;
    unsigned long long s1 = 0ull, s2 = 0ull;
    if (REG) {
      s1 = (unsigned long long)(long long)rint((double)a1.x * (double)a1.y * yscale);
      s2 = (unsigned long long)(long long)rint((double)a2.x * (double)a2.y * yscale);
    }
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      if (j < nfb) {
        if (REG) {
          atomicAdd(&lh_u[j * B + b1[j]], w1);
          atomicAdd(&lh_s[j * B + b1[j]], s1);
          if (w2) {
            atomicAdd(&lh_u[j * B + b2[j]], w2);
            atomicAdd(&lh_s[j * B + b2[j]], s2);
          }
        } else {
          atomicAdd(&lh_u[(j * S + (int)a1.y) * B + b1[j]], w1);
          if (w2) atomicAdd(&lh_u[(j * S + (int)a2.y) * B + b2[j]], w2);
        }
      }
    }
  }
  __syncthreads();
  // fold into the global [node][feature][bin][stat] layout
  const long out_base = ((long)node * nf + f_begin) * B * S;
  const int valid_cells = nfb * B * S;
  const double inv = 1.0 / yscale;
  for (int i = threadIdx.x; i < valid_cells; i += 256) {
    const int j = i / (B * S), rem = i % (B * S), b = rem / S, st = rem % S;
    if (REG && FIXED) {
      // deterministic mode: the cells hold i64 fixed-point integers (two's complement u64
      // atomics add exactly, in any order); srml_rf_hist_fixed_finish converts them to fp64
      const unsigned long long q = st == 0 ? (unsigned long long)lh_u[j * B + b] : lh_s[j * B + b];
      unsigned long long* cell = reinterpret_cast<unsigned long long*>(hist_d) + out_base + i;
      if (excl) *cell = q;
      else if (q) atomicAdd(cell, q);
    } else if (REG) {
      double v;
      if (st == 0) v = (double)lh_u[j * B + b];
      else v = (double)(long long)lh_s[j * B + b] * inv;
      if (excl) hist_d[out_base + i] = v;
      else if (v != 0.0) atomicAdd(&hist_d[out_base + i], v);
    } else {
      const unsigned v = lh_u[(j * S + st) * B + b];
      if (excl) hist_u[out_base + i] = v;
      else if (v) atomicAdd(&hist_u[out_base + i], v);
    }
  }
}

// wy: (weight, label) float pairs aligned with idx
// regression: S must be 2 (weighted count, weighted sum); yscale = fixed-point scale for w*y
// features per work item for a (B, S) histogram: the LDS slab (fb * B * S words) must fit 64 KiB
SRML_API int srml_rf_hist_fb(int B, int S, int regression) {
  const long per = (long)B * (regression ? 3 : S) * (long)sizeof(unsigned);
  long fb = (64 * 1024) / (per > 0 ? per : 1);
  if (fb > FB) fb = FB;
  return (int)(fb < 1 ? (per <= 160 * 1024 ? 1 : 0) : fb);
}

// wy: (weight, label) float pairs aligned with idx; items use feature chunks of `fb` features
// (srml_rf_hist_fb). regression: S must be 2 (weighted count, weighted sum); yscale = fixed-point
// scale for w*y
// il != 0: `bins` is the 32-byte record layout (srml_rf_interleave_u8), else feature-major.
SRML_API int srml_rf_hist(const unsigned char* bins, long m, const int* idx, const float* wy, const int* items,
                          int n_items, const int* node_feats, int nf, int B, int S, int regression, double yscale,
                          int fb, unsigned* hist_u, double* hist_d, int il, hipStream_t stream) {
  if (n_items <= 0) return 0;
  if (regression && S != 2) return -6;
  if (fb < 1 || fb > FB) return -7;
  if (il == 1 && (reinterpret_cast<uintptr_t>(bins) & 15)) return -8;
  const size_t lds = ((size_t)fb * B * (regression ? 3 : S) + 1) * sizeof(unsigned);
  if (lds > 160 * 1024) return -5;
  const float2* w2 = reinterpret_cast<const float2*>(wy);
  const int4* it = reinterpret_cast<const int4*>(items);
#define SRML_RF_HIST(RG, ILV, YS)                                                                                   \
  do {                                                                                                             \
    if (lds > 64 * 1024)                                                                                           \
      (void)hipFuncSetAttribute((const void*)rf_hist_kernel<RG, false, ILV>,                                       \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                             \
    hipLaunchKernelGGL((rf_hist_kernel<RG, false, ILV>), dim3(n_items), dim3(256), lds, stream, bins, m, idx, w2,  \
                       it, node_feats, nf, B, S, fb, YS, hist_u, hist_d);                                          \
  } while (0)
  if (il == 2) {  // row-major bins (m carries the row stride)
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)rf_hist_kernel<false, false, false, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (regression) {
      if (lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void*)rf_hist_kernel<true, false, false, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL((rf_hist_kernel<true, false, false, true>), dim3(n_items), dim3(256), lds, stream, bins, m,
                         idx, w2, it, node_feats, nf, B, S, fb, yscale, hist_u, hist_d);
    } else {
      hipLaunchKernelGGL((rf_hist_kernel<false, false, false, true>), dim3(n_items), dim3(256), lds, stream, bins, m,
                         idx, w2, it, node_feats, nf, B, S, fb, 1.0, hist_u, hist_d);
    }
  } else if (regression) {
    if (il) SRML_RF_HIST(true, true, yscale);
    else SRML_RF_HIST(true, false, yscale);
  } else {
    if (il) SRML_RF_HIST(false, true, 1.0);
    else SRML_RF_HIST(false, false, 1.0);
  }
#undef SRML_RF_HIST
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Wide record-layout histogram for sparse (deep) levels: a block of 1024 threads owns up to fbw
// (~100) of its node's sampled features at once (LDS slab sized to 150 KiB), so each row's
// 32-byte bin records are fetched ONCE per ~100 features instead of once per 8-feature item —
// the row's bytes cross L2 about once per level instead of ~3x (measured: 8-feature record
// items read ~130 GB per 1M x 3000 regression level, L2/MALL-bound at ~65 ms). The feature
// metadata (record group, byte) sits in LDS; the group is made wave-uniform (readfirstlane), so
// the "new record?" test and the byte pick are scalar branches. Same cells, same fold as
// rf_hist_kernel.
// ------------------------------------------------------------------------------------------
constexpr int RHW_T = 1024;

// Byte offset of record (g, r). 32-B records: [g][r]. 64-B records come in line-sized PAIRS: the
// records of groups 2h and 2h + 1 of row r share one 128-B line ([h][r][2][64]), so a row's
// consecutive groups (the wide kernel walks them in order, prefetching the next) hit the line the
// previous load brought in.
template <int RB>
__device__ __forceinline__ long rec_offset(int g, long r, long m) {
  return RB == 64 ? (((long)(g >> 1) * m + r) * 128 + (g & 1) * 64) : (((long)g * m + r) * RB);
}

// byte o (wave-uniform) of a record held as four 16-B pieces: scalar branches pick piece and word
__device__ __forceinline__ int rec_pick(uint4 a, uint4 b, uint4 c, uint4 d, int o) {
  const int t = o >> 4;
  const uint4 piece = t == 0 ? a : t == 1 ? b : t == 2 ? c : d;
  const int wq = (o >> 2) & 3;
  const unsigned word = wq == 0 ? piece.x : wq == 1 ? piece.y : wq == 2 ? piece.z : piece.w;
  return (int)((word >> (8 * (o & 3))) & 0xff);
}

// PACK (regression, non-deterministic): ONE u64 LDS atomic per (row, feature) instead of a u32
// count + u64 sum: cell = (sum w) << 44 | sum w (yq + 2^22), yq = rint(y * yscale) with yscale =
// 2^22 / max|y| (|yq| <= 2^22, so every addend's low field is in [0, w 2^23] and never borrows);
// with sum w <= 2^20 per block (rows per item x max weight, checked by the host) the low field
// stays below 2^43. Count exact; sum quantised to 2^-22 max|y| per row (fp32-level), unpacked at
// the flush. Two LDS words per cell instead of three: ~1.5x the features per block.
constexpr int RF_PACK_SHIFT = 44;
constexpr long long RF_PACK_BIAS = 1LL << 22;

template <bool REG, bool FIXED, int RB, bool PACK = false>
__global__ __launch_bounds__(RHW_T) void rf_hist_wide_kernel(const unsigned char* __restrict__ rec, long m,
                                                              const int* __restrict__ idx,
                                                              const float2* __restrict__ wy,
                                                              const int4* __restrict__ items,
                                                              const int* __restrict__ node_feats, int nf, int B, int S,
                                                              int fbw, double yscale, unsigned* __restrict__ hist_u,
                                                              double* __restrict__ hist_d) {
  extern __shared__ __attribute__((aligned(16))) unsigned hw_u[];
  const int4 it = items[blockIdx.x];
  const bool excl = (it.w >> 30) & 1;
  const int node = it.x, rb = it.y, re = it.z, fc = it.w & 0x3fffffff;
  const int f_begin = fc * fbw;
  const int nfb = min(fbw, nf - f_begin);
  // LDS: [grp | byo] shorts for fbw features, then counts (u32) and, for regression, u64 sums
  short* s_grp = reinterpret_cast<short*>(hw_u);
  short* s_byo = s_grp + fbw;
  unsigned* cnt = hw_u + ((2 * fbw * (int)sizeof(short) + 15) / 16) * 4;
  const int cntw = PACK ? 0 : (fbw * B + 1) & ~1;  // u64 sums stay 8-byte aligned for any B
  unsigned long long* sum = reinterpret_cast<unsigned long long*>(cnt + cntw);
  const int words = PACK ? 2 * fbw * B : REG ? cntw + 2 * fbw * B : fbw * B * S;
  for (int i = threadIdx.x; i < words; i += RHW_T) cnt[i] = 0u;
  for (int j = threadIdx.x; j < fbw; j += RHW_T) {
    const int f = j < nfb ? node_feats[(long)node * nf + f_begin + j] : 0;
    s_grp[j] = (short)(f / RB);
    s_byo[j] = (short)(f % RB);
  }
  __syncthreads();
  // two rows per thread and the next record group prefetched while the current one is binned:
  // four record loads in flight per lane instead of one dependent load per group
  for (int i = rb + threadIdx.x; i < re; i += 2 * RHW_T) {
    const int i2 = i + RHW_T;
    const bool has2 = i2 < re;
    const int r1 = idx[i];
    const int r2 = has2 ? idx[i2] : r1;
    const float2 a1 = wy[i];
    const float2 a2 = has2 ? wy[i2] : make_float2(0.f, 0.f);
    const unsigned w1 = (unsigned)a1.x, w2 = (unsigned)a2.x;
    unsigned long long s1 = 0ull, s2 = 0ull;
    if (PACK) {
      const long long q1 = (long long)rint((double)a1.y * yscale) + RF_PACK_BIAS;
      const long long q2 = (long long)rint((double)a2.y * yscale) + RF_PACK_BIAS;
      s1 = ((unsigned long long)w1 << RF_PACK_SHIFT) + (unsigned long long)w1 * (unsigned long long)q1;
      s2 = ((unsigned long long)w2 << RF_PACK_SHIFT) + (unsigned long long)w2 * (unsigned long long)q2;
    } else if (REG) {
      s1 = (unsigned long long)(long long)rint((double)a1.x * (double)a1.y * yscale);
      s2 = (unsigned long long)(long long)rint((double)a2.x * (double)a2.y * yscale);
    }
    const int c1 = REG ? 0 : (int)a1.y, c2 = REG ? 0 : (int)a2.y;
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    uint4 qa1 = z4, qb1 = z4, qc1 = z4, qd1 = z4, qa2 = z4, qb2 = z4, qc2 = z4, qd2 = z4;
    uint4 na1 = z4, nb1 = z4, nc1 = z4, nd1 = z4, na2 = z4, nb2 = z4, nc2 = z4, nd2 = z4;
#define SRML_REC_LOAD(A, Bq, C, D, G, R)                                                    \
  do {                                                                                     \
    const uint4* p_ = reinterpret_cast<const uint4*>(rec + rec_offset<RB>(G, R, m));         \
    A = p_[0];                                                                             \
    Bq = p_[1];                                                                            \
    if (RB == 64) {                                                                        \
      C = p_[2];                                                                           \
      D = p_[3];                                                                           \
    }                                                                                      \
  } while (0)
    int j = 0;
    int g = __builtin_amdgcn_readfirstlane((int)s_grp[0]);
    SRML_REC_LOAD(qa1, qb1, qc1, qd1, g, r1);
    SRML_REC_LOAD(qa2, qb2, qc2, qd2, g, r2);
    while (j < nfb) {  // one trip per record group of the item's (ascending) features
      int je = j + 1;
      while (je < nfb && __builtin_amdgcn_readfirstlane((int)s_grp[je]) == g) ++je;
      const int gn = je < nfb ? __builtin_amdgcn_readfirstlane((int)s_grp[je]) : g;
      if (je < nfb) {
        SRML_REC_LOAD(na1, nb1, nc1, nd1, gn, r1);
        SRML_REC_LOAD(na2, nb2, nc2, nd2, gn, r2);
      }
      for (int jj = j; jj < je; ++jj) {
        const int o = __builtin_amdgcn_readfirstlane((int)s_byo[jj]);
        const int b1 = rec_pick(qa1, qb1, qc1, qd1, o), b2 = rec_pick(qa2, qb2, qc2, qd2, o);
        if (PACK) {
          atomicAdd(&sum[jj * B + b1], s1);
          if (w2) atomicAdd(&sum[jj * B + b2], s2);
        } else if (REG) {
          atomicAdd(&cnt[jj * B + b1], w1);
          atomicAdd(&sum[jj * B + b1], s1);
          if (w2) {
            atomicAdd(&cnt[jj * B + b2], w2);
            atomicAdd(&sum[jj * B + b2], s2);
          }
        } else {
          atomicAdd(&cnt[(jj * S + c1) * B + b1], w1);
          if (w2) atomicAdd(&cnt[(jj * S + c2) * B + b2], w2);
        }
      }
      if (je < nfb) {
        qa1 = na1; qb1 = nb1; qc1 = nc1; qd1 = nd1;
        qa2 = na2; qb2 = nb2; qc2 = nc2; qd2 = nd2;
      }
      j = je;
      g = gn;
    }
#undef SRML_REC_LOAD
  }
  __syncthreads();
  const long out_base = ((long)node * nf + f_begin) * B * S;
  const int valid_cells = nfb * B * S;
  const double inv = 1.0 / yscale;
  for (int i = threadIdx.x; i < valid_cells; i += RHW_T) {
    const int j = i / (B * S), rem = i % (B * S), b = rem / S, st = rem % S;
    if (PACK) {
      const unsigned long long pk = sum[j * B + b];
      const unsigned long long c = pk >> RF_PACK_SHIFT;
      const long long lo = (long long)(pk & ((1ull << RF_PACK_SHIFT) - 1ull)) - (long long)c * RF_PACK_BIAS;
      const double v = st == 0 ? (double)c : (double)lo * inv;
      if (excl) hist_d[out_base + i] = v;
      else if (v != 0.0) atomicAdd(&hist_d[out_base + i], v);
    } else if (REG && FIXED) {
      const unsigned long long q = st == 0 ? (unsigned long long)cnt[j * B + b] : sum[j * B + b];
      unsigned long long* cell = reinterpret_cast<unsigned long long*>(hist_d) + out_base + i;
      if (excl) *cell = q;
      else if (q) atomicAdd(cell, q);
    } else if (REG) {
      const double v = st == 0 ? (double)cnt[j * B + b] : (double)(long long)sum[j * B + b] * inv;
      if (excl) hist_d[out_base + i] = v;
      else if (v != 0.0) atomicAdd(&hist_d[out_base + i], v);
    } else {
      const unsigned v = cnt[(j * S + st) * B + b];
      if (excl) hist_u[out_base + i] = v;
      else if (v) atomicAdd(&hist_u[out_base + i], v);
    }
  }
}

// Features per item of the wide kernel for (B, S): the LDS slab (metadata + fbw * B * S' words)
// within 150 KiB (S' = 3 for regression: count + 64-bit fixed-point sum).
SRML_API int srml_rf_hist_wide_fb(int B, int S, int regression) {
  // regression > 1: the packed single-u64 cells (2 words per (feature, bin))
  const long per = (long)B * (regression > 1 ? 2 : regression ? 3 : S) * (long)sizeof(unsigned) +
                   2 * (long)sizeof(short);
  const long fbw = (150L * 1024 - 64) / (per > 0 ? per : 1);
  return (int)(fbw > 512 ? 512 : fbw);
}

// items: {node, row_begin, row_end, feature chunk (of fbw features) | exclusive << 30} on the
// record layout `rec` (srml_rf_interleave_u8). fixed: deterministic i64 cells (regression).
SRML_API int srml_rf_hist_wide(const unsigned char* rec, long m, const int* idx, const float* wy, const int* items,
                               int n_items, const int* node_feats, int nf, int B, int S, int regression, double yscale,
                               int fbw, int fixed, int rb, unsigned* hist_u, double* hist_d, hipStream_t stream) {
  // fixed: 1 = deterministic i64 cells, 2 = packed count/sum cells (yscale = 2^22 / max|y|; the
  // caller guarantees sum w <= 2^20 per item)
  if (n_items <= 0) return 0;
  if (regression && S != 2) return -6;
  if (fbw < 1 || (reinterpret_cast<uintptr_t>(rec) & 15)) return -7;
  if (rb != 32 && rb != 64) return -2;
  if (fixed == 2 && !regression) return -2;
  const size_t lds = (size_t)((2 * fbw * sizeof(short) + 15) / 16) * 16 +
                     ((size_t)fbw * B * (fixed == 2 ? 2 : regression ? 3 : S) + 1) * sizeof(unsigned);
  if (lds > 160 * 1024) return -5;
  const float2* w2 = reinterpret_cast<const float2*>(wy);
  const int4* it = reinterpret_cast<const int4*>(items);
#define SRML_RF_HW(RG, FX, RBB, PK, YS)                                                                        \
  do {                                                                                                        \
    (void)hipFuncSetAttribute((const void*)rf_hist_wide_kernel<RG, FX, RBB, PK>,                              \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                          \
    hipLaunchKernelGGL((rf_hist_wide_kernel<RG, FX, RBB, PK>), dim3(n_items), dim3(RHW_T), lds, stream, rec, m, \
                       idx, w2, it, node_feats, nf, B, S, fbw, YS, hist_u, hist_d);                           \
  } while (0)
#define SRML_RF_HW_RB(RBB)                                                \
  do {                                                                    \
    if (regression && fixed == 2) SRML_RF_HW(true, false, RBB, true, yscale); \
    else if (regression && fixed) SRML_RF_HW(true, true, RBB, false, yscale); \
    else if (regression) SRML_RF_HW(true, false, RBB, false, yscale);     \
    else SRML_RF_HW(false, false, RBB, false, 1.0);                       \
  } while (0)
  if (rb == 64) SRML_RF_HW_RB(64);
  else SRML_RF_HW_RB(32);
#undef SRML_RF_HW_RB
#undef SRML_RF_HW
  return srml_status();
}

// 32-byte record layout of a feature-major (n x m) uint8 bin matrix: out[(g * m + r) * 32 + j] =
// bins[(32 g + j) * m + r] (features past n are 0). One thread per row and group: 32 coalesced
// byte reads across the rows, two 16-B stores.
template <int RB>
__global__ __launch_bounds__(256) void rf_interleave_kernel(const unsigned char* __restrict__ bins, long m, int n,
                                                            unsigned char* __restrict__ out) {
  const long r = (long)blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y;
  if (r >= m) return;
  unsigned w[RB / 4];
#pragma unroll
  for (int q = 0; q < RB / 4; ++q) {
    unsigned v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = RB * g + 4 * q + b;
      if (f < n) v |= (unsigned)bins[(long)f * m + r] << (8 * b);
    }
    w[q] = v;
  }
  uint4* dst = reinterpret_cast<uint4*>(out + rec_offset<RB>(g, r, m));
#pragma unroll
  for (int q = 0; q < RB / 16; ++q) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// Four rows per thread (m % 4 == 0): one dword load per feature brings the feature's bins of rows
// r .. r + 3, a byte transpose in registers forms the four rows' records — a quarter of the load
// instructions of one byte load per (row, feature)
template <int RB>
__global__ __launch_bounds__(256) void rf_interleave4_kernel(const unsigned char* __restrict__ bins, long m, int n,
                                                             unsigned char* __restrict__ out) {
  const long r = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  const int g = blockIdx.y;
  if (r >= m) return;
  unsigned w[4][RB / 4];
#pragma unroll
  for (int q = 0; q < RB / 4; ++q) {
    unsigned v[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = RB * g + 4 * q + b;
      v[b] = f < n ? *reinterpret_cast<const unsigned*>(bins + (long)f * m + r) : 0u;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)  // row r + i: byte i of each feature's dword
      w[i][q] = ((v[0] >> (8 * i)) & 0xffu) | (((v[1] >> (8 * i)) & 0xffu) << 8) |
                (((v[2] >> (8 * i)) & 0xffu) << 16) | (((v[3] >> (8 * i)) & 0xffu) << 24);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint4* dst = reinterpret_cast<uint4*>(out + rec_offset<RB>(g, r + i, m));
#pragma unroll
    for (int q = 0; q < RB / 16; ++q)
      dst[q] = make_uint4(w[i][4 * q], w[i][4 * q + 1], w[i][4 * q + 2], w[i][4 * q + 3]);
  }
}

// Row-major copy of the feature-major (n x m) bin matrix: out[r * n + f] = bins[f * m + r] (the
// deep levels' gathers, rf_hist RM / rf_node_split). 64-row x 64-feature byte tiles through LDS:
// 16-B loads along each feature's rows, 8-B stores along each row's features (byte accesses at
// the edges / unaligned shapes): one pass over the matrix each way (torch's strided uint8 copy of
// the transpose took ~16 ms at 1M x 3000).
__global__ __launch_bounds__(256) void rf_transpose_u8_kernel(const unsigned char* __restrict__ in, long m, int n,
                                                              unsigned char* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned char tile[64][68];
  const long r0 = (long)blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  const int t = threadIdx.x;
  {
    const int fl = t >> 2, rc = (t & 3) * 16;
    const int f = f0 + fl;
    const long r = r0 + rc;
    unsigned w[4] = {0u, 0u, 0u, 0u};
    if (f < n) {
      const unsigned char* src = in + (long)f * m + r;
      if (r + 16 <= m && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const uint4 v = *reinterpret_cast<const uint4*>(src);
        w[0] = v.x;
        w[1] = v.y;
        w[2] = v.z;
        w[3] = v.w;
      } else {
        for (int k = 0; k < 16; ++k)
          if (r + k < m) w[k >> 2] |= (unsigned)src[k] << (8 * (k & 3));
      }
    }
    unsigned* d = reinterpret_cast<unsigned*>(&tile[fl][rc]);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = w[q];
  }
  __syncthreads();
  const int rl = t >> 2, fc = (t & 3) * 16;
  const long r = r0 + rl;
  if (r >= m) return;
  unsigned w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    w[q] = (unsigned)tile[fc + 4 * q][rl] | ((unsigned)tile[fc + 4 * q + 1][rl] << 8) |
           ((unsigned)tile[fc + 4 * q + 2][rl] << 16) | ((unsigned)tile[fc + 4 * q + 3][rl] << 24);
  unsigned char* dst = out + r * n + f0 + fc;
  if (f0 + fc + 16 <= n && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
    reinterpret_cast<uint2*>(dst)[0] = make_uint2(w[0], w[1]);
    reinterpret_cast<uint2*>(dst)[1] = make_uint2(w[2], w[3]);
  } else {
    for (int k = 0; k < 16; ++k)
      if (f0 + fc + k < n) dst[k] = (unsigned char)(w[k >> 2] >> (8 * (k & 3)));
  }
}

SRML_API int srml_rf_transpose_u8(const unsigned char* bins, long m, int n, unsigned char* out, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  const long gy = (n + 63) / 64;
  if (gy > 65535) return -2;
  hipLaunchKernelGGL(rf_transpose_u8_kernel, dim3((unsigned)((m + 63) / 64), (unsigned)gy), dim3(256), 0, stream, bins,
                     m, n, out);
  return srml_status();
}

// rb = record bytes (features per record): 32 (the 8-feature item kernel's layout) or 64
SRML_API int srml_rf_interleave_u8(const unsigned char* bins, long m, int n, int rb, unsigned char* out,
                                   hipStream_t stream) {
  if (m <= 0 || n <= 0) return 0;
  if (reinterpret_cast<uintptr_t>(out) & 15) return -8;
  if (rb != 32 && rb != 64) return -2;
  const int G = (n + rb - 1) / rb;
  if (G > 65535) return -2;
  if ((m & 3) == 0 && (reinterpret_cast<uintptr_t>(bins) & 3) == 0) {
    const dim3 grid4((unsigned)((m / 4 + 255) / 256), (unsigned)G);
    if (rb == 32) hipLaunchKernelGGL(rf_interleave4_kernel<32>, grid4, dim3(256), 0, stream, bins, m, n, out);
    else hipLaunchKernelGGL(rf_interleave4_kernel<64>, grid4, dim3(256), 0, stream, bins, m, n, out);
    return srml_status();
  }
  const dim3 grid((unsigned)((m + 255) / 256), (unsigned)G);
  if (rb == 32) hipLaunchKernelGGL(rf_interleave_kernel<32>, grid, dim3(256), 0, stream, bins, m, n, out);
  else hipLaunchKernelGGL(rf_interleave_kernel<64>, grid, dim3(256), 0, stream, bins, m, n, out);
  return srml_status();
}

SRML_API int srml_rf_hist_fb_max() { return FB; }

// Deterministic regression histograms (SRML_DETERMINISTIC): same work items as srml_rf_hist, but
// the cross-chunk fold adds exact i64 fixed-point integers (order-independent) into the fp64
// buffer's bits; srml_rf_hist_fixed_finish then converts every cell in place (count -> double,
// sum -> integer / yscale). Bit-identical results for any block scheduling.
SRML_API int srml_rf_hist_fixed(const unsigned char* bins, long m, const int* idx, const float* wy, const int* items,
                                int n_items, const int* node_feats, int nf, int B, double yscale, int fb,
                                double* hist_d, int il, hipStream_t stream) {
  if (n_items <= 0) return 0;
  if (fb < 1 || fb > FB) return -7;
  if (il == 1 && (reinterpret_cast<uintptr_t>(bins) & 15)) return -8;
  const size_t lds = ((size_t)fb * B * 3 + 1) * sizeof(unsigned);
  if (lds > 160 * 1024) return -5;
  const float2* w2 = reinterpret_cast<const float2*>(wy);
  const int4* it = reinterpret_cast<const int4*>(items);
  if (il) {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)rf_hist_kernel<true, true, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((rf_hist_kernel<true, true, true>), dim3(n_items), dim3(256), lds, stream, bins, m, idx, w2, it,
                       node_feats, nf, B, 2, fb, yscale, nullptr, hist_d);
  } else {
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)rf_hist_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
    hipLaunchKernelGGL((rf_hist_kernel<true, true>), dim3(n_items), dim3(256), lds, stream, bins, m, idx, w2, it,
                       node_feats, nf, B, 2, fb, yscale, nullptr, hist_d);
  }
  return srml_status();
}

__global__ __launch_bounds__(256) void rf_hist_fixed_finish_kernel(double* __restrict__ hist, long pairs, double inv) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= pairs) return;
  const long long* q = reinterpret_cast<const long long*>(hist) + 2 * i;
  const long long c = q[0], s = q[1];
  hist[2 * i] = (double)c;
  hist[2 * i + 1] = (double)s * inv;
}

SRML_API int srml_rf_hist_fixed_finish(double* hist_d, long cells, double yscale, hipStream_t stream) {
  const long pairs = cells / 2;
  if (pairs <= 0) return 0;
  hipLaunchKernelGGL(rf_hist_fixed_finish_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, stream, hist_d,
                     pairs, 1.0 / yscale);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// split search. crit: 0 gini, 1 entropy, 2 variance.  out per node (double[6]):
//   {gain, feature_slot, bin, n_left, n_right, parent_impurity}
// totals per node (double[S]): class counts or (count, sum); the regression gain is the exact
// variance reduction computed from (count, sum) alone, parent impurity is reported as 0 then
// ------------------------------------------------------------------------------------------
template <int SMAX>
__device__ __forceinline__ double impurity(const double* s, int S, int crit, double n) {
  if (n <= 0.0) return 0.0;
  if (crit == 2) {
    const double mean = s[1] / n;
    const double v = s[2] / n - mean * mean;
    return v > 0.0 ? v : 0.0;
  }
  double acc = 0.0;
  if (crit == 0) {
#pragma unroll
    for (int c = 0; c < SMAX; ++c)
      if (c < S) { const double p = s[c] / n; acc += p * p; }
    return 1.0 - acc;
  }
#pragma unroll
  for (int c = 0; c < SMAX; ++c)
    if (c < S && s[c] > 0.0) { const double p = s[c] / n; acc -= p * log2(p); }
  return acc;
}

// classification gain of one threshold (shared by the split kernels, so they agree bit for bit)
template <int SMAX>
__device__ __forceinline__ double class_split_gain(const double* left, const double* tot, int S, int crit, double nl,
                                                   double nr, double ntot, double pimp) {
  double right[SMAX];
#pragma unroll
  for (int c = 0; c < SMAX; ++c) right[c] = tot[c] - left[c];
  return pimp - (nl / ntot) * impurity<SMAX>(left, S, crit, nl) - (nr / ntot) * impurity<SMAX>(right, S, crit, nr);
}

template <int SMAX, bool REG>
__global__ __launch_bounds__(256) void rf_best_split_kernel(const unsigned* __restrict__ hist_u,
                                                            const double* __restrict__ hist_d, int nf, int B, int S,
                                                            int crit, double min_leaf, double min_gain,
                                                            double* __restrict__ out, double* __restrict__ totals) {
  __shared__ double s_gain[256];
  __shared__ int s_key[256];
  __shared__ double s_tot[SMAX];
  const int node = blockIdx.x;
  const long nbase = (long)node * nf * B * S;
  // node totals from feature slot 0 (every feature's histogram sums to the node totals)
  if (threadIdx.x < S) {
    double acc = 0.0;
    for (int b = 0; b < B; ++b) {
      const long i = nbase + (long)b * S + threadIdx.x;
      acc += REG ? hist_d[i] : (double)hist_u[i];
    }
    s_tot[threadIdx.x] = acc;
  }
  __syncthreads();
  double tot[SMAX];
#pragma unroll
  for (int c = 0; c < SMAX; ++c) tot[c] = c < S ? s_tot[c] : 0.0;
  double ntot = 0.0;
  if (REG) {
    ntot = tot[0];
  } else {
#pragma unroll
    for (int c = 0; c < SMAX; ++c) ntot += tot[c];
  }
  const double pimp = (REG && S < 3) ? 0.0 : impurity<SMAX>(tot, S, crit, ntot);
  double best = -1.0;
  int bkey = 0x7fffffff;
  for (int f = threadIdx.x; f < nf; f += 256) {
    double left[SMAX];
#pragma unroll
    for (int c = 0; c < SMAX; ++c) left[c] = 0.0;
    const long fbase = nbase + (long)f * B * S;
    for (int b = 0; b < B - 1; ++b) {
      double nl = 0.0;
#pragma unroll
      for (int c = 0; c < SMAX; ++c) {
        if (c < S) {
          const long i = fbase + (long)b * S + c;
          left[c] += REG ? hist_d[i] : (double)hist_u[i];
        }
      }
      if (REG) {
        nl = left[0];
      } else {
#pragma unroll
        for (int c = 0; c < SMAX; ++c) nl += left[c];
      }
      const double nr = ntot - nl;
      if (nl < min_leaf || nr < min_leaf || nl <= 0.0 || nr <= 0.0) continue;
      double gain;
      if (REG) {
        // variance reduction = (s_L^2/n_L + s_R^2/n_R - s^2/n) / n  (the sums of squares cancel)
        const double sl = left[1], sr = tot[1] - left[1];
        gain = (sl * sl / nl + sr * sr / nr - tot[1] * tot[1] / ntot) / ntot;
      } else {
        gain = class_split_gain<SMAX>(left, tot, S, crit, nl, nr, ntot, pimp);
      }
      const int key = f * 1024 + b;
      if (gain > best || (gain == best && key < bkey)) { best = gain; bkey = key; }
    }
  }
  s_gain[threadIdx.x] = best;
  s_key[threadIdx.x] = bkey;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const double og = s_gain[threadIdx.x + o];
      const int ok = s_key[threadIdx.x + o];
      if (og > s_gain[threadIdx.x] || (og == s_gain[threadIdx.x] && ok < s_key[threadIdx.x])) {
        s_gain[threadIdx.x] = og;
        s_key[threadIdx.x] = ok;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double g = s_gain[0];
    const int key = s_key[0];
    double* o = out + (long)node * 6;
    const bool ok = (g > min_gain || (g >= 0.0 && min_gain < 0.0)) && key != 0x7fffffff && g > 1e-15;
    o[0] = ok ? g : -1.0;
    o[1] = ok ? (double)(key / 1024) : -1.0;
    o[2] = ok ? (double)(key % 1024) : -1.0;
    o[3] = 0.0;
    o[4] = 0.0;
    o[5] = pimp;
    if (ok) {  // left/right weighted counts of the winner
      const int f = key / 1024, bb = key % 1024;
      double nl = 0.0;
      for (int b = 0; b <= bb; ++b) {
        if (REG) {
          nl += hist_d[nbase + ((long)f * B + b) * S];
        } else {
          for (int c = 0; c < S; ++c) nl += (double)hist_u[nbase + ((long)f * B + b) * S + c];
        }
      }
      o[3] = nl;
      o[4] = ntot - nl;
    }
  }
  if (threadIdx.x < S) totals[(long)node * S + threadIdx.x] = s_tot[threadIdx.x];
}

SRML_API int srml_rf_best_split(const unsigned* hist_u, const double* hist_d, int nodes, int nf, int B, int S,
                                int regression, int crit, double min_leaf, double min_gain, double* out,
                                double* totals, hipStream_t stream) {
  if (nodes <= 0) return 0;
#define SRML_RF_SPLIT(SM)                                                                                          \
  do {                                                                                                             \
    if (regression)                                                                                                \
      hipLaunchKernelGGL((rf_best_split_kernel<SM, true>), dim3(nodes), dim3(256), 0, stream, hist_u, hist_d, nf, B, \
                         S, crit, min_leaf, min_gain, out, totals);                                               \
    else                                                                                                           \
      hipLaunchKernelGGL((rf_best_split_kernel<SM, false>), dim3(nodes), dim3(256), 0, stream, hist_u, hist_d, nf, \
                         B, S, crit, min_leaf, min_gain, out, totals);                                            \
  } while (0)
  if (S <= 2) SRML_RF_SPLIT(2);
  else if (S <= 4) SRML_RF_SPLIT(4);
  else if (S <= 8) SRML_RF_SPLIT(8);
  else if (S <= 16) SRML_RF_SPLIT(16);
  else if (S <= 32) SRML_RF_SPLIT(32);
  else return -6;
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Fused histogram + split search for small classification nodes (the deep levels). One 512-thread
// block per node keeps the node's whole histogram ([feature slot][class][bin] u32 weighted counts
// of every sampled feature) in LDS, so nothing goes to HBM between the two phases: the unfused
// level writes nf * B * S cells per node, re-reads them in rf_best_split_kernel and once more
// (cumsum + gather) for the left-child totals, and at the deep levels it launches one 256-thread
// block per 8-feature chunk of a ~200-row node. Rows are gathered from the ROW-MAJOR bin copy: a
// row gets the next power of two >= nf lanes (64 / that rows per wave instruction, NS_U
// instructions in flight) and its lanes fetch the row's sampled features — ascending ids, so one
// row's gathers share cache lines (a 64-feature row is one line) — and add the row's weight into
// their own feature's cells. The split search gives each feature to a wave with the bins spread over the lanes
// (a run of consecutive bins per lane, exclusive wave scan of the class counts) instead of one
// thread per feature. Counts are integers below 2^32 per node, so every left / right total is
// exact and the gains (class_split_gain), the winner (highest gain, then lowest feature slot, then
// lowest bin) and the record equal rf_best_split_kernel's on the same histogram. Outputs per node:
// the rf_best_split record {gain, slot, bin, n_left, n_right, impurity} and the winner's
// left-child class totals (zeros without a split). Reference: tree.py:309-414 (cuML's level-wise
// split search).
// ------------------------------------------------------------------------------------------
constexpr int NS_T = 512;
constexpr int NS_W = NS_T / 64;
constexpr int NS_FL = 4;  // sampled features per lane: nf <= 256
constexpr int NS_U = 4;   // rows in flight per wave

__device__ __forceinline__ unsigned wave_excl_scan_u32(unsigned v, int lane) {
  unsigned x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x - v;
}

__device__ __forceinline__ unsigned wave_sum_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ bool split_better(double g, int k, double bg, int bk) {
  return g > bg || (g == bg && k < bk);
}

template <int SMAX, bool MULTI>
__global__ __launch_bounds__(NS_T) void rf_node_split_kernel(const unsigned char* __restrict__ bins_rm, long ldr,
                                                             const int* __restrict__ idx,
                                                             const float2* __restrict__ wy,
                                                             const int* __restrict__ se,
                                                             const int* __restrict__ node_feats, int nf, int B, int S,
                                                             int crit, double min_leaf, double min_gain,
                                                             double* __restrict__ out, double* __restrict__ left_out,
                                                             int lpr_log2) {
  extern __shared__ __attribute__((aligned(16))) unsigned lh[];  // [nf][S][B]
  __shared__ double s_gain[NS_W];
  __shared__ int s_key[NS_W];
  __shared__ double s_tot[SMAX];
  const int node = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cells = nf * S * B;
  for (int i = threadIdx.x; i < cells; i += NS_T) lh[i] = 0u;
  // lanes per row: the next power of two >= nf (<= 64); a wave instruction covers 64 / LPR rows,
  // lane (sub, fl) = row sub, features fl, fl + LPR, ... (several per lane only when nf > 64)
  // (!MULTI: one row per wave instruction, the row id / weight / class stay wave-uniform)
  const int lg = MULTI ? lpr_log2 : 6;
  const int LPR = 1 << lg, RPW = 64 >> lg;
  const int sub = MULTI ? lane >> lg : 0, fl = MULTI ? (lane & (LPR - 1)) : lane;
  long foff[NS_FL];
#pragma unroll
  for (int q = 0; q < NS_FL; ++q) {
    const int j = fl + LPR * q;
    foff[q] = j < nf ? (long)node_feats[(long)node * nf + j] : 0;
  }
  __syncthreads();
  const int rb = se[2 * node], re = se[2 * node + 1];
  for (int i0 = rb + wave * NS_U * RPW; i0 < re; i0 += NS_W * NS_U * RPW) {
    int r[NS_U], c[NS_U];
    unsigned w[NS_U];
#pragma unroll
    for (int u = 0; u < NS_U; ++u) {
      const int i = i0 + u * RPW + sub;
      const bool v = i < re;
      r[u] = v ? idx[i] : 0;
      const float2 a = v ? wy[i] : make_float2(0.f, 0.f);
      w[u] = (unsigned)a.x;
      c[u] = (int)a.y;
    }
    int bv[NS_U][NS_FL];
#pragma unroll
    for (int u = 0; u < NS_U; ++u)
#pragma unroll
      for (int q = 0; q < NS_FL; ++q)
        bv[u][q] = (fl + LPR * q < nf && w[u]) ? (int)bins_rm[(long)r[u] * ldr + foff[q]] : 0;
#pragma unroll
    for (int u = 0; u < NS_U; ++u)
#pragma unroll
      for (int q = 0; q < NS_FL; ++q) {
        const int j = fl + LPR * q;
        if (j < nf && w[u]) atomicAdd(&lh[(j * S + c[u]) * B + bv[u][q]], w[u]);
      }
  }
  __syncthreads();
  // node totals from feature slot 0 (every slot's histogram sums to them)
  if (wave == 0) {
    for (int cc = 0; cc < S; ++cc) {
      unsigned v = 0;
      for (int b = lane; b < B; b += 64) v += lh[cc * B + b];
      v = wave_sum_u32(v);
      if (lane == 0) s_tot[cc] = (double)v;
    }
  }
  __syncthreads();
  double tot[SMAX];
#pragma unroll
  for (int cc = 0; cc < SMAX; ++cc) tot[cc] = cc < S ? s_tot[cc] : 0.0;
  double ntot = 0.0;
#pragma unroll
  for (int cc = 0; cc < SMAX; ++cc) ntot += tot[cc];
  const double pimp = impurity<SMAX>(tot, S, crit, ntot);
  double best = -1.0;
  int bkey = 0x7fffffff;
  const int bpl = (B + 63) >> 6;
  const int b0 = lane * bpl;
  for (int f = wave; f < nf; f += NS_W) {
    const unsigned* hf = lh + f * S * B;
    unsigned pre[SMAX];
#pragma unroll
    for (int cc = 0; cc < SMAX; ++cc) {
      pre[cc] = 0u;
      if (cc < S) {  // wave-uniform
        unsigned own = 0;
        for (int k = 0; k < bpl; ++k)
          if (b0 + k < B) own += hf[cc * B + b0 + k];
        pre[cc] = wave_excl_scan_u32(own, lane);
      }
    }
    for (int k = 0; k < bpl; ++k) {
      const int b = b0 + k;
      if (b >= B - 1) break;
      double left[SMAX];
      double nl = 0.0;
#pragma unroll
      for (int cc = 0; cc < SMAX; ++cc) {
        if (cc < S) pre[cc] += hf[cc * B + b];
        left[cc] = cc < S ? (double)pre[cc] : 0.0;
      }
#pragma unroll
      for (int cc = 0; cc < SMAX; ++cc) nl += left[cc];
      const double nr = ntot - nl;
      if (nl < min_leaf || nr < min_leaf || nl <= 0.0 || nr <= 0.0) continue;
      const double gain = class_split_gain<SMAX>(left, tot, S, crit, nl, nr, ntot, pimp);
      const int key = f * 1024 + b;
      if (split_better(gain, key, best, bkey)) {
        best = gain;
        bkey = key;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(best, o, 64);
    const int ok = __shfl_xor(bkey, o, 64);
    if (split_better(og, ok, best, bkey)) {
      best = og;
      bkey = ok;
    }
  }
  if (lane == 0) {
    s_gain[wave] = best;
    s_key[wave] = bkey;
  }
  __syncthreads();
  if (wave != 0) return;
  double g = s_gain[0];
  int key = s_key[0];
  for (int k = 1; k < NS_W; ++k)
    if (split_better(s_gain[k], s_key[k], g, key)) {
      g = s_gain[k];
      key = s_key[k];
    }
  const bool ok = (g > min_gain || (g >= 0.0 && min_gain < 0.0)) && key != 0x7fffffff && g > 1e-15;
  const int f = ok ? key / 1024 : 0, bb = ok ? key % 1024 : -1;
  double nl = 0.0;
  for (int cc = 0; cc < S; ++cc) {
    unsigned v = 0;
    for (int b = lane; b <= bb; b += 64) v += lh[(f * S + cc) * B + b];
    v = wave_sum_u32(v);
    if (lane == 0) left_out[(long)node * S + cc] = (double)v;
    nl += (double)v;
  }
  if (lane == 0) {
    double* o = out + (long)node * 6;
    o[0] = ok ? g : -1.0;
    o[1] = ok ? (double)f : -1.0;
    o[2] = ok ? (double)bb : -1.0;
    o[3] = nl;
    o[4] = ok ? ntot - nl : 0.0;
    o[5] = pimp;
  }
}

// whether srml_rf_node_split takes (nf sampled features, B bins, S classes)
SRML_API int srml_rf_node_split_ok(int nf, int B, int S) {
  return nf >= 1 && nf <= 64 * NS_FL && S >= 1 && S <= 8 && B >= 2 && B <= 1024 &&
         (long)nf * S * B * (long)sizeof(unsigned) <= 150 * 1024;
}

// bins_rm: row-major uint8 bins (row r at bins_rm + r * ldr); idx / wy: the level's positions
// (row id, (weight, class)); se: (nodes, 2) int32 [begin, end) positions of each node; node_feats:
// (nodes, nf) ascending sampled feature ids. out: (nodes, 6) fp64, left: (nodes, S) fp64.
SRML_API int srml_rf_node_split(const unsigned char* bins_rm, long ldr, const int* idx, const float* wy, const int* se,
                                int nodes, const int* node_feats, int nf, int B, int S, int crit, double min_leaf,
                                double min_gain, double* out, double* left, hipStream_t stream) {
  if (nodes <= 0) return 0;
  if (!srml_rf_node_split_ok(nf, B, S)) return -6;
  const size_t lds = (size_t)nf * S * B * sizeof(unsigned);
  const float2* w2 = reinterpret_cast<const float2*>(wy);
  int lpr = 0;
  while ((1 << lpr) < nf && lpr < 6) ++lpr;
#define SRML_RF_NODE_SPLIT_L(SM, MU)                                                                               \
  do {                                                                                                             \
    if (lds > 64 * 1024)                                                                                           \
      (void)hipFuncSetAttribute((const void*)rf_node_split_kernel<SM, MU>,                                         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                             \
    hipLaunchKernelGGL((rf_node_split_kernel<SM, MU>), dim3(nodes), dim3(NS_T), lds, stream, bins_rm, ldr, idx, w2, \
                       se, node_feats, nf, B, S, crit, min_leaf, min_gain, out, left, lpr);                        \
  } while (0)
#define SRML_RF_NODE_SPLIT(SM)                      \
  do {                                              \
    if (lpr < 6) SRML_RF_NODE_SPLIT_L(SM, true);    \
    else SRML_RF_NODE_SPLIT_L(SM, false);           \
  } while (0)
  if (S <= 2) SRML_RF_NODE_SPLIT(2);
  else if (S <= 4) SRML_RF_NODE_SPLIT(4);
  else SRML_RF_NODE_SPLIT(8);
#undef SRML_RF_NODE_SPLIT_L
#undef SRML_RF_NODE_SPLIT
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// routing: key[i] = 2*child_base[node]+right for split nodes, INT_MAX for rows leaving the tree.
// seg_node: node slot of each position i (int32), node_feature/node_bin: split per node (-1: leaf)
// ------------------------------------------------------------------------------------------
__global__ void rf_route_kernel(const unsigned char* __restrict__ bins, long m, const int* __restrict__ idx,
                                const int* __restrict__ seg_node, long total, const int* __restrict__ node_feature,
                                const int* __restrict__ node_bin, const int* __restrict__ child_base,
                                int* __restrict__ keys) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int node = seg_node[i];
  const int f = node_feature[node];
  if (f < 0) {
    keys[i] = 0x7fffffff;
    return;
  }
  const int r = idx[i];
  const int right = bins[(long)f * m + r] > node_bin[node] ? 1 : 0;
  keys[i] = child_base[node] + right;
}

SRML_API int srml_rf_route(const unsigned char* bins, long m, const int* idx, const int* seg_node, long total,
                           const int* node_feature, const int* node_bin, const int* child_base, int* keys,
                           hipStream_t stream) {
  if (total <= 0) return 0;
  hipLaunchKernelGGL(rf_route_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, bins, m, idx,
                     seg_node, total, node_feature, node_bin, child_base, keys);
  return srml_status();
}

// segment-bounds variant: the segment of position i is found by binary search over the sorted
// bounds (no per-position segment-id array to materialise each level)
__global__ void rf_route_segments_kernel(const unsigned char* __restrict__ bins, long m, const int* __restrict__ idx,
                                         long total, const long long* __restrict__ bounds, int nseg,
                                         const int* __restrict__ node_feature, const int* __restrict__ node_bin,
                                         const int* __restrict__ child_base, int* __restrict__ keys) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int lo = 0, hi = nseg - 1;  // largest s with bounds[s] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bounds[mid] <= i) lo = mid; else hi = mid - 1;
  }
  const int node = lo;
  const int f = node_feature[node];
  if (f < 0) {
    keys[i] = 0x7fffffff;
    return;
  }
  const int r = idx[i];
  keys[i] = child_base[node] + (bins[(long)f * m + r] > node_bin[node] ? 1 : 0);
}

SRML_API int srml_rf_route_segments(const unsigned char* bins, long m, const int* idx, long total,
                                    const long long* bounds, int nseg, const int* node_feature, const int* node_bin,
                                    const int* child_base, int* keys, hipStream_t stream) {
  if (total <= 0 || nseg <= 0) return 0;
  hipLaunchKernelGGL(rf_route_segments_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, bins, m,
                     idx, total, bounds, nseg, node_feature, node_bin, child_base, keys);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Per-node feature subsets (featureSubsetStrategy): node c draws nf of n features uniformly without
// replacement by selection sampling (Knuth's Algorithm S: feature f is taken with probability
// needed / (n - f)), which emits them in ascending order — the order the histogram items want —
// with no sort. Counter-based randomness (splitmix64 of seed, node, feature): reproducible, the
// same on every rank of a data-parallel fit.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// One wave per node, 64 features per step: the lanes draw their uniforms in parallel and turn the
// test u (n - f) < need into an integer threshold t = floor(u (n - f)) + 1 (need > x <=> need >= t
// for integer need), then one scalar pass over the 64 thresholds resolves the sequential `need`
// chain and the accepted lanes store their features at their prefix-count slots. Bit-identical to
// the one-thread-per-node scan it replaced (3000 dependent draws per node: ~0.4 ms per level).
__global__ __launch_bounds__(256) void rf_sample_features_kernel(int C, int n, int nf, unsigned long long seed,
                                                                 int* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;  // wave-uniform
  const unsigned long long base = mix64(seed ^ mix64((unsigned long long)c + 1));
  int need = nf;
  int* o = out + (long)c * nf;
  for (int f0 = 0; f0 < n && need > 0; f0 += 64) {
    const int f = f0 + lane;
    int t = 0x7fffffff;  // past n: never taken
    if (f < n) {
      const double u = (double)(mix64(base + (unsigned long long)f) >> 11) * 0x1.0p-53;
      t = (int)floor(u * (double)(n - f)) + 1;
    }
    unsigned long long take = 0;
    int k = need;
    for (int j = 0; j < 64; ++j) {
      const int tj = __builtin_amdgcn_readlane(t, j);
      if (k > 0 && k >= tj) {
        take |= 1ull << j;
        --k;
      }
    }
    if ((take >> lane) & 1ull) o[nf - need + __popcll(take & ((1ull << lane) - 1ull))] = f;
    need = k;
  }
}

// Sparse subsets (nf <= n / 8, n <= 16384): Floyd's algorithm, O(nf) draws per node
// instead of Algorithm S's O(n) scan (at sqrt(3000) = 55 of 3000 features the scan cost ~9400
// VALU instructions per node: 0.87 ms per deep level of 100k nodes). One wave per node; the
// node's n-bit membership bitmap lives in registers, 64-bit word w = q * 64 + lane in register q
// of lane `lane` (W registers cover 4096 W features). Draw i (j = n - nf + i): t = floor(u_i (j + 1))
// with u_i = splitmix64(base + i) >> 11 * 2^-53 (the same counter-based draws, per node base);
// take t unless it is taken already, else take j. The set bits are then written out ascending
// (wave prefix of the per-word popcounts). Bit-identical to a sequential Floyd on the same draws.
template <int W>
__global__ __launch_bounds__(256) void rf_sample_features_floyd_kernel(int C, int n, int nf, unsigned long long seed,
                                                                       int* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;  // wave-uniform
  const unsigned long long base = mix64(seed ^ mix64((unsigned long long)c + 1));
  unsigned long long w[W];
#pragma unroll
  for (int q = 0; q < W; ++q) w[q] = 0ull;
  for (int i = 0; i < nf; ++i) {
    const int j = n - nf + i;
    const double u = (double)(mix64(base + (unsigned long long)i) >> 11) * 0x1.0p-53;
    int t = (int)floor(u * (double)(j + 1));
    t = t > j ? j : t;
    // is t taken? word t >> 6 = register (t >> 12) of lane (t >> 6) & 63 (t is wave-uniform)
    // (readlane moves 32 bits: read the half of the word that holds bit t)
    unsigned wt = 0u;
#pragma unroll
    for (int q = 0; q < W; ++q)
      if (q == (t >> 12)) {
        const unsigned half = (unsigned)(w[q] >> (t & 32));
        wt = __builtin_amdgcn_readlane(half, (t >> 6) & 63);
      }
    const int pick = ((wt >> (t & 31)) & 1u) ? j : t;
#pragma unroll
    for (int q = 0; q < W; ++q)
      if (q == (pick >> 12) && lane == ((pick >> 6) & 63)) w[q] |= 1ull << (pick & 63);
  }
  int* o = out + (long)c * nf;
  int pos0 = 0;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const int cnt = __popcll(w[q]);
    int x = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    int pos = pos0 + x - cnt;
    unsigned long long b = w[q];
    const int f0 = (q * 64 + lane) * 64;
    while (b) {
      o[pos++] = f0 + __builtin_ctzll(b);
      b &= b - 1ull;
    }
    pos0 += __shfl(x, 63, 64);
  }
}

SRML_API int srml_rf_sample_features(int C, int n, int nf, unsigned long long seed, int* out, hipStream_t stream) {
  if (C <= 0 || nf <= 0) return 0;
  if (nf > n) return -2;
  const dim3 grid((unsigned)((C + 3) / 4));
  static const int floyd = getenv("SRML_RF_FLOYD") ? atoi(getenv("SRML_RF_FLOYD")) : 1;
  if (floyd && 8L * nf <= n && n <= 4 * 4096) {
#define SRML_FLOYD(W) \
  hipLaunchKernelGGL(rf_sample_features_floyd_kernel<W>, grid, dim3(256), 0, stream, C, n, nf, seed, out)
    if (n <= 4096) SRML_FLOYD(1);
    else if (n <= 2 * 4096) SRML_FLOYD(2);
    else SRML_FLOYD(4);
#undef SRML_FLOYD
    return srml_status();
  }
  hipLaunchKernelGGL(rf_sample_features_kernel, grid, dim3(256), 0, stream, C, n, nf, seed, out);
  return srml_status();
}

// Which sampler srml_rf_sample_features runs for (n, nf): 1 = Floyd, 0 = Algorithm S.
SRML_API int srml_rf_sample_features_floyd(int n, int nf) {
  static const int floyd = getenv("SRML_RF_FLOYD") ? atoi(getenv("SRML_RF_FLOYD")) : 1;
  return (floyd && nf > 0 && 8L * nf <= n && n <= 4 * 4096) ? 1 : 0;
}

// ------------------------------------------------------------------------------------------
// Stable re-partition of the position arrays into child segments (replaces a device radix sort of
// the child keys + searchsorted + two gathers per level). Every split parent segment s (split rank
// j, child_base = 2j) sends its positions to children 2j (left) and 2j + 1 (right), keeping their
// order; positions of unsplit segments leave the tree. With P = exclusive prefix over positions of
// (is_left | is_right << 32) the rank of a position inside its child is a difference of P values,
// the child sizes come from P at the parent's bounds, and the child offsets from a scan over the
// split parents. Kernels: flags + block scans, scan of the block totals, offsets, per-parent
// sizes, child bounds, scatter.
// ------------------------------------------------------------------------------------------
constexpr int PS_T = 256, PS_E = 4, PS_B = PS_T * PS_E;  // 1024 elements per scan block

__device__ __forceinline__ unsigned long long block_excl_scan_u64(unsigned long long v, unsigned long long* s_w,
                                                                  unsigned long long& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  unsigned long long base = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < PS_T / 64; ++w) {
    const unsigned long long tw = s_w[w];
    if (w < wid) base += tw;
    total += tw;
  }
  __syncthreads();
  return base + x - v;
}

// in == nullptr: the values are the partition flags of `keys` (left = even key, right = odd,
// dropped = 0x7fffffff); otherwise a plain u64 exclusive scan of `in`.
__global__ __launch_bounds__(PS_T) void scan_blocks_u64_kernel(const unsigned long long* __restrict__ in,
                                                               const int* __restrict__ keys, long n,
                                                               unsigned long long* __restrict__ out,
                                                               unsigned long long* __restrict__ tot) {
  __shared__ unsigned long long s_w[PS_T / 64];
  const long b0 = (long)blockIdx.x * PS_B + (long)threadIdx.x * PS_E;
  unsigned long long v[PS_E], sum = 0;
#pragma unroll
  for (int e = 0; e < PS_E; ++e) {
    const long i = b0 + e;
    unsigned long long x = 0;
    if (i < n) {
      if (in) {
        x = in[i];
      } else {
        const int k = keys[i];
        x = k == 0x7fffffff ? 0ull : ((k & 1) ? (1ull << 32) : 1ull);
      }
    }
    v[e] = x;
    sum += x;
  }
  unsigned long long total;
  unsigned long long run = block_excl_scan_u64(sum, s_w, total);
#pragma unroll
  for (int e = 0; e < PS_E; ++e) {
    const long i = b0 + e;
    if (i < n) out[i] = run;
    run += v[e];
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = total;
}

// exclusive scan of the nb block totals in place (one block), grand total to *grand
__global__ __launch_bounds__(PS_T) void scan_totals_u64_kernel(unsigned long long* __restrict__ tot, long nb,
                                                               unsigned long long* __restrict__ grand) {
  __shared__ unsigned long long s_w[PS_T / 64];
  unsigned long long carry = 0;
  for (long c0 = 0; c0 < nb; c0 += PS_T) {
    const long i = c0 + threadIdx.x;
    const unsigned long long x = i < nb ? tot[i] : 0ull;
    unsigned long long total;
    const unsigned long long ex = block_excl_scan_u64(x, s_w, total);
    if (i < nb) tot[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(PS_T) void scan_add_u64_kernel(unsigned long long* __restrict__ out, long n,
                                                            const unsigned long long* __restrict__ tot,
                                                            const unsigned long long* __restrict__ grand) {
  const long i = (long)blockIdx.x * PS_T + threadIdx.x;
  if (i < n) out[i] += tot[i / PS_B];
  if (i == n) out[n] = *grand;
}

// out[0..n] = exclusive prefix (out[n] = total) of in[0..n) (or of the partition flags of keys)
static int scan_u64(const unsigned long long* in, const int* keys, long n, unsigned long long* out,
                    unsigned long long* ws, hipStream_t stream) {
  const long nb = (n + PS_B - 1) / PS_B;
  if (nb > 0x7fffffffL) return -3;
  if (nb > 0)
    hipLaunchKernelGGL(scan_blocks_u64_kernel, dim3((unsigned)nb), dim3(PS_T), 0, stream, in, keys, n, out, ws);
  hipLaunchKernelGGL(scan_totals_u64_kernel, dim3(1), dim3(PS_T), 0, stream, ws, nb, ws + nb);
  hipLaunchKernelGGL(scan_add_u64_kernel, dim3((unsigned)((n + 1 + PS_T - 1) / PS_T)), dim3(PS_T), 0, stream, out, n,
                     ws, ws + nb);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Bootstrap bagging of T trees over m rows in one pass (reference: cuML RF bootstrap / Spark
// Poisson(subsamplingRate) bagging): element i = t m + r draws its multiplicity w ~ Poisson(rate)
// by inversion of a counter-based uniform (splitmix64 of seed, i), clamped to 255; the in-bag rows
// are compacted tree-major and ascending (the order the level segments keep). Kernels: per-block
// in-bag counts, scan of the block counts (scan_totals_u64_kernel), scatter with an in-block
// exclusive scan; tree bounds come out of the scatter (element t m marks tree t's start).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int poisson_draw(unsigned long long seed, long i, double rate, double e0) {
  const double u = (double)(mix64(seed ^ mix64((unsigned long long)i + 1)) >> 11) * 0x1.0p-53;
  int k = 0;
  double p = e0, F = e0;  // e0 = exp(-rate)
  while (u > F && k < 255) {
    ++k;
    p *= rate / (double)k;
    F += p;
  }
  return k;
}

__global__ __launch_bounds__(PS_T) void rf_boot_count_kernel(long N, unsigned long long seed, double rate, double e0,
                                                             unsigned long long* __restrict__ tot) {
  __shared__ unsigned long long s_w[PS_T / 64];
  const long b0 = (long)blockIdx.x * PS_B + (long)threadIdx.x * PS_E;
  unsigned long long c = 0;
#pragma unroll
  for (int e = 0; e < PS_E; ++e)
    if (b0 + e < N) c += poisson_draw(seed, b0 + e, rate, e0) > 0 ? 1ull : 0ull;
  unsigned long long total;
  block_excl_scan_u64(c, s_w, total);
  if (threadIdx.x == 0) tot[blockIdx.x] = total;
}

__global__ __launch_bounds__(PS_T) void rf_boot_scatter_kernel(long N, long m, unsigned long long seed, double rate,
                                                               double e0, const unsigned long long* __restrict__ boff,
                                                               const unsigned long long* __restrict__ grand,
                                                               int* __restrict__ idx, float* __restrict__ w,
                                                               long long* __restrict__ tbounds) {
  __shared__ unsigned long long s_w[PS_T / 64];
  const long b0 = (long)blockIdx.x * PS_B + (long)threadIdx.x * PS_E;
  int k[PS_E];
  unsigned long long c = 0;
#pragma unroll
  for (int e = 0; e < PS_E; ++e) {
    k[e] = b0 + e < N ? poisson_draw(seed, b0 + e, rate, e0) : 0;
    c += k[e] > 0 ? 1ull : 0ull;
  }
  unsigned long long total;
  unsigned long long o = boff[blockIdx.x] + block_excl_scan_u64(c, s_w, total);
#pragma unroll
  for (int e = 0; e < PS_E; ++e) {
    const long i = b0 + e;
    if (i >= N) break;
    const long r = i % m;
    if (r == 0) tbounds[i / m] = (long long)o;
    if (k[e] > 0) {
      idx[o] = (int)r;
      w[o] = (float)k[e];
      ++o;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) tbounds[N / m] = (long long)*grand;
}

// idx / w: capacity T m; tbounds: T + 1 (exclusive prefix of the per-tree in-bag counts); ws: at
// least srml_rf_bootstrap_ws(T, m) u64
SRML_API long srml_rf_bootstrap_ws(int T, long m) { return ((long)T * m + PS_B - 1) / PS_B + 1; }

// (weight, label) pairs in position order, the histogram kernels' row stream: wy[i] = (w[i], y[idx[i]])
// in one pass (replaces a gather, two conversions and a stack per tree level)
__global__ __launch_bounds__(256) void rf_pack_wy_kernel(const int* __restrict__ idx, const float* __restrict__ w,
                                                         const float* __restrict__ y, long P, float2* __restrict__ wy) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < P) wy[i] = make_float2(w[i], y[idx[i]]);
}

SRML_API int srml_rf_pack_wy(const int* idx, const float* w, const float* y, long P, float* wy, hipStream_t stream) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(rf_pack_wy_kernel, dim3((unsigned)ceil_div(P, 256)), dim3(256), 0, stream, idx, w, y, P,
                     reinterpret_cast<float2*>(wy));
  return srml_status();
}

SRML_API int srml_rf_bootstrap(int T, long m, double rate, unsigned long long seed, int* idx, float* w,
                               long long* tbounds, unsigned long long* ws, hipStream_t stream) {
  if (T <= 0 || m <= 0) return 0;
  if (!(rate > 0.0) || m > 0x7fffffffL) return -2;
  const long N = (long)T * m;
  const long nb = (N + PS_B - 1) / PS_B;
  if (nb > 0x7fffffffL) return -3;
  const double e0 = exp(-rate);
  hipLaunchKernelGGL(rf_boot_count_kernel, dim3((unsigned)nb), dim3(PS_T), 0, stream, N, seed, rate, e0, ws);
  hipLaunchKernelGGL(scan_totals_u64_kernel, dim3(1), dim3(PS_T), 0, stream, ws, nb, ws + nb);
  hipLaunchKernelGGL(rf_boot_scatter_kernel, dim3((unsigned)nb), dim3(PS_T), 0, stream, N, m, seed, rate, e0, ws,
                     ws + nb, idx, w, tbounds);
  return srml_status();
}

// per split parent j: cnt[j] = |left| + |right|, lcnt[j] = |left|, pstart[j] = the parent's start
__global__ __launch_bounds__(256) void part_parent_kernel(const long long* __restrict__ bounds, int nseg,
                                                          const int* __restrict__ node_feature,
                                                          const int* __restrict__ child_base,
                                                          const unsigned long long* __restrict__ P,
                                                          unsigned long long* __restrict__ cnt,
                                                          long long* __restrict__ lcnt, long long* __restrict__ pstart) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= nseg || node_feature[s] < 0) return;
  const int j = child_base[s] >> 1;
  const unsigned long long a = P[bounds[s]], b = P[bounds[s + 1]];
  const long long l = (long long)((b & 0xffffffffull) - (a & 0xffffffffull));
  const long long r = (long long)((b >> 32) - (a >> 32));
  cnt[j] = (unsigned long long)(l + r);
  lcnt[j] = l;
  pstart[j] = bounds[s];
}

// child bounds nb[2j] = off[j], nb[2j + 1] = off[j] + |left_j|, nb[2k] = kept total
__global__ __launch_bounds__(256) void part_bounds_kernel(const unsigned long long* __restrict__ off, int k,
                                                          const long long* __restrict__ lcnt,
                                                          long long* __restrict__ nb) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < k) {
    nb[2 * j] = (long long)off[j];
    nb[2 * j + 1] = (long long)off[j] + lcnt[j];
  }
  if (j == k) nb[2 * k] = (long long)off[k];
}

__global__ __launch_bounds__(256) void part_scatter_kernel(const int* __restrict__ keys, long total,
                                                           const unsigned long long* __restrict__ P,
                                                           const long long* __restrict__ pstart,
                                                           const long long* __restrict__ nb,
                                                           const int* __restrict__ idx, const float* __restrict__ w,
                                                           int* __restrict__ idx_out, float* __restrict__ w_out) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= total) return;
  const int c = keys[p];
  if (c == 0x7fffffff) return;
  const int j = c >> 1;
  const unsigned long long a = P[pstart[j]], x = P[p];
  const long long rank = (c & 1) ? (long long)((x >> 32) - (a >> 32)) : (long long)((x & 0xffffffffull) - (a & 0xffffffffull));
  const long long q = nb[c] + rank;
  idx_out[q] = idx[p];
  w_out[q] = w[p];
}

// Workspace (u64 elements) for srml_rf_partition with `total` positions and k split parents.
SRML_API long srml_rf_partition_ws(long total, int k) {
  return (total + 1) + ((total + PS_B - 1) / PS_B + 1) + 3L * (k + 1) + ((k + PS_B) / PS_B + 1);
}

// keys: child key per position (srml_rf_route_segments); nseg parent segments (bounds nseg + 1);
// k split parents. Writes idx_out / w_out (kept positions, child order) and nb (2k + 1 bounds).
SRML_API int srml_rf_partition(const int* keys, long total, const long long* bounds, int nseg,
                               const int* node_feature, const int* child_base, int k, const int* idx, const float* w,
                               int* idx_out, float* w_out, long long* nb, unsigned long long* ws, hipStream_t stream) {
  if (total < 0 || k < 0 || total >= (1L << 32)) return -2;
  unsigned long long* P = ws;                                   // total + 1
  unsigned long long* tws = P + total + 1;                      // block totals + grand
  const long nbt = (total + PS_B - 1) / PS_B + 1;
  unsigned long long* cnt = tws + nbt;                          // k + 1 (scanned into offsets)
  long long* lcnt = reinterpret_cast<long long*>(cnt + k + 1);  // k + 1
  long long* pstart = lcnt + k + 1;                             // k + 1
  unsigned long long* tws2 = reinterpret_cast<unsigned long long*>(pstart + k + 1);
  if (k == 0) return (int)hipMemsetAsync(nb, 0, sizeof(long long), stream);  // every position leaves
  int st = scan_u64(nullptr, keys, total, P, tws, stream);
  if (st) return st;
  if (nseg > 0)
    hipLaunchKernelGGL(part_parent_kernel, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, stream, bounds, nseg,
                       node_feature, child_base, P, cnt, lcnt, pstart);
  st = scan_u64(cnt, nullptr, k, cnt, tws2, stream);  // in place: off[0..k]
  if (st) return st;
  hipLaunchKernelGGL(part_bounds_kernel, dim3((unsigned)((k + 1 + 255) / 256)), dim3(256), 0, stream, cnt, k, lcnt, nb);
  if (total > 0)
    hipLaunchKernelGGL(part_scatter_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, keys, total, P,
                       pstart, nb, idx, w, idx_out, w_out);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// per-segment node statistics (replaces cumsum-based segment sums): each block reduces a
// contiguous chunk of positions in registers and flushes one fp64 atomic per (segment, stat)
// it touched; chunks are sorted so a block rarely spans more than a couple of segments.
// regression: (sum w, sum w y, sum w y^2); classification: per-class sum w.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rf_node_stats_kernel(const int* __restrict__ idx,
                                                            const float* __restrict__ wpos,
                                                            const float* __restrict__ label, long total,
                                                            const long long* __restrict__ bounds, int nseg, int S,
                                                            int regression, long chunk, double* __restrict__ out) {
  __shared__ double red[4][32];
  const long p0 = (long)blockIdx.x * chunk;
  const long p1 = min(total, p0 + chunk);
  if (p0 >= p1) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // first segment of the chunk
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (bounds[mid] <= p0) lo = mid; else hi = mid - 1;
  }
  const int NS = regression ? 3 : S;
  for (int seg = lo; seg < nseg && bounds[seg] < p1; ++seg) {
    const long a = max(p0, (long)bounds[seg]), b = min(p1, (long)bounds[seg + 1]);
    if (a >= b) continue;
    double acc[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) acc[k] = 0.0;
    for (long i = a + threadIdx.x; i < b; i += 256) {
      const double w = wpos[i];
      const double y = label[idx[i]];
      if (regression) {
        acc[0] += w;
        acc[1] += w * y;
        acc[2] += w * y * y;
      } else {
        const int c = (int)y;
#pragma unroll
        for (int k = 0; k < 32; ++k)
          if (k == c) acc[k] += w;
      }
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {  // static indices: acc stays in registers (no scratch)
      if (k < NS) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) red[wid][k] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x < NS) {
      const double v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
      if (v != 0.0) atomicAdd(&out[(long)seg * NS + threadIdx.x], v);
    }
    __syncthreads();
  }
}

// deterministic variant (SRML_DETERMINISTIC): one block per segment, strided per-thread sums and
// a fixed-order block reduction, plain stores (no atomics: bit-identical run to run)
__global__ __launch_bounds__(256) void rf_node_stats_seg_kernel(const int* __restrict__ idx,
                                                                const float* __restrict__ wpos,
                                                                const float* __restrict__ label,
                                                                const long long* __restrict__ bounds, int S,
                                                                int regression, double* __restrict__ out) {
  __shared__ double red[4][32];
  const int seg = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int NS = regression ? 3 : S;
  double acc[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) acc[k] = 0.0;
  for (long i = bounds[seg] + threadIdx.x; i < bounds[seg + 1]; i += 256) {
    const double w = wpos[i];
    const double y = label[idx[i]];
    if (regression) {
      acc[0] += w;
      acc[1] += w * y;
      acc[2] += w * y * y;
    } else {
      const int c = (int)y;
#pragma unroll
      for (int k = 0; k < 32; ++k)
        if (k == c) acc[k] += w;
    }
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {  // static indices: acc stays in registers (no scratch)
    if (k < NS) {
      const double v = wave_sum(acc[k]);
      if (lane == 0) red[wid][k] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < NS)
    out[(long)seg * NS + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

SRML_API int srml_rf_node_stats_det(const int* idx, const float* wpos, const float* label,
                                    const long long* bounds, int nseg, int S, int regression, double* out,
                                    hipStream_t stream) {
  if (nseg <= 0) return 0;
  if (!regression && S > 32) return -7;
  hipLaunchKernelGGL(rf_node_stats_seg_kernel, dim3((unsigned)nseg), dim3(256), 0, stream, idx, wpos, label, bounds,
                     S, regression, out);
  return srml_status();
}

SRML_API int srml_rf_node_stats(const int* idx, const float* wpos, const float* label, long total,
                                const long long* bounds, int nseg, int S, int regression, double* out,
                                hipStream_t stream) {
  if (total <= 0 || nseg <= 0) return 0;
  if (!regression && S > 32) return -7;
  long chunk = (total + 4095) / 4096;
  if (chunk < 2048) chunk = 2048;
  const long blocks = (total + chunk - 1) / chunk;
  hipLaunchKernelGGL(rf_node_stats_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, idx, wpos, label, total,
                     bounds, nseg, S, regression, chunk, out);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// inference: trees stored as flat node arrays; roots[t] = first node of tree t.
// feature < 0 => leaf whose value vector (width S) starts at values[value_off[node]].
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rf_predict_kernel(const float* __restrict__ X, long m, long ld,
                                                         const int* __restrict__ roots, int ntrees,
                                                         const int* __restrict__ feature,
                                                         const float* __restrict__ threshold,
                                                         const int* __restrict__ left, const int* __restrict__ right,
                                                         const int* __restrict__ value_off,
                                                         const float* __restrict__ values, int S,
                                                         float* __restrict__ out, int* __restrict__ leaves) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  const float* row = X + r * ld;
  float acc[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) acc[c] = 0.f;
  for (int t = 0; t < ntrees; ++t) {
    int node = roots[t];
    int f = feature[node];
    while (f >= 0) {
      node = (row[f] <= threshold[node]) ? left[node] : right[node];
      f = feature[node];
    }
    if (leaves) leaves[r * ntrees + t] = node - roots[t];
    const float* v = values + value_off[node];
#pragma unroll
    for (int c = 0; c < 32; ++c)
      if (c < S) acc[c] += v[c];
  }
#pragma unroll
  for (int c = 0; c < 32; ++c)
    if (c < S) out[r * S + c] = acc[c];
}

SRML_API int srml_rf_predict(const float* X, long m, long ld, const int* roots, int ntrees, const int* feature,
                             const float* threshold, const int* left, const int* right, const int* value_off,
                             const float* values, int S, float* out, int* leaves, hipStream_t stream) {
  if (m <= 0) return 0;
  if (S > 32) return -7;
  hipLaunchKernelGGL(rf_predict_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, X, m, ld, roots,
                     ntrees, feature, threshold, left, right, value_off, values, S, out, leaves);
  return srml_status();
}

// node: {feature, left, right, threshold bits}; leaf: {-1, value offset, leaf id within its tree, 0}
template <int SV>
__global__ __launch_bounds__(256) void rf_predict_wave_kernel(const float* __restrict__ X, long m, long ld,
                                                              const int4* __restrict__ nodes,
                                                              const int* __restrict__ roots, int ntrees,
                                                              const float* __restrict__ values, int S,
                                                              float* __restrict__ out, int* __restrict__ leaves) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * 4;
  for (long r = wave; r < m; r += nw) {
    const float* row = X + r * ld;
    float acc[SV];
#pragma unroll
    for (int c = 0; c < SV; ++c) acc[c] = 0.f;
    for (int t = lane; t < ntrees; t += 64) {
      int4 nd = nodes[roots[t]];
      while (nd.x >= 0) {
        const float xv = row[nd.x];
        nd = nodes[xv <= __int_as_float(nd.w) ? nd.y : nd.z];
      }
      if (leaves) leaves[r * ntrees + t] = nd.z;
      const float* v = values + nd.y;
#pragma unroll
      for (int c = 0; c < SV; ++c)
        if (c < S) acc[c] += v[c];
    }
    float mine = 0.f;
#pragma unroll
    for (int c = 0; c < SV; ++c) {
      const float tot = wave_sum(acc[c]);
      if (c == lane) mine = tot;
    }
    if (lane < S) out[r * S + lane] = mine;
  }
}

// Rows staged in LDS (n <= RF_LDS_N): each wave streams its row with coalesced 16-B loads into
// its own LDS slice (12 KB at n = 3000), then the lanes' tree walks gather from LDS instead of
// issuing one scattered global load per level; HBM traffic is exactly X once, at full width.
constexpr int RF_LDS_N = 4096;

template <int SV>
__global__ __launch_bounds__(256) void rf_predict_lds_kernel(const float* __restrict__ X, long m, long ld, int n,
                                                             const int4* __restrict__ nodes,
                                                             const int* __restrict__ roots, int ntrees,
                                                             const float* __restrict__ values, int S,
                                                             float* __restrict__ out, int* __restrict__ leaves) {
  extern __shared__ __attribute__((aligned(16))) float srow_all[];  // [4][npad]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int npad = (n + 3) & ~3;
  float* srow = srow_all + wid * npad;
  const long nw = (long)gridDim.x * 4;
  for (long r0 = (long)blockIdx.x * 4; r0 < m; r0 += nw) {
    const long r = r0 + wid;
    const bool active = r < m;
    if (active) {
      const float* row = X + r * ld;
      for (int c = lane * 4; c < npad; c += 256)
        *reinterpret_cast<floatx4*>(&srow[c]) = *reinterpret_cast<const floatx4*>(row + c);
    }
    __syncthreads();
    if (active) {
      float acc[SV];
#pragma unroll
      for (int c = 0; c < SV; ++c) acc[c] = 0.f;
      for (int t = lane; t < ntrees; t += 64) {
        int4 nd = nodes[roots[t]];
        while (nd.x >= 0) nd = nodes[srow[nd.x] <= __int_as_float(nd.w) ? nd.y : nd.z];
        if (leaves) leaves[r * ntrees + t] = nd.z;
        const float* v = values + nd.y;
#pragma unroll
        for (int c = 0; c < SV; ++c)
          if (c < S) acc[c] += v[c];
      }
      float mine = 0.f;
#pragma unroll
      for (int c = 0; c < SV; ++c) {
        const float tot = wave_sum(acc[c]);
        if (c == lane) mine = tot;
      }
      if (lane < S) out[r * S + lane] = mine;
    }
    __syncthreads();
  }
}

SRML_API int srml_rf_predict_nodes2(const float* X, long m, long ld, int n, const int* nodes, const int* roots,
                                    int ntrees, const float* values, int S, float* out, int* leaves,
                                    hipStream_t stream) {
  if (m <= 0) return 0;
  if (S < 1 || S > 32) return -7;
  long blocks = (m + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  const int4* nd = reinterpret_cast<const int4*>(nodes);
  const bool lds = n <= RF_LDS_N && ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   (n % 4 == 0 || (long)((n + 3) & ~3) <= ld);
  if (lds) {
    const size_t shm = (size_t)4 * ((n + 3) & ~3) * sizeof(float);
#define SRML_RF_PRED_LDS(SVV)                                                                                     \
    hipLaunchKernelGGL(rf_predict_lds_kernel<SVV>, dim3((unsigned)blocks), dim3(256), shm, stream, X, m, ld, n, nd, \
                       roots, ntrees, values, S, out, leaves)
    if (S <= 1) SRML_RF_PRED_LDS(1);
    else if (S <= 2) SRML_RF_PRED_LDS(2);
    else if (S <= 4) SRML_RF_PRED_LDS(4);
    else if (S <= 8) SRML_RF_PRED_LDS(8);
    else if (S <= 16) SRML_RF_PRED_LDS(16);
    else SRML_RF_PRED_LDS(32);
#undef SRML_RF_PRED_LDS
    return srml_status();
  }
#define SRML_RF_PRED(SVV)                                                                                        \
  hipLaunchKernelGGL(rf_predict_wave_kernel<SVV>, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, ld, nd, roots, \
                     ntrees, values, S, out, leaves)
  if (S <= 1) SRML_RF_PRED(1);
  else if (S <= 2) SRML_RF_PRED(2);
  else if (S <= 4) SRML_RF_PRED(4);
  else if (S <= 8) SRML_RF_PRED(8);
  else if (S <= 16) SRML_RF_PRED(16);
  else SRML_RF_PRED(32);
#undef SRML_RF_PRED
  return srml_status();
}
