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

// ------------------------------------------------------------------------------------------
// fp16 candidate search, centred on the query list (n <= 128, k <= 32).
//
// Rows of one inverted list sit around its centroid, so a query tile of list c and the items of
// c's probe lists are shifted by C_c while they are staged (fp32 load -> subtract -> fp16 LDS):
// the dot products then see local magnitudes (~ the list radius, not ||x||) and fp16's 11-bit
// mantissa ranks candidates almost like fp32; the caller asks for a few extra neighbours and
// re-ranks them with exact fp32 distances (knn_refine_sort). Per 128 x 128 tile pair:
//  * the query tile is staged ONCE per block (it was re-read for every item tile before), the
//    next item tile is prefetched into registers while the MFMAs run on the current one
//    (`v_mfma_f32_32x32x16_f16`: 16x the fp32 MFMA rate, 8 waves = 2 per SIMD);
//  * item norms ||i - C_c||^2 of the rounded rows come from the staging pass (lane-contiguous
//    coalesced loads: one row is 32 lanes x 16 B, reduced by 4 DPP adds per 16-lane group);
//  * selection is a threshold filter in registers: a lane compares its 32 accumulator values
//    (fmaf(-2, acc, ||i||^2)) with its rows' current k-th best and appends the rare survivors
//    to per-row LDS candidate lists (LDS atomics), which one thread per row merges into its
//    sorted top-k. A row that overflows its 32 slots keeps the values not yet taken (a per-lane
//    mask) and the tile re-runs the append after the merge tightened the thresholds, so no
//    candidate is lost and every value is appended at most once.
namespace {
typedef _Float16 kg_halfx8 __attribute__((ext_vector_type(8)));
typedef _Float16 kg_half2 __attribute__((ext_vector_type(2)));
constexpr int F_BM = 128, F_BN = 128, F_KP = 128, F_RS = F_KP + 8;  // LDS row stride (halves)
constexpr int F_CAP = 32, F_KQ = 32, F_PMAX = 128;

__device__ __forceinline__ float kg_dpp(float v, int ctrl_sel) {
  // ctrl_sel: 0 quad xor 1, 1 quad xor 2, 2 row_ror:4, 3 row_ror:8
  const int x = __float_as_int(v);
  int r;
  switch (ctrl_sel) {
    case 0: r = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xf, 0xf, false); break;
    case 1: r = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xf, 0xf, false); break;
    case 2: r = __builtin_amdgcn_update_dpp(0, x, 0x124, 0xf, 0xf, false); break;
    default: r = __builtin_amdgcn_update_dpp(0, x, 0x128, 0xf, 0xf, false); break;
  }
  return __int_as_float(r);
}

// sum over the 16 lanes of a DPP row, in every lane of it
__device__ __forceinline__ float kg_sum16(float v) {
  v += kg_dpp(v, 0);
  v += kg_dpp(v, 1);
  v += kg_dpp(v, 2);
  v += kg_dpp(v, 3);
  return v;
}

// Wave w stages rows 16w .. 16w + 15 of a 128-row tile: load j covers rows 16w + 2j (lanes 0-31)
// and 16w + 2j + 1 (lanes 32-63), columns 4 (lane & 31) .. + 3.
struct KgPf {
  floatx4 v[8];
};

__device__ __forceinline__ void kg_load(KgPf& pf, const float* __restrict__ X, long ld, long r0, long nvalid, int n,
                                        int wid, int lane) {
  // unconditional loads from clamped addresses (kg_store zeroes what lies outside the tile): a
  // conditional load would make the compiler zero the destination first and wait on the loads
  // still in flight for the other register set
  const int col = min(4 * (lane & 31), n - 4);
  const long rmax = nvalid > 0 ? nvalid - 1 : 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long r = min((long)(16 * wid + 2 * j + (lane >> 5)), rmax);
    pf.v[j] = *reinterpret_cast<const floatx4*>(X + (r0 + r) * ld + col);  // plain: item tiles are re-read through L2
  }
}

__device__ __forceinline__ void kg_store(const KgPf& pf, _Float16* __restrict__ dst, floatx4 cen, int wid, int lane,
                                         long nvalid, int n) {
  const int col = 4 * (lane & 31);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int r = 16 * wid + 2 * j + (lane >> 5);
    const bool ok = r < nvalid && col < n;
    const floatx4 x = ok ? pf.v[j] - cen : floatx4{0.f, 0.f, 0.f, 0.f};
    typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<halfx4*>(dst + r * F_RS + col) =
        halfx4{(_Float16)x[0], (_Float16)x[1], (_Float16)x[2], (_Float16)x[3]};
  }
}

// Wave-wide bitonic sorts of 64 (distance, index) pairs, ascending (index breaks ties), R rows
// at once: the R exchange chains are independent, so their shuffle latencies overlap.
template <int R>
__device__ __forceinline__ void kg_bitonic64(float (&d)[R], int (&id)[R], int lane) {
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const bool up = (lane & size) == 0 || size == 64;
      const bool lower = (lane & stride) == 0;
      float od[R];
      int oi[R];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        od[q] = __shfl_xor(d[q], stride, 64);
        oi[q] = __shfl_xor(id[q], stride, 64);
      }
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const bool other_less = od[q] < d[q] || (od[q] == d[q] && oi[q] < id[q]);
        if ((lower == up) == other_less) {
          d[q] = od[q];
          id[q] = oi[q];
        }
      }
    }
}

// Merge the rows' candidate lists into their sorted top lists (32 slots, +inf padded): wave w
// owns rows 16w .. 16w + 15, one row at a time (4 interleaved rows measured no faster), lanes
// 0..31 holding the top list and lanes 32 + j candidate j. A row is merged when it holds
// >= min_fill candidates.
// Few candidates (the usual case once thresholds are seeded or warm): rank insertion — every
// element's merged position is its rank in its own list plus the number of elements of the other
// list ahead of it, counted in one pass over the m candidates (each broadcast from its lane: one
// compare per lane, one ballot for the tops ahead of it), then one scatter. ~10 instructions per
// candidate instead of the 21 exchange stages of the 64-lane bitonic sort, which stays for rows
// with many candidates (an overflow). Order: (distance, index), a top entry ahead of an equal
// candidate.
constexpr int KG_RANK_MAX = 12;
__device__ __forceinline__ void kg_merge(float (*topd)[F_KQ + 1], int (*topi)[F_KQ + 1], float (*cand_d)[F_CAP + 1],
                                         int (*cand_i)[F_CAP + 1], int* cnt, float* thr_s, int k, int nq, int wid,
                                         int lane, int min_fill) {
  const float inf = __builtin_huge_valf();
  const bool top = lane < 32;
  for (int r = 0; r < F_BM / 8; ++r) {
    const int row = wid * (F_BM / 8) + r;
    const int m = __builtin_amdgcn_readfirstlane(min(cnt[row], F_CAP));
    if (m == 0 || m < min_fill) continue;  // wave-uniform: this row keeps collecting
    const bool ok = top || lane - 32 < m;
    float d = top ? topd[row][lane] : (ok ? cand_d[row][lane - 32] : inf);
    int id = top ? topi[row][lane] : (ok ? cand_i[row][lane - 32] : -1);
    int pos;
    if (m <= KG_RANK_MAX) {
      pos = top ? lane : 0;
      unsigned long long mine = 0ull;  // candidate lanes: the tops ahead of this candidate
      for (int j = 0; j < m; ++j) {
        const float bd = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, d), 32 + j));
        const int bi = __builtin_amdgcn_readlane(id, 32 + j);
        // candidate j ahead of this lane's element (a top wins a full tie; candidates by lane)
        const bool ahead = bd < d || (bd == d && (bi < id || (bi == id && !top && 32 + j < lane)));
        const unsigned long long tops_ahead = __ballot(top && !ahead);
        pos += ahead ? 1 : 0;
        if (lane == 32 + j) mine = tops_ahead;
      }
      pos += top ? 0 : __popcll(mine);
      if (!ok) pos = 64;
      if (pos < F_KQ) {
        topd[row][pos] = d;
        topi[row][pos] = id;
      }
    } else {
      float dd[1] = {d};
      int ii[1] = {id};
      kg_bitonic64<1>(dd, ii, lane);
      d = dd[0];
      id = ii[0];
      pos = lane;
      if (top) {
        topd[row][lane] = d;
        topi[row][lane] = id;
      }
    }
    // (the k-th best only falls; min() also keeps a seeded threshold while fewer than k
    // candidates have been found)
    if (pos == k - 1 && row < nq) thr_s[row] = fminf(thr_s[row], d);
    if (lane == 0) cnt[row] = 0;
  }
}

// Wave w loads query rows 16w .. 16w + 15 of a tile given by row ids (the PAIRS mode's queries
// are gathered: rows that probe the tile's list come from anywhere in X)
__device__ __forceinline__ void kg_load_rows(KgPf& pf, const float* __restrict__ X, long ld,
                                             const int* __restrict__ rows, long nvalid, int n, int wid, int lane) {
  const int col = min(4 * (lane & 31), n - 4);
  const long rmax = nvalid > 0 ? nvalid - 1 : 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long r = min((long)(16 * wid + 2 * j + (lane >> 5)), rmax);
    pf.v[j] = *reinterpret_cast<const floatx4*>(X + (long)rows[r] * ld + col);
  }
}

// Pre-centred fp16 item rows (PAIRS mode: every item of list c is x - C_c, converted once per
// fit, rows of F_KP halves = 256 B): a tile is 128 rows x 16 pieces of 16 B; thread t moves pieces
// t + 512 i (i < 4): 16 consecutive threads cover one row, fully coalesced, no conversion
struct KgPh {
  uint4 v[4];
  float nrm;  // ||item||^2 of this lane's MFMA column (row `col` of the tile), loaded with the tile
};

__device__ __forceinline__ void kg_load_h(KgPh& pf, const _Float16* __restrict__ Xh, const float* __restrict__ xhn,
                                          long r0, long nvalid, int t, int col) {
  const long rmax = nvalid > 0 ? nvalid - 1 : 0;
  pf.nrm = xhn[r0 + min((long)col, rmax)];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = t + 512 * i;
    const long r = min((long)(id >> 4), rmax);
    pf.v[i] = *reinterpret_cast<const uint4*>(Xh + (r0 + r) * F_KP + 8 * (id & 15));
  }
}

__device__ __forceinline__ void kg_store_h(const KgPh& pf, _Float16* __restrict__ dst, long nvalid, int t) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = t + 512 * i;
    const int r = id >> 4;
    *reinterpret_cast<uint4*>(dst + r * F_RS + 8 * (id & 15)) = r < nvalid ? pf.v[i] : make_uint4(0u, 0u, 0u, 0u);
  }
}

// PAIRS = false: a tile is <= 128 consecutive rows of list c = tile_list[b] (its rows X[q0 ..)),
// scanning the lists probes[c][0 .. nprobe); output row = the query's sorted row.
// PAIRS = true (per-query probing, inverted): the (row, probed list) pairs are sorted by list; a
// tile is <= 128 consecutive pairs of list c = tile_list[b] (pair positions q0 .. bounded by
// pair_off[c + 1]), its queries are the rows qrows[q0 ..], gathered, and it scans list c's own
// items (probes[c][0] = c, nprobe = 1). Both operands are centred on C_c, and ||q - C_c||^2 of the
// rounded query is added to the keys, so keys of one row from different lists compare (they are
// the fp16-rounded ||q - i||^2); output row = qslot[pair position] (the caller's per-pair slot).
// H16 (PAIRS only): the items come pre-centred in fp16 (Xh: x - C_list(x), N x F_KP halves, and
// their norms xhn): the per-tile staging is a plain 16-B copy (half the bytes, no conversion) and
// the item norms are loaded, not recomputed from the fragments.
template <bool PAIRS, bool H16 = false>
__global__ __launch_bounds__(512, 1) void knn_lists_f16_kernel(
    const float* __restrict__ X, int n, long ld, const float* __restrict__ C, const long long* __restrict__ list_off,
    const int* __restrict__ probes, int nprobe, const long long* __restrict__ tile_q0,
    const int* __restrict__ tile_list, int ntiles, int k, float* __restrict__ out_d, int* __restrict__ out_i,
    const int* __restrict__ qrows = nullptr, const int* __restrict__ qslot = nullptr,
    const long long* __restrict__ pair_off = nullptr, const float* __restrict__ thr_row = nullptr,
    const _Float16* __restrict__ Xh = nullptr, const float* __restrict__ xhn = nullptr) {
  static_assert(PAIRS || !H16, "pre-centred items are the PAIRS mode's (items centred on their own list)");
  __shared__ __attribute__((aligned(16))) _Float16 Qs[F_BM * F_RS];
  __shared__ __attribute__((aligned(16))) _Float16 Is[F_BN * F_RS];
  __shared__ float cand_d[F_BM][F_CAP + 1];
  __shared__ int cand_i[F_BM][F_CAP + 1];
  __shared__ int cnt[F_BM];
  __shared__ float topd[F_BM][F_KQ + 1];
  __shared__ int topi[F_BM][F_KQ + 1];
  __shared__ __attribute__((aligned(16))) float thr_s[F_BM];
  __shared__ int ovf[2];
  __shared__ long long pl[F_PMAX][2];
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  if (b >= ntiles) return;  // block-uniform
  const int c = tile_list[b];
  const long q0 = tile_q0[b];
  const long q1 = min(q0 + (long)F_BM, (long)(PAIRS ? pair_off : list_off)[c + 1]);
  const int nq = (int)(q1 - q0);
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int wm = wid >> 2, wn = wid & 3;  // wave tile: rows 64 wm .. +64, columns 32 wn .. +32
  __shared__ float qn_s[F_BM];  // PAIRS: ||q - C_c||^2 of the rounded queries
  const int li = lane & 31, lk = lane >> 5;
  const float inf = __builtin_huge_valf();
  for (int i = t; i < F_BM * (F_KQ + 1); i += 512) {
    (&topd[0][0])[i] = inf;
    (&topi[0][0])[i] = -1;
  }
  if (t < F_BM) {
    cnt[t] = 0;
    thr_s[t] = t < nq ? inf : -inf;  // rows past the tile never take candidates
  }
  if (t < 2) ovf[t] = 0;
  floatx4 cen = floatx4{0.f, 0.f, 0.f, 0.f};
  {
    const int col = 4 * li;
    if (col < n) cen = *reinterpret_cast<const floatx4*>(C + (long)c * n + col);
  }
  // probed lists' row ranges, read once into LDS (empty range for a missing probe)
  if (t < nprobe) {
    const int l = probes[(long)c * nprobe + t];
    pl[t][0] = l >= 0 ? list_off[l] : 0;
    pl[t][1] = l >= 0 ? list_off[l + 1] : 0;
  }
  __syncthreads();
  // probe / item-tile iterator (block-uniform)
  int p = -1;
  long c0 = 0, e = 0;
  auto next_tile = [&]() -> bool {
    c0 += F_BN;
    while (c0 >= e) {
      if (++p >= nprobe) return false;
      c0 = pl[p][0];
      e = pl[p][1];
    }
    return true;
  };
  // item tiles flow: registers -> centred fp16 LDS tile -> MFMA. The loads of tile t + 2 are
  // issued right after tile t + 1 is staged (at tile t's first barrier), so they have a whole
  // tile period to arrive.
  // (a second fp16 register buffer keeping tiles t + 1 AND t + 2 in flight measured 5 % slower
  // once the query fragments moved to registers: it spilled, 20M rows 1.205 vs 1.140 s)
  KgPf pfa;
  KgPh pfh;
  const int my_col = wn * 32 + li;  // this lane's item column in every MFMA tile
  float is_nrm = 0.f;              // H16: its item norm for the tile now in Is
  auto load_items = [&](long r0, long nv) {
    if constexpr (H16) kg_load_h(pfh, Xh, xhn, r0, nv, t, my_col);
    else kg_load(pfa, X, ld, r0, nv, n, wid, lane);
  };
  auto store_items = [&](long nv) {
    if constexpr (H16) {
      kg_store_h(pfh, Is, nv, t);
      is_nrm = pfh.nrm;
    } else {
      kg_store(pfa, Is, cen, wid, lane, nv, n);
    }
  };
  bool have = next_tile();  // tile in LDS
  long tc0 = c0, te = e;
  if (have) load_items(c0, e - c0);
  {
    KgPf pq;
    if (PAIRS) kg_load_rows(pq, X, ld, qrows + q0, nq, n, wid, lane);
    else kg_load(pq, X, ld, q0, nq, n, wid, lane);
    kg_store(pq, Qs, cen, wid, lane, nq, n);
  }
  if (have) store_items(te - tc0);
  bool have1 = have && next_tile();  // tile after it, in registers
  long h1c0 = c0, h1e = e;
  if (have1) load_items(c0, e - c0);
  __syncthreads();
  if (PAIRS) {
    // ||q - C_c||^2 of the staged (rounded, centred) queries; padding columns are zero. A seeded
    // row threshold (thr_row: its k-th best squared distance so far, from lists it already
    // scanned) becomes the key threshold thr - ||q - C_c||^2: only items that can enter the row's
    // top k are appended, so the candidate lists rarely fill and the merges all but vanish
    if (t < nq) {
      float a = 0.f;
      for (int j = 0; j < F_KP; j += 2) {
        const kg_half2 h = *reinterpret_cast<const kg_half2*>(Qs + t * F_RS + j);
        a = __builtin_amdgcn_fdot2(h, h, a, false);
      }
      qn_s[t] = a;
      if (thr_row) thr_s[t] = thr_row[qrows[q0 + t]] - a;
    }
    __syncthreads();
  }
  const int nks = (n + 15) >> 4;
  // this wave's query fragments stay in registers for the whole scan: re-reading them from LDS
  // for every item tile made the MFMA operand traffic (24 KB per wave and tile) LDS-bound
  kg_halfx8 areg[2][F_KP / 16];
#pragma unroll
  for (int ks = 0; ks < F_KP / 16; ++ks)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
      areg[mt][ks] = *reinterpret_cast<const kg_halfx8*>(Qs + (wm * 64 + mt * 32 + li) * F_RS + ks * 16 + lk * 8);
  int par = 0;
  while (have) {
    // the next tile to fetch: t + 2
    const bool haveN = have1 && next_tile();
    const long hNc0 = c0, hNe = e;
    floatx16 acc[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
    float nrm = 0.f;  // ||i - C_c||^2 of the rounded item row, from the B fragments themselves
#pragma unroll
    for (int ks = 0; ks < F_KP / 16; ++ks) {
      if (ks >= nks) break;  // block-uniform (zero padding columns past n)
      const kg_halfx8 bv = *reinterpret_cast<const kg_halfx8*>(Is + (wn * 32 + li) * F_RS + ks * 16 + lk * 8);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(areg[mt][ks], bv, acc[mt], 0, 0, 0);
      if constexpr (!H16) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const kg_half2 h = kg_half2{bv[2 * u], bv[2 * u + 1]};
          nrm = __builtin_amdgcn_fdot2(h, h, nrm, false);
        }
      }
    }
    const int col = wn * 32 + li;
    const long cg = tc0 + col;
    if constexpr (H16) nrm = is_nrm;  // came with the tile (no load on the MFMA -> filter path)
    else nrm += __shfl_xor(nrm, 32, 64);  // the other k half of the same item row
    const float inv = cg < te ? nrm : inf;
    unsigned done = 0u;
    bool first = true;
    for (;;) {
      // filter: one bit per accumulator value below its row's threshold, not yet taken
      unsigned pass = 0u;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const floatx4 tv = *reinterpret_cast<const floatx4*>(&thr_s[wm * 64 + mt * 32 + 8 * g + 4 * lk]);
#pragma unroll
          for (int u = 0; u < 4; ++u)
            pass |= (unsigned)(fmaf(-2.f, acc[mt][4 * g + u], inv) < tv[u]) << (mt * 16 + 4 * g + u);
        }
      pass &= ~done;
      if (pass) {
        // groups of 4 values (4 consecutive rows): survivors are rare, so most groups are skipped
        // with one branch; inside a group all slot atomics go out together, then the writes
#pragma unroll
        for (int gq = 0; gq < 8; ++gq) {
          if (pass & (0xFu << (4 * gq))) {
            const int mt = gq >> 2, g = gq & 3;
            const int row0 = wm * 64 + mt * 32 + 8 * g + 4 * lk;
            int slot[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (pass & (1u << (4 * gq + u))) slot[u] = atomicAdd(&cnt[row0 + u], 1);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const unsigned bit = 1u << (4 * gq + u);
              if (pass & bit) {
                if (slot[u] < F_CAP) {
                  cand_d[row0 + u][slot[u]] = fmaf(-2.f, acc[mt][4 * g + u], inv);
                  cand_i[row0 + u][slot[u]] = (int)cg;
                  done |= bit;
                } else {
                  ovf[par] = 1;
                }
              }
            }
          }
        }
      }
      __syncthreads();  // A: candidates visible; every wave is past its MFMAs on Is
      if (first && have1) {
        // pin the prefetched registers behind the barrier: otherwise the compiler hoists the
        // centring/conversion above the append loop and waits for the loads right after the MFMAs
        if constexpr (H16) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            asm volatile("" : "+v"(pfh.v[j].x), "+v"(pfh.v[j].y), "+v"(pfh.v[j].z), "+v"(pfh.v[j].w));
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(pfa.v[j]));
        }
        store_items(h1e - h1c0);
        if (haveN) load_items(hNc0, hNe - hNc0);
      }
      const int full = ovf[par];  // block-uniform: some row ran out of candidate slots
      first = false;
      if (t == 0) ovf[par ^ 1] = 0;
      // every row with candidates is merged when one row overflows: fresher thresholds measured
      // 2 % faster than merging only rows at least half full (4M rows: 0.1533 vs 0.1564 s)
      if (full) kg_merge(topd, topi, cand_d, cand_i, cnt, thr_s, k, nq, wid, lane, 1);
      __syncthreads();  // B: next item tile staged; merged lists and thresholds visible
      par ^= 1;
      if (!full) break;
    }
    tc0 = h1c0;
    te = h1e;
    have = have1;
    h1c0 = hNc0;
    h1e = hNe;
    have1 = haveN;
  }
  kg_merge(topd, topi, cand_d, cand_i, cnt, thr_s, k, nq, wid, lane, 1);  // the last candidates
  __syncthreads();
  if (t < nq) {
    const long base = (PAIRS ? (long)qslot[q0 + t] : q0 + t) * (long)k;
    const float add = PAIRS ? qn_s[t] : 0.f;
    for (int j = 0; j < k; ++j) {
      out_d[base + j] = topd[t][j] + add;
      out_i[base + j] = topi[t][j];
    }
  }
}
}  // namespace

// fp16 centred variant of srml_knn_lists_f32 (see above): C is the nlist x n fp32 centroid table
// (row-major, leading dimension n); out_d holds the centred fp16 partial distances
// ||i - C_c||^2 - 2 (q - C_c).(i - C_c) — a ranking key, re-ranked exactly by the caller.
// Requires n <= 128, n % 4 == 0, ld % 4 == 0, 16-byte aligned X and C, k <= 32.
SRML_API int srml_knn_lists_f16c(const float* X, int n, long ld, const float* C, const long long* list_off,
                                 const int* probes, int nprobe, const long long* tile_q0, const int* tile_list,
                                 int ntiles, int k, float* out_d, int* out_i, hipStream_t stream) {
  if (ntiles <= 0) return 0;
  if (k < 1 || k > F_KQ || n < 1 || n > F_KP || (n & 3) || (ld & 3) || nprobe < 1 || nprobe > F_PMAX ||
      (reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(C) & 15))
    return -8;
  hipLaunchKernelGGL((knn_lists_f16_kernel<false, false>), dim3((unsigned)ntiles), dim3(512), 0, stream, X, n, ld, C,
                     list_off, probes, nprobe, tile_q0, tile_list, ntiles, k, out_d, out_i, nullptr, nullptr, nullptr,
                     nullptr, nullptr, nullptr);
  return srml_status();
}

// Pre-centred fp16 items of the pair search: out[r] = fp16(X[r] - C[list of r]) (F_KP halves per
// row, zero padded), norms[r] = ||out[r]||^2 of the rounded values. 32 lanes per row, 4 columns
// each; list_off (nlist + 1) gives each sorted row's list by binary search.
__global__ __launch_bounds__(256) void center_rows_f16_kernel(const float* __restrict__ X, int n, long ld,
                                                              const float* __restrict__ C,
                                                              const long long* __restrict__ list_off, int nlist, long N,
                                                              _Float16* __restrict__ out, float* __restrict__ norms) {
  const long r = (long)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int l32 = threadIdx.x & 31;
  if (r >= N) return;  // whole 32-lane groups
  int lo = 0, hi = nlist;  // list c with list_off[c] <= r < list_off[c + 1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (list_off[mid] <= r) lo = mid;
    else hi = mid;
  }
  const int col = 4 * l32;
  typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
  halfx4 h = halfx4{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
  if (col < n) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(X + r * ld + col);
    const floatx4 c = *reinterpret_cast<const floatx4*>(C + (long)lo * n + col);
    h = halfx4{(_Float16)(x[0] - c[0]), (_Float16)(x[1] - c[1]), (_Float16)(x[2] - c[2]), (_Float16)(x[3] - c[3])};
  }
  *reinterpret_cast<halfx4*>(out + r * F_KP + col) = h;
  float a = 0.f;
  a = __builtin_amdgcn_fdot2(kg_half2{h[0], h[1]}, kg_half2{h[0], h[1]}, a, false);
  a = __builtin_amdgcn_fdot2(kg_half2{h[2], h[3]}, kg_half2{h[2], h[3]}, a, false);
  for (int o = 16; o > 0; o >>= 1) a += __shfl_xor(a, o, 32);
  if (l32 == 0) norms[r] = a;
}

SRML_API int srml_center_rows_f16(const float* X, int n, long ld, const float* C, const long long* list_off, int nlist,
                                  long N, void* out, float* norms, hipStream_t stream) {
  if (N <= 0) return 0;
  if (n < 1 || n > F_KP || (n & 3) || (ld & 3) || (reinterpret_cast<uintptr_t>(X) & 15) ||
      (reinterpret_cast<uintptr_t>(C) & 15) || (reinterpret_cast<uintptr_t>(out) & 15))
    return -8;
  hipLaunchKernelGGL(center_rows_f16_kernel, dim3((unsigned)((N + 7) / 8)), dim3(256), 0, stream, X, n, ld, C, list_off,
                     nlist, N, reinterpret_cast<_Float16*>(out), norms);
  return srml_status();
}

// Per-query probing (PAIRS mode of the kernel above): (row, probed list) pairs sorted by list,
// qrows[i] = the sorted X row of pair position i, qslot[i] = its output slot, pair_off = nlist + 1
// pair offsets per list; tiles (tile_q0 = first pair position, tile_list = list) of <= 128 pairs.
// out_d / out_i: slot-major (nslots x k): the fp16-rounded ||q - i||^2 (centred on the probed
// list's centre, comparable across one row's lists) and the sorted item positions, ascending.
// thr_row (nullable, indexed by X row): only items with a key below the row's threshold are kept
// (a slot may then hold fewer than k: +inf / -1 padding).
SRML_API int srml_knn_pairs_f16c(const float* X, int n, long ld, const float* C, const long long* list_off,
                                 const long long* pair_off, const int* qrows, const int* qslot,
                                 const long long* tile_q0, const int* tile_list, int ntiles, int k, float* out_d,
                                 int* out_i, const int* self_probe, const float* thr_row, const void* Xh,
                                 const float* xhn, hipStream_t stream) {
  if (ntiles <= 0) return 0;
  if (k < 1 || k > F_KQ || n < 1 || n > F_KP || (n & 3) || (ld & 3) || !qrows || !qslot || !pair_off ||
      !self_probe || (reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(C) & 15))
    return -8;
  // self_probe: nlist ints, self_probe[c] = c (list c scans its own items)
  if (Xh && xhn) {
    if (reinterpret_cast<uintptr_t>(Xh) & 15) return -8;
    hipLaunchKernelGGL((knn_lists_f16_kernel<true, true>), dim3((unsigned)ntiles), dim3(512), 0, stream, X, n, ld, C,
                       list_off, self_probe, 1, tile_q0, tile_list, ntiles, k, out_d, out_i, qrows, qslot, pair_off,
                       thr_row, reinterpret_cast<const _Float16*>(Xh), xhn);
  } else {
    hipLaunchKernelGGL((knn_lists_f16_kernel<true, false>), dim3((unsigned)ntiles), dim3(512), 0, stream, X, n, ld, C,
                       list_off, self_probe, 1, tile_q0, tile_list, ntiles, k, out_d, out_i, qrows, qslot, pair_off,
                       thr_row, nullptr, nullptr);
  }
  return srml_status();
}

