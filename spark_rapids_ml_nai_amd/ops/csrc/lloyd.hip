// Small-k Lloyd step on the matrix cores (k <= 32, n <= 64: the BASELINE KMeans k = 20 on
// 100M x 64) — ONE pass over X per iteration: every row's nearest centre, the per-cluster sums /
// counts by those labels and the inertia, with no host round trip between iterations.
//
// Why not the VALU kernel (kmeans.hip lloyd_small_kernel): its distances read the centres from LDS
// as broadcasts (384 ds_read_b128 per 64 rows x 24 padded centres = 1536 LDS cycles per tile,
// more than the tile's HBM time) and its one-hot sums ran on the f32 MFMA (64 cycles per
// 32x32x2): 14.8 ms per 100M x 64 iteration, ~1.7 TB/s. Here both products run on the bf16
// matrix cores over an EXACT three-way split of the fp32 operands (x = hi + mid + lo, each a
// bf16 value, by truncation: hi keeps the top 8 significand bits, mid the next 8, lo the last 8):
//   * distances D^T = C . X^T (A = centre planes, resident in LDS for the whole kernel; B = the
//     wave's staged rows): the six products of order <= 2^-16 (hh, hm, mh, hl, lh, mm; smallest
//     first), i.e. fp32-level dot products, 48 v_mfma_f32_32x32x16_bf16 per 64 rows;
//   * cluster sums S = onehot(labels)^T . X (A = one-hot, exact in bf16; B = the three planes of
//     the same staged rows, read column-wise): EXACT products accumulated in fp32, 24 MFMAs per
//     64 rows (the f32 one-hot GEMM took 64 x 64-cycle MFMAs for the same tile).
// Each lane of a tile's output holds 16 of the 32 centres of one row, so the arg-min is 16
// in-lane compares plus one exchange with lane ^ 32 (lowest index on ties, like every search).
//
// Layout: 256-thread blocks of 4 waves, persistent (2 blocks per CU, 78 KB LDS each). A wave owns
// 64-row tiles (wave-strided over the grid); tile g + W's rows are loaded lane-linearly into
// registers while tile g is computed, then written to the wave's XOR-swizzled LDS image
// (slot(r, c) = r NV + (c ^ (r & (NV - 1))): conflict-free row-fragment ds_read_b128 and
// column ds_read_b32). At the end the 4 waves' sum accumulators are added in LDS and the block
// adds its k x n partial (+ counts, inertia) into one fp64 output [sums | counts | inertia]: the
// iteration's all-reduce buffer as it stands.
//
// Delta steps (label book): the loop keeps every row's label; once few rows move per step the
// one-hot A becomes onehot(new) - onehot(old) on the moved rows (0 elsewhere), so the same GEMM
// yields the sums' change, and a wave skips it on tiles without a moved row. On uniform 100M x 64
// rows ~0.8 % of the rows keep moving (60 % of the tiles hold none): 6.2 vs 6.95 ms per step.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "common.h"

namespace {

typedef short ll_bf16x8 __attribute__((ext_vector_type(8)));

// exact 3-way split of 2 floats into packed bf16 pairs (element a low, b high)
__device__ __forceinline__ void split2(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  const unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
  const float ra = a - __uint_as_float(ua & 0xffff0000u), rb = b - __uint_as_float(ub & 0xffff0000u);
  const unsigned va = __float_as_uint(ra), vb = __float_as_uint(rb);
  const float la = ra - __uint_as_float(va & 0xffff0000u), lb = rb - __uint_as_float(vb & 0xffff0000u);
  h = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
  m = __builtin_amdgcn_perm(vb, va, 0x07060302u);
  l = __builtin_amdgcn_perm(__float_as_uint(lb), __float_as_uint(la), 0x07060302u);
}

// 8 floats -> the three bf16x8 plane fragments
__device__ __forceinline__ void split8(const float (&x)[8], ll_bf16x8& h, ll_bf16x8& m, ll_bf16x8& l) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 hh, mm, lw;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    unsigned a, b, c;
    split2(x[2 * p], x[2 * p + 1], a, b, c);
    hh[p] = a;
    mm[p] = b;
    lw[p] = c;
  }
  h = __builtin_bit_cast(ll_bf16x8, hh);
  m = __builtin_bit_cast(ll_bf16x8, mm);
  l = __builtin_bit_cast(ll_bf16x8, lw);
}

constexpr int LL_T = 256;  // threads per block (4 waves)
constexpr int LL_KP = 32;  // padded centres (one 32-row MFMA A tile)

template <int NV>
struct LloydSmem {
  static constexpr int KS = NV / 4;              // 16-wide k steps of the distance GEMM
  static constexpr int NQ = (4 * NV + 31) / 32;  // 32-column tiles of the sums
  floatx4 tile[4][64 * NV];                      // per wave: 64 rows x NV float4, swizzled
  ll_bf16x8 cpl[3][KS][64];                      // centre planes, lane-linear A fragments
  float cn[LL_KP];                               // ||c||^2 (+inf for padding centres)
  int lab[4][64];                                // per wave: the tile's labels (-1: no row)
  int lob[4][64];                                // per wave, delta step: a moved row's old label (-1: none)
  float cnt[LL_KP];                              // block counts (exact in fp32 below 2^24 rows/block)
  double in[4];
  unsigned moved;  // rows whose label changed (label book)
};

template <int NV>
__device__ __forceinline__ int slot(int r, int c) {
  return r * NV + (c ^ (r & (NV - 1)));
}

template <int NV>
__global__ __launch_bounds__(LL_T, 2) void lloyd_mfma_kernel(const float* __restrict__ X, long m, int n, long ld,
                                                             const float* __restrict__ C, int k,
                                                             const float* __restrict__ cnorm,
                                                             int* __restrict__ labels, float* __restrict__ dist,
                                                             double* __restrict__ out, const int* __restrict__ done,
                                                             const float* __restrict__ mu, int* __restrict__ book,
                                                             const int* __restrict__ mode) {
  using S = LloydSmem<NV>;
  constexpr int KS = S::KS, NQ = S::NQ;
  __shared__ S sm;
  if (done && *done) return;  // converged: the remaining launches of a batch are no-ops
  // label book: book receives every row's label. *mode != 0, a delta step: book holds the
  // previous step's labels; a row whose label changed moves its count, and the one-hot of the sums
  // GEMM becomes onehot(new) - onehot(old) on the moved rows only (0 elsewhere; +-1 exact in
  // bf16): the GEMM computes the sums' CHANGE, and runs only for the tiles that hold a moved row.
  // (The old label is loaded per 32-row half before its MFMAs: prefetching it with the tile's rows
  // measured slower, 6.3 vs 6.2 ms per 100M x 64 delta step, and cost two more registers.)
  const bool dmode = book != nullptr && mode != nullptr && *mode != 0;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  // ---- centre planes (A fragments: row = centre r32, k = 16 s + 8 hh + j) and norms
  for (int i = t; i < 3 * KS * 64; i += LL_T) {
    const int p = i / (KS * 64), s = (i / 64) % KS, l = i % 64;
    const int cj = l & 31, d0 = 16 * s + 8 * (l >> 5);
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (cj < k && d0 + j < n) ? C[(long)cj * n + d0 + j] : 0.f;
    ll_bf16x8 a, b, c;
    split8(x, a, b, c);
    sm.cpl[p][s][l] = p == 0 ? a : (p == 1 ? b : c);
  }
  if (t < LL_KP) {
    sm.cn[t] = t < k ? cnorm[t] : __builtin_huge_valf();
    sm.cnt[t] = 0.f;
  }
  if (t == 0) sm.moved = 0u;
  __syncthreads();
  float cnr[16];  // this lane half's 16 centre norms, in accumulator-register order
#pragma unroll
  for (int i = 0; i < 16; ++i) cnr[i] = sm.cn[(i & 3) + 8 * (i >> 2) + 4 * hh];
  const bool acc_sums = out != nullptr;
  floatx16 accs[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) accs[q][r] = 0.f;
  double in_sum = 0.0;
  const long tiles = (m + 63) / 64;
  const long W = (long)gridDim.x * 4;
  floatx4* tw = sm.tile[wid];
  int* slab = sm.lab[wid];
  int* slob = sm.lob[wid];
  floatx4 pre[NV];
  // mu (nullable): every staged row is x - mu (C and cnorm are then the centred centres): the
  // sums accumulate in fp32 per wave over ~50k rows, so data far from the origin would lose
  // centre precision to the fp32 accumulator; centred rows keep the sums at the data's spread.
  // A lane always stages the same 4 columns (f % NV = lane % NV: NV divides 64).
  floatx4 mu4 = floatx4{0.f, 0.f, 0.f, 0.f};
  if (mu && 4 * (lane % NV) < n) mu4 = *reinterpret_cast<const floatx4*>(mu + 4 * (lane % NV));
  auto fetch = [&](long g) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = lane + 64 * i, rr = f / NV, comp = f % NV;
      const long r = g * 64 + rr;
      pre[i] = (g < tiles && r < m && 4 * comp < n) ? *reinterpret_cast<const floatx4*>(X + r * ld + 4 * comp)
                                                    : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  };
  long g = (long)blockIdx.x * 4 + wid;
  fetch(g);
  for (; g < tiles; g += W) {
    __builtin_amdgcn_wave_barrier();  // every lane is done reading the previous tile
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = lane + 64 * i, rr = f / NV, comp = f % NV;
      tw[slot<NV>(rr, comp)] = pre[i] - mu4;  // (padding rows: -mu, never labelled or summed)
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    fetch(g + W);  // next tile's rows: in flight under this tile's MFMAs
    bool tile_moved = false;
    // ---- distances: two 32-row N tiles (rolled: the register budget holds one tile's operands)
#pragma unroll 1
    for (int nt = 0; nt < 2; ++nt) {
      const int row = 32 * nt + r32;
      // the book's label of this lane's row, loaded before the MFMAs so they cover its latency
      const int oldv = (dmode && hh == 0 && g * 64 + row < m) ? book[g * 64 + row] : -1;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      float xn = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const floatx4 v0 = tw[slot<NV>(row, 4 * s + 2 * hh)];
        const floatx4 v1 = tw[slot<NV>(row, 4 * s + 2 * hh + 1)];
        const float x[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) xn = fmaf(x[j], x[j], xn);
        ll_bf16x8 xh, xm, xl;
        split8(x, xh, xm, xl);
        const ll_bf16x8 ch = sm.cpl[0][s][lane], cm = sm.cpl[1][s][lane], cl = sm.cpl[2][s][lane];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch, xl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cl, xh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cm, xm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch, xm, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cm, xh, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ch, xh, acc, 0, 0, 0);
      }
      // arg-min over this half's 16 centres (ascending index), then across the halves
      float bv = __builtin_huge_valf();
      int bi = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float d = fmaf(-2.f, acc[i], cnr[i]);
        if (d < bv) {
          bv = d;
          bi = (i & 3) + 8 * (i >> 2) + 4 * hh;
        }
      }
      const float ov = __shfl_xor(bv, 32, 64);
      const int oi = __shfl_xor(bi, 32, 64);
      if (ov < bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
      xn += __shfl_xor(xn, 32, 64);
      const long grow = g * 64 + row;
      const bool live = grow < m;
      bool mv = false;
      int old = -1;
      if (hh == 0) {
        slab[row] = live ? bi : -1;
        slob[row] = -1;
        if (live) {
          float dd = bv + xn;
          dd = dd > 0.f ? dd : 0.f;
          if (labels) labels[grow] = bi;
          if (dist) dist[grow] = dd;
          in_sum += (double)dd;
          if (book) {
            old = oldv;
            book[grow] = bi;
          }
          mv = dmode && old != bi;
          if (acc_sums && !dmode) {
            atomicAdd(&sm.cnt[bi], 1.f);
          } else if (mv) {
            atomicAdd(&sm.cnt[bi], 1.f);
            atomicAdd(&sm.cnt[old], -1.f);
            slob[row] = old;
          } else if (dmode) {
            slab[row] = -1;  // unmoved: no change to sum
          }
        }
      }
      if (dmode) {
        const unsigned long long bal = __ballot(mv);
        if (bal) {
          tile_moved = true;
          if (lane == 0) atomicAdd(&sm.moved, (unsigned)__popcll(bal));
        }
      }
    }
    if (!acc_sums || (dmode && !tile_moved)) continue;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // ---- cluster sums: K = the tile's 64 rows in 4 steps of 16
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
      const int r0 = 16 * s + 8 * hh;
      typedef int i4 __attribute__((ext_vector_type(4)));
      const i4 la = *reinterpret_cast<const i4*>(&slab[r0]);
      const i4 lb = *reinterpret_cast<const i4*>(&slab[r0 + 4]);
      const int lv[8] = {la[0], la[1], la[2], la[3], lb[0], lb[1], lb[2], lb[3]};
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      u4 oh;
#pragma unroll
      for (int p = 0; p < 4; ++p)
        oh[p] = (lv[2 * p] == r32 ? 0x3f80u : 0u) | (lv[2 * p + 1] == r32 ? 0x3f800000u : 0u);
      if (dmode) {  // - onehot(old) of the moved rows (bf16 -1.0 = 0xbf80)
        const i4 oa = *reinterpret_cast<const i4*>(&slob[r0]);
        const i4 ob = *reinterpret_cast<const i4*>(&slob[r0 + 4]);
        const int ov[8] = {oa[0], oa[1], oa[2], oa[3], ob[0], ob[1], ob[2], ob[3]};
#pragma unroll
        for (int p = 0; p < 4; ++p)
          oh[p] |= (ov[2 * p] == r32 ? 0xbf80u : 0u) | (ov[2 * p + 1] == r32 ? 0xbf800000u : 0u);
      }
      const ll_bf16x8 a = __builtin_bit_cast(ll_bf16x8, oh);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int col = 32 * q + r32;
        float x[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rr = r0 + j;
          const float* tf = reinterpret_cast<const float*>(tw);
          x[j] = col < 4 * NV ? tf[4 * slot<NV>(rr, col >> 2) + (col & 3)] : 0.f;
        }
        ll_bf16x8 xh, xm, xl;
        split8(x, xh, xm, xl);
        accs[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xl, accs[q], 0, 0, 0);
        accs[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xm, accs[q], 0, 0, 0);
        accs[q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, xh, accs[q], 0, 0, 0);
      }
    }
  }
  // ---- block totals
  {
    double v = in_sum;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) sm.in[wid] = v;
  }
  __syncthreads();
  if (!acc_sums) return;
  const long kn = (long)k * n;
  if (t == 0) atomicAdd(&out[kn + k], (sm.in[0] + sm.in[1]) + (sm.in[2] + sm.in[3]));
  if (t == 0 && book && sm.moved) atomicAdd(&out[kn + k + 1], (double)sm.moved);
  if (t < k && sm.cnt[t] != 0.f) atomicAdd(&out[kn + t], (double)sm.cnt[t]);
  // accs[q][r] = sums[cluster (r & 3) + 8 (r >> 2) + 4 hh][column 32 q + r32]; the tile images are
  // free now: [4 waves][32 clusters][NQ * 32 columns] floats (<= 8 KB per wave)
  constexpr int RW = NQ * 32;
  float* red = reinterpret_cast<float*>(&sm.tile[0][0]);
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cl = (r & 3) + 8 * (r >> 2) + 4 * hh;
      red[(wid * 32 + cl) * RW + 32 * q + r32] = accs[q][r];
    }
  __syncthreads();
  for (int i = t; i < k * n; i += LL_T) {
    const int cl = i / n, col = i % n;
    const float v = (red[(0 * 32 + cl) * RW + col] + red[(1 * 32 + cl) * RW + col]) +
                    (red[(2 * 32 + cl) * RW + col] + red[(3 * 32 + cl) * RW + col]);
    if (v != 0.f) atomicAdd(&out[i], (double)v);
  }
}

// Centre update of the device Lloyd loop (one block): new centre = sums / counts (empty clusters
// keep theirs), the largest squared shift, convergence flag; fp32 copy + norms for the next
// search. Skips once flags[0] (done) is set. stat: [inertia of the last step, last max shift].
// With a label book (G non-null): buf = [sums | counts | inertia | moved] of this step, a full
// step's (flags[2] == 0) or a delta step's (1) change; G (k n + k) = the running sums / counts
// (G = buf or G += buf); the next step is a delta step when fewer than 1/4 of all ranks' rows
// moved in this one (a full step counts none). A full step cannot count moved rows without
// reading the book, which costs more (+0.6 ms per 100M rows) than a delta step saves early on.
__global__ __launch_bounds__(256) void kmeans_small_update_kernel(const double* __restrict__ buf, int k, int n,
                                                                   double* __restrict__ C64, float* __restrict__ C32,
                                                                   float* __restrict__ cnorm, double tol2,
                                                                   int* __restrict__ flags, double* __restrict__ stat,
                                                                   double* __restrict__ G) {
  if (flags[0]) return;
  __shared__ double shift[LL_KP];
  const int t = threadIdx.x;
  const long kn = (long)k * n;
  if (G) {
    const bool delta = flags[2] == 1;
    for (long i = t; i < kn + k; i += 256) G[i] = delta ? G[i] + buf[i] : buf[i];
    __syncthreads();
  }
  const double* sums = G ? G : buf;
  for (int j = t >> 3; j < k; j += 32) {  // 8 threads per centre
    const double cnt = sums[kn + j];
    double sh = 0.0;
    float nn = 0.f;
    for (int d = t & 7; d < n; d += 8) {
      const double old = C64[(long)j * n + d];
      const double nw = cnt > 0.0 ? sums[(long)j * n + d] / cnt : old;
      sh += (nw - old) * (nw - old);
      C64[(long)j * n + d] = nw;
      const float f = (float)nw;
      C32[(long)j * n + d] = f;
      nn = fmaf(f, f, nn);
    }
    for (int o = 4; o > 0; o >>= 1) {
      sh += __shfl_xor(sh, o, 8);
      nn += __shfl_xor(nn, o, 8);
    }
    if ((t & 7) == 0) {
      shift[j] = sh;
      cnorm[j] = nn;
    }
  }
  __syncthreads();
  if (t == 0) {
    double mx = 0.0;
    for (int j = 0; j < k; ++j) mx = shift[j] > mx ? shift[j] : mx;
    stat[0] = buf[kn + k];
    stat[1] = mx;
    flags[1] += 1;
    if (mx <= tol2) flags[0] = 1;
    if (G) {
      double m_total = 0.0;  // every rank's rows: the reduced running counts
      for (int j = 0; j < k; ++j) m_total += G[kn + j];
      flags[2] = buf[kn + k + 1] * 4.0 < m_total ? 1 : 0;
    }
  }
}

}  // namespace

// Small-k Lloyd step on the bf16 matrix cores (see above). mu (nullable, n floats, 16-B aligned):
// search / sum the rows x - mu against centres C given already centred (C - mu, their norms); the
// sums are then of x - mu. out == nullptr: search only (labels / squared distances). Otherwise
// out = [k x n sums | k counts | inertia] (fp64, zeroed by the caller) accumulates this launch;
// labels / dist may then be nullptr (not written: the Lloyd loop needs neither). done (nullable):
// a device flag; non-zero = return at once.
// Label book (book non-null, out needs k n + k + 2 doubles): book (m int32) receives every row's
// label, out[k n + k + 1] the rows whose label changed; when *mode != 0 the step is a delta step:
// out gets the sums' and counts' CHANGE (the rows whose label differs from book's).
// Needs k <= 32, n <= 64, n % 4 == 0, ld % 4 == 0, 16-B aligned X.
SRML_API int srml_kmeans_lloyd_mfma(const float* X, long m, int n, long ld, const float* C, int k,
                                    const float* cnorm, int* labels, float* dist, double* out, const int* done,
                                    const float* mu, int* book, const int* mode, hipStream_t stream) {
  if (m <= 0) return 0;
  if (k < 1 || k > LL_KP || n < 1 || n > 64 || (n & 3) || (ld & 3) || (reinterpret_cast<uintptr_t>(X) & 15) ||
      (reinterpret_cast<uintptr_t>(mu) & 15) ||
      (book && (!out || !mode)))
    return (int)hipErrorInvalidValue;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const long tiles = (m + 63) / 64;
  const long want = (tiles + 3) / 4;  // 4 waves (tiles in flight) per block
  const unsigned grid = (unsigned)(want < 2L * cus ? want : 2L * cus);
#define SRML_LL(NV)                                                                                                   \
  hipLaunchKernelGGL((lloyd_mfma_kernel<NV>), dim3(grid), dim3(LL_T), 0, stream, X, m, n, ld, C, k, cnorm, labels, \
                     dist, out, done, mu, book, mode)
  if (n <= 16) SRML_LL(4);
  else if (n <= 32) SRML_LL(8);
  else SRML_LL(16);
#undef SRML_LL
  return srml_status();
}

// One centre update of the device Lloyd loop (see kmeans_small_update_kernel). flags = [done,
// iterations, delta mode]; stat = [inertia, max shift] of the last update that ran. G (nullable):
// the label book's running sums / counts.
SRML_API int srml_kmeans_small_update(const double* buf, int k, int n, double* C64, float* C32, float* cnorm,
                                      double tol2, int* flags, double* stat, double* G, hipStream_t stream) {
  if (k < 1 || k > LL_KP || n < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kmeans_small_update_kernel, dim3(1), dim3(256), 0, stream, buf, k, n, C64, C32, cnorm, tol2, flags,
                     stat, G);
  return srml_status();
}
