// Split-bf16 ("bf16x6") fp32-exact distance GEMM for the large-k nearest-centroid search.
//
// gfx950 has no xf32 MFMA: fp32-input MFMA (`v_mfma_f32_32x32x2_f32`) runs at 1/16 of the bf16
// rate (64 vs 1024 FLOP/clk/SIMD). The KMeans distance GEMM (m x n . n x k, e.g. the reference
// headline 1M x 3000 x 1000 per Lloyd iteration, reference cuML KMeansMG / RAFT fusedL2NN) is
// therefore re-expressed on the bf16 matrix cores without giving up fp32 accuracy:
//
//   x = x_h + x_m + x_l   (three bf16 pieces, each the round-to-nearest bf16 of the remaining
//                          fp32 residual; 3 x 8 significant bits = the 24 of fp32, so the split
//                          is exact for normal numbers)
//   x.c ~= h.h + h.m + m.h + h.l + m.m + l.h     (every product of relative weight >= 2^-16)
//
// The dropped products (m.l, l.m, l.l) are <= 2^-24 relative, i.e. below fp32 rounding, and
// each bf16 x bf16 product is exact in the fp32 MFMA accumulator: the result has the accuracy
// of an fp32 FMA dot product at 6/16 of the fp32 MFMA cost.
//
//  * srml_split_bf16x3: X (m x n fp32, ld) -> planes P[3][rows_pad][kp] bf16 (kp = n rounded up
//    to 16, zero padded; rows >= m zero). One pass, 16-B stores.
//  * srml_nearest_centroid_split: packed (dist, index) arg-min of ||c||^2 - 2 x.c over the
//    centroids, the same 64-bit atomicMin contract as srml_nearest_centroid_f32 (kmeans.hip).
//    Block tile 128 rows x 128 centroids, 4 waves as 2 x 2, each wave 2 x 2 tiles of
//    `v_mfma_f32_32x32x16_bf16`; per 16-wide k step the block stages 6 plane tiles (X and C,
//    h/m/l) in LDS (rows padded to 48 B: the 16-B fragment reads of 16 consecutive lanes hit 16
//    distinct 4-bank groups), double-buffered with register prefetch so the next k step's
//    global loads are in flight under the current 24 MFMAs per wave. Grid is 1-D, centroid tile
//    fastest and XCD-remapped so the blocks sharing one X row tile run on one XCD's L2.
#include "common.h"

#include "tile.h"
#include <stdlib.h>

namespace {
using srml_tile::orderable;
using srml_tile::unorderable;

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
typedef unsigned uintx2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned bf16_rn(float f) {  // round-to-nearest-even (finite inputs)
  unsigned u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__device__ __forceinline__ float bf16_f(unsigned b) { return __uint_as_float(b << 16); }

// 4 consecutive elements per thread -> three 8-byte plane stores
__global__ __launch_bounds__(256) void split_kernel(const float* __restrict__ X, long m, int n, long ld, int kp,
                                                    long rows_pad, unsigned short* __restrict__ P) {
  const int q4 = kp >> 2;
  const long total = rows_pad * q4;
  const long plane = rows_pad * (long)kp;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long r = i / q4;
    const int c = (int)(i - r * q4) * 4;
    unsigned h[4], md[4], lo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = (r < m && c + j < n) ? X[r * ld + c + j] : 0.f;
      h[j] = bf16_rn(x);
      const float r1 = x - bf16_f(h[j]);
      md[j] = bf16_rn(r1);
      lo[j] = bf16_rn(r1 - bf16_f(md[j]));
    }
    const long o = r * kp + c;
    *reinterpret_cast<uintx2*>(P + o) = uintx2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
    *reinterpret_cast<uintx2*>(P + plane + o) = uintx2{md[0] | (md[1] << 16), md[2] | (md[3] << 16)};
    *reinterpret_cast<uintx2*>(P + 2 * plane + o) = uintx2{lo[0] | (lo[1] << 16), lo[2] | (lo[3] << 16)};
  }
}

// Tiled + swizzled plane layout for the LDS-DMA kernel: P[3][rows_pad / 256][kp / 16][256][16],
// i.e. every (256-row tile, 16-wide k step) block of a plane is one contiguous 8 KiB image, with
// row r's 16-B half h stored at half h ^ ((r >> 3) & 1) (the bank-conflict-free fragment image).
// A k step of a tile is then streamed with fully sequential 1 KiB LDS-DMA wave loads (every
// 128-B line used whole) instead of 32-B pieces of 256 rows 6 KB apart.
__global__ __launch_bounds__(256) void split_tiled_kernel(const float* __restrict__ X, long m, int n, long ld, int kp,
                                                          long rows_pad, unsigned short* __restrict__ P,
                                                          const float* __restrict__ mu,
                                                          const int* __restrict__ ridx = nullptr) {
  // one thread = one row's 16-wide k step (64 B of X in, one 32-B slot per plane out); a block =
  // the 256 rows of one (tile, k step) image, so each block writes three contiguous 8 KiB images
  const int ks_n = kp >> 4;
  const long total = rows_pad * ks_n;
  const long plane = rows_pad * (long)kp;
  const bool vec = (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long img = i >> 8;  // = tile * ks_n + ks
    const int rr = (int)(i & 255);
    const long tile = img / ks_n;
    const int c0 = (int)(img - tile * ks_n) * 16;
    const long r = tile * 256 + rr;
    const long rs = ridx && r < m ? (long)ridx[r] : r;  // gathered rows (the filter's re-search list)
    float x[16];
    if (vec && r < m && c0 + 16 <= n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(X + rs * ld + c0 + 4 * q);
        x[4 * q] = v[0]; x[4 * q + 1] = v[1]; x[4 * q + 2] = v[2]; x[4 * q + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = (r < m && c0 + j < n) ? X[rs * ld + c0 + j] : 0.f;
    }
    if (mu && r < m) {  // centred planes (x - mu): same distances, smaller operands
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (c0 + j < n) x[j] -= mu[c0 + j];
    }
    unsigned hw[8], mw[8], lw[8];
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      unsigned h2[2], m2[2], l2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        h2[u] = bf16_rn(x[j + u]);
        const float r1 = x[j + u] - bf16_f(h2[u]);
        m2[u] = bf16_rn(r1);
        l2[u] = bf16_rn(r1 - bf16_f(m2[u]));
      }
      hw[j / 2] = h2[0] | (h2[1] << 16);
      mw[j / 2] = m2[0] | (m2[1] << 16);
      lw[j / 2] = l2[0] | (l2[1] << 16);
    }
    const int sw = (rr >> 3) & 1;  // logical half h lands at physical half h ^ sw
    unsigned short* o = P + (img << 12) + rr * 16;
    const unsigned* W[3] = {hw, mw, lw};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      uintx4* d = reinterpret_cast<uintx4*>(o + p * plane);
      d[sw] = uintx4{W[p][0], W[p][1], W[p][2], W[p][3]};
      d[sw ^ 1] = uintx4{W[p][4], W[p][5], W[p][6], W[p][7]};
    }
  }
}

// One fp16 plane of s (x - mu) in the same tiled, swizzled image layout (the fp16 certified
// filter, srml_nearest_centroid_f16_top2): s is a power of two chosen by the caller from
// max |x - mu| so the largest element lands in [2^13, 2^14) (headroom for centroids, which are
// convex combinations of rows); an element with |s v| >= 2^15 (a centroid outside the data's
// range) sets *ovf, and the select phase then re-searches every row exactly.
__global__ __launch_bounds__(256) void split_tiled_f16_kernel(const float* __restrict__ X, long m, int n, long ld, int kp,
                                                              long rows_pad, unsigned short* __restrict__ P,
                                                              const float* __restrict__ mu, float scale,
                                                              int* __restrict__ ovf, const int* __restrict__ ridx = nullptr) {
  const int ks_n = kp >> 4;
  const long total = rows_pad * ks_n;
  const bool vec = (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  bool over = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long img = i >> 8;
    const int rr = (int)(i & 255);
    const long tile = img / ks_n;
    const int c0 = (int)(img - tile * ks_n) * 16;
    const long r = tile * 256 + rr;
    const long rs = ridx && r < m ? (long)ridx[r] : r;
    float x[16];
    if (vec && r < m && c0 + 16 <= n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 v = *reinterpret_cast<const floatx4*>(X + rs * ld + c0 + 4 * q);
        x[4 * q] = v[0]; x[4 * q + 1] = v[1]; x[4 * q + 2] = v[2]; x[4 * q + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = (r < m && c0 + j < n) ? X[rs * ld + c0 + j] : 0.f;
    }
    unsigned hw[8];
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      unsigned h2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float v = x[j + u];
        if (mu && r < m && c0 + j + u < n) v -= mu[c0 + j + u];  // the same fp32 x - mu as the exact search
        v *= scale;                                             // power of two: exact
        if (fabsf(v) >= 32768.f) { over = true; v = v > 0.f ? 32768.f : -32768.f; }
        const _Float16 hv = (_Float16)v;                        // round to nearest even
        h2[u] = (unsigned)__builtin_bit_cast(unsigned short, hv);
      }
      hw[j / 2] = h2[0] | (h2[1] << 16);
    }
    const int sw = (rr >> 3) & 1;
    uintx4* d = reinterpret_cast<uintx4*>(P + (img << 12) + rr * 16);
    d[sw] = uintx4{hw[0], hw[1], hw[2], hw[3]};
    d[sw ^ 1] = uintx4{hw[4], hw[5], hw[6], hw[7]};
  }
  if (over) atomicOr(ovf, 1);
}

constexpr int SBK = 16;
constexpr int ROWB = 24;  // padded LDS row: 16 bf16 + 8 pad = 48 B

// BM x BN block tile, WM x WN waves, each wave (BM/WM) x (BN/WN) = TM x TN tiles of 32x32.
// Staging: thread t owns row (t >> 1), 16-byte half (t & 1) of every plane tile, so
// BM == BN == 2 * threads (both configs below).
template <int BM, int BN, int WM, int WN>
struct SplitCfg {
  static constexpr int NT = WM * WN * 64;
  static constexpr int TM = BM / WM / 32;
  static constexpr int TN = BN / WN / 32;
  static_assert(BM == NT / 2 && BN == NT / 2, "staging assumes one A row and one B row per thread pair");
};

// Fused arg-min epilogue shared by the split kernels: d = ||c||^2 - 2 x.c per accumulator element,
// row-wise arg-min over the wave's columns, then one packed 64-bit atomicMin per row.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void split_epilogue(const floatx16 (&acc)[BM / WM / 32][BN / WN / 32], long row0, int col0,
                                               long m, int k, const float* __restrict__ cnorm,
                                               unsigned long long* __restrict__ best, int wm, int wn, int li, int lk) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  // C/D layout of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5))
  float cn[TN];
  int cj[TN];
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) {
    cj[nt] = col0 + wn * (BN / WN) + nt * 32 + li;
    cn[nt] = (cj[nt] < k) ? cnorm[cj[nt]] : 0.f;
  }
#pragma unroll
  for (int mt = 0; mt < TM; ++mt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float bv = __builtin_huge_valf();
      int bi = 0x7fffffff;
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
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
      if (li == 0 && bi != 0x7fffffff) {
        const long row = row0 + wm * (BM / WM) + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < m) {
          const unsigned long long key = ((unsigned long long)orderable(bv) << 32) | (unsigned)bi;
          atomicMin(&best[row], key);
        }
      }
    }
  }
}

// One merge step of the (best value, best index, best's lower bound, others' lower bound) state
// with the state DPP-moved from another lane; lanes the DPP pattern does not write receive the
// identity (+inf, INT_MAX, +inf, +inf) and keep their state.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void top2_merge_dpp(float& bv, int& bi, float& badj, float& sadj) {
  const float inf = __builtin_huge_valf();
  const float ov = __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(inf), __float_as_int(bv), CTRL, ROW_MASK, 0xf, false));
  const int oi = __builtin_amdgcn_update_dpp(0x7fffffff, bi, CTRL, ROW_MASK, 0xf, false);
  const float oadj = __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(inf), __float_as_int(badj), CTRL, ROW_MASK, 0xf, false));
  const float osadj = __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(inf), __float_as_int(sadj), CTRL, ROW_MASK, 0xf, false));
  if (ov < bv || (ov == bv && oi < bi)) {
    sadj = fminf(fminf(sadj, badj), osadj);
    bv = ov;
    bi = oi;
    badj = oadj;
  } else {
    sadj = fminf(fminf(sadj, oadj), osadj);
  }
}

// Top-2 epilogue for the certified 3-product search. Each candidate j carries an error radius
// e_j = sqrt(||x||^2) * g_j (g_j = 2 tau ||c_j||, the bound on |d~_j - d_j| of the dropped
// products); per (row, wave column slot) it keeps the best (d~, index) and the smallest LOWER
// bound d~_j - e_j over the slot's other candidates, plain stores into keys / lob[slot * m + row]
// (slot = ctile * WN + wn, slot-major: [slot][row]); srml_split_top2_select merges the slots.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void split_epilogue_top2(const floatx16 (&acc)[BM / WM / 32][BN / WN / 32], long row0,
                                                    int col0, int ctile, long m, int k,
                                                    const float* __restrict__ cnorm, const float* __restrict__ cg,
                                                    const float* __restrict__ xnorm,
                                                    unsigned long long* __restrict__ keys, float* __restrict__ lob,
                                                    int nslot, int wm, int wn, int li, int lk, float dscale,
                                                    float xadd) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  float cn[TN], g[TN];
  int cj[TN];
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) {
    cj[nt] = col0 + wn * (BN / WN) + nt * 32 + li;
    cn[nt] = (cj[nt] < k) ? cnorm[cj[nt]] : 0.f;
    g[nt] = (cj[nt] < k) ? cg[cj[nt]] : 0.f;
  }
  const int slot = ctile * WN + wn;
#pragma unroll
  for (int mt = 0; mt < TM; ++mt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long row = row0 + wm * (BM / WM) + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
      const float xs = row < m ? sqrtf(fmaxf(xnorm[row], 0.f)) + xadd : 0.f;
      float bv = __builtin_huge_valf(), badj = __builtin_huge_valf(), sadj = __builtin_huge_valf();
      int bi = 0x7fffffff;
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        if (cj[nt] < k) {
          const float d = fmaf(dscale, acc[mt][nt][r], cn[nt]);
          const float adj = fmaf(-xs, g[nt], d);
          if (d < bv) { sadj = fminf(sadj, badj); bv = d; bi = cj[nt]; badj = adj; }
          else sadj = fminf(sadj, adj);
        }
      }
      // 32-lane merge on DPP (no LDS round trips): quad_perm xor 1 / xor 2, row_half_mirror and
      // row_mirror leave every lane with its 16-lane row's state, row_bcast:15 folds row 0 into
      // row 1 (and row 2 into row 3); lane 31 / 63 then holds the 32-lane result of its lk half
      top2_merge_dpp<0xb1, 0xf>(bv, bi, badj, sadj);
      top2_merge_dpp<0x4e, 0xf>(bv, bi, badj, sadj);
      top2_merge_dpp<0x141, 0xf>(bv, bi, badj, sadj);
      top2_merge_dpp<0x140, 0xf>(bv, bi, badj, sadj);
      top2_merge_dpp<0x142, 0xa>(bv, bi, badj, sadj);
      if (li == 31 && row < m) {
        const long o = (long)slot * m + row;  // slot-major: the select kernel reads rows coalesced
        keys[o] = bi == 0x7fffffff ? ~0ull : (((unsigned long long)orderable(bv) << 32) | (unsigned)bi);
        lob[o] = sadj;
      }
    }
  }
}

// Top-2 epilogue on TRANSPOSED accumulators (acc[mt][nt] = centres x rows: lane (li, lk) holds row
// row0 + wm (BM / WM) + 32 mt + li against centres col0 + wn (BN / WN) + 32 nt + (r & 3) + 8 (r >> 2)
// + 4 lk): same state and output as split_epilogue_top2, but each lane scans its 2 x 16 candidates
// in registers and only the two lk halves are merged (one cross-half exchange per row instead of
// five DPP merges of four values per (row, register)).
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void split_epilogue_top2_t(const floatx16 (&acc)[BM / WM / 32][BN / WN / 32], long row0,
                                                      int col0, int ctile, long m, int k,
                                                      const float* __restrict__ cnorm, const float* __restrict__ cg,
                                                      const float* __restrict__ xnorm,
                                                      unsigned long long* __restrict__ keys, float* __restrict__ lob,
                                                      int nslot, int wm, int wn, int li, int lk, float dscale,
                                                      float xadd) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  // per-row state of the wave's TM rows of this lane; the centre tiles are scanned nt-outer (one
  // tile's 16 norms / radii live at a time: TN = 4 tiles would need 128 more VGPRs), j ascending
  // per lane either way, so ties keep the lower index
  float bv[TM], badj[TM], sadj[TM], xs[TM];
  int bi[TM];
#pragma unroll
  for (int mt = 0; mt < TM; ++mt) {
    const long row = row0 + wm * (BM / WM) + mt * 32 + li;
    xs[mt] = row < m ? sqrtf(fmaxf(xnorm[row], 0.f)) + xadd : 0.f;
    bv[mt] = badj[mt] = sadj[mt] = __builtin_huge_valf();
    bi[mt] = 0x7fffffff;
  }
#pragma unroll
  for (int nt = 0; nt < TN; ++nt) {
    float cn[16], g[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = col0 + wn * (BN / WN) + nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
      cn[r] = j < k ? cnorm[j] : __builtin_huge_valf();  // +inf: never the best, never a bound
      g[r] = j < k ? cg[j] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < TM; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = fmaf(dscale, acc[mt][nt][r], cn[r]);
        const float adj = fmaf(-xs[mt], g[r], d);
        const int j = col0 + wn * (BN / WN) + nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (d < bv[mt]) { sadj[mt] = fminf(sadj[mt], badj[mt]); bv[mt] = d; bi[mt] = j; badj[mt] = adj; }
        else sadj[mt] = fminf(sadj[mt], adj);
      }
  }
  const int slot = ctile * WN + wn;
#pragma unroll
  for (int mt = 0; mt < TM; ++mt) {
    const long row = row0 + wm * (BM / WM) + mt * 32 + li;
    float b = bv[mt], ba = badj[mt], sa = sadj[mt];
    int bj = bi[mt];
    // merge with the other lk half (lane ^ 32: the same row, the other 16 centres of each tile)
    const float ov = __shfl_xor(b, 32, 64);
    const int oi = __shfl_xor(bj, 32, 64);
    const float oadj = __shfl_xor(ba, 32, 64);
    const float osadj = __shfl_xor(sa, 32, 64);
    if (ov < b || (ov == b && oi < bj)) {
      sa = fminf(fminf(sa, ba), osadj);
      b = ov;
      bj = oi;
      ba = oadj;
    } else {
      sa = fminf(fminf(sa, oadj), osadj);
    }
    if (lk == 0 && row < m) {
      const long o = (long)slot * m + row;
      const bool none = bj == 0x7fffffff || !(b < __builtin_huge_valf());
      keys[o] = none ? ~0ull : (((unsigned long long)orderable(b) << 32) | (unsigned)bj);
      lob[o] = sa;
    }
  }
}

// Candidate epilogue of the fp16 re-search pass (transposed accumulators as split_epilogue_top2_t):
// every centre j whose lower bound d~_j - (||x|| + xadd) g_j is <= thr[row] (the row's certified upper
// bound on the best distance from the filter pass) is appended to the row's list (cap entries; the
// count keeps growing past cap so the exact pass can tell an overflow)
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void split_epilogue_cand_t(const floatx16 (&acc)[BM / WM / 32][BN / WN / 32], long row0,
                                                      int col0, long m, int k, const float* __restrict__ cnorm,
                                                      const float* __restrict__ cg, const float* __restrict__ xnorm,
                                                      int wm, int wn, int li, int lk, float dscale, float xadd,
                                                      const float* __restrict__ thr, int* __restrict__ ccount,
                                                      int* __restrict__ cand, int cap) {
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
#pragma unroll
  for (int mt = 0; mt < TM; ++mt) {
    const long row = row0 + wm * (BM / WM) + mt * 32 + li;
    if (row >= m) continue;
    const float xs = sqrtf(fmaxf(xnorm[row], 0.f)) + xadd;
    const float t = thr[row];
#pragma unroll
    for (int nt = 0; nt < TN; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = col0 + wn * (BN / WN) + nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (j < k) {
          const float d = fmaf(dscale, acc[mt][nt][r], cnorm[j]);
          if (fmaf(-xs, cg[j], d) <= t) {
            const int p = atomicAdd(&ccount[row], 1);
            if (p < cap) cand[row * (long)cap + p] = j;
          }
        }
      }
  }
}

template <int BM, int BN>
struct SplitStage {
  unsigned short A[3][BM][ROWB];
  unsigned short B[3][BN][ROWB];
};

template <int BM, int BN, int WM, int WN, int MINB, int PF>
__global__ __launch_bounds__(WM * WN * 64, MINB) void nearest_centroid_split_kernel(
    const unsigned short* __restrict__ XP, long m, long xrows, int kp, const unsigned short* __restrict__ CP, int k,
    long crows, const float* __restrict__ cnorm, unsigned long long* __restrict__ best, int n_ctiles) {
  using Cfg = SplitCfg<BM, BN, WM, WN>;
  constexpr int TM = Cfg::TM, TN = Cfg::TN;
  __shared__ SplitStage<BM, BN> st[2];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const long rtile = bid / n_ctiles;
  const int ctile = bid % n_ctiles;
  const long row0 = rtile * BM;
  const int col0 = ctile * BN;
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int li = lane & 31, lk = lane >> 5;

  const int sr = t >> 1, sh = (t & 1) * 8;
  long xr = row0 + sr;
  if (xr >= xrows) xr = xrows - 1;  // clamp: those rows are never reported
  const long xplane = xrows * (long)kp, cplane = crows * (long)kp;
  const unsigned short* xa = XP + xr * kp + sh;
  const unsigned short* ca = CP + (long)(col0 + sr) * kp + sh;  // crows is a multiple of BN

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // One 16-wide k step of MFMAs on LDS stage `cur` (smallest terms first: l.h, m.m, h.l, m.h, h.m, h.h).
  auto mma_step = [&](int cur) {
    bf16x8 fb[3][TN];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int nt = 0; nt < TN; ++nt)
        fb[p][nt] = *reinterpret_cast<const bf16x8*>(&st[cur].B[p][wn * (BN / WN) + nt * 32 + li][8 * lk]);
#pragma unroll
    for (int mt = 0; mt < TM; ++mt) {
      bf16x8 fa[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        fa[p] = *reinterpret_cast<const bf16x8*>(&st[cur].A[p][wm * (BM / WM) + mt * 32 + li][8 * lk]);
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0][nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1][nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2][nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0][nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1][nt], acc[mt][nt], 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0][nt], acc[mt][nt], 0, 0, 0);
      }
    }
  };
  auto gload = [&](int kt, uintx4 (&a)[3], uintx4 (&b)[3]) {
    const long ko = (long)kt * SBK;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      a[p] = *reinterpret_cast<const uintx4*>(xa + p * xplane + ko);
      b[p] = *reinterpret_cast<const uintx4*>(ca + p * cplane + ko);
    }
  };
  auto lstore = [&](int stage, const uintx4 (&a)[3], const uintx4 (&b)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      *reinterpret_cast<uintx4*>(&st[stage].A[p][sr][sh]) = a[p];
      *reinterpret_cast<uintx4*>(&st[stage].B[p][sr][sh]) = b[p];
    }
  };
  const int nk = kp / SBK;
  if (PF == 1) {
    uintx4 ra[3], rb[3];
    gload(0, ra, rb);
    lstore(0, ra, rb);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) gload(kt + 1, ra, rb);
      mma_step(cur);
      if (more) lstore(cur ^ 1, ra, rb);
      __syncthreads();
      cur ^= 1;
    }
  } else {
    // global loads run two k steps ahead (two register sets): the L2/HBM latency of a step's
    // operands is covered by two steps of MFMAs instead of one
    uintx4 ra0[3], rb0[3], ra1[3], rb1[3];
    gload(0, ra0, rb0);
    if (nk > 1) gload(1, ra1, rb1);
    lstore(0, ra0, rb0);
    __syncthreads();
    int kt = 0;
    for (; kt + 2 <= nk; kt += 2) {
      // step kt on stage 0; data of kt+1 sits in set 1; set 0 is refilled with kt+2
      if (kt + 2 < nk) gload(kt + 2, ra0, rb0);
      mma_step(0);
      lstore(1, ra1, rb1);
      __syncthreads();
      // step kt+1 on stage 1; data of kt+2 sits in set 0; set 1 is refilled with kt+3
      if (kt + 3 < nk) gload(kt + 3, ra1, rb1);
      mma_step(1);
      if (kt + 2 < nk) lstore(0, ra0, rb0);
      __syncthreads();
    }
    if (kt < nk) mma_step(0);  // odd step count: the last step's data is already in stage 0
  }

  split_epilogue<BM, BN, WM, WN>(acc, row0, col0, m, k, cnorm, best, wm, wn, li, lk);
}

// ------------------------------------------------------------------------------------------
// LDS-DMA variant (BM = BN = 256, 8 waves as 2 x 4): operand tiles go global -> LDS with
// `global_load_lds_dwordx4` (no VGPR staging, no ds_write pass) into a 3-stage ring of unpadded
// 32-B rows (3 stages x 6 planes x 256 x 32 B = 144 KiB), two k steps in flight across each raw
// barrier with a counted vmcnt. One LDS-DMA wave-instruction writes 1 KiB lane-linearly (32 rows x
// 32 B), so the bank-conflict swizzle (16-B half h of row r stored at half h ^ ((r >> 3) & 1))
// is applied on the per-lane SOURCE address and undone on the fragment read
// (cdna_hip_programming.md §5 "Async global->LDS copy", rule 21).
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* gbl_vptr;

// TILED: operands in the split_tiled_kernel layout (contiguous, pre-swizzled 8 KiB k-step images).
// NP = 6: the fp32-exact product set; NP = 3: h.h + h.m + m.h only (~2^-16 relative, half the
// MFMAs) for consumers that only need approximate distances (k-means|| D^2 sampling / weighting).
// WN_ = 4: 256 x 256 block tile, 8 waves, one block per CU. WN_ = 2 (3-product only): 256 x 128
// block tile, 4 waves (one per SIMD) and a 3-stage 72 KiB ring, so TWO blocks share a CU: each
// SIMD runs two waves of independent blocks whose barriers and LDS-DMA waits fall at different
// times (the 8-wave block parks all its waves at every barrier together). Same per-wave 128 x 64
// tile and fragment reads; C rows of a 128-wide tile are the first / second half of the 256-row
// tiled image.
// PRIO: s_setprio(1) / (0) around every MFMA cluster: keeps hipcc from moving MFMAs across the
// raw barriers into the load phase (cdna_hip_programming.md T5).
template <bool TILED, int NP = 6, bool TOP2 = false, int WN_ = 4, bool PRIO = false, bool CAND = false, int RING = 0>
__global__ __launch_bounds__(WN_ * 128, WN_ == 4 ? 1 : 2) void nearest_centroid_split_glds_kernel(
    const unsigned short* __restrict__ XP, long m, long xrows, int kp, const unsigned short* __restrict__ CP, int k,
    long crows, const float* __restrict__ cnorm, unsigned long long* __restrict__ best, int n_ctiles,
    float* __restrict__ lob = nullptr, const float* __restrict__ cg = nullptr, const float* __restrict__ xnorm = nullptr,
    float dscale = -2.f, float xadd = 0.f, const float* __restrict__ thr = nullptr, int* __restrict__ ccount = nullptr,
    int* __restrict__ cand = nullptr, int cap = 0) {
  static_assert(!CAND || (NP == 1 && TOP2), "candidate lists come from the fp16 filter");
  static_assert(WN_ == 4 || (WN_ == 2 && NP != 6), "256 x 128 tiles are built for the filter passes");
  static_assert(NP == 6 || NP == 3 || (NP == 1 && TOP2), "NP = 1 is the fp16 certified filter");
  // (128 x 128 wave tiles for the fp16 filter — 4 waves of 16 accumulator tiles, 8 fragment reads
  // per 16 MFMAs — measured 7.8 vs 7.15 ms at 1M x 3000 x 1000: one wave per SIMD exposes every
  // barrier and DMA wait; the 8-wave 128 x 64 layout stays)
  constexpr int BM = 256, WM = 2, WN = WN_, BN = 64 * WN, TM = 4, TN = 2;
  // planes staged per operand: h, m, l for the 6-product set; the 3-product set (h.h, h.m, m.h)
  // never touches the l planes, so it stages 2 per operand (2/3 of the DMA and LDS traffic)
  constexpr int NPL = NP == 6 ? 3 : (NP == 3 ? 2 : 1);
  constexpr int XCH = NPL * (BM / 32), CCH = NPL * (BN / 32);  // 1 KiB staging chunks per stage
  constexpr int CPW = (XCH + CCH) / (WM * WN);                  // ... per wave
  static_assert((XCH + CCH) % (WM * WN) == 0, "chunks split evenly over the waves");
  // ring depth: a 3-product k step is half the MFMA time of a 6-product one, so the 8-wave block's
  // loads get one more step of lead (4 stages x 32 KiB = 128 KiB; the 6-product ring is 3 x 48 KiB);
  // the 4-wave block keeps 3 stages (3 x 24 KiB) so two blocks fit a CU
  // NP = 1 (one fp16 plane per operand, 16 KiB stages): a k step is a third of a 3-product one,
  // so three steps share a barrier and the ring holds three such groups (9 stages, 144 KiB): the
  // loads of group g + 2 are issued while group g computes (two groups of HBM-latency cover)
  // RING (fp16 filter probes, SRML_F16_RING): 10 * KPB + NG overrides the defaults below
  constexpr int KPB = RING ? RING / 10 : NP == 1 ? 3 : (NP == 3 && WN_ == 4 ? 2 : 1);  // k steps per barrier
  constexpr int NG = RING ? RING % 10 : NP == 1 && WN_ == 4 ? 3 : 2;  // groups in the ring (2 x 72 KiB per CU at WN_ = 2)
  static_assert(!RING || (NP == 1 && KPB >= 1 && NG >= 2), "ring override is for the fp16 filter");
  constexpr int NS = (KPB > 1 || RING) ? NG * KPB : 3;
  constexpr int STAGE = NPL * (BM + BN) * 16;  // elements: X planes [NPL][BM][16], then C planes [NPL][BN][16]
  __shared__ __attribute__((aligned(1024))) unsigned short lds[NS][STAGE];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const long rtile = bid / n_ctiles;
  const int ctile = bid % n_ctiles;
  const long row0 = rtile * BM;
  const int col0 = ctile * BN;
  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int li = lane & 31, lk = lane >> 5;
  const long xplane = xrows * (long)kp, cplane = crows * (long)kp;

  // this wave's CPW staging chunks per stage: chunk c = wid * CPW + i -> X plane c / 8 (rows
  // 32 (c % 8) ..) for c < XCH, else C plane (c - XCH) / (BN / 32)
  const unsigned short* src[CPW];
  int dst_off[CPW];  // element offset of the chunk inside one stage
#pragma unroll
  for (int i = 0; i < CPW; ++i) {
    const int c = wid * CPW + i;
    const bool isx = c < XCH;
    const int q = isx ? c / (BM / 32) : (c - XCH) / (BN / 32);
    const int j = isx ? c % (BM / 32) : (c - XCH) % (BN / 32);
    const int r = 32 * j + (lane >> 1);
    const int lh = (lane & 1) ^ ((lane >> 4) & 1);  // logical half stored at physical half (lane & 1)
    if (TILED) {  // the image is already swizzled: lane-linear 16-B pieces of one contiguous 1 KiB
      const int ks_n = kp / SBK;
      if (isx) src[i] = XP + q * xplane + ((rtile * ks_n) << 12) + 512 * j + lane * 8;
      else src[i] = CP + q * cplane + (((long)(col0 >> 8) * ks_n) << 12) + 16 * (col0 & 255) + 512 * j + lane * 8;
    } else if (isx) {
      long xr = row0 + r;
      if (xr >= xrows) xr = xrows - 1;  // clamp: those rows are never reported
      src[i] = XP + q * xplane + xr * kp + 8 * lh;
    } else {
      src[i] = CP + q * cplane + (long)(col0 + r) * kp + 8 * lh;  // crows % 256 == 0
    }
    dst_off[i] = isx ? (q * BM + 32 * j) * 16 : (NPL * BM + q * BN + 32 * j) * 16;
  }
  auto issue = [&](int kt, int stage) {
    unsigned short* base = &lds[stage][0];
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      __builtin_amdgcn_global_load_lds((gbl_vptr)(src[i] + (TILED ? ((long)kt << 12) : (long)kt * SBK)),
                                       (lds_vptr)(base + dst_off[i]), 16, 0, 0);
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int ph = lk ^ ((li >> 3) & 1);  // physical half of this lane's fragment
  const int nk = kp / SBK;
  // one k step of this wave's 32x32 tiles from LDS stage `st`
  auto compute = [&](int st) {
    bf16x8 fb[NPL][TN];
#pragma unroll
    for (int p = 0; p < NPL; ++p)
#pragma unroll
      for (int nt = 0; nt < TN; ++nt)
        fb[p][nt] = *reinterpret_cast<const bf16x8*>(
            &lds[st][(NPL * BM + p * BN + wn * (BN / WN) + nt * 32 + li) * 16 + 8 * ph]);
#pragma unroll
    for (int mt = 0; mt < TM; ++mt) {
      bf16x8 fa[NPL];
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        fa[p] = *reinterpret_cast<const bf16x8*>(&lds[st][(p * BM + wm * (BM / WM) + mt * 32 + li) * 16 + 8 * ph]);
#pragma unroll
      for (int nt = 0; nt < TN; ++nt) {
        if constexpr (NP == 1) {
          // transposed tile (centres x rows): a lane holds ONE data row's 16 centre values per
          // 32 x 32 tile, so the arg-min epilogue is a register scan (split_epilogue_top2_t)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8, fb[0][nt]),
                                                               __builtin_bit_cast(halfx8, fa[0]), acc[mt][nt], 0,
                                                               0, 0);
        } else {
          if constexpr (NP == 6) {
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0][nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1][nt], acc[mt][nt], 0, 0, 0);
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2][nt], acc[mt][nt], 0, 0, 0);
          }
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0][nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1][nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0][nt], acc[mt][nt], 0, 0, 0);
        }
      }
    }
  };
  if constexpr (KPB == 1 && !RING) {
    // 3-stage ring, one k step per barrier, two steps of load lead
    static_assert(CPW == 6, "the counted wait below leaves one step (CPW loads) in flight");
    issue(0, 0);
    if (nk > 1) issue(1, 1);
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // step kt + 1 may stay in flight
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // step kt landed for every wave; every wave finished step kt - 1
      if (kt + 2 < nk) issue(kt + 2, stage == 0 ? 2 : stage - 1);
      if (PRIO) __builtin_amdgcn_s_setprio(1);
      compute(stage);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
      stage = stage == 2 ? 0 : stage + 1;
    }
  } else {
    // 3-product steps carry half the MFMA work (fp16 1-product steps a sixth): KPB k steps per
    // barrier on a 2 KPB-stage ring (group g computes from its KPB stages while group g + 1 lands
    // in the other KPB), so the barrier and the first fragment reads are paid once per KPB steps
    // NG >= 3: the NG - 2 newest groups may stay in flight at the wait (counted vmcnt: those groups
    // are full, else wait for everything)
#pragma unroll
    for (int j = 0; j < (NG - 1) * KPB; ++j)
      if (j < nk) issue(j, j);
    for (int kt = 0; kt < nk; kt += KPB) {
      if (NG >= 3 && kt + (NG - 1) * KPB <= nk)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NG - 2) * KPB * CPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // steps kt .. kt + KPB - 1 landed; every wave finished the previous group
#pragma unroll
      for (int j = 0; j < KPB; ++j)
        if (kt + (NG - 1) * KPB + j < nk) issue(kt + (NG - 1) * KPB + j, (kt + (NG - 1) * KPB + j) % NS);
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < KPB; ++j)
        if (kt + j < nk) compute((kt + j) % NS);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }
  if (CAND)
    split_epilogue_cand_t<BM, BN, WM, WN>(acc, row0, col0, m, k, cnorm, cg, xnorm, wm, wn, li, lk, dscale, xadd, thr,
                                          ccount, cand, cap);
  else if (TOP2 && NP == 1)
    split_epilogue_top2_t<BM, BN, WM, WN>(acc, row0, col0, ctile, m, k, cnorm, cg, xnorm, best, lob, n_ctiles * WN, wm,
                                          wn, li, lk, dscale, xadd);
  else if (TOP2)
    split_epilogue_top2<BM, BN, WM, WN>(acc, row0, col0, ctile, m, k, cnorm, cg, xnorm, best, lob, n_ctiles * WN, wm,
                                        wn, li, lk, dscale, xadd);
  else
    split_epilogue<BM, BN, WM, WN>(acc, row0, col0, m, k, cnorm, best, wm, wn, li, lk);
}

// Merge the slots of every row and certify the 3-product arg-min b: with |d~_j - d_j| <= e_j =
// ||x|| g_j (g_j = 2 tau ||c_j||; tau = ops.certify_tau(n) = 2^-13 for the 3 * 2^-16 dropped
// products + 2 n 2^-24 for the worst-case fp32 accumulation of both searches), d~_j - e_j >
// d~_b + e_b for every j != b proves d_j > d_b, i.e. the fp32 6-product search picks b too.
// Certified rows get their label and distance; the rest are appended to `flagged` (count in
// *n_flagged) for an exact re-search.
__global__ __launch_bounds__(256) void split_top2_select_kernel(const unsigned long long* __restrict__ keys,
                                                                const float* __restrict__ lob, long m, int nslot,
                                                                const float* __restrict__ xnorm,
                                                                const float* __restrict__ cg,
                                                                int* __restrict__ labels, float* __restrict__ dist,
                                                                int* __restrict__ flagged, int* __restrict__ n_flagged,
                                                                float xadd = 0.f, float z = 0.f, float z2 = 0.f,
                                                                const int* __restrict__ ovf = nullptr,
                                                                float* __restrict__ thr_out = nullptr) {
  // fp16 filter (srml_split_top2_select_f16): the radius of candidate j is (||x|| + xadd) g_j +
  // z ||x|| + z2 (the last two terms: subnormal fp16 elements, the same for every j, so they enter
  // the test once per side); an overflowed centroid plane (*ovf) certifies nothing
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  // slot-major layout (keys / lob[slot * m + row]): consecutive lanes read consecutive rows
  unsigned long long k1 = ~0ull;
  int s1 = 0;
  for (int s = 0; s < nslot; ++s) {
    const unsigned long long v = keys[(long)s * m + i];
    if (v < k1) { k1 = v; s1 = s; }
  }
  const float xn = xnorm[i];
  const float xs0 = sqrtf(fmaxf(xn, 0.f));
  const float xs = xs0 + xadd;
  const float c2 = 2.f * fmaf(z, xs0, z2);
  float low = __builtin_huge_valf();  // min over j != b of d~_j - e_j
  for (int s = 0; s < nslot; ++s) {
    low = fminf(low, lob[(long)s * m + i]);
    const unsigned long long v = keys[(long)s * m + i];
    if (s != s1 && v != ~0ull) low = fminf(low, fmaf(-xs, cg[(int)(v & 0xffffffffu)], unorderable((unsigned)(v >> 32))));
  }
  const float bv = unorderable((unsigned)(k1 >> 32));
  if (k1 != ~0ull && !(ovf && *ovf) && low > fmaf(xs, cg[(int)(k1 & 0xffffffffu)], bv) + c2) {
    labels[i] = (int)(k1 & 0xffffffffu);
    const float d = bv + xn;
    dist[i] = d > 0.f ? d : 0.f;
  } else {
    const int p = atomicAdd(n_flagged, 1);
    flagged[p] = (int)i;
    // the row's certified upper bound on its best distance: the re-search keeps every centre whose
    // lower bound does not exceed it (an overflowed centre plane: no bound, every centre)
    if (thr_out)
      thr_out[p] = (k1 != ~0ull && !(ovf && *ovf)) ? fmaf(xs, cg[(int)(k1 & 0xffffffffu)], bv) + c2
                                                   : __builtin_huge_valf();
  }
}

// Exact pass of the fp16 re-search: one wave per flagged row, squared distances to its candidate
// centres in fp64 ((x - mu) and (c - mu) as the fp32 values every search uses; each term exact in
// fp64, the 3000-term sum ~n 2^-53 relative), arg-min with the lowest index on ties; a row whose
// list overflowed (count > cap) scans every centre.
__global__ __launch_bounds__(256) void cand_exact_kernel(const float* __restrict__ X, long ld,
                                                         const float* __restrict__ mu, const float* __restrict__ W,
                                                         long ldw, int n, int k, const int* __restrict__ rows, int nf,
                                                         const int* __restrict__ ccount, const int* __restrict__ cand,
                                                         int cap, int* __restrict__ labels, float* __restrict__ dist) {
  const int lane = threadIdx.x & 63;
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nf) return;
  const long i = rows[w];
  const float* xr = X + i * ld;
  const int cnt = ccount[w];
  const bool full = cnt > cap || cnt <= 0;
  const int nc = full ? k : cnt;
  double bd = __builtin_huge_val();
  int bj = 0x7fffffff;
  for (int q = 0; q < nc; ++q) {
    const int j = full ? q : cand[w * (long)cap + q];
    const float* wr = W + (long)j * ldw;
    double acc = 0.0;
    for (int l = lane; l < n; l += 64) {
      const double dv = (double)(xr[l] - mu[l]) - (double)wr[l];
      acc = fma(dv, dv, acc);
    }
    acc = wave_sum(acc);
    if (acc < bd || (acc == bd && j < bj)) { bd = acc; bj = j; }
  }
  if (lane == 0) {
    labels[i] = bj;
    dist[i] = (float)bd;
  }
}

// Same pass with the row's fp32 (x - mu) held in registers as NV float4 per lane (n <= 1024 NV,
// n % 4 == 0, 16-B aligned rows): per candidate only its centre row is read, with all NV
// vector loads of it in flight at once (the scalar kernel re-read x and mu for every candidate
// and walked each row in a latency-bound 4-B loop).
template <int NV>
__global__ __launch_bounds__(256) void cand_exact_vec_kernel(const float* __restrict__ X, long ld,
                                                             const float* __restrict__ mu, const float* __restrict__ W,
                                                             long ldw, int n, int k, const int* __restrict__ rows,
                                                             int nf, const int* __restrict__ ccount,
                                                             const int* __restrict__ cand, int cap,
                                                             int* __restrict__ labels, float* __restrict__ dist) {
  const int lane = threadIdx.x & 63;
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nf) return;
  const long i = rows[w];
  const int n4 = n >> 2;
  const floatx4* xr = reinterpret_cast<const floatx4*>(X + i * ld);
  const floatx4* m4 = reinterpret_cast<const floatx4*>(mu);
  floatx4 xm[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = v * 64 + lane;
    xm[v] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (c < n4) {
      const floatx4 a = xr[c], b = m4[c];
      xm[v] = floatx4{a[0] - b[0], a[1] - b[1], a[2] - b[2], a[3] - b[3]};  // the fp32 x - mu of every search
    }
  }
  const int cnt = ccount[w];
  const bool full = cnt > cap || cnt <= 0;
  const int nc = full ? k : cnt;
  double bd = __builtin_huge_val();
  int bj = 0x7fffffff;
  for (int q = 0; q < nc; ++q) {
    const int j = full ? q : cand[w * (long)cap + q];
    const floatx4* wr = reinterpret_cast<const floatx4*>(W + (long)j * ldw);
    floatx4 wv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = v * 64 + lane;
      wv[v] = c < n4 ? wr[c] : floatx4{0.f, 0.f, 0.f, 0.f};
    }
    double acc = 0.0;
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double dv = (double)xm[v][e] - (double)wv[v][e];
        acc = fma(dv, dv, acc);
      }
    acc = wave_sum(acc);
    if (acc < bd || (acc == bd && j < bj)) { bd = acc; bj = j; }
  }
  if (lane == 0) {
    labels[i] = bj;
    dist[i] = (float)bd;
  }
}

__global__ __launch_bounds__(256) void split_scatter_refined_kernel(const unsigned long long* __restrict__ best,
                                                                    const int* __restrict__ rows, int nf,
                                                                    const float* __restrict__ xnorm,
                                                                    int* __restrict__ labels, float* __restrict__ dist) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= nf) return;
  const int r = rows[j];
  const unsigned long long key = best[j];
  labels[r] = (int)(key & 0xffffffffu);
  const float d = unorderable((unsigned)(key >> 32)) + xnorm[r];
  dist[r] = d > 0.f ? d : 0.f;
}
}  // namespace

// P: [3][rows_pad][kp] bf16 (uint16), kp % 16 == 0, kp >= n, rows_pad >= m
SRML_API int srml_split_bf16x3(const float* X, long m, int n, long ld, int kp, long rows_pad, unsigned short* P,
                               hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || kp < n || rows_pad < m) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) != 0) return -5;
  long total = rows_pad * (long)(kp / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(split_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, kp, rows_pad, P);
  return srml_status();
}

// XP: planes of X ([3][xrows][kp]), CP: planes of the centroids ([3][crows][kp], crows % 128 == 0
// (% 256 when k > 256), crows >= k). best: m packed keys, initialised to ~0 by the caller.
SRML_API int srml_nearest_centroid_split(const unsigned short* XP, long m, long xrows, int kp,
                                         const unsigned short* CP, int k, long crows, const float* cnorm,
                                         unsigned long long* best, hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  static const int tile_env = getenv("SRML_SPLIT_TILE") ? atoi(getenv("SRML_SPLIT_TILE")) : 0;
  const bool big = tile_env ? tile_env == 256 : k > 256;  // 256 x 256 tiles: half the L2 bytes per MFMA of 128 x 128
  const int T = big ? 256 : 128;
  if ((kp & 15) || xrows < m || crows < k || (crows % T) != 0) return -2;
  if ((reinterpret_cast<uintptr_t>(XP) & 15) || (reinterpret_cast<uintptr_t>(CP) & 15)) return -5;
  const long rt = (m + T - 1) / T;
  const int ct = (k + T - 1) / T;
  const long nb = rt * ct;
  if (nb > srml_max_blocks(big ? 512 : 256)) return -3;
  static const int pf = getenv("SRML_SPLIT_PF") ? atoi(getenv("SRML_SPLIT_PF")) : 2;
  static const int glds = getenv("SRML_SPLIT_GLDS") ? atoi(getenv("SRML_SPLIT_GLDS")) : 0;
  if (big && glds)
    hipLaunchKernelGGL(nearest_centroid_split_glds_kernel<false>, dim3((unsigned)nb), dim3(512), 0, stream, XP, m, xrows, kp,
                       CP, k, crows, cnorm, best, ct);
  else if (big && pf == 2)
    hipLaunchKernelGGL((nearest_centroid_split_kernel<256, 256, 2, 4, 1, 2>), dim3((unsigned)nb), dim3(512), 0, stream,
                       XP, m, xrows, kp, CP, k, crows, cnorm, best, ct);
  else if (big)
    hipLaunchKernelGGL((nearest_centroid_split_kernel<256, 256, 2, 4, 1, 1>), dim3((unsigned)nb), dim3(512), 0, stream,
                       XP, m, xrows, kp, CP, k, crows, cnorm, best, ct);
  else if (pf == 2)
    hipLaunchKernelGGL((nearest_centroid_split_kernel<128, 128, 2, 2, 2, 2>), dim3((unsigned)nb), dim3(256), 0, stream,
                       XP, m, xrows, kp, CP, k, crows, cnorm, best, ct);
  else
    hipLaunchKernelGGL((nearest_centroid_split_kernel<128, 128, 2, 2, 2, 1>), dim3((unsigned)nb), dim3(256), 0, stream,
                       XP, m, xrows, kp, CP, k, crows, cnorm, best, ct);
  return srml_status();
}

// Tiled layout (split_tiled_kernel): P = [3][rows_pad / 256][kp / 16][256][16], rows_pad % 256 == 0.
SRML_API int srml_split_bf16x3_tiled(const float* X, long m, int n, long ld, int kp, long rows_pad, unsigned short* P,
                                     hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || kp < n || rows_pad < m || (rows_pad & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) != 0) return -5;
  long total = rows_pad * (long)(kp / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(split_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, kp, rows_pad, P,
                     (const float*)nullptr);
  return srml_status();
}

// Tiled planes of X - mu (mu: n floats): the certified KMeans search works on centred data, where
// the dropped-product error bound (relative to ||x - mu|| ||c - mu||) is small next to the gaps.
SRML_API int srml_split_bf16x3_tiled_centered(const float* X, long m, int n, long ld, const float* mu, int kp,
                                              long rows_pad, unsigned short* P, hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || kp < n || rows_pad < m || (rows_pad & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) != 0) return -5;
  long total = rows_pad * (long)(kp / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(split_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, kp, rows_pad, P,
                     mu);
  return srml_status();
}

// Tiled centred planes of the rows X[ridx[0..m)] (a gathered copy never exists): the re-search
// operand of the certified filters' flagged rows
SRML_API int srml_split_bf16x3_tiled_centered_rows(const float* X, long ld, const int* ridx, long m, int n,
                                                   const float* mu, int kp, long rows_pad, unsigned short* P,
                                                   hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || kp < n || rows_pad < m || (rows_pad & 255) || !ridx) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) != 0) return -5;
  long total = rows_pad * (long)(kp / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(split_tiled_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, kp, rows_pad, P,
                     mu, ridx);
  return srml_status();
}

// Block tile of the 3-product passes: 256 x 256 (one 8-wave block per CU) unless
// SRML_SPLIT_BN3=128 (256 x 128, two 4-wave blocks per CU: measured equal, 16.8 vs 16.7 ms).
static int split3_bn() {
  static const int bn = getenv("SRML_SPLIT_BN3") && atoi(getenv("SRML_SPLIT_BN3")) == 128 ? 128 : 256;
  return bn;
}

// Nearest centroid on tiled planes of X (xrows % 256 == 0) and of the centroids (crows % 256 == 0).
// nprod: 6 (fp32-exact) or 3 (approximate, half the MFMAs).
SRML_API int srml_nearest_centroid_split_tiled_np(const unsigned short* XP, long m, long xrows, int kp,
                                                  const unsigned short* CP, int k, long crows, const float* cnorm,
                                                  unsigned long long* best, int nprod, hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  if ((kp & 15) || xrows < m || crows < k || (crows & 255) || (xrows & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(XP) & 15) || (reinterpret_cast<uintptr_t>(CP) & 15)) return -5;
  const long rt = (m + 255) / 256;
  const int bn = nprod == 3 ? split3_bn() : 256;
  const int ct = (k + bn - 1) / bn;
  const long nb = rt * ct;
  if (nb > srml_max_blocks(512)) return -3;  // 2^32 work-item grid
  if (nprod == 3 && bn == 128)
    hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 3, false, 2>), dim3((unsigned)nb), dim3(256), 0, stream,
                       XP, m, xrows, kp, CP, k, crows, cnorm, best, (int)ct);
  else if (nprod == 3)
    hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 3>), dim3((unsigned)nb), dim3(512), 0, stream, XP, m,
                       xrows, kp, CP, k, crows, cnorm, best, (int)ct);
  else if (nprod == 6)
    hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 6>), dim3((unsigned)nb), dim3(512), 0, stream, XP, m,
                       xrows, kp, CP, k, crows, cnorm, best, (int)ct);
  else
    return -2;
  return srml_status();
}

SRML_API int srml_nearest_centroid_split_tiled(const unsigned short* XP, long m, long xrows, int kp,
                                               const unsigned short* CP, int k, long crows, const float* cnorm,
                                               unsigned long long* best, hipStream_t stream) {
  return srml_nearest_centroid_split_tiled_np(XP, m, xrows, kp, CP, k, crows, cnorm, best, 6, stream);
}

// Certified 3-product nearest-centroid search, phase 1 (tiled planes, as
// srml_nearest_centroid_split_tiled_np): best + lower-bound slots per row, keys / lob sized
// m * srml_nearest_centroid_split_top2_nslot(k); cg = 2 tau ||c_j|| per centroid, xnorm = ||x||^2 of the (centred) rows.
SRML_API int srml_nearest_centroid_split_top2(const unsigned short* XP, long m, long xrows, int kp,
                                              const unsigned short* CP, int k, long crows, const float* cnorm,
                                              const float* cg, const float* xnorm, unsigned long long* keys,
                                              float* lob, hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  if ((kp & 15) || xrows < m || crows < k || (crows & 255) || (xrows & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(XP) & 15) || (reinterpret_cast<uintptr_t>(CP) & 15)) return -5;
  const long rt = (m + 255) / 256;
  const int bn = split3_bn();
  const int ct = (k + bn - 1) / bn;
  const long nb = rt * ct;
  if (nb > srml_max_blocks(512)) return -3;  // 2^32 work-item grid
  // s_setprio around the MFMA clusters: 16.7 -> 16.4 ms per pass on the 256 x 256 tile (neutral
  // on 256 x 128); SRML_SPLIT_PRIO=0 turns it off
  static const bool prio = !(getenv("SRML_SPLIT_PRIO") && atoi(getenv("SRML_SPLIT_PRIO")) == 0);
#define SRML_TOP2(WNN, PR, T)                                                                                    \
  hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 3, true, WNN, PR>), dim3((unsigned)nb), dim3(T), 0, \
                     stream, XP, m, xrows, kp, CP, k, crows, cnorm, keys, (int)ct, lob, cg, xnorm)
  if (bn == 128 && prio) SRML_TOP2(2, true, 256);
  else if (bn == 128) SRML_TOP2(2, false, 256);
  else if (prio) SRML_TOP2(4, true, 512);
  else SRML_TOP2(4, false, 512);
#undef SRML_TOP2
  return srml_status();
}

// (row, slot) pairs of the top-2 phase: one slot per (centroid tile, wave column)
SRML_API int srml_nearest_centroid_split_top2_nslot(int k) {
  const int bn = split3_bn();
  return ((k + bn - 1) / bn) * (bn / 64);
}

// phase 2: merge slots, certify, emit labels / distances of certified rows, list the others
SRML_API int srml_split_top2_select(const unsigned long long* keys, const float* lob, long m, int nslot,
                                    const float* xnorm, const float* cg, int* labels, float* dist, int* flagged,
                                    int* n_flagged, hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(split_top2_select_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, keys, lob, m,
                     nslot, xnorm, cg, labels, dist, flagged, n_flagged);
  return srml_status();
}

// phase 3 epilogue: exact keys of the re-searched rows -> labels / distances at their positions
SRML_API int srml_split_scatter_refined(const unsigned long long* best, const int* rows, int nf, const float* xnorm,
                                        int* labels, float* dist, hipStream_t stream) {
  if (nf <= 0) return 0;
  hipLaunchKernelGGL(split_scatter_refined_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, stream, best,
                     rows, nf, xnorm, labels, dist);
  return srml_status();
}

// ---- fp16 certified filter -----------------------------------------------------------------
// Centroid-tile width of the fp16 filter: 256 (256 x 256 tile, one 8-wave block per CU, 3-group
// ring) or SRML_F16_BN=128 (256 x 128 tiles, two 4-wave blocks per CU, 2-group rings)
static int f16_bn() {
  static const int bn = getenv("SRML_F16_BN") && atoi(getenv("SRML_F16_BN")) == 128 ? 128 : 256;
  return bn;
}
// result slots per centroid tile: one per 64-wide wave column
static int f16_slots_per_tile() { return f16_bn() / 64; }

// Centre operands of one fp16 filter search, in one launch (was ~10 torch launches per Lloyd
// iteration): W = fp32(C - mu) (C fp64 or fp32 rows, k x n), cn = fp32 of the fp64 norm of W's
// rows, cg = 2 tau sqrt(cn) (0 when approx), and the overflow / flagged counters zeroed. One
// 64-lane wave per centre.
template <typename T>
__global__ __launch_bounds__(256) void f16_centre_prep_kernel(const T* __restrict__ C, int k, int n,
                                                              const float* __restrict__ mu, float tau2, int approx,
                                                              float* __restrict__ W, float* __restrict__ cn,
                                                              float* __restrict__ cg, int* __restrict__ zero2) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x < 2) zero2[threadIdx.x] = 0;
  if (j >= k) return;  // whole waves
  double a = 0.0;
  for (int d = lane; d < n; d += 64) {
    const float w = (float)((double)C[(long)j * n + d] - (double)mu[d]);
    W[(long)j * n + d] = w;
    a += (double)w * (double)w;
  }
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (lane == 0) {
    const float c = (float)a;
    cn[j] = c;
    cg[j] = approx ? 0.f : tau2 * sqrtf(c > 0.f ? c : 0.f);
  }
}

SRML_API int srml_f16_centre_prep(const void* C, int c_f64, int k, int n, const float* mu, float tau2, int approx,
                                  float* W, float* cn, float* cg, int* zero2, hipStream_t stream) {
  if (k <= 0) return 0;
  const dim3 grid((unsigned)((k + 3) / 4));
  if (c_f64)
    hipLaunchKernelGGL(f16_centre_prep_kernel<double>, grid, dim3(256), 0, stream,
                       reinterpret_cast<const double*>(C), k, n, mu, tau2, approx, W, cn, cg, zero2);
  else
    hipLaunchKernelGGL(f16_centre_prep_kernel<float>, grid, dim3(256), 0, stream, reinterpret_cast<const float*>(C),
                       k, n, mu, tau2, approx, W, cn, cg, zero2);
  return srml_status();
}

// One tiled fp16 plane of scale * (x - mu) (mu may be null), rows padded to rows_pad (% 256 == 0):
// P = [rows_pad / 256][kp / 16][256][16]; *ovf |= 1 if an element of |scale v| >= 2^15 was clamped.
SRML_API int srml_split_f16_tiled_centered(const float* X, long m, int n, long ld, const float* mu, int kp,
                                           long rows_pad, float scale, unsigned short* P, int* ovf,
                                           hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || kp < n || rows_pad < m || (rows_pad & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) != 0) return -5;
  const long total = rows_pad * (long)(kp / 16);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(split_tiled_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, kp, rows_pad, P,
                     mu, scale, ovf);
  return srml_status();
}

// Certified fp16 filter, phase 1: one fp16 MFMA product per (row, centroid) on the scaled planes
// (XP, CP from srml_split_f16_tiled_centered with the same scale s); d~ = ||c||^2 + dscale acc with
// dscale = -2 / s^2; lower bounds use the radius (||x|| + xadd) g_j. 256 x 256 tiles, keys / lob
// sized m * srml_nearest_centroid_split_top2_nslot(k) as the 3-product pass at SRML_SPLIT_BN3=256.
SRML_API int srml_nearest_centroid_f16_top2(const unsigned short* XP, long m, long xrows, int kp,
                                            const unsigned short* CP, int k, long crows, const float* cnorm,
                                            const float* cg, const float* xnorm, float dscale, float xadd,
                                            unsigned long long* keys, float* lob, hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  if ((kp & 15) || xrows < m || crows < k || (crows & 255) || (xrows & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(XP) & 15) || (reinterpret_cast<uintptr_t>(CP) & 15)) return -5;
  const long rt = (m + 255) / 256;
  const int bn = f16_bn();
  const int ct = (k + bn - 1) / bn;
  const long nb = rt * ct;
  if (nb > srml_max_blocks(bn * 2)) return -3;  // 2^32 work-item grid
  static const bool prio = !(getenv("SRML_SPLIT_PRIO") && atoi(getenv("SRML_SPLIT_PRIO")) == 0);
#define SRML_F16(WNN, PR, T)                                                                                      \
  hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 1, true, WNN, PR>), dim3((unsigned)nb), dim3(T), 0, \
                     stream, XP, m, xrows, kp, CP, k, crows, cnorm, keys, (int)ct, lob, cg, xnorm, dscale, xadd)
  static const int ring = getenv("SRML_F16_RING") ? atoi(getenv("SRML_F16_RING")) : 0;
#define SRML_F16R(RG)                                                                                               \
  hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 1, true, 4, true, false, RG>), dim3((unsigned)nb),      \
                     dim3(512), 0, stream, XP, m, xrows, kp, CP, k, crows, cnorm, keys, (int)ct, lob, cg, xnorm,       \
                     dscale, xadd)
  if (f16_bn() == 128) {
    if (prio) SRML_F16(2, true, 256);
    else SRML_F16(2, false, 256);
  } else if (ring == 23) {
    SRML_F16R(23);
  } else if (ring == 24) {
    SRML_F16R(24);
  } else if (ring == 42) {
    SRML_F16R(42);
  } else if (ring == 18) {
    SRML_F16R(18);
  } else if (ring == 25) {
    SRML_F16R(25);
  } else {
    if (prio) SRML_F16(4, true, 512);
    else SRML_F16(4, false, 512);
  }
#undef SRML_F16R
#undef SRML_F16
  return srml_status();
}

// (row, slot) pairs of the fp16 filter (one slot per wave column of each centroid tile)
SRML_API int srml_nearest_centroid_f16_top2_nslot(int k) {
  const int bn = f16_bn();
  return ((k + bn - 1) / bn) * f16_slots_per_tile();
}

// phase 2 of the fp16 filter: as srml_split_top2_select with the extra radius terms (see kernel)
SRML_API int srml_split_top2_select_f16(const unsigned long long* keys, const float* lob, long m, int nslot,
                                        const float* xnorm, const float* cg, float xadd, float z, float z2,
                                        const int* ovf, int* labels, float* dist, int* flagged, int* n_flagged,
                                        hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(split_top2_select_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, keys, lob, m,
                     nslot, xnorm, cg, labels, dist, flagged, n_flagged, xadd, z, z2, ovf);
  return srml_status();
}

// ---- fp16 filter re-search (candidate lists + fp64 exact distances) -------------------------
// fp16 plane of the gathered rows X[ridx[0..m)] (same scale / layout as srml_split_f16_tiled_centered)
SRML_API int srml_split_f16_tiled_centered_rows(const float* X, long ld, const int* ridx, long m, int n,
                                                const float* mu, int kp, long rows_pad, float scale, unsigned short* P,
                                                int* ovf, hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || kp < n || rows_pad < m || (rows_pad & 255) || !ridx) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) != 0) return -5;
  const long total = rows_pad * (long)(kp / 16);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(split_tiled_f16_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, X, m, n, ld, kp, rows_pad, P,
                     mu, scale, ovf, ridx);
  return srml_status();
}

// Gather rows of an existing tiled fp16 plane (the filter's X plane) into a new tiled plane: row
// r of the output = row ridx[r] of the source, bit-identical to converting X[ridx[r]] again but
// reading 32 B of fp16 per (row, k step) instead of 64 B of fp32; one thread per (row, k step),
// each 32-B slot moved as two 16-B halves with the source / destination swizzles undone / applied.
// xn / xn_out (nullable): also gather the rows' norms; zero_out (nullable): m ints zeroed (the
// candidate search's per-row counters), so the re-search needs no separate fill / gather launches.
__global__ __launch_bounds__(256) void f16_plane_gather_kernel(const uintx4* __restrict__ src, int ks_n,
                                                               const int* __restrict__ ridx, long m, long rows_pad,
                                                               uintx4* __restrict__ dst,
                                                               const float* __restrict__ xn = nullptr,
                                                               float* __restrict__ xn_out = nullptr,
                                                               int* __restrict__ zero_out = nullptr) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < m; i += (long)gridDim.x * 256) {
    if (xn_out) xn_out[i] = xn[ridx[i]];
    if (zero_out) zero_out[i] = 0;
  }
  const long total = rows_pad * ks_n;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long img = i >> 8;
    const int rr = (int)(i & 255);
    const long tile = img / ks_n;
    const long ks = img - tile * ks_n;
    const long r = tile * 256 + rr;
    uintx4 lo = uintx4{0u, 0u, 0u, 0u}, hi = lo;  // padding rows: zeros, as the converting kernel writes
    if (r < m) {
      const long rs = ridx[r];
      const int ssw = (int)((rs >> 3) & 1);
      const uintx4* s = src + ((((rs >> 8) * ks_n + ks) << 12) + (rs & 255) * 16) / 8;
      lo = s[ssw];
      hi = s[ssw ^ 1];
    }
    const int dsw = (rr >> 3) & 1;
    uintx4* d = dst + ((img << 12) + rr * 16) / 8;
    d[dsw] = lo;
    d[dsw ^ 1] = hi;
  }
}

SRML_API int srml_f16_plane_gather_rows_ex(const unsigned short* P, long src_rows_pad, int kp, const int* ridx, long m,
                                           long rows_pad, unsigned short* out, const float* xn, float* xn_out,
                                           int* zero_out, hipStream_t stream) {
  if (rows_pad <= 0) return 0;
  if ((kp & 15) || rows_pad < m || (rows_pad & 255) || (src_rows_pad & 255) || !ridx) return -2;
  if ((reinterpret_cast<uintptr_t>(P) & 15) || (reinterpret_cast<uintptr_t>(out) & 15)) return -5;
  if (xn_out && !xn) return -2;
  const long total = rows_pad * (long)(kp / 16);
  long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(f16_plane_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     reinterpret_cast<const uintx4*>(P), kp / 16, ridx, m, rows_pad, reinterpret_cast<uintx4*>(out), xn,
                     xn_out, zero_out);
  return srml_status();
}

SRML_API int srml_f16_plane_gather_rows(const unsigned short* P, long src_rows_pad, int kp, const int* ridx, long m,
                                        long rows_pad, unsigned short* out, hipStream_t stream) {
  return srml_f16_plane_gather_rows_ex(P, src_rows_pad, kp, ridx, m, rows_pad, out, nullptr, nullptr, nullptr, stream);
}

// select of the filter pass with the flagged rows' thresholds (thr_out[p] for flagged[p])
SRML_API int srml_split_top2_select_f16_thr(const unsigned long long* keys, const float* lob, long m, int nslot,
                                            const float* xnorm, const float* cg, float xadd, float z, float z2,
                                            const int* ovf, int* labels, float* dist, int* flagged, int* n_flagged,
                                            float* thr_out, hipStream_t stream) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(split_top2_select_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, keys, lob, m,
                     nslot, xnorm, cg, labels, dist, flagged, n_flagged, xadd, z, z2, ovf, thr_out);
  return srml_status();
}

// candidate pass over the flagged rows' fp16 plane XP (m rows): ccount (m, zeroed by the caller),
// cand (m x cap) — same tile / launch rules as srml_nearest_centroid_f16_top2
SRML_API int srml_nearest_centroid_f16_cand(const unsigned short* XP, long m, long xrows, int kp,
                                            const unsigned short* CP, int k, long crows, const float* cnorm,
                                            const float* cg, const float* xnorm, float dscale, float xadd,
                                            const float* thr, int* ccount, int* cand, int cap, hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  if ((kp & 15) || xrows < m || crows < k || (crows & 255) || (xrows & 255) || cap < 1) return -2;
  if ((reinterpret_cast<uintptr_t>(XP) & 15) || (reinterpret_cast<uintptr_t>(CP) & 15)) return -5;
  const long rt = (m + 255) / 256;
  const int ct = (k + 255) / 256;
  const long nb = rt * ct;
  if (nb > srml_max_blocks(512)) return -3;
  hipLaunchKernelGGL((nearest_centroid_split_glds_kernel<true, 1, true, 4, true, true>), dim3((unsigned)nb), dim3(512),
                     0, stream, XP, m, xrows, kp, CP, k, crows, cnorm, (unsigned long long*)nullptr, (int)ct,
                     (float*)nullptr, cg, xnorm, dscale, xadd, thr, ccount, cand, cap);
  return srml_status();
}

// exact fp64 arg-min of each flagged row over its candidate list -> labels / dist at the row
SRML_API int srml_kmeans_cand_exact(const float* X, long ld, const float* mu, const float* W, long ldw, int n, int k,
                                    const int* rows, int nf, const int* ccount, const int* cand, int cap, int* labels,
                                    float* dist, hipStream_t stream) {
  if (nf <= 0) return 0;
  const dim3 grid((unsigned)((nf + 3) / 4));
  const bool vec = (n & 3) == 0 && (ld & 3) == 0 && (ldw & 3) == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(W) & 15) == 0 && (reinterpret_cast<uintptr_t>(mu) & 15) == 0;
  const int nv = (n / 4 + 63) / 64;
  static const bool scalar = getenv("SRML_CAND_EXACT") && atoi(getenv("SRML_CAND_EXACT")) == 0;  // 0: scalar kernel
#define SRML_CE(NVV)                                                                                                  \
  hipLaunchKernelGGL(cand_exact_vec_kernel<NVV>, grid, dim3(256), 0, stream, X, ld, mu, W, ldw, n, k, rows, nf, ccount, \
                     cand, cap, labels, dist)
  if (vec && !scalar && nv <= 4) SRML_CE(4);
  else if (vec && !scalar && nv <= 8) SRML_CE(8);
  else if (vec && !scalar && nv <= 12) SRML_CE(12);
  else if (vec && !scalar && nv <= 16) SRML_CE(16);
  else
    hipLaunchKernelGGL(cand_exact_kernel, grid, dim3(256), 0, stream, X, ld, mu, W, ldw, n, k, rows, nf, ccount, cand,
                       cap, labels, dist);
#undef SRML_CE
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Arg-min over ALL centres per row in one block per 256-row tile: the IVF bucketing / quantiser
// labels (approximate: the fp16 planes' arg-min, lowest index on ties) for short rows (kp = 128:
// 8 k steps) and many centres. The top-2 filter above writes one (key, bound) slot per (row,
// 64-centre tile) — at 20M rows x 19.5k lists that is 73 GB of slots written and re-read by the
// select, while the products themselves are ~100 TFLOP: the rows' fragments here stay in
// registers for the whole scan, the centre tiles (64 KB of fp16 images + their norms) stream
// through a 2-buffer LDS ring by LDS-DMA, and each lane keeps its row's running minimum (the
// transposed 32 x 32 tiles of split_epilogue_top2_t: 16 centres per lane and tile), so a row costs
// 4 bytes of output.
namespace {
template <int KS>
__global__ __launch_bounds__(512, 1) void nearest_f16_rowloop_kernel(const unsigned short* __restrict__ XP, long m,
                                                                     const unsigned short* __restrict__ CP, int k,
                                                                     int n_ctiles, const float* __restrict__ cnorm,
                                                                     float dscale, int* __restrict__ labels) {
  constexpr int CT = 256;             // centres per staged tile
  constexpr int IMG = CT * 16;        // halves per (tile, k step) image (8 KB)
  constexpr int CHUNKS = KS * 8;      // 1 KB DMA chunks per centre tile
  constexpr int CPW = CHUNKS / 8;     // ... per wave
  __shared__ __attribute__((aligned(1024))) unsigned short lds[2][KS * IMG];
  __shared__ __attribute__((aligned(1024))) float cn_s[2][CT];
  const long tile = xcd_remap(blockIdx.x, gridDim.x);
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6, li = lane & 31, lk = lane >> 5;
  const int rr = 32 * wid + li;  // this lane's row in the tile (B operand column)
  halfx8 xb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    xb[ks] = *reinterpret_cast<const halfx8*>(XP + ((tile * KS + ks) << 12) + rr * 16 + 8 * (lk ^ ((rr >> 3) & 1)));
  auto issue = [&](int c, int buf) {
    const unsigned short* src = CP + ((long)c * KS << 12);
#pragma unroll
    for (int i = 0; i < CPW; ++i) {
      const int ch = wid * CPW + i;
      __builtin_amdgcn_global_load_lds((gbl_vptr)(src + ch * 512 + lane * 8), (lds_vptr)(&lds[buf][ch * 512]), 16, 0,
                                       0);
    }
    if (wid == 0) {
#pragma unroll
      for (int i = 0; i < CT / 64; ++i)
        __builtin_amdgcn_global_load_lds((gbl_vptr)(cnorm + (long)c * CT + i * 64 + lane), (lds_vptr)(&cn_s[buf][i * 64]),
                                         4, 0, 0);
    }
  };
  float best = __builtin_huge_valf();
  int bi = 0x7fffffff;
  issue(0, 0);
  if (n_ctiles > 1) issue(1, 1);
  for (int c = 0; c < n_ctiles; ++c) {
    const int buf = c & 1;
    // tile c landed for every wave (tile c + 1 may stay in flight), every wave is past tile c - 1
    if (c + 1 < n_ctiles) {
      if (wid == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(CPW + CT / 64) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(CPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const bool last = c == n_ctiles - 1;
    const int cbase = c * CT;
#pragma unroll 2
    for (int nt = 0; nt < CT / 32; ++nt) {
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int cl = nt * 32 + li;  // this lane's centre row of the A fragment
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const halfx8 a = *reinterpret_cast<const halfx8*>(&lds[buf][ks * IMG + cl * 16 + 8 * (lk ^ ((cl >> 3) & 1))]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, xb[ks], acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 cn = *reinterpret_cast<const floatx4*>(&cn_s[buf][nt * 32 + 8 * q + 4 * lk]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = cbase + nt * 32 + 8 * q + 4 * lk + u;
          float d = fmaf(dscale, acc[4 * q + u], cn[u]);
          if (last && j >= k) d = __builtin_huge_valf();
          if (d < best) {
            best = d;
            bi = j;
          }
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done with buffer `buf`
    if (c + 2 < n_ctiles) issue(c + 2, buf);
  }
  const float ov = __shfl_xor(best, 32, 64);
  const int oi = __shfl_xor(bi, 32, 64);
  if (ov < best || (ov == best && oi < bi)) {
    best = ov;
    bi = oi;
  }
  const long row = tile * 256 + rr;
  if (lk == 0 && row < m) labels[row] = bi == 0x7fffffff ? 0 : bi;
}
}  // namespace

// labels[r] = arg-min_j (cnorm[j] + dscale <P_r, CP_j>) over j < k (lowest index on ties): XP / CP
// tiled fp16 planes with kp = 128 (rows padded to 256), cnorm readable for crows = n_ctiles * 256
// entries (entries past k are ignored). Returns -2 for other widths (the caller takes the top-2 path).
SRML_API int srml_nearest_f16_rowloop(const unsigned short* XP, long m, long xrows, int kp, const unsigned short* CP,
                                      int k, long crows, const float* cnorm, float dscale, int* labels,
                                      hipStream_t stream) {
  if (m <= 0 || k <= 0) return 0;
  if (kp != 128 || xrows < m || (xrows & 255) || crows < k || (crows & 255)) return -2;
  if ((reinterpret_cast<uintptr_t>(XP) & 15) || (reinterpret_cast<uintptr_t>(CP) & 15) ||
      (reinterpret_cast<uintptr_t>(cnorm) & 3))
    return -5;
  const long nb = (m + 255) / 256;
  if (nb > srml_max_blocks(512)) return -3;
  hipLaunchKernelGGL(nearest_f16_rowloop_kernel<8>, dim3((unsigned)nb), dim3(512), 0, stream, XP, m, CP, k,
                     (int)(crows / 256), cnorm, dscale, labels);
  return srml_status();
}
