// Per-level bookkeeping of the level-synchronous forest builder (models/forest.py
// `_level_one_sync`) as four small kernels instead of ~55 torch library launches per level:
//
//   * rf_left_totals: a candidate's left-child class totals, the prefix of its winning feature's
//     histogram up to the split bin (zeros when the candidate does not split);
//   * rf_gather_feature: the winning feature id of every candidate (its record's slot into the
//     node's feature sample), as fp64 next to the record;
//   * rf_decide_scan (one block): the splitting candidates' exclusive rank r (children 2r, 2r + 1)
//     and their count k;
//   * rf_decide_apply: the routing arrays of the level's segments (feature, bin, child base) at
//     the splitting candidates, and for classification the children's totals (left = prefix,
//     right = parent - left) with the rows past 2k zeroed;
//   * rf_level_pack: ONE fp64 buffer for the level's single read-back — child bounds, per-child
//     [leaf value(s) | weight | impurity] (the formulas of forest.py `_seg_stats`), the split
//     records and the winning feature ids.
// Reference behaviour: python/src/spark_rapids_ml/tree.py:309-414 (cuML RF node splitting, leaf
// values and impurities per node).
#include <hip/hip_runtime.h>

#include "common.h"

namespace {

constexpr int RL_THREADS = 256;

// left[c, s] = sum_{bin <= b} hist[c, slot, bin, s] for (slot, b) = out[c, 1..2], zeros if slot < 0
template <typename H>
__global__ __launch_bounds__(RL_THREADS) void rf_left_totals_kernel(const H* __restrict__ hist, long C, int nslot,
                                                                    int B, int S, const double* __restrict__ out,
                                                                    double* __restrict__ left) {
  const long i = (long)blockIdx.x * RL_THREADS + threadIdx.x;
  if (i >= C * S) return;
  const long c = i / S;
  const int s = (int)(i - c * S);
  const int slot = (int)out[c * 6 + 1];
  double a = 0.0;
  if (slot >= 0) {
    const int b = (int)out[c * 6 + 2];
    const H* h = hist + ((c * nslot + slot) * (long)B) * S + s;
    for (int j = 0; j <= b && j < B; ++j) a += (double)h[(long)j * S];
  }
  left[i] = a;
}

__global__ __launch_bounds__(RL_THREADS) void rf_gather_feature_kernel(const int* __restrict__ feats, long ld,
                                                                       const double* __restrict__ out, long C,
                                                                       double* __restrict__ fsel) {
  const long c = (long)blockIdx.x * RL_THREADS + threadIdx.x;
  if (c >= C) return;
  const int slot = (int)out[c * 6 + 1];
  fsel[c] = (double)feats[c * ld + (slot > 0 ? slot : 0)];
}

// one 1024-thread block: pos[j] = # splitting candidates before j, tot[0] = their count
__global__ __launch_bounds__(1024) void rf_decide_scan_kernel(const double* __restrict__ out, long C,
                                                              int* __restrict__ pos, long long* __restrict__ tot) {
  __shared__ long long s[1024];
  const int t = threadIdx.x;
  const long per = (C + 1023) / 1024;
  const long a = (long)t * per, e = a + per < C ? a + per : C;
  long long sum = 0;
  for (long j = a; j < e; ++j) sum += out[j * 6 + 1] >= 0.0 ? 1 : 0;
  s[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const long long v = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  long long run = s[t] - sum;
  for (long j = a; j < e; ++j) {
    pos[j] = (int)run;
    run += out[j * 6 + 1] >= 0.0 ? 1 : 0;
  }
  if (t == 1023) tot[0] = s[1023];
}

// node arrays pre-filled by the caller (feature -1, bin 0, child base 0)
__global__ __launch_bounds__(RL_THREADS) void rf_decide_apply_kernel(
    const double* __restrict__ out, const double* __restrict__ fsel, const long long* __restrict__ cand, long C,
    const int* __restrict__ pos, const long long* __restrict__ tot_k, int* __restrict__ node_feature,
    int* __restrict__ node_bin, int* __restrict__ child_base, const double* __restrict__ left,
    const double* __restrict__ tot, int S, double* __restrict__ tot_n) {
  const long j = (long)blockIdx.x * RL_THREADS + threadIdx.x;
  if (j < C && out[j * 6 + 1] >= 0.0) {
    const long seg = cand[j];
    const int r = pos[j];
    node_feature[seg] = (int)fsel[j];
    node_bin[seg] = (int)out[j * 6 + 2];
    child_base[seg] = 2 * r;
    if (tot_n) {
      for (int s = 0; s < S; ++s) {
        const double l = left[j * S + s];
        tot_n[(2L * r) * S + s] = l;
        tot_n[(2L * r + 1) * S + s] = tot[seg * S + s] - l;
      }
    }
  }
  if (tot_n) {  // children past the k real ones: empty segments
    const long k = (long)tot_k[0];
    const long z0 = 2 * k * S, z1 = 2 * C * S;
    for (long i = z0 + (long)blockIdx.x * RL_THREADS + threadIdx.x; i < z1; i += (long)gridDim.x * RL_THREADS)
      tot_n[i] = 0.0;
  }
}

// hb = [bounds (2C + 1) | stats (2C x V2) | out (6C) | fsel (C)], V2 = 3 (regression: mean, n,
// variance) or S + 2 (class probabilities, n, gini / entropy)
__global__ __launch_bounds__(RL_THREADS) void rf_level_pack_kernel(const long long* __restrict__ bounds, long C,
                                                                   const double* __restrict__ tot_n, int S,
                                                                   int regression, int crit,
                                                                   const double* __restrict__ out,
                                                                   const double* __restrict__ fsel,
                                                                   double* __restrict__ hb) {
  const long rows = 2 * C;
  const int V2 = regression ? 3 : S + 2;
  const long o_st = rows + 1, o_out = o_st + rows * V2, o_fs = o_out + 6 * C, total = o_fs + C;
  for (long i = (long)blockIdx.x * RL_THREADS + threadIdx.x; i < total; i += (long)gridDim.x * RL_THREADS) {
    if (i < o_st) {
      hb[i] = (double)bounds[i];
    } else if (i < o_out) {
      const long q = i - o_st;
      const long r = q / V2;
      const int v = (int)(q - r * V2);
      const double* t = tot_n + r * S;  // S: tot_n's columns (regression: n, sum, sum of squares)
      double val;
      if (regression) {
        const double n = t[0];
        const double mu = n > 0.0 ? t[1] / n : 0.0;
        if (v == 0) val = mu;
        else if (v == 1) val = n;
        else val = n > 0.0 ? fmax(t[2] / n - mu * mu, 0.0) : 0.0;
      } else {
        double n = 0.0;
        for (int s = 0; s < S; ++s) n += t[s];
        const double safe = n > 0.0 ? n : 1.0;
        if (v < S) {
          val = n > 0.0 ? t[v] / safe : 0.0;
        } else if (v == S) {
          val = n;
        } else if (n > 0.0) {
          double a = 0.0;
          if (crit == 0) {
            for (int s = 0; s < S; ++s) a += (t[s] / safe) * (t[s] / safe);
            val = 1.0 - a;
          } else {
            for (int s = 0; s < S; ++s) {
              const double p = t[s] / safe;
              if (p > 0.0) a += p * log2(p);
            }
            val = -a;
          }
        } else {
          val = 0.0;
        }
      }
      hb[i] = val;
    } else if (i < o_fs) {
      hb[i] = out[i - o_out];
    } else {
      hb[i] = fsel[i - o_fs];
    }
  }
}

}  // namespace

// left (C x S fp64) of the winning split per candidate from its histogram (C, nslot, B, S):
// hist_f64 = 0: int32 counts, 1: fp64 sums
SRML_API int srml_rf_left_totals(const void* hist, int hist_f64, long C, int nslot, int B, int S, const double* out,
                                 double* left, hipStream_t stream) {
  if (C <= 0) return 0;
  if (nslot <= 0 || B <= 0 || S <= 0) return -2;
  const unsigned g = ceil_div(C * S, RL_THREADS);
  if (hist_f64)
    hipLaunchKernelGGL(rf_left_totals_kernel<double>, dim3(g), dim3(RL_THREADS), 0, stream,
                       reinterpret_cast<const double*>(hist), C, nslot, B, S, out, left);
  else
    hipLaunchKernelGGL(rf_left_totals_kernel<int>, dim3(g), dim3(RL_THREADS), 0, stream,
                       reinterpret_cast<const int*>(hist), C, nslot, B, S, out, left);
  return srml_status();
}

// fsel[c] = feats[c, max(out[c, 1], 0)] as fp64 (feats: int32, row stride ld)
SRML_API int srml_rf_gather_feature(const int* feats, long ld, const double* out, long C, double* fsel,
                                    hipStream_t stream) {
  if (C <= 0) return 0;
  hipLaunchKernelGGL(rf_gather_feature_kernel, dim3(ceil_div(C, RL_THREADS)), dim3(RL_THREADS), 0, stream, feats, ld,
                     out, C, fsel);
  return srml_status();
}

// The level's split decisions: pos (C int32) / k (tot_k[0]) from out[:, 1] >= 0, then the node
// arrays (pre-filled: feature -1, bin 0, child base 0; L entries indexed by cand) and, with tot_n
// (2C x S fp64), the children's totals from left (C x S) and the parents' tot (L x S).
SRML_API int srml_rf_decide(const double* out, const double* fsel, const long long* cand, long C, int* pos,
                            long long* tot_k, int* node_feature, int* node_bin, int* child_base, const double* left,
                            const double* tot, int S, double* tot_n, hipStream_t stream) {
  if (C <= 0) return 0;
  if (tot_n && (!left || !tot || S <= 0)) return -2;
  hipLaunchKernelGGL(rf_decide_scan_kernel, dim3(1), dim3(1024), 0, stream, out, C, pos, tot_k);
  hipLaunchKernelGGL(rf_decide_apply_kernel, dim3(ceil_div(C, RL_THREADS)), dim3(RL_THREADS), 0, stream, out, fsel,
                     cand, C, pos, tot_k, node_feature, node_bin, child_base, left, tot, S, tot_n);
  return srml_status();
}

// hb (fp64, 2C + 1 + 2C V2 + 7C) for the level's one read-back (see rf_level_pack_kernel)
SRML_API int srml_rf_level_pack(const long long* bounds, long C, const double* tot_n, int S, int regression, int crit,
                                const double* out, const double* fsel, double* hb, hipStream_t stream) {
  if (C <= 0) return 0;
  const int V2 = regression ? 3 : S + 2;
  const long total = 2 * C + 1 + 2 * C * V2 + 7 * C;
  long blocks = (total + RL_THREADS - 1) / RL_THREADS;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(rf_level_pack_kernel, dim3((unsigned)blocks), dim3(RL_THREADS), 0, stream, bounds, C, tot_n, S,
                     regression, crit, out, fsel, hb);
  return srml_status();
}

namespace {
// out[j, c] = start[j] + lower_bound(idx[start[j] .. start[j] + count[j]), vals[c])
__global__ __launch_bounds__(RL_THREADS) void seg_lower_bound_kernel(const int* __restrict__ idx,
                                                                     const long long* __restrict__ start,
                                                                     const long long* __restrict__ count, long nseg,
                                                                     const int* __restrict__ vals, int nv,
                                                                     long long* __restrict__ out) {
  const long i = (long)blockIdx.x * RL_THREADS + threadIdx.x;
  if (i >= nseg * nv) return;
  const long j = i / nv;
  const int c = (int)(i - j * nv);
  const int v = vals[c];
  long lo = start[j], hi = start[j] + count[j];
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (idx[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  out[i] = lo;
}
}  // namespace

// Per-segment lower bounds of nv values in ascending segments of idx (the streamed root level's
// chunk boundaries inside every tree's bootstrap rows): out (nseg x nv, int64) = global positions.
SRML_API int srml_seg_lower_bound(const int* idx, const long long* start, const long long* count, long nseg,
                                  const int* vals, int nv, long long* out, hipStream_t stream) {
  if (nseg <= 0 || nv <= 0) return 0;
  hipLaunchKernelGGL(seg_lower_bound_kernel, dim3(ceil_div(nseg * nv, RL_THREADS)), dim3(RL_THREADS), 0, stream, idx,
                     start, count, nseg, vals, nv, out);
  return srml_status();
}
