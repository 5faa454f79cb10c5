// Device bookkeeping of the large-k Lloyd loop (models/kmeans.py `_lloyd_f16_loop`): everything an
// iteration does besides the certified nearest-centre search and the cluster-sum kernels, so the
// loop launches only its own kernels (the torch versions were ~37 library launches per iteration:
// compare / nonzero / index_select / cat / fill / add / where / div / pow / sum / max).
//
//   * moved rows: per-block counts of rows whose label changed, one-block exclusive scan (block
//     offsets + total), then an in-order compaction into the delta update's list — moved rows as
//     `row` under their new label followed by `~row` under their old one (the sorted-sum kernel
//     subtracts a `~row`), with the per-cluster counts updated by exact fp64 +-1 atomics;
//   * counts of a full pass from the label sort's segment offsets;
//   * the inertia (sum of the fp32 squared distances) in fp64, per-block partials folded in block
//     order (bit-identical run to run);
//   * the centre update from the all-reduced [sums | counts | inertia] buffer: C = sums / counts
//     (an empty cluster keeps its centre), in place, and the largest squared centre shift (one
//     block per centre, then a one-block max) — read back together with the inertia in one copy.
// Reference behaviour: python/src/spark_rapids_ml/clustering.py:348-384 (cuML KMeans fit: Lloyd
// iterations until the centre shift falls under tol).
#include <hip/hip_runtime.h>

#include "common.h"

namespace {

constexpr int LB_THREADS = 256;
constexpr int LB_ROWS = 4 * LB_THREADS;  // rows per block of the moved-row passes
constexpr int LB_SUM_BLOCKS = 512;       // fixed grid of the inertia partials (deterministic fold)

__device__ __forceinline__ double block_sum(double v, double* ws) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) ws[wid] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += ws[w];  // fixed order
  return s;
}

__global__ __launch_bounds__(LB_THREADS) void moved_count_kernel(const int* __restrict__ lab,
                                                                 const int* __restrict__ prev, long m,
                                                                 long long* __restrict__ blk) {
  __shared__ double ws[LB_THREADS / 64];
  const long base = (long)blockIdx.x * LB_ROWS;
  int c = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long i = base + j * LB_THREADS + threadIdx.x;
    c += (i < m && lab[i] != prev[i]) ? 1 : 0;
  }
  const double s = block_sum((double)c, ws);
  if (threadIdx.x == 0) blk[blockIdx.x] = (long long)s;
}

// one 1024-thread block: blk[b] <- exclusive prefix of the block counts, tot[0] <- their total
__global__ __launch_bounds__(1024) void moved_scan_kernel(long long* __restrict__ blk, long nblk,
                                                          long long* __restrict__ tot) {
  __shared__ long long s[1024];
  const int t = threadIdx.x;
  const long per = (nblk + 1023) / 1024;
  const long a = (long)t * per, e = a + per < nblk ? a + per : nblk;
  long long sum = 0;
  for (long i = a; i < e; ++i) sum += blk[i];
  s[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const long long v = t >= o ? s[t - o] : 0;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  long long run = s[t] - sum;
  for (long i = a; i < e; ++i) {
    const long long v = blk[i];
    blk[i] = run;
    run += v;
  }
  if (t == 1023) tot[0] = s[1023];
}

// rows in ascending order: block b writes its moved rows from offset blk[b], in (pass j, lane) order
__global__ __launch_bounds__(LB_THREADS) void moved_compact_kernel(const int* __restrict__ lab,
                                                                   const int* __restrict__ prev, long m,
                                                                   const long long* __restrict__ blk, long nm,
                                                                   int* __restrict__ rows2, int* __restrict__ lab2,
                                                                   double* __restrict__ counts) {
  __shared__ int wtot[LB_THREADS / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long base = (long)blockIdx.x * LB_ROWS;
  long run = (long)blk[blockIdx.x];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long i = base + j * LB_THREADS + threadIdx.x;
    const bool mv = i < m && lab[i] != prev[i];
    const unsigned long long bal = __ballot(mv);
    if (lane == 0) wtot[wid] = __popcll(bal);
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < LB_THREADS / 64; ++w) {
      before += w < wid ? wtot[w] : 0;
      all += wtot[w];
    }
    if (mv) {
      const long p = run + before + __popcll(bal & ((1ull << lane) - 1ull));
      const int nl = lab[i], ol = prev[i];
      rows2[p] = (int)i;
      rows2[nm + p] = ~(int)i;
      lab2[p] = nl;
      lab2[nm + p] = ol;
      atomicAdd(&counts[nl], 1.0);  // exact: integer-valued fp64
      atomicAdd(&counts[ol], -1.0);
    }
    run += all;
    __syncthreads();  // wtot is rewritten by the next pass
  }
}

__global__ __launch_bounds__(LB_THREADS) void counts_from_off_kernel(const long long* __restrict__ off, int k,
                                                                     double* __restrict__ counts) {
  const int c = blockIdx.x * LB_THREADS + threadIdx.x;
  if (c < k) counts[c] = (double)(off[c + 1] - off[c]);
}

__global__ __launch_bounds__(LB_THREADS) void sum_f32_part_kernel(const float* __restrict__ x, long m,
                                                                  double* __restrict__ part) {
  __shared__ double ws[LB_THREADS / 64];
  double a = 0.0;
  for (long i = (long)blockIdx.x * LB_THREADS + threadIdx.x; i < m; i += (long)gridDim.x * LB_THREADS) a += x[i];
  const double s = block_sum(a, ws);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(LB_THREADS) void fold_sum_kernel(const double* __restrict__ part, int np,
                                                              double* __restrict__ out) {
  __shared__ double ws[LB_THREADS / 64];
  double a = 0.0;
  for (int i = threadIdx.x; i < np; i += LB_THREADS) a += part[i];
  const double s = block_sum(a, ws);
  if (threadIdx.x == 0) out[0] = s;
}

// block c: centre c <- sums / counts (kept when the cluster is empty), part[c] <- squared shift
__global__ __launch_bounds__(LB_THREADS) void centre_update_kernel(const double* __restrict__ G, int k, int n,
                                                                   double* __restrict__ C,
                                                                   double* __restrict__ part) {
  __shared__ double ws[LB_THREADS / 64];
  const int c = blockIdx.x;
  const double cnt = G[(long)k * n + c];
  const double* s = G + (long)c * n;
  double* cr = C + (long)c * n;
  double d = 0.0;
  for (int j = threadIdx.x; j < n; j += LB_THREADS) {
    const double old = cr[j];
    const double nc = cnt > 0.0 ? s[j] / cnt : old;
    d += (nc - old) * (nc - old);
    cr[j] = nc;
  }
  const double tot = block_sum(d, ws);
  if (threadIdx.x == 0) part[c] = tot;
}

// out[0] <- max squared centre shift, out[1] <- the all-reduced inertia G[k n + k]
__global__ __launch_bounds__(LB_THREADS) void shift_max_kernel(const double* __restrict__ part, int k,
                                                               const double* __restrict__ G, long kn,
                                                               double* __restrict__ out) {
  __shared__ double ws[LB_THREADS / 64];
  double v = 0.0;
  for (int i = threadIdx.x; i < k; i += LB_THREADS) v = fmax(v, part[i]);
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) ws[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0.0;
    for (int w = 0; w < LB_THREADS / 64; ++w) r = fmax(r, ws[w]);
    out[0] = r;
    out[1] = G[kn + k];
  }
}

}  // namespace

// workspace (long long elements) of srml_lloyd_moved_count for m rows
SRML_API long srml_lloyd_moved_ws(long m) { return (m + LB_ROWS - 1) / LB_ROWS; }

// Rows whose label changed (lab[i] != prev[i]): blk (srml_lloyd_moved_ws(m) elements) <- per-block
// exclusive offsets, tot[0] <- the count (device; the caller reads it back to size the update).
SRML_API int srml_lloyd_moved_count(const int* lab, const int* prev, long m, long long* blk, long long* tot,
                                    hipStream_t stream) {
  if (m <= 0 || m > 0x7FFFFFFFL) return -2;
  const long nb = (m + LB_ROWS - 1) / LB_ROWS;
  hipLaunchKernelGGL(moved_count_kernel, dim3((unsigned)nb), dim3(LB_THREADS), 0, stream, lab, prev, m, blk);
  hipLaunchKernelGGL(moved_scan_kernel, dim3(1), dim3(1024), 0, stream, blk, nb, tot);
  return srml_status();
}

// The delta update's list (after srml_lloyd_moved_count, nm = its total): rows2[0, nm) = moved
// rows ascending, rows2[nm, 2 nm) = ~ those rows; lab2 = their new / old labels; counts[k] (fp64,
// the loop's local count vector) += 1 for every new label, -= 1 for every old one.
SRML_API int srml_lloyd_moved_compact(const int* lab, const int* prev, long m, const long long* blk, long nm,
                                      int* rows2, int* lab2, double* counts, hipStream_t stream) {
  if (m <= 0 || nm <= 0) return 0;
  if (m > 0x7FFFFFFFL) return -2;
  const long nb = (m + LB_ROWS - 1) / LB_ROWS;
  hipLaunchKernelGGL(moved_compact_kernel, dim3((unsigned)nb), dim3(LB_THREADS), 0, stream, lab, prev, m, blk, nm,
                     rows2, lab2, counts);
  return srml_status();
}

// counts[c] = off[c + 1] - off[c] as fp64 (a full pass's cluster sizes from the label sort)
SRML_API int srml_counts_from_offsets(const long long* off, int k, double* counts, hipStream_t stream) {
  if (k <= 0) return 0;
  hipLaunchKernelGGL(counts_from_off_kernel, dim3(ceil_div(k, LB_THREADS)), dim3(LB_THREADS), 0, stream, off, k,
                     counts);
  return srml_status();
}

// workspace (doubles) of srml_sum_f32_f64
SRML_API long srml_sum_f32_ws() { return LB_SUM_BLOCKS; }

// out[0] = sum of x[0, m) in fp64, folded in a fixed order (part: srml_sum_f32_ws() doubles)
SRML_API int srml_sum_f32_f64(const float* x, long m, double* part, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(sum_f32_part_kernel, dim3(LB_SUM_BLOCKS), dim3(LB_THREADS), 0, stream, x, m < 0 ? 0 : m, part);
  hipLaunchKernelGGL(fold_sum_kernel, dim3(1), dim3(LB_THREADS), 0, stream, part, LB_SUM_BLOCKS, out);
  return srml_status();
}

// Centre update from the all-reduced buffer G = [sums (k x n) | counts (k) | inertia]: C (k x n
// fp64, in place) = sums / counts where counts > 0; part: k doubles; out[0] = max squared shift,
// out[1] = inertia.
SRML_API int srml_lloyd_centre_update(const double* G, int k, int n, double* C, double* part, double* out,
                                      hipStream_t stream) {
  if (k <= 0 || n <= 0) return -2;
  hipLaunchKernelGGL(centre_update_kernel, dim3((unsigned)k), dim3(LB_THREADS), 0, stream, G, k, n, C, part);
  hipLaunchKernelGGL(shift_max_kernel, dim3(1), dim3(LB_THREADS), 0, stream, part, k, G, (long)k * n, out);
  return srml_status();
}
