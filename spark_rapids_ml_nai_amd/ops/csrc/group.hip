// Grouping rows by a small integer label on the device: stable counting sort and label counts.
//
// Replaces the library sorts (rocprim radix / merge sort behind torch.sort / argsort) and
// torch.bincount (which reads the label maximum back to the host first) in the fit paths that
// group rows by cluster / IVF list: KMeans cluster sums (label-sorted segments), the k-means||
// candidate weights, the IVF list build of ApproximateNearestNeighbors and of the UMAP kNN graph,
// the class histogram of LogisticRegression.
//
// Counting sort for labels in [0, k) (k + 1 buckets: a label outside the range goes to bucket k,
// after every valid row, so a bad label cannot write out of bounds):
//   1. one wave per tile of LS_R rows: LDS histogram of the tile -> counts[l * nb + tile]
//      (label-major, so the exclusive scan of the flat matrix IS the output offset of every
//      (label, tile) pair: all tiles of label l precede every row of label l + 1);
//   2. exclusive scan of the (k + 1) * nb counts (block scans, one-block scan of the block
//      totals, add);
//   3. the same wave re-walks its tile in row order, 64 rows at a time: lanes with equal labels
//      are grouped with ballots (leader's label broadcast, peers = ballot(label == leader's)),
//      each lane's rank is the popcount of its lower peers, and the leader advances the label's
//      LDS cursor. Rows keep their order within a label: the sort is stable.
#include "common.h"

namespace {
constexpr int LS_R = 2048;        // rows per tile (one wave)
constexpr int LS_KMAX = 16383;    // k + 1 u32 cursors in 64 KiB of LDS
constexpr int GS_T = 256, GS_E = 4, GS_B = GS_T * GS_E;  // scan blocks of 1024 elements

__global__ __launch_bounds__(64) void ls_hist_kernel(const int* __restrict__ lab, long m, int k, long nb,
                                                     unsigned long long* __restrict__ cnt) {
  extern __shared__ unsigned h[];
  const int lane = threadIdx.x;
  const int kb = k + 1;
  for (int l = lane; l < kb; l += 64) h[l] = 0u;
  __syncthreads();
  const long r0 = (long)blockIdx.x * LS_R;
  const long r1 = r0 + LS_R < m ? r0 + LS_R : m;
  for (long i = r0 + lane; i < r1; i += 64) {
    const int l = lab[i];
    atomicAdd(&h[(unsigned)l < (unsigned)k ? l : k], 1u);
  }
  __syncthreads();
  for (int l = lane; l < kb; l += 64) cnt[(long)l * nb + blockIdx.x] = h[l];
}

__device__ __forceinline__ unsigned long long block_scan_excl(unsigned long long v, unsigned long long* s_w,
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
  for (int w = 0; w < GS_T / 64; ++w) {
    const unsigned long long tw = s_w[w];
    if (w < wid) base += tw;
    total += tw;
  }
  __syncthreads();
  return base + x - v;
}

// in place: a[i] <- sum_{j < i} a[j] within each 1024-element block; tot[block] = block sum
__global__ __launch_bounds__(GS_T) void gs_scan_blocks_kernel(unsigned long long* __restrict__ a, long n,
                                                              unsigned long long* __restrict__ tot) {
  __shared__ unsigned long long s_w[GS_T / 64];
  const long b0 = (long)blockIdx.x * GS_B + (long)threadIdx.x * GS_E;
  unsigned long long v[GS_E], sum = 0;
#pragma unroll
  for (int e = 0; e < GS_E; ++e) {
    v[e] = b0 + e < n ? a[b0 + e] : 0ull;
    sum += v[e];
  }
  unsigned long long total;
  unsigned long long run = block_scan_excl(sum, s_w, total);
#pragma unroll
  for (int e = 0; e < GS_E; ++e) {
    if (b0 + e < n) a[b0 + e] = run;
    run += v[e];
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = total;
}

__global__ __launch_bounds__(GS_T) void gs_scan_totals_kernel(unsigned long long* __restrict__ tot, long nb) {
  __shared__ unsigned long long s_w[GS_T / 64];
  unsigned long long carry = 0;
  for (long c0 = 0; c0 < nb; c0 += GS_T) {
    const long i = c0 + threadIdx.x;
    const unsigned long long x = i < nb ? tot[i] : 0ull;
    unsigned long long total;
    const unsigned long long ex = block_scan_excl(x, s_w, total);
    if (i < nb) tot[i] = carry + ex;
    carry += total;
  }
}

__global__ __launch_bounds__(GS_T) void gs_scan_add_kernel(unsigned long long* __restrict__ a, long n,
                                                           const unsigned long long* __restrict__ tot) {
  const long i = (long)blockIdx.x * GS_T + threadIdx.x;
  if (i < n) a[i] += tot[i / GS_B];
}

// Lanes holding the same `bits`-bit digit as this lane, among the `valid` lanes: one ballot per
// digit bit (wave-level multisplit), independent of how many distinct digits the 64 lanes hold.
__device__ __forceinline__ unsigned long long match_peers(unsigned d, bool valid, int bits) {
  unsigned long long peers = __ballot(valid);
  for (int b = 0; b < bits; ++b) {
    const bool set = (d >> b) & 1u;
    const unsigned long long B = __ballot(valid && set);
    peers &= set ? B : ~B;
  }
  return peers;
}

__global__ __launch_bounds__(64) void ls_scatter_kernel(const int* __restrict__ lab, long m, int k, long nb,
                                                        const unsigned long long* __restrict__ off,
                                                        int* __restrict__ perm, int* __restrict__ slab) {
  extern __shared__ unsigned cur[];
  const int lane = threadIdx.x;
  const int kb = k + 1;
  const int bits = 32 - __clz(k);  // buckets 0..k
  for (int l = lane; l < kb; l += 64) cur[l] = (unsigned)off[(long)l * nb + blockIdx.x];
  __syncthreads();
  const long r0 = (long)blockIdx.x * LS_R;
  const long r1 = r0 + LS_R < m ? r0 + LS_R : m;
  const unsigned long long lower = (1ull << lane) - 1ull;
  for (long c0 = r0; c0 < r1; c0 += 64) {
    const long i = c0 + lane;
    const bool valid = i < r1;
    int l = 0;
    if (valid) {
      const int v = lab[i];
      l = (unsigned)v < (unsigned)k ? v : k;
    }
    const unsigned long long peers = match_peers((unsigned)l, valid, bits);
    // every lane reads its bucket's cursor, then the lowest lane of each group advances it (the
    // reads and the writes are two in-order LDS instructions of this one wave)
    const unsigned base = valid ? cur[l] : 0u;
    if (valid && (peers & lower) == 0) cur[l] = base + (unsigned)__popcll(peers);
    if (valid) {
      const unsigned pos = base + (unsigned)__popcll(peers & lower);
      perm[pos] = (int)i;
      if (slab) slab[pos] = l;
    }
  }
}

// ---- stable LSD radix sort of (u64 key, u32 value) pairs, 8-bit digits, same tile scheme ----
constexpr int RS_R = 4096;  // elements per tile (one wave)

__global__ __launch_bounds__(64) void rs_hist_kernel(const unsigned long long* __restrict__ keys, long n, int shift,
                                                     long nb, unsigned long long* __restrict__ cnt) {
  __shared__ unsigned h[256];
  const int lane = threadIdx.x;
  for (int d = lane; d < 256; d += 64) h[d] = 0u;
  __syncthreads();
  const long r0 = (long)blockIdx.x * RS_R;
  const long r1 = r0 + RS_R < n ? r0 + RS_R : n;
  for (long i = r0 + lane; i < r1; i += 64) atomicAdd(&h[(unsigned)(keys[i] >> shift) & 255u], 1u);
  __syncthreads();
  for (int d = lane; d < 256; d += 64) cnt[(long)d * nb + blockIdx.x] = h[d];
}

__global__ __launch_bounds__(64) void rs_scatter_kernel(const unsigned long long* __restrict__ kin,
                                                        const unsigned* __restrict__ vin, long n, int shift, long nb,
                                                        const unsigned long long* __restrict__ off,
                                                        unsigned long long* __restrict__ kout,
                                                        unsigned* __restrict__ vout) {
  __shared__ unsigned long long cur[256];
  const int lane = threadIdx.x;
  for (int d = lane; d < 256; d += 64) cur[d] = off[(long)d * nb + blockIdx.x];
  __syncthreads();
  const long r0 = (long)blockIdx.x * RS_R;
  const long r1 = r0 + RS_R < n ? r0 + RS_R : n;
  const unsigned long long lower = (1ull << lane) - 1ull;
  for (long c0 = r0; c0 < r1; c0 += 64) {
    const long i = c0 + lane;
    const bool valid = i < r1;
    unsigned long long key = 0ull;
    unsigned val = 0u;
    if (valid) {
      key = kin[i];
      val = vin[i];
    }
    const unsigned d = (unsigned)(key >> shift) & 255u;
    const unsigned long long peers = match_peers(d, valid, 8);
    const unsigned long long base = valid ? cur[d] : 0ull;
    if (valid && (peers & lower) == 0) cur[d] = base + (unsigned long long)__popcll(peers);
    if (valid) {
      const unsigned long long pos = base + (unsigned long long)__popcll(peers & lower);
      kout[pos] = key;
      vout[pos] = val;
    }
  }
}

__global__ __launch_bounds__(256) void ls_offsets_kernel(const unsigned long long* __restrict__ off, int k, long nb,
                                                         long long* __restrict__ out) {
  const int l = blockIdx.x * 256 + threadIdx.x;
  if (l <= k) out[l] = (long long)off[(long)l * nb];
}

__global__ __launch_bounds__(256) void ls_count_kernel(const int* __restrict__ lab, long m, int k,
                                                       unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned h[];
  for (int l = threadIdx.x; l < k; l += 256) h[l] = 0u;
  __syncthreads();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < m; i += (long)gridDim.x * 256) {
    const int l = lab[i];
    if ((unsigned)l < (unsigned)k) atomicAdd(&h[l], 1u);
  }
  __syncthreads();
  for (int l = threadIdx.x; l < k; l += 256)
    if (h[l]) atomicAdd(&counts[l], (unsigned long long)h[l]);
}
}  // namespace

SRML_API int srml_label_sort_kmax() { return LS_KMAX - 1; }

// workspace (u64 elements) of srml_label_sort: the (k + 1) x tiles count matrix + scan totals
SRML_API long srml_label_sort_ws(long m, int k) {
  const long nb = (m + LS_R - 1) / LS_R;
  const long n = (long)(k + 1) * (nb > 0 ? nb : 1);
  return n + (n + GS_B - 1) / GS_B + 1;
}

// Stable grouping of the m labels in [0, k): perm[p] = row ids in (label, row) order, off[0..k]
// = the start of every label's run (off[k] = rows with a valid label), slab (optional) = the
// sorted labels. Rows with a label outside [0, k) follow at perm[off[k]..m).
SRML_API int srml_label_sort(const int* lab, long m, int k, int* perm, int* slab, long long* off,
                             unsigned long long* ws, hipStream_t stream) {
  if (m < 0 || k < 1 || k > LS_KMAX - 1 || m >= (1L << 31)) return -2;
  const long nb = (m + LS_R - 1) / LS_R;
  if (m == 0) return (int)hipMemsetAsync(off, 0, (size_t)(k + 1) * sizeof(long long), stream);
  const long n = (long)(k + 1) * nb;
  unsigned long long* tot = ws + n;
  const size_t lds = (size_t)(k + 1) * sizeof(unsigned);
  hipLaunchKernelGGL(ls_hist_kernel, dim3((unsigned)nb), dim3(64), lds, stream, lab, m, k, nb, ws);
  const long sb = (n + GS_B - 1) / GS_B;
  hipLaunchKernelGGL(gs_scan_blocks_kernel, dim3((unsigned)sb), dim3(GS_T), 0, stream, ws, n, tot);
  hipLaunchKernelGGL(gs_scan_totals_kernel, dim3(1), dim3(GS_T), 0, stream, tot, sb);
  hipLaunchKernelGGL(gs_scan_add_kernel, dim3(ceil_div(n, GS_T)), dim3(GS_T), 0, stream, ws, n, tot);
  hipLaunchKernelGGL(ls_scatter_kernel, dim3((unsigned)nb), dim3(64), lds, stream, lab, m, k, nb, ws, perm, slab);
  hipLaunchKernelGGL(ls_offsets_kernel, dim3(ceil_div(k + 1, 256)), dim3(256), 0, stream, ws, k, nb, off);
  return srml_status();
}

// workspace (u64 elements) of srml_radix_sort_u64 for n pairs
SRML_API long srml_radix_sort_ws(long n) {
  const long nb = (n + RS_R - 1) / RS_R;
  const long c = 256L * (nb > 0 ? nb : 1);
  return c + (c + GS_B - 1) / GS_B + 1;
}

// Stable ascending sort of n (key, value) pairs by the low `key_bits` bits of the keys (8-bit LSD
// passes; keys must be < 2^key_bits). The result is in keys / vals; keys_alt / vals_alt are
// scratch of the same sizes.
SRML_API int srml_radix_sort_u64(unsigned long long* keys, unsigned* vals, unsigned long long* keys_alt,
                                 unsigned* vals_alt, long n, int key_bits, unsigned long long* ws,
                                 hipStream_t stream) {
  if (n < 0 || key_bits < 1 || key_bits > 64) return -2;
  if (n <= 1) return 0;
  const long nb = (n + RS_R - 1) / RS_R;
  if (nb > 0x7fffffffL) return -3;
  const long c = 256L * nb;
  unsigned long long* tot = ws + c;
  const long sb = (c + GS_B - 1) / GS_B;
  unsigned long long *ki = keys, *ko = keys_alt;
  unsigned *vi = vals, *vo = vals_alt;
  for (int shift = 0; shift < key_bits; shift += 8) {
    hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)nb), dim3(64), 0, stream, ki, n, shift, nb, ws);
    hipLaunchKernelGGL(gs_scan_blocks_kernel, dim3((unsigned)sb), dim3(GS_T), 0, stream, ws, c, tot);
    hipLaunchKernelGGL(gs_scan_totals_kernel, dim3(1), dim3(GS_T), 0, stream, tot, sb);
    hipLaunchKernelGGL(gs_scan_add_kernel, dim3(ceil_div(c, GS_T)), dim3(GS_T), 0, stream, ws, c, tot);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3((unsigned)nb), dim3(64), 0, stream, ki, vi, n, shift, nb, ws, ko, vo);
    unsigned long long* tk = ki;
    ki = ko;
    ko = tk;
    unsigned* tv = vi;
    vi = vo;
    vo = tv;
  }
  if (ki != keys) {  // odd pass count: the result sits in the scratch pair
    hipError_t e = hipMemcpyAsync(keys, ki, (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(vals, vi, (size_t)n * sizeof(unsigned), hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return (int)e;
  }
  return srml_status();
}

// counts[l] += #rows with label l, l in [0, k) (u64; labels outside the range are not counted)
SRML_API int srml_label_counts(const int* lab, long m, int k, unsigned long long* counts, hipStream_t stream) {
  if (m <= 0) return 0;
  if (k < 1 || k > LS_KMAX) return -2;
  long blocks = (m + 256 * 16 - 1) / (256 * 16);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(ls_count_kernel, dim3((unsigned)blocks), dim3(256), (size_t)k * sizeof(unsigned), stream, lab, m,
                     k, counts);
  return srml_status();
}
