// UMAP layout optimisation: one SGD epoch over the fuzzy-graph edges (reference: cuML UMAP
// optimize_layout, reached through umap.py:924-958 fit and 1203-1230 transform).
//
// One thread per edge, edges sorted by head vertex so neighbouring threads hit neighbouring
// embedding rows. A sampled edge pulls head and (when move_other) tail together; then it draws
// its due number of negative samples from a counter-based hash RNG (seed, epoch, edge, draw) and
// pushes the head away from them. The head row is kept in registers across the whole edge update
// (attraction + all repulsions); the per-edge head deltas of one run of equal heads in a wave are
// summed by a segmented shuffle scan and committed ONCE by the run's first lane. Float atomics
// execute at the memory side (~17x slower for one-row-per-lane shapes, worse under contention),
// so the "pull" form of a symmetric graph (fit: fuzzy union = A + A^T - A.A^T has both
// directions of every pair) moves heads only, with the pair's two attraction halves applied by
// its two directed edges: no tail atomics, and a run that starts and ends inside its wave is
// committed with a plain store. Gradients are clipped to [-4, 4] as in umap-learn.
//
// Fuzzy simplicial set of a kNN graph (umap-learn smooth_knn_dist / compute_membership_strengths
// / fuzzy union; cuML UMAP's fuzzy_simplicial_set):
//  * srml_umap_smooth_knn — one thread per row: rho = local_connectivity-th smallest non-zero
//    distance (interpolated), sigma by the 64-step bisection on sum_j exp(-(d_j - rho)/sigma) =
//    log2(k)·bandwidth in fp64 (umap-learn's loop, same early exit and MIN_K_DIST_SCALE floors),
//    then the row's membership strengths written directly (self / missing neighbours -> 0);
//  * srml_umap_fuzzy_union_knn — one thread per directed edge i->c: v_ci is found by scanning
//    row c's k neighbours, the union value mix·(v + v' - v v') + (1 - mix)·v v' goes to slot 2e
//    as (i, c), and when c->i is not an edge of A (or has zero weight) the transposed entry
//    (c, i) goes to slot 2e+1, so every entry of A ∪ Aᵀ is produced exactly once, no hashing.
#include "common.h"

namespace {

__device__ __forceinline__ unsigned hash3(unsigned a, unsigned b, unsigned c) {
  // lowbias32-style mixing of three words
  unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ float clip4(float v) { return fminf(fmaxf(v, -4.f), 4.f); }

// x^b for x > 0 on the hardware log2 / exp2 (v_log_f32 / v_exp_f32): __powf lowers to the
// full-precision OCML pow (~200 instructions), which made the epoch kernel VALU-bound
__device__ __forceinline__ float fast_pow(float x, float b) {
  return __builtin_amdgcn_exp2f(b * __builtin_amdgcn_logf(x));
}

template <int D>
__global__ __launch_bounds__(256) void umap_epoch_kernel(
    const int* __restrict__ head, const int* __restrict__ tail, long n_edges, const float* __restrict__ eps,
    float* __restrict__ next_sample, float* __restrict__ next_neg, const float* __restrict__ eps_neg,
    float* __restrict__ emb_head, float* __restrict__ emb_tail, int n_tail_vertices, int dim, float a, float b,
    float gamma, float alpha, float epoch, int move_other, int pull, unsigned seed,
    const float* __restrict__ neg_tab, const int* __restrict__ neg_ids, int neg_lines) {
  constexpr int DM = D > 0 ? D : 32;
  const int lane = threadIdx.x & 63;
  // XCD-remapped: each XCD sweeps a contiguous edge range, so the head / tail rows of a
  // list-ordered graph stay in its L2
  const long e = (long)xcd_remap(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  const bool in = e < n_edges;
  const float eps_e = in ? eps[e] : 0.f;
  const bool act = eps_e > 0.f && next_sample[in ? e : 0] <= epoch;
  if (__ballot(act) == 0ull) return;  // whole wave idle this epoch (uniform exit: no lane left behind)
  const int dd = D > 0 ? D : dim;
  const int j = in ? head[e] : -1;
  float* hj = emb_head + (long)(j < 0 ? 0 : j) * dd;
  float cur[DM], orig[DM];
#pragma unroll
  for (int d = 0; d < DM; ++d) cur[d] = orig[d] = 0.f;
  if (act) {
    const int k = tail[e];
    float* tk = emb_tail + (long)k * dd;
    float dist2 = 0.f;
#pragma unroll
    for (int d = 0; d < DM; ++d) {
      if (d < dd) {
        cur[d] = hj[d];
        orig[d] = cur[d];
        const float diff = cur[d] - tk[d];
        dist2 = fmaf(diff, diff, dist2);
      }
    }
    float coef = 0.f;
    if (dist2 > 0.f) {
      const float pb = fast_pow(dist2, b);
      coef = __fdividef(-2.f * a * b * pb, dist2 * (a * pb + 1.f));
    }
    // pull: the graph holds both directions of every pair, so the reverse edge moves the tail
    // and the head takes both halves of the pair's attraction here (no tail writes at all)
    const float ascale = pull ? 2.f * alpha : alpha;
#pragma unroll
    for (int d = 0; d < DM; ++d) {
      if (d < dd) {
        const float g = clip4(coef * (cur[d] - tk[d]));
        cur[d] += g * ascale;
        if (move_other && !pull) atomicAdd(&tk[d], -g * alpha);
      }
    }
    next_sample[e] += eps_e;
    const float en = eps_neg[e];
    const int n_neg = en > 0.f ? (int)((epoch - next_neg[e]) / en) : 0;
    // negative samples: their rows depend only on the hash, so for small layouts all draws of a
    // group are loaded before any is used (one memory latency per group instead of one per draw)
    constexpr int NPF = (D > 0 && D <= 4) ? 8 : 1;
    for (int p0 = 0; p0 < n_neg; p0 += NPF) {
      float tnv[NPF][DM];
      int kkv[NPF];
#pragma unroll
      for (int q = 0; q < NPF; ++q) {
        const int p = p0 + q;
        kkv[q] = -1;
        if (p < n_neg) {
          const float* tn;
          if (neg_tab != nullptr) {
            // line-shared draw: the 8 edges e & ~7 .. e | 7 take the 8 consecutive rows of ONE
            // random 8-row line of the randomly permuted negative table (one 64 B request for
            // 8 lanes instead of 8); the rows of a line are unrelated vertices
            const unsigned h = hash3(seed ^ (unsigned)(e >> 3), (unsigned)epoch, (unsigned)p + 0x2545F491u);
            const long pos = (long)(((unsigned long long)h * (unsigned)neg_lines) >> 32) * 8 + (e & 7);
            tn = neg_tab + pos * dd;
            kkv[q] = (int)pos;  // a table position; resolved to a vertex id only on a zero distance
          } else {
            // uniform draw in [0, n): high half of hash * n (no integer division)
            const unsigned h =
                hash3(seed ^ (unsigned)e, (unsigned)epoch, (unsigned)p + 0x51ED27u * (unsigned)(e >> 32));
            kkv[q] = (int)(((unsigned long long)h * (unsigned)n_tail_vertices) >> 32);
            tn = emb_tail + (long)kkv[q] * dd;
          }
#pragma unroll
          for (int d = 0; d < DM; ++d)
            if (d < dd) tnv[q][d] = tn[d];
        }
      }
#pragma unroll
      for (int q = 0; q < NPF; ++q) {
        if (p0 + q >= n_neg) break;
        float d2 = 0.f;
#pragma unroll
        for (int d = 0; d < DM; ++d) {
          if (d < dd) {
            const float diff = cur[d] - tnv[q][d];
            d2 = fmaf(diff, diff, d2);
          }
        }
        float c = 0.f;
        if (d2 > 0.f) {
          c = __fdividef(2.f * gamma * b, (0.001f + d2) * (a * fast_pow(d2, b) + 1.f));
        } else if (j == (neg_tab != nullptr ? neg_ids[kkv[q]] : kkv[q])) {
          continue;
        }
#pragma unroll
        for (int d = 0; d < DM; ++d) {
          if (d < dd) {
            const float g = c > 0.f ? clip4(c * (cur[d] - tnv[q][d])) : 4.f;
            cur[d] += g * alpha;
          }
        }
      }
    }
    next_neg[e] += (float)n_neg * en;
  }
  // Edges are sorted by head: sum the head deltas of each run of equal heads inside the wave
  // (segmented doubling scan; runs are contiguous, so an equal head o lanes on closes the gap)
  float dl[DM];
#pragma unroll
  for (int d = 0; d < DM; ++d) dl[d] = cur[d] - orig[d];
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int jo = __shfl_down(j, o);
    const bool take = lane + o < 64 && jo == j;
#pragma unroll
    for (int d = 0; d < DM; ++d) {
      if (d < dd) {
        const float v = __shfl_down(dl[d], o);
        if (take) dl[d] += v;
      }
    }
  }
  const int jprev = __shfl_up(j, 1);
  const bool leader = j >= 0 && (lane == 0 || jprev != j);
  // does the run continue in the previous / next wave's edges?
  int jp = -2, jn = -2;
  if (lane == 0 && e > 0 && e - 1 < n_edges) jp = head[e - 1];
  if (lane == 63 && e + 1 < n_edges) jn = head[e + 1];
  jp = __shfl(jp, 0);
  jn = __shfl(jn, 63);
  const int j63 = __shfl(j, 63);
  if (!leader) return;
  bool nz = false;
#pragma unroll
  for (int d = 0; d < DM; ++d)
    if (d < dd) nz |= dl[d] != 0.f;
  if (!nz) return;
  const bool crosses = (lane == 0 && jp == j) || (j63 == j && jn == j);
  // a head is written only by its own run unless tails are moved: then one plain store per run
  if ((pull || !move_other) && !crosses) {
    if (!act) {
#pragma unroll
      for (int d = 0; d < DM; ++d)
        if (d < dd) orig[d] = hj[d];
    }
#pragma unroll
    for (int d = 0; d < DM; ++d)
      if (d < dd) hj[d] = orig[d] + dl[d];
  } else {
#pragma unroll
    for (int d = 0; d < DM; ++d)
      if (d < dd) atomicAdd(&hj[d], dl[d]);
  }
}

}  // namespace

namespace {
__global__ __launch_bounds__(256) void umap_neg_table_kernel(const float* __restrict__ emb, const int* __restrict__ ids,
                                                             long rows, int dim, float* __restrict__ tab) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * dim) return;
  const long r = i / dim;
  tab[i] = emb[(long)ids[r] * dim + (i - r * dim)];
}
}  // namespace

// tab[r] = emb[ids[r]] (rows x dim): the per-epoch snapshot of the layout in a random vertex order
// that the line-shared negative draws read (srml_umap_epoch neg_tab).
SRML_API int srml_umap_neg_table(const float* emb, const int* ids, long rows, int dim, float* tab, hipStream_t stream) {
  if (rows <= 0) return 0;
  const long tot = rows * (long)dim;
  hipLaunchKernelGGL(umap_neg_table_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, emb, ids, rows,
                     dim, tab);
  return srml_status();
}

SRML_API int srml_umap_epoch(const int* head, const int* tail, long n_edges, const float* eps, float* next_sample,
                             float* next_neg, const float* eps_neg, float* emb_head, float* emb_tail,
                             int n_tail_vertices, int dim, float a, float b, float gamma, float alpha, float epoch,
                             int move_other, int pull, unsigned seed, const float* neg_tab, const int* neg_ids,
                             int neg_lines, hipStream_t stream) {
  if (n_edges <= 0) return 0;
  if (dim < 1 || dim > 32 || n_tail_vertices < 1) return -8;
  const dim3 grid((unsigned)((n_edges + 255) / 256));
#define SRML_UMAP_LAUNCH(DD)                                                                                         \
  hipLaunchKernelGGL(umap_epoch_kernel<DD>, grid, dim3(256), 0, stream, head, tail, n_edges, eps, next_sample,       \
                     next_neg, eps_neg, emb_head, emb_tail, n_tail_vertices, dim, a, b, gamma, alpha, epoch,         \
                     move_other, pull, seed, neg_tab, neg_ids, neg_lines)
  switch (dim) {
    case 2: SRML_UMAP_LAUNCH(2); break;
    case 3: SRML_UMAP_LAUNCH(3); break;
    case 4: SRML_UMAP_LAUNCH(4); break;
    case 8: SRML_UMAP_LAUNCH(8); break;
    case 16: SRML_UMAP_LAUNCH(16); break;
    default: SRML_UMAP_LAUNCH(0); break;
  }
#undef SRML_UMAP_LAUNCH
  return srml_status();
}

// ------------------------------------------------------------------------------------------
namespace {
constexpr double SMOOTH_K_TOLERANCE = 1e-5;
constexpr double MIN_K_DIST_SCALE = 1e-3;

// t-th smallest (0-based, with multiplicity) strictly positive value of d[0..k)
__device__ double nth_positive(const float* d, int k, int t) {
  double cur = 0.0;
  int count = 0;
  while (true) {
    double nxt = __builtin_huge_val();
    for (int j = 0; j < k; ++j) {
      const double v = d[j];
      if (v > cur && v < nxt) nxt = v;
    }
    if (nxt == __builtin_huge_val()) return cur;
    int mult = 0;
    for (int j = 0; j < k; ++j) mult += ((double)d[j] == nxt) ? 1 : 0;
    if (count + mult > t) return nxt;
    count += mult;
    cur = nxt;
  }
}

__global__ __launch_bounds__(256) void umap_smooth_knn_kernel(const float* __restrict__ dist, const long long* __restrict__ idx,
                                                              long m, int k, long ld, double target, double local_conn,
                                                              int n_iter, const double* __restrict__ mean_all,
                                                              int self_rows, double* __restrict__ sigma_out,
                                                              double* __restrict__ rho_out, float* __restrict__ w) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const float* d = dist + i * ld;
  int n_nz = 0;
  double mean_row = 0.0, max_nz = 0.0;
  for (int j = 0; j < k; ++j) {
    const double v = d[j];
    mean_row += v;
    if (v > 0.0) { ++n_nz; max_nz = v > max_nz ? v : max_nz; }
  }
  mean_row /= (double)k;
  double rho = 0.0;
  const int index = (int)floor(local_conn);
  const double interp = local_conn - (double)index;
  if ((double)n_nz >= local_conn) {
    if (index > 0) {
      const double base = nth_positive(d, k, index - 1);
      rho = base;
      if (interp > SMOOTH_K_TOLERANCE && index < k) rho = base + interp * (nth_positive(d, k, index) - base);
    } else {
      rho = interp * nth_positive(d, k, 0);
    }
  } else if (n_nz > 0) {
    rho = max_nz;
  }
  double lo = 0.0, hi = __builtin_huge_val(), mid = 1.0;
  for (int it = 0; it < n_iter; ++it) {
    double psum = 0.0;
    for (int j = 1; j < k; ++j) {
      const double dd = (double)d[j] - rho;
      psum += dd > 0.0 ? exp(-(dd / mid)) : 1.0;
    }
    if (fabs(psum - target) < SMOOTH_K_TOLERANCE) break;
    if (psum > target) {
      hi = mid;
      mid = (lo + hi) * 0.5;
    } else {
      lo = mid;
      mid = (hi == __builtin_huge_val()) ? mid * 2.0 : (lo + hi) * 0.5;
    }
  }
  double sig = mid;
  const double floor_v = MIN_K_DIST_SCALE * (rho > 0.0 ? mean_row : mean_all[0]);
  if (sig < floor_v) sig = floor_v;
  sigma_out[i] = sig;
  rho_out[i] = rho;
  if (w) {
    const long long* row_idx = idx + i * ld;
    for (int j = 0; j < k; ++j) {
      const long long c = row_idx[j];
      float v;
      if (c < 0 || (self_rows && c == i)) {
        v = 0.f;
      } else {
        const double dd = (double)d[j] - rho;
        v = (dd <= 0.0 || sig == 0.0) ? 1.f : (float)exp(-(dd / sig));
      }
      w[i * ld + j] = v;
    }
  }
}

__global__ __launch_bounds__(256) void umap_fuzzy_union_knn_kernel(const long long* __restrict__ idx,
                                                                   const float* __restrict__ w, long m, int k, long ld,
                                                                   float mix, unsigned long long* __restrict__ keys,
                                                                   float* __restrict__ vals,
                                                                   unsigned long long* __restrict__ kept) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = e < m * (long)k;
  const unsigned long long none = (unsigned long long)m * (unsigned long long)m;  // sorts after every entry
  unsigned long long k0 = none, k1 = none;
  float o0 = 0.f, o1 = 0.f;
  if (live) {
    const long i = e / k;
    const int j = (int)(e % k);
    const long long c = idx[i * ld + j];
    const float v = w[i * ld + j];
    if (c >= 0 && c < m && v > 0.f) {
      float vt = 0.f;
      const long long* rc = idx + c * ld;
      for (int q = 0; q < k; ++q)
        if (rc[q] == i) { vt = w[c * ld + q]; break; }
      const float prod = v * vt;
      o0 = mix * (v + vt - prod) + (1.f - mix) * prod;
      if (o0 > 0.f) k0 = (unsigned long long)i * m + c;
      if (!(vt > 0.f)) {  // (c, i) is only in Aᵀ: emit it here
        o1 = mix * v;
        if (o1 > 0.f) k1 = (unsigned long long)c * m + i;
      }
    }
    keys[2 * e] = k0;
    keys[2 * e + 1] = k1;
    vals[2 * e] = o0;
    vals[2 * e + 1] = o1;
  }
  // emitted-entry count: one atomic per wave
  const unsigned long long n0 = __ballot(k0 != none), n1 = __ballot(k1 != none);
  if ((threadIdx.x & 63) == 0 && (n0 | n1)) atomicAdd(kept, (unsigned long long)(__popcll(n0) + __popcll(n1)));
}
}  // namespace

// dist fp32 / idx int64 [m][k] (leading dim ld); mean_all: device fp64 scalar (mean of all dist);
// outputs sigma, rho (fp64 [m]) and, when w != null, membership strengths fp32 [m][ld].
SRML_API int srml_umap_smooth_knn(const float* dist, const long long* idx, long m, int k, long ld, double target,
                                  double local_conn, int n_iter, const double* mean_all, int self_rows, double* sigma,
                                  double* rho, float* w, hipStream_t stream) {
  if (m <= 0) return 0;
  if (k < 1 || ld < k || !mean_all) return -1;
  hipLaunchKernelGGL(umap_smooth_knn_kernel, dim3(ceil_div(m, 256)), dim3(256), 0, stream, dist, idx, m, k, ld, target,
                     local_conn, n_iter, mean_all, self_rows, sigma, rho, w);
  return srml_status();
}

// keys u64 [2 m k] (row * m + col; m * m = no entry, sorting after every entry), vals fp32
// [2 m k]; *kept (zeroed by the caller) += number of entries.
SRML_API int srml_umap_fuzzy_union_knn(const long long* idx, const float* w, long m, int k, long ld, float mix,
                                       unsigned long long* keys, float* vals, unsigned long long* kept,
                                       hipStream_t stream) {
  if (m <= 0) return 0;
  if (k < 1 || ld < k || m >= (1L << 31)) return -1;
  hipLaunchKernelGGL(umap_fuzzy_union_knn_kernel, dim3(ceil_div(m * (long)k, 256)), dim3(256), 0, stream, idx, w, m, k,
                     ld, mix, keys, vals, kept);
  return srml_status();
}

// ------------------------------------------------------------------------------------------
// Supervised UMAP: categorical simplicial-set intersection on the (row, col)-sorted fuzzy union
// (umap-learn's categorical_simplicial_set_intersection + reset_local_connectivity + the second
// fuzzy union), in place of a library unique / scatter-max / coalesce. The union's pattern is
// symmetric, so every edge's transpose is found by a binary search in the other row's sorted
// column run — no re-sort, the output keeps the input pattern and order:
//   K1 row pointers (binary search per row), K2 scaled values v = w * exp(-unknown_dist) for an
//   unknown label / * exp(-far_dist) for differing labels and the per-row max (one thread per
//   row), K3 per edge a = v_ij / max_i, b = v_ji / max_j, out = mix (a + b - ab) + (1 - mix) ab.
// ------------------------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(256) void ucat_indptr_kernel(const long long* __restrict__ rows, long nnz, long N,
                                                          long long* __restrict__ indptr) {
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r <= N; r += (long)gridDim.x * 256) {
    long lo = 0, hi = nnz;
    while (lo < hi) {
      const long mid = (lo + hi) >> 1;
      if (rows[mid] < r) lo = mid + 1;
      else hi = mid;
    }
    indptr[r] = lo;
  }
}

__global__ __launch_bounds__(256) void ucat_scale_kernel(const long long* __restrict__ indptr,
                                                         const long long* __restrict__ cols,
                                                         const float* __restrict__ vals, const long long* __restrict__ y,
                                                         long N, double f_unknown, double f_far,
                                                         double* __restrict__ v, double* __restrict__ rmax) {
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < N; r += (long)gridDim.x * 256) {
    const long long yr = y[r];
    double mx = 0.0;
    for (long long e = indptr[r]; e < indptr[r + 1]; ++e) {
      const long long yc = y[cols[e]];
      double x = (double)vals[e];
      if (yr == -1 || yc == -1) x *= f_unknown;
      else if (yr != yc) x *= f_far;
      v[e] = x;
      mx = x > mx ? x : mx;
    }
    rmax[r] = mx;
  }
}

__global__ __launch_bounds__(256) void ucat_union_kernel(const long long* __restrict__ rows,
                                                         const long long* __restrict__ cols,
                                                         const long long* __restrict__ indptr,
                                                         const double* __restrict__ v, const double* __restrict__ rmax,
                                                         long nnz, double mix, float* __restrict__ out) {
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < nnz; e += (long)gridDim.x * 256) {
    const long long i = rows[e], j = cols[e];
    const double a = v[e] / (rmax[i] > 1e-30 ? rmax[i] : 1e-30);
    long long lo = indptr[j], hi = indptr[j + 1];
    while (lo < hi) {
      const long long mid = (lo + hi) >> 1;
      if (cols[mid] < i) lo = mid + 1;
      else hi = mid;
    }
    const double b = (lo < indptr[j + 1] && cols[lo] == i) ? v[lo] / (rmax[j] > 1e-30 ? rmax[j] : 1e-30) : 0.0;
    const double ab = a * b;
    out[e] = (float)(mix * (a + b - ab) + (1.0 - mix) * ab);
  }
}

inline unsigned ucat_grid(long work) {
  long b = (work + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}
}  // namespace

// rows / cols: int64 (row, col)-sorted union edges (symmetric pattern), vals fp32, y int64 labels
// (-1 unknown). out: fp32 new values (same pattern). ws: (N + 1) int64 + nnz + N fp64 (= 8-byte words).
SRML_API long srml_umap_categorical_ws(long N, long nnz) { return (N + 1) + nnz + N; }

SRML_API int srml_umap_categorical(const long long* rows, const long long* cols, const float* vals, long nnz,
                                   const long long* y, long N, double unknown_dist, double far_dist, double mix,
                                   float* out, void* ws, hipStream_t stream) {
  if (nnz <= 0 || N <= 0) return 0;
  long long* indptr = reinterpret_cast<long long*>(ws);
  double* v = reinterpret_cast<double*>(indptr + (N + 1));
  double* rmax = v + nnz;
  hipLaunchKernelGGL(ucat_indptr_kernel, dim3(ucat_grid(N + 1)), dim3(256), 0, stream, rows, nnz, N, indptr);
  hipLaunchKernelGGL(ucat_scale_kernel, dim3(ucat_grid(N)), dim3(256), 0, stream, indptr, cols, vals, y, N,
                     exp(-unknown_dist), exp(-far_dist), v, rmax);
  hipLaunchKernelGGL(ucat_union_kernel, dim3(ucat_grid(nnz)), dim3(256), 0, stream, rows, cols, indptr, v, rmax, nnz,
                     mix, out);
  return srml_status();
}
