// UMAP layout optimisation: one SGD epoch over the fuzzy-graph edges (reference: cuML UMAP
// optimize_layout, reached through umap.py:924-958 fit and 1203-1230 transform).
//
// One thread per edge, edges sorted by head vertex so neighbouring threads hit neighbouring
// embedding rows. A sampled edge pulls head and (when move_other) tail together; then it draws
// its due number of negative samples from a counter-based hash RNG (seed, epoch, edge, draw) and
// pushes the head away from them. The head row is kept in registers across the whole edge update
// (attraction + all repulsions) and committed with one atomicAdd per coordinate, the tail
// update is an atomicAdd too (Hogwild-style like the CPU/GPU references, but without lost
// updates). Gradients are clipped to [-4, 4] as in umap-learn.
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

template <int D>
__global__ __launch_bounds__(256) void umap_epoch_kernel(
    const int* __restrict__ head, const int* __restrict__ tail, long n_edges, const float* __restrict__ eps,
    float* __restrict__ next_sample, float* __restrict__ next_neg, const float* __restrict__ eps_neg,
    float* __restrict__ emb_head, float* __restrict__ emb_tail, int n_tail_vertices, int dim, float a, float b,
    float gamma, float alpha, float epoch, int move_other, unsigned seed) {
  constexpr int DM = D > 0 ? D : 32;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_edges) return;
  const float eps_e = eps[e];
  if (eps_e <= 0.f || next_sample[e] > epoch) return;
  const int dd = D > 0 ? D : dim;
  const int j = head[e], k = tail[e];
  float cur[DM], orig[DM];
  float* hj = emb_head + (long)j * dd;
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
    const float pb = __powf(dist2, b);
    coef = (-2.f * a * b * pb / dist2) / (a * pb + 1.f);
  }
#pragma unroll
  for (int d = 0; d < DM; ++d) {
    if (d < dd) {
      const float g = clip4(coef * (cur[d] - tk[d]));
      cur[d] += g * alpha;
      if (move_other) atomicAdd(&tk[d], -g * alpha);
    }
  }
  next_sample[e] += eps_e;
  const float en = eps_neg[e];
  const int n_neg = en > 0.f ? (int)((epoch - next_neg[e]) / en) : 0;
  for (int p = 0; p < n_neg; ++p) {
    const int kk = (int)(hash3(seed ^ (unsigned)e, (unsigned)epoch, (unsigned)p + 0x51ED27u * (unsigned)(e >> 32)) %
                         (unsigned)n_tail_vertices);
    const float* tn = emb_tail + (long)kk * dd;
    float d2 = 0.f;
#pragma unroll
    for (int d = 0; d < DM; ++d) {
      if (d < dd) {
        const float diff = cur[d] - tn[d];
        d2 = fmaf(diff, diff, d2);
      }
    }
    float c = 0.f;
    if (d2 > 0.f) {
      c = 2.f * gamma * b / ((0.001f + d2) * (a * __powf(d2, b) + 1.f));
    } else if (j == kk) {
      continue;
    }
#pragma unroll
    for (int d = 0; d < DM; ++d) {
      if (d < dd) {
        const float g = c > 0.f ? clip4(c * (cur[d] - tn[d])) : 4.f;
        cur[d] += g * alpha;
      }
    }
  }
  next_neg[e] += (float)n_neg * en;
#pragma unroll
  for (int d = 0; d < DM; ++d)
    if (d < dd) atomicAdd(&hj[d], cur[d] - orig[d]);
}

}  // namespace

SRML_API int srml_umap_epoch(const int* head, const int* tail, long n_edges, const float* eps, float* next_sample,
                             float* next_neg, const float* eps_neg, float* emb_head, float* emb_tail,
                             int n_tail_vertices, int dim, float a, float b, float gamma, float alpha, float epoch,
                             int move_other, unsigned seed, hipStream_t stream) {
  if (n_edges <= 0) return 0;
  if (dim < 1 || dim > 32 || n_tail_vertices < 1) return -8;
  const dim3 grid((unsigned)((n_edges + 255) / 256));
#define SRML_UMAP_LAUNCH(DD)                                                                                         \
  hipLaunchKernelGGL(umap_epoch_kernel<DD>, grid, dim3(256), 0, stream, head, tail, n_edges, eps, next_sample,       \
                     next_neg, eps_neg, emb_head, emb_tail, n_tail_vertices, dim, a, b, gamma, alpha, epoch,         \
                     move_other, seed)
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
