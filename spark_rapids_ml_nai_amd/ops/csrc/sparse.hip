// CSR (sparse-feature) kernels: the device path of LogisticRegression's sparse input mode.
//
// Reference: the reference hands a cupyx CSR matrix to cuML's QN solver when
// `enable_sparse_data_optim` is on (classification.py:957-1151, core.py:192-246); cuML then runs
// one sparse SpMV for the margins and a second transposed SpMV for the gradient, i.e. two passes
// over the non-zeros per function evaluation. Here:
//
//  * srml_csr_logreg_binary_{f32,f64} — ONE pass over the non-zeros per L-BFGS evaluation:
//        z_r = x_r . w + b ; loss += softplus(z_r) - y_r z_r ; g[col] += (sigmoid(z_r) - y_r) x_rc
//    A group of G lanes (G in {4,8,16,32,64}, picked from the mean row length) owns one row: the
//    lanes stride the row's non-zeros, reduce the dot product with intra-group shuffles, then
//    reuse the same (index, value) registers for the scatter of the gradient (fp64 atomics in
//    L2; sparse columns rarely collide within a wave). Non-zeros beyond 4*G per row are re-read.
//  * srml_csr_spmm_{f32,f64}   — Z (m x K fp32) = X W + bias, W (n x K fp32 row-major), K <= 16
//    (K > 4: one lane per output column; also the SpMM of UMAP's spectral initialisation):
//    multinomial margins for every class in one pass.
//  * srml_csr_spmtm_{f32,f64}  — out (n x K fp64) += X^T R, R (m x K fp32): multinomial gradient.
//  * srml_csr_col_moments_{f32,f64} — column sum and sum of squares (fp64) over the non-zeros
//    (standardisation statistics; zeros contribute nothing to either moment).
//
// Row offsets are int64, column indices int32 (the layout the ingest path builds from Arrow
// sparse VectorUDT columns, core/dataframe.py:vector_column_to_csr).
#include "common.h"

template <int G, typename V>
__device__ __forceinline__ V group_sum(V v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// fold one fp64 value per row group into a global accumulator (one atomic per block)
template <int GPB>
__device__ __forceinline__ void block_fold2(double a, double b, bool holder, int g, double* outa, double* outb) {
  __shared__ double red[2][GPB];
  if (holder) {
    red[0][g] = a;
    red[1][g] = b;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int i = 0; i < GPB; ++i) s += red[threadIdx.x][i];
    atomicAdd(threadIdx.x == 0 ? outa : outb, s);
  }
}

// ------------------------------------------------------------------------------------------
template <typename T, int G>
__global__ __launch_bounds__(256) void csr_logreg_binary_kernel(const long* __restrict__ indptr,
                                                                const int* __restrict__ indices,
                                                                const T* __restrict__ data, long m,
                                                                const float* __restrict__ y,
                                                                const double* __restrict__ w, double b_in,
                                                                const double* __restrict__ bptr,
                                                                const int* __restrict__ flag,
                                                                double* __restrict__ grad,
                                                                double* __restrict__ tail) {
  if (flag && *flag) return;  // on-device quasi-Newton driver finished
  const double b = bptr ? *bptr : b_in;
  constexpr int GPB = 256 / G;  // row groups per block
  constexpr int CACHE = 4;      // non-zeros per lane kept in registers between the two phases
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  double gb = 0.0, loss = 0.0;
  for (long r = (long)blockIdx.x * GPB + g; r < m; r += (long)gridDim.x * GPB) {
    const long p0 = indptr[r], p1 = indptr[r + 1];
    int ci[CACHE];
    double cv[CACHE];
    double dot = 0.0;
#pragma unroll
    for (int t = 0; t < CACHE; ++t) {
      const long p = p0 + t * G + l;
      ci[t] = -1;
      cv[t] = 0.0;
      if (p < p1) {
        ci[t] = indices[p];
        cv[t] = (double)data[p];
        dot = fma(cv[t], w[ci[t]], dot);
      }
    }
    for (long p = p0 + CACHE * G + l; p < p1; p += G) dot = fma((double)data[p], w[indices[p]], dot);
    dot = group_sum<G>(dot);
    double res, lt;
    logistic_terms(dot + b, (double)y[r], res, lt);
    if (l == 0) {
      gb += res;
      loss += lt;
    }
#pragma unroll
    for (int t = 0; t < CACHE; ++t)
      if (ci[t] >= 0) atomicAdd(&grad[ci[t]], res * cv[t]);
    for (long p = p0 + CACHE * G + l; p < p1; p += G) atomicAdd(&grad[indices[p]], res * (double)data[p]);
  }
  block_fold2<GPB>(gb, loss, l == 0, g, tail, tail + 1);
}

// ------------------------------------------------------------------------------------------
template <typename T, int G, int K>
__global__ __launch_bounds__(256) void csr_spmm_kernel(const long* __restrict__ indptr, const int* __restrict__ indices,
                                                       const T* __restrict__ data, long m,
                                                       const float* __restrict__ W, int kk,
                                                       const float* __restrict__ bias, float* __restrict__ Z,
                                                       long ldw, long ldz) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  for (long r = (long)blockIdx.x * GPB + g; r < m; r += (long)gridDim.x * GPB) {
    float acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.f;
    const long p1 = indptr[r + 1];
    for (long p = indptr[r] + l; p < p1; p += G) {
      const float v = (float)data[p];
      const float* wr = W + (long)indices[p] * ldw;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (k < kk) acc[k] = fmaf(v, wr[k], acc[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = group_sum<G>(acc[k]);
    // lane k of the group writes column k
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < kk && (k % G) == l) Z[r * ldz + k] = acc[k] + (bias ? bias[k] : 0.f);
  }
}

// Column-per-lane variant for 4 < K <= 16: a group of G >= K lanes owns one row and lane k
// accumulates output column k over the row's non-zeros (no cross-lane reduction, where the
// nnz-split kernel spent 4 shuffles per column per row). The row's (index, value) pairs are read
// G at a time, one per lane (coalesced), and handed round the group by shuffles, so the G
// W-row gathers of a chunk are independent loads in flight together instead of a chain of
// index load -> W load pairs.
template <typename T, int G>
__global__ __launch_bounds__(256) void csr_spmm_cols_kernel(const long* __restrict__ indptr,
                                                            const int* __restrict__ indices,
                                                            const T* __restrict__ data, long m,
                                                            const float* __restrict__ W, int kk,
                                                            const float* __restrict__ bias, float* __restrict__ Z,
                                                            long ldw, long ldz) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const bool act = l < kk;
  const float b0 = (bias && act) ? bias[l] : 0.f;
  // one row group per block, XCD-remapped: each XCD sweeps a contiguous row range, so the W rows
  // of a list-ordered graph's neighbours stay in that XCD's L2 (round-robin blocks spread every
  // XCD's gathers over the whole active window: 10 % L2 hits)
  {
    const long r = (long)xcd_remap(blockIdx.x, gridDim.x) * GPB + g;
    const bool rv = r < m;
    const long p0 = rv ? indptr[r] : 0, p1 = rv ? indptr[r + 1] : 0;
    float a0 = 0.f, a1 = 0.f;
    for (long base = p0; __any(base < p1); base += G) {
      const long p = base + l;
      int c = 0;
      float v = 0.f;
      if (p < p1) {
        c = indices[p];
        v = (float)data[p];
      }
#pragma unroll
      for (int s2 = 0; s2 < G; s2 += 2) {
        const int cs0 = __shfl(c, s2, G), cs1 = __shfl(c, s2 + 1, G);
        const float vs0 = __shfl(v, s2, G), vs1 = __shfl(v, s2 + 1, G);
        if (act && base + s2 < p1) a0 = fmaf(vs0, W[(long)cs0 * ldw + l], a0);
        if (act && base + s2 + 1 < p1) a1 = fmaf(vs1, W[(long)cs1 * ldw + l], a1);
      }
    }
    if (rv && act) Z[r * ldz + l] = a0 + a1 + b0;
  }
}

template <typename T, int G, int K>
__global__ __launch_bounds__(256) void csr_spmtm_kernel(const long* __restrict__ indptr, const int* __restrict__ indices,
                                                        const T* __restrict__ data, long m,
                                                        const float* __restrict__ R, int kk, double* __restrict__ out,
                                                        long ldr, long ldo) {
  constexpr int GPB = 256 / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  for (long r = (long)blockIdx.x * GPB + g; r < m; r += (long)gridDim.x * GPB) {
    float rr[K];
#pragma unroll
    for (int k = 0; k < K; ++k) rr[k] = k < kk ? R[r * ldr + k] : 0.f;
    const long p1 = indptr[r + 1];
    for (long p = indptr[r] + l; p < p1; p += G) {
      const double v = (double)data[p];
      double* o = out + (long)indices[p] * ldo;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (k < kk && rr[k] != 0.f) atomicAdd(&o[k], v * (double)rr[k]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void csr_col_moments_kernel(const int* __restrict__ indices, const T* __restrict__ data,
                                                              long nnz, double* __restrict__ s, double* __restrict__ q) {
  for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < nnz; p += (long)gridDim.x * 256) {
    const double v = (double)data[p];
    if (v != 0.0) {
      atomicAdd(&s[indices[p]], v);
      atomicAdd(&q[indices[p]], v * v);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Lanes per row: the smallest power of two >= mean nnz / 2 (so each lane handles ~2 non-zeros),
// clamped to [4, 64].
static int pick_group(long m, long nnz) {
  const double mean = m > 0 ? (double)nnz / (double)m : 0.0;
  int G = 4;
  while (G < 64 && G * 2 < mean) G <<= 1;
  return G;
}

static unsigned grid_for(long rows, int G) {
  const long groups_per_block = 256 / G;
  long blocks = (rows + groups_per_block - 1) / groups_per_block;
  if (blocks > 8192) blocks = 8192;  // grid-stride beyond 32 blocks per CU
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

template <typename T>
static int csr_logreg_launch(const long* indptr, const int* indices, const T* data, long m, long nnz, const float* y,
                             const double* w, double b, const double* bptr, const int* flag, double* grad,
                             double* tail, hipStream_t s) {
  if (m <= 0) return 0;
  const int G = pick_group(m, nnz);
  const dim3 grid(grid_for(m, G)), blk(256);
#define SRML_CSR_LR(GG)                                                                                           \
  hipLaunchKernelGGL((csr_logreg_binary_kernel<T, GG>), grid, blk, 0, s, indptr, indices, data, m, y, w, b, bptr, flag, \
                     grad, tail)
  switch (G) {
    case 4: SRML_CSR_LR(4); break;
    case 8: SRML_CSR_LR(8); break;
    case 16: SRML_CSR_LR(16); break;
    case 32: SRML_CSR_LR(32); break;
    default: SRML_CSR_LR(64); break;
  }
#undef SRML_CSR_LR
  return srml_status();
}

template <typename T, int K>
static void csr_spmm_k(int G, dim3 grid, hipStream_t s, const long* indptr, const int* indices, const T* data, long m,
                       const float* W, int kk, const float* bias, float* Z, long ldw, long ldz) {
#define SRML_CSR_MM(GG) \
  hipLaunchKernelGGL((csr_spmm_kernel<T, GG, K>), grid, dim3(256), 0, s, indptr, indices, data, m, W, kk, bias, Z, ldw, ldz)
  switch (G) {
    case 4: SRML_CSR_MM(4); break;
    case 8: SRML_CSR_MM(8); break;
    case 16: SRML_CSR_MM(16); break;
    case 32: SRML_CSR_MM(32); break;
    default: SRML_CSR_MM(64); break;
  }
#undef SRML_CSR_MM
}

template <typename T, int K>
static void csr_spmtm_k(int G, dim3 grid, hipStream_t s, const long* indptr, const int* indices, const T* data, long m,
                        const float* R, int kk, double* out, long ldr, long ldo) {
#define SRML_CSR_TM(GG) \
  hipLaunchKernelGGL((csr_spmtm_kernel<T, GG, K>), grid, dim3(256), 0, s, indptr, indices, data, m, R, kk, out, ldr, ldo)
  switch (G) {
    case 4: SRML_CSR_TM(4); break;
    case 8: SRML_CSR_TM(8); break;
    case 16: SRML_CSR_TM(16); break;
    case 32: SRML_CSR_TM(32); break;
    default: SRML_CSR_TM(64); break;
  }
#undef SRML_CSR_TM
}

template <typename T>
static int csr_spmm_launch(const long* indptr, const int* indices, const T* data, long m, long nnz, const float* W,
                           int kk, const float* bias, float* Z, long ldw, long ldz, hipStream_t s) {
  if (m <= 0) return 0;
  if (kk < 1 || kk > 16 || ldw < kk || ldz < kk) return (int)hipErrorInvalidValue;
  if (kk > 4) {  // column-per-lane groups, one block per 256 / Gc rows (no grid stride: see kernel)
    const int Gc = kk <= 8 ? 8 : 16;
    if ((m + 256 / Gc - 1) / (256 / Gc) > 0x7fffffffL) return (int)hipErrorInvalidValue;
    const dim3 gridc((unsigned)((m + 256 / Gc - 1) / (256 / Gc)));
    if (Gc == 8)
      hipLaunchKernelGGL((csr_spmm_cols_kernel<T, 8>), gridc, dim3(256), 0, s, indptr, indices, data, m, W, kk, bias, Z,
                         ldw, ldz);
    else
      hipLaunchKernelGGL((csr_spmm_cols_kernel<T, 16>), gridc, dim3(256), 0, s, indptr, indices, data, m, W, kk, bias, Z,
                         ldw, ldz);
    return srml_status();
  }
  const int G = pick_group(m, nnz);
  const dim3 grid(grid_for(m, G));
  if (kk <= 4) csr_spmm_k<T, 4>(G, grid, s, indptr, indices, data, m, W, kk, bias, Z, ldw, ldz);
  else if (kk <= 8) csr_spmm_k<T, 8>(G, grid, s, indptr, indices, data, m, W, kk, bias, Z, ldw, ldz);
  else csr_spmm_k<T, 16>(G, grid, s, indptr, indices, data, m, W, kk, bias, Z, ldw, ldz);
  return srml_status();
}

template <typename T>
static int csr_spmtm_launch(const long* indptr, const int* indices, const T* data, long m, long nnz, const float* R,
                            int kk, double* out, long ldr, long ldo, hipStream_t s) {
  if (m <= 0) return 0;
  if (kk < 1 || kk > 16 || ldr < kk || ldo < kk) return (int)hipErrorInvalidValue;
  const int G = pick_group(m, nnz);
  const dim3 grid(grid_for(m, G));
  if (kk <= 4) csr_spmtm_k<T, 4>(G, grid, s, indptr, indices, data, m, R, kk, out, ldr, ldo);
  else if (kk <= 8) csr_spmtm_k<T, 8>(G, grid, s, indptr, indices, data, m, R, kk, out, ldr, ldo);
  else csr_spmtm_k<T, 16>(G, grid, s, indptr, indices, data, m, R, kk, out, ldr, ldo);
  return srml_status();
}

template <typename T>
static int csr_moments_launch(const int* indices, const T* data, long nnz, double* sum, double* sq, hipStream_t s) {
  if (nnz <= 0) return 0;
  long blocks = (nnz + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL((csr_col_moments_kernel<T>), dim3((unsigned)blocks), dim3(256), 0, s, indices, data, nnz, sum, sq);
  return srml_status();
}

// out: [grad (n) | grad_b | loss], fp64, accumulated (caller zeroes it)
SRML_API int srml_csr_logreg_binary_f32(const long* indptr, const int* indices, const float* data, long m, int n,
                                        long nnz, const float* y, const double* w, double b, const double* bptr,
                                        const int* flag, double* out, hipStream_t s) {
  return csr_logreg_launch<float>(indptr, indices, data, m, nnz, y, w, b, bptr, flag, out, out + n, s);
}
SRML_API int srml_csr_logreg_binary_f64(const long* indptr, const int* indices, const double* data, long m, int n,
                                        long nnz, const float* y, const double* w, double b, const double* bptr,
                                        const int* flag, double* out, hipStream_t s) {
  return csr_logreg_launch<double>(indptr, indices, data, m, nnz, y, w, b, bptr, flag, out, out + n, s);
}
SRML_API int srml_csr_spmm_f32(const long* indptr, const int* indices, const float* data, long m, long nnz,
                               const float* W, int k, const float* bias, float* Z, hipStream_t s) {
  return csr_spmm_launch<float>(indptr, indices, data, m, nnz, W, k, bias, Z, k, k, s);
}
SRML_API int srml_csr_spmm_f64(const long* indptr, const int* indices, const double* data, long m, long nnz,
                               const float* W, int k, const float* bias, float* Z, hipStream_t s) {
  return csr_spmm_launch<double>(indptr, indices, data, m, nnz, W, k, bias, Z, k, k, s);
}
SRML_API int srml_csr_spmtm_f32(const long* indptr, const int* indices, const float* data, long m, long nnz,
                                const float* R, int k, double* out, hipStream_t s) {
  return csr_spmtm_launch<float>(indptr, indices, data, m, nnz, R, k, out, k, k, s);
}
SRML_API int srml_csr_spmtm_f64(const long* indptr, const int* indices, const double* data, long m, long nnz,
                                const float* R, int k, double* out, hipStream_t s) {
  return csr_spmtm_launch<double>(indptr, indices, data, m, nnz, R, k, out, k, k, s);
}
SRML_API int srml_csr_col_moments_f32(const int* indices, const float* data, long nnz, double* sum, double* sq,
                                      hipStream_t s) {
  return csr_moments_launch<float>(indices, data, nnz, sum, sq, s);
}
SRML_API int srml_csr_col_moments_f64(const int* indices, const double* data, long nnz, double* sum, double* sq,
                                      hipStream_t s) {
  return csr_moments_launch<double>(indices, data, nnz, sum, sq, s);
}

// Strided panels (K > 16 classes in 16-column panels, no gather / scatter copies): W rows of
// leading dim ldw, Z rows of leading dim ldz; R rows of leading dim ldr, out rows of ldo.
SRML_API int srml_csr_spmm_ld_f32(const long* indptr, const int* indices, const float* data, long m, long nnz,
                                  const float* W, int k, long ldw, const float* bias, float* Z, long ldz,
                                  hipStream_t s) {
  return csr_spmm_launch<float>(indptr, indices, data, m, nnz, W, k, bias, Z, ldw, ldz, s);
}
SRML_API int srml_csr_spmm_ld_f64(const long* indptr, const int* indices, const double* data, long m, long nnz,
                                  const float* W, int k, long ldw, const float* bias, float* Z, long ldz,
                                  hipStream_t s) {
  return csr_spmm_launch<double>(indptr, indices, data, m, nnz, W, k, bias, Z, ldw, ldz, s);
}
SRML_API int srml_csr_spmtm_ld_f32(const long* indptr, const int* indices, const float* data, long m, long nnz,
                                   const float* R, int k, long ldr, double* out, long ldo, hipStream_t s) {
  return csr_spmtm_launch<float>(indptr, indices, data, m, nnz, R, k, out, ldr, ldo, s);
}
SRML_API int srml_csr_spmtm_ld_f64(const long* indptr, const int* indices, const double* data, long m, long nnz,
                                   const float* R, int k, long ldr, double* out, long ldo, hipStream_t s) {
  return csr_spmtm_launch<double>(indptr, indices, data, m, nnz, R, k, out, ldr, ldo, s);
}

// Row sums of a CSR matrix, accumulated in fp64 (one thread per row, no atomics): the UMAP
// spectral-init degrees of the fuzzy graph.
template <typename T>
__global__ __launch_bounds__(256) void csr_row_sums_kernel(const long* __restrict__ indptr, const T* __restrict__ data,
                                                           long m, double* __restrict__ out) {
  for (long r = (long)blockIdx.x * 256 + threadIdx.x; r < m; r += (long)gridDim.x * 256) {
    double acc = 0.0;
    const long p1 = indptr[r + 1];
    for (long p = indptr[r]; p < p1; ++p) acc += (double)data[p];
    out[r] = acc;
  }
}

SRML_API int srml_csr_row_sums_f32(const long* indptr, const float* data, long m, double* out, hipStream_t s) {
  if (m <= 0) return 0;
  long blocks = (m + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL((csr_row_sums_kernel<float>), dim3((unsigned)blocks), dim3(256), 0, s, indptr, data, m, out);
  return srml_status();
}
