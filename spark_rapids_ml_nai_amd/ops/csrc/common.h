// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of libsrml_ops.so.
//
// Conventions used by every kernel in this library:
//  * wave64: every cross-lane idiom is written for 64 lanes (shuffles over 64, 64-bit ballots);
//  * matrices are row-major with an explicit leading dimension (Arrow/pandas feature blocks
//    land row-major, so no transposes on ingest);
//  * every exported entry point is `extern "C"`, takes a hipStream_t, launches asynchronously
//    and returns the launch status (hipGetLastError) so the Python side can raise loudly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SRML_API extern "C" __attribute__((visibility("default")))

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef double doublex2 __attribute__((ext_vector_type(2)));
typedef double doublex4 __attribute__((ext_vector_type(4)));

static constexpr int kWave = 64;

// Wave64 all-reduce on DPP (no LDS): quad_perm swaps and row mirrors reduce within each 16-lane
// row, row_bcast:15 / row_bcast:31 fold the four rows into lane 63, readlane broadcasts the
// result as a wave-uniform value. __shfl_xor lowers to ds_bpermute (an LDS round trip per step),
// which made per-row reductions the bottleneck of the row-streaming kernels.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xf, false));
}

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xb1>(v);        // quad_perm [1,0,3,2]
  v += dpp_f<0x4e>(v);        // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);       // row_half_mirror
  v += dpp_f<0x140>(v);       // row_mirror   -> every lane holds its 16-lane row sum
  v += dpp_f<0x142, 0xa>(v);  // row_bcast:15 into rows 1,3
  v += dpp_f<0x143, 0xc>(v);  // row_bcast:31 into rows 2,3 -> lane 63 holds the total
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_d<0xb1>(v);
  v += dpp_d<0x4e>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// fast fp32 / full-precision fp64 exp and log for kernels templated on the value type
__device__ __forceinline__ float fexp(float x) { return __expf(x); }
__device__ __forceinline__ double fexp(double x) { return exp(x); }
__device__ __forceinline__ float flog(float x) { return __logf(x); }
__device__ __forceinline__ double flog(double x) { return log(x); }

// Bijective XCD-aware remap of a 1-D block id (MI355X: 8 XCDs, blocks b and b+8 share one
// XCD's L2). Consecutive *logical* ids land on the same XCD so neighbouring tiles that share
// operand panels hit in that L2 (cdna_hip_programming.md §5.5 T1, bijective variant).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int nxcd = 8;
  if (nblocks < nxcd) return bid;
  int xcd = bid % nxcd;
  int q = nblocks / nxcd, r = nblocks % nxcd;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / nxcd;
}

// Per-row logistic terms. The piecewise-linear parts of the loss (max(z,0) - y z) stay in fp64 so
// the objective is smooth for the line search; the bounded transcendental part log1p(exp(-|z|))
// and the sigmoid use the fp32 hardware exp/log (v_exp_f32 / v_log_f32): fp64 exp/log1p are long
// software sequences that made the kernel VALU-bound.
__device__ __forceinline__ void logistic_terms(double z, double y, double& res, double& loss) {
  const float zf = (float)z;
  const float e = __expf(-fabsf(zf));             // in (0, 1]
  const float p = zf >= 0.f ? 1.f / (1.f + e) : e / (1.f + e);
  res = (double)p - y;
  loss = (z > 0.0 ? z : 0.0) - y * z + (double)log1pf(e);
}

static inline int srml_status() { return (int)hipGetLastError(); }

// An AMD dispatch packet carries the grid size in WORK-ITEMS as a 32-bit field: blocks * threads
// per block must stay below 2^32 (a 1-D launch of 2^24 256-thread blocks silently covers nothing
// past that). Tile-product launches (rows x centroid tiles) are split or checked against this.
static inline long srml_max_blocks(int threads) { return 0xFFFFFFFFL / (long)threads; }

// Ordered fold of per-block partials (deterministic mode, defined in glm.hip):
// out[(i / inner) * so_outer + (i % inner) * so_inner] += sum_{p = 0..parts-1} ws[p * pstride + i], i < width,
// summed in block order so the result is bit-identical run to run; skipped once *flag != 0.
SRML_API int srml_fold_partials_f64(const double* ws, long parts, long pstride, long width, long inner, double* out,
                                    long so_outer, long so_inner, const int* flag, hipStream_t stream);

// keep the first failing HIP runtime status of a multi-call host routine in `err`
#define SRML_TRY(err, call)                                  \
  do {                                                       \
    hipError_t e_ = (call);                                  \
    if (e_ != hipSuccess && (err) == hipSuccess) (err) = e_; \
  } while (0)

static inline unsigned ceil_div(long a, long b) { return (unsigned)((a + b - 1) / b); }
