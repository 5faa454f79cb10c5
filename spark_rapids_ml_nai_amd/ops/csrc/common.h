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
typedef double doublex4 __attribute__((ext_vector_type(4)));

static constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

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

static inline int srml_status() { return (int)hipGetLastError(); }

static inline unsigned ceil_div(long a, long b) { return (unsigned)((a + b - 1) / b); }
