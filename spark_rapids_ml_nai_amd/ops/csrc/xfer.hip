// Small-transfer helpers for host-driven iterative solvers (L-BFGS evaluations): one
// hipMemcpyAsync on the caller's stream, without torch's per-copy pinned-block event bookkeeping
// (~40 us per copy on this stack, a sixth of a 125k-row LogisticRegression evaluation). The
// caller owns the ordering: a page-locked source is reused only after a later synchronising
// transfer on the same stream.
#include "common.h"

SRML_API int srml_memcpy_h2d_async(void* dst, const void* src, long bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, stream);
}

// device -> host, then wait for the stream (the host buffer is valid on return)
SRML_API int srml_memcpy_d2h_sync(void* dst, const void* src, long bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  hipError_t err = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, stream);
  if (err != hipSuccess) return (int)err;
  return (int)hipStreamSynchronize(stream);
}

SRML_API int srml_memset_async(void* dst, int value, long bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemsetAsync(dst, value, (size_t)bytes, stream);
}
