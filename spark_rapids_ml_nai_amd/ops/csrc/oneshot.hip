// One-shot small-message all-reduce over peer-mapped (IPC) device buffers (SURVEY §2.7 / §7.4.5;
// the latency-bound payloads of the solver loops: the LogReg gradient, KMeans k=20 sums).
//
// A ring all-reduce over xGMI costs 2(W-1) dependent link hops per call; for <= 256 KB payloads
// that latency, not bandwidth, is the cost. One-shot: every rank publishes its payload into its
// OWN uncached buffer, raises an epoch flag, waits for every peer's flag and reads all W payloads
// directly over the point-to-point links, summing them in rank order — one hop, and the result is
// bit-identical on every rank.
//
// Buffer of each rank (hipDeviceMallocUncached, IPC-exported): [flag u64 | pad to 256 B]
// [slot 0: max_elems fp64][slot 1: max_elems fp64]. Epoch e (1, 2, ...) uses slot e & 1: when a
// rank reaches epoch e every peer has raised flag >= e-1, i.e. has finished reading slot (e & 1)
// of epoch e-2, so two slots make the reuse safe without a second barrier.
// Spins are bounded: a peer that does not arrive within `timeout_cycles` sets the sticky *err, the
// output is poisoned with NaN and the kernel exits; later calls see *err, publish nothing (so the
// peers time out too) and return NaN. The host polls *err (Communicator.poll/check) and raises.
#include "common.h"

#include <string.h>

namespace {
constexpr int OS_T = 1024;
constexpr long OS_HDR = 256 / sizeof(double);  // header (flag) in doubles

template <typename T>
__global__ __launch_bounds__(OS_T) void oneshot_allreduce_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                                 long n, double* const* __restrict__ bufs,
                                                                 int world, int rank, unsigned long long epoch,
                                                                 long max_elems, long long timeout_cycles,
                                                                 int* __restrict__ err) {
  __shared__ int s_fail;
  const int t = threadIdx.x;
  if (t == 0) s_fail = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_fail) {  // sticky: a rank that already lost a peer publishes nothing and returns NaN
    for (long i = t; i < n; i += OS_T) out[i] = (T)__builtin_nan("");
    return;
  }
  double* mine = bufs[rank];
  const long slot = OS_HDR + (long)(epoch & 1ull) * max_elems;
  for (long i = t; i < n; i += OS_T) mine[slot + i] = (double)in[i];
  __threadfence_system();
  __syncthreads();
  if (t == 0)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(mine), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < world) {
    unsigned long long* f = reinterpret_cast<unsigned long long*>(bufs[t]);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (wall_clock64() - t0 > timeout_cycles) {
        atomicExch(&s_fail, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (s_fail) {  // never leave the local partial in `out`: poison it, flag the error
    for (long i = t; i < n; i += OS_T) out[i] = (T)__builtin_nan("");
    if (t == 0) atomicExch(err, 1);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  for (long i = t; i < n; i += OS_T) {
    double s = 0.0;
    for (int p = 0; p < world; ++p) s += bufs[p][slot + i];  // rank order: identical on every rank
    out[i] = (T)s;
  }
}
}  // namespace

// Allocate one rank's exchange buffer (zeroed) and export its IPC handle (64 bytes).
SRML_API int srml_oneshot_alloc(long max_elems, void** ptr, void* handle_out) {
  const size_t bytes = (size_t)(OS_HDR + 2 * max_elems) * sizeof(double);
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, *ptr);
  if (e != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

SRML_API int srml_oneshot_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

SRML_API int srml_oneshot_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

SRML_API int srml_oneshot_free(void* ptr) { return (int)hipFree(ptr); }

// out[i] = sum over ranks of in[i] (n <= max_elems); bufs: device array of the W buffer pointers
// (own buffer at index rank). dtype: 0 = fp32, 1 = fp64.
SRML_API int srml_oneshot_allreduce(const void* in, void* out, long n, int dtype, void* const* bufs, int world,
                                    int rank, unsigned long long epoch, long max_elems, long long timeout_cycles,
                                    int* err, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > max_elems || world < 1 || rank < 0 || rank >= world || epoch == 0) return -2;
  double* const* b = reinterpret_cast<double* const*>(bufs);
  if (dtype == 1)
    hipLaunchKernelGGL(oneshot_allreduce_kernel<double>, dim3(1), dim3(OS_T), 0, stream,
                       static_cast<const double*>(in), static_cast<double*>(out), n, b, world, rank, epoch, max_elems,
                       timeout_cycles, err);
  else
    hipLaunchKernelGGL(oneshot_allreduce_kernel<float>, dim3(1), dim3(OS_T), 0, stream,
                       static_cast<const float*>(in), static_cast<float*>(out), n, b, world, rank, epoch, max_elems,
                       timeout_cycles, err);
  return srml_status();
}
