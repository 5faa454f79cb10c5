// Managed-memory allocator for the UVM mode (reference: spark.rapids.ml.uvm.enabled -> RMM managed
// memory, core.py:706-714). Plugged into a torch MemPool (CUDAPluggableAllocator ABI), so only the
// ingest buffers of an opted-in fit live in hipMallocManaged memory: partitions larger than the
// 288 GB of HBM3E page in on demand, with the owning GPU as preferred location.
#include "common.h"

SRML_API void* srml_managed_malloc(ssize_t size, int device, hipStream_t stream) {
  (void)stream;
  void* p = nullptr;
  if (size <= 0) size = 1;
  if (hipMallocManaged(&p, (size_t)size, hipMemAttachGlobal) != hipSuccess) return nullptr;
  (void)hipMemAdvise(p, (size_t)size, hipMemAdviseSetPreferredLocation, device);
  (void)hipMemAdvise(p, (size_t)size, hipMemAdviseSetAccessedBy, device);
  return p;
}

SRML_API void srml_managed_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)device;
  (void)stream;
  if (ptr) (void)hipFree(ptr);
}
