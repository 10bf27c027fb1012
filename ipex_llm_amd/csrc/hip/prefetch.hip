// Infinity-Cache (L3) warm-up: stream a byte range of a device buffer through
// the memory hierarchy and drop the data, so the next reader of that range
// hits the 256 MiB die-level cache instead of HBM (MI355X_MICROARCH.md
// "Infinity Cache": a range stays resident while it plus everything streamed
// after it fits in ~256 MiB).  The decode step uses it to pull the next
// projection's weights in while a latency-bound kernel (attention, combine,
// norm) leaves HBM bandwidth idle.
//
// Each lane keeps four 16-B loads in flight per iteration; the loaded words
// fold into one XOR that is stored (vector store) only on a value no real
// data produces in practice, so the loads cannot be dropped.
#include "illm_device.h"
#include "kernels.h"

namespace illm {

namespace {

__global__ void __launch_bounds__(256) l3_prefetch_kernel(const uint4* p, size_t n16, unsigned* sink) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t k = i + (size_t)j * 256;
      v[j] = k < n16 ? p[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  if (acc == 0x5bd1e995u) sink[threadIdx.x & 63] = acc;
}

}  // namespace

void launch_l3_prefetch(const void* p, size_t nbytes, int wgs, unsigned* sink, hipStream_t st) {
  const size_t n16 = nbytes / 16;
  if (n16 == 0) return;
  const size_t need = (n16 + 1023) / 1024;
  const unsigned g = (unsigned)std::min<size_t>(need, (size_t)std::max(1, wgs));
  hipLaunchKernelGGL(l3_prefetch_kernel, dim3(g), dim3(256), 0, st, (const uint4*)p, n16, sink);
}

}  // namespace illm
