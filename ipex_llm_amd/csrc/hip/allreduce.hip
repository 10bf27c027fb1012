// One-shot peer-to-peer all-reduce over xGMI for small tensor-parallel
// messages (row-parallel o_proj / down_proj outputs during decode).
//
// Reference capability: the patched oneCCL "DG2 LL256" all-reduce
// (CCL_PATCH:180-830) that exchanges Level-Zero IPC handles
// and polls flag lines in peer memory.  MI355X design:
//   * every rank owns one hipMalloc'd buffer = [signal area | data half 0 |
//     data half 1]; the buffers are exchanged once as hipIpcMemHandles and
//     mapped into every peer (fully connected xGMI: each GPU reads the 7
//     peers over 7 separate links at once, which a ring cannot do);
//   * block b of every rank handles the same contiguous slice of the
//     message: it copies its slice of the input into its own buffer, then
//     stores the call's epoch into slot [parity][b][rank] of every peer's
//     signal area (system-scope release), waits for all ranks' epochs in
//     its own signal area, and sums the slice from all peers' buffers (f32
//     accumulation) into the output.  Synchronisation is therefore per block
//     slice, no grid-wide barrier is needed;
//   * the data area is double-buffered by epoch parity, so no end-of-call
//     barrier is needed: a rank can only start call N+2 (which overwrites the
//     parity of call N) after every peer signalled call N+1, i.e. after every
//     peer finished reading call N;
//   * epochs are device-resident per-block counters (all advanced every
//     call, so all blocks share one parity), so the launch is
//     hipGraph-capturable (no host-side state changes between replays);
//   * every wait loop is bounded: on timeout the kernel raises an error flag
//     and continues instead of hanging the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

__device__ __forceinline__ uint32_t* ar_sig(uint8_t* base, int parity, int blk, int src) {
  return (uint32_t*)base + (parity * AR_MAX_BLOCKS + blk) * AR_MAX_RANKS + src;
}

template <typename T>
__device__ __forceinline__ void acc_vec(float (&s)[8], uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    s[2 * i] += to_f32<T>((uint16_t)(w[i] & 0xffff));
    s[2 * i + 1] += to_f32<T>((uint16_t)(w[i] >> 16));
  }
}

template <typename T, int W>
__global__ void __launch_bounds__(AR_THREADS) one_shot_all_reduce(AllReduceArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint32_t epoch = a.counter[b] + 1;
  const int parity = epoch & 1;
  const int64_t per = (a.nvec + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = b * per, v1 = min(a.nvec, v0 + per);

  // 1. my slice -> my buffer (data half `parity`)
  uint4* mine = (uint4*)(a.bufs[a.rank] + AR_SIGNAL_BYTES + parity * a.cap);
  for (int64_t v = v0 + tid; v < v1; v += AR_THREADS) mine[v] = a.in[v];
  __threadfence_system();
  __syncthreads();

  // 2. publish the epoch to every rank; 3. wait for every rank's epoch
  if (tid < W) {
    __hip_atomic_store(ar_sig(a.bufs[tid], parity, b, a.rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mysig = ar_sig(a.bufs[a.rank], parity, b, tid);
    int64_t spins = 0;
    while (__hip_atomic_load(mysig, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (++spins > (1ll << 26)) {  // ~seconds: a peer is gone; report, do not hang
        atomicExch(a.err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();

  // 4. sum the slice over all ranks (f32), 16 B per thread per step
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* src[W];
#pragma unroll
  for (int r = 0; r < W; r++) src[r] = (const u32x4*)(a.bufs[r] + AR_SIGNAL_BYTES + parity * a.cap);
  for (int64_t v = v0 + tid; v < v1; v += AR_THREADS) {
    uint4 x[W];
#pragma unroll
    for (int r = 0; r < W; r++) {
      const u32x4 t = __builtin_nontemporal_load(src[r] + v);  // peer data: bypass stale cache lines
      x[r] = make_uint4(t.x, t.y, t.z, t.w);
    }
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < W; r++) acc_vec<T>(s, x[r]);
    a.out[v] = make_uint4(pack2<T>(s[0], s[1]), pack2<T>(s[2], s[3]), pack2<T>(s[4], s[5]),
                          pack2<T>(s[6], s[7]));
  }
  // all AR_MAX_BLOCKS epochs advance every call (blocks beyond this grid are
  // advanced by block 0), so every block of a call uses the same parity
  if (tid == 0) a.counter[b] = epoch;
  if (b == 0 && tid >= (int)gridDim.x && tid < AR_MAX_BLOCKS) a.counter[tid] = epoch;
}

int custom_all_reduce_blocks(int64_t nvec) {
  int64_t nb = (nvec + 4 * AR_THREADS - 1) / (4 * AR_THREADS);
  return (int)std::max<int64_t>(1, std::min<int64_t>(nb, AR_MAX_BLOCKS));
}

void launch_custom_all_reduce(bool bf16, const AllReduceArgs& a, hipStream_t st) {
  const int nb = custom_all_reduce_blocks(a.nvec);
#define ARK(TT, WW) hipLaunchKernelGGL((one_shot_all_reduce<TT, WW>), dim3(nb), dim3(AR_THREADS), 0, st, a)
#define ARW(TT)                       \
  switch (a.world) {                  \
    case 1: ARK(TT, 1); break;        \
    case 2: ARK(TT, 2); break;        \
    case 3: ARK(TT, 3); break;        \
    case 4: ARK(TT, 4); break;        \
    case 5: ARK(TT, 5); break;        \
    case 6: ARK(TT, 6); break;        \
    case 7: ARK(TT, 7); break;        \
    default: ARK(TT, 8); break;       \
  }
  if (bf16) { ARW(BF16) } else { ARW(F16) }
#undef ARW
#undef ARK
}

}  // namespace illm
