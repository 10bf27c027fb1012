// Expert-parallel token dispatch / combine over xGMI peer memory (BASELINE
// config 3, Mixtral 8x7B on 8x MI355X; the reference honours vLLM's
// expert_map in its fused MoE, VLLM_PATCH:11514-11516, and has no EP of its
// own -- SURVEY §2.4).
//
// MI355X design: every rank owns one hipMalloc'd, IPC-mapped buffer
//   [signals: u32 [2 phases][EP_BLOCKS][8 src] | counts: i32 [8 src] |
//    meta: i32 [W src][cap] expert ids | recv: 16-bit [W src][cap][H] |
//    ret: 16-bit [W dst][cap][H]]
// and each (source, destination) pair owns a fixed region of the
// destination's buffer, so a source never needs the other sources' counts:
//   dispatch   the source's pairs, sorted by destination rank on the device
//              (moe_align over rank ids), are written straight into the
//              destination's recv region [src] (16-B stores over the link to
//              that peer -- EXACTLY T * k rows of H leave a rank, no padding),
//              then the pair count and a per-block epoch flag (system-scope
//              release);
//   wait/mask  the destination waits for every (source, block) flag and
//              marks region slots past each source's count as empty (-1), so
//              the grouped expert GEMM (moe_align over the meta ids + the
//              FlashMoE grouped GEMM) touches only real pairs;
//   return     each computed row goes back into the SOURCE's ret region [dst]
//              (same slot), then per-block phase-1 flags;
//   combine    the source waits, and every token sums its k returned rows
//              times the routing weights (no atomics, fixed order).
// The epoch is a device tensor advanced once per call, so the whole exchange
// is hipGraph-capturable.  Regions are reused without double-buffering: a
// rank only starts call N+1 after its combine saw every peer's call-N
// return, i.e. after every peer finished reading its recv regions.  Every
// wait is bounded: a missing peer sets ERR_PEER in the kernel error word and
// poisons the output with NaN instead of hanging or summing stale rows.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "illm_device.h"
#include "kernels_dist.h"

namespace illm {

namespace {

__device__ __forceinline__ uint32_t* ep_sig(uint8_t* base, int phase, int blk, int src) {
  return (uint32_t*)base + (phase * EP_BLOCKS + blk) * EP_MAX_RANKS + src;
}
__device__ __forceinline__ int32_t* ep_cnt(uint8_t* base) { return (int32_t*)(base + EP_SIG_BYTES); }
__device__ __forceinline__ int32_t* ep_meta(uint8_t* base) { return (int32_t*)(base + EP_SIG_BYTES + EP_CNT_BYTES); }
__device__ __forceinline__ uint16_t* ep_recv(const EpA2AArgs& a, uint8_t* base) {
  return (uint16_t*)(base + EP_SIG_BYTES + EP_CNT_BYTES + (size_t)a.world * a.cap * 4);
}
__device__ __forceinline__ uint16_t* ep_ret(const EpA2AArgs& a, uint8_t* base) {
  return ep_recv(a, base) + (size_t)a.world * a.cap * a.H;
}

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// copy one H-element 16-bit row with the block's threads (16 B each)
__device__ __forceinline__ void row_copy(uint16_t* dst, const uint16_t* src, int H) {
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) ((v4u*)dst)[v] = __builtin_nontemporal_load((const v4u*)src + v);
}

__device__ __forceinline__ bool wait_flag(uint32_t* p, uint32_t epoch, const EpA2AArgs& a) {
  // bounded by wall time (100 MHz constant clock): a peer silent for
  // a.timeout ticks is gone -- report, never hang
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
    if (wall_clock64() - t0 > a.timeout) {
      kerr(a.err, ERR_PEER);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// grid EP_BLOCKS x 256: pairs in destination order, block-strided
__global__ void __launch_bounds__(256) ep_dispatch_kernel(const EpA2AArgs a) {
  const uint32_t epoch = *a.epoch;
  const int P = a.off[a.world];            // pairs with an expert on some rank
  for (int i = blockIdx.x; i < P; i += gridDim.x) {
    const int p = a.rows[i];
    const int32_t e = a.ids[p];
    const int d = e / a.el;
    const int slot = i - a.off[d];
    uint8_t* peer = a.bufs[d];
    row_copy(ep_recv(a, peer) + ((size_t)a.rank * a.cap + slot) * a.H, a.x + (size_t)(p / a.k) * a.H, a.H);
    if (threadIdx.x == 0) {
      ep_meta(peer)[(size_t)a.rank * a.cap + slot] = e;
      a.pos[p] = i;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < a.world) {
    const int d = threadIdx.x;
    if (blockIdx.x == 0)
      __hip_atomic_store(ep_cnt(a.bufs[d]) + a.rank, a.off[d + 1] - a.off[d], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ep_sig(a.bufs[d], 0, blockIdx.x, a.rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one workgroup per source: wait for its EP_BLOCKS flags, then mark its
// region's slots past the count empty (on a timeout: the whole region)
__global__ void __launch_bounds__(256) ep_wait_mask_kernel(const EpA2AArgs a) {
  const uint32_t epoch = *a.epoch;
  const int src = blockIdx.x;
  uint8_t* own = a.bufs[a.rank];
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  if (threadIdx.x < EP_BLOCKS && !wait_flag(ep_sig(own, 0, threadIdx.x, src), epoch, a)) ok = 0;
  __syncthreads();
  const int cnt = ok ? __hip_atomic_load(ep_cnt(own) + src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
  int32_t* meta = ep_meta(own) + (size_t)src * a.cap;
  for (int64_t s = cnt + threadIdx.x; s < a.cap; s += blockDim.x) meta[s] = -1;
  if (threadIdx.x == 0) a.counts[src] = cnt;
}

// grid EP_BLOCKS x 256: computed rows (slot-indexed) back to their sources
__global__ void __launch_bounds__(256) ep_return_kernel(const EpA2AArgs a) {
  const uint32_t epoch = *a.epoch;
  int64_t total = 0;
  for (int s = 0; s < a.world; s++) total += a.counts[s];
  for (int64_t i = blockIdx.x; i < total; i += gridDim.x) {
    int64_t j = i;
    int src = 0;
    while (src < a.world - 1 && j >= a.counts[src]) j -= a.counts[src++];
    row_copy(ep_ret(a, a.bufs[src]) + ((size_t)a.rank * a.cap + j) * a.H,
             a.out_rows + ((size_t)src * a.cap + j) * a.H, a.H);
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < a.world)
    __hip_atomic_store(ep_sig(a.bufs[threadIdx.x], 1, blockIdx.x, a.rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// one workgroup: wait for every (destination, block) return flag; the result
// (1 = all arrived) goes to counts[W] for the combine
__global__ void __launch_bounds__(512) ep_wait_ret_kernel(const EpA2AArgs a) {
  const uint32_t epoch = *a.epoch;
  uint8_t* own = a.bufs[a.rank];
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  for (int f = threadIdx.x; f < a.world * EP_BLOCKS; f += blockDim.x)
    if (!wait_flag(ep_sig(own, 1, f % EP_BLOCKS, f / EP_BLOCKS), epoch, a)) ok = 0;
  __syncthreads();
  if (threadIdx.x == 0) a.counts[a.world] = ok;
}

// one workgroup per token: y[t] = sum_j w[t, j] * ret[dst_j][slot_j] (NaN
// when a peer never returned)
__global__ void __launch_bounds__(256) ep_combine_kernel(const EpA2AArgs a) {
  const int t = blockIdx.x;
  uint8_t* own = a.bufs[a.rank];
  const int ok = a.counts[a.world];
  const uint16_t* ret = ep_ret(a, own);
  for (int v = threadIdx.x; v < a.H / 8; v += blockDim.x) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < a.k; j++) {
      const int p = t * a.k + j;
      const int d = a.ids[p] / a.el;
      if (a.ids[p] < 0 || d >= a.world) continue;   // dropped by the align (ERR_EXPERT there)
      const int slot = a.pos[p] - a.off[d];
      const v4u x = __builtin_nontemporal_load((const v4u*)(ret + ((size_t)d * a.cap + slot) * a.H) + v);
      const float wt = a.w[p];
      const uint32_t u[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        s[2 * q] += wt * (a.bf16 ? bf16_to_f32(u[q] & 0xffff) : f16_to_f32(u[q] & 0xffff));
        s[2 * q + 1] += wt * (a.bf16 ? bf16_to_f32(u[q] >> 16) : f16_to_f32(u[q] >> 16));
      }
    }
    if (!ok) {
#pragma unroll
      for (int q = 0; q < 8; q++) s[q] = __builtin_nanf("");
    }
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; q++) o[q] = a.bf16 ? pack2<BF16>(s[2 * q], s[2 * q + 1]) : pack2<F16>(s[2 * q], s[2 * q + 1]);
    ((uint4*)(a.y + (size_t)t * a.H))[v] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

void launch_ep_dispatch(const EpA2AArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ep_dispatch_kernel, dim3(EP_BLOCKS), dim3(256), 0, st, a);
  hipLaunchKernelGGL(ep_wait_mask_kernel, dim3(a.world), dim3(256), 0, st, a);
}

void launch_ep_return(const EpA2AArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ep_return_kernel, dim3(EP_BLOCKS), dim3(256), 0, st, a);
}

void launch_ep_combine(const EpA2AArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(ep_wait_ret_kernel, dim3(1), dim3(512), 0, st, a);
  if (a.T > 0) hipLaunchKernelGGL(ep_combine_kernel, dim3(a.T), dim3(256), 0, st, a);
}

}  // namespace illm
