// Peer-to-peer all-reduce over xGMI for tensor-parallel messages (row-parallel
// o_proj / down_proj outputs, including the decoder's f32 split-K
// accumulators, and MoE expert-parallel partial sums).
//
// Reference capability: the patched oneCCL "DG2 LL256" all-reduce
// (CCL_PATCH:180-830, dg2_ll256_allreduce :624, dg2_allreduce
// :809) that exchanges Level-Zero IPC handles and polls flag lines in peer
// memory.  MI355X design:
//   * every rank owns one hipMalloc'd buffer = [signal area | data p0 | data p1
//     | result p0 | result p1]; the buffers are exchanged once as
//     hipIpcMemHandles and mapped into every peer (fully connected xGMI: each
//     GPU reads its 7 peers over 7 separate links at once, which a ring cannot);
//   * ONE-SHOT (small messages, decode): block b of every rank copies its
//     slice of the input into its own data half, publishes the call's epoch
//     into slot [0][parity][b][rank] of every peer (system-scope release),
//     waits for all ranks' epochs in its own signal area and sums the slice
//     from all peers' buffers (f32 accumulation);
//   * TWO-SHOT (medium messages, prefill chunks / large batches): after the
//     same publish + wait, rank r reduces only sub-slice r of the block's
//     slice (W x fewer peer bytes per rank), writes it to its result half,
//     publishes a phase-2 epoch and gathers the W reduced sub-slices from the
//     peers' result halves: 2 (W-1)/W of the message crosses the links per
//     rank instead of (W-1);
//   * the data/result halves are double-buffered by epoch parity: a rank
//     starts call N+2 (which overwrites the halves of call N) only after every
//     peer signalled call N+1, i.e. after every peer's call-N kernel finished;
//   * epochs are device-resident per-block counters (all advanced every call),
//     so the launch is hipGraph-capturable;
//   * every wait loop is bounded (AR_TIMEOUT_S of wall time): on timeout the
//     kernel sets the communicator's flag and ERR_PEER in the device error word
//     (ops.check_kernel_errors raises) and writes NaN instead of a sum of stale
//     peer data, so a lost peer can never become a silently wrong result.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

__device__ __forceinline__ uint32_t* ar_sig(uint8_t* base, int phase, int parity, int blk, int src) {
  return (uint32_t*)base + ((phase * 2 + parity) * AR_MAX_BLOCKS + blk) * AR_MAX_RANKS + src;
}

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

// 16-byte vector -> 8 (16-bit) or 4 (f32) accumulator lanes
template <int DT>
__device__ __forceinline__ void acc_vec(float (&s)[8], u32x4v v) {
  if constexpr (DT == AR_F32) {
    s[0] += __uint_as_float(v.x); s[1] += __uint_as_float(v.y);
    s[2] += __uint_as_float(v.z); s[3] += __uint_as_float(v.w);
  } else {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if constexpr (DT == AR_BF16) {
        s[2 * i] += to_f32<BF16>((uint16_t)(w[i] & 0xffff));
        s[2 * i + 1] += to_f32<BF16>((uint16_t)(w[i] >> 16));
      } else {
        s[2 * i] += to_f32<F16>((uint16_t)(w[i] & 0xffff));
        s[2 * i + 1] += to_f32<F16>((uint16_t)(w[i] >> 16));
      }
    }
  }
}
template <int DT>
__device__ __forceinline__ uint4 pack_vec(const float (&s)[8]) {
  if constexpr (DT == AR_F32) return make_uint4(__float_as_uint(s[0]), __float_as_uint(s[1]), __float_as_uint(s[2]),
                                                __float_as_uint(s[3]));
  else if constexpr (DT == AR_BF16)
    return make_uint4(pack2<BF16>(s[0], s[1]), pack2<BF16>(s[2], s[3]), pack2<BF16>(s[4], s[5]), pack2<BF16>(s[6], s[7]));
  else return make_uint4(pack2<F16>(s[0], s[1]), pack2<F16>(s[2], s[3]), pack2<F16>(s[4], s[5]), pack2<F16>(s[6], s[7]));
}

// publish `epoch` to every rank's slot (phase, parity, b, rank); wait for all
// ranks' epochs in the own signal area.  Threads 0..W-1 take part.
// `ok` (block-shared, 1 on entry) drops to 0 when a peer stays silent.
constexpr int AR_TIMEOUT_S = 10;
template <int W>
__device__ __forceinline__ void ar_exchange(const AllReduceArgs& a, int phase, int parity, uint32_t epoch, int& ok) {
  const int tid = threadIdx.x, b = blockIdx.x;
  if (tid < W) {
    __hip_atomic_store(ar_sig(a.bufs[tid], phase, parity, b, a.rank), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mysig = ar_sig(a.bufs[a.rank], phase, parity, b, tid);
    const uint64_t t0 = wall_clock64();     // 100 MHz constant clock
    while (__hip_atomic_load(mysig, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (wall_clock64() - t0 > (uint64_t)AR_TIMEOUT_S * 100000000ull) {  // a peer is gone
        ok = 0;
        kerr(a.err, 1);
        kerr(a.kerr, ERR_PEER);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
}

template <int DT, int W>
__global__ void __launch_bounds__(AR_THREADS) peer_all_reduce(AllReduceArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint32_t epoch = a.counter[b] + 1;
  const int parity = epoch & 1;
  const int64_t per = (a.nvec + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = b * per, v1 = min(a.nvec, v0 + per);
  __shared__ int ok;
  if (tid == 0) ok = 1;

  // 1. my slice -> my data half `parity`
  u32x4v* mine = (u32x4v*)(a.bufs[a.rank] + AR_SIGNAL_BYTES + parity * a.cap);
  const u32x4v* in = (const u32x4v*)a.in;
  for (int64_t v = v0 + tid; v < v1; v += AR_THREADS) mine[v] = in[v];
  __threadfence_system();
  __syncthreads();
  ar_exchange<W>(a, 0, parity, epoch, ok);

  const u32x4v* src[W];
#pragma unroll
  for (int r = 0; r < W; r++) src[r] = (const u32x4v*)(a.bufs[r] + AR_SIGNAL_BYTES + parity * a.cap);
  auto reduce_range = [&](int64_t s0, int64_t s1, u32x4v* dst) {
    for (int64_t v = s0 + tid; v < s1; v += AR_THREADS) {
      u32x4v x[W];
#pragma unroll
      for (int r = 0; r < W; r++) x[r] = __builtin_nontemporal_load(src[r] + v);   // peer data: bypass caches
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < W; r++) acc_vec<DT>(s, x[r]);
      if (!ok) {
#pragma unroll
        for (int q = 0; q < 8; q++) s[q] = __builtin_nanf("");
      }
      const uint4 o = pack_vec<DT>(s);
      dst[v] = u32x4v{o.x, o.y, o.z, o.w};
    }
  };
  if (!a.two_shot) {
    // 2. sum the slice over all ranks (f32), 16 B per thread per step
    reduce_range(v0, v1, (u32x4v*)a.out);
  } else {
    // 2a. reduce sub-slice `rank` of this block's slice into my result half
    const int64_t sub = (v1 - v0 + W - 1) / W;
    const int64_t r0 = min(v1, v0 + a.rank * sub), r1 = min(v1, r0 + sub);
    u32x4v* res = (u32x4v*)(a.bufs[a.rank] + AR_SIGNAL_BYTES + (2 + parity) * a.cap);
    reduce_range(r0, r1, res);
    __threadfence_system();
    __syncthreads();
    ar_exchange<W>(a, 1, parity, epoch, ok);
    // 2b. gather every rank's reduced sub-slice
    u32x4v* out = (u32x4v*)a.out;
#pragma unroll
    for (int r = 0; r < W; r++) {
      const u32x4v* rr = (const u32x4v*)(a.bufs[r] + AR_SIGNAL_BYTES + (2 + parity) * a.cap);
      const int64_t g0 = min(v1, v0 + r * sub), g1 = min(v1, g0 + sub);
      for (int64_t v = g0 + tid; v < g1; v += AR_THREADS)
        out[v] = ok ? __builtin_nontemporal_load(rr + v) : u32x4v{0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
    }
  }
  // all AR_MAX_BLOCKS epochs advance every call (blocks beyond this grid are
  // advanced by block 0), so every block of a call uses the same parity
  if (tid == 0) a.counter[b] = epoch;
  if (b == 0 && tid >= (int)gridDim.x && tid < AR_MAX_BLOCKS) a.counter[tid] = epoch;
}

// all-gather over the same buffers: block b copies its slice of the local
// message into its data half, exchanges epochs (phase 0) like the all-reduce,
// then reads every rank's slice and writes it at column block r of the
// [rows, W * inner] output (last-dim concatenation, no permute afterwards)
template <int W>
__global__ void __launch_bounds__(AR_THREADS) peer_all_gather(AllReduceArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const uint32_t epoch = a.counter[b] + 1;
  const int parity = epoch & 1;
  const int64_t per = (a.nvec + gridDim.x - 1) / gridDim.x;
  const int64_t v0 = b * per, v1 = min(a.nvec, v0 + per);
  __shared__ int ok;
  if (tid == 0) ok = 1;
  u32x4v* mine = (u32x4v*)(a.bufs[a.rank] + AR_SIGNAL_BYTES + parity * a.cap);
  const u32x4v* in = (const u32x4v*)a.in;
  for (int64_t v = v0 + tid; v < v1; v += AR_THREADS) mine[v] = in[v];
  __threadfence_system();
  __syncthreads();
  ar_exchange<W>(a, 0, parity, epoch, ok);
  u32x4v* out = (u32x4v*)a.out;
  const int64_t inner = a.inner;
#pragma unroll
  for (int r = 0; r < W; r++) {
    const u32x4v* src = (const u32x4v*)(a.bufs[r] + AR_SIGNAL_BYTES + parity * a.cap);
    for (int64_t v = v0 + tid; v < v1; v += AR_THREADS) {
      const int64_t row = v / inner, c = v - row * inner;
      out[(row * W + r) * inner + c] =
          ok ? __builtin_nontemporal_load(src + v) : u32x4v{0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
    }
  }
  if (tid == 0) a.counter[b] = epoch;
  if (b == 0 && tid >= (int)gridDim.x && tid < AR_MAX_BLOCKS) a.counter[tid] = epoch;
}

int custom_all_reduce_blocks(int64_t nvec) {
  int64_t nb = (nvec + 4 * AR_THREADS - 1) / (4 * AR_THREADS);
  return (int)std::max<int64_t>(1, std::min<int64_t>(nb, AR_MAX_BLOCKS));
}

template <int DT>
static void launch_dt(const AllReduceArgs& a, int nb, hipStream_t st) {
#define ARK(WW) hipLaunchKernelGGL((peer_all_reduce<DT, WW>), dim3(nb), dim3(AR_THREADS), 0, st, a)
  switch (a.world) {
    case 1: ARK(1); break;
    case 2: ARK(2); break;
    case 3: ARK(3); break;
    case 4: ARK(4); break;
    case 5: ARK(5); break;
    case 6: ARK(6); break;
    case 7: ARK(7); break;
    default: ARK(8); break;
  }
#undef ARK
}

void launch_custom_all_reduce(const AllReduceArgs& a, hipStream_t st) {
  const int nb = custom_all_reduce_blocks(a.nvec);
  if (a.dtype == AR_F32) launch_dt<AR_F32>(a, nb, st);
  else if (a.dtype == AR_BF16) launch_dt<AR_BF16>(a, nb, st);
  else launch_dt<AR_F16>(a, nb, st);
}

void launch_custom_all_gather(const AllReduceArgs& a, hipStream_t st) {
  const int nb = custom_all_reduce_blocks(a.nvec);
#define AGK(WW) hipLaunchKernelGGL((peer_all_gather<WW>), dim3(nb), dim3(AR_THREADS), 0, st, a)
  switch (a.world) {
    case 1: AGK(1); break;
    case 2: AGK(2); break;
    case 3: AGK(3); break;
    case 4: AGK(4); break;
    case 5: AGK(5); break;
    case 6: AGK(6); break;
    case 7: AGK(7); break;
    default: AGK(8); break;
  }
#undef AGK
}

}  // namespace illm
