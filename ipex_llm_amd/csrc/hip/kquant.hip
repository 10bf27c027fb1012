// k-quant (q4_K / q5_K / q6_K / q2_K, GGUF super-block layouts, common/kquant.h)
// and IQ lattice (iq2_xxs / iq2_xs / iq1_s / iq1_m, common/iquant.h; codebooks in
// constant memory) decoders on gfx950: dequantize to bf16/f16 (prefill GEMM input, QLoRA
// backward) and the decode GEMV (M <= 8) straight from the GGUF blocks.
//
// Reference capability: the k-quant qtypes and the gguf_q4k_s/m mixed
// policies of SRC/transformers/utils.py:286-401 decoded by xe_linear on the
// XPU.  MI355X design: the GGUF block bytes are the device
// layout (GGUF tensors load without re-quantization; bits per weight equal
// the reference formats).  GEMV: one wave per output row; per 256-weight
// super-block each lane decodes 4 consecutive weights from ONE 32-bit code
// load (the 4 share a sub-block scale) and multiplies them against every
// activation row, the row sum is a wave reduction.  Sub-block scales are
// decoded per lane from the block header (L1-resident: 64 lanes share it).
#include <hip/hip_runtime.h>

#include "../common/kquant.h"
#include "illm_device.h"
#include "kernels.h"

namespace illm {

// the IQ codebooks (common/iq_grids.h) in constant memory
__constant__ uint64_t d_iq2xxs_grid[256] = ILLM_IQ2XXS_GRID;
__constant__ uint64_t d_iq2xs_grid[512] = ILLM_IQ2XS_GRID;
__constant__ uint64_t d_iq1s_grid[2048] = ILLM_IQ1S_GRID;

__device__ __forceinline__ float kq_h(const uint8_t* p) { return f16_to_f32(*(const uint16_t*)p); }
// q6_K blocks are 210 B: odd blocks start 2 mod 4, so its 32-bit code reads
// are assembled from two 16-bit loads (every other format is 4-B aligned)
__device__ __forceinline__ uint32_t ld32_a2(const uint8_t* p) {
  return (uint32_t)*(const uint16_t*)p | ((uint32_t)*(const uint16_t*)(p + 2) << 16);
}

// 4 consecutive weights e0..e0+3 (e0 % 4 == 0) of one super-block
template <int FMT>
__device__ __forceinline__ void kq_dec4(const uint8_t* b, int e0, float* w) {
  if constexpr (is_iq(FMT)) {
    // IQ: decode the lane's 8-weight chunk, keep its half
    float w8[8];
    const uint64_t* grid = FMT == FMT_IQ2XXS ? d_iq2xxs_grid : (FMT == FMT_IQ2XS ? d_iq2xs_grid : d_iq1s_grid);  // iq1_m: iq1_s grid
    iq_dec8(FMT, b, e0 >> 3, grid, w8);
    const int o = e0 & 4;
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = w8[o + i];
  } else if constexpr (FMT == FMT_Q4K || FMT == FMT_Q5K) {
    const int j = e0 >> 6, hi = (e0 >> 5) & 1, l = e0 & 31, sub = 2 * j + hi;
    int s, m;
    kq_scale_min_k4(sub, b + 4, &s, &m);
    const float d = kq_h(b) * s, dm = kq_h(b + 2) * m;
    const uint32_t q = *(const uint32_t*)(b + (FMT == FMT_Q5K ? 48 : 16) + 32 * j + l);
    uint32_t qh = 0;
    if constexpr (FMT == FMT_Q5K) qh = *(const uint32_t*)(b + 16 + l);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      int v = (q >> (8 * i + 4 * hi)) & 0xF;
      if constexpr (FMT == FMT_Q5K) v += ((qh >> (8 * i + sub)) & 1) << 4;
      w[i] = d * v - dm;
    }
  } else if constexpr (FMT == FMT_Q6K) {
    const int half = e0 >> 7, r = e0 & 127, quarter = r >> 5, l = r & 31;
    const uint8_t* ql = b + 64 * half;
    const uint8_t* qh = b + 128 + 32 * half;
    const int8_t* sc = (const int8_t*)(b + 192) + 8 * half;
    const float d = kq_h(b + 208) * sc[(l >> 4) + 2 * quarter];
    const uint32_t lo = ld32_a2(ql + l + ((quarter & 1) ? 32 : 0));
    const uint32_t hh = ld32_a2(qh + l);
    const int lsh = (quarter >> 1) * 4, hsh = 2 * quarter;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int v = (int)(((lo >> (8 * i + lsh)) & 0xF) | (((hh >> (8 * i + hsh)) & 3) << 4)) - 32;
      w[i] = d * v;
    }
  } else {  // q2_K
    const int half = e0 >> 7, r = e0 & 127, j = r >> 5, l32 = r & 31, hs = l32 >> 4, l = l32 & 15;
    const uint8_t sc = b[8 * half + 2 * j + hs];
    const float dl = kq_h(b + 80) * (sc & 0xF), ml = kq_h(b + 82) * (sc >> 4);
    const uint32_t q = *(const uint32_t*)(b + 16 + 32 * half + 16 * hs + l);
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = dl * ((q >> (8 * i + 2 * j)) & 3) - ml;
  }
}

template <int FMT, typename T>
__global__ void __launch_bounds__(256) kq_dequant_kernel(const uint8_t* __restrict__ w, int64_t nblocks,
                                                         uint16_t* __restrict__ out) {
  // thread -> 4 consecutive weights; 64 threads per super-block
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t blk = t >> 6;
  if (blk >= nblocks) return;
  const int e0 = (int)(t & 63) * 4;
  float v[4];
  kq_dec4<FMT>(w + blk * kq_block_bytes(FMT), e0, v);
  uint16_t* o = out + blk * QK_K + e0;
  *(uint2*)o = make_uint2(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]));
}

template <int FMT, typename T, int MM>
__global__ void __launch_bounds__(256) kq_gemv_kernel(const uint16_t* __restrict__ x, int M, int64_t K,
                                                      const uint8_t* __restrict__ w, int64_t N,
                                                      uint16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t nb = K / QK_K;
  const uint8_t* wr = w + row * nb * kq_block_bytes(FMT);
  float acc[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) acc[m] = 0.f;
  const int e0 = lane * 4;
  for (int64_t b = 0; b < nb; b++) {
    float wv[4];
    kq_dec4<FMT>(wr + b * kq_block_bytes(FMT), e0, wv);
    const int64_t k0 = b * QK_K + e0;
#pragma unroll
    for (int m = 0; m < MM; m++) {
      if (m < M) {
        const uint2 xv = *(const uint2*)(x + m * K + k0);
        acc[m] += wv[0] * to_f32<T>(xv.x & 0xffff) + wv[1] * to_f32<T>(xv.x >> 16) +
                  wv[2] * to_f32<T>(xv.y & 0xffff) + wv[3] * to_f32<T>(xv.y >> 16);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MM; m++) {
    if (m < M) {
      const float s = wave_sum(acc[m]);
      if (lane == 0) out[m * N + row] = from_f32<T>(s);
    }
  }
}

template <int FMT>
static void dq_fmt(bool bf16, const uint8_t* w, int64_t n, int64_t k, uint16_t* out, hipStream_t st) {
  const int64_t nblocks = n * (k / QK_K);
  const dim3 grid((unsigned)((nblocks * 64 + 255) / 256));
  if (bf16) hipLaunchKernelGGL((kq_dequant_kernel<FMT, BF16>), grid, dim3(256), 0, st, w, nblocks, out);
  else hipLaunchKernelGGL((kq_dequant_kernel<FMT, F16>), grid, dim3(256), 0, st, w, nblocks, out);
}

void launch_kq_dequant(int fmt, bool bf16, const uint8_t* w, int64_t n, int64_t k, uint16_t* out, hipStream_t st) {
  switch (fmt) {
    case FMT_Q4K: dq_fmt<FMT_Q4K>(bf16, w, n, k, out, st); break;
    case FMT_Q5K: dq_fmt<FMT_Q5K>(bf16, w, n, k, out, st); break;
    case FMT_Q6K: dq_fmt<FMT_Q6K>(bf16, w, n, k, out, st); break;
    case FMT_IQ2XXS: dq_fmt<FMT_IQ2XXS>(bf16, w, n, k, out, st); break;
    case FMT_IQ2XS: dq_fmt<FMT_IQ2XS>(bf16, w, n, k, out, st); break;
    case FMT_IQ1S: dq_fmt<FMT_IQ1S>(bf16, w, n, k, out, st); break;
    case FMT_IQ1M: dq_fmt<FMT_IQ1M>(bf16, w, n, k, out, st); break;
    default: dq_fmt<FMT_Q2K>(bf16, w, n, k, out, st); break;
  }
}

template <int FMT>
static void gv_fmt(bool bf16, const uint16_t* x, int M, int64_t K, const uint8_t* w, int64_t N, uint16_t* out,
                   hipStream_t st) {
  const dim3 grid((unsigned)((N + 3) / 4));
#define KQ_GV(TT, MMV) hipLaunchKernelGGL((kq_gemv_kernel<FMT, TT, MMV>), grid, dim3(256), 0, st, x, M, K, w, N, out)
  if (bf16) {
    if (M <= 1) KQ_GV(BF16, 1); else if (M <= 4) KQ_GV(BF16, 4); else KQ_GV(BF16, 8);
  } else {
    if (M <= 1) KQ_GV(F16, 1); else if (M <= 4) KQ_GV(F16, 4); else KQ_GV(F16, 8);
  }
#undef KQ_GV
}

void launch_kq_gemv(int fmt, bool bf16, const uint16_t* x, int M, int64_t K, const uint8_t* w, int64_t N,
                    uint16_t* out, hipStream_t st) {
  switch (fmt) {
    case FMT_Q4K: gv_fmt<FMT_Q4K>(bf16, x, M, K, w, N, out, st); break;
    case FMT_Q5K: gv_fmt<FMT_Q5K>(bf16, x, M, K, w, N, out, st); break;
    case FMT_Q6K: gv_fmt<FMT_Q6K>(bf16, x, M, K, w, N, out, st); break;
    case FMT_IQ2XXS: gv_fmt<FMT_IQ2XXS>(bf16, x, M, K, w, N, out, st); break;
    case FMT_IQ2XS: gv_fmt<FMT_IQ2XS>(bf16, x, M, K, w, N, out, st); break;
    case FMT_IQ1S: gv_fmt<FMT_IQ1S>(bf16, x, M, K, w, N, out, st); break;
    case FMT_IQ1M: gv_fmt<FMT_IQ1M>(bf16, x, M, K, w, N, out, st); break;
    default: gv_fmt<FMT_Q2K>(bf16, x, M, K, w, N, out, st); break;
  }
}

}  // namespace illm
