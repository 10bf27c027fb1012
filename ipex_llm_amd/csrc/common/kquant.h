// GGML k-quant super-block formats (256 weights per block), shared by the
// host quantizers (csrc/cpu/kquant.cpp) and the HIP decoders
// (csrc/hip/kquant.hip).  Byte layouts are the GGUF / llama.cpp ones, so a
// GGUF tensor of these types is used as-is (no re-quantization) and the
// bits per weight equal the reference's k-quant qtypes
// (SRC/ggml/quantize.py:28-60: q2_k = 23, q6_k = 26, q4_k = 27, q5_k = 28):
//
//   q4_K  144 B = 4.5    bpw   { f16 d, f16 dmin, u8 scales[12], u8 qs[128] }
//   q5_K  176 B = 5.5    bpw   { f16 d, f16 dmin, u8 scales[12], u8 qh[32], u8 qs[128] }
//   q6_K  210 B = 6.5625 bpw   { u8 ql[128], u8 qh[64], i8 scales[16], f16 d }
//   q2_K   84 B = 2.625  bpw   { u8 scales[16], u8 qs[64], f16 d, f16 dmin }
//
// A weight W[N, K] (K % 256 == 0) is N rows of K / 256 consecutive blocks,
// on the host and on the device alike.
#pragma once
#include <stdint.h>

#include "iquant.h"        // IQ lattice formats (15..18) share the super-block plumbing
#include "quant_block.h"   // ILLM_HD (host / host+device inline)

namespace illm {

enum KqFmt : int { FMT_Q4K = 11, FMT_Q5K = 12, FMT_Q6K = 13, FMT_Q2K = 14 };
constexpr int QK_K = 256;

// super-block formats: the k-quants and the IQ lattice formats (iquant.h)
constexpr bool is_kq(int f) { return f >= FMT_Q4K && f <= FMT_IQ1M; }
constexpr int kq_block_bytes(int f) {
  return f == FMT_Q4K ? 144 : f == FMT_Q5K ? 176 : f == FMT_Q6K ? 210 : f == FMT_Q2K ? 84 : iq_block_bytes(f);
}
constexpr int64_t kq_total_bytes(int f, int64_t n, int64_t k) { return n * (k / QK_K) * kq_block_bytes(f); }

// 6-bit (scale, min) pair j (0..7) of a q4_K / q5_K block
ILLM_HD void kq_scale_min_k4(int j, const uint8_t* q, int* d, int* m) {
  if (j < 4) {
    *d = q[j] & 63;
    *m = q[j + 4] & 63;
  } else {
    *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
    *m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
  }
}

}  // namespace illm
