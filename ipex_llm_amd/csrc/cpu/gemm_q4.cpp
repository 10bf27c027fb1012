// Host low-bit GEMV/GEMM for the 4-bit integer formats (sym_int4 = ggml q4_0
// values, asym_int4 = q4_1) with activations quantized per 64-block to int8:
// the CPU path of LowBitLinear for decode-size M (BASELINE config "Llama-2 7B
// INT4 load_in_4bit greedy decode on CPU").
//
// Reference: ggml_compute_forward_mul_mat_q_fp32 through ctypes
// (SRC/transformers/low_bit_linear.py:494-529, llama_cpp.py:1154-1185), which
// ggml runs as q4 x q8 integer dot products in per-ISA builds (AVX2 / AVX512 /
// VNNI).  Here one source, two code paths chosen at run time:
//   * AVX-512 VNNI: the 64 codes of a block (32 packed bytes -> low nibbles =
//     elements 0..31, high = 32..63) form ONE zmm of u8, the block's int8
//     activations another; vpdpbusd gives 16 int32 partial dots, converted and
//     FMA'd with the block scale product into a 16-lane f32 accumulator (one
//     horizontal sum per output element);
//   * AVX2 (x86-64-v3 baseline): vpmaddubsw + vpmaddwd on 32-byte halves.
// The code offset / min is folded outside the integer dot:
//   sum_j (q_j d + c) x_j ~= d dx sum_j q_j xq_j + c sx,  sx = dx * sum_j xq_j
// with c = -8 d (sym_int4) or the block min (asym_int4).
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../common/formats.h"
#include "../common/quant_block.h"

using namespace illm;

namespace {

constexpr int QB = QBLOCK;   // 64

// x[m, k] f32 -> per (row, block): int8 codes, scale dx, dx * sum(codes)
void quantize_x(const float* x, int64_t m, int64_t k, int8_t* xq, float* xd, float* xs) {
  const int64_t nb = k / QB;
#pragma omp parallel for schedule(static) if (m * k > 65536)
  for (int64_t t = 0; t < m * nb; t++) {
    const float* v = x + t * QB;
    float amax = 0.f;
    for (int j = 0; j < QB; j++) amax = std::max(amax, fabsf(v[j]));
    const float d = amax / 127.f;
    const float id = d > 0.f ? 1.f / d : 0.f;
    int sum = 0;
    for (int j = 0; j < QB; j++) {
      const int q = (int)lrintf(v[j] * id);
      xq[t * QB + j] = (int8_t)q;
      sum += q;
    }
    xd[t] = d;
    xs[t] = d * (float)sum;
  }
}

// max activation rows handled per pass over a weight row (accumulators in registers)
constexpr int MR = 8;

__attribute__((target("avx512f,avx512bw,avx512vnni,avx512vl")))
void rows_avx512(int fmt, const int8_t* xq, const float* xd, const float* xs, int64_t m, const uint8_t* codes,
                 const uint16_t* scales, const uint16_t* mins, int64_t r0, int64_t r1, int64_t k, int64_t n,
                 float* y) {
  const int64_t nb = k / QB;
  const __m256i lo4 = _mm256_set1_epi8(0x0F);
  for (int64_t r = r0; r < r1; r++) {
    const uint8_t* row = codes + r * (k / 2);
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m512 acc[MR];
      float corr[MR];
      for (int i = 0; i < MR; i++) { acc[i] = _mm512_setzero_ps(); corr[i] = 0.f; }
      for (int64_t b = 0; b < nb; b++) {
        const __m256i c = _mm256_loadu_si256((const __m256i*)(row + b * 32));
        const __m256i lo = _mm256_and_si256(c, lo4);
        const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(c, 4), lo4);
        const __m512i q = _mm512_inserti64x4(_mm512_castsi256_si512(lo), hi, 1);
        const float d = hd_f16_to_f32(scales[r * nb + b]);
        const float cst = fmt == FMT_SYM_INT4 ? -8.f * d : hd_f16_to_f32(mins[r * nb + b]);
        for (int i = 0; i < mi; i++) {
          const int64_t t = (i0 + i) * nb + b;
          const __m512i xv = _mm512_loadu_si512((const void*)(xq + t * QB));
          const __m512i dp = _mm512_dpbusd_epi32(_mm512_setzero_si512(), q, xv);
          acc[i] = _mm512_fmadd_ps(_mm512_cvtepi32_ps(dp), _mm512_set1_ps(d * xd[t]), acc[i]);
          corr[i] += cst * xs[t];
        }
      }
      for (int i = 0; i < mi; i++) y[(i0 + i) * n + r] = _mm512_reduce_add_ps(acc[i]) + corr[i];
    }
  }
}

static inline float hsum256(__m256 v) {
  __m128 s = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
  s = _mm_add_ps(s, _mm_movehl_ps(s, s));
  s = _mm_add_ss(s, _mm_movehdup_ps(s));
  return _mm_cvtss_f32(s);
}

void rows_avx2(int fmt, const int8_t* xq, const float* xd, const float* xs, int64_t m, const uint8_t* codes,
               const uint16_t* scales, const uint16_t* mins, int64_t r0, int64_t r1, int64_t k, int64_t n,
               float* y) {
  const int64_t nb = k / QB;
  const __m256i lo4 = _mm256_set1_epi8(0x0F);
  const __m256i ones = _mm256_set1_epi16(1);
  for (int64_t r = r0; r < r1; r++) {
    const uint8_t* row = codes + r * (k / 2);
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m256 acc[MR];
      float corr[MR];
      for (int i = 0; i < MR; i++) { acc[i] = _mm256_setzero_ps(); corr[i] = 0.f; }
      for (int64_t b = 0; b < nb; b++) {
        const __m256i c = _mm256_loadu_si256((const __m256i*)(row + b * 32));
        const __m256i lo = _mm256_and_si256(c, lo4);
        const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(c, 4), lo4);
        const float d = hd_f16_to_f32(scales[r * nb + b]);
        const float cst = fmt == FMT_SYM_INT4 ? -8.f * d : hd_f16_to_f32(mins[r * nb + b]);
        for (int i = 0; i < mi; i++) {
          const int64_t t = (i0 + i) * nb + b;
          const __m256i x0 = _mm256_loadu_si256((const __m256i*)(xq + t * QB));
          const __m256i x1 = _mm256_loadu_si256((const __m256i*)(xq + t * QB + 32));
          // codes <= 15, |x| <= 127: the pairwise s16 sums cannot saturate
          const __m256i p = _mm256_add_epi32(_mm256_madd_epi16(_mm256_maddubs_epi16(lo, x0), ones),
                                             _mm256_madd_epi16(_mm256_maddubs_epi16(hi, x1), ones));
          acc[i] = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p), _mm256_set1_ps(d * xd[t]), acc[i]);
          corr[i] += cst * xs[t];
        }
      }
      for (int i = 0; i < mi; i++) y[(i0 + i) * n + r] = hsum256(acc[i]) + corr[i];
    }
  }
}

bool has_vnni512() {
  static const int v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                       __builtin_cpu_supports("avx512vnni");
  return v != 0;
}

}  // namespace

extern "C" {

// 1 if (fmt) has the integer-dot fast path
int illm_cpu_q4_supported(int fmt) { return fmt == FMT_SYM_INT4 || fmt == FMT_ASYM_INT4; }

// y[m, n] = x[m, k] @ W[n, k]^T, W in canonical planes of a 4-bit integer format
void illm_cpu_gemm_q4(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                      const uint16_t* mins, int64_t n, int64_t k, float* y, int isa) {
  const int64_t nb = k / QB;
  std::vector<int8_t> xq((size_t)(m * k));
  std::vector<float> xd((size_t)(m * nb)), xs((size_t)(m * nb));
  quantize_x(x, m, k, xq.data(), xd.data(), xs.data());
  const bool v512 = isa == 2 || (isa == 0 && has_vnni512());
  constexpr int64_t RB = 16;   // output rows per task
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t r1 = std::min(n, r0 + RB);
    if (v512) rows_avx512(fmt, xq.data(), xd.data(), xs.data(), m, codes, scales, mins, r0, r1, k, n, y);
    else rows_avx2(fmt, xq.data(), xd.data(), xs.data(), m, codes, scales, mins, r0, r1, k, n, y);
  }
}

}  // extern "C"
