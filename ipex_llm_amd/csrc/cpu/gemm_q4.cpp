// Host low-bit GEMV/GEMM: the CPU path of LowBitLinear for decode-size M
// (BASELINE config "Llama-2 7B INT4 load_in_4bit greedy decode on CPU").
//   * integer formats -- sym_int4 (ggml q4_0 values), asym_int4 (q4_1),
//     sym_int8 / sym_int5 (signed byte codes), asym_int5 (byte codes + min):
//     activations quantized per 64-block to int8, integer dot products;
//   * LUT / minifloat formats -- nf4 / fp4 / nf3 (16-entry code table) and
//     fp8_e4m3 / fp8_e5m2 / fp6: codes expanded to f32 in registers (AVX-512
//     vpermps on a one-register table, or the exponent-rebias trick for the
//     minifloats), f32 FMAs against exact f32 activations -- the dense
//     weight is never materialised.
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

// ---- 8-bit integer codes (sym_int8 / sym_int5: signed; asym_int5: unsigned + min)
// VNNI: vpdpbusd wants u8 x s8 -- signed codes are biased by 128 (c ^ 0x80)
// and the bias folds into the per-block correction: cst = -128 d.
__attribute__((target("avx512f,avx512bw,avx512vnni,avx512vl")))
void rows8_avx512(int fmt, const int8_t* xq, const float* xd, const float* xs, int64_t m, const uint8_t* codes,
                  const uint16_t* scales, const uint16_t* mins, int64_t r0, int64_t r1, int64_t k, int64_t n,
                  float* y) {
  const int64_t nb = k / QB;
  const bool sgn = fmt != FMT_ASYM_INT5;
  const __m512i bias = _mm512_set1_epi8((char)0x80);
  for (int64_t r = r0; r < r1; r++) {
    const uint8_t* row = codes + r * k;
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m512 acc[MR];
      float corr[MR];
      for (int i = 0; i < MR; i++) { acc[i] = _mm512_setzero_ps(); corr[i] = 0.f; }
      for (int64_t b = 0; b < nb; b++) {
        __m512i q = _mm512_loadu_si512((const void*)(row + b * QB));
        if (sgn) q = _mm512_xor_si512(q, bias);
        const float d = hd_f16_to_f32(scales[r * nb + b]);
        const float cst = sgn ? -128.f * d : hd_f16_to_f32(mins[r * nb + b]);
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

// AVX2: signed codes through the sign trick (|w| as u8, sign(x, w) as s8:
// pairwise s16 sums <= 2 * 128 * 127, no saturation, no correction term)
void rows8_avx2(int fmt, const int8_t* xq, const float* xd, const float* xs, int64_t m, const uint8_t* codes,
                const uint16_t* scales, const uint16_t* mins, int64_t r0, int64_t r1, int64_t k, int64_t n,
                float* y) {
  const int64_t nb = k / QB;
  const bool sgn = fmt != FMT_ASYM_INT5;
  const __m256i ones = _mm256_set1_epi16(1);
  for (int64_t r = r0; r < r1; r++) {
    const uint8_t* row = codes + r * k;
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m256 acc[MR];
      float corr[MR];
      for (int i = 0; i < MR; i++) { acc[i] = _mm256_setzero_ps(); corr[i] = 0.f; }
      for (int64_t b = 0; b < nb; b++) {
        const __m256i c0 = _mm256_loadu_si256((const __m256i*)(row + b * QB));
        const __m256i c1 = _mm256_loadu_si256((const __m256i*)(row + b * QB + 32));
        const __m256i a0 = sgn ? _mm256_sign_epi8(c0, c0) : c0, a1 = sgn ? _mm256_sign_epi8(c1, c1) : c1;
        const float d = hd_f16_to_f32(scales[r * nb + b]);
        const float cst = sgn ? 0.f : hd_f16_to_f32(mins[r * nb + b]);
        for (int i = 0; i < mi; i++) {
          const int64_t t = (i0 + i) * nb + b;
          __m256i x0 = _mm256_loadu_si256((const __m256i*)(xq + t * QB));
          __m256i x1 = _mm256_loadu_si256((const __m256i*)(xq + t * QB + 32));
          if (sgn) { x0 = _mm256_sign_epi8(x0, c0); x1 = _mm256_sign_epi8(x1, c1); }
          const __m256i p = _mm256_add_epi32(_mm256_madd_epi16(_mm256_maddubs_epi16(a0, x0), ones),
                                             _mm256_madd_epi16(_mm256_maddubs_epi16(a1, x1), ones));
          acc[i] = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p), _mm256_set1_ps(d * xd[t]), acc[i]);
          corr[i] += cst * xs[t];
        }
      }
      for (int i = 0; i < mi; i++) y[(i0 + i) * n + r] = hsum256(acc[i]) + corr[i];
    }
  }
}

// ---- LUT / minifloat codes against f32 activations
inline bool is_lut4(int fmt) { return fmt == FMT_NF4 || fmt == FMT_FP4 || fmt == FMT_NF3; }
inline bool is_mini8(int fmt) { return fmt == FMT_FP8E4 || fmt == FMT_FP8E5 || fmt == FMT_FP6; }

// 16 minifloat bytes (zero-extended to i32) -> f32: magnitude bits moved to the
// f32 exponent / mantissa field and rescaled by 2^(127 - bias) -- exact for
// normals and subnormals alike; the sign bit moved to bit 31
__attribute__((target("avx512f,avx512bw,avx512vl")))
inline __m512 mini_to_f32_512(__m512i v, bool e5m2) {
  const __m512i mag = _mm512_slli_epi32(_mm512_and_si512(v, _mm512_set1_epi32(0x7f)), e5m2 ? 21 : 20);
  const __m512 f = _mm512_mul_ps(_mm512_castsi512_ps(mag), _mm512_set1_ps(e5m2 ? 0x1p112f : 0x1p120f));
  const __m512i sg = _mm512_slli_epi32(_mm512_and_si512(v, _mm512_set1_epi32(0x80)), 24);
  return _mm512_castsi512_ps(_mm512_or_si512(_mm512_castps_si512(f), sg));
}
inline __m256 mini_to_f32_256(__m256i v, bool e5m2) {
  const __m256i mag = _mm256_slli_epi32(_mm256_and_si256(v, _mm256_set1_epi32(0x7f)), e5m2 ? 21 : 20);
  const __m256 f = _mm256_mul_ps(_mm256_castsi256_ps(mag), _mm256_set1_ps(e5m2 ? 0x1p112f : 0x1p120f));
  const __m256i sg = _mm256_slli_epi32(_mm256_and_si256(v, _mm256_set1_epi32(0x80)), 24);
  return _mm256_castsi256_ps(_mm256_or_si256(_mm256_castps_si256(f), sg));
}

__attribute__((target("avx512f,avx512bw,avx512vl")))
void rows_lut_avx512(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                     int64_t r0, int64_t r1, int64_t k, int64_t n, float* y) {
  const int64_t nb = k / QB;
  alignas(64) float lut[16];
  for (int c = 0; c < 16; c++) lut[c] = is_lut4(fmt) ? hd_lut4(fmt, c) : 0.f;
  const __m512 lz = _mm512_load_ps(lut);
  const bool e5 = fmt == FMT_FP8E5;
  for (int64_t r = r0; r < r1; r++) {
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m512 acc[MR];
      for (int i = 0; i < MR; i++) acc[i] = _mm512_setzero_ps();
      for (int64_t b = 0; b < nb; b++) {
        const __m512 d = _mm512_set1_ps(hd_f16_to_f32(scales[r * nb + b]));
        __m512 w[4];
        if (is_lut4(fmt)) {
          // 32 bytes: low nibbles = elements 0..31, high = 32..63
          const uint8_t* src = codes + r * (k / 2) + b * 32;
          const __m128i c0 = _mm_loadu_si128((const __m128i*)src), c1 = _mm_loadu_si128((const __m128i*)(src + 16));
          const __m512i i0v = _mm512_cvtepu8_epi32(c0), i1v = _mm512_cvtepu8_epi32(c1);
          const __m512i m4 = _mm512_set1_epi32(15);
          w[0] = _mm512_permutexvar_ps(_mm512_and_si512(i0v, m4), lz);
          w[1] = _mm512_permutexvar_ps(_mm512_and_si512(i1v, m4), lz);
          w[2] = _mm512_permutexvar_ps(_mm512_srli_epi32(i0v, 4), lz);
          w[3] = _mm512_permutexvar_ps(_mm512_srli_epi32(i1v, 4), lz);
        } else {
          const uint8_t* src = codes + r * k + b * QB;
          for (int q = 0; q < 4; q++)
            w[q] = mini_to_f32_512(_mm512_cvtepu8_epi32(_mm_loadu_si128((const __m128i*)(src + 16 * q))), e5);
        }
        for (int q = 0; q < 4; q++) w[q] = _mm512_mul_ps(w[q], d);
        for (int i = 0; i < mi; i++) {
          const float* xv = x + (i0 + i) * k + b * QB;
          for (int q = 0; q < 4; q++) acc[i] = _mm512_fmadd_ps(w[q], _mm512_loadu_ps(xv + 16 * q), acc[i]);
        }
      }
      for (int i = 0; i < mi; i++) y[(i0 + i) * n + r] = _mm512_reduce_add_ps(acc[i]);
    }
  }
}

void rows_lut_avx2(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                   int64_t r0, int64_t r1, int64_t k, int64_t n, float* y) {
  const int64_t nb = k / QB;
  alignas(32) float lut[16];
  for (int c = 0; c < 16; c++) lut[c] = is_lut4(fmt) ? hd_lut4(fmt, c) : 0.f;
  const __m256 llo = _mm256_load_ps(lut), lhi = _mm256_load_ps(lut + 8);
  const bool e5 = fmt == FMT_FP8E5;
  // 8 codes (i32) -> table values: vpermps on each half of the table, blend on bit 3
  auto lut8 = [&](__m256i idx) {
    const __m256 a = _mm256_permutevar8x32_ps(llo, idx), bb = _mm256_permutevar8x32_ps(lhi, idx);
    return _mm256_blendv_ps(a, bb, _mm256_castsi256_ps(_mm256_slli_epi32(idx, 28)));
  };
  for (int64_t r = r0; r < r1; r++) {
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m256 acc[MR];
      for (int i = 0; i < MR; i++) acc[i] = _mm256_setzero_ps();
      for (int64_t b = 0; b < nb; b++) {
        const __m256 d = _mm256_set1_ps(hd_f16_to_f32(scales[r * nb + b]));
        __m256 w[8];
        if (is_lut4(fmt)) {
          const uint8_t* src = codes + r * (k / 2) + b * 32;
          const __m256i m4 = _mm256_set1_epi32(15);
          for (int q = 0; q < 4; q++) {
            const __m256i iv = _mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)(src + 8 * q)));
            w[q] = lut8(_mm256_and_si256(iv, m4));                          // elements 8q .. 8q + 7
            w[4 + q] = lut8(_mm256_srli_epi32(iv, 4));                      // elements 32 + 8q ..
          }
        } else {
          const uint8_t* src = codes + r * k + b * QB;
          for (int q = 0; q < 8; q++)
            w[q] = mini_to_f32_256(_mm256_cvtepu8_epi32(_mm_loadl_epi64((const __m128i*)(src + 8 * q))), e5);
        }
        for (int q = 0; q < 8; q++) w[q] = _mm256_mul_ps(w[q], d);
        for (int i = 0; i < mi; i++) {
          const float* xv = x + (i0 + i) * k + b * QB;
          for (int q = 0; q < 8; q++) acc[i] = _mm256_fmadd_ps(w[q], _mm256_loadu_ps(xv + 8 * q), acc[i]);
        }
      }
      for (int i = 0; i < mi; i++) y[(i0 + i) * n + r] = hsum256(acc[i]);
    }
  }
}

bool has_avx512() {
  static const int v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                       __builtin_cpu_supports("avx512vl");
  return v != 0;
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
int illm_cpu_i8_supported(int fmt) { return fmt == FMT_SYM_INT8 || fmt == FMT_SYM_INT5 || fmt == FMT_ASYM_INT5; }
int illm_cpu_lut_supported(int fmt) { return is_lut4(fmt) || is_mini8(fmt); }

// y[m, n] = x[m, k] @ W[n, k]^T for the 8-bit integer formats (int8 activations)
void illm_cpu_gemm_i8(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                      const uint16_t* mins, int64_t n, int64_t k, float* y, int isa) {
  const int64_t nb = k / QB;
  std::vector<int8_t> xq((size_t)(m * k));
  std::vector<float> xd((size_t)(m * nb)), xs((size_t)(m * nb));
  quantize_x(x, m, k, xq.data(), xd.data(), xs.data());
  const bool v512 = (isa == 2 || isa == 0) && has_vnni512();   // a forced 2 on a host without VNNI runs AVX2
  constexpr int64_t RB = 16;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t r1 = std::min(n, r0 + RB);
    if (v512) rows8_avx512(fmt, xq.data(), xd.data(), xs.data(), m, codes, scales, mins, r0, r1, k, n, y);
    else rows8_avx2(fmt, xq.data(), xd.data(), xs.data(), m, codes, scales, mins, r0, r1, k, n, y);
  }
}

// y[m, n] = x[m, k] @ W[n, k]^T for the LUT / minifloat formats (f32 activations)
void illm_cpu_gemm_lut(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                       int64_t n, int64_t k, float* y, int isa) {
  const bool v512 = (isa == 2 || isa == 0) && has_avx512();
  constexpr int64_t RB = 16;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t r1 = std::min(n, r0 + RB);
    if (v512) rows_lut_avx512(fmt, x, m, codes, scales, r0, r1, k, n, y);
    else rows_lut_avx2(fmt, x, m, codes, scales, r0, r1, k, n, y);
  }
}

// y[m, n] = x[m, k] @ W[n, k]^T, W in canonical planes of a 4-bit integer format
void illm_cpu_gemm_q4(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                      const uint16_t* mins, int64_t n, int64_t k, float* y, int isa) {
  const int64_t nb = k / QB;
  std::vector<int8_t> xq((size_t)(m * k));
  std::vector<float> xd((size_t)(m * nb)), xs((size_t)(m * nb));
  quantize_x(x, m, k, xq.data(), xd.data(), xs.data());
  const bool v512 = (isa == 2 || isa == 0) && has_vnni512();   // a forced 2 on a host without VNNI runs AVX2
  constexpr int64_t RB = 16;   // output rows per task
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t r1 = std::min(n, r0 + RB);
    if (v512) rows_avx512(fmt, xq.data(), xd.data(), xs.data(), m, codes, scales, mins, r0, r1, k, n, y);
    else rows_avx2(fmt, xq.data(), xd.data(), xs.data(), m, codes, scales, mins, r0, r1, k, n, y);
  }
}

}  // extern "C"
