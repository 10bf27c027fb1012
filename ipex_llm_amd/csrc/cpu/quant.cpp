// Host-side low-bit library: quantizers, dequantizers, MI355X tile repacker
// and a CPU low-bit GEMM.  Plain C++ (OpenMP), no torch headers -- wrapped as
// torch ops in csrc/torch/ops.cpp.
//
// Reference behaviour being matched (semantics, not code):
//   ggml_quantize_tensor / _with_weights / _rtn   (SRC/transformers/low_bit_linear.py:157-189)
//   ggml_dequantize                               (low_bit_linear.py:256-279)
//   ggml_q_format_convet_cpu2xpu / xpu2cpu       (low_bit_linear.py:198-253)
//   ggml_compute_forward_mul_mat_q_fp32           (low_bit_linear.py:494-529)
#include "quant_api.h"

#include <string.h>

#include <vector>

#include "../common/formats.h"
#include "../common/quant_block.h"

using namespace illm;

extern "C" {

int illm_fmt_bits(int fmt) { return fmt_bits(fmt); }

void illm_quantize(int fmt, const float* src, int64_t n, int64_t k, const float* imatrix,
                   int scale_search, uint8_t* codes, uint16_t* scales, uint16_t* mins) {
  const int64_t nb = k / QBLOCK;
  const int bits = fmt_bits(fmt);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n; r++) {
    uint8_t c[QBLOCK];
    for (int64_t b = 0; b < nb; b++) {
      const float* x = src + r * k + b * QBLOCK;
      const float* w = imatrix ? imatrix + b * QBLOCK : nullptr;
      float d, m;
      hd_quant_block(fmt, x, w, scale_search != 0, c, &d, &m);
      scales[r * nb + b] = hd_f32_to_f16(d);
      if (mins) mins[r * nb + b] = hd_f32_to_f16(m);
      uint8_t* dst = codes + (r * k + b * QBLOCK) * bits / 8;
      if (bits == 4) {
        for (int j = 0; j < 32; j++) dst[j] = (uint8_t)((c[j] & 15) | ((c[j + 32] & 15) << 4));
      } else {
        memcpy(dst, c, QBLOCK);
      }
    }
  }
}

void illm_dequantize(int fmt, const uint8_t* codes, const uint16_t* scales, const uint16_t* mins,
                     int64_t n, int64_t k, float* dst) {
  const int64_t nb = k / QBLOCK;
  const int bits = fmt_bits(fmt);
  float lut[256];
  for (int c = 0; c < (bits == 4 ? 16 : 256); c++) lut[c] = hd_code_value(fmt, c);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n; r++) {
    for (int64_t b = 0; b < nb; b++) {
      float d = hd_f16_to_f32(scales[r * nb + b]);
      float m = mins ? hd_f16_to_f32(mins[r * nb + b]) : 0.f;
      const uint8_t* src = codes + (r * k + b * QBLOCK) * bits / 8;
      float* o = dst + r * k + b * QBLOCK;
      for (int j = 0; j < QBLOCK; j++) {
        int code = bits == 4 ? ((j < 32 ? src[j] : src[j - 32] >> 4) & 15) : src[j];
        o[j] = lut[code] * d + m;
      }
    }
  }
}

static inline int canon_code_at(int fmt, int bits, const uint8_t* codes, int64_t n, int64_t k,
                                int64_t r, int64_t kk) {
  if (r >= n || kk >= k) return fmt == FMT_SYM_INT4 ? 8 : 0;  // decodes to 0
  const uint8_t* row = codes + r * k * bits / 8;
  if (bits == 4) {
    int64_t b = kk / QBLOCK, j = kk % QBLOCK;
    uint8_t byte = row[b * 32 + (j & 31)];
    return j < 32 ? (byte & 15) : (byte >> 4);
  }
  return row[kk];
}

// canonical planes -> MI355X tiled device blob (see formats.h)
void illm_repack_to_device(int fmt, const uint8_t* codes, const uint16_t* scales,
                           const uint16_t* mins, int64_t n, int64_t k, uint8_t* dev) {
  const int bits = fmt_bits(fmt);
  const int64_t Np = pad_to(n, TILE_N), Kp = pad_to(k, CHUNK_K);
  const int64_t KC = Kp / CHUNK_K, NT = Np / TILE_N;
  const int64_t nb = k / QBLOCK;
  const int64_t TB = dev_tile_bytes(fmt, KC);
#pragma omp parallel for collapse(2) schedule(static)
  for (int64_t t = 0; t < NT; t++) {
    for (int64_t c = 0; c < KC; c++) {
      uint8_t* tile = dev + t * TB;
      uint8_t* rec = tile + c * dev_code_chunk(fmt);
      for (int l = 0; l < 64; l++) {
        int r = l & 15, g = l >> 4;
        int64_t row = t * TILE_N + r;
        if (bits == 4) {
          uint32_t* out = (uint32_t*)(rec + l * 16);
          for (int s = 0; s < 4; s++) {
            uint32_t u = 0;
            for (int j = 0; j < 8; j++) {
              int64_t kk = c * CHUNK_K + 32 * s + 8 * g + j;
              u |= (uint32_t)(canon_code_at(fmt, bits, codes, n, k, row, kk) & 15)
                   << (4 * dev_nib_pos(fmt, j));
            }
            out[s] = u;
          }
        } else {
          for (int h = 0; h < 2; h++) {
            uint8_t* out = rec + (h * 64 + l) * 16;
            for (int ss = 0; ss < 2; ss++) {
              int s = 2 * h + ss;
              for (int j = 0; j < 8; j++) {
                int64_t kk = c * CHUNK_K + 32 * s + 8 * g + j;
                out[ss * 8 + j] = (uint8_t)canon_code_at(fmt, bits, codes, n, k, row, kk);
              }
            }
          }
        }
      }
      for (int r = 0; r < TILE_N; r++)
        for (int blk = 0; blk < 2; blk++) {
          int64_t row = t * TILE_N + r;
          int64_t b = c * 2 + blk;
          bool in = row < n && b < nb;
          ((uint16_t*)(tile + dev_scale_off(fmt, KC, r, c)))[blk] = in ? scales[row * nb + b] : 0;
          if (fmt_has_min(fmt))
            ((uint16_t*)(tile + dev_min_off(fmt, KC, r, c)))[blk] = (in && mins) ? mins[row * nb + b] : 0;
        }
    }
  }
}

// MI355X tiled device blob -> canonical planes (inverse of the above)
void illm_repack_from_device(int fmt, const uint8_t* dev, int64_t n, int64_t k, uint8_t* codes,
                             uint16_t* scales, uint16_t* mins) {
  const int bits = fmt_bits(fmt);
  const int64_t KC = pad_to(k, CHUNK_K) / CHUNK_K;
  const int64_t nb = k / QBLOCK;
  const int64_t TB = dev_tile_bytes(fmt, KC);
#pragma omp parallel for schedule(static)
  for (int64_t row = 0; row < n; row++) {
    int64_t t = row / TILE_N;
    int r = (int)(row % TILE_N);
    uint8_t* crow = codes + row * k * bits / 8;
    for (int64_t kk = 0; kk < k; kk++) {
      int64_t c = kk / CHUNK_K;
      const uint8_t* rec = dev + t * TB + c * dev_code_chunk(fmt);
      int kin = (int)(kk % CHUNK_K);
      int s = kin / 32, g = (kin % 32) / 8, j = kin % 8;
      int l = g * 16 + r;
      if (bits == 4) {
        const uint32_t* in = (const uint32_t*)(rec + l * 16);
        int code = (in[s] >> (4 * dev_nib_pos(fmt, j))) & 15;
        int64_t b = kk / QBLOCK, jj = kk % QBLOCK;
        uint8_t& byte = crow[b * 32 + (jj & 31)];
        if (jj < 32) byte = (uint8_t)((byte & 0xf0) | code);
        else byte = (uint8_t)((byte & 0x0f) | (code << 4));
      } else {
        int h = s / 2, ss = s % 2;
        crow[kk] = rec[(h * 64 + l) * 16 + ss * 8 + j];
      }
    }
    for (int64_t b = 0; b < nb; b++) {
      int64_t c = b / 2;
      const uint8_t* tile = dev + t * TB;
      scales[row * nb + b] = ((const uint16_t*)(tile + dev_scale_off(fmt, KC, r, c)))[b % 2];
      if (mins && fmt_has_min(fmt)) mins[row * nb + b] = ((const uint16_t*)(tile + dev_min_off(fmt, KC, r, c)))[b % 2];
    }
  }
}

// y[M,N] = x[M,K] @ W[N,K]^T with W in canonical planes (fp32 math).
// The CPU path of LowBitLinear (BASELINE config 1: Llama-2 7B INT4 on CPU).
void illm_cpu_gemm(int fmt, const float* x, int64_t m, const uint8_t* codes,
                   const uint16_t* scales, const uint16_t* mins, int64_t n, int64_t k,
                   float* y) {
  const int64_t nb = k / QBLOCK;
  const int bits = fmt_bits(fmt);
  float lutv[256];
  for (int c = 0; c < (bits == 4 ? 16 : 256); c++) lutv[c] = hd_code_value(fmt, c);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t r = 0; r < n; r++) {
    float tmp[QBLOCK];
    std::vector<float> acc((size_t)m, 0.f);
    const uint8_t* row = codes + r * k * bits / 8;
    for (int64_t b = 0; b < nb; b++) {
      float d = hd_f16_to_f32(scales[r * nb + b]);
      float mn = mins ? hd_f16_to_f32(mins[r * nb + b]) : 0.f;
      if (bits == 4) {
        const uint8_t* src = row + b * 32;
        for (int j = 0; j < 32; j++) {
          tmp[j] = lutv[src[j] & 15] * d + mn;
          tmp[j + 32] = lutv[src[j] >> 4] * d + mn;
        }
      } else {
        const uint8_t* src = row + b * QBLOCK;
        for (int j = 0; j < QBLOCK; j++) tmp[j] = lutv[src[j]] * d + mn;
      }
      for (int64_t i = 0; i < m; i++) {
        const float* xv = x + i * k + b * QBLOCK;
        float s = 0.f;
#pragma omp simd reduction(+ : s)
        for (int j = 0; j < QBLOCK; j++) s += tmp[j] * xv[j];
        acc[(size_t)i] += s;
      }
    }
    for (int64_t i = 0; i < m; i++) y[i * n + r] = acc[(size_t)i];
  }
}

void illm_f32_to_fp8(const float* src, int64_t n, int e5m2, uint8_t* dst) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) dst[i] = e5m2 ? hd_f32_to_e5m2(src[i]) : hd_f32_to_e4m3(src[i]);
}

}  // extern "C"
