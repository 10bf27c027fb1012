// Block quantizer shared by the host library (g++) and the HIP quantize
// kernel (hipcc), so that GPU-side quantize-on-load produces bit-identical
// codes and scales to the CPU path.
#pragma once
#include <math.h>
#include <stdint.h>

#include "formats.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ILLM_HD __host__ __device__ __forceinline__
#else
#define ILLM_HD inline
#endif

namespace illm {

ILLM_HD uint32_t hd_f2u(float f) {
  union { float f; uint32_t u; } c;
  c.f = f;
  return c.u;
}
ILLM_HD float hd_u2f(uint32_t u) {
  union { float f; uint32_t u; } c;
  c.u = u;
  return c.f;
}

// f32 -> f16 bits, round-to-nearest-even (finite inputs)
ILLM_HD uint16_t hd_f32_to_f16(float f) {
  uint32_t x = hd_f2u(f);
  uint32_t sign = (x >> 16) & 0x8000u;
  int32_t exp = (int32_t)((x >> 23) & 0xff) - 127 + 15;
  uint32_t mant = x & 0x7fffffu;
  if (((x >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0));
  if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
  if (exp <= 0) {
    if (exp < -10) return (uint16_t)sign;
    mant |= 0x800000u;
    uint32_t shift = (uint32_t)(14 - exp);
    uint32_t half = mant >> shift;
    uint32_t rem = mant & ((1u << shift) - 1);
    uint32_t mid = 1u << (shift - 1);
    if (rem > mid || (rem == mid && (half & 1))) half++;
    return (uint16_t)(sign | half);
  }
  uint32_t h = sign | ((uint32_t)exp << 10) | (mant >> 13);
  uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) h++;
  return (uint16_t)h;
}
ILLM_HD float hd_f16_to_f32(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t mant = h & 0x3ffu;
  if (exp == 0) {
    float v = (float)mant * 5.9604644775390625e-8f;  // 2^-24
    return sign ? -v : v;
  }
  if (exp == 31) return hd_u2f(sign | 0x7f800000u | (mant << 13));
  return hd_u2f(sign | ((exp + 127 - 15) << 23) | (mant << 13));
}
ILLM_HD float hd_round_f16(float f) { return hd_f16_to_f32(hd_f32_to_f16(f)); }

// Generic minifloat encoder (no inf/nan produced; saturates to maxv).
// Returns the magnitude code ((E+bias) << mbits | m); sign handled by caller.
ILLM_HD int hd_encode_minifloat(float a, int mbits, int bias, int maxcode) {
  const float sub_step = ldexpf(1.f, 1 - bias - mbits);
  const float min_normal = ldexpf(1.f, 1 - bias);
  if (!(a > 0.f)) return 0;
  int code;
  if (a < min_normal) {
    code = (int)rintf(a / sub_step);
  } else {
    int ex;
    float fr = frexpf(a, &ex);  // a = fr * 2^ex, fr in [0.5, 1)
    int E = ex - 1;
    float mant = fr * 2.f - 1.f;
    int mq = (int)rintf(mant * (float)(1 << mbits));
    if (mq == (1 << mbits)) { mq = 0; E++; }
    code = ((E + bias) << mbits) | mq;
  }
  return code > maxcode ? maxcode : code;
}
ILLM_HD float hd_decode_minifloat(int code, int mbits, int bias) {
  int e = code >> mbits, m = code & ((1 << mbits) - 1);
  if (e == 0) return ldexpf((float)m, 1 - bias - mbits);
  return ldexpf((float)((1 << mbits) + m), e - bias - mbits);
}
// OCP e4m3fn (max code 0x7e = 448) / e5m2 (max 0x7b = 57344) / e3m2 (28)
ILLM_HD uint8_t hd_f32_to_e4m3(float v) {
  int c = hd_encode_minifloat(fabsf(v), 3, 7, 0x7e);
  return (uint8_t)(c | ((v < 0.f && c) ? 0x80 : 0));
}
ILLM_HD uint8_t hd_f32_to_e5m2(float v) {
  int c = hd_encode_minifloat(fabsf(v), 2, 15, 0x7b);
  return (uint8_t)(c | ((v < 0.f && c) ? 0x80 : 0));
}
ILLM_HD float hd_e4m3_to_f32(uint8_t b) {
  float r = hd_decode_minifloat(b & 0x7f, 3, 7);
  return (b & 0x80) ? -r : r;
}
ILLM_HD float hd_e5m2_to_f32(uint8_t b) {
  float r = hd_decode_minifloat(b & 0x7f, 2, 15);
  return (b & 0x80) ? -r : r;
}
// fp6 = e3m2 grid (max 28), stored as its exact e4m3 code
ILLM_HD uint8_t hd_f32_to_fp6_as_e4m3(float v) {
  int c = hd_encode_minifloat(fabsf(v), 2, 3, 0x1f);
  float q = hd_decode_minifloat(c, 2, 3);
  return hd_f32_to_e4m3(v < 0.f ? -q : q);
}

ILLM_HD float hd_lut4(int f, int code) {
  const float nf4[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f,
                         -0.39491748809814453f, -0.28444138169288635f, -0.18477343022823334f,
                         -0.09105003625154495f, 0.0f, 0.07958029955625534f,
                         0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
                         0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};
  const float nf3[8] = {-1.0f, -0.5350227355957031f, -0.2469314038753510f, 0.0f,
                        0.1833375245332718f, 0.3819939494132996f, 0.6229856610298157f, 1.0f};
  const float fp4[16] = {0.0f, 0.5f, 1.0f, 1.5f, 2.0f, 3.0f, 4.0f, 6.0f,
                         -0.0f, -0.5f, -1.0f, -1.5f, -2.0f, -3.0f, -4.0f, -6.0f};
  if (f == FMT_NF4) return nf4[code & 15];
  if (f == FMT_NF3) return nf3[code & 7];
  return fp4[code & 15];
}

// value of a code before the block scale / min are applied
ILLM_HD float hd_code_value(int f, int code) {
  switch (f) {
    case FMT_SYM_INT4: return (float)(code - 8);
    case FMT_ASYM_INT4: case FMT_ASYM_INT5: return (float)code;
    case FMT_NF4: case FMT_FP4: case FMT_NF3: return hd_lut4(f, code);
    case FMT_SYM_INT8: case FMT_SYM_INT5: return (float)(int8_t)(uint8_t)code;
    case FMT_FP8E4: case FMT_FP6: return hd_e4m3_to_f32((uint8_t)code);
    case FMT_FP8E5: return hd_e5m2_to_f32((uint8_t)code);
  }
  return 0.f;
}

ILLM_HD int hd_encode(int f, float v, float d, float m) {
  float id = d != 0.f ? 1.f / d : 0.f;
  switch (f) {
    case FMT_SYM_INT4: {
      int q = (int)floorf(v * id + 8.5f);
      return q < 0 ? 0 : (q > 15 ? 15 : q);
    }
    case FMT_ASYM_INT4: case FMT_ASYM_INT5: {
      int qmax = f == FMT_ASYM_INT4 ? 15 : 31;
      int q = (int)floorf((v - m) * id + 0.5f);
      return q < 0 ? 0 : (q > qmax ? qmax : q);
    }
    case FMT_NF4: case FMT_FP4: case FMT_NF3: {
      float t = v * id;
      int ncode = f == FMT_NF3 ? 8 : 16, best = 0;
      float be = 1e30f;
      for (int c = 0; c < ncode; c++) {
        float e = fabsf(t - hd_lut4(f, c));
        if (e < be) { be = e; best = c; }
      }
      return best;
    }
    case FMT_SYM_INT8: case FMT_SYM_INT5: {
      int qm = f == FMT_SYM_INT8 ? 127 : 15, qn = f == FMT_SYM_INT8 ? -127 : -16;
      int q = (int)rintf(v * id);
      q = q < qn ? qn : (q > qm ? qm : q);
      return (int)(uint8_t)(int8_t)q;
    }
    case FMT_FP8E4: return hd_f32_to_e4m3(v * id);
    case FMT_FP8E5: return hd_f32_to_e5m2(v * id);
    case FMT_FP6: return hd_f32_to_fp6_as_e4m3(v * id);
  }
  return 0;
}

// Quantize one 64-element block: codes[64] (one per byte), scale, min.
// w: importance weights (imatrix) or nullptr; search: RTN scale search.
ILLM_HD void hd_quant_block(int f, const float* x, const float* w, bool search, uint8_t* codes,
                            float* d_out, float* m_out) {
  float amax = 0.f, vmax = 0.f, mn = x[0], mx = x[0];
  for (int i = 0; i < QBLOCK; i++) {
    float a = fabsf(x[i]);
    if (a > amax) { amax = a; vmax = x[i]; }
    mn = x[i] < mn ? x[i] : mn;
    mx = x[i] > mx ? x[i] : mx;
  }
  float d = 0.f, m = 0.f;
  switch (f) {
    case FMT_SYM_INT4: d = vmax / -8.f; break;  // max-|x| element -> code 0 (ggml q4_0)
    case FMT_ASYM_INT4: d = (mx - mn) / 15.f; m = mn; break;
    case FMT_ASYM_INT5: d = (mx - mn) / 31.f; m = mn; break;
    case FMT_NF4: case FMT_NF3: d = amax; break;
    case FMT_FP4: d = amax / 6.f; break;
    case FMT_SYM_INT8: d = amax / 127.f; break;
    case FMT_SYM_INT5: d = amax / 15.f; break;
    case FMT_FP8E4: d = amax / 448.f; break;
    case FMT_FP8E5: d = amax / 57344.f; break;
    case FMT_FP6: d = amax / 28.f; break;
  }
  if (search && amax > 0.f && (f == FMT_SYM_INT4 || f == FMT_SYM_INT8 || f == FMT_NF4 ||
                               f == FMT_FP4 || f == FMT_SYM_INT5)) {
    // weighted RTN scale search around the absmax scale
    float best = -1.f, bd = d;
    for (int is = -9; is <= 9; is++) {
      float dd = hd_round_f16(d * (1.f + 0.0125f * (float)is));
      float e = 0.f;
      for (int i = 0; i < QBLOCK; i++) {
        float r = x[i] - hd_code_value(f, hd_encode(f, x[i], dd, 0.f)) * dd;
        e += (w ? w[i] : 1.f) * r * r;
      }
      if (best < 0.f || e < best) { best = e; bd = dd; }
    }
    d = bd;
  }
  d = hd_round_f16(d);
  m = hd_round_f16(m);
  for (int i = 0; i < QBLOCK; i++) codes[i] = (uint8_t)hd_encode(f, x[i], d, m);
  *d_out = d;
  *m_out = m;
}

}  // namespace illm
