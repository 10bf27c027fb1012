// Host k-quant quantizers / dequantizers / GEMM (q4_K, q5_K, q6_K, q2_K).
//
// Reference capability: the ggml k-quant quantizers the reference reaches
// through ctypes (ggml_quantize_tensor / _with_weights, SRC/transformers/
// low_bit_linear.py:157-190; llama_cpp.py:946-991) for its q2_k / q4_k /
// q5_k / q6_k qtypes and the gguf_q4k_s / gguf_q4k_m mixed policies
// (SRC/transformers/utils.py:286-401).  The block layouts are GGUF's
// (common/kquant.h); the search procedures follow the published ggml design:
//   * q4_K / q5_K / q2_K: per sub-block an affine (scale, min) fitted by a
//     weighted least-squares search over candidate inverse scales
//     (fit_affine), sub-block scales / mins quantized to 6 (4) bits against
//     a per-block f16 d / dmin, then every weight re-rounded against its
//     quantized (scale, min);
//   * q6_K: per 16-weight sub-block a symmetric scale searched around
//     -32 / max (fit_sym), 8-bit sub-block scales against an f16 d.
// The optional importance matrix (imatrix, one weight per input column)
// multiplies the least-squares weights, as in the reference's
// ggml_quantize_tensor_with_weights.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "../common/kquant.h"
#include "../common/quant_block.h"

namespace illm {
void iq_quantize_block(int fmt, const float* x, const float* im, uint8_t* out);   // iquant.cpp
void iq_dequant_block(int fmt, const uint8_t* b, float* y);
}

namespace {

using illm::QK_K;

inline int nearest_int(float v) { return (int)lrintf(v); }

// affine fit of n values onto levels 0..nmax: returns scale, *the_min = -min
float fit_affine(int n, int nmax, const float* x, const float* w, uint8_t* L, float* the_min, uint8_t* Laux,
                 float rmin, float rdelta, int nstep, bool use_mad) {
  float mn = x[0], mx = x[0], sum_w = w[0], sum_x = w[0] * x[0];
  for (int i = 1; i < n; ++i) {
    mn = std::min(mn, x[i]);
    mx = std::max(mx, x[i]);
    sum_w += w[i];
    sum_x += w[i] * x[i];
  }
  if (mn > 0) mn = 0;
  if (mx == mn) {
    for (int i = 0; i < n; ++i) L[i] = 0;
    *the_min = -mn;
    return 0.f;
  }
  float iscale = nmax / (mx - mn);
  float scale = 1.f / iscale;
  float best = 0;
  for (int i = 0; i < n; ++i) {
    const int l = std::max(0, std::min(nmax, nearest_int(iscale * (x[i] - mn))));
    L[i] = (uint8_t)l;
    float d = scale * l + mn - x[i];
    d = use_mad ? fabsf(d) : d * d;
    best += w[i] * d;
  }
  for (int is = 0; is <= nstep; ++is) {
    iscale = (rmin + rdelta * is + nmax) / (mx - mn);
    float sum_l = 0, sum_l2 = 0, sum_xl = 0;
    for (int i = 0; i < n; ++i) {
      const int l = std::max(0, std::min(nmax, nearest_int(iscale * (x[i] - mn))));
      Laux[i] = (uint8_t)l;
      sum_l += w[i] * l;
      sum_l2 += w[i] * l * l;
      sum_xl += w[i] * l * x[i];
    }
    const float D = sum_w * sum_l2 - sum_l * sum_l;
    if (D > 0) {
      float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
      float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
      if (this_min > 0) {
        this_min = 0;
        this_scale = sum_xl / sum_l2;
      }
      float err = 0;
      for (int i = 0; i < n; ++i) {
        float d = this_scale * Laux[i] + this_min - x[i];
        d = use_mad ? fabsf(d) : d * d;
        err += w[i] * d;
      }
      if (err < best) {
        for (int i = 0; i < n; ++i) L[i] = Laux[i];
        best = err;
        scale = this_scale;
        mn = this_min;
      }
    }
  }
  *the_min = -mn;
  return scale;
}

// symmetric fit onto -nmax..nmax-1 (stored biased by nmax), weights w (or x^2)
float fit_sym(int n, int nmax, const float* x, const float* w, int8_t* L) {
  float mx = 0, amax = 0;
  for (int i = 0; i < n; ++i) {
    const float ax = fabsf(x[i]);
    if (ax > amax) { amax = ax; mx = x[i]; }
  }
  if (amax < 1e-15f) {
    for (int i = 0; i < n; ++i) L[i] = 0;
    return 0.f;
  }
  auto weight = [&](int i) { return w ? w[i] : x[i] * x[i]; };
  float iscale = -nmax / mx;
  float sumlx = 0, suml2 = 0;
  for (int i = 0; i < n; ++i) {
    const int l = std::max(-nmax, std::min(nmax - 1, nearest_int(iscale * x[i])));
    L[i] = (int8_t)l;
    sumlx += weight(i) * x[i] * l;
    suml2 += weight(i) * l * l;
  }
  float scale = suml2 > 0 ? sumlx / suml2 : 0.f;
  float best = scale * sumlx;
  for (int is = -9; is <= 9; ++is) {
    if (is == 0) continue;
    iscale = -(nmax + 0.1f * is) / mx;
    float slx = 0, sl2 = 0;
    for (int i = 0; i < n; ++i) {
      const int l = std::max(-nmax, std::min(nmax - 1, nearest_int(iscale * x[i])));
      slx += weight(i) * x[i] * l;
      sl2 += weight(i) * l * l;
    }
    if (sl2 > 0 && slx * slx > best * sl2) {
      for (int i = 0; i < n; ++i) L[i] = (int8_t)std::max(-nmax, std::min(nmax - 1, nearest_int(iscale * x[i])));
      scale = slx / sl2;
      best = scale * slx;
    }
  }
  return scale;
}

inline uint16_t h(float v) { return illm::hd_f32_to_f16(v); }
inline float f(uint16_t v) { return illm::hd_f16_to_f32(v); }

// least-squares weights of one sub-block: imatrix-weighted when given
void sub_weights(const float* x, const float* im, int n, float* w, bool plain_abs) {
  float s2 = 0;
  for (int i = 0; i < n; ++i) s2 += x[i] * x[i];
  const float sigma2 = s2 / n;
  for (int i = 0; i < n; ++i) {
    if (im) w[i] = im[i] * sqrtf(sigma2 + x[i] * x[i]);
    else w[i] = plain_abs ? fabsf(x[i]) : sqrtf(sigma2) + fabsf(x[i]);
  }
}

void quant_q4k_q5k(const float* x, const float* im, uint8_t* out, bool five) {
  const int nmax = five ? 31 : 15;
  float scales[8], mins[8], w[32];
  uint8_t L[QK_K], Laux[32];
  float max_scale = 0, max_min = 0;
  for (int j = 0; j < 8; ++j) {
    sub_weights(x + 32 * j, im ? im + 32 * j : nullptr, 32, w, false);
    scales[j] = fit_affine(32, nmax, x + 32 * j, w, L + 32 * j, &mins[j], Laux, five ? -0.5f : -1.f, 0.1f,
                           five ? 15 : 20, false);
    max_scale = std::max(max_scale, scales[j]);
    max_min = std::max(max_min, mins[j]);
  }
  uint16_t* hd = (uint16_t*)out;
  uint8_t* sc = out + 4;
  memset(sc, 0, 12);
  const float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
  const float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
  for (int j = 0; j < 8; ++j) {
    const uint8_t ls = (uint8_t)std::min(63, nearest_int(inv_scale * scales[j]));
    const uint8_t lm = (uint8_t)std::min(63, nearest_int(inv_min * mins[j]));
    if (j < 4) {
      sc[j] = ls;
      sc[j + 4] = lm;
    } else {
      sc[j + 4] = (ls & 0xF) | ((lm & 0xF) << 4);
      sc[j - 4] |= ((ls >> 4) << 6);
      sc[j] |= ((lm >> 4) << 6);
    }
  }
  hd[0] = h(max_scale / 63.f);
  hd[1] = h(max_min / 63.f);
  for (int j = 0; j < 8; ++j) {
    int s, m;
    illm::kq_scale_min_k4(j, sc, &s, &m);
    const float d = f(hd[0]) * s;
    if (d == 0.f) continue;
    const float dm = f(hd[1]) * m;
    for (int i = 0; i < 32; ++i) L[32 * j + i] = (uint8_t)std::max(0, std::min(nmax, nearest_int((x[32 * j + i] + dm) / d)));
  }
  if (!five) {
    uint8_t* q = out + 16;
    for (int j = 0; j < QK_K; j += 64, q += 32)
      for (int l = 0; l < 32; ++l) q[l] = L[j + l] | (L[j + l + 32] << 4);
  } else {
    uint8_t* qh = out + 16;
    uint8_t* ql = out + 48;
    memset(qh, 0, 32);
    uint8_t m1 = 1, m2 = 2;
    for (int n = 0; n < QK_K; n += 64, ql += 32) {
      for (int j = 0; j < 32; ++j) {
        int l1 = L[n + j], l2 = L[n + j + 32];
        if (l1 > 15) { l1 -= 16; qh[j] |= m1; }
        if (l2 > 15) { l2 -= 16; qh[j] |= m2; }
        ql[j] = (uint8_t)(l1 | (l2 << 4));
      }
      m1 <<= 2;
      m2 <<= 2;
    }
  }
}

void quant_q6k(const float* x, const float* im, uint8_t* out) {
  float scales[16], w[16];
  int8_t Ls[QK_K];
  uint8_t L[QK_K];
  float max_scale = 0, max_abs = 0;
  for (int ib = 0; ib < 16; ++ib) {
    if (im) sub_weights(x + 16 * ib, im + 16 * ib, 16, w, false);
    const float s = fit_sym(16, 32, x + 16 * ib, im ? w : nullptr, Ls + 16 * ib);
    scales[ib] = s;
    if (fabsf(s) > max_abs) { max_abs = fabsf(s); max_scale = s; }
  }
  uint8_t* ql = out;
  uint8_t* qh = out + 128;
  int8_t* sc = (int8_t*)(out + 192);
  uint16_t* hd = (uint16_t*)(out + 208);
  if (max_abs < 1e-15f) {
    memset(out, 0, 210);
    return;
  }
  const float iscale = -128.f / max_scale;
  hd[0] = h(1.f / iscale);
  for (int ib = 0; ib < 16; ++ib) sc[ib] = (int8_t)std::min(127, nearest_int(iscale * scales[ib]));
  for (int j = 0; j < 16; ++j) {
    const float d = f(hd[0]) * sc[j];
    for (int i = 0; i < 16; ++i) {
      const int l = d == 0.f ? 0 : std::max(-32, std::min(31, nearest_int(x[16 * j + i] / d)));
      L[16 * j + i] = (uint8_t)(l + 32);
    }
  }
  for (int j = 0; j < QK_K; j += 128, ql += 64, qh += 32) {
    for (int l = 0; l < 32; ++l) {
      const uint8_t q1 = L[j + l] & 0xF, q2 = L[j + l + 32] & 0xF, q3 = L[j + l + 64] & 0xF, q4 = L[j + l + 96] & 0xF;
      ql[l] = q1 | (q3 << 4);
      ql[l + 32] = q2 | (q4 << 4);
      qh[l] = (L[j + l] >> 4) | ((L[j + l + 32] >> 4) << 2) | ((L[j + l + 64] >> 4) << 4) | ((L[j + l + 96] >> 4) << 6);
    }
  }
}

void quant_q2k(const float* x, const float* im, uint8_t* out) {
  float scales[16], mins[16], w[16];
  uint8_t L[QK_K], Laux[16];
  float max_scale = 0, max_min = 0;
  for (int j = 0; j < 16; ++j) {
    sub_weights(x + 16 * j, im ? im + 16 * j : nullptr, 16, w, true);
    scales[j] = fit_affine(16, 3, x + 16 * j, w, L + 16 * j, &mins[j], Laux, -0.5f, 0.1f, 15, true);
    max_scale = std::max(max_scale, scales[j]);
    max_min = std::max(max_min, mins[j]);
  }
  uint8_t* sc = out;
  uint8_t* qs = out + 16;
  uint16_t* hd = (uint16_t*)(out + 80);
  if (max_scale > 0) {
    const float is = 15.f / max_scale;
    for (int j = 0; j < 16; ++j) sc[j] = (uint8_t)std::min(15, nearest_int(is * scales[j]));
    hd[0] = h(max_scale / 15.f);
  } else {
    for (int j = 0; j < 16; ++j) sc[j] = 0;
    hd[0] = h(0.f);
  }
  if (max_min > 0) {
    const float is = 15.f / max_min;
    for (int j = 0; j < 16; ++j) sc[j] |= (uint8_t)(std::min(15, nearest_int(is * mins[j])) << 4);
    hd[1] = h(max_min / 15.f);
  } else {
    hd[1] = h(0.f);
  }
  for (int j = 0; j < 16; ++j) {
    const float d = f(hd[0]) * (sc[j] & 0xF);
    if (d == 0.f) continue;
    const float dm = f(hd[1]) * (sc[j] >> 4);
    for (int i = 0; i < 16; ++i) L[16 * j + i] = (uint8_t)std::max(0, std::min(3, nearest_int((x[16 * j + i] + dm) / d)));
  }
  for (int j = 0; j < QK_K; j += 128)
    for (int l = 0; l < 32; ++l)
      qs[j / 4 + l] = L[j + l] | (L[j + l + 32] << 2) | (L[j + l + 64] << 4) | (L[j + l + 96] << 6);
}

void dequant_block(int fmt, const uint8_t* b, float* y) {
  if (illm::is_iq(fmt)) {
    illm::iq_dequant_block(fmt, b, y);
  } else if (fmt == illm::FMT_Q4K || fmt == illm::FMT_Q5K) {
    const float d = f(((const uint16_t*)b)[0]), dmin = f(((const uint16_t*)b)[1]);
    const uint8_t* sc = b + 4;
    const bool five = fmt == illm::FMT_Q5K;
    const uint8_t* qh = b + 16;
    const uint8_t* q = b + (five ? 48 : 16);
    int is = 0;
    uint8_t u1 = 1, u2 = 2;
    for (int j = 0; j < QK_K; j += 64, q += 32, is += 2) {
      int s, m;
      illm::kq_scale_min_k4(is, sc, &s, &m);
      const float d1 = d * s, m1 = dmin * m;
      illm::kq_scale_min_k4(is + 1, sc, &s, &m);
      const float d2 = d * s, m2 = dmin * m;
      for (int l = 0; l < 32; ++l) {
        const int lo = (q[l] & 0xF) + (five && (qh[l] & u1) ? 16 : 0);
        const int hi = (q[l] >> 4) + (five && (qh[l] & u2) ? 16 : 0);
        y[j + l] = d1 * lo - m1;
        y[j + 32 + l] = d2 * hi - m2;
      }
      u1 <<= 2;
      u2 <<= 2;
    }
  } else if (fmt == illm::FMT_Q6K) {
    const uint8_t* ql = b;
    const uint8_t* qh = b + 128;
    const int8_t* sc = (const int8_t*)(b + 192);
    const float d = f(*(const uint16_t*)(b + 208));
    for (int n = 0; n < QK_K; n += 128, ql += 64, qh += 32, sc += 8) {
      for (int l = 0; l < 32; ++l) {
        const int is = l / 16;
        const int q1 = (int)((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
        const int q2 = (int)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
        const int q3 = (int)((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
        const int q4 = (int)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
        y[n + l] = d * sc[is] * q1;
        y[n + l + 32] = d * sc[is + 2] * q2;
        y[n + l + 64] = d * sc[is + 4] * q3;
        y[n + l + 96] = d * sc[is + 6] * q4;
      }
    }
  } else {  // q2_K
    const uint8_t* sc = b;
    const uint8_t* q = b + 16;
    const float d = f(*(const uint16_t*)(b + 80)), dmin = f(*(const uint16_t*)(b + 82));
    int is = 0;
    for (int n = 0; n < QK_K; n += 128, q += 32) {
      int shift = 0;
      for (int j = 0; j < 4; ++j, shift += 2) {
        int s = sc[is++];
        float dl = d * (s & 0xF), ml = dmin * (s >> 4);
        for (int l = 0; l < 16; ++l) y[n + 32 * j + l] = dl * ((q[l] >> shift) & 3) - ml;
        s = sc[is++];
        dl = d * (s & 0xF);
        ml = dmin * (s >> 4);
        for (int l = 0; l < 16; ++l) y[n + 32 * j + 16 + l] = dl * ((q[l + 16] >> shift) & 3) - ml;
      }
    }
  }
}

}  // namespace

extern "C" {

int64_t illm_kq_total_bytes(int fmt, int64_t n, int64_t k) { return illm::kq_total_bytes(fmt, n, k); }

// src f32 [n, k] (k % 256 == 0); imatrix f32 [k] or null
void illm_kq_quantize(int fmt, const float* src, int64_t n, int64_t k, const float* imatrix, uint8_t* dst) {
  const int64_t nb = k / QK_K;
  const int bb = illm::kq_block_bytes(fmt);
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t r = 0; r < n; ++r) {
    for (int64_t b = 0; b < nb; ++b) {
      const float* x = src + r * k + b * QK_K;
      const float* im = imatrix ? imatrix + b * QK_K : nullptr;
      uint8_t* o = dst + (r * nb + b) * bb;
      if (illm::is_iq(fmt)) illm::iq_quantize_block(fmt, x, im, o);
      else if (fmt == illm::FMT_Q4K) quant_q4k_q5k(x, im, o, false);
      else if (fmt == illm::FMT_Q5K) quant_q4k_q5k(x, im, o, true);
      else if (fmt == illm::FMT_Q6K) quant_q6k(x, im, o);
      else quant_q2k(x, im, o);
    }
  }
}

void illm_kq_dequantize(int fmt, const uint8_t* src, int64_t n, int64_t k, float* dst) {
  const int64_t nb = k / QK_K;
  const int bb = illm::kq_block_bytes(fmt);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n; ++r)
    for (int64_t b = 0; b < nb; ++b) dequant_block(fmt, src + (r * nb + b) * bb, dst + r * k + b * QK_K);
}

// y [m, n] = x [m, k] @ W^T (f32), one block row dequantized at a time
void illm_kq_gemm(int fmt, const float* x, int64_t m, const uint8_t* w, int64_t n, int64_t k, float* y) {
  const int64_t nb = k / QK_K;
  const int bb = illm::kq_block_bytes(fmt);
#pragma omp parallel
  {
    std::vector<float> row(k);
#pragma omp for schedule(dynamic, 8)
    for (int64_t r = 0; r < n; ++r) {
      for (int64_t b = 0; b < nb; ++b) dequant_block(fmt, w + (r * nb + b) * bb, row.data() + b * QK_K);
      for (int64_t i = 0; i < m; ++i) {
        const float* xi = x + i * k;
        float s = 0.f;
        for (int64_t c = 0; c < k; ++c) s += xi[c] * row[c];
        y[i * n + r] = s;
      }
    }
  }
}

}  // extern "C"
