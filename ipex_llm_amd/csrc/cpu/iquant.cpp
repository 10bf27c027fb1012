// Host quantizers of the IQ lattice formats (iq2_xxs / iq2_xs / iq1_s / iq1_m,
// common/iquant.h): the gguf_iq2_xxs / gguf_iq2_xs / gguf_iq1_s qtypes the
// reference produces through ggml_quantize_tensor_with_weights with an
// importance matrix (SRC/transformers/low_bit_linear.py:153-190,
// SRC/transformers/model.py:334-346).
//
// Search (per 8-weight chunk, per candidate group scale):
//   * every weight is first rounded to its nearest codebook LEVEL (IQ2:
//     magnitudes {8, 25, 43}; IQ1: {-1, 0, +1} after the +-1/8 shift), which
//     names one of the 3^8 level vectors; a table built once maps each level
//     vector to its 16 nearest codebook entries (plain L2), and the entry
//     with the smallest importance-weighted error is taken;
//   * IQ2 signs are stored for 7 weights, the 8th is implied by even parity:
//     an odd count of negative weights flips the sign of the weight whose
//     flip costs least (w_j |x_j| g_j);
//   * group scales are searched over a fixed set of candidates around
//     amax / level_max, then quantized against the super-block f16 d (4-bit
//     IQ2 scales, 3-bit IQ1) and every chunk is re-searched at the final
//     scale.
// Weights: imatrix[k] * sqrt(sigma2 + x^2) (ggml's form; sigma2 = 2 <x^2>),
// or sqrt(sigma2 + x^2) without an imatrix.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "../common/iquant.h"
#include "../common/kquant.h"
#include "../common/quant_block.h"

namespace {

const uint64_t G2XXS[256] = ILLM_IQ2XXS_GRID;
const uint64_t G2XS[512] = ILLM_IQ2XS_GRID;
const uint64_t G1S[2048] = ILLM_IQ1S_GRID;
constexpr int NB = 16;            // codebook candidates per level vector
constexpr int NLV = 6561;         // 3^8 level vectors

struct Neighbors {
  std::vector<uint16_t> idx;      // [NLV][NB]
};

inline float lvl2(int i) { return i == 0 ? 8.f : (i == 1 ? 25.f : 43.f); }
inline float grid_val(const uint64_t* grid, bool ternary, int e, int j) {
  const uint8_t b = (uint8_t)((grid[e] >> (8 * j)) & 0xff);
  return ternary ? (float)(int8_t)b : (float)b;
}

Neighbors build(const uint64_t* grid, int n, bool ternary) {
  Neighbors nb;
  nb.idx.resize((size_t)NLV * NB);
  std::vector<std::pair<float, int>> dist((size_t)n);
  for (int key = 0; key < NLV; key++) {
    float v[8];
    int t = key;
    for (int j = 0; j < 8; j++, t /= 3) v[j] = ternary ? (float)(t % 3 - 1) : lvl2(t % 3);
    for (int e = 0; e < n; e++) {
      float s = 0.f;
      for (int j = 0; j < 8; j++) {
        const float dd = v[j] - grid_val(grid, ternary, e, j);
        s += dd * dd;
      }
      dist[(size_t)e] = {s, e};
    }
    std::partial_sort(dist.begin(), dist.begin() + NB, dist.end());
    for (int q = 0; q < NB; q++) nb.idx[(size_t)key * NB + q] = (uint16_t)dist[(size_t)q].second;
  }
  return nb;
}

const Neighbors& neighbors(int fmt) {
  static std::once_flag f0, f1, f2;
  static Neighbors n0, n1, n2;
  if (fmt == illm::FMT_IQ2XXS) { std::call_once(f0, [] { n0 = build(G2XXS, 256, false); }); return n0; }
  if (fmt == illm::FMT_IQ2XS) { std::call_once(f1, [] { n1 = build(G2XS, 512, false); }); return n1; }
  std::call_once(f2, [] { n2 = build(G1S, 2048, true); });
  return n2;
}

// best codebook entry for one IQ2 chunk: a = |x| (8), w = weights, s = scale
// (reconstruction s * grid); returns the entry and its weighted error
inline int iq2_chunk(const uint64_t* grid, const Neighbors& nb, const float* a, const float* w, float s, float* err) {
  int key = 0, mul = 1;
  for (int j = 0; j < 8; j++, mul *= 3) {
    const float t = a[j] / s;
    key += mul * (t < 16.5f ? 0 : (t < 34.f ? 1 : 2));
  }
  int best = 0;
  float be = 3.4e38f;
  for (int q = 0; q < NB; q++) {
    const int e = nb.idx[(size_t)key * NB + q];
    float er = 0.f;
    for (int j = 0; j < 8; j++) {
      const float d = a[j] - s * grid_val(grid, false, e, j);
      er += w[j] * d * d;
    }
    if (er < be) { be = er; best = e; }
  }
  *err = be;
  return best;
}

// signs of one chunk with even parity: returns the 8 sign bits (1 = minus)
// and adds the flip cost to *err
inline uint32_t iq2_signs(const uint64_t* grid, int e, const float* x, const float* w, float s, float* err) {
  uint32_t sg = 0;
  for (int j = 0; j < 8; j++)
    if (x[j] < 0.f) sg |= 1u << j;
  if (__builtin_popcount(sg) & 1) {
    int jm = 0;
    float cm = 3.4e38f;
    for (int j = 0; j < 8; j++) {
      const float c = w[j] * fabsf(x[j]) * grid_val(grid, false, e, j);
      if (c < cm) { cm = c; jm = j; }
    }
    sg ^= 1u << jm;
    *err += 4.f * s * cm;
  }
  return sg;
}

void weights_of(const float* x, const float* im, float* w) {
  float s2 = 0.f;
  for (int i = 0; i < 256; i++) s2 += x[i] * x[i];
  const float sigma2 = 2.f * s2 / 256.f;
  for (int i = 0; i < 256; i++) w[i] = (im ? im[i] : 1.f) * sqrtf(sigma2 + x[i] * x[i]);
}

constexpr float SCALE_F[] = {0.55f, 0.65f, 0.75f, 0.85f, 0.95f, 1.05f, 1.15f, 1.3f};

// search the scale of `n8` consecutive chunks (a group / half group) of an IQ2 format
float iq2_group_scale(const uint64_t* grid, const Neighbors& nb, const float* x, const float* w, int n8) {
  float amax = 0.f;
  for (int i = 0; i < 8 * n8; i++) amax = std::max(amax, fabsf(x[i]));
  if (amax == 0.f) return 0.f;
  float best_s = amax / 43.f, best_e = 3.4e38f;
  for (float f : SCALE_F) {
    const float s = amax / 43.f * f;
    float tot = 0.f;
    for (int c = 0; c < n8; c++) {
      float a[8], er;
      for (int j = 0; j < 8; j++) a[j] = fabsf(x[8 * c + j]);
      const int e = iq2_chunk(grid, nb, a, w + 8 * c, s, &er);
      iq2_signs(grid, e, x + 8 * c, w + 8 * c, s, &er);
      tot += er;
    }
    if (tot < best_e) { best_e = tot; best_s = s; }
  }
  return best_s;
}

void quant_iq2(int fmt, const float* x, const float* im, uint8_t* out) {
  const bool xxs = fmt == illm::FMT_IQ2XXS;
  const uint64_t* grid = xxs ? G2XXS : G2XS;
  const Neighbors& nb = neighbors(fmt);
  float w[256];
  weights_of(x, im, w);
  // group (xxs: 32 weights) / half-group (xs: 16) scales
  const int per = xxs ? 4 : 2, ns = 32 / per;
  float sc[16];
  float smax = 0.f;
  for (int g = 0; g < ns; g++) {
    sc[g] = iq2_group_scale(grid, nb, x + 8 * per * g, w + 8 * per * g, per);
    smax = std::max(smax, sc[g]);
  }
  const float d = smax / (15.5f * 0.25f);
  const uint16_t dh = illm::hd_f32_to_f16(d);
  const float dq = illm::hd_f16_to_f32(dh);
  memset(out, 0, illm::iq_block_bytes(fmt));
  out[0] = (uint8_t)(dh & 0xff);
  out[1] = (uint8_t)(dh >> 8);
  int ls[16];
  for (int g = 0; g < ns; g++) {
    const int l = dq > 0.f ? (int)lrintf(sc[g] / (0.25f * dq) - 0.5f) : 0;
    ls[g] = std::min(15, std::max(0, l));
  }
  for (int c = 0; c < 32; c++) {
    const int g = c / per;
    const float s = dq * (0.5f + (float)ls[g]) * 0.25f;
    float a[8], er = 0.f;
    for (int j = 0; j < 8; j++) a[j] = fabsf(x[8 * c + j]);
    const int e = s > 0.f ? iq2_chunk(grid, nb, a, w + 8 * c, s, &er) : 0;
    const uint32_t sg = iq2_signs(grid, e, x + 8 * c, w + 8 * c, s > 0.f ? s : 1.f, &er);
    if (xxs) {
      uint8_t* grp = out + 2 + 8 * (c >> 2);
      grp[c & 3] = (uint8_t)e;
      uint32_t aux = illm::iq_rd32(grp + 4);
      aux |= (sg & 127u) << (7 * (c & 3));
      if ((c & 3) == 0) aux |= (uint32_t)ls[g] << 28;
      memcpy(grp + 4, &aux, 4);
    } else {
      const uint16_t q = (uint16_t)((uint32_t)e | ((sg & 127u) << 9));
      memcpy(out + 2 + 2 * c, &q, 2);
      if ((c & 1) == 0) out[66 + (c >> 2)] |= (uint8_t)(ls[g] << (4 * ((c >> 1) & 1)));
    }
  }
}

// IQ1: best ternary entry for x / s - shift
inline int iq1_chunk(const Neighbors& nb, const float* x, const float* w, float s, float sh, float* err) {
  int key = 0, mul = 1;
  for (int j = 0; j < 8; j++, mul *= 3) {
    const float t = x[j] / s - sh;
    key += mul * (t < -0.5f ? 0 : (t < 0.5f ? 1 : 2));
  }
  int best = 0;
  float be = 3.4e38f;
  for (int q = 0; q < NB; q++) {
    const int e = nb.idx[(size_t)key * NB + q];
    float er = 0.f;
    for (int j = 0; j < 8; j++) {
      const float d = x[j] - s * (grid_val(G1S, true, e, j) + sh);
      er += w[j] * d * d;
    }
    if (er < be) { be = er; best = e; }
  }
  *err = be;
  return best;
}

void quant_iq1s(const float* x, const float* im, uint8_t* out) {
  const Neighbors& nb = neighbors(illm::FMT_IQ1S);
  float w[256];
  weights_of(x, im, w);
  float sc[8];
  int shn[8];
  float smax = 0.f;
  for (int g = 0; g < 8; g++) {
    const float* xg = x + 32 * g;
    float amax = 0.f;
    for (int i = 0; i < 32; i++) amax = std::max(amax, fabsf(xg[i]));
    float bs = amax, be = 3.4e38f;
    int bsh = 0;
    if (amax > 0.f) {
      for (float f : SCALE_F)
        for (int sn = 0; sn < 2; sn++) {
          const float s = amax / 1.125f * f, sh = sn ? -illm::IQ1S_DELTA : illm::IQ1S_DELTA;
          float tot = 0.f;
          for (int c = 0; c < 4; c++) {
            float er;
            iq1_chunk(nb, xg + 8 * c, w + 32 * g + 8 * c, s, sh, &er);
            tot += er;
          }
          if (tot < be) { be = tot; bs = s; bsh = sn; }
        }
    }
    sc[g] = amax > 0.f ? bs : 0.f;
    shn[g] = bsh;
    smax = std::max(smax, sc[g]);
  }
  const float d = smax / 15.f;
  const uint16_t dh = illm::hd_f32_to_f16(d);
  const float dq = illm::hd_f16_to_f32(dh);
  memset(out, 0, illm::iq_block_bytes(illm::FMT_IQ1S));
  out[0] = (uint8_t)(dh & 0xff);
  out[1] = (uint8_t)(dh >> 8);
  for (int g = 0; g < 8; g++) {
    const int l = dq > 0.f ? (int)lrintf((sc[g] / dq - 1.f) * 0.5f) : 0;
    const int ls = std::min(7, std::max(0, l));
    const float s = dq * (float)(2 * ls + 1);
    const float sh = shn[g] ? -illm::IQ1S_DELTA : illm::IQ1S_DELTA;
    uint32_t h = ((uint32_t)ls << 12) | ((uint32_t)shn[g] << 15);
    for (int c = 0; c < 4; c++) {
      float er;
      const int e = s > 0.f ? iq1_chunk(nb, x + 32 * g + 8 * c, w + 32 * g + 8 * c, s, sh, &er) : 0;
      out[2 + 4 * g + c] = (uint8_t)(e & 0xff);
      h |= (uint32_t)(e >> 8) << (3 * c);
    }
    const uint16_t h16 = (uint16_t)h;
    memcpy(out + 34 + 2 * g, &h16, 2);
  }
}

// IQ1_M chunk: the better of the two shift signs (returns the entry, *neg = sign)
inline int iq1m_chunk(const Neighbors& nb, const float* x, const float* w, float s, int* neg, float* err) {
  float e0, e1;
  const int a = iq1_chunk(nb, x, w, s, illm::IQ1M_DELTA, &e0);
  const int b = iq1_chunk(nb, x, w, s, -illm::IQ1M_DELTA, &e1);
  *neg = e1 < e0;
  *err = e1 < e0 ? e1 : e0;
  return e1 < e0 ? b : a;
}

// iq1_m: a 3-bit scale per 16 weights and a shift sign per 8 (finer than
// iq1_s's per-32 scale and shift, 1.75 instead of 1.5625 bpw): per 16-weight
// sub-block the scale is searched over the same multipliers as iq1_s, every
// chunk taking its best (entry, shift sign); then d = max scale / 15 is
// rounded to f16 and the entries re-chosen for the 3-bit quantized scales
void quant_iq1m(const float* x, const float* im, uint8_t* out) {
  const Neighbors& nb = neighbors(illm::FMT_IQ1S);
  float w[256];
  weights_of(x, im, w);
  float sc[16];
  float smax = 0.f;
  for (int g = 0; g < 16; g++) {
    const float* xg = x + 16 * g;
    float amax = 0.f;
    for (int i = 0; i < 16; i++) amax = std::max(amax, fabsf(xg[i]));
    float bs = amax, be = 3.4e38f;
    if (amax > 0.f) {
      for (float f : SCALE_F) {
        const float sv = amax / 1.125f * f;
        float tot = 0.f;
        for (int c = 0; c < 2; c++) {
          float er;
          int ng;
          iq1m_chunk(nb, xg + 8 * c, w + 16 * g + 8 * c, sv, &ng, &er);
          tot += er;
        }
        if (tot < be) { be = tot; bs = sv; }
      }
    }
    sc[g] = amax > 0.f ? bs : 0.f;
    smax = std::max(smax, sc[g]);
  }
  const float d = smax / 15.f;
  const uint16_t dh = illm::hd_f32_to_f16(d);
  const float dq = illm::hd_f16_to_f32(dh);
  memset(out, 0, illm::iq_block_bytes(illm::FMT_IQ1M));
  uint16_t sw[4] = {0, 0, 0, 0};
  for (int g = 0; g < 16; g++) {
    const int l = dq > 0.f ? (int)lrintf((sc[g] / dq - 1.f) * 0.5f) : 0;
    const int ls = std::min(7, std::max(0, l));
    const float sv = dq * (float)(2 * ls + 1);
    const int ib = g >> 1, hf = g & 1;
    sw[ib >> 1] |= (uint16_t)(ls << (6 * (ib & 1) + 3 * hf));
    for (int c2 = 0; c2 < 2; c2++) {
      const int c = 2 * g + c2;
      float er;
      int ng = 0;
      const int e = sv > 0.f ? iq1m_chunk(nb, x + 8 * c, w + 8 * c, sv, &ng, &er) : 0;
      out[c] = (uint8_t)(e & 0xff);
      out[32 + (c >> 1)] |= (uint8_t)((((e >> 8) & 7) | (ng << 3)) << (4 * (c & 1)));
    }
  }
  for (int i = 0; i < 4; i++) {
    sw[i] |= (uint16_t)(((dh >> (4 * i)) & 15) << 12);
    memcpy(out + 48 + 2 * i, &sw[i], 2);
  }
}

}  // namespace

namespace illm {

// one 256-weight super-block of an IQ format (imatrix slice or null)
void iq_quantize_block(int fmt, const float* x, const float* im, uint8_t* out) {
  if (fmt == FMT_IQ1S) quant_iq1s(x, im, out);
  else if (fmt == FMT_IQ1M) quant_iq1m(x, im, out);
  else quant_iq2(fmt, x, im, out);
}

void iq_dequant_block(int fmt, const uint8_t* b, float* y) {
  const uint64_t* grid = fmt == FMT_IQ2XXS ? G2XXS : (fmt == FMT_IQ2XS ? G2XS : G1S);   // iq1_s / iq1_m: G1S
  for (int c = 0; c < 32; c++) iq_dec8(fmt, b, c, grid, y + 8 * c);
}

}  // namespace illm
