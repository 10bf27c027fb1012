// Host GEMV/GEMM straight from GGUF super-blocks (k-quants q2_K / q4_K /
// q5_K / q6_K and the IQ lattice formats iq2_xxs / iq2_xs / iq1_s / iq1_m):
// the CPU path of KQuantLinear for decode-size M.
//
// Reference: ggml_compute_forward_mul_mat_q_fp32 through ctypes
// (SRC/transformers/low_bit_linear.py:494-529, llama_cpp.py:1154-1185), which
// runs every qtype as an integer dot product against 8-bit activations (q8_K
// for the k-quants).  Design here, one integer kernel for all super-block
// formats:
//   * activations are quantized per 64-element block to int8 (one f32 scale
//     dx; ggml's q8_K uses one per 256) with the 8-element sums of the codes
//     kept (the offset term);
//   * each weight super-block is unpacked once per output row into 256
//     UNSIGNED byte codes plus a (scale, offset) pair per 16 weights such that
//     w = ds * c - dm: q4_K / q5_K / q2_K codes as stored (the min is dm),
//     q6_K codes 0..63 with dm = 32 ds, IQ2 signed grid values biased by 64,
//     IQ1 ternary values + 1 with dm = ds (1 - shift);
//   * the dot product is u8 x s8: AVX-512 VNNI vpdpbusd over 64-byte rows
//     (16 int32 lanes = 4 per 16-weight group, scaled per lane in f32), or
//     AVX2 vpmaddubsw + vpmaddwd (pairwise s16 sums <= 2 * 107 * 127, no
//     saturation);  y = sum_g dx ds_g (c . xq)_g - dx dm_g sum_g(xq).
// The weight is never expanded to f32 and every activation row reuses the
// unpacked block (MR rows per pass).
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../common/iq_grids.h"
#include "../common/kquant.h"

using namespace illm;

namespace {

const uint64_t KG2XXS[256] = ILLM_IQ2XXS_GRID;
const uint64_t KG2XS[512] = ILLM_IQ2XS_GRID;
const uint64_t KG1S[2048] = ILLM_IQ1S_GRID;

inline float h2f(const uint8_t* p) { return hd_f16_to_f32((uint16_t)(p[0] | (p[1] << 8))); }

struct Unpacked {
  alignas(64) uint8_t c[QK_K];
  float ds[16], dm[16];
};

// one super-block -> unsigned codes + per-16 (scale, offset): w = ds * c - dm
void unpack(int fmt, const uint8_t* b, Unpacked& u) {
  if (fmt == FMT_Q4K || fmt == FMT_Q5K) {
    const float d = h2f(b), dmin = h2f(b + 2);
    const bool five = fmt == FMT_Q5K;
    const uint8_t* qh = b + 16;
    const uint8_t* q = b + (five ? 48 : 16);
    for (int j = 0; j < 4; j++) {                 // 64 weights: sub-blocks 2j (low nibbles), 2j + 1 (high)
      for (int hi = 0; hi < 2; hi++) {
        int s, m;
        kq_scale_min_k4(2 * j + hi, b + 4, &s, &m);
        const int sub = 2 * j + hi;
        u.ds[2 * sub] = u.ds[2 * sub + 1] = d * (float)s;
        u.dm[2 * sub] = u.dm[2 * sub + 1] = dmin * (float)m;
        for (int l = 0; l < 32; l++) {
          int v = (q[32 * j + l] >> (4 * hi)) & 15;
          if (five) v |= ((qh[l] >> sub) & 1) << 4;
          u.c[64 * j + 32 * hi + l] = (uint8_t)v;
        }
      }
    }
  } else if (fmt == FMT_Q6K) {
    const uint8_t* ql = b;
    const uint8_t* qh = b + 128;
    const int8_t* sc = (const int8_t*)(b + 192);
    const float d = h2f(b + 208);
    for (int half = 0; half < 2; half++) {
      for (int l = 0; l < 32; l++) {
        const uint8_t* L = ql + 64 * half;
        const uint8_t H = qh[32 * half + l];
        const int base = 128 * half;
        u.c[base + l] = (uint8_t)((L[l] & 15) | (((H >> 0) & 3) << 4));
        u.c[base + 32 + l] = (uint8_t)((L[l + 32] & 15) | (((H >> 2) & 3) << 4));
        u.c[base + 64 + l] = (uint8_t)((L[l] >> 4) | (((H >> 4) & 3) << 4));
        u.c[base + 96 + l] = (uint8_t)((L[l + 32] >> 4) | (((H >> 6) & 3) << 4));
      }
    }
    for (int g = 0; g < 16; g++) {                // 16 weights per int8 scale, value = c - 32
      u.ds[g] = d * (float)sc[g];
      u.dm[g] = 32.f * u.ds[g];
    }
  } else if (fmt == FMT_Q2K) {
    const float d = h2f(b + 80), dmin = h2f(b + 82);
    const uint8_t* q = b + 16;
    for (int half = 0; half < 2; half++)
      for (int j = 0; j < 4; j++)
        for (int l = 0; l < 32; l++) u.c[128 * half + 32 * j + l] = (uint8_t)((q[32 * half + l] >> (2 * j)) & 3);
    for (int g = 0; g < 16; g++) {
      u.ds[g] = d * (float)(b[g] & 15);
      u.dm[g] = dmin * (float)(b[g] >> 4);
    }
  } else if (fmt == FMT_IQ2XXS || fmt == FMT_IQ2XS) {
    // grid magnitudes with per-weight signs: c = sign * mag + 64, dm = 64 ds
    const float d = h2f(b);
    for (int ch = 0; ch < 32; ch++) {
      float db;
      uint32_t s;
      uint64_t q;
      if (fmt == FMT_IQ2XXS) {
        const uint8_t* gp = b + 2 + 8 * (ch >> 2);
        const uint32_t aux = iq_rd32(gp + 4);
        db = d * (0.5f + (float)(aux >> 28)) * 0.25f;
        s = (aux >> (7 * (ch & 3))) & 127;
        q = KG2XXS[gp[ch & 3]];
      } else {
        const uint32_t q16 = iq_rd16(b + 2 + 2 * ch);
        const uint8_t sc = b[66 + (ch >> 2)];
        db = d * (0.5f + (float)((sc >> (4 * ((ch >> 1) & 1))) & 15)) * 0.25f;
        s = q16 >> 9;
        q = KG2XS[q16 & 511];
      }
      s |= (uint32_t)iq_parity7(s) << 7;
      for (int j = 0; j < 8; j++) {
        const int mag = (int)((q >> (8 * j)) & 0xff);
        u.c[8 * ch + j] = (uint8_t)(64 + ((s >> j) & 1 ? -mag : mag));
      }
      u.ds[ch >> 1] = db;                          // both chunks of a 16-group share the scale
      u.dm[ch >> 1] = 64.f * db;
    }
  } else {  // iq1_s / iq1_m: ternary grid + shift, c = g + 1, dm = ds (1 - shift)
    for (int ch = 0; ch < 32; ch++) {
      float db, sh;
      int idx;
      if (fmt == FMT_IQ1S) {
        const float d = h2f(b);
        const uint32_t h = iq_rd16(b + 34 + 2 * (ch >> 2));
        idx = (int)b[2 + ch] | (int)(((h >> (3 * (ch & 3))) & 7) << 8);
        db = d * (float)(2 * ((h >> 12) & 7) + 1);
        sh = (h & 0x8000) ? -IQ1S_DELTA : IQ1S_DELTA;
      } else {
        const uint8_t* sc = b + 48;
        const float d = hd_f16_to_f32(iq1m_d16(sc));
        const int ib = ch >> 2, hf = (ch >> 1) & 1;
        const uint32_t sw = iq_rd16(sc + 2 * (ib >> 1));
        db = d * (float)(2 * ((sw >> (6 * (ib & 1) + 3 * hf)) & 7) + 1);
        const uint32_t h = (uint32_t)(b[32 + (ch >> 1)] >> (4 * (ch & 1))) & 15;
        idx = (int)b[ch] | (int)((h & 7) << 8);
        sh = (h & 8) ? -IQ1M_DELTA : IQ1M_DELTA;
      }
      const uint64_t q = KG1S[idx];
      for (int j = 0; j < 8; j++) u.c[8 * ch + j] = (uint8_t)((int8_t)((q >> (8 * j)) & 0xff) + 1);
      // iq1_s: one shift per 32 weights, iq1_m: per 8 -- a 16-group holds 2
      // chunks; when their shifts differ the offset is applied per chunk below
      u.ds[ch >> 1] = db;
      u.dm[ch >> 1] = db * (1.f - sh);
    }
  }
}

// iq1_m chunks of one 16-group may carry opposite shifts: the per-group dm
// above is then wrong for one chunk -- such blocks take this exact per-chunk
// offset instead (returns true when the block needs it)
bool iq1m_split_offsets(const uint8_t* b, float* dm8) {
  const uint8_t* sc = b + 48;
  const float d = hd_f16_to_f32(iq1m_d16(sc));
  bool split = false;
  for (int ch = 0; ch < 32; ch++) {
    const int ib = ch >> 2, hf = (ch >> 1) & 1;
    const uint32_t sw = iq_rd16(sc + 2 * (ib >> 1));
    const float db = d * (float)(2 * ((sw >> (6 * (ib & 1) + 3 * hf)) & 7) + 1);
    const uint32_t h = (uint32_t)(b[32 + (ch >> 1)] >> (4 * (ch & 1))) & 15;
    const float sh = (h & 8) ? -IQ1M_DELTA : IQ1M_DELTA;
    dm8[ch] = db * (1.f - sh);
    if ((ch & 1) && dm8[ch] != dm8[ch - 1]) split = true;
  }
  return split;
}

// x[m, k] f32 -> per (row, 64-element block): int8 codes and scale (4 per
// super-block: a 4x finer activation grid than ggml's per-256 q8_K), plus the
// 8-element code sums (the offset terms)
void quantize_x(const float* x, int64_t m, int64_t k, int8_t* xq, float* xd, int* xs8) {
  const int64_t nq = k / 64;
#pragma omp parallel for schedule(static) if (m * k > 65536)
  for (int64_t t = 0; t < m * nq; t++) {
    const float* v = x + t * 64;
    float amax = 0.f;
    for (int j = 0; j < 64; j++) amax = std::max(amax, fabsf(v[j]));
    const float d = amax / 127.f;
    const float id = d > 0.f ? 1.f / d : 0.f;
    for (int c = 0; c < 8; c++) {
      int s = 0;
      for (int j = 0; j < 8; j++) {
        const int q = (int)lrintf(v[8 * c + j] * id);
        xq[t * 64 + 8 * c + j] = (int8_t)q;
        s += q;
      }
      xs8[t * 8 + c] = s;
    }
    xd[t] = d;
  }
}

constexpr int MR = 8;

// sum over the block of dm * (dx * code sum): per 16-group, or per 8-chunk
// where an iq1_m group's two chunks carry different shifts
inline float offset_term(const Unpacked& u, bool split, const float* dm8, const int* s8, const float* dx4) {
  float c = 0.f;
  if (split) {
    for (int ch = 0; ch < 32; ch++) c += dm8[ch] * dx4[ch >> 3] * (float)s8[ch];
  } else {
    for (int g = 0; g < 16; g++) c += u.dm[g] * dx4[g >> 2] * (float)(s8[2 * g] + s8[2 * g + 1]);
  }
  return c;
}

// per-16-group integer dots of one unpacked block against one activation row
__attribute__((target("avx512f,avx512bw,avx512vnni,avx512vl")))
inline void dots_avx512(const Unpacked& u, const int8_t* xq, const float* dx4, __m512& acc) {
  for (int z = 0; z < 4; z++) {                   // 64 codes = 4 groups of 16
    const __m512i q = _mm512_load_si512((const void*)(u.c + 64 * z));
    const __m512i xv = _mm512_loadu_si512((const void*)(xq + 64 * z));
    const __m512i dp = _mm512_dpbusd_epi32(_mm512_setzero_si512(), q, xv);
    // lane l holds a 4-element partial of group 4 z + l / 4
    const __m512 sc = _mm512_set_ps(u.ds[4 * z + 3], u.ds[4 * z + 3], u.ds[4 * z + 3], u.ds[4 * z + 3],
                                    u.ds[4 * z + 2], u.ds[4 * z + 2], u.ds[4 * z + 2], u.ds[4 * z + 2],
                                    u.ds[4 * z + 1], u.ds[4 * z + 1], u.ds[4 * z + 1], u.ds[4 * z + 1],
                                    u.ds[4 * z], u.ds[4 * z], u.ds[4 * z], u.ds[4 * z]);
    acc = _mm512_fmadd_ps(_mm512_cvtepi32_ps(dp), _mm512_mul_ps(sc, _mm512_set1_ps(dx4[z])), acc);
  }
}

__attribute__((target("avx512f,avx512bw,avx512vnni,avx512vl")))
void rows_avx512(int fmt, const int8_t* xq, const float* xd, const int* xs8, int64_t m, const uint8_t* w,
                 int64_t r0, int64_t r1, int64_t k, int64_t n, float* y) {
  const int64_t nb = k / QK_K;
  const int bb = kq_block_bytes(fmt);
  Unpacked u;
  float dm8[32];
  for (int64_t r = r0; r < r1; r++) {
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m512 acc[MR];
      float corr[MR];
      for (int i = 0; i < MR; i++) { acc[i] = _mm512_setzero_ps(); corr[i] = 0.f; }
      for (int64_t b = 0; b < nb; b++) {
        const uint8_t* blk = w + (r * nb + b) * bb;
        unpack(fmt, blk, u);
        const bool split = fmt == FMT_IQ1M && iq1m_split_offsets(blk, dm8);
        for (int i = 0; i < mi; i++) {
          const int64_t t = (i0 + i) * nb + b;
          const float* dx4 = xd + 4 * t;
          dots_avx512(u, xq + t * QK_K, dx4, acc[i]);
          corr[i] -= offset_term(u, split, dm8, xs8 + t * 32, dx4);
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

void rows_avx2(int fmt, const int8_t* xq, const float* xd, const int* xs8, int64_t m, const uint8_t* w,
               int64_t r0, int64_t r1, int64_t k, int64_t n, float* y) {
  const int64_t nb = k / QK_K;
  const int bb = kq_block_bytes(fmt);
  const __m256i ones = _mm256_set1_epi16(1);
  Unpacked u;
  float dm8[32];
  for (int64_t r = r0; r < r1; r++) {
    for (int64_t i0 = 0; i0 < m; i0 += MR) {
      const int mi = (int)std::min<int64_t>(MR, m - i0);
      __m256 acc[MR];
      float corr[MR];
      for (int i = 0; i < MR; i++) { acc[i] = _mm256_setzero_ps(); corr[i] = 0.f; }
      for (int64_t b = 0; b < nb; b++) {
        const uint8_t* blk = w + (r * nb + b) * bb;
        unpack(fmt, blk, u);
        const bool split = fmt == FMT_IQ1M && iq1m_split_offsets(blk, dm8);
        for (int i = 0; i < mi; i++) {
          const int64_t t = (i0 + i) * nb + b;
          const int8_t* xr = xq + t * QK_K;
          const float* dx4 = xd + 4 * t;
          for (int z = 0; z < 8; z++) {            // 32 codes = 2 groups: lanes 0-3 group 2z, 4-7 group 2z + 1
            const __m256i q = _mm256_load_si256((const __m256i*)(u.c + 32 * z));
            const __m256i xv = _mm256_loadu_si256((const __m256i*)(xr + 32 * z));
            const __m256i p = _mm256_madd_epi16(_mm256_maddubs_epi16(q, xv), ones);
            const __m256 sc = _mm256_set_ps(u.ds[2 * z + 1], u.ds[2 * z + 1], u.ds[2 * z + 1], u.ds[2 * z + 1],
                                            u.ds[2 * z], u.ds[2 * z], u.ds[2 * z], u.ds[2 * z]);
            acc[i] = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p), _mm256_mul_ps(sc, _mm256_set1_ps(dx4[z >> 1])), acc[i]);
          }
          corr[i] -= offset_term(u, split, dm8, xs8 + t * 32, dx4);
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

// y[m, n] = x[m, k] @ W[n, k]^T, W in GGUF super-blocks (isa: 0 auto, 1 AVX2, 2 AVX-512 VNNI)
void illm_kq_gemm_int(int fmt, const float* x, int64_t m, const uint8_t* w, int64_t n, int64_t k, float* y,
                      int isa) {
  const int64_t nb = k / QK_K;
  std::vector<int8_t> xq((size_t)(m * k));
  std::vector<float> xd((size_t)(m * nb * 4));
  std::vector<int> xs8((size_t)(m * nb * 32));
  quantize_x(x, m, k, xq.data(), xd.data(), xs8.data());
  const bool v512 = (isa == 2 || isa == 0) && has_vnni512();   // a forced 2 on a host without VNNI runs AVX2
  constexpr int64_t RB = 8;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t r0 = 0; r0 < n; r0 += RB) {
    const int64_t r1 = std::min(n, r0 + RB);
    if (v512) rows_avx512(fmt, xq.data(), xd.data(), xs8.data(), m, w, r0, r1, k, n, y);
    else rows_avx2(fmt, xq.data(), xd.data(), xs8.data(), m, w, r0, r1, k, n, y);
  }
}

}  // extern "C"
