// Low-bit weight x bf16/f16 activation "skinny GEMM" for M <= 64 rows
// (decode, batched decode, speculative verify) on gfx950 MFMA.
//
// Reference op: xe_linear.forward_new / xe_batch.batch_forward /
// xe_linear.mlp_forward_xpu (SRC/transformers/low_bit_linear.py:698-708,
// models/common.py:146-161).  Design is MI355X-first:
//   * weights are pre-tiled (formats.h) so one wave64 streams a 16-row x
//     128-k chunk record with ONE global_load_dwordx4 per lane per KiB of
//     codes (fully coalesced) plus one 16-B scale load from the same record;
//     no LDS round trip for the weight stream;
//   * dequant happens in registers straight into the MFMA A fragment
//     (int4: the bf16 0x4300|q / f16 0x6400|q magic, fp4/fp8: the gfx950
//     v_cvt_scalef32_pk_* converters, nf4: a 256-entry pair table in LDS);
//   * the zero-point/offset of integer formats is folded in with one extra
//     MFMA against an all-ones A fragment (sum of x per block) instead of
//     per-element VALU subtracts;
//   * per-64-block scales are applied on the 4 f32 accumulators per lane;
//   * two kernels: lowbit_gemv4_kernel (M <= 16, the decode hot path: x in
//     LDS, pre-scaled f16 A fragments, one accumulator per tile) and
//     lowbit_gemv_kernel (17..64 rows: MT 16-row M tiles per wave, 4 waves
//     split K and reduce through LDS);
//   * a workgroup-level split-K over blockIdx.y writes f32 partial slabs that
//     are summed by the consumer (fused add+RMSNorm / reduce) kernel.
#pragma once
#include <type_traits>

#include "../common/quant_block.h"
#include "gemv_args.h"
#include "illm_device.h"

namespace illm {

template <typename T> struct Magic;
template <> struct Magic<BF16> {
  static constexpr uint32_t k4 = 0x43004300u;  // bf16(128 + q)
  static constexpr float off = 128.f;
  static constexpr uint32_t one2 = 0x3F803F80u;
};
template <> struct Magic<F16> {
  static constexpr uint32_t k4 = 0x64006400u;  // f16(1024 + q)
  static constexpr float off = 1024.f;
  static constexpr uint32_t one2 = 0x3C003C00u;
};

// ---- decoders: one 8-code group (k-step) -> 16-byte A fragment ------------
template <int DK, typename T>
__device__ __forceinline__ uint4 decode4(uint32_t u, const uint32_t* lut2) {
  uint4 r;
  if constexpr (DK == DK_INT4S || DK == DK_INT4A) {
    r.x = (u & 0x000F000Fu) | Magic<T>::k4;
    r.y = ((u >> 4) & 0x000F000Fu) | Magic<T>::k4;
    r.z = ((u >> 8) & 0x000F000Fu) | Magic<T>::k4;
    r.w = ((u >> 12) & 0x000F000Fu) | Magic<T>::k4;
  } else if constexpr (DK == DK_FP4) {
    if constexpr (std::is_same<T, BF16>::value) {
      r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 0));
      r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 1));
      r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 2));
      r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 3));
    } else {
      r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 0));
      r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 1));
      r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 2));
      r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 3));
    }
  } else {  // DK_LUT4
    r.x = lut2[u & 0xff];
    r.y = lut2[(u >> 8) & 0xff];
    r.z = lut2[(u >> 16) & 0xff];
    r.w = lut2[u >> 24];
  }
  return r;
}

template <int DK, typename T>
__device__ __forceinline__ uint32_t dec8_pair(uint32_t u, bool hi) {
  if constexpr (DK == DK_FP8E4) {
    if constexpr (std::is_same<T, BF16>::value)
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u, 1.0f, false));
    else
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u, 1.0f, false));
  } else if constexpr (DK == DK_FP8E5) {
    if constexpr (std::is_same<T, BF16>::value)
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u, 1.0f, false));
    else
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u, 1.0f, false));
  } else {
    // integer bytes: signed codes are biased by 128 (xor 0x80) so every code
    // is an exact small non-negative integer in bf16/f16
    if constexpr (DK == DK_INT8S) u ^= 0x80808080u;
    const int sh = hi ? 16 : 0;
    return pack2<T>((float)((u >> sh) & 0xff), (float)((u >> (sh + 8)) & 0xff));
  }
}

// 8 bytes (two dwords) -> 16-byte A fragment
template <int DK, typename T>
__device__ __forceinline__ uint4 decode8(uint32_t lo, uint32_t hi) {
  uint4 r;
  r.x = dec8_pair<DK, T>(lo, false);
  r.y = dec8_pair<DK, T>(lo, true);
  r.z = dec8_pair<DK, T>(hi, false);
  r.w = dec8_pair<DK, T>(hi, true);
  return r;
}

// per-block coefficients: acc += cd * P + cx * X
template <int DK, typename T>
__device__ __forceinline__ void block_coef(float d, float m, float& cd, float& cx) {
  cd = d;
  if constexpr (DK == DK_INT4S) cx = -(Magic<T>::off + 8.f) * d;
  else if constexpr (DK == DK_INT4A) cx = m - Magic<T>::off * d;
  else if constexpr (DK == DK_INT8S) cx = -128.f * d;
  else if constexpr (DK == DK_INT8A) cx = m;
  else cx = 0.f;
}

template <int DK, typename T, int MT, int EPI>
__global__ void __launch_bounds__(256) lowbit_gemv_kernel(const GemvArgs a) {
  constexpr int BITS = dk_bits(DK);
  constexpr bool NEEDX = dk_needx(DK);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  __shared__ float4 red[4][MT][64];
  __shared__ uint32_t lut2[DK == DK_LUT4 ? 256 : 1];
  if constexpr (DK == DK_LUT4) {
    const int i = threadIdx.x;
    lut2[i] = pack2<T>(hd_lut4(a.lut_fmt, i & 15), hd_lut4(a.lut_fmt, i >> 4));
    __syncthreads();
  }

  int tile, wk, nwk;
  if constexpr (EPI == EPI_GLU) {
    tile = blockIdx.x * 2 + (wave >> 1);
    wk = blockIdx.y * 2 + (wave & 1);
    nwk = gridDim.y * 2;
  } else {
    tile = blockIdx.x;
    wk = blockIdx.y * 4 + wave;
    nwk = gridDim.y * 4;
  }
  const int cpw = (a.KC + nwk - 1) / nwk;
  const int c0 = wk * cpw;
  const int c1 = min(a.KC, c0 + cpw);

  // activation row pointers (clamped, masked after load)
  const uint16_t* xr[MT];
  bool mok[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) {
    int m = mt * 16 + r16;
    mok[mt] = m < a.M;
    xr[mt] = a.x + (size_t)(mok[mt] ? m : 0) * a.ldx;
  }
  const uint4 ones = make_uint4(Magic<T>::one2, Magic<T>::one2, Magic<T>::one2, Magic<T>::one2);

  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; mt++) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const uint8_t* tptr = a.w + (size_t)tile * dk_tile_bytes(DK, a.KC);
  // Software pipeline: a ring of PF chunks is always in flight.  Loads are
  // issued unconditionally (clamped index: tail re-loads are L2 hits) so
  // hipcc keeps counted vmcnt waits instead of branching around loads.
  struct Chunk {
    uint4 q0, q1, sc, mn;
    uint4 xb[4][MT];
  };
  auto load_chunk = [&](Chunk& ch, int c) {
    c = min(c, c1 - 1);
    const uint8_t* rec = tptr + (size_t)c * dk_code_chunk(DK);
    ch.q0 = *(const uint4*)(rec + lane * 16);
    if constexpr (BITS == 8) ch.q1 = *(const uint4*)(rec + 1024 + lane * 16);
    // C-fragment rows 4g..4g+3: one dword (blk0 | blk1 << 16) per row and chunk
    const uint32_t* sp = (const uint32_t*)(tptr + (size_t)a.KC * dk_code_chunk(DK)) + (size_t)(4 * g) * a.KC + c;
    ch.sc = make_uint4(sp[0], sp[a.KC], sp[2 * a.KC], sp[3 * a.KC]);
    if constexpr (dk_has_min(DK)) {
      const uint32_t* mp = sp + 16 * a.KC;
      ch.mn = make_uint4(mp[0], mp[a.KC], mp[2 * a.KC], mp[3 * a.KC]);
    }
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int kk = c * 128 + 32 * s + 8 * g;
      const bool kok = kk < a.K;
#pragma unroll
      for (int mt = 0; mt < MT; mt++) {
        const uint4 B = *(const uint4*)(xr[mt] + (kok ? kk : 0));
        ch.xb[s][mt] = (mok[mt] && kok) ? B : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto compute_chunk = [&](const Chunk& ch) {
#pragma unroll
    for (int blk = 0; blk < 2; blk++) {
      f32x4 P[MT], X[MT];
#pragma unroll
      for (int mt = 0; mt < MT; mt++) {
        P[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        X[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ss = 0; ss < 2; ss++) {
        const int s = blk * 2 + ss;
        uint4 A;
        if constexpr (BITS == 4) {
          const uint32_t u = s == 0 ? ch.q0.x : (s == 1 ? ch.q0.y : (s == 2 ? ch.q0.z : ch.q0.w));
          A = decode4<DK, T>(u, lut2);
        } else {
          const uint4& qq = blk == 0 ? ch.q0 : ch.q1;
          A = ss == 0 ? decode8<DK, T>(qq.x, qq.y) : decode8<DK, T>(qq.z, qq.w);
        }
#pragma unroll
        for (int mt = 0; mt < MT; mt++) {
          P[mt] = mfma16<T>(A, ch.xb[s][mt], P[mt]);
          if constexpr (NEEDX) X[mt] = mfma16<T>(ones, ch.xb[s][mt], X[mt]);
        }
      }
      // this 64-block's scales: lane rows n = 4g + i
      const int sh = blk * 16;
      const float d[4] = {f16_to_f32((ch.sc.x >> sh) & 0xffff), f16_to_f32((ch.sc.y >> sh) & 0xffff),
                          f16_to_f32((ch.sc.z >> sh) & 0xffff), f16_to_f32((ch.sc.w >> sh) & 0xffff)};
      float mm[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (dk_has_min(DK)) {
        mm[0] = f16_to_f32((ch.mn.x >> sh) & 0xffff); mm[1] = f16_to_f32((ch.mn.y >> sh) & 0xffff);
        mm[2] = f16_to_f32((ch.mn.z >> sh) & 0xffff); mm[3] = f16_to_f32((ch.mn.w >> sh) & 0xffff);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        float cd, cx;
        block_coef<DK, T>(d[i], mm[i], cd, cx);
#pragma unroll
        for (int mt = 0; mt < MT; mt++) {
          acc[mt][i] += cd * P[mt][i];
          if constexpr (NEEDX) acc[mt][i] += cx * X[mt][i];
        }
      }
    }
  };
  constexpr int PF = MT == 1 ? 4 : 2;
  if (c0 < c1) {
    Chunk ring[PF];
#pragma unroll
    for (int u = 0; u < PF; u++) load_chunk(ring[u], c0 + u);
    for (int c = c0; c < c1; c += PF) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        if (c + u < c1) compute_chunk(ring[u]);
        load_chunk(ring[u], c + u + PF);
      }
    }
  }

#pragma unroll
  for (int mt = 0; mt < MT; mt++) red[wave][mt][lane] = make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
  __syncthreads();
  if (wave != 0) return;

  if constexpr (EPI == EPI_GLU) {
    // tile pair p: rows of tile 2p are gate rows, tile 2p+1 up rows
    const int p = blockIdx.x;
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
      const int m = mt * 16 + r16;
      float4 g0 = red[0][mt][lane], g1 = red[1][mt][lane], u0 = red[2][mt][lane], u1 = red[3][mt][lane];
      float gv[4] = {g0.x + g1.x, g0.y + g1.y, g0.z + g1.z, g0.w + g1.w};
      float uv[4] = {u0.x + u1.x, u0.y + u1.y, u0.z + u1.z, u0.w + u1.w};
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; i++) o[i] = (a.act == 0 ? silu_f(gv[i]) : gelu_tanh_f(gv[i])) * uv[i];
      const int n0 = p * 16 + 4 * g;
      if (m < a.M && n0 < a.N) {
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n0;
        if (n0 + 3 < a.N) {
          *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
        } else {
          for (int i = 0; i < 4 && n0 + i < a.N; i++) y[i] = from_f32<T>(o[i]);
        }
      }
    }
  } else {
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
      const int m = mt * 16 + r16;
      float4 v0 = red[0][mt][lane], v1 = red[1][mt][lane], v2 = red[2][mt][lane], v3 = red[3][mt][lane];
      float o[4] = {v0.x + v1.x + v2.x + v3.x, v0.y + v1.y + v2.y + v3.y,
                    v0.z + v1.z + v2.z + v3.z, v0.w + v1.w + v2.w + v3.w};
      const int n0 = tile * 16 + 4 * g;
      if (m >= a.M || n0 >= a.N) continue;
      if constexpr (EPI == EPI_PARTIAL) {
        float* ws = (float*)a.out + ((size_t)blockIdx.y * a.M + m) * a.N + n0;
        if (n0 + 3 < a.N && (a.N & 3) == 0) {
          *(float4*)ws = make_float4(o[0], o[1], o[2], o[3]);
        } else {
          for (int i = 0; i < 4 && n0 + i < a.N; i++) ws[i] = o[i];
        }
      } else {
        if (a.bias) {
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] += (n0 + i < a.N) ? to_f32<T>(a.bias[n0 + i]) : 0.f;
        }
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n0;
        if (n0 + 3 < a.N && ((a.ldo | n0) & 3) == 0) {
          *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
        } else {
          for (int i = 0; i < 4 && n0 + i < a.N; i++) y[i] = from_f32<T>(o[i]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// v4 (M <= 16): pre-scaled f16 A fragments, one MFMA accumulator per tile.
// x[0:M, K-slice] is staged once per workgroup in LDS (16-B vector loads,
// read back as MFMA B fragments with ds_read_b128); each wave owns TPW whole
// 16-row tiles over the workgroup's K range (TPW = 2 for GLU: gate tile + up
// tile in the same lanes -> act(g) * u in registers), so there is no
// cross-wave reduction, and only weight records live in the PF-deep register
// prefetch ring.  Why pre-scaled: v1 accumulates each 64-element block in a fresh MFMA accumulator and then
// read it out (v_accvgpr_read) to apply the block scale: a dependent
// MFMA -> VALU chain per block that, at the ~2 waves/SIMD a GEMV grid gives,
// is not hidden.  Here the block scale (and min) is applied to the decoded
// weights with packed f16 VALU (exact (q-8) via the 0x6400 magic, then one
// rounding of (q-8)*d), so all chunks of a tile chain into ONE accumulator,
// the all-ones offset MFMA disappears and there is no per-block readout.
// Activations are converted to f16 while being staged into LDS (clamped to
// the f16 range), accumulation stays f32, outputs are written in T.
// ---------------------------------------------------------------------------
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t as_u(h2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t bytes01(uint32_t u) { return __builtin_amdgcn_perm(0u, u, 0x0c010c00u); }
__device__ __forceinline__ uint32_t bytes23(uint32_t u) { return __builtin_amdgcn_perm(0u, u, 0x0c030c02u); }

// scaled A fragment (8 f16) for one k-step; d2 / m2 = (d, d) / (m, m)
template <int DK>
__device__ __forceinline__ uint4 scaled_a4(uint32_t u, h2 d2, h2 m2, const uint32_t* lut2) {
  uint32_t w[4];
  if constexpr (DK == DK_INT4S || DK == DK_INT4A) {
    w[0] = (u & 0x000F000Fu) | 0x64006400u;
    w[1] = ((u >> 4) & 0x000F000Fu) | 0x64006400u;
    w[2] = ((u >> 8) & 0x000F000Fu) | 0x64006400u;
    w[3] = ((u >> 12) & 0x000F000Fu) | 0x64006400u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if constexpr (DK == DK_INT4S) w[i] = as_u((as_h2(w[i]) - h2{(_Float16)1032.f, (_Float16)1032.f}) * d2);
      else w[i] = as_u(__builtin_elementwise_fma(as_h2(w[i]) - h2{(_Float16)1024.f, (_Float16)1024.f}, d2, m2));
    }
  } else {
    if constexpr (DK == DK_FP4) {
      w[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 0));
      w[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 1));
      w[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 2));
      w[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 3));
    } else {  // DK_LUT4: f16 pair table
      w[0] = lut2[u & 0xff];
      w[1] = lut2[(u >> 8) & 0xff];
      w[2] = lut2[(u >> 16) & 0xff];
      w[3] = lut2[u >> 24];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = as_u(as_h2(w[i]) * d2);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int DK>
__device__ __forceinline__ uint4 scaled_a8(uint32_t lo, uint32_t hi, h2 d2, h2 m2) {
  uint32_t w[4];
  if constexpr (DK == DK_FP8E4 || DK == DK_FP8E5) {
    if constexpr (DK == DK_FP8E4) {
      w[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(lo, 1.0f, false));
      w[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(lo, 1.0f, true));
      w[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(hi, 1.0f, false));
      w[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(hi, 1.0f, true));
    } else {
      w[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(lo, 1.0f, false));
      w[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(lo, 1.0f, true));
      w[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(hi, 1.0f, false));
      w[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(hi, 1.0f, true));
    }
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = as_u(as_h2(w[i]) * d2);
  } else {
    // bytes -> f16(1024 + byte) via v_perm + magic; signed codes biased by 128
    if constexpr (DK == DK_INT8S) { lo ^= 0x80808080u; hi ^= 0x80808080u; }
    w[0] = bytes01(lo) | 0x64006400u;
    w[1] = bytes23(lo) | 0x64006400u;
    w[2] = bytes01(hi) | 0x64006400u;
    w[3] = bytes23(hi) | 0x64006400u;
    const _Float16 off = DK == DK_INT8S ? (_Float16)1152.f : (_Float16)1024.f;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if constexpr (DK == DK_INT8S) w[i] = as_u((as_h2(w[i]) - h2{off, off}) * d2);
      else w[i] = as_u(__builtin_elementwise_fma(as_h2(w[i]) - h2{off, off}, d2, m2));
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// MOE = grouped GEMV over experts (FlashMoE decode): blockIdx.z = expert e,
// its token-expert pairs are moe_rows[moe_off[e] .. moe_off[e+1]) (<= 16),
// weights at a.w + e * w_stride, x row = pair / moe_xdiv, output row = pair.
// QS = quad scales: the workgroup's chunk range starts at a multiple of 4 and
// KC % 4 == 0, so a row's scales (and mins) of 4 consecutive chunks arrive in
// ONE 16-B load per 4 code loads (one scale load per chunk measured ~10%
// slower); the quad for chunks c+4..c+7 is fetched while c..c+3 compute.
template <int DK, typename T, int EPI, int TPW, bool MOE = false, bool QS = true>
__global__ void __launch_bounds__(512) lowbit_gemv4_kernel(const GemvArgs a) {
  constexpr int BITS = dk_bits(DK);
  constexpr int PF = 4;
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  __shared__ uint32_t lut2[DK == DK_LUT4 ? 256 : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  int Mloc = a.M;
  const uint8_t* wbase = a.w;
  const int32_t* prow = nullptr;
  if constexpr (MOE) {
    const int e = blockIdx.z;
    const int m0 = a.moe_off[e];
    Mloc = min(16, a.moe_off[e + 1] - m0);
    if (Mloc <= 0) return;                // expert not routed to: whole block exits
    wbase += (size_t)e * a.w_stride;
    prow = a.moe_rows + m0;
  }
  auto xrow_of = [&](int m) -> int { if constexpr (MOE) return prow[m] / a.moe_xdiv; else return m; };
  auto orow_of = [&](int m) -> int { if constexpr (MOE) return prow[m]; else return m; };

  const int nks = gridDim.y;
  const int cpk = a.cpk > 0 ? a.cpk : (a.KC + nks - 1) / nks;
  const int c0 = blockIdx.y * cpk;
  const int c1 = min(a.KC, c0 + cpk);
  const int kbase = c0 * 128;
  const int kw = (c1 - c0) * 128;
  const int lds_ld = kw + 8;
  const int NT = (a.N * (EPI == EPI_GLU ? 2 : 1) + 15) / 16;
  const int tile0 = (blockIdx.x * (int)(blockDim.x >> 6) + wave) * TPW;
  const bool wave_on = tile0 < NT && c0 < c1;
  const size_t TB = (size_t)dk_tile_bytes(DK, a.KC);
  const size_t soff = (size_t)a.KC * dk_code_chunk(DK) + (size_t)r16 * a.KC * 4;   // this row's scale dwords
  const size_t moff = soff + (size_t)16 * a.KC * 4;
  const uint8_t* tb[TPW];
#pragma unroll
  for (int t = 0; t < TPW; t++) tb[t] = wbase + (size_t)min(tile0 + t, NT - 1) * TB;

  struct Chunk {
    uint4 q[TPW][BITS / 4];
    uint32_t sc[TPW];     // !QS only
    uint32_t mn[TPW];
  };
  auto load_chunk = [&](Chunk& ch, int c) {
    c = min(c, c1 - 1);
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      const uint8_t* rec = tb[t] + (size_t)c * dk_code_chunk(DK);
      ch.q[t][0] = *(const uint4*)(rec + lane * 16);
      if constexpr (BITS == 8) ch.q[t][1] = *(const uint4*)(rec + 1024 + lane * 16);
      if constexpr (!QS) {
        ch.sc[t] = *(const uint32_t*)(tb[t] + soff + (size_t)c * 4);
        if constexpr (dk_has_min(DK)) ch.mn[t] = *(const uint32_t*)(tb[t] + moff + (size_t)c * 4);
      }
    }
  };
  uint4 sq[TPW], sqn[TPW], mq[TPW], mqn[TPW];     // quad scale / min registers
  const int last_quad = ((c1 - 1) >> 2) << 2;
  auto load_quad = [&](uint4 (&s)[TPW], uint4 (&m)[TPW], int c) {
    c = min(c, last_quad);
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      s[t] = *(const uint4*)(tb[t] + soff + (size_t)c * 4);
      if constexpr (dk_has_min(DK)) m[t] = *(const uint4*)(tb[t] + moff + (size_t)c * 4);
    }
  };
  Chunk ring[PF];
  if (wave_on) {
    if constexpr (QS) load_quad(sq, mq, c0);
#pragma unroll
    for (int u = 0; u < PF; u++) load_chunk(ring[u], c0 + u);
  }
  if constexpr (DK == DK_LUT4) {
    if (threadIdx.x < 256)
      lut2[threadIdx.x] = pack2<F16>(hd_lut4(a.lut_fmt, threadIdx.x & 15), hd_lut4(a.lut_fmt, threadIdx.x >> 4));
  }
  {  // stage x[0:M, kbase:kbase+kw] -> LDS as f16
    const int vpr = kw / 8;
    for (int v = threadIdx.x; v < Mloc * vpr; v += blockDim.x) {
      const int m = v / vpr, kk = (v % vpr) * 8;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (kbase + kk < a.K && a.xpart) {
        // fused activation of the gate/up GEMV: 8 consecutive k stay inside one 16-column tile
        const int k0 = kbase + kk;
        const size_t gc = (size_t)(k0 >> 4) * 32 + (k0 & 15);
        const size_t ld = (size_t)2 * a.K;
        float gv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, uv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int sp = 0; sp < a.xpart_ns; sp++) {
          const float* row = a.xpart + ((size_t)sp * a.M + xrow_of(m)) * ld;
          const float4 g0 = *(const float4*)(row + gc), g1 = *(const float4*)(row + gc + 4);
          const float4 u0 = *(const float4*)(row + gc + 16), u1 = *(const float4*)(row + gc + 20);
          gv[0] += g0.x; gv[1] += g0.y; gv[2] += g0.z; gv[3] += g0.w;
          gv[4] += g1.x; gv[5] += g1.y; gv[6] += g1.z; gv[7] += g1.w;
          uv[0] += u0.x; uv[1] += u0.y; uv[2] += u0.z; uv[3] += u0.w;
          uv[4] += u1.x; uv[5] += u1.y; uv[6] += u1.z; uv[7] += u1.w;
        }
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float o2[2];
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const float gg = gv[2 * i + j];
            // activation output rounded to T (what the GLU epilogue would have written)
            const float act = to_f32<T>(from_f32<T>((a.act == 0 ? silu_f(gg) : gelu_tanh_f(gg)) * uv[2 * i + j]));
            o2[j] = fminf(fmaxf(act, -65504.f), 65504.f);
          }
          w[i] = pack2<F16>(o2[0], o2[1]);
        }
        val = make_uint4(w[0], w[1], w[2], w[3]);
      } else if (kbase + kk < a.K) {
        val = *(const uint4*)(a.x + (size_t)xrow_of(m) * a.ldx + kbase + kk);
        if constexpr (std::is_same<T, BF16>::value) {
          uint32_t w[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const float lo = fminf(fmaxf(bf16_to_f32(w[i] & 0xffff), -65504.f), 65504.f);
            const float hi = fminf(fmaxf(bf16_to_f32(w[i] >> 16), -65504.f), 65504.f);
            w[i] = pack2<F16>(lo, hi);
          }
          val = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
      *(uint4*)(xs + m * lds_ld + kk) = val;
    }
  }
  __syncthreads();
  if (!wave_on) return;

  const bool mok = r16 < Mloc;
  const uint16_t* xrow = xs + (mok ? r16 : 0) * lds_ld + 8 * g;
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto pick = [&](uint32_t v, int blk) -> h2 {
    // broadcast half blk of the row's scale dword to both halves of an h2
    return as_h2(__builtin_amdgcn_perm(0u, v, blk == 0 ? 0x01000100u : 0x03020302u));
  };
  auto comp = [](const uint4& v, int u) -> uint32_t { return u == 0 ? v.x : (u == 1 ? v.y : (u == 2 ? v.z : v.w)); };
  // u = position of the chunk inside its quad (static in the unrolled loops)
  auto compute_chunk = [&](const Chunk& ch, int c, int u) {
    const uint16_t* xc = xrow + (c - c0) * 128;
    uint4 B[4];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint4 v = *(const uint4*)(xc + 32 * s);
      B[s] = mok ? v : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      const uint32_t scw = QS ? comp(sq[t], u) : ch.sc[t];
      const uint32_t mnw = dk_has_min(DK) ? (QS ? comp(mq[t], u) : ch.mn[t]) : 0u;
#pragma unroll
      for (int blk = 0; blk < 2; blk++) {
        const h2 d2 = pick(scw, blk);
        h2 m2 = h2{(_Float16)0.f, (_Float16)0.f};
        if constexpr (dk_has_min(DK)) m2 = pick(mnw, blk);
#pragma unroll
        for (int ss = 0; ss < 2; ss++) {
          const int s = blk * 2 + ss;
          uint4 A;
          if constexpr (BITS == 4) {
            const uint4& q0 = ch.q[t][0];
            const uint32_t w = s == 0 ? q0.x : (s == 1 ? q0.y : (s == 2 ? q0.z : q0.w));
            A = scaled_a4<DK>(w, d2, m2, lut2);
          } else {
            const uint4& qq = ch.q[t][blk];
            A = ss == 0 ? scaled_a8<DK>(qq.x, qq.y, d2, m2) : scaled_a8<DK>(qq.z, qq.w, d2, m2);
          }
          acc[t] = mfma16<F16>(A, B[s], acc[t]);
        }
      }
    }
  };
  auto next_quad = [&]() {
    if constexpr (QS) {
#pragma unroll
      for (int t = 0; t < TPW; t++) {
        sq[t] = sqn[t];
        if constexpr (dk_has_min(DK)) mq[t] = mqn[t];
      }
    }
  };

  // Steady state: unconditional loads (hipcc keeps exact counted vmcnt
  // waits); the last < 2*PF chunks run a guarded tail.
  const int c1u = __builtin_amdgcn_readfirstlane(c1);
  int c = __builtin_amdgcn_readfirstlane(c0);
  for (; c + 2 * PF <= c1u; c += PF) {
#pragma unroll
    for (int u = 0; u < PF; u++) {
      compute_chunk(ring[u], c + u, u);
      load_chunk(ring[u], c + u + PF);
      if (QS && u == 0) load_quad(sqn, mqn, c + PF);
    }
    next_quad();
  }
#pragma unroll
  for (int u = 0; u < PF; u++) {
    if (c + u < c1u) compute_chunk(ring[u], c + u, u);
    load_chunk(ring[u], c + u + PF);
    if (QS && u == 0) load_quad(sqn, mqn, c + PF);
  }
  next_quad();
  c += PF;
#pragma unroll
  for (int u = 0; u < PF; u++)
    if (c + u < c1u) compute_chunk(ring[u], c + u, u);

  // ---- epilogue: lane holds rows 16*tile + 4g + i, column r16
  if (r16 >= Mloc) return;
  const int m = orow_of(r16);
  if constexpr (EPI == EPI_GLU) {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const float gv = acc[0][i], uv = acc[TPW - 1][i];
      o[i] = (a.act == 0 ? silu_f(gv) : gelu_tanh_f(gv)) * uv;
    }
    const int n0 = (tile0 / 2) * 16 + 4 * g;
    if (n0 < a.N) {
      uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n0;
      if (n0 + 3 < a.N) *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
      else for (int i = 0; i < 4 && n0 + i < a.N; i++) y[i] = from_f32<T>(o[i]);
    }
  } else {
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      const int n0 = (tile0 + t) * 16 + 4 * g;
      if (tile0 + t >= NT || n0 >= a.N) continue;
      float o[4] = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
      if constexpr (EPI == EPI_PARTIAL) {
        float* ws = (float*)a.out + ((size_t)blockIdx.y * a.M + m) * a.N + n0;
        if (n0 + 3 < a.N && (a.N & 3) == 0) *(float4*)ws = make_float4(o[0], o[1], o[2], o[3]);
        else for (int i = 0; i < 4 && n0 + i < a.N; i++) ws[i] = o[i];
      } else {
        if (a.bias) {
#pragma unroll
          for (int i = 0; i < 4; i++) o[i] += (n0 + i < a.N) ? to_f32<T>(a.bias[n0 + i]) : 0.f;
        }
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n0;
        if (n0 + 3 < a.N && ((a.ldo | n0) & 3) == 0) *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
        else for (int i = 0; i < 4 && n0 + i < a.N; i++) y[i] = from_f32<T>(o[i]);
      }
    }
  }
}

// launch helper: 150 KiB dynamic LDS allowed once per instantiation
template <typename K>
inline void launch4(K kern, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(kern, grid, dim3(64 * (a.waves ? a.waves : 4)), shmem, st, a);
}

template <int DK, typename T, bool MOE, bool QS>
inline void launch4_epi(int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  if (epi == EPI_STORE) launch4(lowbit_gemv4_kernel<DK, T, EPI_STORE, 1, MOE, QS>, grid, shmem, a, st);
  else if (epi == EPI_PARTIAL) launch4(lowbit_gemv4_kernel<DK, T, EPI_PARTIAL, 1, MOE, QS>, grid, shmem, a, st);
  else launch4(lowbit_gemv4_kernel<DK, T, EPI_GLU, 2, MOE, QS>, grid, shmem, a, st);
}

template <int DK>
void launch_gemv4_dk(bool bf16, int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  // quad scale loads need chunk ranges starting at multiples of 4
  const int cpk = a.cpk > 0 ? a.cpk : (a.KC + (int)grid.y - 1) / (int)grid.y;
  const bool qs = (a.KC % 4 == 0) && (cpk % 4 == 0);
  const bool moe = a.moe_off != nullptr;
  if (moe && epi == EPI_STORE) epi = EPI_PARTIAL;   // grouped launches write slabs or GLU rows
  if (bf16) {
    if (moe) { if (qs) launch4_epi<DK, BF16, true, true>(epi, grid, shmem, a, st); else launch4_epi<DK, BF16, true, false>(epi, grid, shmem, a, st); }
    else if (qs) launch4_epi<DK, BF16, false, true>(epi, grid, shmem, a, st);
    else launch4_epi<DK, BF16, false, false>(epi, grid, shmem, a, st);
  } else {
    if (moe) { if (qs) launch4_epi<DK, F16, true, true>(epi, grid, shmem, a, st); else launch4_epi<DK, F16, true, false>(epi, grid, shmem, a, st); }
    else if (qs) launch4_epi<DK, F16, false, true>(epi, grid, shmem, a, st);
    else launch4_epi<DK, F16, false, false>(epi, grid, shmem, a, st);
  }
}

template <int DK, typename T, int MT>
inline void launch_gemv_t(int epi, dim3 grid, const GemvArgs& a, hipStream_t st) {
  if (epi == EPI_STORE) hipLaunchKernelGGL((lowbit_gemv_kernel<DK, T, MT, EPI_STORE>), grid, dim3(256), 0, st, a);
  else if (epi == EPI_PARTIAL) hipLaunchKernelGGL((lowbit_gemv_kernel<DK, T, MT, EPI_PARTIAL>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((lowbit_gemv_kernel<DK, T, MT, EPI_GLU>), grid, dim3(256), 0, st, a);
}

template <int DK>
void launch_gemv_dk(bool bf16, int mt, int epi, dim3 grid, const GemvArgs& a, hipStream_t st) {
  if (bf16) {
    if (mt == 1) launch_gemv_t<DK, BF16, 1>(epi, grid, a, st);
    else if (mt == 2) launch_gemv_t<DK, BF16, 2>(epi, grid, a, st);
    else launch_gemv_t<DK, BF16, 4>(epi, grid, a, st);
  } else {
    if (mt == 1) launch_gemv_t<DK, F16, 1>(epi, grid, a, st);
    else if (mt == 2) launch_gemv_t<DK, F16, 2>(epi, grid, a, st);
    else launch_gemv_t<DK, F16, 4>(epi, grid, a, st);
  }
}

}  // namespace illm
