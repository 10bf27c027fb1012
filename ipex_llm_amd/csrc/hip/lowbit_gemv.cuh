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
//   * two kernels: lowbit_gemv5_kernel (M <= 16, the decode hot path,
//     lowbit_gemv5.cuh) and lowbit_gemv_kernel (17..64 rows: MT 16-row M
//     tiles per wave, 4 waves split K and reduce through LDS);
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
    // chunk-major scale plane: rows 4g..4g+3 of chunk c are one 16-B record
    const uint32_t* sp = (const uint32_t*)(tptr + (size_t)a.KC * dk_code_chunk(DK)) + (size_t)c * 16 + 4 * g;
    ch.sc = *(const uint4*)sp;
    if constexpr (dk_has_min(DK)) ch.mn = *(const uint4*)(sp + 16 * a.KC);
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

}  // namespace illm

#include "lowbit_gemv5.cuh"

namespace illm {

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
