// In-register decoders of the tiled low-bit weight blob (formats.h) into
// f16 MFMA operand fragments, shared by the prefill GEMMs (gemm.hip: A
// fragments straight to the MFMA; gemm_mfma.hip: fragments decoded once per
// workgroup into LDS).  One code dword of a 4-bit chunk record = the 8
// codes of one lane's k-step, nibble order = the magic-number pair order, so
// (u >> 4q) & 0x000F000F is the packed f16 pair (2q, 2q+1).
//
// Numerics: (q - 8) * d is formed in f16 from the exact code (1024 + q via
// the 0x6400 exponent trick, minus 1032 exactly) and rounded once by the
// multiply -- the same single rounding as the reference's fp16 dequant.
#pragma once
#include <stdint.h>

#include "gemv_args.h"
#include "illm_device.h"

namespace illm {

typedef _Float16 gh2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gh2 g_as_h2(uint32_t u) { return __builtin_bit_cast(gh2, u); }
__device__ __forceinline__ uint32_t g_as_u(gh2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t g_bytes01(uint32_t u) { return __builtin_amdgcn_perm(0u, u, 0x0c010c00u); }
__device__ __forceinline__ uint32_t g_bytes23(uint32_t u) { return __builtin_amdgcn_perm(0u, u, 0x0c030c02u); }

// pre-scaled f16 A fragment (8 weights of one k-step); d2 / m2 = (d, d) / (min, min)
template <int DK>
__device__ __forceinline__ uint4 gemm_a4(uint32_t u, gh2 d2, gh2 m2, const uint32_t* lut2) {
  uint32_t w[4];
  if constexpr (DK == DK_INT4S || DK == DK_INT4A) {
    w[0] = (u & 0x000F000Fu) | 0x64006400u;
    w[1] = ((u >> 4) & 0x000F000Fu) | 0x64006400u;
    w[2] = ((u >> 8) & 0x000F000Fu) | 0x64006400u;
    w[3] = ((u >> 12) & 0x000F000Fu) | 0x64006400u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if constexpr (DK == DK_INT4S) w[i] = g_as_u((g_as_h2(w[i]) - gh2{(_Float16)1032.f, (_Float16)1032.f}) * d2);
      else w[i] = g_as_u(__builtin_elementwise_fma(g_as_h2(w[i]) - gh2{(_Float16)1024.f, (_Float16)1024.f}, d2, m2));
    }
  } else {
    if constexpr (DK == DK_FP4) {
      w[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 0));
      w[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 1));
      w[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 2));
      w[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(u, 1.0f, 3));
    } else {  // DK_LUT4
      w[0] = lut2[u & 0xff];
      w[1] = lut2[(u >> 8) & 0xff];
      w[2] = lut2[(u >> 16) & 0xff];
      w[3] = lut2[u >> 24];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = g_as_u(g_as_h2(w[i]) * d2);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int DK>
__device__ __forceinline__ uint4 gemm_a8(uint32_t lo, uint32_t hi, gh2 d2, gh2 m2) {
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
    for (int i = 0; i < 4; i++) w[i] = g_as_u(g_as_h2(w[i]) * d2);
  } else {
    // bytes -> f16(1024 + byte) via v_perm + magic; signed codes biased by 128
    if constexpr (DK == DK_INT8S) { lo ^= 0x80808080u; hi ^= 0x80808080u; }
    w[0] = g_bytes01(lo) | 0x64006400u;
    w[1] = g_bytes23(lo) | 0x64006400u;
    w[2] = g_bytes01(hi) | 0x64006400u;
    w[3] = g_bytes23(hi) | 0x64006400u;
    const _Float16 off = DK == DK_INT8S ? (_Float16)1152.f : (_Float16)1024.f;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if constexpr (DK == DK_INT8S) w[i] = g_as_u((g_as_h2(w[i]) - gh2{off, off}) * d2);
      else w[i] = g_as_u(__builtin_elementwise_fma(g_as_h2(w[i]) - gh2{off, off}, d2, m2));
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// (d, d) f16 pair of scale block `blk` from a (blk0 | blk1 << 16) scale dword
__device__ __forceinline__ gh2 g_pick(uint32_t v, int blk) {
  return g_as_h2(__builtin_amdgcn_perm(0u, v, blk == 0 ? 0x01000100u : 0x03020302u));
}

}  // namespace illm
