// Fused rotary embedding + KV-cache append for the decode/prefill step.
//
// Reference ops: xe_addons.rotary_half_inplaced / rotary_two_inplaced /
// rotary_*_with_cache_inplaced (models/common.py:354-367, llama.py:158-162,
// chatglm2.py:251) and the KV write of kv.py / models/utils.py:65-74
// (append_kv_cache) + quantize_key_value (utils.py:133-191).
//
// One wave64 per (head, token): q/k/v rows come straight from the fused QKV
// projection output; q is rotated (optionally per-head RMS-normalised first,
// qwen3) and written contiguous; k is rotated and v copied into the paged KV
// cache at slots[t] (block * bs + offset), in the activation dtype or fp8.
// Positions and slots are device tensors, so the kernel is graph-capturable.
#include "../common/quant_block.h"
#include "illm_device.h"
#include "kernels.h"

namespace illm {

__device__ __forceinline__ void store_kv(uint8_t* base, size_t idx, float v, int kv_fp8, float scale,
                                         bool bf16) {
  if (kv_fp8 == 1) {
    base[idx] = hd_f32_to_e5m2(v / scale);
  } else if (kv_fp8 == 2) {
    base[idx] = hd_f32_to_e4m3(v / scale);
  } else {
    ((uint16_t*)base)[idx] = bf16 ? f32_to_bf16(v) : f32_to_f16(v);
  }
}

template <typename T>
__global__ void __launch_bounds__(64) rope_kv_kernel(const RopeKVArgs a) {
  const int h = blockIdx.x, t = blockIdx.y, lane = threadIdx.x;
  const int D = a.D, half = a.rot_dim / 2;
  const bool is_q = h < a.Hq, is_k = !is_q && h < a.Hq + a.Hkv;
  const size_t col0 = (size_t)h * D;
  const uint16_t* src = a.part ? nullptr : a.qkv + (size_t)t * a.ld_qkv + col0;
  constexpr bool BF = std::is_same<T, BF16>::value;
  // projection output element d of this head (split-K partials summed here,
  // rounded to T like the standalone GEMV output)
  const float rs = a.pss ? rsqrtf(a.pss[t] / (float)a.pss_n + a.pss_eps) : 1.f;   // deferred input norm
  auto raw = [&](int d) -> float {
    if (!a.part) return to_f32<T>(src[d]);
    float s = 0.f;
#pragma unroll 4
    for (int k = 0; k < a.nsplit; k++) s += a.part[((size_t)k * a.T + t) * a.ld_qkv + col0 + d];
    s *= rs;
    if (a.bias) s += to_f32<T>(a.bias[col0 + d]);
    return to_f32<T>(from_f32<T>(s));
  };
  // two elements at once: both columns' split-K loads are in flight together
  // (the per-split loads are independent; only the adds are ordered)
  auto raw2 = [&](int d0, int d1, float& r0, float& r1) {
    if (!a.part) {
      r0 = to_f32<T>(src[d0]);
      r1 = to_f32<T>(src[d1]);
      return;
    }
    float s0 = 0.f, s1 = 0.f;
    const float* pk = a.part + (size_t)t * a.ld_qkv + col0;
    const size_t kstride = (size_t)a.T * a.ld_qkv;
#pragma unroll 4
    for (int k = 0; k < a.nsplit; k++) {
      s0 += pk[d0];
      s1 += pk[d1];
      pk += kstride;
    }
    s0 *= rs;
    s1 *= rs;
    if (a.bias) {
      s0 += to_f32<T>(a.bias[col0 + d0]);
      s1 += to_f32<T>(a.bias[col0 + d1]);
    }
    r0 = to_f32<T>(from_f32<T>(s0));
    r1 = to_f32<T>(from_f32<T>(s1));
  };

  // per-head RMSNorm (qwen3 q_norm / k_norm): sum of squares over D
  const uint16_t* nw = is_q ? a.q_norm : (is_k ? a.k_norm : nullptr);
  float inv = 1.f;
  if (nw) {
    float ss = 0.f;
    for (int d = lane; d < D; d += 64) {
      float v = raw(d);
      ss += v * v;
    }
    ss = wave_sum(ss);
    inv = rsqrtf(ss / (float)D + a.norm_eps);
  }
  auto val = [&](int d) -> float {
    float v = raw(d);
    if (nw) v = to_f32<T>(from_f32<T>(to_f32<T>(nw[d]) * to_f32<T>(from_f32<T>(v * inv))));
    return v;
  };

  const float p = (float)a.pos[t];
  int64_t slot = 0;
  uint8_t* cache = nullptr;
  float cscale = 1.f;
  if (!is_q) {
    if (a.slots) {
      slot = a.slots[t];
    } else {
      // cache index = rotary position - per-sequence offset (compressed KV keeps fewer entries)
      const int64_t pp = a.pos[t] - (a.pos_offset ? a.pos_offset[t / a.tq] : 0);
      slot = (int64_t)a.block_tables[(size_t)(t / a.tq) * a.max_blocks + pp / a.bs] * a.bs + pp % a.bs;
    }
    const bool oob = a.num_blocks > 0 && slot >= (int64_t)a.num_blocks * a.bs;
    if (oob && lane == 0) kerr(a.err, ERR_SLOT);
    if (slot < 0 || oob) {   // padding token (or a bad slot): nothing to write, keep the accumulator zeroed
      if (a.part && a.zero_part)
        for (int d = lane; d < D; d += 64) ((float*)a.part)[(size_t)t * a.ld_qkv + col0 + d] = 0.f;
      return;
    }
    cache = is_k ? a.k_cache : a.v_cache;
    cscale = is_k ? a.k_scale : a.v_scale;
  }
  const int hk = is_q ? h : (is_k ? h - a.Hq : h - a.Hq - a.Hkv);
  const size_t crow = is_q ? 0 : (((size_t)(slot / a.bs) * a.Hkv + hk) * a.bs + (size_t)(slot % a.bs)) * D;
  uint16_t* qdst = is_q ? a.q_out + ((size_t)t * a.Hq + h) * D : nullptr;

  auto put = [&](int d, float v) {
    if (is_q) qdst[d] = from_f32<T>(v * a.attn_scale_q);
    else store_kv(cache, crow + d, v, a.kv_fp8, cscale, BF);
  };

  if (is_q || is_k) {
    for (int i = lane; i < half; i += 64) {
      int d0, d1;
      if (a.interleaved) { d0 = 2 * i; d1 = 2 * i + 1; }
      else { d0 = i; d1 = i + half; }
      float s, c;
      if (a.cos_sin) {
        const float2 cs = ((const float2*)a.cos_sin)[(size_t)a.pos[t] * half + i];
        c = cs.x;
        s = cs.y;
      } else {
        sincosf(p * a.inv_freq[i], &s, &c);
      }
      // HF casts cos/sin to the activation dtype before the rotation
      c = to_f32<T>(from_f32<T>(c));
      s = to_f32<T>(from_f32<T>(s));
      float x0, x1;
      if (nw) {
        x0 = val(d0);
        x1 = val(d1);
      } else {
        raw2(d0, d1, x0, x1);
      }
      put(d0, to_f32<T>(from_f32<T>(x0 * c)) - to_f32<T>(from_f32<T>(x1 * s)));
      put(d1, to_f32<T>(from_f32<T>(x1 * c)) + to_f32<T>(from_f32<T>(x0 * s)));
    }
    for (int d = a.rot_dim + lane; d < D; d += 64) put(d, val(d));
  } else {
    int d = lane;
    for (; d + 64 < D; d += 128) {
      float v0, v1;
      raw2(d, d + 64, v0, v1);
      put(d, v0);
      put(d + 64, v1);
    }
    if (d < D) put(d, raw(d));
  }
  if (a.part && a.zero_part) {
    // every read of this head's columns above was made by this wave
    for (int d = lane; d < D; d += 64) ((float*)a.part)[(size_t)t * a.ld_qkv + col0 + d] = 0.f;
  }
}

// Fast path (full-width NeoX rotary from the cos/sin table, no per-head norm,
// 16-bit cache; input = the projection output in T, or one f32 atomic
// accumulator slab + bias, re-zeroed here): D / 16 lanes per (token, head)
// row, each rotating 8 consecutive dims of both halves with 16-B accesses;
// 256-thread workgroups.  Same rounding sequence as the general kernel.  The one-wave-per-row kernel with 2-byte accesses took 27.8 us per
// Llama-3-8B layer at 1024 prompt tokens.
template <typename T>
__global__ void __launch_bounds__(256) rope_kv_vec_kernel(const RopeKVArgs a) {
  const int D = a.D, half = D / 2, LPR = D / 16;
  const int HT = a.Hq + 2 * a.Hkv;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / LPR;
  if (row >= (int64_t)a.T * HT) return;
  const int i0 = (int)(gid % LPR) * 8;
  const int t = (int)(row / HT), h = (int)(row % HT);
  const bool is_q = h < a.Hq, is_k = !is_q && h < a.Hq + a.Hkv;
  const uint16_t* src = a.part ? nullptr : a.qkv + (size_t)t * a.ld_qkv + (size_t)h * D;
  uint16_t* d0p;
  uint16_t* d1p;
  if (is_q) {
    d0p = a.q_out + ((size_t)t * a.Hq + h) * D + i0;
  } else {
    int64_t slot;
    if (a.slots) {
      slot = a.slots[t];
    } else {
      const int64_t pp = a.pos[t] - (a.pos_offset ? a.pos_offset[t / a.tq] : 0);
      slot = (int64_t)a.block_tables[(size_t)(t / a.tq) * a.max_blocks + pp / a.bs] * a.bs + pp % a.bs;
    }
    const bool oob = a.num_blocks > 0 && slot >= (int64_t)a.num_blocks * a.bs;
    if (oob) kerr(a.err, ERR_SLOT);
    if (slot < 0 || oob) {                             // padding token (or a bad slot): nothing to write
      if (a.part && a.zero_part) {
        float* pp = (float*)a.part + (size_t)t * a.ld_qkv + (size_t)h * D;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        *(float4*)(pp + i0) = z; *(float4*)(pp + i0 + 4) = z;
        *(float4*)(pp + i0 + half) = z; *(float4*)(pp + i0 + half + 4) = z;
      }
      return;
    }
    const int hk = is_k ? h - a.Hq : h - a.Hq - a.Hkv;
    d0p = (uint16_t*)(is_k ? a.k_cache : a.v_cache) +
          (((size_t)(slot / a.bs) * a.Hkv + hk) * a.bs + (size_t)(slot % a.bs)) * D + i0;
  }
  d1p = d0p + half;
  uint4 x0, x1;
  if (a.part) {
    // rnd(bias + acc) like the GEMV output, then the accumulator is re-zeroed
    float* pp = (float*)a.part + (size_t)t * a.ld_qkv + (size_t)h * D;
    float4* p0 = (float4*)(pp + i0);
    float4* p1 = (float4*)(pp + i0 + half);
    float4 f[4] = {p0[0], p0[1], p1[0], p1[1]};
    if (a.pss) {                                       // deferred input norm: one scale per token row
      const float rs = rsqrtf(a.pss[t] / (float)a.pss_n + a.pss_eps);
#pragma unroll
      for (int e = 0; e < 4; e++) { f[e].x *= rs; f[e].y *= rs; f[e].z *= rs; f[e].w *= rs; }
    }
    uint32_t wv[8];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int dd = (e < 2 ? i0 : i0 + half) + 4 * (e & 1);
      float bb[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.bias) {
        const uint2 bu = *(const uint2*)(a.bias + (size_t)h * D + dd);
        bb[0] = to_f32<T>((uint16_t)(bu.x & 0xffff)); bb[1] = to_f32<T>((uint16_t)(bu.x >> 16));
        bb[2] = to_f32<T>((uint16_t)(bu.y & 0xffff)); bb[3] = to_f32<T>((uint16_t)(bu.y >> 16));
      }
      wv[2 * e] = pack2<T>(bb[0] + f[e].x, bb[1] + f[e].y);
      wv[2 * e + 1] = pack2<T>(bb[2] + f[e].z, bb[3] + f[e].w);
    }
    x0 = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    x1 = make_uint4(wv[4], wv[5], wv[6], wv[7]);
    if (a.zero_part) {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      p0[0] = z; p0[1] = z; p1[0] = z; p1[1] = z;
    }
  } else {
    x0 = *(const uint4*)(src + i0);
    x1 = *(const uint4*)(src + i0 + half);
  }
  if (!is_q && !is_k) {                                // v: copy
    *(uint4*)d0p = x0;
    *(uint4*)d1p = x1;
    return;
  }
  const float4* cs = (const float4*)((const float2*)a.cos_sin + (size_t)a.pos[t] * half + i0);
  const uint32_t w0[4] = {x0.x, x0.y, x0.z, x0.w}, w1[4] = {x1.x, x1.y, x1.z, x1.w};
  const float osc = is_q ? a.attn_scale_q : 1.f;
  auto rnd = [](float v) { return to_f32<T>(from_f32<T>(v)); };
  uint32_t o0[4], o1[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const float4 q = cs[e];                            // (cos, sin) of dims i0 + 2e, i0 + 2e + 1
    float r0[2], r1[2];
#pragma unroll
    for (int u = 0; u < 2; u++) {
      // HF casts cos/sin to the activation dtype before the rotation
      const float c = rnd(u ? q.z : q.x), sn = rnd(u ? q.w : q.y);
      const float a0 = to_f32<T>((uint16_t)(w0[e] >> (16 * u))), a1 = to_f32<T>((uint16_t)(w1[e] >> (16 * u)));
      r0[u] = (rnd(a0 * c) - rnd(a1 * sn)) * osc;
      r1[u] = (rnd(a1 * c) + rnd(a0 * sn)) * osc;
    }
    o0[e] = pack2<T>(r0[0], r0[1]);
    o1[e] = pack2<T>(r1[0], r1[1]);
  }
  *(uint4*)d0p = make_uint4(o0[0], o0[1], o0[2], o0[3]);
  *(uint4*)d1p = make_uint4(o1[0], o1[1], o1[2], o1[3]);
}

void launch_rope_kv(bool bf16, const RopeKVArgs& a, hipStream_t st) {
  if ((!a.part || a.nsplit == 1) && !a.q_norm && !a.k_norm && !a.interleaved && a.rot_dim == a.D &&
      a.kv_fp8 == 0 && a.cos_sin && a.D % 16 == 0 && a.ld_qkv % 8 == 0) {
    const int64_t n = (int64_t)a.T * (a.Hq + 2 * a.Hkv) * (a.D / 16);
    dim3 g((unsigned)((n + 255) / 256));
    if (bf16) hipLaunchKernelGGL(rope_kv_vec_kernel<BF16>, g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(rope_kv_vec_kernel<F16>, g, dim3(256), 0, st, a);
    return;
  }
  dim3 grid(a.Hq + 2 * a.Hkv, a.T);
  if (bf16) hipLaunchKernelGGL(rope_kv_kernel<BF16>, grid, dim3(64), 0, st, a);
  else hipLaunchKernelGGL(rope_kv_kernel<F16>, grid, dim3(64), 0, st, a);
}

}  // namespace illm
