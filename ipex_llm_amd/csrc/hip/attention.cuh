// Decode / short-query attention over a paged KV cache (flash-decoding).
//
// Reference ops: xe_addons.sdp / sdp_fp8 (decode, q_len <= 32, native GQA;
// models/common.py:250-286), gemma2_sdp (softcap, sliding window;
// models/gemma2.py:133-155) and the vLLM-XPU paged_attention_v1/v2 GQA
// kernels (VLLM_PATCH:3380-3460).
//
// MI355X design: one wave64 per (batch, kv-head, 64-key split).  All query
// rows that share the kv head (GQA group x new tokens, R <= 16) are handled
// by the same wave, so every K/V byte is read from HBM once.  QK^T: lane =
// key, the K row is streamed in 16-B pieces and dotted against the q rows
// held in LDS (broadcast reads).  Softmax per row with wave64 shuffles.  PV:
// lane = head dim, V rows are read coalesced (one row per wave instruction).
// Per-split (m, l, o) partials are merged by a second small kernel.  Sequence
// lengths and block tables are device tensors: the launch geometry depends
// only on the max length bucket, so the whole thing is hipGraph-capturable.
#pragma once
#include <cstdlib>
#include "../common/quant_block.h"
#include "illm_device.h"
#include "kernels.h"

namespace illm {

constexpr int SPLIT = 64;
constexpr int RMAX = 16;

template <typename T, int KVF>
__device__ __forceinline__ void kv_load8(const uint8_t* p, float scale, float* v) {
  if constexpr (KVF == 0) {
    uint4 u = *(const uint4*)p;
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      v[2 * i] = to_f32<T>(w[i] & 0xffff);
      v[2 * i + 1] = to_f32<T>(w[i] >> 16);
    }
  } else {
    uint2 u = *(const uint2*)p;
    uint32_t w[2] = {u.x, u.y};
#pragma unroll
    for (int i = 0; i < 2; i++) {
      auto f0 = KVF == 1 ? __builtin_amdgcn_cvt_pk_f32_bf8(w[i], false) : __builtin_amdgcn_cvt_pk_f32_fp8(w[i], false);
      auto f1 = KVF == 1 ? __builtin_amdgcn_cvt_pk_f32_bf8(w[i], true) : __builtin_amdgcn_cvt_pk_f32_fp8(w[i], true);
      v[4 * i + 0] = f0[0] * scale;
      v[4 * i + 1] = f0[1] * scale;
      v[4 * i + 2] = f1[0] * scale;
      v[4 * i + 3] = f1[1] * scale;
    }
  }
}

template <typename T, int KVF>
__device__ __forceinline__ float kv_load1(const uint8_t* base, size_t idx, float scale) {
  if constexpr (KVF == 0) return to_f32<T>(((const uint16_t*)base)[idx]);
  else if constexpr (KVF == 1) return hd_e5m2_to_f32(base[idx]) * scale;
  else return hd_e4m3_to_f32(base[idx]) * scale;
}

// key count beyond the sequence's block-table row, or more keys than the
// split grid covers: the sequence's splits leave (reported once, by split 0)
__device__ __forceinline__ bool bad_len(const AttnDecodeArgs& a, int len, int split) {
  const bool bad = (int64_t)len > (int64_t)a.max_blocks * a.bs || (int64_t)a.nsplit * SPLIT < len;
  if (bad && split == 0 && threadIdx.x == 0) kerr(a.err, ERR_SEQ_LEN);
  return bad;
}

template <typename T, int D, int KVF>
__global__ void __launch_bounds__(64) attn_decode_kernel(const AttnDecodeArgs a) {
  constexpr int EB = KVF == 0 ? 2 : 1;  // bytes per cached element
  constexpr int DV = (D + 63) / 64;     // head dims per lane in PV
  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x;
  const int len = a.seq_lens[b];
  const int k0 = split * SPLIT;
  if (k0 >= len || bad_len(a, len, split)) return;
  const int group = a.Hq / a.Hkv;
  const int R = group * a.Tq;  // rows: r = t * group + gi

  __shared__ float qs[RMAX][D];
  __shared__ float ps[RMAX][SPLIT];

  // q rows of this kv head -> LDS (f32)
  for (int i = lane; i < R * D; i += 64) {
    const int r = i / D, d = i % D;
    const int t = r / group, h = kvh * group + r % group;
    qs[r][d] = to_f32<T>(a.q[(((size_t)b * a.Tq + t) * a.Hq + h) * D + d]);
  }
  __syncthreads();

  const int blk = a.block_tables[(size_t)b * a.max_blocks + k0 / a.bs];
  if (bad_block(blk, a.num_blocks)) {
    if (lane == 0) kerr(a.err, ERR_BLOCK_ID);
    return;
  }
  const size_t base = (((size_t)blk * a.Hkv + kvh) * a.bs + (k0 % a.bs)) * D;
  const uint8_t* kb = a.k_cache + base * EB;
  const uint8_t* vb = a.v_cache + base * EB;

  // ---- S = q k^T : lane = key
  const int key = k0 + lane;
  const bool kin = key < len;
  float s[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; r++) s[r] = 0.f;
  if (kin) {
    const uint8_t* krow = kb + (size_t)lane * D * EB;
#pragma unroll 4
    for (int c = 0; c < D; c += 8) {
      float kv[8];
      kv_load8<T, KVF>(krow + c * EB, a.k_scale, kv);
#pragma unroll
      for (int r = 0; r < RMAX; r++) {
        if (r < R) {
          float acc = s[r];
#pragma unroll
          for (int i = 0; i < 8; i++) acc += qs[r][c + i] * kv[i];
          s[r] = acc;
        }
      }
    }
  }
  const int qpos0 = len - a.Tq;  // absolute position of query token 0
#pragma unroll
  for (int r = 0; r < RMAX; r++) {
    if (r >= R) break;
    const int t = r / group, h = kvh * group + r % group;
    const int qpos = qpos0 + t;
    float v = s[r] * a.scale;
    if (a.softcap > 0.f) v = a.softcap * tanhf(v / a.softcap);
    if (a.alibi) v += a.alibi[h] * (float)key;
    bool ok = kin && key <= qpos;
    if (a.sliding_window > 0 && key <= qpos - a.sliding_window) ok = false;
    s[r] = ok ? v : -INFINITY;
  }

  // ---- softmax pieces per row
  float m[RMAX], l[RMAX];
#pragma unroll
  for (int r = 0; r < RMAX; r++) {
    if (r >= R) break;
    m[r] = wave_max(s[r]);
    const float p = m[r] == -INFINITY ? 0.f : __expf(s[r] - m[r]);
    l[r] = wave_sum(p);
    ps[r][lane] = p;
  }
  __syncthreads();

  // ---- O = P V : lane = head dim
  float o[RMAX][DV];
#pragma unroll
  for (int r = 0; r < RMAX; r++)
#pragma unroll
    for (int j = 0; j < DV; j++) o[r][j] = 0.f;
  const int nk = min(SPLIT, len - k0);
  for (int kk = 0; kk < nk; kk++) {
    float vv[DV];
#pragma unroll
    for (int j = 0; j < DV; j++) {
      const int d = lane + 64 * j;
      vv[j] = (d < D) ? kv_load1<T, KVF>(vb, (size_t)kk * D + d, a.v_scale) : 0.f;
    }
#pragma unroll
    for (int r = 0; r < RMAX; r++) {
      if (r < R) {
        const float p = ps[r][kk];
#pragma unroll
        for (int j = 0; j < DV; j++) o[r][j] += p * vv[j];
      }
    }
  }

  // ---- partials
#pragma unroll
  for (int r = 0; r < RMAX; r++) {
    if (r >= R) break;
    const int t = r / group, h = kvh * group + r % group;
    const size_t row = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit + split;
#pragma unroll
    for (int j = 0; j < DV; j++) {
      const int d = lane + 64 * j;
      if (d < D) a.part_o[row * D + d] = o[r][j];
    }
    if (lane == 0) {
      a.part_ml[row * 2] = m[r];
      a.part_ml[row * 2 + 1] = l[r];
    }
  }
}

// ---------------------------------------------------------------------------
// v2: MFMA flash-decoding for D in {64, 128, 256}.  One wave per 64-key split.
// Every K and V byte of the split is requested up front (16 + 16 x 16-B
// loads per lane, 1 KiB per wave instruction), so the wave pays one memory
// latency instead of one per key.
//   S^T = K Q^T on 16x16x32 MFMA: A = K rows (key on the lane, 16 B of one
//   key row per lane straight from HBM), B = Q^T (query row on the lane).
//   The result puts (key = 16 kt + 4 g + i, row = lane & 15) in registers,
//   so the softmax row max/sum is a 16-value register reduction + 2 shuffles.
//   O = P V on the VALU: lane (dg = lane & 15, kg = lane >> 4) owns D/16
//   head dims of 16 keys; P comes back through 4 KiB of LDS; the 4 key
//   groups are summed with 2 shuffles.
// ---------------------------------------------------------------------------
template <typename T, int KVF>
__device__ __forceinline__ uint4 kv_frag8(const uint8_t* p) {
  // 8 cached elements -> 8 x 16-bit A/B fragment (f32 scale applied later)
  if constexpr (KVF == 0) {
    return *(const uint4*)p;
  } else {
    const uint2 u = *(const uint2*)p;
    uint4 r;
    constexpr bool BF = std::is_same<T, BF16>::value;
    if constexpr (KVF == 1) {
      if constexpr (BF) {
        r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u.x, 1.0f, false));
        r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u.x, 1.0f, true));
        r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u.y, 1.0f, false));
        r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u.y, 1.0f, true));
      } else {
        r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u.x, 1.0f, false));
        r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u.x, 1.0f, true));
        r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u.y, 1.0f, false));
        r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u.y, 1.0f, true));
      }
    } else {
      if constexpr (BF) {
        r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u.x, 1.0f, false));
        r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u.x, 1.0f, true));
        r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u.y, 1.0f, false));
        r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u.y, 1.0f, true));
      } else {
        r.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u.x, 1.0f, false));
        r.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u.x, 1.0f, true));
        r.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u.y, 1.0f, false));
        r.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u.y, 1.0f, true));
      }
    }
    return r;
  }
}

template <typename T, bool SC1 = false>
__device__ __forceinline__ void combine_row(const AttnDecodeArgs& a, int b, int h, int t, float* wsh);
template <typename T, bool SC1, int NR>
__device__ __forceinline__ bool combine_fast(const AttnDecodeArgs& a, int b, const int* hs, const int* ts, int nr);

// LATEV: issue the V loads after Q K^T (K registers are dead by then): fewer
// VGPRs and the V stream overlaps the QK/softmax of the co-resident wave.
// Chosen for grids larger than one wave per SIMD (measured on MI355X at
// batch 8, 1088 waves: 2.564 -> 2.524 ms/step; ILLM_ATTN_LATEV=0/1 forces it)
//
// PVM: P V on the matrix cores as O^T = V^T P^T (the prefill kernel's form):
// the split's V tile is staged in LDS ([key][D], 16-B XOR swizzle) and read
// back transposed by ds_read_b64_tr_b16 as the A operand; the B operand is the
// lane's own softmax numerators (key order of the S^T C layout), so P never
// leaves registers.  16 MFMAs per 64-key split (D = 128) instead of the
// per-lane FMA loop and its 2 x RT x DPL cross-lane reductions.
//
// NWV = 2 (PVM only): two waves per 64-key split, each owning 32 keys (half
// the K/V loads, QK^T and P V work of the one-wave form, so half its serial
// instruction chain); the split's softmax max / sum meet in LDS and wave 1's
// P V accumulator is added by wave 0, which writes the split partial.
template <typename T, int D, int KVF, int RT, bool RQ = false, bool LATEV = false, bool PVM = false, int NWV = 1>
__global__ void __launch_bounds__(64 * NWV) attn_decode_v2_kernel(const AttnDecodeArgs a) {
  static_assert(NWV == 1 || PVM, "two-wave splits need the MFMA P V form");
  constexpr int KTW = 4 / NWV;        // 16-key tiles per wave
  constexpr int EB = KVF == 0 ? 2 : 1;
  constexpr int KSTEP = D / 32;       // MFMA k-steps over the head dim
  constexpr int DPL = D / 16;         // head dims per lane in P.V
  constexpr int VCH = DPL / 8 > 0 ? DPL / 8 : 1;  // 8-element fragments per key per lane
  constexpr int VU = D / 8;           // PVM staging: 16-B chunks per key = chunks per lane
  constexpr int KPJ = 64 / VU;        // keys per staging step (lane -> key lane / VU, chunk lane % VU)
  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, r16 = lane & 15, g = lane >> 4;
  const int wv = NWV > 1 ? (int)(threadIdx.x >> 6) : 0;
  const int len = a.seq_lens[b];
  const int k0 = split * SPLIT;
  if (k0 >= len || bad_len(a, len, split)) return;
  const int nk = min(SPLIT, len - k0);
  const int group = a.Hq / a.Hkv;
  const int R = group * a.Tq;

  __shared__ float ps[PVM ? 1 : SPLIT][RT];
  __shared__ float mx[NWV > 1 ? 2 * NWV : 1][16];      // NWV > 1: per-wave row max / sum
  __shared__ __attribute__((aligned(16))) uint16_t vl[PVM ? SPLIT * D : 8];

  // ---- fused RoPE (rq_part): q/k/v of the new token from the qkv accumulator,
  // rounded exactly like rope_kv_fused (GEMV output in T, cos/sin in T, each
  // product in T, q scaled then stored in T)
  // separate instantiation: the plain kernel keeps its register allocation
  constexpr bool RQ_OK = RQ && KVF == 0 && D / 16 >= 8;
  constexpr bool rq = RQ_OK;
  auto rnd = [](float v) { return to_f32<T>(from_f32<T>(v)); };
  // deferred RMSNorm of the qkv GEMV input (lowbit_gemv5.cuh ndefer): one scale per sequence row
  const float rq_rs = (rq && a.rq_ss) ? rsqrtf(a.rq_ss[b] / (float)a.rq_ss_n + a.rq_ss_eps) : 1.f;
  auto rq_raw = [&](int col) -> float {
    float s = a.rq_bias ? to_f32<T>(a.rq_bias[col]) : 0.f;
    s += rq_rs * a.rq_part[(size_t)b * a.rq_ld + col];
    return rnd(s);
  };
  const int64_t rpos = rq ? a.rq_pos[b] : 0;
  auto rq_rot = [&](int col0, int d) -> float {
    const int half = a.rq_rot / 2;
    if (d >= a.rq_rot) return rq_raw(col0 + d);
    int i, d0, d1;
    bool first;
    if (a.rq_interleaved) { i = d >> 1; d0 = 2 * i; d1 = d0 + 1; first = (d & 1) == 0; }
    else { first = d < half; i = first ? d : d - half; d0 = i; d1 = i + half; }
    const float2 cs = ((const float2*)a.rq_cos_sin)[(size_t)rpos * half + i];
    const float c = rnd(cs.x), sn = rnd(cs.y);
    const float x0 = rq_raw(col0 + d0), x1 = rq_raw(col0 + d1);
    return first ? rnd(x0 * c) - rnd(x1 * sn) : rnd(x1 * c) + rnd(x0 * sn);
  };
  const bool has_new = rq && k0 + nk == len;        // this split holds the new key (position len - 1)
  uint4 vnew[VCH];                                  // the new value row (re-applied after a late V load)
  const int colk = (a.Hq + kvh) * D, colv = (a.Hq + a.Hkv + kvh) * D;

  const int blk = a.block_tables[(size_t)b * a.max_blocks + k0 / a.bs];
  if (bad_block(blk, a.num_blocks)) {                // wave-uniform: the whole split leaves
    if (threadIdx.x == 0) kerr(a.err, ERR_BLOCK_ID);
    return;
  }
  const size_t base = (((size_t)blk * a.Hkv + kvh) * a.bs + (k0 % a.bs)) * D;
  const uint8_t* kb = a.k_cache + base * EB;
  const uint8_t* vb = a.v_cache + base * EB;

  // ---- issue every load of the split
  uint4 kf[KTW][KSTEP];
#pragma unroll
  for (int kt = 0; kt < KTW; kt++) {
    const int kk = min((wv * KTW + kt) * 16 + r16, nk - 1);
#pragma unroll
    for (int s = 0; s < KSTEP; s++) kf[kt][s] = kv_frag8<T, KVF>(kb + ((size_t)kk * D + 32 * s + 8 * g) * EB);
  }
  const int dg = r16, kg = g;
  uint4 vf[PVM ? 1 : 16][VCH];
  constexpr int VUW = PVM ? VU / NWV : 1;           // staging steps of this wave's keys
  uint4 vm[VUW];
  auto load_v = [&]() {
    if constexpr (PVM) {
#pragma unroll
      for (int j = 0; j < VUW; j++) {
        const int kk = min((wv * VUW + j) * KPJ + lane / VU, nk - 1);
        vm[j] = kv_frag8<T, KVF>(vb + ((size_t)kk * D + 8 * (lane % VU)) * EB);
      }
    } else if constexpr (DPL >= 8) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const int kk = min(4 * i + kg, nk - 1);
#pragma unroll
        for (int c = 0; c < VCH; c++) vf[i][c] = kv_frag8<T, KVF>(vb + ((size_t)kk * D + DPL * dg + 8 * c) * EB);
      }
    }
  };
  if constexpr (!LATEV) load_v();
  uint4 qf[KSTEP];
  if constexpr (rq) {
    // a lane's q / k dims are 32 s + 8 g + j (s < KSTEP, j < 8): with full-width
    // rotary (rot == D) the rotation partner of chunk s is chunk s +- KSTEP/2 of
    // the same lane, so every operand arrives in 16-B vector loads
    auto lane_raw = [&](int col0, float (&v)[KSTEP][8]) {
#pragma unroll
      for (int s = 0; s < KSTEP; s++) {
        const float4* p = (const float4*)(a.rq_part + (size_t)b * a.rq_ld + col0 + 32 * s + 8 * g);
        const float4 f0 = p[0], f1 = p[1];
        float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (a.rq_bias) {
          const uint4 u = *(const uint4*)(a.rq_bias + col0 + 32 * s + 8 * g);
          const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int e = 0; e < 4; e++) {
            bb[2 * e] = to_f32<T>((uint16_t)(w[e] & 0xffff));
            bb[2 * e + 1] = to_f32<T>((uint16_t)(w[e] >> 16));
          }
        }
        const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
        for (int j = 0; j < 8; j++) v[s][j] = rnd(bb[j] + rq_rs * f[j]);
      }
    };
    auto lane_rot = [&](int col0, float scale_out, uint4* outf) {
      float v[KSTEP][8];
      lane_raw(col0, v);
      if (a.rq_prerot) {
        // the qkv GEMV rotated its partial sums: round, scale, pack
#pragma unroll
        for (int s = 0; s < KSTEP; s++) {
          uint32_t w[4];
#pragma unroll
          for (int j = 0; j < 4; j++) w[j] = pack2<T>(v[s][2 * j] * scale_out, v[s][2 * j + 1] * scale_out);
          outf[s] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      } else if (a.rq_rot == D && !a.rq_interleaved) {
        constexpr int HS = KSTEP / 2;
        const float4* csp = (const float4*)a.rq_cos_sin + (size_t)rpos * (D / 4);   // float2 pairs, 2 per float4
#pragma unroll
        for (int s = 0; s < HS; s++) {
          float cc[8], ss[8];
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const float4 q = csp[(32 * s + 8 * g) / 2 + e];
            cc[2 * e] = rnd(q.x); ss[2 * e] = rnd(q.y); cc[2 * e + 1] = rnd(q.z); ss[2 * e + 1] = rnd(q.w);
          }
          uint32_t lo[4], hi[4];
#pragma unroll
          for (int e = 0; e < 4; e++) {
            float r0[2], r1[2];
#pragma unroll
            for (int t = 0; t < 2; t++) {
              const int j = 2 * e + t;
              const float x0 = v[s][j], x1 = v[s + HS][j];
              r0[t] = (rnd(x0 * cc[j]) - rnd(x1 * ss[j])) * scale_out;
              r1[t] = (rnd(x1 * cc[j]) + rnd(x0 * ss[j])) * scale_out;
            }
            lo[e] = pack2<T>(r0[0], r0[1]);
            hi[e] = pack2<T>(r1[0], r1[1]);
          }
          outf[s] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
          outf[s + HS] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
        }
      } else {
#pragma unroll
        for (int s = 0; s < KSTEP; s++) {
          uint32_t w[4];
#pragma unroll
          for (int j = 0; j < 4; j++)
            w[j] = pack2<T>(rq_rot(col0, 32 * s + 8 * g + 2 * j) * scale_out,
                            rq_rot(col0, 32 * s + 8 * g + 2 * j + 1) * scale_out);
          outf[s] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    };
    {
      const int row = r16 < R ? r16 : 0;
      lane_rot((kvh * group + row % group) * D, a.rq_qscale, qf);
      if (r16 >= R)
#pragma unroll
        for (int s = 0; s < KSTEP; s++) qf[s] = make_uint4(0, 0, 0, 0);
    }
    if (has_new) {
      // the new key / value replace the (not yet written) cache entry in
      // registers and are appended to the paged cache for later steps
      const int kn = nk - 1, pos = len - 1;
      const int nb = a.block_tables[(size_t)b * a.max_blocks + pos / a.bs];
      const size_t crow = (((size_t)nb * a.Hkv + kvh) * a.bs + (size_t)(pos % a.bs)) * D;
      if (bad_block(nb, a.num_blocks)) {
        if (threadIdx.x == 0) kerr(a.err, ERR_BLOCK_ID);
      } else if (r16 == (kn & 15) && (kn >> 4) / KTW == wv) {
        uint4 kq[KSTEP];
        lane_rot(colk, 1.f, kq);
#pragma unroll
        for (int kt = 0; kt < KTW; kt++)
          if (wv * KTW + kt == (kn >> 4))
#pragma unroll
            for (int s = 0; s < KSTEP; s++) kf[kt][s] = kq[s];
#pragma unroll
        for (int s = 0; s < KSTEP; s++) *(uint4*)((uint16_t*)a.k_cache + crow + 32 * s + 8 * g) = kq[s];
      }
      if constexpr (PVM) {
        if (lane / VU == kn % KPJ && (kn / KPJ) / VUW == wv) {
          const int d0 = 8 * (lane % VU);
          const float4* p = (const float4*)(a.rq_part + (size_t)b * a.rq_ld + colv + d0);
          const float4 f0 = p[0], f1 = p[1];
          const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
          float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if (a.rq_bias) {
            const uint4 u = *(const uint4*)(a.rq_bias + colv + d0);
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
              bb[2 * e] = to_f32<T>((uint16_t)(w[e] & 0xffff));
              bb[2 * e + 1] = to_f32<T>((uint16_t)(w[e] >> 16));
            }
          }
          uint32_t w[4];
#pragma unroll
          for (int e = 0; e < 4; e++) w[e] = pack2<T>(rnd(bb[2 * e] + rq_rs * f[2 * e]), rnd(bb[2 * e + 1] + rq_rs * f[2 * e + 1]));
          const uint4 vq = make_uint4(w[0], w[1], w[2], w[3]);
          vnew[0] = vq;
#pragma unroll
          for (int j = 0; j < VUW; j++)
            if (wv * VUW + j == kn / KPJ) vm[j] = vq;
          if (!bad_block(nb, a.num_blocks)) *(uint4*)((uint16_t*)a.v_cache + crow + d0) = vq;
        }
      } else if constexpr (DPL >= 8) {
        if (kg == (kn & 3)) {
#pragma unroll
          for (int c = 0; c < VCH; c++) {
            const int d0 = DPL * dg + 8 * c;
            const float4* p = (const float4*)(a.rq_part + (size_t)b * a.rq_ld + colv + d0);
            const float4 f0 = p[0], f1 = p[1];
            const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
            float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (a.rq_bias) {
              const uint4 u = *(const uint4*)(a.rq_bias + colv + d0);
              const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
              for (int e = 0; e < 4; e++) {
                bb[2 * e] = to_f32<T>((uint16_t)(w[e] & 0xffff));
                bb[2 * e + 1] = to_f32<T>((uint16_t)(w[e] >> 16));
              }
            }
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 4; e++) w[e] = pack2<T>(rnd(bb[2 * e] + rq_rs * f[2 * e]), rnd(bb[2 * e + 1] + rq_rs * f[2 * e + 1]));
            const uint4 vq = make_uint4(w[0], w[1], w[2], w[3]);
            vnew[c] = vq;
#pragma unroll
            for (int i = 0; i < 16; i++)
              if (i == (kn >> 2)) vf[i][c] = vq;
            if (!bad_block(nb, a.num_blocks)) *(uint4*)((uint16_t*)a.v_cache + crow + d0) = vq;
          }
        }
      }
    }
  } else {
    const int row = r16 < R ? r16 : 0;
    const int t = row / group, h = kvh * group + row % group;
    const uint16_t* qr = a.q + (((size_t)b * a.Tq + t) * a.Hq + h) * D;
#pragma unroll
    for (int s = 0; s < KSTEP; s++) {
      uint4 v = *(const uint4*)(qr + 32 * s + 8 * g);
      qf[s] = r16 < R ? v : make_uint4(0, 0, 0, 0);
    }
  }

  // ---- S^T tiles: lane holds (key = 16 kt + 4 g + i, row = r16)
  f32x4 st[KTW];
#pragma unroll
  for (int kt = 0; kt < KTW; kt++) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSTEP; s++) acc = mfma16<T>(kf[kt][s], qf[s], acc);
    st[kt] = acc;
  }
  if constexpr (LATEV) {
    load_v();
    if constexpr (rq && DPL >= 8) {
      // the cache row of the new value was written by this wave above: take it
      // from registers, not from a load that may race the store
      const int kn = nk - 1;
      if constexpr (PVM) {
        if (has_new && lane / VU == kn % KPJ && (kn / KPJ) / VUW == wv) {
#pragma unroll
          for (int j = 0; j < VUW; j++)
            if (wv * VUW + j == kn / KPJ) vm[j] = vnew[0];
        }
      } else if (has_new && kg == (kn & 3)) {
#pragma unroll
        for (int c = 0; c < VCH; c++)
#pragma unroll
          for (int i = 0; i < 16; i++)
            if (i == (kn >> 2)) vf[i][c] = vnew[c];
      }
    }
  }
  const int row = r16;
  const int t = row / group;
  const int h = kvh * group + (row % group);
  const int qpos = len - a.Tq + t;
  const float sc = a.scale * (KVF ? a.k_scale : 1.f);
#ifndef ILLM_ATTN_SCORE_BF
#define ILLM_ATTN_SCORE_BF 1
#endif
#if ILLM_ATTN_SCORE_BF
  // the optional soft-cap / ALiBi terms are uniform branches around whole
  // loops and the mask is branch-free (per-score branches split the score
  // pass into dozens of basic blocks)
#pragma unroll
  for (int kt = 0; kt < KTW; kt++)
#pragma unroll
    for (int i = 0; i < 4; i++) st[kt][i] *= sc;
  if (a.softcap > 0.f) {
#pragma unroll
    for (int kt = 0; kt < KTW; kt++)
#pragma unroll
      for (int i = 0; i < 4; i++) st[kt][i] = a.softcap * tanhf(st[kt][i] / a.softcap);
  }
  if (a.alibi) {
    const float slope = row < R ? a.alibi[h] : 0.f;
#pragma unroll
    for (int kt = 0; kt < KTW; kt++)
#pragma unroll
      for (int i = 0; i < 4; i++) st[kt][i] += slope * (float)(k0 + (wv * KTW + kt) * 16 + 4 * g + i);
  }
  const int win = a.sliding_window > 0 ? qpos - a.sliding_window : -1;
  const int klim = min(nk, qpos - k0 + 1);          // keys kk < klim are visible
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < KTW; kt++) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int kk = (wv * KTW + kt) * 16 + 4 * g + i;
      const bool ok = row < R && kk < klim && k0 + kk > win;
      const float v = ok ? st[kt][i] : -INFINITY;
      st[kt][i] = v;
      m = fmaxf(m, v);
    }
  }
#else
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < KTW; kt++) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int kk = (wv * KTW + kt) * 16 + 4 * g + i;
      const int key = k0 + kk;
      float v = st[kt][i] * sc;
      if (a.softcap > 0.f) v = a.softcap * tanhf(v / a.softcap);
      if (a.alibi && row < R) v += a.alibi[h] * (float)key;
      bool ok = row < R && kk < nk && key <= qpos;
      if (a.sliding_window > 0 && key <= qpos - a.sliding_window) ok = false;
      v = ok ? v : -INFINITY;
      st[kt][i] = v;
      m = fmaxf(m, v);
    }
  }
#endif
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  if constexpr (NWV > 1) {                         // split-wide row max
    if (g == 0) mx[wv][r16] = m;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NWV; w++) m = fmaxf(m, mx[w][r16]);
  }
  float l = 0.f;
  const float vs = KVF ? a.v_scale : 1.f;
  const bool handoff = a.counters != nullptr;
  if constexpr (PVM) {
    // P^T fragments (16-bit pairs, key order 16 kt + 4 g + i) and the V tile in LDS
    uint32_t pk[KTW][2];
#pragma unroll
    for (int kt = 0; kt < KTW; kt++) {
      float p[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        p[i] = m == -INFINITY ? 0.f : __expf(st[kt][i] - m);
        l += p[i];
      }
      pk[kt][0] = pack2<T>(p[0], p[1]);
      pk[kt][1] = pack2<T>(p[2], p[3]);
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int j = 0; j < VUW; j++) *(uint4*)(vl + pf_off<D>((wv * VUW + j) * KPJ + lane / VU, lane % VU)) = vm[j];
    if constexpr (NWV > 1) {
      if (g == 0) mx[NWV + wv][r16] = l;
    }
    __syncthreads();
    if constexpr (NWV > 1) {
      l = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; w++) l += mx[NWV + w][r16];
    }
    constexpr int DT = D / 16;
    f32x4 o[DT];
#pragma unroll
    for (int d = 0; d < DT; d++) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int qq = r16 >> 2, pp = r16 & 3;
#pragma unroll
    for (int kk = 0; kk < 2 / NWV; kk++) {
      const int row0 = 32 * (wv * (2 / NWV) + kk) + 4 * g + qq, row1 = row0 + 16;
      const uint4 pb = make_uint4(pk[2 * kk][0], pk[2 * kk][1], pk[2 * kk + 1][0], pk[2 * kk + 1][1]);
#pragma unroll
      for (int d = 0; d < DT; d++) {
        const int col = 16 * d + 4 * pp;
        const uint2 v0 = ds_read_tr16(vl + pf_off<D>(row0, col >> 3) + (col & 7));
        const uint2 v1 = ds_read_tr16(vl + pf_off<D>(row1, col >> 3) + (col & 7));
        o[d] = mfma16<T>(make_uint4(v0.x, v0.y, v1.x, v1.y), pb, o[d]);
      }
    }
    if constexpr (NWV > 1) {
      // wave 1's P V sums join wave 0's through LDS (the V tile is dead now)
      float* ob = (float*)vl;
      __syncthreads();
      if (wv == 1) {
#pragma unroll
        for (int d = 0; d < DT; d++) *(float4*)(ob + (d * 64 + lane) * 4) = make_float4(o[d][0], o[d][1], o[d][2], o[d][3]);
      }
      __syncthreads();
      if (wv == 0) {
#pragma unroll
        for (int d = 0; d < DT; d++) {
          const float4 u = *(const float4*)(ob + (d * 64 + lane) * 4);
          o[d][0] += u.x; o[d][1] += u.y; o[d][2] += u.z; o[d][3] += u.w;
        }
      }
    }
    // lane holds O^T[16 d + 4 g + i][row r16]
    if (row < R && wv == 0) {
      const size_t prow = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit + split;
      float* po = a.part_o + prow * D + 4 * g;
#pragma unroll
      for (int d = 0; d < DT; d++) {
        if (handoff) {
          st16_sc1(a.part_o, (size_t)(po - a.part_o) + 16 * d,
                   make_float4(o[d][0] * vs, o[d][1] * vs, o[d][2] * vs, o[d][3] * vs));
        } else {
          *(float4*)(po + 16 * d) = make_float4(o[d][0] * vs, o[d][1] * vs, o[d][2] * vs, o[d][3] * vs);
        }
      }
    }
  } else {
#pragma unroll
  for (int kt = 0; kt < 4; kt++) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const float p = m == -INFINITY ? 0.f : __expf(st[kt][i] - m);
      l += p;
      if (row < RT) ps[kt * 16 + 4 * g + i][row] = p;
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  __syncthreads();

  // ---- O = P V: lane (dg, kg) owns dims [DPL*dg, DPL*dg + DPL) of keys 4i + kg
  float o[RT][DPL];
#pragma unroll
  for (int r = 0; r < RT; r++)
#pragma unroll
    for (int d = 0; d < DPL; d++) o[r][d] = 0.f;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int kk = 4 * i + kg;
    float v[DPL];
    if constexpr (DPL >= 8) {
#pragma unroll
      for (int c = 0; c < VCH; c++) {
        const uint32_t w[4] = {vf[i][c].x, vf[i][c].y, vf[i][c].z, vf[i][c].w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          v[8 * c + 2 * e] = to_f32<T>(w[e] & 0xffff);
          v[8 * c + 2 * e + 1] = to_f32<T>(w[e] >> 16);
        }
      }
    } else {
      const int kc = min(kk, nk - 1);
#pragma unroll
      for (int d = 0; d < DPL; d++) v[d] = kv_load1<T, KVF>(vb, (size_t)kc * D + DPL * dg + d, 1.f);
    }
#pragma unroll
    for (int r = 0; r < RT; r++) {
      const float p = ps[kk][r];
#pragma unroll
      for (int d = 0; d < DPL; d++) o[r][d] += p * v[d];
    }
  }
#pragma unroll
  for (int r = 0; r < RT; r++)
#pragma unroll
    for (int d = 0; d < DPL; d++) {
      float x = o[r][d];
      x += __shfl_xor(x, 16, 64);
      x += __shfl_xor(x, 32, 64);
      o[r][d] = x;
    }
  if (kg == 0) {
#pragma unroll
    for (int r = 0; r < RT; r++) {
      if (r < R) {
        const int tt = r / group, hh = kvh * group + r % group;
        const size_t prow = (((size_t)b * a.Hq + hh) * a.Tq + tt) * a.nsplit + split;
        float* po = a.part_o + prow * D + DPL * dg;
        if (handoff) {
#pragma unroll
          for (int d = 0; d < DPL; d += 4)
            st16_sc1(a.part_o, (size_t)(po - a.part_o) + d,
                     make_float4(o[r][d] * vs, o[r][d + 1] * vs, o[r][d + 2] * vs, o[r][d + 3] * vs));
        } else {
#pragma unroll
          for (int d = 0; d < DPL; d += 4)
            *(float4*)(po + d) = make_float4(o[r][d] * vs, o[r][d + 1] * vs, o[r][d + 2] * vs, o[r][d + 3] * vs);
        }
      }
    }
  }
  }
  if (g == 0 && row < R && wv == 0) {
    const size_t prow = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit + split;
    if (handoff) {
      st8_sc1(a.part_ml + prow * 2, m, l);
    } else {
      a.part_ml[prow * 2] = m;
      a.part_ml[prow * 2 + 1] = l;
    }
  }
  if (!handoff) return;
  // ---- fused combine: the last split (one wave = one workgroup) of this
  // (b, kv head) to arrive merges the partials of its R query rows (saves the
  // combine launch).  The counter is reset by the merging wave, so graph
  // replays start from zero.
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's sc1 stores are done
  __syncthreads();
  if (lane == 0) {
    const int ns = min(a.nsplit, (len + SPLIT - 1) / SPLIT);
    int* ctr = a.counters + (size_t)b * a.Hkv + kvh;
    const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = prev == ns - 1;
    if (is_last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!is_last) return;
  float* wsh = PVM ? (float*)vl : &ps[0][0];        // LDS scratch of the split, reused
  for (int r0 = 0; r0 < R; r0 += 4) {
    const int nr = min(4, R - r0);
    int hs[4], ts[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int rr = r0 + min(r, nr - 1);
      hs[r] = kvh * group + rr % group;
      ts[r] = rr / group;
    }
    if (!combine_fast<T, true, 4>(a, b, hs, ts, nr))
      for (int r = 0; r < nr; r++) combine_row<T, true>(a, b, hs[r], ts[r], wsh);
  }
  if constexpr (rq) {
    // fused-RoPE decode: every split of this (b, kv head) has read its q / k / v
    // columns of the qkv accumulator: re-zero them for the next layer's GEMV
    float* prow = (float*)a.rq_part + (size_t)b * a.rq_ld;
    for (int hh = kvh * group; hh < (kvh + 1) * group; hh++)
      for (int d = lane * 4; d < D; d += 256) *(float4*)(prow + hh * D + d) = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int d = lane * 4; d < D; d += 256) {
      *(float4*)(prow + (a.Hq + kvh) * D + d) = make_float4(0.f, 0.f, 0.f, 0.f);
      *(float4*)(prow + (a.Hq + a.Hkv + kvh) * D + d) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// merge NR (<= 4) rows (b, hs[r], ts[r]) in ONE memory round trip: lane
// (quad q, phase p) requests its partial quads of splits p, p + P, ... of
// every row together with the rows' (m, l) pairs before any of them is
// needed (the split weights only scale what is already in flight); the P
// phases are summed with shuffles.  A loop over splits waited on one
// dependent L2 round trip per few splits (5.8 us at 17 splits, B = 1), and
// merging rows one after another in the fused combine put R such chains in
// series.  Returns false (nothing done) when the splits do not fit one round.
template <typename T, bool SC1, int NR>
__device__ __forceinline__ bool combine_fast(const AttnDecodeArgs& a, int b, const int* hs, const int* ts, int nr) {
  constexpr int CH = 12;                             // quads in flight per lane per row
  const int lane = threadIdx.x;
  const int len = a.seq_lens[b];
  const int ns = min(a.nsplit, (len + SPLIT - 1) / SPLIT);
  const int Q = a.D / 4;
  if (!(Q == 16 || Q == 32 || Q == 64)) return false;
  const int P = 64 / Q, q = lane % Q, p = lane / Q;
  if (ns > CH * P) return false;
  auto ld4 = [&](const float* x) -> float4 {
    if constexpr (SC1) return ld16_sc1(a.part_o, (size_t)(x - a.part_o));
    else return *(const float4*)x;
  };
  auto ld1 = [](const float* x) -> float {
    if constexpr (SC1) return ld_sc1(x); else return *x;
  };
  float4 pv[NR][CH];
  float2 ml[NR];
  size_t row0[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int rr = min(r, nr - 1);
    row0[r] = (((size_t)b * a.Hq + hs[rr]) * a.Tq + ts[rr]) * a.nsplit;
    const float* po = a.part_o + row0[r] * a.D + 4 * q;
#pragma unroll
    for (int j = 0; j < CH; j++) pv[r][j] = ld4(po + (size_t)min(p + j * P, ns - 1) * a.D);
    ml[r] = make_float2(-INFINITY, 0.f);
    if (lane < ns) {
      if constexpr (SC1) ml[r] = ld8_sc1(a.part_ml + (row0[r] + lane) * 2);
      else ml[r] = make_float2(ld1(a.part_ml + (row0[r] + lane) * 2), ld1(a.part_ml + (row0[r] + lane) * 2 + 1));
    }
  }
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const float M = wave_max(ml[r].x);
    const float w = ml[r].x == -INFINITY ? 0.f : __expf(ml[r].x - M);
    const float L = wave_sum(w * ml[r].y);
    const float invL = L > 0.f ? 1.f / L : 0.f;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < CH; j++) {
      const int s = p + j * P;
      // an unused split holds unwritten bytes: select, never multiply
      const float ws = __shfl(w, s & 63, 64);
      const bool on = s < ns && ws != 0.f;
      o.x += on ? ws * pv[r][j].x : 0.f; o.y += on ? ws * pv[r][j].y : 0.f;
      o.z += on ? ws * pv[r][j].z : 0.f; o.w += on ? ws * pv[r][j].w : 0.f;
    }
    for (int off = Q; off < 64; off <<= 1) {
      o.x += __shfl_xor(o.x, off, 64); o.y += __shfl_xor(o.y, off, 64);
      o.z += __shfl_xor(o.z, off, 64); o.w += __shfl_xor(o.w, off, 64);
    }
    if (p == 0 && r < nr) {
      uint16_t* out = a.out + (((size_t)b * a.Tq + ts[r]) * a.Hq + hs[r]) * a.D + 4 * q;
      *(uint2*)out = make_uint2(pack2<T>(o.x * invL, o.y * invL), pack2<T>(o.z * invL, o.w * invL));
    }
  }
  return true;
}

// merge the nsplit partial (o, m, l) of one (b, h, t) row: split weights
// lane-parallel into LDS, then every lane sums its head dims with
// independent loads.
template <typename T, bool SC1>
__device__ __forceinline__ void combine_row(const AttnDecodeArgs& a, int b, int h, int t, float* wsh) {
  // SC1: the partials were handed over by other waves of this launch (sc1 loads)
  auto ld = [](const float* p) -> float {
    if constexpr (SC1) return ld_sc1(p); else return *p;
  };
  const int lane = threadIdx.x;
  const int len = a.seq_lens[b];
  const int ns = min(a.nsplit, (len + SPLIT - 1) / SPLIT);
  const size_t row0 = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit;
  float M = -INFINITY, L = 0.f;
  if (ns > 1024) {
    // more splits than the LDS weight scratch holds (> 64 Ki keys): every
    // lane recomputes the split weights it needs (rare, long-context only)
    for (int s = lane; s < ns; s += 64) M = fmaxf(M, ld(a.part_ml + (row0 + s) * 2));
    M = wave_max(M);
    uint16_t* out = a.out + (((size_t)b * a.Tq + t) * a.Hq + h) * a.D;
    const float* po = a.part_o + row0 * a.D;
    for (int d = lane; d < a.D; d += 64) {
      float x = 0.f, l = 0.f;
      for (int s = 0; s < ns; s++) {
        const float2 ml = make_float2(ld(a.part_ml + (row0 + s) * 2), ld(a.part_ml + (row0 + s) * 2 + 1));
        const float w = ml.x == -INFINITY ? 0.f : __expf(ml.x - M);
        l += w * ml.y;
        x += w * ld(po + (size_t)s * a.D + d);
      }
      out[d] = from_f32<T>(l > 0.f ? x / l : 0.f);
    }
    __syncthreads();
    return;
  }
  {
    const int hs[1] = {h}, ts[1] = {t};
    if (combine_fast<T, SC1, 1>(a, b, hs, ts, 1)) return;
  }
  if (ns <= 64) {
    // one (m, l) pair per lane, loaded once
    float2 ml = make_float2(-INFINITY, 0.f);
    if (lane < ns) ml = make_float2(ld(a.part_ml + (row0 + lane) * 2), ld(a.part_ml + (row0 + lane) * 2 + 1));
    M = wave_max(ml.x);
    const float w = ml.x == -INFINITY ? 0.f : __expf(ml.x - M);
    L = w * ml.y;
    if (lane < ns) wsh[lane] = w;
  } else {
    for (int s = lane; s < ns; s += 64) M = fmaxf(M, ld(a.part_ml + (row0 + s) * 2));
    M = wave_max(M);
    for (int s = lane; s < ns; s += 64) {
      const float2 ml = make_float2(ld(a.part_ml + (row0 + s) * 2), ld(a.part_ml + (row0 + s) * 2 + 1));
      const float w = ml.x == -INFINITY ? 0.f : __expf(ml.x - M);
      L += w * ml.y;
      if (s < 1024) wsh[s] = w;
    }
  }
  L = wave_sum(L);
  __syncthreads();
  const float invL = L > 0.f ? 1.f / L : 0.f;
  uint16_t* out = a.out + (((size_t)b * a.Tq + t) * a.Hq + h) * a.D;
  const float* po = a.part_o + row0 * a.D;
  // two head dims per lane (d, d + 64) so both columns' split loads are in
  // flight together: half the dependent memory round trips at D = 128
  for (int d = lane; d < a.D; d += 128) {
    const bool two = d + 64 < a.D;
    const int e = two ? d + 64 : d;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f, y0 = 0.f, y1 = 0.f, y2 = 0.f, y3 = 0.f;
    int s = 0;
    for (; s + 4 <= ns; s += 4) {
      const float* p0 = po + (size_t)s * a.D;
      const float u0 = ld(p0 + d), u1 = ld(p0 + a.D + d), u2 = ld(p0 + 2 * a.D + d), u3 = ld(p0 + 3 * a.D + d);
      const float v0 = ld(p0 + e), v1 = ld(p0 + a.D + e), v2 = ld(p0 + 2 * a.D + e), v3 = ld(p0 + 3 * a.D + e);
      x0 += wsh[s] * u0;
      x1 += wsh[s + 1] * u1;
      x2 += wsh[s + 2] * u2;
      x3 += wsh[s + 3] * u3;
      y0 += wsh[s] * v0;
      y1 += wsh[s + 1] * v1;
      y2 += wsh[s + 2] * v2;
      y3 += wsh[s + 3] * v3;
    }
    for (; s < ns; s++) {
      x0 += wsh[s] * ld(po + (size_t)s * a.D + d);
      y0 += wsh[s] * ld(po + (size_t)s * a.D + e);
    }
    out[d] = from_f32<T>((x0 + x1 + x2 + x3) * invL);
    if (two) out[e] = from_f32<T>((y0 + y1 + y2 + y3) * invL);
  }
  __syncthreads();
}

// fused-RoPE decode: every split has read the qkv accumulator by now, so the
// combine re-zeroes it for the next layer's atomic GEMV (block (h, b): q head
// h and the k/v column blocks dealt over the Hq blocks -- all of them are
// covered for any Hq / Hkv ratio, MHA included)
__device__ __forceinline__ void combine_zero_rq(const AttnDecodeArgs& a, int h, int b, int tid, int nthr) {
  float* row = (float*)a.rq_part + (size_t)b * a.rq_ld;
  const int D = a.D;
  for (int d = tid * 4; d < D; d += 4 * nthr) *(float4*)(row + h * D + d) = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int hh = h; hh < 2 * a.Hkv; hh += a.Hq)
    for (int d = tid * 4; d < D; d += 4 * nthr)
      *(float4*)(row + (a.Hq + hh) * D + d) = make_float4(0.f, 0.f, 0.f, 0.f);
}

template <typename T>
__global__ void __launch_bounds__(64) attn_combine_kernel(const AttnDecodeArgs a) {
  __shared__ float wsh[1024];
  combine_row<T>(a, blockIdx.z, blockIdx.x, blockIdx.y, wsh);
  if (a.rq_part != nullptr && blockIdx.y == 0) combine_zero_rq(a, blockIdx.x, blockIdx.z, threadIdx.x, 64);
}

// long contexts (more splits than one wave merges in a round trip; 32 K keys
// = 513 splits): 8 waves per (b, h, t) row.  Split weights for every split go
// to LDS first; then lane (quad q, phase p) of wave w streams splits
// w P + p + j (8 P) with 16 partial quads in flight per round, and the
// (wave, phase) partial sums meet in LDS.  One wave looping over the splits
// (the kernel above) spent 57.7 us per layer at 32 K keys, longer than the
// split attention itself (37.2 us).
constexpr int CW_NW = 8, CW_MAXS = 4096;
template <typename T>
__global__ void __launch_bounds__(CW_NW * 64) attn_combine_wide_kernel(const AttnDecodeArgs a) {
  __shared__ float wsh[CW_MAXS];
  __shared__ float4 red[CW_NW * 64];
  __shared__ float rsum[CW_NW];
  const int h = blockIdx.x, t = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int len = a.seq_lens[b];
  const int ns = min(a.nsplit, (len + SPLIT - 1) / SPLIT);
  const size_t row0 = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit;
  // ---- split weights: block max, exp, block sum of w * l
  float mx = -INFINITY;
  for (int s = tid; s < ns; s += CW_NW * 64) mx = fmaxf(mx, a.part_ml[(row0 + s) * 2]);
  mx = wave_max(mx);
  if (lane == 0) rsum[wave] = mx;
  __syncthreads();
  float M = rsum[0];
#pragma unroll
  for (int w = 1; w < CW_NW; w++) M = fmaxf(M, rsum[w]);
  float L = 0.f;
  for (int s = tid; s < ns; s += CW_NW * 64) {
    const float2 ml = *(const float2*)(a.part_ml + (row0 + s) * 2);
    const float w = ml.x == -INFINITY ? 0.f : __expf(ml.x - M);
    wsh[s] = w;
    L += w * ml.y;
  }
  L = wave_sum(L);
  __syncthreads();                                  // rsum (max) read by all
  if (lane == 0) rsum[wave] = L;
  __syncthreads();
  L = 0.f;
#pragma unroll
  for (int w = 0; w < CW_NW; w++) L += rsum[w];
  const float invL = L > 0.f ? 1.f / L : 0.f;
  // ---- weighted sum of the partial rows
  const int Q = a.D / 4, P = 64 / Q, q = lane % Q, p = lane / Q;
  const int gp = wave * P + p, GS = CW_NW * P;     // phase of this lane, phase stride
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p < P) {
    constexpr int U = 16;
    const float* po = a.part_o + row0 * a.D + 4 * q;
    for (int s0 = gp; s0 < ns; s0 += U * GS) {
      float4 pv[U];
#pragma unroll
      for (int j = 0; j < U; j++) pv[j] = *(const float4*)(po + (size_t)min(s0 + j * GS, ns - 1) * a.D);
#pragma unroll
      for (int j = 0; j < U; j++) {
        const int s = s0 + j * GS;
        // an unused split holds unwritten bytes: select, never multiply
        const float ws = s < ns ? wsh[s] : 0.f;
        const bool on = ws != 0.f;
        o.x += on ? ws * pv[j].x : 0.f; o.y += on ? ws * pv[j].y : 0.f;
        o.z += on ? ws * pv[j].z : 0.f; o.w += on ? ws * pv[j].w : 0.f;
      }
    }
  }
  red[tid] = o;
  __syncthreads();
  if (tid < Q) {
    float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int w = 0; w < CW_NW; w++)
      for (int pp = 0; pp < P; pp++) {
        const float4 v = red[w * 64 + pp * Q + tid];
        r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
      }
    uint16_t* out = a.out + (((size_t)b * a.Tq + t) * a.Hq + h) * a.D + 4 * tid;
    *(uint2*)out = make_uint2(pack2<T>(r.x * invL, r.y * invL), pack2<T>(r.z * invL, r.w * invL));
  }
  if (a.rq_part != nullptr && t == 0) combine_zero_rq(a, h, b, tid, CW_NW * 64);
}

// the combine launch for a.nsplit splits (the max over the batch)
template <typename T>
static void launch_combine(const AttnDecodeArgs& a, hipStream_t st) {
  if (a.nsplit > 24 && a.nsplit <= CW_MAXS && a.D % 4 == 0)
    hipLaunchKernelGGL((attn_combine_wide_kernel<T>), dim3(a.Hq, a.Tq, a.B), dim3(CW_NW * 64), 0, st, a);
  else
    hipLaunchKernelGGL((attn_combine_kernel<T>), dim3(a.Hq, a.Tq, a.B), dim3(64), 0, st, a);
}

template <typename T, int D, int RT, bool PVM = false>
static void launch_v2(const AttnDecodeArgs& a0, hipStream_t st) {
  AttnDecodeArgs a = a0;
  // combine fused into the split kernel when the merge fits its LDS scratch
  if (a.nsplit > SPLIT * RT || a.no_combine) a.counters = nullptr;
  dim3 grid(a.nsplit, a.Hkv, a.B);
  static int simds = 0;
  if (simds == 0) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    simds = 4 * (cus > 0 ? cus : 256);
  }
  static const int latev_env = getenv("ILLM_ATTN_LATEV") ? atoi(getenv("ILLM_ATTN_LATEV")) : -1;
  const bool latev = latev_env >= 0 ? latev_env == 1 : (long)a.nsplit * a.Hkv * a.B > simds;
  // two waves per split (PVM, 16-bit KV, no in-kernel combine) while the doubled
  // grid still has at most one wave per SIMD: MI355X, Llama-3-8B at 1K keys
  // (same-box A/B, profiles/bench_b*_r3_nwv*.json): B=1 1.654 -> 1.646 ms/token,
  // but B=8 (1024 split waves) 2.366 -> 2.419 ms/step, so larger grids keep one.
  // ILLM_ATTN_NWV=1 / 2 forces either form
  static const int nwv_env = getenv("ILLM_ATTN_NWV") ? atoi(getenv("ILLM_ATTN_NWV")) : 0;
  const bool small_grid = 2L * a.nsplit * a.Hkv * a.B <= simds;
  const bool two = PVM && a.counters == nullptr && a.kv_fp8 == 0 && (nwv_env == 2 || (nwv_env == 0 && small_grid));
  if constexpr (D / 16 >= 8) {
    if (a.rq_part != nullptr) {
      if constexpr (PVM) {
        if (two) {
          if (latev) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, true, true, PVM, 2>), grid, dim3(128), 0, st, a);
          else hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, true, false, PVM, 2>), grid, dim3(128), 0, st, a);
          if (!a.no_combine) launch_combine<T>(a, st);
          return;
        }
      }
      if (latev) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, true, true, PVM>), grid, dim3(64), 0, st, a);
      else hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, true, false, PVM>), grid, dim3(64), 0, st, a);
      if (a.counters == nullptr && !a.no_combine)
        launch_combine<T>(a, st);
      return;
    }
  }
  if constexpr (PVM) {
    if (two) {
      if (latev) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, false, true, PVM, 2>), grid, dim3(128), 0, st, a);
      else hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, false, false, PVM, 2>), grid, dim3(128), 0, st, a);
      if (!a.no_combine) launch_combine<T>(a, st);
      return;
    }
  }
  if (latev) {
    if (a.kv_fp8 == 1) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 1, RT, false, true, PVM>), grid, dim3(64), 0, st, a);
    else if (a.kv_fp8 == 2) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 2, RT, false, true, PVM>), grid, dim3(64), 0, st, a);
    else hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, false, true, PVM>), grid, dim3(64), 0, st, a);
  } else {
    if (a.kv_fp8 == 1) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 1, RT, false, false, PVM>), grid, dim3(64), 0, st, a);
    else if (a.kv_fp8 == 2) hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 2, RT, false, false, PVM>), grid, dim3(64), 0, st, a);
    else hipLaunchKernelGGL((attn_decode_v2_kernel<T, D, 0, RT, false, false, PVM>), grid, dim3(64), 0, st, a);
  }
  if (a.counters == nullptr && !a.no_combine)
    launch_combine<T>(a, st);
}

}  // namespace illm
#include "attn_dec_v3.cuh"
namespace illm {

template <typename T, int D>
void launch_d(const AttnDecodeArgs& a, hipStream_t st) {
  const int R = (a.Hq / a.Hkv) * a.Tq;
  if constexpr (D == 64 || D == 128) {
    if (v3_ok(a, D)) {
      if constexpr (D == 128) {
        if (a.rq_part != nullptr)
          return a.rq_prerot && a.rq_bias == nullptr ? launch_v3<T, D, 2>(a, st) : launch_v3<T, D, 1>(a, st);
      }
      return launch_v3<T, D, 0>(a, st);
    }
  }
  // P V on MFMA (ILLM_ATTN_PVM=0 keeps the per-lane FMA form, for A/B runs)
  static const bool pvm = getenv("ILLM_ATTN_PVM") ? atoi(getenv("ILLM_ATTN_PVM")) != 0 : true;
  if constexpr (D == 64 || D == 128) {
    if (pvm && R <= 16) return launch_v2<T, D, 16, true>(a, st);
  }
  if constexpr (D == 64 || D == 128 || D == 256) {
    if (R <= 4) return launch_v2<T, D, 4>(a, st);
    if (R <= 8) return launch_v2<T, D, 8>(a, st);
    if (D <= 128) return launch_v2<T, D, 16>(a, st);
  }
  dim3 grid(a.nsplit, a.Hkv, a.B);
  if (a.kv_fp8 == 1) hipLaunchKernelGGL((attn_decode_kernel<T, D, 1>), grid, dim3(64), 0, st, a);
  else if (a.kv_fp8 == 2) hipLaunchKernelGGL((attn_decode_kernel<T, D, 2>), grid, dim3(64), 0, st, a);
  else hipLaunchKernelGGL((attn_decode_kernel<T, D, 0>), grid, dim3(64), 0, st, a);
  if (!a.no_combine) launch_combine<T>(a, st);
}

}  // namespace illm
