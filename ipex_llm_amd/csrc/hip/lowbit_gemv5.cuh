// v5 low-bit GEMV for M <= 16 rows: the decode hot path (xe_linear.forward_new
// / xe_batch.batch_forward / xe_linear.mlp_forward_xpu at batch <= 16,
// SRC/transformers/low_bit_linear.py:698-708, models/common.py:146-161; the
// FlashMoE decode GEMV moe_forward_vec, models/qwen3_moe.py:88-105).
//
// Why v5 (measured on MI355X with rocprofv3 PMC, gate_up 28672x4096 M=1):
// the v4 kernel issued 24 VALU per MFMA (scale/offset applied to every
// decoded weight with packed f16 ops, per-k-step exec-masked LDS reads) and
// ran ~1 wave per SIMD, so it was VALU- and latency-bound at 3.0-3.5 TB/s.
// v5 keeps the weights as raw codes in the MFMA A operand and moves all
// per-block arithmetic to the accumulator side:
//   * A fragment = raw code value (int4: bf16 0x4300|q = 128+q / f16
//     0x6400|q = 1024+q via ONE v_and_or_b32 per packed pair; fp4 / fp8 via
//     the gfx950 v_cvt_scalef32_pk_* converters; nf4/nf3 via an LDS pair
//     table in f16), exact in the MFMA input type;
//   * each 64-element block accumulates into a fresh 4-float P, then per
//     row i: acc += d_i * (P_i - OFF * sx_blk) (+ min_i * sx_blk for asym),
//     where sx_blk = sum of the block's activations, computed ONCE per
//     workgroup while x is staged in LDS (no per-element subtract, no
//     all-ones MFMA): ~11 VALU per k-step instead of ~25;
//   * unused MFMA columns (m >= M) read a clamped valid row: D's column j
//     depends only on B's column j, so no masking is needed;
//   * KW waves of a workgroup split the chunk range of the same tile(s)
//     and reduce through LDS, so the grid reaches 3-4 waves per SIMD
//     without split-K slabs (the GLU cannot split K across workgroups);
//   * scales are stored chunk-major (formats.h): one 16-B load gives the 4
//     C-fragment rows' (blk0, blk1) scales of a chunk.
#pragma once
#include <cstdio>
#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "../common/quant_block.h"
#include "gemv_args.h"
#include "illm_device.h"

namespace illm {

// packed-pair nibble extract (x & m) | c as ONE v_and_or_b32: hipcc splits
// the pattern into v_and + v_or (gfx9 VOP3 takes no literal and one
// constant-bus read), so the mask is an SGPR and the magic a VGPR operand
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m_s, uint32_t c_v) {
  uint32_t r;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(m_s), "v"(c_v));
  return r;
}

template <typename C> struct Raw;
template <> struct Raw<BF16> {
  static constexpr uint32_t k4 = 0x43004300u;   // bf16(128 + q)
  static constexpr float off4 = 128.f;
};
template <> struct Raw<F16> {
  static constexpr uint32_t k4 = 0x64006400u;   // f16(1024 + q)
  static constexpr float off4 = 1024.f;
};

// raw value offset per decoder: value = code_raw - OFF (before scale)
template <int DK, typename C>
__host__ __device__ constexpr float raw_off() {
  return DK == DK_INT4S ? Raw<C>::off4 + 8.f
       : DK == DK_INT4A ? Raw<C>::off4
       : DK == DK_INT8S ? 128.f
       : 0.f;
}

template <int DK, typename C>
__device__ __forceinline__ uint4 raw_a4(uint32_t u, uint32_t mask_s, uint32_t magic_v, const uint32_t* lut2) {
  uint4 r;
  if constexpr (DK == DK_INT4S || DK == DK_INT4A) {
    r.x = and_or(u, mask_s, magic_v);
    r.y = and_or(u >> 4, mask_s, magic_v);
    r.z = and_or(u >> 8, mask_s, magic_v);
    r.w = and_or(u >> 12, mask_s, magic_v);
  } else if constexpr (DK == DK_FP4) {
    if constexpr (std::is_same<C, BF16>::value) {
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
  } else {  // DK_LUT4 (C = F16 pair table)
    r.x = lut2[u & 0xff];
    r.y = lut2[(u >> 8) & 0xff];
    r.z = lut2[(u >> 16) & 0xff];
    r.w = lut2[u >> 24];
  }
  return r;
}

template <int DK, typename C>
__device__ __forceinline__ uint32_t raw_pair8(uint32_t u, bool hi) {
  if constexpr (DK == DK_FP8E4) {
    if constexpr (std::is_same<C, BF16>::value)
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(u, 1.0f, false));
    else
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(u, 1.0f, false));
  } else if constexpr (DK == DK_FP8E5) {
    if constexpr (std::is_same<C, BF16>::value)
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8(u, 1.0f, false));
    else
      return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u, 1.0f, true)
                                             : __builtin_amdgcn_cvt_scalef32_pk_f16_bf8(u, 1.0f, false));
  } else {
    // integer bytes through the exact small-integer float conversion;
    // signed codes are biased by 128 (raw_off = 128)
    if constexpr (DK == DK_INT8S) u ^= 0x80808080u;
    const int sh = hi ? 16 : 0;
    return pack2<C>((float)((u >> sh) & 0xff), (float)((u >> (sh + 8)) & 0xff));
  }
}

template <int DK, typename C>
__device__ __forceinline__ uint4 raw_a8(uint32_t lo, uint32_t hi) {
  return make_uint4(raw_pair8<DK, C>(lo, false), raw_pair8<DK, C>(lo, true), raw_pair8<DK, C>(hi, false),
                    raw_pair8<DK, C>(hi, true));
}

// LDS plan of one workgroup (bytes): x slice [rows][kw + 8] in C, then per
// (row, chunk) float4 {-OFF*sx0, -OFF*sx1, sx0, sx1}, then the KW reduction
// area [<= 8 waves][2 tiles][64] float4, then (attention-combine prologue only)
// the split weights [rows][heads of the slice][ans + 1] f32.
// x rows are padded to whole 1-KB LDS-DMA pieces (512 16-bit elements): a
// row's last piece is issued with every lane active (no exec-masked LDS-DMA)
// and its tail lands in the row's own padding; + 8 elements keep the 16 rows
// of a fragment read on distinct banks
__host__ __device__ constexpr int gemv5_x_ld(int kw) { return (kw + 511) / 512 * 512 + 8; }
__host__ __device__ constexpr size_t gemv5_shmem(int rows, int cpk) {
  return ((size_t)rows * gemv5_x_ld(cpk * 128) * 2 + 15) / 16 * 16 + (size_t)rows * cpk * 16 + 8 * 2 * 64 * 16;
}
__host__ __device__ constexpr int gemv5_attn_heads(int cpk, int D) { return (cpk * 128 + D - 1) / D + 1; }
__host__ __device__ constexpr size_t gemv5_attn_shmem(int rows, int cpk, int D, int ns) {
  return (size_t)rows * gemv5_attn_heads(cpk, D) * (ns + 1) * 4;
}

// weight stream loads: read once per decode step by one CU (the model's
// weights are far larger than the 256 MB MALL, nothing survives to the next
// hipGraph replay), so they take the non-temporal policy.  Same-box A/B on
// MI355X (Llama-3-8B, 256 steps x 2, profiles/gemv_nt_ab_samebox.txt):
// B=1 1.780 -> 1.732 ms/token, B=8 2.381 -> 2.356 ms/step.  ILLM_GEMV_NT=0
// at build time restores default-policy loads.
#ifndef ILLM_GEMV_NT
#define ILLM_GEMV_NT 1
#endif
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// ablation knobs for tools/probe/gemv5_probe.hip (timing only; results are
// wrong when set): bit 0 = no dequant/MFMA (loads are xor-folded), bit 1 =
// no norm/x-staging prologue, bit 2 = no epilogue stores/atomics
#ifndef ILLM_GEMV5_ABL
#define ILLM_GEMV5_ABL 0
#endif
__device__ __forceinline__ uint4 ldw16(const uint8_t* p) {
#if ILLM_GEMV_NT
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v[0], v[1], v[2], v[3]);
#else
  return *(const uint4*)p;
#endif
}

// minimum waves per SIMD the register allocation must allow (1 = unconstrained)
#ifndef ILLM_GEMV5_MINW
#define ILLM_GEMV5_MINW 1
#endif
// scale words shared across lanes (SCL above); ILLM_GEMV5_SCL=0 at build time
// restores the per-lane scale loads in the chunk ring
#ifndef ILLM_GEMV5_SCL
#define ILLM_GEMV5_SCL 1
#endif
// x staging by LDS-DMA (buffer_load ... lds: 16 B per lane straight into LDS,
// no VGPR round trip, every row requested at once) for launches whose x slice
// needs more than one batch of register-staged loads per thread (the batch-8
// gate/up GEMV: 64 KB per workgroup, two dependent L2 round trips before).
// Issued from inline asm like the 8-phase GEMM's (gemm_8p.hip dma16).
#ifndef ILLM_GEMV5_XDMA
#define ILLM_GEMV5_XDMA 1
#endif
// x-side loads (activations, norm-in accumulator / residual / weight) issued
// ahead of the weight ring (gemv5_body); ILLM_GEMV5_EARLYX=0 at build time
// restores the round-5 order (A/B builds, tools/ab_lib.sh)
#ifndef ILLM_GEMV5_EARLYX
#define ILLM_GEMV5_EARLYX 1
#endif
typedef int32_t gv5_rsrc __attribute__((ext_vector_type(4)));
__device__ __forceinline__ gv5_rsrc gv5_make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)(uintptr_t)base;
  return gv5_rsrc{(int32_t)(uint32_t)p, (int32_t)((uint32_t)(p >> 32) & 0xffffu), (int32_t)bytes, 0x00020000};
}
__device__ __forceinline__ void gv5_dma16(const gv5_rsrc& rs, const void* lds, uint32_t voff) {
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)lds);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :: "s"(la), "v"(voff), "s"(rs) : "memory", "m0");
}

// per-workgroup timeline stamps (tools/probe/gemv5_probe.hip PROBE_MODE=s,
// built with its own definition): 0 entry, 1 x staged, 2 chunks computed,
// 3 epilogue issued.  Empty in the library.
#ifndef ILLM_GEMV5_STAMP
#define ILLM_GEMV5_STAMP(i) ((void)0)
#endif

// block coordinates of one GEMV workgroup (blockIdx / gridDim of the launch)
struct G5Blk {
  int x, y, z, gx, gy, gz;
};

// EPI_ATOMIC norm-out epilogue (gemv_args.h lctr ...): the last-arriving
// split-K workgroup of column block blk.x turns the block's finished f32 sums
// into the next layer half's inputs, so the standalone residual-add + RMSNorm
// launch between o_proj and the gate/up GEMV goes away.  Hand-off: the adds
// are memory-side f32 atomics, every wave waits for its own (vmcnt(0)) before
// the workgroup's one agent-scope ticket, the last arriver reads the sums with
// sc1 (L1-bypassing) loads -- the MI355X form used by the fused attention
// combine (attn_dec_v3.cuh).  Thread v handles 4 consecutive columns of row
// v / C4; a row's C4 threads are one aligned lane group (shuffle reduce).
template <typename T>
__device__ __forceinline__ void gemv5_norm_out(const GemvArgs& a, const G5Blk& blk, int Mloc, int nb, int NC,
                                               int nthr) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* ctr = a.lctr + blk.x;
    const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == blk.gy - 1;
    if (prev == blk.gy - 1) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  auto rnd = [](float v) { return to_f32<T>(from_f32<T>(v)); };
  const int C4 = NC / 4;                        // 16 or 32 (host-checked)
  float* ws = (float*)a.out;
  for (int v = threadIdx.x; v < Mloc * C4; v += nthr) {
    const int m = v / C4, n = nb + 4 * (v % C4);
    float ss = 0.f;
    if (n < a.N) {                              // N % 4 == 0 (host-checked)
      const size_t e = (size_t)m * a.N + n;
      const float4 s = ld16_sc1(ws, e);
      const uint2 r = *(const uint2*)(a.lres + e);
      const uint2 w = *(const uint2*)(a.lnw + n);
      const float sv[4] = {s.x, s.y, s.z, s.w};
      const uint32_t rw[2] = {r.x, r.y}, ww[2] = {w.x, w.y};
      float h[4], xo[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t rr = rw[i >> 1], wr = ww[i >> 1];
        const float rv = to_f32<T>((uint16_t)((i & 1) ? rr >> 16 : rr & 0xffff));
        float wv = to_f32<T>((uint16_t)((i & 1) ? wr >> 16 : wr & 0xffff));
        if (a.lunit) wv = rnd(1.f + wv);
        h[i] = rnd(rnd(sv[i]) + rv);
        xo[i] = wv * h[i];
        ss += h[i] * h[i];
      }
      *(uint2*)(a.lres_out + e) = make_uint2(pack2<T>(h[0], h[1]), pack2<T>(h[2], h[3]));
      *(uint2*)(a.lxo + e) = make_uint2(pack2<T>(xo[0], xo[1]), pack2<T>(xo[2], xo[3]));
      *(float4*)(ws + e) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int o = C4 >> 1; o > 0; o >>= 1) ss += __shfl_xor(ss, o, C4);
    if ((v & (C4 - 1)) == 0) __hip_atomic_fetch_add(a.lss + m, ss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// XM (x mode): 0 = every input form, chosen at run time; 1 = plain 16-bit x
// staged by LDS-DMA only (the launcher checks the arguments).  A separate
// instantiation because hipcc's wait insertion is path-insensitive: the
// loads of the other staging forms, merged at the join, made it drain
// vmcnt(0) right behind the DMA staging's counted wait, i.e. wait for every
// weight chunk in flight before the first MFMA (seen in the .s).
template <int DK, typename T, int EPI, int TPW, int KW, bool MOE, int NW, int PF, bool SCL, int XM = 0, int XS = 1>
__device__ __forceinline__ void gemv5_body(const GemvArgs& a, const G5Blk& blk) {
  // PF: chunks in flight per wave (4; 8 = every chunk of a decode split-K
  // slice of <= 8 chunks requested before the prologue)
  using C = typename std::conditional<DK == DK_LUT4, F16, T>::type;   // MFMA input type
  constexpr int BITS = dk_bits(DK);
  constexpr int TG = NW / KW;          // tile groups per workgroup (NW waves)
  constexpr float OFF = raw_off<DK, C>();
  constexpr bool HASMIN = dk_has_min(DK);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint32_t lut2[DK == DK_LUT4 ? 256 : 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  int Mloc = a.M;
  const uint8_t* wbase = a.w;
  const int32_t* prow = nullptr;
  if constexpr (MOE) {
    const int e = blk.z;
    const int m0 = a.moe_off[e];
    Mloc = min(16, a.moe_off[e + 1] - m0);
    if (Mloc <= 0) return;                // expert not routed to: the whole block exits
    wbase += (size_t)e * a.w_stride;
    prow = a.moe_rows + m0;
  }
  auto xrow_of = [&](int m) -> int { if constexpr (MOE) return prow[m] / a.moe_xdiv; else return m; };
  auto orow_of = [&](int m) -> int { if constexpr (MOE) return prow[m]; else return m; };

  const int nks = blk.gy;
  const int cpk = a.cpk > 0 ? a.cpk : (a.KC + nks - 1) / nks;
  const int c0 = blk.y * cpk;
  const int c1 = min(a.KC, c0 + cpk);
  const int kbase = c0 * 128;
  const int kw = (c1 - c0) * 128;
  const int ldx = gemv5_x_ld(kw);
  uint16_t* xs = (uint16_t*)smem;
  float4* sxs = (float4*)(smem + ((size_t)Mloc * ldx * 2 + 15) / 16 * 16);        // [Mloc][c1-c0]
  float4* red = (float4*)((uint8_t*)sxs + (size_t)Mloc * (c1 - c0) * 16);          // [4][TPW][64]
  float* aw = (float*)(red + 8 * 2 * 64);                                          // attention split weights

  const int NT = (a.N * (EPI == EPI_GLU ? 2 : 1) + 15) / 16;
  const int tg = wave / KW, kp = wave % KW;
  const int tile0 = (blk.x * TG + tg) * TPW;
  const int per = (c1 - c0 + KW - 1) / KW;
  const int wc0 = c0 + kp * per;
  const int wc1 = min(c1, wc0 + per);
  const bool wave_on = tile0 < NT && wc0 < wc1;
  // debug build: the host geometry must cover every output tile and K chunk
  if (ILLM_DCHECK_FAILS((int64_t)blk.gx * TG * TPW >= NT && (int64_t)nks * cpk >= a.KC && Mloc <= 16, a.err,
                        ERR_GEOMETRY))
    return;
  ILLM_GEMV5_STAMP(0);
  const size_t TB = (size_t)dk_tile_bytes(DK, a.KC);
  const size_t soff = (size_t)a.KC * dk_code_chunk(DK) + (size_t)g * 16;   // + c * 64: rows 4g..4g+3
  const size_t moff = soff + (size_t)16 * a.KC * 4;
  const uint8_t* tb[TPW];
#pragma unroll
  for (int t = 0; t < TPW; t++) tb[t] = wbase + (size_t)min(tile0 + t, NT - 1) * TB;

  // SCL: the 16 lanes that share a k-group g hold the scale words of 16
  // consecutive chunks (lane 16 g + j: chunk sw0 + j, rows 4g..4g+3) instead of
  // each lane re-loading its chunk's word into the ring: a chunk in flight
  // costs 4 VGPRs (codes) instead of 8, so twice the chunks fit in flight;
  // the word is fetched with a ds_bpermute when the chunk is computed
  struct Chunk {
    uint4 q[TPW][BITS / 4];
    uint4 sc[SCL ? 1 : TPW];
    uint4 mn[(SCL || !HASMIN) ? 1 : TPW];
  };
  auto load_chunk = [&](Chunk& ch, int c) {
    c = min(c, wc1 - 1);
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      const uint8_t* rec = tb[t] + (size_t)c * dk_code_chunk(DK);
      ch.q[t][0] = ldw16(rec + lane * 16);
      if constexpr (BITS == 8) ch.q[t][1] = ldw16(rec + 1024 + lane * 16);
      if constexpr (!SCL) {
        ch.sc[t] = ldw16(tb[t] + soff + (size_t)c * 64);
        if constexpr (HASMIN) ch.mn[t] = ldw16(tb[t] + moff + (size_t)c * 64);
      }
    }
  };
  uint4 scl[TPW], mnl[TPW];
  const int sw0 = wc0;
  auto load_scl = [&](int cb) {
    const int cc = min(cb + r16, wc1 - 1);
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      scl[t] = ldw16(tb[t] + soff + (size_t)cc * 64);
      if constexpr (HASMIN) mnl[t] = ldw16(tb[t] + moff + (size_t)cc * 64);
    }
  };
  // GLU over a deferred-norm input staged elsewhere (gemv5_norm_out): the
  // row's sum of squares, requested first, used by the epilogue
  float xss_raw = 0.f;
  if constexpr (EPI == EPI_GLU)
    if (a.xpss != nullptr && a.xpart == nullptr) xss_raw = a.xpss[orow_of(min(r16, Mloc - 1))];
  // ---- zero a consumed atomic accumulator (its readers ran earlier in the
  // stream), spread over every workgroup of the grid (up to ~1 MB at M = 8)
  if (a.nzero) {
    const int nthr = NW * 64;
    const size_t nb = (size_t)blk.gx * blk.gy * blk.gz;
    const size_t bid = ((size_t)blk.z * blk.gy + blk.y) * blk.gx + blk.x;
    const size_t nv = (size_t)a.nzero_n / 4;
    for (size_t i = bid * nthr + threadIdx.x; i < nv; i += nb * nthr)
      ((float4*)a.nzero)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // ---- x-side loads BEFORE the weight ring.  Vector-memory loads retire in
  // issue order, so x loads issued behind the ring (as before round 6) could
  // be staged only once every weight chunk had arrived: the LDS staging, the
  // block sums and the barrier sat behind the HBM round trip (per-workgroup
  // stamps, profiles/gemv5_stamps_r6.jsonl).
  //   XM 1 / 2 (the decode forms, their own instantiations): the thread's XS
  //   16-B slots of x (XM 1) or of the deferred-norm inputs -- accumulator,
  //   residual, norm weight (XM 2) -- go to registers first, clamped and
  //   unconditional; hipcc then waits for exactly these (counted vmcnt).  An
  //   LDS-DMA form with a hand-counted wait produced NaN once the ring was
  //   refilled (K >= 2048): LDS-DMA and register loads are not retired in one
  //   order, so the count cannot isolate the DMA pieces.
  //   XM 0: x requested first by LDS-DMA, waited for with vmcnt(0).
  const int xvpr = kw / 8, xtotal = Mloc * xvpr;
  const bool defer = XM == 2 || (XM == 0 && a.nacc != nullptr && a.ndefer != 0);
  const bool plain_x = XM == 1 || (XM == 0 && !a.apo && !a.xpart && !defer && !a.nacc);
  // XM 0 LDS-DMA: 16-bit x that needs no conversion, whole K chunks inside K;
  // each row in whole 1-KB pieces (64 lanes x 16 B) into its padded LDS row
  const bool dma_x = XM == 0 && ILLM_GEMV5_XDMA && !(ILLM_GEMV5_ABL & 2) && plain_x && !MOE &&
                     std::is_same<C, T>::value && kbase + kw <= a.K &&
                     (ILLM_GEMV5_EARLYX || Mloc * xvpr > 4 * NW * 64);
  constexpr int XR = XM == 0 ? 1 : XS;
  uint4 xr[XR], er[XR], ew[XR];
  float4 ea0[XR], ea1[XR];
  if constexpr (XM == 1) {
#pragma unroll
    for (int u = 0; u < XS; u++) {
      const int vv = min((int)threadIdx.x + u * NW * 64, xtotal - 1);
      const int m = vv / xvpr, kk = (vv % xvpr) * 8;
      xr[u] = *(const uint4*)(a.x + (size_t)m * a.ldx + kbase + kk);
    }
  } else if constexpr (XM == 2) {
#pragma unroll
    for (int u = 0; u < XS; u++) {
      const int vv = min((int)threadIdx.x + u * NW * 64, xtotal - 1);
      const int m = vv / xvpr, k = kbase + (vv % xvpr) * 8;
      const float4* pa = (const float4*)(a.nacc + (size_t)m * a.K + k);
      ea0[u] = pa[0];
      ea1[u] = pa[1];
      er[u] = *(const uint4*)(a.nres + (size_t)m * a.K + k);
      ew[u] = *(const uint4*)(a.nweight + k);
    }
  }
  if (dma_x) {
    const int per_row = (xvpr + 63) >> 6, nins = Mloc * per_row;
    const gv5_rsrc rx = gv5_make_rsrc(a.x, (uint32_t)((size_t)a.M * a.ldx * 2));
    for (int i = wave; i < nins; i += NW) {      // wave-uniform: one whole row piece per instruction
      const int m = i / per_row, j = i - m * per_row;
      gv5_dma16(rx, xs + m * ldx + j * 512, (uint32_t)(((size_t)m * a.ldx + kbase + j * 512 + lane * 8) * 2));
    }
  }
  asm volatile("" ::: "memory");             // the ring loads stay behind these

  Chunk ring[PF];
  // XM 1 / 2: issued unconditionally (clamped, valid addresses) -- behind a
  // wave_on branch hipcc counted the no-ring path at the join and drained the
  // ring before staging x
  if (XM != 0 || wave_on) {
    if constexpr (SCL) load_scl(wc0);
#pragma unroll
    for (int u = 0; u < PF; u++) load_chunk(ring[u], max(wc0, 0) + u);
  }
  if constexpr (DK == DK_LUT4) {
    if (threadIdx.x < 256)
      lut2[threadIdx.x] = pack2<F16>(hd_lut4(a.lut_fmt, threadIdx.x & 15), hd_lut4(a.lut_fmt, threadIdx.x >> 4));
  }

  // ---- attention-combine prologue: per (row, head) split weights exp(m_s - M) / L
  const int a_h0 = XM == 0 && a.apo ? kbase / a.aD : 0;
  const int a_nh = XM == 0 && a.apo ? (kbase + kw - 1) / a.aD - a_h0 + 1 : 0;
  if (XM == 0 && a.apo) {
    // 16 lanes per (row, head) pair, one split per lane (all (m, l) loads in
    // flight at once; a serial per-thread loop was latency-bound)
    const int sub = threadIdx.x & 15;
    for (int v = threadIdx.x >> 4; v < Mloc * a_nh; v += NW * 4) {
      const int m = v / a_nh, h = min(a_h0 + v % a_nh, a.aHq - 1);
      float* wr = aw + (size_t)v * (a.ans + 1);
      const int b = m / a.aTq, t = m % a.aTq;
      const int ns = min(a.ans, (a.alens[b] + 63) / 64);
      const float2* ml = (const float2*)a.aml + (((size_t)b * a.aHq + h) * a.aTq + t) * a.ans;
      float M = -INFINITY;
      for (int s = sub; s < ns; s += 16) M = fmaxf(M, ml[s].x);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 16));
      float L = 0.f;
      for (int s = sub; s < a.ans; s += 16) {
        float w = 0.f;
        if (s < ns) {
          const float2 q = ml[s];
          w = q.x == -INFINITY ? 0.f : __expf(q.x - M);
          L += w * q.y;
        }
        wr[s] = w;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) L += __shfl_xor(L, o, 16);
      if (sub == 0) wr[a.ans] = L > 0.f ? 1.f / L : 0.f;
    }
    __syncthreads();
  }


  // ---- residual-add + RMSNorm prologue (replaces the standalone norm launch):
  // h = rnd(rnd(acc) + res) exactly as add_rms_norm rounds it; every workgroup
  // needs 1/rms of the FULL row (16 KB f32 + 8 KB residual per row, L2-resident)
  __shared__ float ninv[16];
  auto rnd = [](float v) { return to_f32<T>(from_f32<T>(v)); };
  auto ni_h = [&](int m, int k, float* h) {
    const float4* p = (const float4*)(a.nacc + (size_t)m * a.K + k);
    const float4 p0 = p[0], p1 = p[1];
    const uint4 r = *(const uint4*)(a.nres + (size_t)m * a.K + k);
    const float av[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    const uint32_t rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
      h[2 * i] = rnd(rnd(av[2 * i]) + to_f32<T>((uint16_t)(rw[i] & 0xffff)));
      h[2 * i + 1] = rnd(rnd(av[2 * i + 1]) + to_f32<T>((uint16_t)(rw[i] >> 16)));
    }
  };
  if (defer) {                    // per-row sum of squares of this workgroup's K slice (staging below)
    if (threadIdx.x < 16) ninv[threadIdx.x] = 0.f;
    __syncthreads();
  }
  if (XM == 0 && a.nacc && !defer && !(ILLM_GEMV5_ABL & 2)) {
    if (threadIdx.x < 16) ninv[threadIdx.x] = 0.f;
    __syncthreads();
    const bool wres = a.nres_out != nullptr && blk.x == 0 && blk.y == 0;
    const int vpr = a.K / 8;
    uint16_t* xst = (uint16_t*)smem;
    const int ldxs = gemv5_x_ld(kw);
    // every row's loads of a thread's (up to HPF) slots are requested before
    // the first use: one L2 round trip per HPF slots instead of one per row
    // (the per-row loop serialised Mloc round trips: at batch 8 the norm-in
    // GLU cost 24.7 us vs 19.7 on a normed x, profiles/gemv5_defer_r3.jsonl)
    constexpr int HPF = 4;
    const int nthr = NW * 64, total = Mloc * vpr;
    for (int v0 = threadIdx.x; v0 < total; v0 += HPF * nthr) {
      float4 hp0[HPF], hp1[HPF];
      uint4 hr[HPF];
#pragma unroll
      for (int u = 0; u < HPF; u++) {
        const int vv = min(v0 + u * nthr, total - 1);
        const int m = vv / vpr, k = (vv % vpr) * 8;
        const float4* p = (const float4*)(a.nacc + (size_t)m * a.K + k);
        hp0[u] = p[0];
        hp1[u] = p[1];
        hr[u] = *(const uint4*)(a.nres + (size_t)m * a.K + k);
      }
#pragma unroll
      for (int u = 0; u < HPF; u++) {
        const int v = v0 + u * nthr;
        if (v >= total) break;                  // per 8-lane group when vpr % 8 == 0
        const int m = v / vpr, k = (v % vpr) * 8;
        const float av[8] = {hp0[u].x, hp0[u].y, hp0[u].z, hp0[u].w, hp1[u].x, hp1[u].y, hp1[u].z, hp1[u].w};
        const uint32_t rw[4] = {hr[u].x, hr[u].y, hr[u].z, hr[u].w};
        float h[8], ss = 0.f;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          h[2 * i] = rnd(rnd(av[2 * i]) + to_f32<T>((uint16_t)(rw[i] & 0xffff)));
          h[2 * i + 1] = rnd(rnd(av[2 * i + 1]) + to_f32<T>((uint16_t)(rw[i] >> 16)));
        }
#pragma unroll
        for (int i = 0; i < 8; i++) ss += h[i] * h[i];
        const uint4 hp =
            make_uint4(pack2<T>(h[0], h[1]), pack2<T>(h[2], h[3]), pack2<T>(h[4], h[5]), pack2<T>(h[6], h[7]));
        if (wres) *(uint4*)(a.nres_out + (size_t)m * a.K + k) = hp;
        // this workgroup's K slice: keep h (exact in T) in the x staging area,
        // the staging pass below normalises it in place (no second global read)
        const int kk = k - kbase;
        if (kk >= 0 && kk < kw) *(uint4*)(xst + m * ldxs + kk) = hp;
        if ((vpr & 7) == 0) {
          // the 8 lanes of an 8-vector group share the row: shuffle, one LDS add
          ss += __shfl_xor(ss, 1, 8);
          ss += __shfl_xor(ss, 2, 8);
          ss += __shfl_xor(ss, 4, 8);
          if ((v & 7) == 0) atomicAdd(&ninv[m], ss);
        } else {
          atomicAdd(&ninv[m], ss);
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < Mloc) ninv[threadIdx.x] = rsqrtf(ninv[threadIdx.x] / (float)a.K + a.neps);
    __syncthreads();
  }

  // ---- stage x[0:Mloc, kbase:kbase+kw] -> LDS in C
  const int vpr = kw / 8;
  // the staged value's LDS store and its per-(row, 64-block) sums: the 8
  // lanes of a block are 8 consecutive threads (vpr is a multiple of 16),
  // reduced with shuffles instead of a second LDS pass behind another barrier
  auto commit_x = [&](int v, uint4 val) {
    const int m = v / vpr, kk = (v % vpr) * 8;
    *(uint4*)(xs + m * ldx + kk) = val;
    const uint32_t sw[4] = {val.x, val.y, val.z, val.w};
    float bsum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) bsum += to_f32<C>((uint16_t)(sw[i] & 0xffff)) + to_f32<C>((uint16_t)(sw[i] >> 16));
    bsum += __shfl_xor(bsum, 1, 8);
    bsum += __shfl_xor(bsum, 2, 8);
    bsum += __shfl_xor(bsum, 4, 8);
    if ((v & 7) == 0) {
      const int blk = kk >> 6, nch = c1 - c0;
      float* rec = (float*)(sxs + m * nch + (blk >> 1));
      rec[blk & 1] = -OFF * bsum;
      rec[2 + (blk & 1)] = bsum;
    }
  };
  auto to_c = [](uint4 val) -> uint4 {
    if constexpr (!std::is_same<C, T>::value) {   // bf16 activations -> f16 (LUT formats)
      uint32_t w[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const float lo = fminf(fmaxf(bf16_to_f32(w[i] & 0xffff), -65504.f), 65504.f);
        const float hi = fminf(fmaxf(bf16_to_f32(w[i] >> 16), -65504.f), 65504.f);
        w[i] = pack2<F16>(lo, hi);
      }
      return make_uint4(w[0], w[1], w[2], w[3]);
    }
    return val;
  };
  if constexpr (XM == 2) {
    // deferred RMSNorm from the early registers (the generic branch below does
    // the same from global memory): h = rnd(rnd(acc) + res), x' = rnd(w * h),
    // the rows' sums of squares into ninv, grid column 0 writes the residual out
#pragma unroll
    for (int u = 0; u < XS; u++) {
      const int v = (int)threadIdx.x + u * NW * 64;
      if (v >= xtotal) break;                   // whole 8-lane groups (xvpr % 16 == 0)
      const int m = v / vpr, kk = (v % vpr) * 8;
      const float av[8] = {ea0[u].x, ea0[u].y, ea0[u].z, ea0[u].w, ea1[u].x, ea1[u].y, ea1[u].z, ea1[u].w};
      const uint32_t rw[4] = {er[u].x, er[u].y, er[u].z, er[u].w}, wv[4] = {ew[u].x, ew[u].y, ew[u].z, ew[u].w};
      float h[8], ssq = 0.f;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        h[2 * i] = rnd(rnd(av[2 * i]) + to_f32<T>((uint16_t)(rw[i] & 0xffff)));
        h[2 * i + 1] = rnd(rnd(av[2 * i + 1]) + to_f32<T>((uint16_t)(rw[i] >> 16)));
      }
#pragma unroll
      for (int i = 0; i < 8; i++) ssq += h[i] * h[i];
      ssq += __shfl_xor(ssq, 1, 8);
      ssq += __shfl_xor(ssq, 2, 8);
      ssq += __shfl_xor(ssq, 4, 8);
      if ((v & 7) == 0) atomicAdd(&ninv[m], ssq);
      if (a.nres_out && blk.x == 0)
        *(uint4*)(a.nres_out + (size_t)m * a.K + kbase + kk) =
            make_uint4(pack2<T>(h[0], h[1]), pack2<T>(h[2], h[3]), pack2<T>(h[4], h[5]), pack2<T>(h[6], h[7]));
      uint32_t o4[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        float w0 = to_f32<T>((uint16_t)(wv[i] & 0xffff)), w1 = to_f32<T>((uint16_t)(wv[i] >> 16));
        if (a.nunit) { w0 = rnd(1.f + w0); w1 = rnd(1.f + w1); }
        o4[i] = pack2<C>(rnd(w0 * h[2 * i]), rnd(w1 * h[2 * i + 1]));
      }
      commit_x(v, make_uint4(o4[0], o4[1], o4[2], o4[3]));
    }
  } else if constexpr (XM == 1) {
#pragma unroll
    for (int u = 0; u < XS; u++) {
      const int v = (int)threadIdx.x + u * NW * 64;
      if (v >= xtotal) break;
      commit_x(v, xr[u]);
    }
  } else if (dma_x) {
    // the row pieces were requested before the weight ring (top): wait for
    // them only -- every load issued later is one of this thread's ring loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // the per-(row, 64-block) sums from the staged rows (8 lanes per block)
    const int nthr = NW * 64, total = Mloc * vpr;
    for (int v = threadIdx.x; v < total; v += nthr) {
      const int m = v / vpr, kk = (v % vpr) * 8;
      const uint4 val = *(const uint4*)(xs + m * ldx + kk);
      const uint32_t sw[4] = {val.x, val.y, val.z, val.w};
      float bsum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; i++) bsum += to_f32<C>((uint16_t)(sw[i] & 0xffff)) + to_f32<C>((uint16_t)(sw[i] >> 16));
      bsum += __shfl_xor(bsum, 1, 8);
      bsum += __shfl_xor(bsum, 2, 8);
      bsum += __shfl_xor(bsum, 4, 8);
      if ((v & 7) == 0) {
        const int blk = kk >> 6, nch = c1 - c0;
        float* rec = (float*)(sxs + m * nch + (blk >> 1));
        rec[blk & 1] = -OFF * bsum;
        rec[2 + (blk & 1)] = bsum;
      }
    }
  } else if (XM == 0 && !(ILLM_GEMV5_ABL & 2) && plain_x) {
    // plain activations: every load of a thread's (up to XPF) staging slots is
    // requested before the first LDS store / shuffle reduction -- one L2 round
    // trip instead of one per slot (the loop form below serialised them:
    // ~3.8 us of a 19.9 us gate/up GEMV prologue at M = 8, 8 slots per thread,
    // profiles/gemv5_ablation2_r3.jsonl abl 1 vs 3)
    constexpr int XPF = 4;
    const int nthr = NW * 64, total = Mloc * vpr;
    {
      for (int v0 = threadIdx.x; v0 < total; v0 += XPF * nthr) {
        uint4 xv[XPF];
#pragma unroll
        for (int u = 0; u < XPF; u++) {
          const int vv = min(v0 + u * nthr, total - 1);
          const int m = vv / vpr, kk = (vv % vpr) * 8;
          xv[u] = kbase + kk < a.K ? *(const uint4*)(a.x + (size_t)xrow_of(m) * a.ldx + kbase + kk)
                                   : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < XPF; u++)
          if (v0 + u * nthr < total) commit_x(v0 + u * nthr, to_c(xv[u]));
      }
    }
  } else if (XM == 0 && !(ILLM_GEMV5_ABL & 2) && a.nacc && !defer && !a.apo && !a.xpart) {
    // norm-in: h (exact in T) is already in LDS from the prologue; x = w * rnd(h * inv).
    // The norm weight loads of a thread's XPF slots are requested together (the
    // generic loop below made each slot's weight load a round trip of its own:
    // Mloc x vpr / threads of them at batch 8)
    constexpr int XPF = 4;
    const int nthr = NW * 64, total = Mloc * vpr;
    for (int v0 = threadIdx.x; v0 < total; v0 += XPF * nthr) {
      uint4 wq[XPF];
#pragma unroll
      for (int u = 0; u < XPF; u++) {
        const int vv = min(v0 + u * nthr, total - 1);
        const int kk = (vv % vpr) * 8;
        wq[u] = kbase + kk < a.K ? *(const uint4*)(a.nweight + kbase + kk) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < XPF; u++) {
        const int v = v0 + u * nthr;
        if (v >= total) break;                  // whole 8-lane groups (vpr % 16 == 0)
        const int m = v / vpr, kk = (v % vpr) * 8;
        uint4 val = make_uint4(0, 0, 0, 0);
        if (kbase + kk < a.K) {
          const uint4 hq = *(const uint4*)(xs + m * ldx + kk);
          const uint32_t hw[4] = {hq.x, hq.y, hq.z, hq.w};
          const uint32_t wv[4] = {wq[u].x, wq[u].y, wq[u].z, wq[u].w};
          const float inv = ninv[m];
          uint32_t o4[4];
#pragma unroll
          for (int i = 0; i < 4; i++) {
            float w0 = to_f32<T>((uint16_t)(wv[i] & 0xffff)), w1 = to_f32<T>((uint16_t)(wv[i] >> 16));
            if (a.nunit) { w0 = rnd(1.f + w0); w1 = rnd(1.f + w1); }
            const float h0 = to_f32<T>((uint16_t)(hw[i] & 0xffff)), h1 = to_f32<T>((uint16_t)(hw[i] >> 16));
            float v0f = rnd(w0 * rnd(h0 * inv)), v1f = rnd(w1 * rnd(h1 * inv));
            if constexpr (!std::is_same<C, T>::value) {
              v0f = fminf(fmaxf(v0f, -65504.f), 65504.f);
              v1f = fminf(fmaxf(v1f, -65504.f), 65504.f);
            }
            o4[i] = pack2<C>(v0f, v1f);
          }
          val = make_uint4(o4[0], o4[1], o4[2], o4[3]);
        }
        commit_x(v, val);
      }
    }
  } else if (XM == 0 && !(ILLM_GEMV5_ABL & 2)) {
    for (int v = threadIdx.x; v < Mloc * vpr; v += NW * 64) {
      const int m = v / vpr, kk = (v % vpr) * 8;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (kbase + kk < a.K && a.apo) {
        // combine the flash-decoding partials of this 8-dim group (8 | D)
        const int k0 = kbase + kk, h = k0 / a.aD, d = k0 % a.aD;
        const int b = m / a.aTq, t = m % a.aTq;
        const float* wr = aw + (size_t)(m * a_nh + (h - a_h0)) * (a.ans + 1);
        const float* po = a.apo + ((((size_t)b * a.aHq + h) * a.aTq + t) * a.ans) * a.aD + d;
        float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // unconditional loads (a branch per split serialises them); an unused or
        // fully masked split (w == 0) holds unwritten bytes, so select, never multiply
#pragma unroll 4
        for (int s = 0; s < a.ans; s++) {
          const float w = wr[s];
          const float4 p0 = *(const float4*)(po + (size_t)s * a.aD), p1 = *(const float4*)(po + (size_t)s * a.aD + 4);
          const bool on = w != 0.f;
          o[0] += on ? w * p0.x : 0.f; o[1] += on ? w * p0.y : 0.f; o[2] += on ? w * p0.z : 0.f;
          o[3] += on ? w * p0.w : 0.f; o[4] += on ? w * p1.x : 0.f; o[5] += on ? w * p1.y : 0.f;
          o[6] += on ? w * p1.z : 0.f; o[7] += on ? w * p1.w : 0.f;
        }
        const float invL = wr[a.ans];
        uint32_t w4[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          // rounded to T: what the separate combine kernel would have written
          float v0 = to_f32<T>(from_f32<T>(o[2 * i] * invL)), v1 = to_f32<T>(from_f32<T>(o[2 * i + 1] * invL));
          if constexpr (std::is_same<C, F16>::value) {
            v0 = fminf(fmaxf(v0, -65504.f), 65504.f);
            v1 = fminf(fmaxf(v1, -65504.f), 65504.f);
          }
          w4[i] = pack2<C>(v0, v1);
        }
        val = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      } else if (kbase + kk < a.K && a.xpart) {
        // fused activation input: x = act(gate) * up from the gate/up GEMV's split-K slabs
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
        if (a.xpss) {              // deferred RMSNorm of the gate/up input: one scale per row
          const float sc = rsqrtf(a.xpss[xrow_of(m)] / (float)a.xpss_n + a.xpss_eps);
#pragma unroll
          for (int i = 0; i < 8; i++) { gv[i] *= sc; uv[i] *= sc; }
        }
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float o2[2];
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const float gg = gv[2 * i + j];
            // rounded to T: what the GLU epilogue would have written
            float act = to_f32<T>(from_f32<T>((a.act == 0 ? silu_f(gg) : gelu_tanh_f(gg)) * uv[2 * i + j]));
            if constexpr (std::is_same<C, F16>::value) act = fminf(fmaxf(act, -65504.f), 65504.f);
            o2[j] = act;
          }
          w[i] = pack2<C>(o2[0], o2[1]);
        }
        val = make_uint4(w[0], w[1], w[2], w[3]);
      } else if (kbase + kk < a.K && defer) {
        // deferred RMSNorm: h = rnd(rnd(acc) + res) of this slice, x' = rnd(w * h);
        // sum of squares per row -> ninv[m] (LDS), grid column 0 writes the residual out
        float h[8];
        ni_h(m, kbase + kk, h);
        float ssq = 0.f;
#pragma unroll
        for (int i = 0; i < 8; i++) ssq += h[i] * h[i];
        ssq += __shfl_xor(ssq, 1, 8);
        ssq += __shfl_xor(ssq, 2, 8);
        ssq += __shfl_xor(ssq, 4, 8);
        if ((v & 7) == 0) atomicAdd(&ninv[m], ssq);
        if (a.nres_out && blk.x == 0)
          *(uint4*)(a.nres_out + (size_t)m * a.K + kbase + kk) =
              make_uint4(pack2<T>(h[0], h[1]), pack2<T>(h[2], h[3]), pack2<T>(h[4], h[5]), pack2<T>(h[6], h[7]));
        const uint4 wq = *(const uint4*)(a.nweight + kbase + kk);
        const uint32_t wv[4] = {wq.x, wq.y, wq.z, wq.w};
        uint32_t o4[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float w0 = to_f32<T>((uint16_t)(wv[i] & 0xffff)), w1 = to_f32<T>((uint16_t)(wv[i] >> 16));
          if (a.nunit) { w0 = rnd(1.f + w0); w1 = rnd(1.f + w1); }
          float v0 = rnd(w0 * h[2 * i]), v1 = rnd(w1 * h[2 * i + 1]);
          if constexpr (!std::is_same<C, T>::value) {
            v0 = fminf(fmaxf(v0, -65504.f), 65504.f);
            v1 = fminf(fmaxf(v1, -65504.f), 65504.f);
          }
          o4[i] = pack2<C>(v0, v1);
        }
        val = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      } else if (kbase + kk < a.K && a.nacc) {
        // normalised residual stream: w * rnd(h * inv), rounded to T like the norm kernel's output
        float h[8];
        {
          const uint4 hq = *(const uint4*)(xs + m * ldx + kk);      // h of the prologue, exact in T
          const uint32_t hw[4] = {hq.x, hq.y, hq.z, hq.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            h[2 * i] = to_f32<T>((uint16_t)(hw[i] & 0xffff));
            h[2 * i + 1] = to_f32<T>((uint16_t)(hw[i] >> 16));
          }
        }
        const float inv = ninv[m];
        const uint4 wq = *(const uint4*)(a.nweight + kbase + kk);
        const uint32_t wv[4] = {wq.x, wq.y, wq.z, wq.w};
        uint32_t o4[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float w0 = to_f32<T>((uint16_t)(wv[i] & 0xffff)), w1 = to_f32<T>((uint16_t)(wv[i] >> 16));
          if (a.nunit) { w0 = rnd(1.f + w0); w1 = rnd(1.f + w1); }
          float v0 = rnd(w0 * rnd(h[2 * i] * inv)), v1 = rnd(w1 * rnd(h[2 * i + 1] * inv));
          if constexpr (!std::is_same<C, T>::value) {
            v0 = fminf(fmaxf(v0, -65504.f), 65504.f);
            v1 = fminf(fmaxf(v1, -65504.f), 65504.f);
          }
          o4[i] = pack2<C>(v0, v1);
        }
        val = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      } else if (kbase + kk < a.K) {
        val = to_c(*(const uint4*)(a.x + (size_t)xrow_of(m) * a.ldx + kbase + kk));
      }
      commit_x(v, val);
    }
  }
  __syncthreads();
  ILLM_GEMV5_STAMP(1);
#ifdef ILLM_GEMV5_DUMP
  ILLM_GEMV5_DUMP();   // debug hook (tools/probe/xm_check.hip: the staged x of workgroup 0)
#endif
  if (defer) {
    if constexpr (EPI == EPI_GLU) {
      // full K staged here: the row scale is known locally (applied before the activation)
      __syncthreads();
      if (threadIdx.x < Mloc) ninv[threadIdx.x] = rsqrtf(ninv[threadIdx.x] / (float)a.K + a.neps);
      __syncthreads();
    } else if (blk.x == 0 && threadIdx.x < Mloc && a.nss) {
      __hip_atomic_fetch_add(a.nss + threadIdx.x, ninv[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }

  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (wave_on) {
    const int mrow = min(r16, Mloc - 1);          // unused columns read a valid row (no masking)
    const uint16_t* xrow = xs + mrow * ldx + 8 * g;
    const float4* srow = sxs + mrow * (c1 - c0);
    const uint32_t mask_s = a.nib_mask, magic_v = a.nib_magic;

    auto compute_chunk = [&](const Chunk& ch, int c) {
      if constexpr ((ILLM_GEMV5_ABL & 1) != 0) {
#pragma unroll
        for (int t = 0; t < TPW; t++)        // every tile folds into acc[0]: no load is dead
          acc[0][0] += __uint_as_float((ch.q[t][0].x ^ ch.q[t][0].y ^ ch.q[t][0].z ^ ch.q[t][0].w ^
                                        (SCL ? scl[t].x : ch.sc[t].x)) & 0x3fffffu);
        return;
      }
      const uint16_t* xc = xrow + (c - c0) * 128;
      uint4 B[4];
#pragma unroll
      for (int s = 0; s < 4; s++) B[s] = *(const uint4*)(xc + 32 * s);
      const float4 sx = srow[c - c0];
      uint4 scv[TPW], mnv[TPW];
      if constexpr (SCL) {
        // one window covers the wave's chunk range (launch guarantees <= 16 chunks:
        // a reload here would make hipcc wait for every load in flight)
        const int src = (16 * g + (c - sw0)) * 4;
#pragma unroll
        for (int t = 0; t < TPW; t++) {
          scv[t] = make_uint4(__builtin_amdgcn_ds_bpermute(src, scl[t].x), __builtin_amdgcn_ds_bpermute(src, scl[t].y),
                              __builtin_amdgcn_ds_bpermute(src, scl[t].z), __builtin_amdgcn_ds_bpermute(src, scl[t].w));
          if constexpr (HASMIN)
            mnv[t] = make_uint4(__builtin_amdgcn_ds_bpermute(src, mnl[t].x), __builtin_amdgcn_ds_bpermute(src, mnl[t].y),
                                __builtin_amdgcn_ds_bpermute(src, mnl[t].z), __builtin_amdgcn_ds_bpermute(src, mnl[t].w));
        }
      } else {
#pragma unroll
        for (int t = 0; t < TPW; t++) {
          scv[t] = ch.sc[t];
          if constexpr (HASMIN) mnv[t] = ch.mn[t];
        }
      }
#pragma unroll
      for (int t = 0; t < TPW; t++) {
#pragma unroll
        for (int blk = 0; blk < 2; blk++) {
          f32x4 P = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ss = 0; ss < 2; ss++) {
            const int s = blk * 2 + ss;
            uint4 A;
            if constexpr (BITS == 4) {
              const uint4& q0 = ch.q[t][0];
              const uint32_t w = s == 0 ? q0.x : (s == 1 ? q0.y : (s == 2 ? q0.z : q0.w));
              A = raw_a4<DK, C>(w, mask_s, magic_v, lut2);
            } else {
              const uint4& qq = ch.q[t][blk];
              A = ss == 0 ? raw_a8<DK, C>(qq.x, qq.y) : raw_a8<DK, C>(qq.z, qq.w);
            }
            P = mfma16<C>(A, B[s], P);
          }
          const float nsx = blk == 0 ? sx.x : sx.y;
          const float sxv = blk == 0 ? sx.z : sx.w;
          const uint32_t scw[4] = {scv[t].x, scv[t].y, scv[t].z, scv[t].w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const float d = f16_to_f32((uint16_t)(scw[i] >> (16 * blk)));
            if constexpr (OFF != 0.f) acc[t][i] = __builtin_fmaf(d, P[i] + nsx, acc[t][i]);
            else acc[t][i] = __builtin_fmaf(d, P[i], acc[t][i]);
            if constexpr (HASMIN) {
              const uint32_t mnw[4] = {mnv[t].x, mnv[t].y, mnv[t].z, mnv[t].w};
              acc[t][i] = __builtin_fmaf(f16_to_f32((uint16_t)(mnw[i] >> (16 * blk))), sxv, acc[t][i]);
            }
          }
        }
      }
    };

    // steady state: unconditional clamped loads (hipcc keeps counted vmcnt)
    const int c1u = __builtin_amdgcn_readfirstlane(wc1);
    int c = __builtin_amdgcn_readfirstlane(wc0);
    for (; c + 2 * PF <= c1u; c += PF) {
#pragma unroll
      for (int u = 0; u < PF; u++) {
        compute_chunk(ring[u], c + u);
        load_chunk(ring[u], c + u + PF);
      }
    }
#pragma unroll
    for (int u = 0; u < PF; u++) {
      if (c + u < c1u) compute_chunk(ring[u], c + u);
      if (PF < 8 || c + u + PF < c1u) load_chunk(ring[u], c + u + PF);   // PF 8: no clamped re-loads
    }
    c += PF;
#pragma unroll
    for (int u = 0; u < PF; u++)
      if (c + u < c1u) compute_chunk(ring[u], c + u);
  }

  ILLM_GEMV5_STAMP(2);
  if constexpr ((ILLM_GEMV5_ABL & 4) != 0) {
    if (acc[0][0] == 1234.5f) ((float*)a.out)[threadIdx.x] = acc[0][1];
    return;
  }
  // ---- reduce the KW k-parts of each tile group through LDS
  constexpr bool ATOMIC_T = EPI == EPI_ATOMIC && !MOE;   // block-transposed atomic epilogue
  if constexpr (KW > 1) {
#pragma unroll
    for (int t = 0; t < TPW; t++)
      red[(wave * TPW + t) * 64 + lane] = make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
    __syncthreads();
    if (!ATOMIC_T && kp != 0) return;
    if (kp == 0) {
#pragma unroll
      for (int t = 0; t < TPW; t++) {
#pragma unroll
        for (int j = 1; j < KW; j++) {
          const float4 v = red[((wave + j) * TPW + t) * 64 + lane];
          acc[t][0] += v.x; acc[t][1] += v.y; acc[t][2] += v.z; acc[t][3] += v.w;
        }
      }
    }
  }
  if constexpr (ATOMIC_T) {
    // split-K f32 atomics, one row segment per wave instruction: the
    // workgroup's [Mloc][TG * TPW * 16] block goes through LDS so consecutive
    // lanes add to consecutive columns of ONE row (a lane-per-(row, 4 cols)
    // pattern spreads each instruction over Mloc rows; measured ~1.4x the
    // slab-store cost at M = 8 on MI355X).  The staging reuses `red`.
    constexpr int NTL = TG * TPW;
    constexpr int NC = NTL * 16;                       // columns per workgroup (<= 128)
    float* tbuf = (float*)red;                         // Mloc * NC floats <= 8 KiB
    __syncthreads();                                   // KW partners done reading red
    if (kp == 0 && tile0 < NT && r16 < Mloc) {
#pragma unroll
      for (int t = 0; t < TPW; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) tbuf[r16 * NC + (tg * TPW + t) * 16 + 4 * g + i] = acc[t][i];
    }
    __syncthreads();
    const int nb = blk.x * NC;
    float* ws = (float*)a.out;
    for (int v = threadIdx.x; v < Mloc * NC; v += NW * 64) {
      const int m = v / NC, n = nb + v % NC;
      if (n < a.N) {
        float val = tbuf[v];
        if (a.rcs != nullptr && n < a.rcols) {
          // rotate_half RoPE of this workgroup's partial (partner column in the
          // same head, same LDS row); cos/sin rounded to T as HF casts them
          const int half = a.rD >> 1, d = n % a.rD, i = d % half;
          const float2 cs = ((const float2*)a.rcs)[(size_t)a.rpos[m] * half + i];
          const float c = to_f32<T>(from_f32<T>(cs.x)), sn = to_f32<T>(from_f32<T>(cs.y));
          const float pv = tbuf[d < half ? v + half : v - half];
          val = d < half ? val * c - pv * sn : val * c + pv * sn;
        }
        __hip_atomic_fetch_add(ws + (size_t)m * a.N + n, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    ILLM_GEMV5_STAMP(3);
    if (a.lctr != nullptr) gemv5_norm_out<T>(a, blk, Mloc, nb, NC, NW * 64);
    return;
  }
  if (tile0 >= NT) return;

  // ---- epilogue: lane holds rows 16*tile + 4g + i, column r16
  if (r16 >= Mloc) return;
  const int m = orow_of(r16);
  if constexpr (EPI == EPI_GLU) {
    float o[4];
    const float rs = defer ? ninv[r16]
                           : (a.xpss != nullptr && a.xpart == nullptr ? rsqrtf(xss_raw / (float)a.xpss_n + a.xpss_eps)
                                                                      : 1.f);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const float gv = acc[0][i] * rs, uv = acc[TPW - 1][i] * rs;
      o[i] = (a.act == 0 ? silu_f(gv) : gelu_tanh_f(gv)) * uv;
    }
    const int n0 = (tile0 / 2) * 16 + 4 * g;
    if (n0 < a.N) {
      uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n0;
      if (n0 + 3 < a.N) *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
      else for (int i = 0; i < 4 && n0 + i < a.N; i++) y[i] = from_f32<T>(o[i]);
    }
    ILLM_GEMV5_STAMP(3);
  } else {
    float abest = -INFINITY;         // argmax partial (EPI_STORE + a.amax)
    int abi = 0x7fffffff;
#pragma unroll
    for (int t = 0; t < TPW; t++) {
      const int n0 = (tile0 + t) * 16 + 4 * g;
      if (tile0 + t >= NT || n0 >= a.N) continue;
      float o[4] = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
      if constexpr (EPI == EPI_ATOMIC) {
        int orow = m;
        if constexpr (MOE) {
          if (a.moe_w) {            // routing-weighted combine straight into the token's row
            const float rw = a.moe_w[m];
#pragma unroll
            for (int i = 0; i < 4; i++) o[i] *= rw;
            orow = m / a.moe_odiv;
          }
        }
        float* ws = (float*)a.out + (size_t)orow * a.N + n0;
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (n0 + i < a.N) __hip_atomic_fetch_add(ws + i, o[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if constexpr (EPI == EPI_PARTIAL) {
        float* ws = (float*)a.out + ((size_t)blk.y * a.M + m) * a.N + n0;
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
        if constexpr (EPI == EPI_STORE && !MOE) {
          if (a.amax) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const float v = to_f32<T>(from_f32<T>(o[i]));   // the stored logit
              if (n0 + i < a.N && v > abest) { abest = v; abi = n0 + i; }
            }
          }
        }
      }
    }
    if constexpr (EPI == EPI_STORE && !MOE) {
      if (a.amax) {
        // the 4 k-groups of this row hold 4 disjoint column sets (first index on ties)
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) {
          const float ov = __shfl_xor(abest, off, 64);
          const int oi = __shfl_xor(abi, off, 64);
          if (ov > abest || (ov == abest && oi < abi)) { abest = ov; abi = oi; }
        }
        if (g == 0) a.amax[((size_t)blk.x * TG + tg) * a.M + m] = make_float2(abest, __int_as_float(abi));
      }
    }
  }
}

template <int DK, typename T, int EPI, int TPW, int KW, bool MOE, int NW, int PF = 4, bool SCL = ILLM_GEMV5_SCL != 0,
          int XM = 0, int XS = 1>
__global__ void __launch_bounds__(NW * 64, ILLM_GEMV5_MINW) lowbit_gemv5_kernel(const GemvArgs a) {
  gemv5_body<DK, T, EPI, TPW, KW, MOE, NW, PF, SCL, XM, XS>(
      a, G5Blk{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.x, (int)gridDim.y, (int)gridDim.z});
}

// launch helper.  A launch over 64 KiB of dynamic LDS first raises the
// kernel's limit to what it asks for (per kernel: every instantiation has one
// function type, so a static flag in this template would cover only the first
// kernel launched); a refused request is cleared so that it does not surface
// as a later op's error.  ILLM_GEMV5_TRACE=1 prints each launch.
template <typename K>
inline void launch5(K kern, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  if (shmem > 64 * 1024) {
    static std::mutex mu;
    static std::unordered_map<const void*, size_t> lim;
    std::lock_guard<std::mutex> g(mu);
    size_t& l = lim[(const void*)kern];
    if (l < shmem) {
      if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem) == hipSuccess)
        l = shmem;
      else
        (void)hipGetLastError();
    }
  }
  static const bool trace = getenv("ILLM_GEMV5_TRACE") != nullptr;
  if (trace)
    fprintf(stderr, "[gemv5] kern=%p M=%d N=%d K=%d grid=%u,%u,%u nw=%d lds=%zu\n", (const void*)kern, a.M, a.N, a.K,
            grid.x, grid.y, grid.z, a.nw, shmem);
  hipLaunchKernelGGL(kern, grid, dim3(64 * (a.nw == 8 ? 8 : 4)), shmem, st, a);
}

// chunks in flight per wave.  The shared scale window would fit 8 in the
// ring VGPRs of 4, but 8 measured slower on MI355X at every decode shape
// (profiles/gemv5_scl_r3.jsonl: qkv M=1 8.9 vs 6.1 us, GLU 23.0 vs 17.6);
// with 4 the window only pays for the two-tile GLU launch (M=1 17.1 vs 17.6,
// deferred-norm 18.0 vs 19.0 us), so that is the one launch that takes it
#ifndef ILLM_GEMV5_PFD
#define ILLM_GEMV5_PFD 4
#endif
template <int DK, typename T, int KW, bool MOE, int NW, bool S>
inline void launch5_epi_s(int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  constexpr int PFD = S ? ILLM_GEMV5_PFD : 4;
  // all loads of a short split-K slice up front (decode projections: 8 chunks)
  const bool pf8 = a.pf8 && !MOE && KW == 1 && a.cpk > 0 && a.cpk <= 8;
  if (epi == EPI_STORE) launch5(lowbit_gemv5_kernel<DK, T, EPI_STORE, 1, KW, MOE, NW, PFD, S>, grid, shmem, a, st);
  else if (epi == EPI_PARTIAL) {
    if (pf8) launch5(lowbit_gemv5_kernel<DK, T, EPI_PARTIAL, 1, KW, MOE, NW, 8, S>, grid, shmem, a, st);
    else launch5(lowbit_gemv5_kernel<DK, T, EPI_PARTIAL, 1, KW, MOE, NW, PFD, S>, grid, shmem, a, st);
  } else if (epi == EPI_ATOMIC) {
    if (pf8) launch5(lowbit_gemv5_kernel<DK, T, EPI_ATOMIC, 1, KW, MOE, NW, 8, S>, grid, shmem, a, st);
    else launch5(lowbit_gemv5_kernel<DK, T, EPI_ATOMIC, 1, KW, MOE, NW, PFD, S>, grid, shmem, a, st);
  } else launch5(lowbit_gemv5_kernel<DK, T, EPI_GLU, 2, KW, MOE, NW, PFD, S>, grid, shmem, a, st);
}

template <int DK, typename T, int KW, bool MOE, int NW>
inline void launch5_epi(int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  // the shared scale window holds 16 chunks: longer per-wave ranges keep the
  // per-lane scale words
  const int cpk = a.cpk > 0 ? a.cpk : (a.KC + (int)grid.y - 1) / (int)grid.y;
  if (ILLM_GEMV5_SCL && epi == EPI_GLU && (cpk + KW - 1) / KW <= 16)
    return launch5(lowbit_gemv5_kernel<DK, T, EPI_GLU, 2, KW, MOE, NW, ILLM_GEMV5_PFD, true>, grid, shmem, a, st);
  return launch5_epi_s<DK, T, KW, MOE, NW, false>(epi, grid, shmem, a, st);
}

// the XM 1 / 2 instantiations (x or the deferred-norm inputs in registers
// ahead of the weight ring): the decode hot path -- sym_int4, bf16, whole K
// chunks -- for the geometries plan5 picks there.  Per launch at Llama-3-8B
// decode shapes (tools/probe/gemv5_probe.hip, profiles/gemv5_xm_forms_r6.txt):
// o 5.3 -> 4.4 us, qkv 6.0 -> 5.4, down 8.8 -> 8.2, gate/up B=8 18.6 -> 16.2.
// Not enabled by default (ILLM_GEMV5_XM_RT below): some forms compute wrong
// outputs, with and without -amdgpu-mfma-vgpr-form.
#ifndef ILLM_GEMV5_XM
#define ILLM_GEMV5_XM ILLM_GEMV5_EARLYX
#endif
// The XM kernels are instantiated in their own translation unit
// (gemv_int4_xm.hip, built without -amdgpu-mfma-vgpr-form; the generic kernels
// keep the flag): launch5_xm_int4s is defined there, or here when
// ILLM_GEMV5_XM_IMPL is set (that TU, the standalone probes).
bool launch5_xm_int4s(int kw, int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st);

template <int DK, typename T, bool MOE>
inline bool launch5_xm(int kw, int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  if constexpr (DK != DK_INT4S || !std::is_same<T, BF16>::value || MOE || !ILLM_GEMV5_XM) {
    return false;
  } else {
    return launch5_xm_int4s(kw, epi, grid, shmem, a, st);
  }
}

#ifdef ILLM_GEMV5_XM_IMPL
bool launch5_xm_int4s(int kw, int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  constexpr int DK = DK_INT4S;
  using T = BF16;
  {
    // ILLM_GEMV5_XM_RT (run time): 0 = generic kernels only, 1 = XM 1 only, 2 (default) = XM 1 and 2.
    // Only the forms that tools/probe/xm_check.hip (random inputs, each form against the
    // generic kernel, three repeats) found exact are taken: split-K forms whose wave range
    // never reaches the steady-state ring loop (cpk < 2 PF; the decode split-K plans: 4-7
    // chunks), and the 8-slot GLU form.  Wrong outputs were found in the others --
    // split-K forms once the ring is refilled (run-to-run different) and the 2-slot
    // GLU form at 4 waves (deterministic) -- and with -amdgpu-mfma-vgpr-form in more
    // (profiles/gemv5_xm_forms_r6.txt); gemv_int4.hip is built without that flag.
    static const int rt = getenv("ILLM_GEMV5_XM_RT") ? atoi(getenv("ILLM_GEMV5_XM_RT")) : 2;
    if (rt <= 0 || a.apo != nullptr || a.xpart != nullptr || a.K % 128 != 0 || a.pf8 || kw > 2) return false;
    const int cpk = a.cpk > 0 ? a.cpk : (a.KC + (int)grid.y - 1) / (int)grid.y;
    const int nthr = a.nw == 8 ? 512 : 256;
    const int slots = (a.M * cpk * 16 + nthr - 1) / nthr;     // 16-B x vectors per thread
    const bool w8 = a.nw == 8;
    static const bool trace = getenv("ILLM_GEMV5_TRACE") != nullptr;
#define ILLM_XM_LAUNCH(EPI_, TPW_, KW_, PF_, SCL_, XM_, XS_)                                                  \
    do {                                                                                                      \
      if (trace) fprintf(stderr, "[gemv5] XM %d XS %d epi %d slots %d cpk %d\n", XM_, XS_, EPI_, slots, cpk); \
      if (w8) launch5(lowbit_gemv5_kernel<DK, T, EPI_, TPW_, KW_, false, 8, PF_, SCL_, XM_, XS_>, grid, shmem, a, st); \
      else launch5(lowbit_gemv5_kernel<DK, T, EPI_, TPW_, KW_, false, 4, PF_, SCL_, XM_, XS_>, grid, shmem, a, st);    \
      return true;                                                                                            \
    } while (0)
    const bool glu_ok = kw == 2 && ILLM_GEMV5_SCL && (cpk + 1) / 2 <= 16;
    const bool atomic_ok = epi == EPI_ATOMIC && kw == 1 && cpk < 2 * 4;      // PF 4: no ring refill loop
    if (a.x == nullptr && a.nacc != nullptr && a.ndefer != 0) {
      // XM 2: deferred-norm input (decode qkv).  The 8-slot gate/up form (ILLM_GEMV5_XM_RT=3)
      // measured slower at batch 1: 1.594-1.597 vs 1.569-1.577 ms (profiles/xm2_glu_ab_r6.jsonl)
      if (rt < 2) return false;
      if (atomic_ok && slots <= 1) ILLM_XM_LAUNCH(EPI_ATOMIC, 1, 1, 4, false, 2, 1);
      if (atomic_ok && slots <= 2) ILLM_XM_LAUNCH(EPI_ATOMIC, 1, 1, 4, false, 2, 2);
      if (epi == EPI_GLU && glu_ok && slots <= 8 && rt >= 3) ILLM_XM_LAUNCH(EPI_GLU, 2, 2, ILLM_GEMV5_PFD, true, 2, 8);
      return false;
    }
    if (a.x == nullptr || a.nacc != nullptr) return false;
    if (atomic_ok && slots <= 1) ILLM_XM_LAUNCH(EPI_ATOMIC, 1, 1, 4, false, 1, 1);
    if (atomic_ok && slots <= 2) ILLM_XM_LAUNCH(EPI_ATOMIC, 1, 1, 4, false, 1, 2);
    if (epi == EPI_GLU && glu_ok && slots <= 8) ILLM_XM_LAUNCH(EPI_GLU, 2, 2, ILLM_GEMV5_PFD, true, 1, 8);
#undef ILLM_XM_LAUNCH
    return false;
  }
}
#endif  // ILLM_GEMV5_XM_IMPL

template <int DK, typename T, bool MOE>
inline void launch5_kw(int kw, int epi, dim3 grid, size_t shmem, const GemvArgs& a0, hipStream_t st) {
  using C = typename std::conditional<DK == DK_LUT4, F16, T>::type;
  GemvArgs a = a0;
  a.nib_mask = 0x000F000Fu;
  a.nib_magic = Raw<C>::k4;
  if (launch5_xm<DK, T, MOE>(kw, epi, grid, shmem, a, st)) return;
  // workgroup size: 4 or 8 waves (a.nw); 8 shares one LDS copy of x among
  // twice the tiles (the x-staging cost of kw > 1 at larger M)
  if (a.nw == 8) {
    if (kw == 1) launch5_epi<DK, T, 1, MOE, 8>(epi, grid, shmem, a, st);
    else if (kw == 2) launch5_epi<DK, T, 2, MOE, 8>(epi, grid, shmem, a, st);
    else launch5_epi<DK, T, 4, MOE, 8>(epi, grid, shmem, a, st);
  } else {
    if (kw == 1) launch5_epi<DK, T, 1, MOE, 4>(epi, grid, shmem, a, st);
    else if (kw == 2) launch5_epi<DK, T, 2, MOE, 4>(epi, grid, shmem, a, st);
    else launch5_epi<DK, T, 4, MOE, 4>(epi, grid, shmem, a, st);
  }
}

// grid.x = workgroups of (nw / kw) tile groups (GLU: tile pairs), grid.y = split-K
template <int DK>
void launch_gemv5_dk(bool bf16, int kw, int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st) {
  const bool moe = a.moe_off != nullptr;
  if (moe && epi == EPI_STORE) epi = EPI_PARTIAL;   // grouped launches write slabs or GLU rows
  if (bf16) {
    if (moe) launch5_kw<DK, BF16, true>(kw, epi, grid, shmem, a, st);
    else launch5_kw<DK, BF16, false>(kw, epi, grid, shmem, a, st);
  } else {
    if (moe) launch5_kw<DK, F16, true>(kw, epi, grid, shmem, a, st);
    else launch5_kw<DK, F16, false>(kw, epi, grid, shmem, a, st);
  }
}

}  // namespace illm
