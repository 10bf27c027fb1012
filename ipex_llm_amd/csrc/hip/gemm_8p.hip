// Dense bf16 NT GEMM, y[M, N] = x[M, K] @ w[N, K]^T (+ bias), on the gfx950
// 256 x 256 "8-phase" schedule (cdna_hip_programming.md §5, 'The 256² 8-phase
// template'): the compute-bound projection / LM-head / LoRA-base GEMMs of
// prefill and training (reference: the dense fp16/bf16 paths of
// SRC/transformers/low_bit_linear.py:780-860 FP16Linear / BF16Linear, which
// the reference runs on oneDNN).
//
// Structure (one 512-thread workgroup = 8 waves as 2 (m) x 4 (n), 256 x 256
// output tile, each wave 128 (m) x 64 (n) = 8 x 4 MFMA tiles of 16 x 16):
//   * K is walked in 64-deep tiles; every tile is split into four
//     half-tiles (A0/A1: the first / second 64 rows of each wave-row's 128
//     x rows, B0/B1: the first / second 32 of each wave-column's 64 w rows),
//     each 128 rows x 128 B, staged global -> LDS by LDS-DMA
//     (buffer_load ... lds, 16 B per lane, two per lane per half-tile) into
//     one of two buffers -- no VGPR round trip, no staging instructions;
//   * four phases per K-tile, one C quadrant each: (mh0, nh0) (mh1, nh0)
//     (mh0, nh1) (mh1, nh1); fragments are read once per tile (A halves kept
//     in registers across phases, the B half re-read once): 24 ds_read_b128
//     per wave per tile, the minimum;
//   * every phase issues ONE half-tile for a future tile (A1(u+1), B1(u+1),
//     A0(u+2), B0(u+2) in phases 0..3 of tile u -- each two or more phases
//     after that LDS half was last read), then waits with a COUNTED
//     `s_waitcnt vmcnt(8)` (four half-tiles stay in flight across the
//     barriers, never drained in the loop), raw s_barrier, lgkmcnt(0),
//     s_setprio(1) around the 16-MFMA cluster, s_barrier;
//   * the LDS images are XOR-swizzled on the 16-B chunk ((row >> 1) & 7),
//     applied to the per-lane SOURCE address of the LDS-DMA (its LDS side is
//     lane-linear) and to the fragment reads: the 16 rows of a 16-lane read
//     group land on 16 distinct bank slots;
//   * out = C^T orientation (w rows are the MFMA A operand), so a lane holds
//     4 consecutive output columns of one row: 8-byte stores;
//   * the two wave-rows run STAGGERED by one barrier (wave-row 1 enters the
//     loop one barrier late): on every SIMD one wave issues its MFMA cluster
//     while the other reads fragments / issues DMA, so the matrix pipe does
//     not idle through the read-and-wait half of each phase;
//   * XCD-aware block order (bijective remap) with 4 m-blocks per group, so
//     concurrently running blocks of one XCD share x and w panels in its L2.
// All LDS lives in ONE __shared__ array (a second LDS object can make hipcc
// drain vmcnt before every ds_read, §5 item 4(a)).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../common/quant_block.h"
#include "gemv_args.h"
#include "illm_device.h"
#include "kernels_g8.h"
#include "mfg_common.h"

namespace illm {
namespace g8 {

constexpr int ROWB = 128;               // bytes per LDS image row (64 bf16)
constexpr int IMG = 256 * ROWB;         // one operand image, 32 KB
constexpr int BUFB = 2 * IMG;           // A + B images of one K-tile
constexpr int LDS_BYTES = 2 * BUFB;     // two buffers, 128 KB

typedef int32_t g8_rsrc __attribute__((ext_vector_type(4)));

// buffer descriptor: base, num_records = bytes (reads past it return 0)
__device__ __forceinline__ g8_rsrc make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)(uintptr_t)base;
  return g8_rsrc{(int32_t)(uint32_t)p, (int32_t)((uint32_t)(p >> 32) & 0xffffu), (int32_t)bytes, 0x00020000};
}

// 16-B LDS-DMA per lane (LDS side: wave-uniform base + lane * 16).  Issued
// from inline asm ON PURPOSE: hipcc cannot tell these LDS writes from the
// fragment ds_reads of the other buffer and would otherwise drain vmcnt(0)
// before every phase's reads (measured in the .s) -- the counted
// `s_waitcnt vmcnt(N)` + barrier below are the only ordering they need.
__device__ __forceinline__ void dma16(const g8_rsrc& rs, const uint8_t* lds, uint32_t voff, int soff) {
  const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)lds);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(la), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
}

// image row of half-tile h, half-tile row q in [0, 128)
__device__ __forceinline__ int a_row(int h, int q) { return (q < 64 ? q : q + 64) + 64 * h; }
__device__ __forceinline__ int b_row(int h, int q) { return (q >> 5) * 64 + 32 * h + (q & 31); }

__device__ __forceinline__ void wait_vm8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// LDS map.  Dense: [A buf0 | B buf0 | A buf1 | B buf1] (128 KB).  Low-bit:
// [A buf0 | A buf1 | B (single) | codes ring 2 x 16 KB | scales ring 2 x 1 KB |
//  LUT 2 KB] (132 KB) -- the B image is decoded just in time, so one buffer.
template <int DK> struct G8Lds;
template <> struct G8Lds<-1> {
  static constexpr int A0 = 0, ASTR = BUFB, B0 = IMG, BSTR = BUFB, BYTES = LDS_BYTES;
};
template <> struct G8Lds<-2> : G8Lds<-1> {};     // fp8 (e4m3 w): the dense layout, 128 k per 128-B row
template <> struct G8Lds<-3> : G8Lds<-1> {};     // fp8 (e5m2 w)
template <int DK> struct G8Lds {
  static constexpr int A0 = 0, ASTR = IMG, B0 = 2 * IMG, BSTR = 0;
  static constexpr int CODES = 3 * IMG, SCALES = CODES + 2 * 16384, LUT = SCALES + 2 * 1024, BYTES = LUT + 2048;
};

// 8 weights of one 4-bit code dword -> 8 bf16 (one ds_write_b128 chunk).
// INT4S nibble order = the pair order of lowbit_decode.h ((u >> 4 i) & 0x000F000F
// = elements 2 i, 2 i + 1); (128 + q) from the bf16 exponent trick, then
// (q - 8) d formed exactly in f32 and rounded once to bf16 -- bit-identical
// to dequantize-to-bf16.  LUT4: byte j = elements 2 j (low nibble), 2 j + 1.
template <int DK>
__device__ __forceinline__ uint4 dec8_bf16(uint32_t u, float d, float md, const float2* lut) {
  uint32_t o[4];
  if constexpr (DK == DK_INT4S) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t q = ((u >> (4 * i)) & 0x000F000Fu) | 0x43004300u;
      o[i] = pack2<BF16>(fmaf(__uint_as_float(q << 16), d, md), fmaf(__uint_as_float(q & 0xffff0000u), d, md));
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const float2 l = lut[(u >> (8 * j)) & 0xff];
      o[j] = pack2<BF16>(l.x * d, l.y * d);
    }
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

typedef int32_t g8_i32x8 __attribute__((ext_vector_type(8)));

template <int DK, int G8S = 0>
__global__ void __launch_bounds__(512) gemm8p_kernel(const G8Args a) {
  constexpr bool DENSE = DK < 0;          // both operands staged by LDS-DMA (bf16 or fp8)
  constexpr bool FP8 = DK <= G8_FP8;      // 128 k per K-tile, 16x16x128 block-scaled fp8 MFMA
  constexpr int FMTW = DK == G8_FP8 - 1 ? 1 : 0;   // w operand format (0 e4m3, 1 e5m2): a compile-time
                                                   // constant -- a runtime select made hipcc issue both MFMAs
  using L = G8Lds<DK>;
  __shared__ __attribute__((aligned(1024))) uint8_t smem[L::BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int g = lane >> 4, r16 = lane & 15;

  // ---- block -> (m-block, n-block): XCD remap, then groups of 4 m-blocks
  const int MB = (a.M + 255) / 256, NB = (a.N + 255) / 256;
  const int S = DENSE && a.ksplit > 1 ? a.ksplit : 1;
  const int total = MB * NB * S;
  // split-K: the S workgroups of one output tile are adjacent ids (one XCD's
  // L2 serves their shared nothing but keeps the grouping of the tiles intact)
  const int id0 = mfg::xcd_remap((int)blockIdx.x, total);
  const int ks = id0 % S, id = id0 / S;
  const int GM = a.gm > 0 ? a.gm : 4;
  const int per_group = GM * NB;
  const int grp = id / per_group, rem = id % per_group;
  const int gm = min(GM, MB - grp * GM);
  const int mb = grp * GM + rem % gm, nb = rem / gm;
  const int m0 = mb * 256, n0 = nb * 256;
  const int Tall = FP8 ? a.K / 128 : a.K / 64;
  const int kt0 = (int)((int64_t)Tall * ks / S);
  const int T = (int)((int64_t)Tall * (ks + 1) / S) - kt0;   // this workgroup's K-tiles
  constexpr int ES = FP8 ? 1 : 2;         // element bytes

  // ---- per-lane LDS-DMA source offsets (bytes; + k-tile via soff) for the
  // two 16-B pieces of each half-tile, and the wave-uniform LDS row bases
  uint32_t xo[2][2], wo[2][2];
  int ar0[2][2], br0[2][2];
#pragma unroll
  for (int h = 0; h < 2; h++)
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int q0 = (i * 8 + wave) * 8, q = q0 + (lane >> 3), c = lane & 7;
      const int ra = a_row(h, q), rb = b_row(h, q);
      ar0[h][i] = a_row(h, q0);
      br0[h][i] = b_row(h, q0);
      xo[h][i] = (uint32_t)(m0 + ra) * (uint32_t)a.ldx * ES + 16u * (uint32_t)(c ^ ((ra >> 1) & 7));
      wo[h][i] = DENSE ? (uint32_t)(n0 + rb) * (uint32_t)a.ldw * ES + 16u * (uint32_t)(c ^ ((rb >> 1) & 7)) : 0u;
    }
  const g8_rsrc rx = make_rsrc(a.x, a.x_bytes), rw = make_rsrc(a.w, a.w_bytes);
  auto a_img = [&](int t) -> uint8_t* { return smem + L::A0 + (t & 1) * L::ASTR; };
  auto b_img = [&](int t) -> uint8_t* { return smem + L::B0 + (t & 1) * L::BSTR; };
  auto stage_a = [&](int h, int t) {          // half-tile A_h of k-tile t -> buffer t & 1
    const int tt = kt0 + min(t, T - 1);       // past the end: harmless reload (keeps the vmcnt count)
    const uint8_t* img = a_img(t);
#pragma unroll
    for (int i = 0; i < 2; i++) dma16(rx, img + ar0[h][i] * ROWB, xo[h][i], tt * 128);
  };
  auto stage_b = [&](int h, int t) {          // dense only
    const int tt = kt0 + min(t, T - 1);
    const uint8_t* img = b_img(t);
#pragma unroll
    for (int i = 0; i < 2; i++) dma16(rw, img + br0[h][i] * ROWB, wo[h][i], tt * 128);
  };

  // ---- low-bit B: codes / scales of 128-k chunk c staged into ring slot
  // c & 1 (one 16-B DMA per lane each), decoded into the B image half h of
  // k-tile t just in time (see the schedule at the loop)
  const int KC = a.K / 128;
  const int NTt = (a.N + 15) / 16;
  const uint32_t TB = (uint32_t)(DENSE ? 0 : dk_tile_bytes(DK < 0 ? 0 : DK, KC));
  // codes: wave w <-> block row-tile j = w of half h: rt = (w >> 1) * 4 + 2 h + (w & 1)
  uint32_t co[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int rt = (wave >> 1) * 4 + 2 * h + (wave & 1);
    co[h] = (uint32_t)min(n0 / 16 + rt, NTt - 1) * TB + (uint32_t)lane * 16u;
  }
  // scales: lane l <-> block row-tile l >> 2, 16-B piece l & 3 of its 64 B
  const uint32_t so = (uint32_t)min(n0 / 16 + (lane >> 2), NTt - 1) * TB + (uint32_t)KC * 1024u +
                      (uint32_t)(lane & 3) * 16u;
  auto stage_codes = [&](int h, int c) {
    if constexpr (!DENSE) {
      const int cc = min(c, KC - 1);
      dma16(rw, smem + L::CODES + (c & 1) * 16384 + h * 8192 + wave * 1024, co[h], cc * 1024);
    }
  };
  auto stage_scales = [&](int c) {            // every wave loads the same 1 KB (uniform vmcnt)
    if constexpr (!DENSE) {
      const int cc = min(c, KC - 1);
      dma16(rw, smem + L::SCALES + (c & 1) * 1024, so, cc * 64);
    }
  };
  // decode half h of k-tile t: this thread's 16 weights = row (wave, r16) of
  // the half, k 8 g .. 8 g + 7 (part 0) and 32 + 8 g .. + 7 (part 1) of the tile
  uint2 cw = make_uint2(0u, 0u);
  uint32_t sd = 0u;
  auto dec_load = [&](int h, int t) {
    if constexpr (!DENSE) {
      const int c = t >> 1, kh = t & 1;
      cw = *(const uint2*)(smem + L::CODES + (c & 1) * 16384 + h * 8192 + wave * 1024 + lane * 16 + kh * 8);
      const int nl = (wave >> 1) * 64 + 32 * h + (wave & 1) * 16 + r16;
      sd = *(const uint32_t*)(smem + L::SCALES + (c & 1) * 1024 + nl * 4);
    }
  };
  auto dec_vals = [&](int t, int part) -> uint4 {
    if constexpr (!DENSE) {
      const int kh = t & 1;
      const float d = f16_to_f32((uint16_t)(kh ? (sd >> 16) : (sd & 0xffffu)));
      const float md = DK == DK_INT4S ? -136.f * d : 0.f;
      const float2* lut = (const float2*)(smem + (DENSE ? 0 : L::LUT));
      return dec8_bf16<DK>(part ? cw.y : cw.x, d, md, lut);
    }
    return make_uint4(0u, 0u, 0u, 0u);
  };
  auto dec_put = [&](int h, int part, const uint4& v) {
    if constexpr (!DENSE) {
      const int R = (wave >> 1) * 64 + 32 * h + (wave & 1) * 16 + r16;
      const int sw = (R >> 1) & 7;
      *(uint4*)(b_img(0) + R * ROWB + ((((part ? 4 : 0) + g) ^ sw) & 7) * 16) = v;
    }
  };
  auto dec_store = [&](int h, int t) {
    const uint4 v0 = dec_vals(t, 0), v1 = dec_vals(t, 1);
    dec_put(h, 0, v0);
    dec_put(h, 1, v1);
  };

  // ---- fragment read offsets: image row R + r16, logical chunk 4 s + g at
  // physical chunk (4 s + g) ^ ((r16 >> 1) & 7)
  const int sw = (r16 >> 1) & 7;
  // (fp8: the lane's 32-byte fragment = logical chunks 2 g, 2 g + 1)
  const int c0 = FP8 ? 2 * g : g, c1 = FP8 ? 2 * g + 1 : 4 + g;
  const uint32_t fo0 = (uint32_t)r16 * ROWB + (uint32_t)((c0 ^ sw) & 7) * 16;
  const uint32_t fo1 = (uint32_t)r16 * ROWB + (uint32_t)((c1 ^ sw) & 7) * 16;
  const uint32_t a_base = (uint32_t)(wr * 128) * ROWB, b_base = (uint32_t)(wc * 64) * ROWB;

  f32x4 acc[4][8];                            // [n-tile][m-tile], C^T tiles
#pragma unroll
  for (int nt = 0; nt < 4; nt++)
#pragma unroll
    for (int mt = 0; mt < 8; mt++) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 fa0[4][2], fa1[4][2], fb[2][2];       // A (m) halves, B (n) half; [tile][k-step]

  auto read_a = [&](uint4 (&f)[4][2], const uint8_t* img, int mh) {
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
      const uint8_t* p = img + a_base + (uint32_t)(mh * 64 + mt * 16) * ROWB;
      f[mt][0] = *(const uint4*)(p + fo0);
      f[mt][1] = *(const uint4*)(p + fo1);
    }
  };
  auto read_b = [&](const uint8_t* img, int nh) {
#pragma unroll
    for (int nt = 0; nt < 2; nt++) {
      const uint8_t* p = img + b_base + (uint32_t)(nh * 32 + nt * 16) * ROWB;
      fb[nt][0] = *(const uint4*)(p + fo0);
      fb[nt][1] = *(const uint4*)(p + fo1);
    }
  };
  auto mma = [&](const uint4 (&f)[4][2], int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (FP8) {
#pragma unroll
      for (int nt = 0; nt < 2; nt++) {
        const g8_i32x8 wb = {(int)fb[nt][0].x, (int)fb[nt][0].y, (int)fb[nt][0].z, (int)fb[nt][0].w,
                             (int)fb[nt][1].x, (int)fb[nt][1].y, (int)fb[nt][1].z, (int)fb[nt][1].w};
#pragma unroll
        for (int mt = 0; mt < 4; mt++) {
          const g8_i32x8 xa = {(int)f[mt][0].x, (int)f[mt][0].y, (int)f[mt][0].z, (int)f[mt][0].w,
                               (int)f[mt][1].x, (int)f[mt][1].y, (int)f[mt][1].z, (int)f[mt][1].w};
          // unit E8M0 block scales (127): the row / column scales go to the epilogue
          acc[nh * 2 + nt][mh * 4 + mt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              wb, xa, acc[nh * 2 + nt][mh * 4 + mt], FMTW, 0, 0, 127, 0, 127);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 2; s++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
#pragma unroll
          for (int mt = 0; mt < 4; mt++)
            acc[nh * 2 + nt][mh * 4 + mt] = mfma16<BF16>(fb[nt][s], f[mt][s], acc[nh * 2 + nt][mh * 4 + mt]);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  // the phase's 16 MFMAs with NP decode parts (8 weights each) computed in
  // their shadow: the decode VALU is placed inside the setprio region (a
  // scheduling boundary) and interleaved NV per MFMA, so it issues in the
  // MFMA's vector-issue gaps instead of after the cluster
  auto mma_dec = [&](const uint4 (&f)[4][2], int mh, int nh, int t, int p0, int np, uint4 (&v)[2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++)
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
          acc[nh * 2 + nt][mh * 4 + mt] = mfma16<BF16>(fb[nt][s], f[mt][s], acc[nh * 2 + nt][mh * 4 + mt]);
    v[0] = dec_vals(t, p0);
    if (np > 1) v[1] = dec_vals(t, 1);
#pragma unroll
    for (int i = 0; i < 16; i++) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (DENSE) {
    // ---- prologue: tile 0 complete, tile 1's A0 / B0 in flight
    stage_a(0, 0);
    stage_b(0, 0);
    stage_a(1, 0);
    stage_b(1, 0);
    stage_a(0, 1);
    stage_b(0, 1);
    wait_vm8();                                  // A0(0), B0(0) landed
    barrier();
    if (wr == 1) barrier();                      // stagger: wave-row 1 runs half a phase behind
    for (int u = 0; u < T; u++) {
      const uint8_t* ai = a_img(u);
      const uint8_t* bi = b_img(u);
      // phase 0: (mh0, nh0)
      read_a(fa0, ai, 0);
      read_b(bi, 0);
      stage_a(1, u + 1);
      wait_vm8();
      barrier();
      wait_lgkm0();
      mma(fa0, 0, 0);
      barrier();
      // phase 1: (mh1, nh0)
      read_a(fa1, ai, 1);
      stage_b(1, u + 1);
      wait_vm8();
      barrier();
      wait_lgkm0();
      mma(fa1, 1, 0);
      barrier();
      // phase 2: (mh0, nh1)
      read_b(bi, 1);
      stage_a(0, u + 2);
      wait_vm8();
      barrier();
      wait_lgkm0();
      mma(fa0, 0, 1);
      barrier();
      // phase 3: (mh1, nh1)
      stage_b(0, u + 2);
      wait_vm8();
      barrier();
      mma(fa1, 1, 1);
      barrier();
    }
    if (wr == 0) barrier();                      // close the stagger
  } else {
    // ---- low-bit schedule (global phase P = 4 t + p; chunk c = k-tiles 2c, 2c+1):
    //   p0: frags A(mh0) B(nh0);               DMA A1(t+1)
    //   p1: frags A(mh1); decode B0(t+1);      DMA t even: scales(t/2+1) again, t odd: scales((t+3)/2)
    //   p2: frags B(nh1);                      DMA A0(t+2)
    //   p3: decode B1(t+1);                    DMA t even: codes0(t/2+2), t odd: codes1((t+3)/2)
    // -> every 4 consecutive phases issue 6 DMAs per lane: vmcnt(6) each
    // phase keeps exactly the last 4 phases' stages in flight; every code /
    // scale stage lands >= 5 phases before its first decode and is re-staged
    // >= 2 phases after its last.  A decode writes its B-image half after the
    // phase's first barrier, one phase after that half's last read and two
    // phases before its next read, so the single B image is race-free even
    // with the two wave-rows staggered by a barrier.
    if constexpr (DK == DK_LUT4) {
      if (tid < 256) {
        const float2 v = make_float2(hd_lut4(a.lut_fmt, tid & 15), hd_lut4(a.lut_fmt, tid >> 4));
        *(float2*)(smem + L::LUT + tid * 8) = v;
      }
    }
    stage_codes(0, 0);
    stage_codes(1, 0);
    stage_scales(0);
    stage_a(0, 0);
    stage_a(1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    dec_load(0, 0);
    dec_store(0, 0);                             // B0, B1 of tile 0
    dec_load(1, 0);
    dec_store(1, 0);
    stage_codes(0, 1);
    stage_scales(1);
    stage_a(0, 1);
    stage_codes(1, 1);
    wait_lgkm0();
    barrier();
    if (wr == 1) barrier();                      // stagger: wave-row 1 runs half a phase behind
    for (int u = 0; u < T; u++) {
      const uint8_t* ai = a_img(u);
      const uint8_t* bi = b_img(u);
      const bool odd = u & 1;
      uint4 dv[2];
      // phase 0
      read_a(fa0, ai, 0);
      read_b(bi, 0);
      stage_a(1, u + 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      barrier();
      wait_lgkm0();
      mma(fa0, 0, 0);
      barrier();
      // phase 1
      read_a(fa1, ai, 1);
      dec_load(0, u + 1);
      stage_scales(odd ? (u + 3) >> 1 : (u >> 1) + 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      barrier();
      wait_lgkm0();
      if constexpr (G8S == 0) {
        mma(fa1, 1, 0);
        if (u + 1 < T) dec_store(0, u + 1);
      } else {
        // unconditional: a computed-but-unstored decode would be sunk into a
        // branch, out of the MFMA region (past the last tile the decode
        // writes a B half nobody reads again)
        mma_dec(fa1, 1, 0, u + 1, 0, 2, dv);
        dec_put(0, 0, dv[0]);
        dec_put(0, 1, dv[1]);
      }
      barrier();
      // phase 2
      read_b(bi, 1);
      stage_a(0, u + 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      barrier();
      wait_lgkm0();
      mma(fa0, 0, 1);
      barrier();
      // phase 3
      dec_load(1, u + 1);
      if (odd) stage_codes(1, (u + 3) >> 1);
      else stage_codes(0, (u >> 1) + 2);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      barrier();
      wait_lgkm0();
      if constexpr (G8S == 0) {
        mma(fa1, 1, 1);
        if (u + 1 < T) dec_store(1, u + 1);
      } else {
        mma_dec(fa1, 1, 1, u + 1, 0, 2, dv);
        dec_put(1, 0, dv[0]);
        dec_put(1, 1, dv[1]);
      }
      barrier();
    }
    if (wr == 0) barrier();                      // close the stagger
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's reloads

  // ---- epilogue: lane holds out[m][n .. n + 3], m = m-tile row r16, n = 4 g
  if (S > 1) {                                 // split-K: this split's f32 slab of the workspace
#pragma unroll
    for (int nt = 0; nt < 4; nt++) {
      const int n = n0 + wc * 64 + nt * 16 + 4 * g;
      if (n >= a.N) continue;
#pragma unroll
      for (int mt = 0; mt < 8; mt++) {
        const int m = m0 + wr * 128 + mt * 16 + r16;
        if (m >= a.M) continue;
        float* y = a.ws + ((size_t)ks * a.M + m) * a.N + n;
        if (n + 3 < a.N && (a.N & 3) == 0) {
          *(float4*)y = make_float4(acc[nt][mt][0], acc[nt][mt][1], acc[nt][mt][2], acc[nt][mt][3]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; i++)
            if (n + i < a.N) y[i] = acc[nt][mt][i];
        }
      }
    }
    return;
  }
  if (a.glu) {
    // w tiles alternate gate / up every 16 rows (the wave's 64 rows = 2
    // pairs): act(gate) * up in f32, one rounding, out column = pair * 16 + 4 g + i
    const int I = a.N / 2;
#pragma unroll
    for (int pr = 0; pr < 2; pr++) {
      const int c0 = ((n0 + wc * 64) / 32 + pr) * 16 + 4 * g;
      if (c0 >= I) continue;
#pragma unroll
      for (int mt = 0; mt < 8; mt++) {
        const int m = m0 + wr * 128 + mt * 16 + r16;
        if (m >= a.M) continue;
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float gv = acc[2 * pr][mt][i], uv = acc[2 * pr + 1][mt][i];
          o[i] = (a.act == 0 ? silu_f(gv) : gelu_tanh_f(gv)) * uv;
        }
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + c0;
        if (c0 + 3 < I && ((a.ldo | c0) & 3) == 0) *(uint2*)y = make_uint2(pack2<BF16>(o[0], o[1]), pack2<BF16>(o[2], o[3]));
        else for (int i = 0; i < 4 && c0 + i < I; i++) y[i] = from_f32<BF16>(o[i]);
      }
    }
    return;
  }
#pragma unroll
  for (int nt = 0; nt < 4; nt++) {
    const int n = n0 + wc * 64 + nt * 16 + 4 * g;
    if (n >= a.N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f}, cs[4] = {1.f, 1.f, 1.f, 1.f};
    if (a.bias != nullptr)
#pragma unroll
      for (int i = 0; i < 4; i++)
        bv[i] = n + i < a.N ? (a.out_f16 ? f16_to_f32(a.bias[n + i]) : bf16_to_f32(a.bias[n + i])) : 0.f;
    if constexpr (FP8) {
#pragma unroll
      for (int i = 0; i < 4; i++) cs[i] = a.sw_per_channel ? (n + i < a.N ? a.sw[n + i] : 0.f) : a.sw[0];
    }
#pragma unroll
    for (int mt = 0; mt < 8; mt++) {
      const int m = m0 + wr * 128 + mt * 16 + r16;
      if (m >= a.M) continue;
      const float rsx = FP8 ? a.sx[m] : 1.f;
      const float o0 = acc[nt][mt][0] * rsx * cs[0] + bv[0], o1 = acc[nt][mt][1] * rsx * cs[1] + bv[1];
      const float o2 = acc[nt][mt][2] * rsx * cs[2] + bv[2], o3 = acc[nt][mt][3] * rsx * cs[3] + bv[3];
      if (FP8 && a.out_f16) {
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n;
        if (n + 3 < a.N && ((a.ldo | n) & 3) == 0) *(uint2*)y = make_uint2(pack2<F16>(o0, o1), pack2<F16>(o2, o3));
        else {
          const float o[4] = {o0, o1, o2, o3};
          for (int i = 0; i < 4 && n + i < a.N; i++) y[i] = from_f32<F16>(o[i]);
        }
        continue;
      }
      if (a.out_f32) {
        float* y = (float*)a.out + (size_t)m * a.ldo + n;
        if (n + 3 < a.N && ((a.ldo | n) & 3) == 0) {
          float4 v = make_float4(o0, o1, o2, o3);
          if (a.accum) {
            const float4 ov = *(const float4*)y;
            v.x += ov.x, v.y += ov.y, v.z += ov.z, v.w += ov.w;
          }
          *(float4*)y = v;
        } else {
          const float o[4] = {o0, o1, o2, o3};
          for (int i = 0; i < 4 && n + i < a.N; i++) y[i] = o[i] + (a.accum ? y[i] : 0.f);
        }
      } else {
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n;
        if (n + 3 < a.N && ((a.ldo | n) & 3) == 0) {
          float q0 = o0, q1 = o1, q2 = o2, q3 = o3;
          if (a.accum) {                   // y += x w^T: one rounding of (old + sum)
            const uint2 ov = *(const uint2*)y;
            q0 += bf16_to_f32(ov.x & 0xffff), q1 += bf16_to_f32(ov.x >> 16);
            q2 += bf16_to_f32(ov.y & 0xffff), q3 += bf16_to_f32(ov.y >> 16);
          }
          *(uint2*)y = make_uint2(pack2<BF16>(q0, q1), pack2<BF16>(q2, q3));
        } else {
          const float o[4] = {o0, o1, o2, o3};
          for (int i = 0; i < 4 && n + i < a.N; i++)
            y[i] = from_f32<BF16>(o[i] + (a.accum ? bf16_to_f32(y[i]) : 0.f));
        }
      }
    }
  }
}

}  // namespace g8

// split-K epilogue: 4 consecutive outputs per thread (GLU: 4 consecutive
// outputs of one 16-row gate/up pair), bias, one rounding
__global__ void __launch_bounds__(256) gemm8p_finish_kernel(const G8Args a) {
  const int N = a.N, NO = a.glu ? N / 2 : N;
  const size_t q = (size_t)blockIdx.x * 256 + threadIdx.x;      // group of 4 outputs
  const int gpr = (NO + 3) / 4;
  const size_t m = q / gpr;
  if (m >= (size_t)a.M) return;
  const int c0 = (int)(q % gpr) * 4;
  const size_t slab = (size_t)a.M * N;
  const float* row = a.ws + m * N;
  auto at = [&](int c) {                      // the S slabs of element (m, c), summed in split order
    float v = row[c];
    for (int s = 1; s < a.ksplit; s++) v += row[s * slab + c];
    return v;
  };
  uint16_t* y = (uint16_t*)a.out + m * a.ldo;
  float o[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int c = min(c0 + i, NO - 1);
    if (a.glu) {
      const int pr = c / 16, j = c % 16;
      const float gv = at(pr * 32 + j), uv = at(pr * 32 + 16 + j);
      o[i] = (a.act == 0 ? silu_f(gv) : gelu_tanh_f(gv)) * uv;
    } else if (a.w_fmt == G8_FP8) {              // fp8: row x column scales, 16-bit bias
      const float cs = a.sw_per_channel ? a.sw[c] : a.sw[0];
      o[i] = at(c) * a.sx[m] * cs + (a.bias ? (a.out_f16 ? f16_to_f32(a.bias[c]) : bf16_to_f32(a.bias[c])) : 0.f);
    } else {
      o[i] = at(c) + (a.bias ? bf16_to_f32(a.bias[c]) : 0.f);
    }
  }
  if (a.out_f16) {
    uint16_t* yh = (uint16_t*)a.out + m * a.ldo;
    if (c0 + 3 < NO && ((a.ldo | c0) & 3) == 0) *(uint2*)(yh + c0) = make_uint2(pack2<F16>(o[0], o[1]), pack2<F16>(o[2], o[3]));
    else for (int i = 0; i < 4 && c0 + i < NO; i++) yh[c0 + i] = from_f32<F16>(o[i]);
    return;
  }
  if (a.out_f32) {
    float* yf = (float*)a.out + m * a.ldo;
    for (int i = 0; i < 4 && c0 + i < NO; i++) yf[c0 + i] = o[i] + (a.accum ? yf[c0 + i] : 0.f);
  } else if (c0 + 3 < NO && ((a.ldo | c0) & 3) == 0) {
    if (a.accum) {
      const uint2 ov = *(const uint2*)(y + c0);
      o[0] += bf16_to_f32(ov.x & 0xffff), o[1] += bf16_to_f32(ov.x >> 16);
      o[2] += bf16_to_f32(ov.y & 0xffff), o[3] += bf16_to_f32(ov.y >> 16);
    }
    *(uint2*)(y + c0) = make_uint2(pack2<BF16>(o[0], o[1]), pack2<BF16>(o[2], o[3]));
  } else {
    for (int i = 0; i < 4 && c0 + i < NO; i++) y[c0 + i] = from_f32<BF16>(o[i] + (a.accum ? bf16_to_f32(y[c0 + i]) : 0.f));
  }
}

int gemm8p_auto_split(int64_t M, int64_t N, int64_t ktiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  if (tiles * 2 > cus) return 1;
  int64_t s = cus / tiles;
  s = s < 8 ? s : 8;
  s = s < ktiles / 8 ? s : ktiles / 8;
  return (int)(s > 1 ? s : 1);
}

void launch_gemm8p_finish(const G8Args& a, hipStream_t st) {
  const int NO = a.glu ? a.N / 2 : a.N;
  const size_t groups = (size_t)a.M * ((NO + 3) / 4);
  hipLaunchKernelGGL(gemm8p_finish_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st, a);
}

void launch_gemm8p(const G8Args& a0, hipStream_t st) {
  G8Args a = a0;
  if (a.gm <= 0) {
    static const int gm_env = [] {
      const char* e = getenv("ILLM_G8_GM");
      return e ? atoi(e) : 0;
    }();
    a.gm = gm_env;
  }
  const int MB = (a.M + 255) / 256, NB = (a.N + 255) / 256;
  const int S = (a.w_fmt == -1 || a.w_fmt == G8_FP8) && a.ksplit > 1 ? a.ksplit : 1;
  const dim3 grid((unsigned)(MB * NB * S)), blk(512);
  if (a.w_fmt == G8_FP8 && a.w_e5m2) hipLaunchKernelGGL(g8::gemm8p_kernel<G8_FP8 - 1>, grid, blk, 0, st, a);
  else if (a.w_fmt == G8_FP8) hipLaunchKernelGGL(g8::gemm8p_kernel<G8_FP8>, grid, blk, 0, st, a);
  else if (a.w_fmt < 0) hipLaunchKernelGGL((g8::gemm8p_kernel<-1, 0>), grid, blk, 0, st, a);
  else {
    // decode interleaved into the MFMA clusters (1, default; +3 % at M = 8192,
    // profiles/g8_sched_sweep_r5.jsonl) or after them (ILLM_G8_SCHED=0)
    static const int sched = [] {
      const char* e = getenv("ILLM_G8_SCHED");
      return e ? atoi(e) : 1;
    }();
    const bool i4 = fmt_to_dk(a.w_fmt) == DK_INT4S;
    void (*k)(const G8Args) = i4 ? g8::gemm8p_kernel<DK_INT4S, 1> : g8::gemm8p_kernel<DK_LUT4, 1>;
    if (sched == 0) k = i4 ? g8::gemm8p_kernel<DK_INT4S, 0> : g8::gemm8p_kernel<DK_LUT4, 0>;
    hipLaunchKernelGGL(k, grid, blk, 0, st, a);
  }
}

bool gemm8p_supports(int fmt) { return fmt == -1 || fmt_to_dk(fmt) == DK_INT4S || fmt_to_dk(fmt) == DK_LUT4; }

}  // namespace illm
