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
//   * XCD-aware block order (bijective remap) with 4 m-blocks per group, so
//     concurrently running blocks of one XCD share x and w panels in its L2.
// All LDS lives in ONE __shared__ array (a second LDS object can make hipcc
// drain vmcnt before every ds_read, §5 item 4(a)).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

__global__ void __launch_bounds__(512) gemm8p_kernel(const G8Args a) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int g = lane >> 4, r16 = lane & 15;

  // ---- block -> (m-block, n-block): XCD remap, then groups of 4 m-blocks
  const int MB = (a.M + 255) / 256, NB = (a.N + 255) / 256;
  const int total = MB * NB;
  const int id = mfg::xcd_remap((int)blockIdx.x, total);
  constexpr int GM = 4;
  const int per_group = GM * NB;
  const int grp = id / per_group, rem = id % per_group;
  const int gm = min(GM, MB - grp * GM);
  const int mb = grp * GM + rem % gm, nb = rem / gm;
  const int m0 = mb * 256, n0 = nb * 256;
  const int T = a.K / 64;

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
      xo[h][i] = ((uint32_t)(m0 + ra) * (uint32_t)a.ldx + 8u * (uint32_t)(c ^ ((ra >> 1) & 7))) * 2u;
      wo[h][i] = ((uint32_t)(n0 + rb) * (uint32_t)a.ldw + 8u * (uint32_t)(c ^ ((rb >> 1) & 7))) * 2u;
    }
  const g8_rsrc rx = make_rsrc(a.x, a.x_bytes), rw = make_rsrc(a.w, a.w_bytes);
  auto stage_a = [&](int h, int t) {          // half-tile A_h of k-tile t -> buffer t & 1
    const int tt = min(t, T - 1);             // past the end: harmless reload (keeps the vmcnt count)
    const uint8_t* img = smem + (t & 1) * BUFB;
#pragma unroll
    for (int i = 0; i < 2; i++) dma16(rx, img + ar0[h][i] * ROWB, xo[h][i], tt * 128);
  };
  auto stage_b = [&](int h, int t) {
    const int tt = min(t, T - 1);
    const uint8_t* img = smem + (t & 1) * BUFB + IMG;
#pragma unroll
    for (int i = 0; i < 2; i++) dma16(rw, img + br0[h][i] * ROWB, wo[h][i], tt * 128);
  };

  // ---- fragment read offsets: image row R + r16, logical chunk 4 s + g at
  // physical chunk (4 s + g) ^ ((r16 >> 1) & 7)
  const int sw = (r16 >> 1) & 7;
  const uint32_t fo0 = (uint32_t)r16 * ROWB + (uint32_t)((g ^ sw) & 7) * 16;
  const uint32_t fo1 = (uint32_t)r16 * ROWB + (uint32_t)(((4 + g) ^ sw) & 7) * 16;
  const uint32_t a_base = (uint32_t)(wr * 128) * ROWB, b_base = IMG + (uint32_t)(wc * 64) * ROWB;

  f32x4 acc[4][8];                            // [n-tile][m-tile], C^T tiles
#pragma unroll
  for (int nt = 0; nt < 4; nt++)
#pragma unroll
    for (int mt = 0; mt < 8; mt++) acc[nt][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint4 fa0[4][2], fa1[4][2], fb[2][2];       // A (m) halves, B (n) half; [tile][k-step]

  auto read_a = [&](uint4 (&f)[4][2], const uint8_t* buf, int mh) {
#pragma unroll
    for (int mt = 0; mt < 4; mt++) {
      const uint8_t* p = buf + a_base + (uint32_t)(mh * 64 + mt * 16) * ROWB;
      f[mt][0] = *(const uint4*)(p + fo0);
      f[mt][1] = *(const uint4*)(p + fo1);
    }
  };
  auto read_b = [&](const uint8_t* buf, int nh) {
#pragma unroll
    for (int nt = 0; nt < 2; nt++) {
      const uint8_t* p = buf + b_base + (uint32_t)(nh * 32 + nt * 16) * ROWB;
      fb[nt][0] = *(const uint4*)(p + fo0);
      fb[nt][1] = *(const uint4*)(p + fo1);
    }
  };
  auto mma = [&](const uint4 (&f)[4][2], int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++)
#pragma unroll
        for (int mt = 0; mt < 4; mt++)
          acc[nh * 2 + nt][mh * 4 + mt] = mfma16<BF16>(fb[nt][s], f[mt][s], acc[nh * 2 + nt][mh * 4 + mt]);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: tile 0 complete, tile 1's A0 / B0 in flight
  stage_a(0, 0);
  stage_b(0, 0);
  stage_a(1, 0);
  stage_b(1, 0);
  stage_a(0, 1);
  stage_b(0, 1);
  wait_vm8();                                  // A0(0), B0(0) landed
  barrier();

  for (int u = 0; u < T; u++) {
    const uint8_t* buf = smem + (u & 1) * BUFB;
    // phase 0: (mh0, nh0)
    read_a(fa0, buf, 0);
    read_b(buf, 0);
    stage_a(1, u + 1);
    wait_vm8();
    barrier();
    wait_lgkm0();
    mma(fa0, 0, 0);
    barrier();
    // phase 1: (mh1, nh0)
    read_a(fa1, buf, 1);
    stage_b(1, u + 1);
    wait_vm8();
    barrier();
    wait_lgkm0();
    mma(fa1, 1, 0);
    barrier();
    // phase 2: (mh0, nh1)
    read_b(buf, 1);
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's reloads

  // ---- epilogue: lane holds out[m][n .. n + 3], m = m-tile row r16, n = 4 g
#pragma unroll
  for (int nt = 0; nt < 4; nt++) {
    const int n = n0 + wc * 64 + nt * 16 + 4 * g;
    if (n >= a.N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias != nullptr)
#pragma unroll
      for (int i = 0; i < 4; i++) bv[i] = n + i < a.N ? bf16_to_f32(a.bias[n + i]) : 0.f;
#pragma unroll
    for (int mt = 0; mt < 8; mt++) {
      const int m = m0 + wr * 128 + mt * 16 + r16;
      if (m >= a.M) continue;
      const float o0 = acc[nt][mt][0] + bv[0], o1 = acc[nt][mt][1] + bv[1];
      const float o2 = acc[nt][mt][2] + bv[2], o3 = acc[nt][mt][3] + bv[3];
      if (a.out_f32) {
        float* y = (float*)a.out + (size_t)m * a.ldo + n;
        if (n + 3 < a.N && ((a.ldo | n) & 3) == 0) *(float4*)y = make_float4(o0, o1, o2, o3);
        else {
          const float o[4] = {o0, o1, o2, o3};
          for (int i = 0; i < 4 && n + i < a.N; i++) y[i] = o[i];
        }
      } else {
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n;
        if (n + 3 < a.N && ((a.ldo | n) & 3) == 0) *(uint2*)y = make_uint2(pack2<BF16>(o0, o1), pack2<BF16>(o2, o3));
        else {
          const float o[4] = {o0, o1, o2, o3};
          for (int i = 0; i < 4 && n + i < a.N; i++) y[i] = from_f32<BF16>(o[i]);
        }
      }
    }
  }
}

}  // namespace g8

void launch_gemm8p(const G8Args& a, hipStream_t st) {
  const int MB = (a.M + 255) / 256, NB = (a.N + 255) / 256;
  hipLaunchKernelGGL(g8::gemm8p_kernel, dim3((unsigned)(MB * NB)), dim3(512), 0, st, a);
}

}  // namespace illm
