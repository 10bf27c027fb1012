// Dense bf16 NT GEMM on 4 waves x (128 x 128) -- the one-wave-per-SIMD
// tiling of the vendor library's MT256x256x64 kernels, written in HIP:
// y[M, N] = x[M, K] @ w[N, K]^T.  Experimental sibling of gemm_8p.hip,
// selected by the benchmark / tests only.
//
// Why: the 8-wave 8-phase kernel (128 x 64 per wave) moves ~192 KB of LDS
// fragment reads per 64-deep tile per CU; 128 x 128 per wave reads 128 KB
// (each A / B fragment feeds twice the MFMAs).  The 256 f32 accumulators per
// lane live in AGPRs (one wave per SIMD leaves the whole 512-entry register
// file to it).
//
// Schedule (tile u in LDS buffer u & 1; the wave's 128 x 128 is four 64 x 64
// quadrants q0 (m0, n0), q1 (m0, n1), q2 (m1, n1), q3 (m1, n0)):
//   q0: MFMA(A0, B0)   || ds_read B1          (same tile)
//   q1: MFMA(A0, B1)   || ds_read A1
//   --- s_waitcnt vmcnt(0) (tile u+1 landed) + lgkmcnt(0) + s_barrier:
//       every wave is done reading buffer u & 1 and tile u+1 is visible
//   issue the LDS-DMA of tile u+2 into buffer u & 1
//   q2: MFMA(A1, B1)   || ds_read A0'         (tile u+1)
//   q3: MFMA(A1, B0)   || ds_read B0'         (tile u+1)
// so fragment reads overlap the MFMAs of the previous quadrant inside the
// wave (no second wave to hide them) and one barrier per tile remains.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "illm_device.h"
#include "kernels_g8.h"
#include "mfg_common.h"

namespace illm {
namespace g4 {

constexpr int ROWB = 128;
constexpr int IMG = 256 * ROWB;       // 32 KB
constexpr int BUFB = 2 * IMG;         // A + B of one tile
constexpr int LDS_BYTES = 2 * BUFB;   // 128 KB

typedef int32_t rsrc_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)(uintptr_t)base;
  return rsrc_t{(int32_t)(uint32_t)p, (int32_t)((uint32_t)(p >> 32) & 0xffffu), (int32_t)bytes, 0x00020000};
}

// la = LDS byte address (wave-uniform)
__device__ __forceinline__ void dma16(const rsrc_t& rs, uint32_t la, uint32_t voff, int soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(la), "v"(voff), "s"(rs), "s"(soff) : "memory", "m0");
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm4w_kernel(const G8Args a) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int g = lane >> 4, r16 = lane & 15;

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

  // DMA: wave w, instruction i (0..7) stages image rows (i * 4 + w) * 8 ..+ 7
  // of A and of B (8 rows x 128 B = one wave instruction)
  uint32_t xo[8], wo[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int r = (i * 4 + wave) * 8 + (lane >> 3), c = lane & 7;
    const int sc = c ^ ((r >> 1) & 7);
    xo[i] = ((uint32_t)(m0 + r) * (uint32_t)a.ldx + 8u * (uint32_t)sc) * 2u;
    wo[i] = ((uint32_t)(n0 + r) * (uint32_t)a.ldw + 8u * (uint32_t)sc) * 2u;
  }
  const rsrc_t rx = make_rsrc(a.x, a.x_bytes), rw = make_rsrc(a.w, a.w_bytes);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)smem + (uint32_t)(wave * 8 * ROWB));
  auto stage = [&](int t) {
    const int tt = min(t, T - 1);
    const uint32_t buf = lds0 + (uint32_t)((t & 1) * BUFB);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      dma16(rx, buf + (uint32_t)(i * 32 * ROWB), xo[i], tt * 128);
      dma16(rw, buf + (uint32_t)(IMG + i * 32 * ROWB), wo[i], tt * 128);
    }
  };

  // 32 x 32 x 16 fragments: lane l holds row (l & 31), k chunk 2 s + (l >> 5)
  const int r32 = lane & 31, kh = lane >> 5;
  const int sw = (r32 >> 1) & 7;
  uint32_t fo[4];
#pragma unroll
  for (int s = 0; s < 4; s++) fo[s] = (uint32_t)r32 * ROWB + (uint32_t)(((2 * s + kh) ^ sw) & 7) * 16;
  const uint32_t a_base = (uint32_t)(wr * 128) * ROWB, b_base = IMG + (uint32_t)(wc * 128) * ROWB;

  f32x16 acc[4][4];                               // [n-block][m-block]
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = f32x16{};
  uint4 fa0[2][4], fa1[2][4], fb0[2][4], fb1[2][4];   // [32-row block][k step]

  auto rd = [&](uint4 (&f)[2][4], const uint8_t* buf, uint32_t base, int h) {
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
      for (int s = 0; s < 4; s++) f[t][s] = *(const uint4*)(buf + base + (uint32_t)(h * 64 + t * 32) * ROWB + fo[s]);
  };
  auto mma = [&](const uint4 (&fa)[2][4], const uint4 (&fb)[2][4], int mh, int nh) {
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int nt = 0; nt < 2; nt++)
#pragma unroll
        for (int mt = 0; mt < 2; mt++)
          acc[nh * 2 + nt][mh * 2 + mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              __builtin_bit_cast(bf16x8, fb[nt][s]), __builtin_bit_cast(bf16x8, fa[mt][s]),
              acc[nh * 2 + nt][mh * 2 + mt], 0, 0, 0);
  };

  // prologue: tiles 0 and 1 staged, tile 0's A0 / B0 fragments read
  stage(0);
  stage(1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");    // tile 0 (the first 16 DMAs) landed
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  rd(fa0, smem, a_base, 0);
  rd(fb0, smem, b_base, 0);
  // one quadrant: 16 MFMAs with the 8 fragment reads of the next one
  // spread over the first half (1 read : 1 MFMA)
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // B0 of tile u is in rb0 and its B1 goes to rb1; tile u+1's B0 lands in
  // rb1 (free after q2), so the B roles swap every tile (unrolled by 2)
  auto tile = [&](int u, uint4 (&rb0)[2][4], uint4 (&rb1)[2][4]) {
    const uint8_t* buf = smem + (u & 1) * BUFB;
    const uint8_t* nbuf = smem + ((u + 1) & 1) * BUFB;
    rd(rb1, buf, b_base, 1);                             // q0
    mma(fa0, rb0, 0, 0);
    interleave();
    rd(fa1, buf, a_base, 1);                             // q1
    mma(fa0, rb1, 0, 1);
    interleave();
    // every wave's reads of this buffer done, tile u+1 landed
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stage(u + 2);                                        // into this buffer (past the end: harmless reload)
    __builtin_amdgcn_sched_barrier(0);
    rd(fa0, nbuf, a_base, 0);                            // q2 reads tile u+1's A0
    mma(fa1, rb1, 1, 1);
    interleave();
    rd(rb1, nbuf, b_base, 0);                            // q3 reads tile u+1's B0
    mma(fa1, rb0, 1, 0);
    interleave();
  };
  for (int u = 0; u < T; u += 2) {                     // K % 128 == 0 (host-checked)
    tile(u, fb0, fb1);
    tile(u + 1, fb1, fb0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: acc[nt][mt][4 q + i] = out[m][n + i], m = row r32 of m-block mt,
  // n = 8 q + 4 kh of n-block nt
#pragma unroll
  for (int mt = 0; mt < 4; mt++) {
    const int m = m0 + wr * 128 + mt * 32 + r32;
    if (m >= a.M) continue;
    uint16_t* yr = (uint16_t*)a.out + (size_t)m * a.ldo;
#pragma unroll
    for (int nt = 0; nt < 4; nt++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int n = n0 + wc * 128 + nt * 32 + q * 8 + 4 * kh;
        const f32x16& c = acc[nt][mt];
        const float o0 = c[4 * q], o1 = c[4 * q + 1], o2 = c[4 * q + 2], o3 = c[4 * q + 3];
        if (n + 3 < a.N && ((a.ldo | n) & 3) == 0) {
          *(uint2*)(yr + n) = make_uint2(pack2<BF16>(o0, o1), pack2<BF16>(o2, o3));
        } else {
          if (n < a.N) yr[n] = from_f32<BF16>(o0);
          if (n + 1 < a.N) yr[n + 1] = from_f32<BF16>(o1);
          if (n + 2 < a.N) yr[n + 2] = from_f32<BF16>(o2);
          if (n + 3 < a.N) yr[n + 3] = from_f32<BF16>(o3);
        }
      }
  }
}

}  // namespace g4

void launch_gemm4w(const G8Args& a, hipStream_t st) {
  const int MB = (a.M + 255) / 256, NB = (a.N + 255) / 256;
  hipLaunchKernelGGL(g4::gemm4w_kernel, dim3((unsigned)(MB * NB)), dim3(256), 0, st, a);
}

}  // namespace illm
