// Prefill / training GEMM engine (xe_linear.forward_new at prefill M and the
// MatMulLowBit training forward: SRC/transformers/low_bit_linear.py:540-545,
// 704-708; the reference's ESIMD GEMM dequantizes inside the kernel, never to
// a dense weight in memory).  out[M, N] = x[M, K] . W[N, K]^T (+ bias) with W
// either the tiled low-bit device blob (formats.h) or a dense 16-bit matrix.
//
// MI355X design (gfx950, wave64, 256 CUs):
//   * workgroup = 8 waves (512 threads) = one BN (weights) x BM (tokens)
//     output block, 256 x 256 at large M; each wave owns WN 16-row weight
//     tiles x WM 16-row token tiles of v_mfma_f32_16x16x32 (acc[WN][WM]);
//   * K advances in 64-deep steps through two LDS stages (64 KiB each at
//     256 x 256); one barrier per step, the next step's operands land while
//     the current one computes;
//   * activations (and dense weights) go global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, 8 rows x 128 B per wave instruction, full
//     cache lines) into an XOR-swizzled [row][64] image: 16-B chunk c of row
//     r sits at chunk c ^ (r & 7), so the b128 fragment reads of 16 rows are
//     bank-conflict free; the swizzle is applied on the per-lane SOURCE
//     address (LDS-DMA writes lane-linear);
//   * low-bit weights: each 1 KiB (tile, chunk) code record is loaded ONCE
//     per workgroup (16 B per lane = exactly the lane's MFMA A fragments of
//     four k-steps), decoded in registers to pre-scaled f16 ((q - 8) * d,
//     lowbit_decode.h) and written to a fragment-linear LDS image that the
//     waves sharing those weight rows read conflict-free -- the decode runs
//     once per weight element per workgroup (not once per wave) and hides
//     among the MFMAs of the current step;
//   * bf16 activations reach the f16 MFMA through a per-row power-of-two
//     normalisation (launch_x_to_f16_rowscale: exact for every element
//     above 2^-28 of the row's max, no saturation at 65504, no underflow of
//     small gradients); the row scale is undone in the epilogue;
//   * XCD-aware block order: blocks that share id % 8 (one XCD, one L2) get
//     consecutive output blocks of one weight panel;
//   * split-K (grid.y) writes f32 slabs (reduced by launch_reduce_partials)
//     for the narrow-N / deep-K shapes that would not fill 256 CUs.
#include <cstdlib>

#include "../common/quant_block.h"
#include "gemv_args.h"
#include "illm_device.h"
#include "kernels.h"
#include "lowbit_decode.h"

namespace illm {

namespace mfg {

// 16-B LDS-DMA through a raw buffer descriptor on `base` (bytes past
// `bytes` read as zero).  A device function, not inline in the kernel's
// lambdas: a lambda that names __amdgpu_buffer_rsrc_t makes hipcc silently
// drop the kernel's host stub.
__device__ __forceinline__ void buf_lds16(const void* base, uint32_t bytes, uint16_t* lds, uint32_t voff, int soff) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// byte offset (in halves) of the b128 fragment read of row `r` (r & 7 known),
// logical 16-B chunk c, in a swizzled [row][64] image
__device__ __forceinline__ int sw_off(int r, int c) { return r * 64 + ((c ^ (r & 7)) << 3); }

template <int DK, typename TM, int WN, int WM, int WAVES_N>
__global__ void __launch_bounds__(512, 1) mfg_nt_kernel(const MfgArgs a) {
  constexpr int WAVES_M = 8 / WAVES_N;
  constexpr int BN = WAVES_N * WN * 16, BM = WAVES_M * WM * 16;
  constexpr int NTILE = BN / 16;
  constexpr bool DENSE = DK == DK_DENSE;
  constexpr int BITS = DENSE ? 16 : dk_bits(DK);
  constexpr int TPW = NTILE / 8;           // low-bit: weight tiles decoded per wave
  static_assert(NTILE % 8 == 0, "BN must be a multiple of 128");
  constexpr int XI = BM / 64;              // LDS-DMA instructions per wave per stage (x)
  constexpr int WI = BN / 64;              // same, dense weights
  constexpr int XS = BM * 64, WS = BN * 64;
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (XS + WS) + (DK == DK_LUT4 ? 512 : 0)];
  // weight stages first: their many per-tile read bases stay below 64 KiB
  // (ds_read immediates), the two x read bases carry the offset
  uint16_t* const W0 = smem;
  uint16_t* const W1 = smem + WS;
  uint16_t* const X0 = smem + 2 * WS;
  uint16_t* const X1 = smem + 2 * WS + XS;
  uint32_t* const lut2 = (uint32_t*)(smem + 2 * (XS + WS));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int wn = wave % WAVES_N, wm = wave / WAVES_N;

  // ---- block -> output block (XCD-aware, bijective over the grid)
  const int NB = (a.N + BN - 1) / BN, MB = (a.M + BM - 1) / BM;
  const int total = NB * MB;
  const int id = blockIdx.x;
  const int xcd = id & 7, q8 = total >> 3, r8 = total & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
  const int nb = wg / MB, mb = wg % MB;
  const int m0 = mb * BM, n0 = nb * BN;

  // ---- K range of this split (64-deep steps; K % 128 == 0, sps even)
  const int T = a.K / 64;
  const int t_beg = blockIdx.y * a.sps;
  const int t_end = min(T, t_beg + a.sps);

  // ---- activation LDS-DMA: buffer_load_dwordx4 ... lds through a buffer
  // descriptor (rows past M read as zeros, no clamping; one offset VGPR per
  // instruction, the k-step in the scalar offset).  Instruction i of a wave
  // covers image rows (wave * XI + i) * 8 + lane / 8, lane & 7 = the physical
  // chunk, i.e. logical chunk (lane & 7) ^ (lane >> 3) (the image's swizzle)
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int sch = (lane & 7) ^ (lane >> 3);
  uint32_t xoff[XI];
#pragma unroll
  for (int i = 0; i < XI; i++)
    xoff[i] = ((uint32_t)(m0 + (wv * XI + i) * 8 + (lane >> 3)) * (uint32_t)a.ldx + 8u * sch) * 2u;
  auto stage_x = [&](uint16_t* buf, int t) {
#pragma unroll
    for (int i = 0; i < XI; i++) buf_lds16(a.x, a.x_bytes, buf + (wv * XI + i) * 512, xoff[i], t * 128);
  };
  uint32_t woff[DENSE ? WI : 1];
  if constexpr (DENSE) {
#pragma unroll
    for (int i = 0; i < WI; i++)
      woff[i] = ((uint32_t)(n0 + (wv * WI + i) * 8 + (lane >> 3)) * (uint32_t)a.ldw + 8u * sch) * 2u;
  }
  auto stage_w = [&](uint16_t* buf, int t) {
    if constexpr (DENSE) {
#pragma unroll
      for (int i = 0; i < WI; i++) buf_lds16(a.w, a.w_bytes, buf + (wv * WI + i) * 512, woff[i], t * 128);
    }
  };

  // ---- low-bit weight records (codes of one 128-deep chunk + scales)
  struct Codes {
    uint4 q[DENSE ? 1 : TPW][BITS == 8 ? 2 : 1];
    uint32_t sc[DENSE ? 1 : TPW], mn[DENSE ? 1 : TPW];
  };
  const uint8_t* tbp[DENSE ? 1 : TPW];
  size_t soff = 0, moff = 0;
  if constexpr (!DENSE) {
    const int NT = (a.N + 15) / 16;
    const size_t TB = (size_t)dk_tile_bytes(DK, a.KC);
#pragma unroll
    for (int i = 0; i < TPW; i++) tbp[i] = a.w + (size_t)min(nb * NTILE + wave * TPW + i, NT - 1) * TB;
    soff = (size_t)a.KC * dk_code_chunk(DK) + (size_t)r16 * 4;
    moff = soff + (size_t)16 * a.KC * 4;
  }
  auto load_codes = [&](Codes& cs, int c) {
    if constexpr (!DENSE) {
#pragma unroll
      for (int i = 0; i < TPW; i++) {
        const uint8_t* rec = tbp[i] + (size_t)c * dk_code_chunk(DK);
        cs.q[i][0] = *(const uint4*)(rec + lane * 16);
        if constexpr (BITS == 8) cs.q[i][1] = *(const uint4*)(rec + 1024 + lane * 16);
        cs.sc[i] = *(const uint32_t*)(tbp[i] + soff + (size_t)c * 64);
        if constexpr (dk_has_min(DK)) cs.mn[i] = *(const uint32_t*)(tbp[i] + moff + (size_t)c * 64);
        else cs.mn[i] = 0u;
      }
    }
  };
  // decode step-half h (k-steps 2h, 2h+1 of the chunk) into a fragment-linear
  // image: [tile][k-step][lane] x 16 B
  auto decode_w = [&](uint16_t* buf, const Codes& cs, int h) {
    if constexpr (!DENSE) {
#pragma unroll
      for (int i = 0; i < TPW; i++) {
        const int lt = wave * TPW + i;
        const gh2 d2 = g_pick(cs.sc[i], h);
        const gh2 m2 = dk_has_min(DK) ? g_pick(cs.mn[i], h) : gh2{(_Float16)0.f, (_Float16)0.f};
#pragma unroll
        for (int sl = 0; sl < 2; sl++) {
          uint4 A;
          if constexpr (BITS == 4) {
            const uint4& q = cs.q[i][0];
            const uint32_t u = h == 0 ? (sl == 0 ? q.x : q.y) : (sl == 0 ? q.z : q.w);
            A = gemm_a4<DK>(u, d2, m2, lut2);
          } else {
            const uint4& q = cs.q[i][h];
            A = sl == 0 ? gemm_a8<DK>(q.x, q.y, d2, m2) : gemm_a8<DK>(q.z, q.w, d2, m2);
          }
          *(uint4*)(buf + ((lt * 2 + sl) * 64 + lane) * 8) = A;
        }
      }
    }
  };

  f32x4 acc[WN][WM];
#pragma unroll
  for (int t = 0; t < WN; t++)
#pragma unroll
    for (int mt = 0; mt < WM; mt++) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one 64-deep step: per 32-deep k-step the wave's WN weight fragments, then
  // its WM token fragments one at a time (the next one read while the WN
  // MFMAs of the current one issue); sched_group_barrier pins that order so
  // the fragments of a whole step are never live at once (128 accumulators +
  // 16 + 2 x 4 operand registers at 256 x 256)
  auto compute = [&](const uint16_t* xb, const uint16_t* wb) {
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int co = ((4 * s + g) ^ (r16 & 7)) << 3;
      uint4 A[WN];
#pragma unroll
      for (int t = 0; t < WN; t++) {
        if constexpr (DENSE) A[t] = *(const uint4*)(wb + ((wn * WN + t) * 16 + r16) * 64 + co);
        else A[t] = *(const uint4*)(wb + (((wn * WN + t) * 2 + s) * 64 + lane) * 8);
      }
      uint4 Bc = *(const uint4*)(xb + ((wm * WM) * 16 + r16) * 64 + co);
      __builtin_amdgcn_sched_group_barrier(0x100, WN + 1, 0);
#pragma unroll
      for (int mt = 0; mt < WM; mt++) {
        uint4 Bn = Bc;
        if (mt + 1 < WM) Bn = *(const uint4*)(xb + ((wm * WM + mt + 1) * 16 + r16) * 64 + co);
#pragma unroll
        for (int t = 0; t < WN; t++) acc[t][mt] = mfma16<TM>(A[t], Bc, acc[t][mt]);
        if (mt + 1 < WM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, WN, 0);
        Bc = Bn;
      }
    }
  };

  if constexpr (DK == DK_LUT4) {
    if (tid < 256) lut2[tid] = pack2<F16>(hd_lut4(a.lut_fmt, tid & 15), hd_lut4(a.lut_fmt, tid >> 4));
  }
  // software pipeline over 128-deep chunks (two 64-deep steps; LDS stage
  // parity static inside the body).  The codes of chunk c + 1 are loaded at
  // the start of step 2c + 1 and decoded at its end (one code set live)
  Codes cur;
  const int c_beg = t_beg >> 1, c_end = t_end >> 1;
  load_codes(cur, c_beg);
  stage_x(X0, t_beg);
  stage_w(W0, t_beg);
  if constexpr (DK == DK_LUT4) __syncthreads();
  decode_w(W0, cur, 0);
  __syncthreads();
  for (int c = c_beg; c < c_end; c++) {
    const bool more = c + 1 < c_end;
    stage_x(X1, 2 * c + 1);
    stage_w(W1, 2 * c + 1);
    compute(X0, W0);
    decode_w(W1, cur, 1);
    __syncthreads();
    if (more) {
      load_codes(cur, c + 1);
      stage_x(X0, 2 * c + 2);
      stage_w(W0, 2 * c + 2);
    }
    compute(X1, W1);
    if (more) decode_w(W0, cur, 0);
    __syncthreads();
  }

  // ---- epilogue: lane holds out[m = 16 mt + r16][n = 16 tile + 4 g + i]
  const int gt0 = nb * NTILE + wn * WN;                  // first global weight tile of the wave
  float rsv[WM];
#pragma unroll
  for (int mt = 0; mt < WM; mt++) {
    const int m = m0 + (wm * WM + mt) * 16 + r16;
    rsv[mt] = (a.rs != nullptr && m < a.M) ? a.rs[m] : 1.f;
  }
  if (a.glu) {
    const int I = a.N / 2;
#pragma unroll
    for (int pr = 0; pr < WN / 2; pr++) {
      const int n = ((gt0 >> 1) + pr) * 16 + 4 * g;
      if (n >= I) continue;
#pragma unroll
      for (int mt = 0; mt < WM; mt++) {
        const int m = m0 + (wm * WM + mt) * 16 + r16;
        if (m >= a.M) continue;
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float gv = acc[2 * pr][mt][i] * rsv[mt], uv = acc[2 * pr + 1][mt][i] * rsv[mt];
          o[i] = (a.act == 0 ? silu_f(gv) : gelu_tanh_f(gv)) * uv;
        }
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n;
        if (a.out_bf16) *(uint2*)y = make_uint2(pack2<BF16>(o[0], o[1]), pack2<BF16>(o[2], o[3]));
        else *(uint2*)y = make_uint2(pack2<F16>(o[0], o[1]), pack2<F16>(o[2], o[3]));
      }
    }
    return;
  }
  if (a.lora_x != nullptr) {
    // LoRA: acc = acc * rs + x_a . B^T as extra bf16 MFMA k-steps over the
    // (padded) rank -- fragments straight from the small L2-resident operands
#pragma unroll
    for (int t = 0; t < WN; t++)
#pragma unroll
      for (int mt = 0; mt < WM; mt++) {
        acc[t][mt] *= rsv[mt];
      }
#pragma unroll
    for (int mt = 0; mt < WM; mt++) rsv[mt] = 1.f;
    for (int s = 0; s < a.lora_rp / 32; s++) {
      uint4 Al[WN];
#pragma unroll
      for (int t = 0; t < WN; t++) {
        const int n = min((gt0 + t) * 16 + r16, a.N - 1);
        Al[t] = *(const uint4*)(a.lora_w + (size_t)n * a.lora_rp + 32 * s + 8 * g);
      }
#pragma unroll
      for (int mt = 0; mt < WM; mt++) {
        const int m = min(m0 + (wm * WM + mt) * 16 + r16, a.M - 1);
        const uint4 Bl = *(const uint4*)(a.lora_x + (size_t)m * a.lora_rp + 32 * s + 8 * g);
#pragma unroll
        for (int t = 0; t < WN; t++) acc[t][mt] = mfma16<BF16>(Al[t], Bl, acc[t][mt]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < WN; t++) {
    const int n = (gt0 + t) * 16 + 4 * g;
    if (n >= a.N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias != nullptr && blockIdx.y == 0) {
#pragma unroll
      for (int i = 0; i < 4; i++) bv[i] = a.bias_bf16 ? bf16_to_f32(a.bias[n + i]) : f16_to_f32(a.bias[n + i]);
    }
#pragma unroll
    for (int mt = 0; mt < WM; mt++) {
      const int m = m0 + (wm * WM + mt) * 16 + r16;
      if (m >= a.M) continue;
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; i++) o[i] = acc[t][mt][i] * rsv[mt] + bv[i];
      if (a.out_f32) {
        float* y = (float*)a.out + (size_t)blockIdx.y * a.slab + (size_t)m * a.ldo + n;
        *(float4*)y = make_float4(o[0], o[1], o[2], o[3]);
      } else {
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + n;
        if (a.out_bf16) *(uint2*)y = make_uint2(pack2<BF16>(o[0], o[1]), pack2<BF16>(o[2], o[3]));
        else *(uint2*)y = make_uint2(pack2<F16>(o[0], o[1]), pack2<F16>(o[2], o[3]));
      }
    }
  }
}

// one workgroup per row: amax -> power-of-two shift s.t. the row max lands in
// [2^14, 2^15); y = x * 2^shift exactly in f16, rs = 2^-shift
__global__ void __launch_bounds__(256) x_to_f16_rowscale_kernel(const uint16_t* x, int64_t ldx, int K, int in_bf16,
                                                                 uint16_t* y, float* rs) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const uint16_t* xr = x + row * ldx;
  uint16_t* yr = y + row * (int64_t)K;
  float amax = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const uint4 v = *(const uint4*)(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const float lo = in_bf16 ? bf16_to_f32(w[j] & 0xffff) : f16_to_f32(w[j] & 0xffff);
      const float hi = in_bf16 ? bf16_to_f32(w[j] >> 16) : f16_to_f32(w[j] >> 16);
      amax = fmaxf(amax, fmaxf(fabsf(lo), fabsf(hi)));
    }
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int shift = 0;
  if (amax > 0.f && amax <= 3.0e38f) {
    int e;
    frexpf(amax, &e);              // amax = f * 2^e, f in [0.5, 1)
    shift = 15 - e;                // amax * 2^shift in [2^14, 2^15)
    shift = max(-120, min(120, shift));
  }
  const float sc = ldexpf(1.f, shift);
  if (threadIdx.x == 0) rs[row] = ldexpf(1.f, -shift);
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const uint4 v = *(const uint4*)(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const float lo = in_bf16 ? bf16_to_f32(w[j] & 0xffff) : f16_to_f32(w[j] & 0xffff);
      const float hi = in_bf16 ? bf16_to_f32(w[j] >> 16) : f16_to_f32(w[j] >> 16);
      o[j] = pack2<F16>(lo * sc, hi * sc);
    }
    *(uint4*)(yr + k) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// the row normalisation above plus the LoRA down-projection of the same row:
// xa[row, r] = bf16(alpha * sum_k x[row, k] * la[r, k]) for r < R (zero up to
// rp = R rounded to 32) -- one pass over x serves the f16 copy, the row scale
// and the adapter input (RR = compile-time bound on R)
template <int RR>
__global__ void __launch_bounds__(256) x_rowscale_lora_kernel(const uint16_t* x, int64_t ldx, int K, int in_bf16,
                                                               uint16_t* y, float* rs, const uint16_t* la, int R,
                                                               float alpha, uint16_t* xa, int rp) {
  __shared__ float red[4];
  __shared__ float dots[4][RR];
  const int64_t row = blockIdx.x;
  const uint16_t* xr = x + row * ldx;
  uint16_t* yr = y + row * (int64_t)K;
  float amax = 0.f;
  float d[RR];
#pragma unroll
  for (int r = 0; r < RR; r++) d[r] = 0.f;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const uint4 v = *(const uint4*)(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float xv[8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      xv[2 * j] = in_bf16 ? bf16_to_f32(w[j] & 0xffff) : f16_to_f32(w[j] & 0xffff);
      xv[2 * j + 1] = in_bf16 ? bf16_to_f32(w[j] >> 16) : f16_to_f32(w[j] >> 16);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf(xv[j]));
#pragma unroll
    for (int r = 0; r < RR; r++) {
      if (r < R) {
        const uint4 av = *(const uint4*)(la + (size_t)r * K + k);
        const uint32_t aw[4] = {av.x, av.y, av.z, av.w};
#pragma unroll
        for (int j = 0; j < 4; j++)
          d[r] += xv[2 * j] * bf16_to_f32(aw[j] & 0xffff) + xv[2 * j + 1] * bf16_to_f32(aw[j] >> 16);
      }
    }
  }
  amax = wave_max(amax);
#pragma unroll
  for (int r = 0; r < RR; r++) d[r] = wave_sum(d[r]);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[wv] = amax;
#pragma unroll
    for (int r = 0; r < RR; r++) dots[wv][r] = d[r];
  }
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  for (int r = threadIdx.x; r < rp; r += 256) {
    const float s = r < R && r < RR ? (dots[0][r] + dots[1][r] + dots[2][r] + dots[3][r]) * alpha : 0.f;
    xa[row * rp + r] = f32_to_bf16(s);
  }
  int shift = 0;
  if (amax > 0.f && amax <= 3.0e38f) {
    int e;
    frexpf(amax, &e);
    shift = max(-120, min(120, 15 - e));
  }
  const float sc = ldexpf(1.f, shift);
  if (threadIdx.x == 0) rs[row] = ldexpf(1.f, -shift);
  if (y == nullptr) return;
  for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const uint4 v = *(const uint4*)(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const float lo = in_bf16 ? bf16_to_f32(w[j] & 0xffff) : f16_to_f32(w[j] & 0xffff);
      const float hi = in_bf16 ? bf16_to_f32(w[j] >> 16) : f16_to_f32(w[j] >> 16);
      o[j] = pack2<F16>(lo * sc, hi * sc);
    }
    *(uint4*)(yr + k) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

template <int DK, typename TM, int WN, int WM, int WAVES_N>
void launch_cfg(const MfgArgs& a, int ksplit, hipStream_t st) {
  constexpr int BN = WAVES_N * WN * 16, BM = (8 / WAVES_N) * WM * 16;
  const int NB = (a.N + BN - 1) / BN, MB = (a.M + BM - 1) / BM;
  hipLaunchKernelGGL((mfg_nt_kernel<DK, TM, WN, WM, WAVES_N>), dim3((unsigned)(NB * MB), (unsigned)ksplit),
                     dim3(512), 0, st, a);
}

template <int DK, typename TM>
void launch_tile(int tile, const MfgArgs& a, int ksplit, hipStream_t st) {
  switch (tile) {
    case MFG_TILE_256x128: launch_cfg<DK, TM, 4, 4, 4>(a, ksplit, st); break;
    case MFG_TILE_128x256: launch_cfg<DK, TM, 2, 8, 4>(a, ksplit, st); break;
    default: launch_cfg<DK, TM, 4, 8, 4>(a, ksplit, st); break;
  }
}

}  // namespace mfg

int mfg_block_n(int tile) { return tile == MFG_TILE_128x256 ? 128 : 256; }
int mfg_block_m(int tile) { return tile == MFG_TILE_256x128 ? 128 : 256; }

void launch_mfgemm(int fmt, bool dense_bf16, int tile, const MfgArgs& a, int ksplit, hipStream_t st) {
  if (fmt < 0) {
    if (dense_bf16) mfg::launch_tile<DK_DENSE, BF16>(tile, a, ksplit, st);
    else mfg::launch_tile<DK_DENSE, F16>(tile, a, ksplit, st);
    return;
  }
  switch (fmt_to_dk(fmt)) {
    case DK_INT4S: mfg::launch_tile<DK_INT4S, F16>(tile, a, ksplit, st); break;
    case DK_INT4A: mfg::launch_tile<DK_INT4A, F16>(tile, a, ksplit, st); break;
    case DK_LUT4: mfg::launch_tile<DK_LUT4, F16>(tile, a, ksplit, st); break;
    case DK_FP4: mfg::launch_tile<DK_FP4, F16>(tile, a, ksplit, st); break;
    case DK_INT8S: mfg::launch_tile<DK_INT8S, F16>(tile, a, ksplit, st); break;
    case DK_INT8A: mfg::launch_tile<DK_INT8A, F16>(tile, a, ksplit, st); break;
    case DK_FP8E4: mfg::launch_tile<DK_FP8E4, F16>(tile, a, ksplit, st); break;
    case DK_FP8E5: mfg::launch_tile<DK_FP8E5, F16>(tile, a, ksplit, st); break;
  }
}

void launch_x_rowscale_lora(bool bf16, const uint16_t* x, int64_t M, int64_t ldx, int K, uint16_t* y, float* rs,
                            const uint16_t* la, int R, float alpha, uint16_t* xa, int rp, hipStream_t st) {
  if (M <= 0) return;
  const dim3 grid((unsigned)M), blk(256);
  const int ib = bf16 ? 1 : 0;
  if (R <= 8) hipLaunchKernelGGL(mfg::x_rowscale_lora_kernel<8>, grid, blk, 0, st, x, ldx, K, ib, y, rs, la, R, alpha, xa, rp);
  else if (R <= 16) hipLaunchKernelGGL(mfg::x_rowscale_lora_kernel<16>, grid, blk, 0, st, x, ldx, K, ib, y, rs, la, R, alpha, xa, rp);
  else if (R <= 32) hipLaunchKernelGGL(mfg::x_rowscale_lora_kernel<32>, grid, blk, 0, st, x, ldx, K, ib, y, rs, la, R, alpha, xa, rp);
  else hipLaunchKernelGGL(mfg::x_rowscale_lora_kernel<64>, grid, blk, 0, st, x, ldx, K, ib, y, rs, la, R, alpha, xa, rp);
}

void launch_x_to_f16_rowscale(bool bf16, const uint16_t* x, int64_t M, int64_t ldx, int K, uint16_t* y, float* rs,
                              hipStream_t st) {
  if (M <= 0) return;
  hipLaunchKernelGGL(mfg::x_to_f16_rowscale_kernel, dim3((unsigned)M), dim3(256), 0, st, x, ldx, K, bf16 ? 1 : 0, y, rs);
}

}  // namespace illm
