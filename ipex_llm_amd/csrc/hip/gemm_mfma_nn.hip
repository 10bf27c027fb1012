// Transposed-weight GEMM of the engine: out[M, K] = g[M, N] . W[N, K] -- the
// grad_x of a linear y = x W^T (MatMulLowBit.backward, reference
// SRC/transformers/low_bit_linear.py:553-573, which dequantizes W to a dense
// [N, K] tensor and calls a dense matmul) and the lm_head input gradient.
//
// MI355X design: the same 512-thread / 256 x 256 block and 64-deep LDS
// stages as gemm_mfma.hip, reduction over the weight's ROW index n.  Each
// 1 KiB (tile, chunk) code record of the tiled blob is decoded once per
// workgroup (one record per wave per step) into a row-major [n][256] f16
// image; the MFMA A operand (rows = output k, reduction = n) is read from it
// TRANSPOSED with ds_read_b64_tr_b16 -- no dense W, no transpose pass.  The
// image's 16-B chunks are XOR-swizzled by row (mfg_common.h nn_swz) so both
// the decode writes and the transposed reads are bank-conflict free.  Dense
// weights (lm_head) fill the same image by LDS-DMA with the swizzle applied
// to the source address.  Requires N % 64 == 0 (the reduction runs in
// 64-row steps over g's columns) and K % 256 == 0 for low-bit weights.
#include <cstdlib>

#include "../common/quant_block.h"
#include "gemv_args.h"
#include "illm_device.h"
#include "kernels.h"
#include "lowbit_decode.h"
#include "mfg_common.h"

namespace illm {
namespace mfg {

// a.x = g [M, ldx] (MFMA type), a.K = reduction length (the weight's rows),
// a.N = output width (the weight's columns), a.KC = a.N / 128 (blob chunks),
// a.ldw = dense row stride
template <int DK, typename TM, int WN, int WM, int WAVES_N>
__global__ void __launch_bounds__(512, 1) mfg_nn_kernel(const MfgArgs a) {
  constexpr int WAVES_M = 8 / WAVES_N;
  constexpr int BO = WAVES_N * WN * 16, BM = WAVES_M * WM * 16;   // output columns x rows per block
  constexpr bool DENSE = DK == DK_DENSE;
  static_assert(DENSE || BO == 256, "low-bit NN blocks decode 4 tiles x 2 chunks per step");
  constexpr int XI = BM / 64;
  constexpr int WROW = BO * 2;                 // bytes per image row
  constexpr int WI = 64 * WROW / 1024 / 8;     // dense: LDS-DMA instructions per wave per stage
  constexpr int RPI = 1024 / WROW;             // dense: image rows per instruction
  constexpr int XS = BM * 64, WS = 64 * BO;
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
  const int wv = __builtin_amdgcn_readfirstlane(wave);

  const int OB = (a.N + BO - 1) / BO, MB = (a.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, OB * MB);
  const int ob = wg / MB, mb = wg % MB;
  const int m0 = mb * BM, o0 = ob * BO;

  const int T = a.K / 64;
  const int t_beg = blockIdx.y * a.sps;
  const int t_end = min(T, t_beg + a.sps);

  // ---- g staging (as x in the NT kernel): [m][64] XOR-swizzled image
  const int sch = (lane & 7) ^ (lane >> 3);
  uint32_t xoff[XI];
#pragma unroll
  for (int i = 0; i < XI; i++)
    xoff[i] = ((uint32_t)(m0 + (wv * XI + i) * 8 + (lane >> 3)) * (uint32_t)a.ldx + 8u * sch) * 2u;
  auto stage_x = [&](uint16_t* buf, int t) {
#pragma unroll
    for (int i = 0; i < XI; i++) buf_lds16(a.x, a.x_bytes, buf + (wv * XI + i) * 512, xoff[i], t * 128);
  };

  // ---- dense weights: [64 n][BO] image rows by LDS-DMA, swizzle on the source
  uint32_t woff[DENSE ? WI : 1];
  if constexpr (DENSE) {
#pragma unroll
    for (int i = 0; i < WI; i++) {
      const int row = (wv * WI + i) * RPI + lane / (64 / RPI);
      const int ch = (lane % (64 / RPI)) ^ nn_swz(row);
      woff[i] = ((uint32_t)row * (uint32_t)a.ldw + (uint32_t)o0 + 8u * ch) * 2u;
    }
  }
  auto stage_w = [&](uint16_t* buf, int t) {
    if constexpr (DENSE) {
#pragma unroll
      for (int i = 0; i < WI; i++)
        buf_lds16(a.w, a.w_bytes, buf + (wv * WI + i) * 512, woff[i], t * 64 * a.ldw * 2);
    }
  };

  // ---- low-bit: wave w decodes record (tile t*4 + w/2, chunk o0/128 + w%2)
  const int tl = wave >> 1, cl = wave & 1;
  const size_t TB = DENSE ? 0 : (size_t)dk_tile_bytes(DK, a.KC);
  const int cg = o0 / 128 + cl;
  const size_t cofs = (size_t)cg * dk_code_chunk(DK);
  const size_t sofs = DENSE ? 0 : (size_t)a.KC * dk_code_chunk(DK) + ((size_t)cg * 16 + r16) * 4;
  const size_t mofs = sofs + (size_t)16 * a.KC * 4;
  constexpr int BITS = DENSE ? 16 : dk_bits(DK);
  struct Rec {
    uint4 q[BITS == 8 ? 2 : 1];
    uint32_t sc, mn;
  };
  auto load_rec = [&](Rec& r, int t) {
    if constexpr (!DENSE) {
      const uint8_t* tb = a.w + (size_t)(t * 4 + tl) * TB;
      r.q[0] = *(const uint4*)(tb + cofs + lane * 16);
      if constexpr (BITS == 8) r.q[1] = *(const uint4*)(tb + cofs + 1024 + lane * 16);
      r.sc = *(const uint32_t*)(tb + sofs);
      r.mn = dk_has_min(DK) ? *(const uint32_t*)(tb + mofs) : 0u;
    }
  };
  auto decode_w = [&](uint16_t* buf, const Rec& r) {
    if constexpr (!DENSE) {
      const int n = tl * 16 + r16;
      const int sw = nn_swz(n);
#pragma unroll
      for (int s = 0; s < 4; s++) {
        const gh2 d2 = g_pick(r.sc, s >> 1);
        const gh2 m2 = dk_has_min(DK) ? g_pick(r.mn, s >> 1) : gh2{(_Float16)0.f, (_Float16)0.f};
        uint4 A;
        if constexpr (BITS == 4) {
          const uint32_t u = s == 0 ? r.q[0].x : (s == 1 ? r.q[0].y : (s == 2 ? r.q[0].z : r.q[0].w));
          A = gemm_a4<DK>(u, d2, m2, lut2);
        } else {
          const uint4& q = r.q[s >> 1];
          A = (s & 1) == 0 ? gemm_a8<DK>(q.x, q.y, d2, m2) : gemm_a8<DK>(q.z, q.w, d2, m2);
        }
        const int ch = cl * 16 + 4 * s + g;
        *(uint4*)(buf + n * BO + ((ch ^ sw) << 3)) = A;
      }
    }
  };

  f32x4 acc[WN][WM];
#pragma unroll
  for (int t = 0; t < WN; t++)
#pragma unroll
    for (int mt = 0; mt < WM; mt++) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed A reads: lane (q, p) of its 16-lane group -> row n_base + q,
  // columns 4p..4p+3 of the wave's output tile
  const int q4 = r16 >> 2, p4 = r16 & 3;
  auto compute = [&](const uint16_t* xb, const uint16_t* wb) {
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int co = ((4 * s + g) ^ (r16 & 7)) << 3;
      uint4 A[WN];
#pragma unroll
      for (int t = 0; t < WN; t++) {
        const int kt = wn * WN + t;
        const int ch = kt * 2 + (p4 >> 1);
        const int n1 = 32 * s + 8 * g + q4, n2 = n1 + 4;
        const uint2 v1 = ds_read_tr16(wb + n1 * BO + ((ch ^ nn_swz(n1)) << 3) + (p4 & 1) * 4);
        const uint2 v2 = ds_read_tr16(wb + n2 * BO + ((ch ^ nn_swz(n2)) << 3) + (p4 & 1) * 4);
        A[t] = make_uint4(v1.x, v1.y, v2.x, v2.y);
      }
      uint4 Bc = *(const uint4*)(xb + ((wm * WM) * 16 + r16) * 64 + co);
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * WN + 1, 0);
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
    __syncthreads();
  }
  Rec cur;
  load_rec(cur, t_beg);
  stage_x(X0, t_beg);
  stage_w(W0, t_beg);
  decode_w(W0, cur);
  __syncthreads();
  // two steps per iteration (stage parity static; an even step count per
  // split: a mid-body exit doubles the live accumulators)
  for (int t = t_beg; t < t_end; t += 2) {
    const bool more = t + 2 < t_end;
    load_rec(cur, t + 1);
    stage_x(X1, t + 1);
    stage_w(W1, t + 1);
    compute(X0, W0);
    decode_w(W1, cur);
    __syncthreads();
    if (more) {
      load_rec(cur, t + 2);
      stage_x(X0, t + 2);
      stage_w(W0, t + 2);
    }
    compute(X1, W1);
    if (more) decode_w(W0, cur);
    __syncthreads();
  }

  // ---- epilogue: lane holds out[m = 16 mt + r16][o = 16 kt + 4 g + i]
  float rsv[WM];
#pragma unroll
  for (int mt = 0; mt < WM; mt++) {
    const int m = m0 + (wm * WM + mt) * 16 + r16;
    rsv[mt] = (a.rs != nullptr && m < a.M) ? a.rs[m] : 1.f;
  }
  if (a.lora_x != nullptr) {
    // LoRA input gradient: acc = acc * rs + (s g B) . A as bf16 MFMA k-steps
    // over the padded rank (lora_w = A^T [N, rp])
#pragma unroll
    for (int t = 0; t < WN; t++)
#pragma unroll
      for (int mt = 0; mt < WM; mt++) acc[t][mt] *= rsv[mt];
#pragma unroll
    for (int mt = 0; mt < WM; mt++) rsv[mt] = 1.f;
    for (int s = 0; s < a.lora_rp / 32; s++) {
      uint4 Al[WN];
#pragma unroll
      for (int t = 0; t < WN; t++) {
        const int o = min(o0 + (wn * WN + t) * 16 + r16, a.N - 1);
        Al[t] = *(const uint4*)(a.lora_w + (size_t)o * a.lora_rp + 32 * s + 8 * g);
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
    const int o = o0 + (wn * WN + t) * 16 + 4 * g;
    if (o >= a.N) continue;
#pragma unroll
    for (int mt = 0; mt < WM; mt++) {
      const int m = m0 + (wm * WM + mt) * 16 + r16;
      if (m >= a.M) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; i++) v[i] = acc[t][mt][i] * rsv[mt];
      if (a.out_f32) {
        float* y = (float*)a.out + (size_t)blockIdx.y * a.slab + (size_t)m * a.ldo + o;
        *(float4*)y = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint16_t* y = (uint16_t*)a.out + (size_t)m * a.ldo + o;
        if (a.out_bf16) *(uint2*)y = make_uint2(pack2<BF16>(v[0], v[1]), pack2<BF16>(v[2], v[3]));
        else *(uint2*)y = make_uint2(pack2<F16>(v[0], v[1]), pack2<F16>(v[2], v[3]));
      }
    }
  }
}

template <int DK, typename TM, int WN, int WM, int WAVES_N>
void launch_nn_cfg(const MfgArgs& a, int ksplit, hipStream_t st) {
  constexpr int BO = WAVES_N * WN * 16, BM = (8 / WAVES_N) * WM * 16;
  const int OB = (a.N + BO - 1) / BO, MB = (a.M + BM - 1) / BM;
  hipLaunchKernelGGL((mfg_nn_kernel<DK, TM, WN, WM, WAVES_N>), dim3((unsigned)(OB * MB), (unsigned)ksplit),
                     dim3(512), 0, st, a);
}

template <int DK, typename TM>
void launch_nn_tile(int tile, const MfgArgs& a, int ksplit, hipStream_t st) {
  if (tile == MFG_TILE_256x128) launch_nn_cfg<DK, TM, 4, 4, 4>(a, ksplit, st);
  else launch_nn_cfg<DK, TM, 4, 8, 4>(a, ksplit, st);
}

}  // namespace mfg

void launch_mfgemm_nn(int fmt, bool dense_bf16, int tile, const MfgArgs& a, int ksplit, hipStream_t st) {
  if (fmt < 0) {
    if (dense_bf16) mfg::launch_nn_tile<DK_DENSE, BF16>(tile, a, ksplit, st);
    else mfg::launch_nn_tile<DK_DENSE, F16>(tile, a, ksplit, st);
    return;
  }
  switch (fmt_to_dk(fmt)) {
    case DK_INT4S: mfg::launch_nn_tile<DK_INT4S, F16>(tile, a, ksplit, st); break;
    case DK_INT4A: mfg::launch_nn_tile<DK_INT4A, F16>(tile, a, ksplit, st); break;
    case DK_LUT4: mfg::launch_nn_tile<DK_LUT4, F16>(tile, a, ksplit, st); break;
    case DK_FP4: mfg::launch_nn_tile<DK_FP4, F16>(tile, a, ksplit, st); break;
    case DK_INT8S: mfg::launch_nn_tile<DK_INT8S, F16>(tile, a, ksplit, st); break;
    case DK_INT8A: mfg::launch_nn_tile<DK_INT8A, F16>(tile, a, ksplit, st); break;
    case DK_FP8E4: mfg::launch_nn_tile<DK_FP8E4, F16>(tile, a, ksplit, st); break;
    case DK_FP8E5: mfg::launch_nn_tile<DK_FP8E5, F16>(tile, a, ksplit, st); break;
  }
}

}  // namespace illm
