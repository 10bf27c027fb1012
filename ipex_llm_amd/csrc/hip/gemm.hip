// Low-bit weight x f16/bf16 activation GEMM for prefill-size M (> 64 rows):
// the MFMA path of xe_linear.forward_new at prefill
// (SRC/transformers/low_bit_linear.py:704-708; the reference dequantizes
// inside its ESIMD/XeTLA GEMM, never to a dense weight in memory).
//
// MI355X design (gfx950, v_mfma_f32_16x16x32_f16, wave64):
//   * workgroup = 4 waves = a 128 (n) x 128 (m) output block; wave w owns
//     weight tiles 2w, 2w+1 (32 rows) against all 128 tokens, so each
//     decoded A fragment feeds 8 MFMAs and each B fragment read from LDS
//     feeds 2;
//   * weights stream straight from the tiled device blob (formats.h): one
//     16-B code load per lane per (tile, 128-k chunk) is exactly the MFMA A
//     fragment of the 4 k-steps; codes are decoded and pre-scaled in f16
//     registers ((q - 8) * d: exact code, one rounding), never written to
//     memory (the dequantize + hipBLASLt path wrote 2 B per weight);
//   * activations: the 128 x 128 x-chunk is staged global -> registers ->
//     LDS as f16 (double buffered, one chunk ahead), padded rows (272 B) so
//     the B-fragment ds_read_b128 of 16 rows hit distinct banks.  bf16
//     activations are converted to f16 ONCE per call with a per-row
//     power-of-two normalisation (launch_x_to_f16_rowscale, shared with the
//     MFMA engine): every bf16 value keeps its f16 mantissa, nothing
//     saturates at 65504, and the epilogue multiplies the row scale back.
//     Converting while staging repeated the work for every n-block and was
//     ~90 % of the kernel's VALU instructions (rocprofv3 PMC, gate_up M=1024);
//   * XCD-aware block order: the 8 m-blocks of one n-block run on one XCD
//     (ids b, b + 8, ...), so a weight chunk comes from HBM once per XCD
//     and is re-read by the other m-blocks from that XCD's L2.
#include <cstdlib>
#include <type_traits>

#include "../common/quant_block.h"
#include "gemv_args.h"
#include "illm_device.h"
#include "kernels.h"
#include "lowbit_decode.h"

namespace illm {

constexpr int GLDX = 128 + 8;     // LDS row stride of the x chunk (halves)

// WN weight tiles (16 rows each) x WM token tiles (16 rows each) per wave; the
// 4 waves of a block form a WA (along n) x 4/WA (along m) grid:
// block = (WA WN 16) n x (4/WA WM 16) m.
//   <2, 8, WA 4>: 128 n x 128 m, every x fragment read from LDS feeds 2 MFMAs;
//   <4, 4, WA 4>: 256 n x 64 m, 4 MFMAs per x fragment, 4 decoded tiles per wave;
//   <4, 4, WA 2>: 128 n x 128 m, 4 MFMAs per x fragment (half the LDS reads of
//                 <2, 8>) at the same accumulator count; each weight tile is
//                 decoded by the two m-halves' waves (L1 hits for the second).
template <int DK, typename T, int WN, int WM, int PFW, int WA = 4>
__global__ void __launch_bounds__(256) lowbit_gemm_kernel(const GemmArgs a) {
  constexpr int BITS = dk_bits(DK);
  constexpr int GBM = (4 / WA) * WM * 16, GBN = WA * WN * 16;
  __shared__ __attribute__((aligned(16))) uint16_t xs[2][GBM * GLDX];
  __shared__ uint32_t lut2[DK == DK_LUT4 ? 256 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;

  // XCD-aware block order: the MB m-blocks of n-block nb get ids that share id % 8
  const bool grouped = a.moe_off != nullptr;
  const int NB = (a.N + GBN - 1) / GBN;
  const int MB = grouped ? (a.M + GBM - 1) / GBM + a.moe_el : (a.M + GBM - 1) / GBM;
  const int id = blockIdx.x;
  const int grp = id / (8 * MB), rem = id % (8 * MB);
  int mb = rem / 8;
  const int nb = grp * 8 + rem % 8;
  if (nb >= NB) return;
  // grouped: global m-block mb -> (local expert e, its m-block); every thread
  // scans a slice of the experts (block-uniform result, no host sync)
  int Mrows = a.M, e_sel = 0, pos0 = 0;
  const uint8_t* wbase = a.w;
  if (grouped) {
    __shared__ int mb_tot[256];
    __shared__ int sel[3];
    const int per = (a.moe_el + 255) / 256;            // experts per thread (contiguous)
    int cnt_blocks = 0;
    for (int j = 0; j < per; j++) {
      const int e = tid * per + j;
      if (e < a.moe_el) cnt_blocks += (a.moe_off[e + 1] - a.moe_off[e] + GBM - 1) / GBM;
    }
    mb_tot[tid] = cnt_blocks;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {                 // inclusive scan of m-blocks per thread slice
      const int v = tid >= o ? mb_tot[tid - o] : 0;
      __syncthreads();
      mb_tot[tid] += v;
      __syncthreads();
    }
    if (tid == 0) sel[0] = -1;
    __syncthreads();
    const int ex = mb_tot[tid] - cnt_blocks;
    if (mb >= ex && mb < mb_tot[tid]) {
      int r = mb - ex;
      for (int j = 0; j < per; j++) {
        const int e = tid * per + j;
        const int c = (a.moe_off[e + 1] - a.moe_off[e] + GBM - 1) / GBM;
        if (r < c) { sel[0] = e; sel[1] = r; break; }
        r -= c;
      }
    }
    __syncthreads();
    if (sel[0] < 0) return;                             // past the last expert's rows
    e_sel = sel[0];
    mb = sel[1];
    pos0 = a.moe_off[e_sel];
    Mrows = a.moe_off[e_sel + 1] - pos0;
    wbase = a.w + (size_t)e_sel * a.w_stride;
  }
  const int m0 = mb * GBM;
  const int NT = (a.N + 15) / 16;
  const int wn = wave % WA, wm = wave / WA;           // wave position in the block
  const int tile0 = nb * (WA * WN) + wn * WN;
  const size_t TB = (size_t)dk_tile_bytes(DK, a.KC);
  const uint8_t* tb[WN];
#pragma unroll
  for (int t = 0; t < WN; t++) tb[t] = wbase + (size_t)min(tile0 + t, NT - 1) * TB;
  const size_t soff = (size_t)a.KC * dk_code_chunk(DK) + (size_t)r16 * 4;   // + c * 64: row r16 of chunk c
  const size_t moff = soff + (size_t)16 * a.KC * 4;

  if constexpr (DK == DK_LUT4) {
    lut2[tid] = pack2<F16>(hd_lut4(a.lut_fmt, tid & 15), hd_lut4(a.lut_fmt, tid >> 4));
  }

  // ---- x staging: thread -> rows (tid / 16) + 16 j, 8 columns at (tid % 16) * 8
  constexpr int XJ = GBM / 16;
  uint4 xr[XJ];
  int xrow[XJ];                                         // source row of staged row j (-1: padding)
#pragma unroll
  for (int j = 0; j < XJ; j++) {
    const int m = m0 + (tid >> 4) + 16 * j;
    if (m >= Mrows) xrow[j] = -1;
    else if (!grouped) xrow[j] = m;
    else xrow[j] = a.moe_x_sorted ? pos0 + m : a.moe_rows[pos0 + m] / a.moe_xdiv;
  }
  auto stage_load = [&](int c) {
    const int kk = c * 128 + (tid & 15) * 8;
#pragma unroll
    for (int j = 0; j < XJ; j++) {
      const bool ok = xrow[j] >= 0 && kk < a.K;
      const uint4 v = *(const uint4*)(a.x + (size_t)(ok ? xrow[j] : 0) * a.ldx + (ok ? kk : 0));
      xr[j] = ok ? v : make_uint4(0, 0, 0, 0);
    }
  };
  auto stage_store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < XJ; j++) {
      uint4 v = xr[j];
      if (std::is_same<T, BF16>::value && !a.x_f16) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float lo = fminf(fmaxf(bf16_to_f32(w[i] & 0xffff), -65504.f), 65504.f);
          const float hi = fminf(fmaxf(bf16_to_f32(w[i] >> 16), -65504.f), 65504.f);
          w[i] = pack2<F16>(lo, hi);
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *(uint4*)(&xs[buf][((tid >> 4) + 16 * j) * GLDX + (tid & 15) * 8]) = v;
    }
  };

  // ---- weight chunk records (A fragments of 4 k-steps) + row-r16 scales
  struct WChunk {
    uint4 q[WN][BITS / 4];
    uint32_t sc[WN], mn[WN];
  };
  auto load_w = [&](WChunk& wc, int c) {
#pragma unroll
    for (int t = 0; t < WN; t++) {
      const uint8_t* rec = tb[t] + (size_t)c * dk_code_chunk(DK);
      wc.q[t][0] = *(const uint4*)(rec + lane * 16);
      if constexpr (BITS == 8) wc.q[t][1] = *(const uint4*)(rec + 1024 + lane * 16);
      wc.sc[t] = *(const uint32_t*)(tb[t] + soff + (size_t)c * 64);
      if constexpr (dk_has_min(DK)) wc.mn[t] = *(const uint32_t*)(tb[t] + moff + (size_t)c * 64);
      else wc.mn[t] = 0u;
    }
  };

  f32x4 acc[WN][WM];
#pragma unroll
  for (int t = 0; t < WN; t++)
#pragma unroll
    for (int mt = 0; mt < WM; mt++) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weight ring: PFW chunks in flight (one chunk of MFMA work, ~1k cycles,
  // does not cover an HBM round trip under load); loads are unconditional
  // (clamped) so hipcc keeps counted vmcnt waits
  const int KC = a.KC;
  auto load_wc = [&](WChunk& wc, int c) { load_w(wc, min(c, KC - 1)); };
  WChunk ring[PFW];
#pragma unroll
  for (int u = 0; u < PFW; u++) load_wc(ring[u], u);
  stage_load(0);
  stage_store(0);
  __syncthreads();

  auto pick = [](uint32_t v, int blk) -> gh2 {
    return g_as_h2(__builtin_amdgcn_perm(0u, v, blk == 0 ? 0x01000100u : 0x03020302u));
  };
  auto compute = [&](const WChunk& cur, int buf) {
    const uint16_t* xb = &xs[buf][(wm * WM * 16 + r16) * GLDX + 8 * g];
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int blk = s >> 1;
      uint4 A[WN];
#pragma unroll
      for (int t = 0; t < WN; t++) {
        const gh2 d2 = pick(cur.sc[t], blk);
        const gh2 m2 = dk_has_min(DK) ? pick(cur.mn[t], blk) : gh2{(_Float16)0.f, (_Float16)0.f};
        if constexpr (BITS == 4) {
          const uint4& q0 = cur.q[t][0];
          const uint32_t w = s == 0 ? q0.x : (s == 1 ? q0.y : (s == 2 ? q0.z : q0.w));
          A[t] = gemm_a4<DK>(w, d2, m2, lut2);
        } else {
          const uint4& qq = cur.q[t][blk];
          A[t] = (s & 1) == 0 ? gemm_a8<DK>(qq.x, qq.y, d2, m2) : gemm_a8<DK>(qq.z, qq.w, d2, m2);
        }
      }
      uint4 B[WM];
#pragma unroll
      for (int mt = 0; mt < WM; mt++) B[mt] = *(const uint4*)(xb + mt * 16 * GLDX + 32 * s);
#pragma unroll
      for (int mt = 0; mt < WM; mt++)
#pragma unroll
        for (int t = 0; t < WN; t++) acc[t][mt] = mfma16<F16>(A[t], B[mt], acc[t][mt]);
    }
  };
  for (int c0 = 0; c0 < KC; c0 += PFW) {
#pragma unroll
    for (int u = 0; u < PFW; u++) {
      const int c = c0 + u;
      if (c < KC) {                        // block-uniform
        const bool more = c + 1 < KC;
        if (more) stage_load(c + 1);
        compute(ring[u], c & 1);
        load_wc(ring[u], c + PFW);
        if (more) stage_store((c + 1) & 1);
        __syncthreads();
      }
    }
  }

  // ---- epilogue: lane holds out[m0 + 16 mt + r16][16 tile + 4 g + i]
  // undo the per-row activation normalisation first (exact: powers of two)
  if (a.rs != nullptr) {
#pragma unroll
    for (int mt = 0; mt < WM; mt++) {
      const int mm = m0 + (wm * WM + mt) * 16 + r16;
      float rsv = 1.f;
      if (mm < Mrows)
        rsv = a.rs[!grouped ? mm : (a.moe_x_sorted ? pos0 + mm : a.moe_rows[pos0 + mm] / a.moe_xdiv)];
#pragma unroll
      for (int t = 0; t < WN; t++)
#pragma unroll
        for (int i = 0; i < 4; i++) acc[t][mt][i] *= rsv;
    }
  }
  if (a.glu) {
    // the wave's tiles are gate/up pairs (16-row interleave, tile0 even):
    // act(gate) * up in f32, one rounding (as the decode GLU GEMV epilogue)
    const int I = a.N / 2;
#pragma unroll
    for (int pr = 0; pr < WN / 2; pr++) {
      if (tile0 + 2 * pr + 1 >= NT) continue;
      const int n0 = (tile0 / 2 + pr) * 16 + 4 * g;
      if (n0 >= I) continue;
#pragma unroll
      for (int mt = 0; mt < WM; mt++) {
        const int mm = m0 + (wm * WM + mt) * 16 + r16;
        if (mm >= Mrows) continue;
        const int m = !grouped ? mm : (a.moe_out_sorted ? pos0 + mm : a.moe_rows[pos0 + mm]);
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const float gv = acc[2 * pr][mt][i], uv = acc[2 * pr + 1][mt][i];
          o[i] = (a.act == 0 ? silu_f(gv) : gelu_tanh_f(gv)) * uv;
        }
        uint16_t* y = a.out + (size_t)m * a.ldo + n0;
        if (n0 + 3 < I && ((a.ldo | n0) & 3) == 0) *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
        else for (int i = 0; i < 4 && n0 + i < I; i++) y[i] = from_f32<T>(o[i]);
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < WN; t++) {
    const int tile = tile0 + t;
    if (tile >= NT) continue;
    const int n0 = tile * 16 + 4 * g;
    if (n0 >= a.N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias)
#pragma unroll
      for (int i = 0; i < 4; i++) bv[i] = n0 + i < a.N ? to_f32<T>(a.bias[n0 + i]) : 0.f;
#pragma unroll
    for (int mt = 0; mt < WM; mt++) {
      const int mm = m0 + (wm * WM + mt) * 16 + r16;
      if (mm >= Mrows) continue;
      const int m = !grouped ? mm : (a.moe_out_sorted ? pos0 + mm : a.moe_rows[pos0 + mm]);
      const float o[4] = {acc[t][mt][0] + bv[0], acc[t][mt][1] + bv[1], acc[t][mt][2] + bv[2],
                          acc[t][mt][3] + bv[3]};
      if (a.out_f32) {
        float* yf = (float*)a.out + (size_t)m * a.ldo + n0;
        if (n0 + 3 < a.N && ((a.ldo | n0) & 3) == 0) *(float4*)yf = make_float4(o[0], o[1], o[2], o[3]);
        else for (int i = 0; i < 4 && n0 + i < a.N; i++) yf[i] = o[i];
        continue;
      }
      uint16_t* y = a.out + (size_t)m * a.ldo + n0;
      if (n0 + 3 < a.N && ((a.ldo | n0) & 3) == 0) *(uint2*)y = make_uint2(pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]));
      else for (int i = 0; i < 4 && n0 + i < a.N; i++) y[i] = from_f32<T>(o[i]);
    }
  }
}

template <int DK, int WN, int WM, int PFW, int WA = 4>
static void launch_gemm_v(bool bf16, const GemmArgs& a, hipStream_t st) {
  constexpr int GBM = (4 / WA) * WM * 16, GBN = WA * WN * 16;
  const int NB = (a.N + GBN - 1) / GBN;
  // grouped: every expert may end with a partial m-block
  const int MB = a.moe_off ? (a.M + GBM - 1) / GBM + a.moe_el : (a.M + GBM - 1) / GBM;
  const int NBp = (NB + 7) / 8 * 8;
  dim3 grid((unsigned)(NBp * MB));
  if (bf16) hipLaunchKernelGGL((lowbit_gemm_kernel<DK, BF16, WN, WM, PFW, WA>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((lowbit_gemm_kernel<DK, F16, WN, WM, PFW, WA>), grid, dim3(256), 0, st, a);
}

template <int DK>
static void launch_gemm_dk(bool bf16, const GemmArgs& a, hipStream_t st) {
  // ILLM_GEMM_TILE: 0 = 128 n x 128 m blocks (2 tiles x 8 m-tiles per wave), 2 = 256 n x 64 m
  // (half the LDS x traffic per MFMA but 268 registers -> 1 wave per SIMD; M = 1024 qkv/o/down
  // +1..14 %, gate_up -12 %, M = 8192 -15..18 %), 3/4 = 2 x 2 wave grid (slower everywhere),
  // 6 = 128 n x 64 m with 6 weight chunks in flight.  Unset: 6 up to M = 768 (and to 1024
  // without the GLU epilogue), 0 above -- MI355X, Llama-3-8B shapes, sym_int4
  // (profiles/prefill_gemm_r3_*tile*.jsonl): twice the blocks on 256 CUs, M = 128 down 188 ->
  // 113 us, qkv 62 -> 40, M = 1024 qkv 95 -> 82, down 214 -> 184 (gate_up 318 -> 333: kept 0);
  // from M = 2048 the 128 x 128 block's x reuse wins (o 97 vs 108, gate_up 580 vs 640)
  static const int tile_env = getenv("ILLM_GEMM_TILE") ? atoi(getenv("ILLM_GEMM_TILE")) : -1;
  const int rows = a.moe_off != nullptr ? a.M / max(1, a.moe_el) : a.M;     // grouped: rows per expert
  const int tile = tile_env >= 0 ? tile_env : ((rows <= 768 || (rows <= 1024 && !a.glu)) ? 6 : 0);
  if (a.moe_off != nullptr) {                                                 // grouped MoE
    if (tile == 6) return launch_gemm_v<DK, 2, 4, 6>(bf16, a, st);
    return launch_gemm_v<DK, 2, 8, 4>(bf16, a, st);
  }
  const int tile_env2 = tile;
  if (tile_env2 == 2) launch_gemm_v<DK, 4, 4, 2>(bf16, a, st);
  else if (tile_env2 == 3) launch_gemm_v<DK, 4, 4, 2, 2>(bf16, a, st);
  else if (tile_env2 == 4) launch_gemm_v<DK, 4, 4, 3, 2>(bf16, a, st);
  else if (tile_env2 == 5) launch_gemm_v<DK, 2, 4, 4>(bf16, a, st);
  else if (tile_env2 == 6) launch_gemm_v<DK, 2, 4, 6>(bf16, a, st);
  else launch_gemm_v<DK, 2, 8, 4>(bf16, a, st);
}

__global__ void bf16_to_f16_sat_kernel(const uint4* x, uint4* y, int64_t n8) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const uint4 v = x[i];
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const float lo = fminf(fmaxf(bf16_to_f32(w[j] & 0xffff), -65504.f), 65504.f);
    const float hi = fminf(fmaxf(bf16_to_f32(w[j] >> 16), -65504.f), 65504.f);
    w[j] = pack2<F16>(lo, hi);
  }
  y[i] = make_uint4(w[0], w[1], w[2], w[3]);
}

void launch_bf16_to_f16_sat(const uint16_t* x, uint16_t* y, int64_t n, hipStream_t st) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  hipLaunchKernelGGL(bf16_to_f16_sat_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st,
                     (const uint4*)x, (uint4*)y, n8);
}

void launch_lowbit_gemm(bool bf16, int fmt, const GemmArgs& a, hipStream_t st) {
  switch (fmt_to_dk(fmt)) {
    case DK_INT4S: launch_gemm_dk<DK_INT4S>(bf16, a, st); break;
    case DK_INT4A: launch_gemm_dk<DK_INT4A>(bf16, a, st); break;
    case DK_LUT4: launch_gemm_dk<DK_LUT4>(bf16, a, st); break;
    case DK_FP4: launch_gemm_dk<DK_FP4>(bf16, a, st); break;
    case DK_INT8S: launch_gemm_dk<DK_INT8S>(bf16, a, st); break;
    case DK_INT8A: launch_gemm_dk<DK_INT8A>(bf16, a, st); break;
    case DK_FP8E4: launch_gemm_dk<DK_FP8E4>(bf16, a, st); break;
    case DK_FP8E5: launch_gemm_dk<DK_FP8E5>(bf16, a, st); break;
  }
}


// ---- per-row power-of-two normalisation of 16-bit x to f16 (the f16 MFMA
// input of the fused prefill GEMM, exact: x = y * rs)
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

void launch_x_to_f16_rowscale(bool bf16, const uint16_t* x, int64_t M, int64_t ldx, int K, uint16_t* y, float* rs,
                              hipStream_t st) {
  if (M <= 0) return;
  hipLaunchKernelGGL(x_to_f16_rowscale_kernel, dim3((unsigned)M), dim3(256), 0, st, x, ldx, K, bf16 ? 1 : 0, y, rs);
}

}  // namespace illm
