// Elementwise / small kernels: GLU activation, on-device quantize-on-load and
// dequant, split-K partial reduction, MoE router top-k.
//
// Reference ops: xe_addons.mlp_silu_mul_inplaced (models/qwen2.py:325-329),
// xe_linear.dequant (low_bit_linear.py:566-570), xe_addons.moe_softmax_topk /
// moe_group_topk (models/common.py:342-375), ggml_quantize_tensor done on
// the GPU instead of the host (low_bit_linear.py:180).
#include "../common/quant_block.h"
#include "illm_device.h"
#include "kernels.h"

namespace illm {

// ---- GLU: out[m, i] = act(gu[m, i]) * gu[m, I + i] ---------------------------
// tile > 0: gate / up interleaved in tile-row groups (the fused gate_up weight
// layout: columns [2 tile j, 2 tile j + tile) gate, the next tile up)
template <typename T>
__global__ void glu_kernel(const uint16_t* gu, int ld, uint16_t* out, int M, int I, int act, int tile) {
  const int64_t n8 = (int64_t)M * I / 8;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n8;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 8;
    const int m = (int)(e / I), i = (int)(e % I);
    const int gc = tile > 0 ? (i / tile) * 2 * tile + i % tile : i;
    const uint4 g = *(const uint4*)(gu + (size_t)m * ld + gc);
    const uint4 u = *(const uint4*)(gu + (size_t)m * ld + gc + (tile > 0 ? tile : I));
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, uw[4] = {u.x, u.y, u.z, u.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      float g0 = to_f32<T>(gw[j] & 0xffff), g1 = to_f32<T>(gw[j] >> 16);
      float u0 = to_f32<T>(uw[j] & 0xffff), u1 = to_f32<T>(uw[j] >> 16);
      // HF: act(gate) rounded to dtype, then * up rounded
      g0 = to_f32<T>(from_f32<T>(act == 0 ? silu_f(g0) : gelu_tanh_f(g0)));
      g1 = to_f32<T>(from_f32<T>(act == 0 ? silu_f(g1) : gelu_tanh_f(g1)));
      o[j] = pack2<T>(g0 * u0, g1 * u1);
    }
    *(uint4*)(out + (size_t)m * I + i) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void launch_glu(bool bf16, const uint16_t* gu, int ld, uint16_t* out, int M, int I, int act, int tile,
                hipStream_t st) {
  const int64_t n8 = (int64_t)M * I / 8;
  const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 4096);
  if (bf16) hipLaunchKernelGGL(glu_kernel<BF16>, dim3(blocks), dim3(256), 0, st, gu, ld, out, M, I, act, tile);
  else hipLaunchKernelGGL(glu_kernel<F16>, dim3(blocks), dim3(256), 0, st, gu, ld, out, M, I, act, tile);
}

// ---- in-place row softmax (eager attention weights) -------------------------
// Reference op: xe_addons.attn_softmax_inplaced (models/common.py:174-181).
// One wave64 per row, four rows per workgroup; f32 math, result rounded to T.
// A fully masked row (max = -inf) is written as zeros.
template <typename T>
__global__ void __launch_bounds__(256) softmax_rows_kernel(uint16_t* x, int64_t rows, int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  if (row >= rows) return;   // whole wave leaves together; no block barrier below
  const int lane = threadIdx.x & 63;
  uint16_t* p = x + row * (int64_t)L;
  float m = -INFINITY;
  for (int i = lane; i < L; i += 64) m = fmaxf(m, to_f32<T>(p[i]));
  m = wave_max(m);
  float s = 0.f;
  if (m != -INFINITY)
    for (int i = lane; i < L; i += 64) s += __expf(to_f32<T>(p[i]) - m);
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  for (int i = lane; i < L; i += 64) p[i] = from_f32<T>(s > 0.f ? __expf(to_f32<T>(p[i]) - m) * inv : 0.f);
}

void launch_softmax_rows(bool bf16, uint16_t* x, int64_t rows, int L, hipStream_t st) {
  const int64_t blocks = (rows + 3) / 4;
  if (bf16) hipLaunchKernelGGL(softmax_rows_kernel<BF16>, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, L);
  else hipLaunchKernelGGL(softmax_rows_kernel<F16>, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, L);
}

// ---- quantize on device: dense [n, k] -> MI355X tiled blob ------------------
__device__ __forceinline__ float load_in(const void* w, int kind, size_t i) {
  if (kind == 0) return ((const float*)w)[i];
  if (kind == 1) return bf16_to_f32(((const uint16_t*)w)[i]);
  return f16_to_f32(((const uint16_t*)w)[i]);
}

__global__ void quantize_device_kernel(int fmt, int kind, const void* w, int64_t n, int64_t k,
                                       uint8_t* blob, int search) {
  const int64_t nb = k / QBLOCK;
  const int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (id >= n * nb) return;
  const int64_t row = id / nb, b = id % nb;
  float x[QBLOCK];
  for (int i = 0; i < QBLOCK; i++) x[i] = load_in(w, kind, (size_t)row * k + b * QBLOCK + i);
  uint8_t codes[QBLOCK];
  float d, m;
  hd_quant_block(fmt, x, nullptr, search != 0, codes, &d, &m);

  const int bits = fmt_bits(fmt);
  const int64_t KC = pad_to(k, CHUNK_K) / CHUNK_K;
  const int64_t t = row / TILE_N;
  const int r = (int)(row % TILE_N);
  const int64_t c = b / 2;
  const int blk = (int)(b % 2);
  uint8_t* tile = blob + t * dev_tile_bytes(fmt, KC);
  uint8_t* rec = tile + c * dev_code_chunk(fmt);
  if (bits == 4) {
    for (int ss = 0; ss < 2; ss++) {
      const int s = 2 * blk + ss;
      for (int g = 0; g < 4; g++) {
        uint32_t u = 0;
        for (int j = 0; j < 8; j++) u |= (uint32_t)(codes[32 * ss + 8 * g + j] & 15) << (4 * dev_nib_pos(fmt, j));
        const int l = g * 16 + r;
        ((uint32_t*)(rec + l * 16))[s] = u;
      }
    }
  } else {
    for (int g = 0; g < 4; g++) {
      const int l = g * 16 + r;
      uint8_t* o = rec + (blk * 64 + l) * 16;
      uint32_t wv[4];
      for (int q = 0; q < 4; q++) {
        const int ss = q / 2, j0 = (q % 2) * 4;
        const uint8_t* cc = codes + 32 * ss + 8 * g + j0;
        wv[q] = (uint32_t)cc[0] | ((uint32_t)cc[1] << 8) | ((uint32_t)cc[2] << 16) | ((uint32_t)cc[3] << 24);
      }
      *(uint4*)o = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
  }
  ((uint16_t*)(tile + dev_scale_off(fmt, KC, r, c)))[blk] = hd_f32_to_f16(d);
  if (fmt_has_min(fmt)) ((uint16_t*)(tile + dev_min_off(fmt, KC, r, c)))[blk] = hd_f32_to_f16(m);
}

void launch_quantize_device(int fmt, int in_kind, const void* w, int64_t n, int64_t k,
                            uint8_t* blob, int search, hipStream_t st) {
  hipMemsetAsync(blob, 0, dev_total_bytes(fmt, n, k), st);
  const int64_t tot = n * (k / QBLOCK);
  hipLaunchKernelGGL(quantize_device_kernel, dim3((unsigned)((tot + 127) / 128)), dim3(128), 0, st, fmt,
                     in_kind, w, n, k, blob, search);
}

// ---- dequantize on device: tiled blob -> dense [n, k] ------------------------
// Used by the library-GEMM prefill path (a transient dense weight per call).
// A workgroup of 4 waves decodes 4 consecutive 128-k chunks of one 16-row
// tile: each lane decodes its MFMA-fragment codes (row l & 15, k-group l >> 4,
// the GEMV's lane mapping, full 1 KiB wave loads) into an LDS [16][512] row
// block, then every wave store writes 1 KiB of ONE output row.  Storing the
// fragments directly left each wave store as 16 separate 64-B row pieces
// (~4.2 TB/s of weight bytes in + out on MI355X).  The format is a template
// parameter so the per-element code decode folds to constants.
constexpr int DQ_CH = 4;                                  // chunks per workgroup
constexpr int DQ_LD = DQ_CH * CHUNK_K + 8;                // LDS row stride (elements)
template <typename T, int FMT>
__global__ void __launch_bounds__(256) dequantize_tiled_kernel(const uint8_t* blob, int64_t n, int64_t k,
                                                               uint16_t* out) {
  constexpr int fmt = FMT;
  constexpr int bits = fmt_bits(fmt);
  __shared__ __attribute__((aligned(16))) uint16_t rows[TILE_N * DQ_LD];
  // 16-entry code tables (nf4 / fp4 / nf3) from LDS: a dynamically indexed
  // local array goes to scratch (nf4 ran at 3-4 TB/s vs 5-6 for sym_int4)
  constexpr bool LUT = fmt == FMT_NF4 || fmt == FMT_FP4 || fmt == FMT_NF3;
  __shared__ float lut[16];
  if constexpr (LUT) {
    if (threadIdx.x < 16) lut[threadIdx.x] = hd_lut4(fmt, threadIdx.x);
    __syncthreads();
  }
  const int64_t KC = pad_to(k, CHUNK_K) / CHUNK_K;
  const int64_t ncg = (KC + DQ_CH - 1) / DQ_CH;
  const int64_t t = blockIdx.x / ncg, cg = blockIdx.x % ncg;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int r = l & 15, g = l >> 4;
  const int64_t c = cg * DQ_CH + w;
  const uint8_t* tile = blob + t * dev_tile_bytes(fmt, KC);
  if (c < KC) {
    const uint8_t* rec = tile + c * dev_code_chunk(fmt);
    uint32_t wd[bits == 4 ? 4 : 8];
    {
      const uint4 q = *(const uint4*)(rec + l * 16);
      wd[0] = q.x; wd[1] = q.y; wd[2] = q.z; wd[3] = q.w;
      if constexpr (bits != 4) {
        const uint4 q1 = *(const uint4*)(rec + (64 + l) * 16);
        wd[4] = q1.x; wd[5] = q1.y; wd[6] = q1.z; wd[7] = q1.w;
      }
    }
    const uint16_t* sp = (const uint16_t*)(tile + dev_scale_off(fmt, KC, r, c));
    const uint16_t* mp = fmt_has_min(fmt) ? (const uint16_t*)(tile + dev_min_off(fmt, KC, r, c)) : nullptr;
#pragma unroll
    for (int s = 0; s < 4; s++) {                          // k-step s: elements 32 s + 8 g .. + 7
      const int blk = s >> 1;
      const float d = f16_to_f32(sp[blk]);
      const float m = fmt_has_min(fmt) ? f16_to_f32(mp[blk]) : 0.f;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        int code;
        // 4-bit: dword s = k-step s; 8-bit: half h = s / 2, dwords 2 (s % 2) .. + 1
        if (bits == 4) code = (wd[s] >> (4 * dev_nib_pos(fmt, j))) & 15;
        else code = (wd[4 * (s >> 1) + 2 * (s & 1) + (j >> 2)] >> (8 * (j & 3))) & 0xff;
        v[j] = (LUT ? lut[code & 15] : hd_code_value(fmt, code)) * d + m;
      }
      *(uint4*)(rows + r * DQ_LD + w * CHUNK_K + 32 * s + 8 * g) =
          make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7]));
    }
  }
  __syncthreads();
  // row segment [cg * 512, cg * 512 + 512) of rows t * 16 .. + 15: 64 x 16-B pieces per row
  const int64_t k0 = cg * DQ_CH * CHUNK_K;
#pragma unroll
  for (int j = 0; j < TILE_N * DQ_CH * CHUNK_K / 8 / 256; j++) {
    const int v = tid + 256 * j;
    const int rr = v / (DQ_CH * CHUNK_K / 8), col = (v % (DQ_CH * CHUNK_K / 8)) * 8;
    const int64_t row = t * TILE_N + rr, kk = k0 + col;
    if (row < n && kk + 8 <= k) *(uint4*)(out + (size_t)row * k + kk) = *(const uint4*)(rows + rr * DQ_LD + col);
  }
}

// Transposed output [k, n] (the W^T operand of grad_x = g W): a workgroup
// decodes ONE 128-k chunk of FOUR consecutive 16-row tiles (one per wave) into
// LDS [64 n][128 k], then stores per k one 128-B run of 64 n values, 8 lanes
// per run.  The row-block kernel above wrote 32-B runs (its tile's 16 n per k).
constexpr int DQT_TILES = 4;
constexpr int DQT_LD = CHUNK_K + 8;
template <typename T, int FMT>
__global__ void __launch_bounds__(256) dequantize_tiled_tr_kernel(const uint8_t* blob, int64_t n, int64_t k,
                                                                  uint16_t* out) {
  constexpr int fmt = FMT;
  constexpr int bits = fmt_bits(fmt);
  __shared__ __attribute__((aligned(16))) uint16_t rows[DQT_TILES * TILE_N * DQT_LD];
  // 16-entry code tables (nf4 / fp4 / nf3) from LDS: a dynamically indexed
  // local array goes to scratch (nf4 ran at 3-4 TB/s vs 5-6 for sym_int4)
  constexpr bool LUT = fmt == FMT_NF4 || fmt == FMT_FP4 || fmt == FMT_NF3;
  __shared__ float lut[16];
  if constexpr (LUT) {
    if (threadIdx.x < 16) lut[threadIdx.x] = hd_lut4(fmt, threadIdx.x);
    __syncthreads();
  }
  const int64_t KC = pad_to(k, CHUNK_K) / CHUNK_K, NT = pad_to(n, TILE_N) / TILE_N;
  const int64_t tg = blockIdx.x / KC, c = blockIdx.x % KC;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int r = l & 15, g = l >> 4;
  const int64_t t = tg * DQT_TILES + w;
  if (t < NT) {
    const uint8_t* tile = blob + t * dev_tile_bytes(fmt, KC);
    const uint8_t* rec = tile + c * dev_code_chunk(fmt);
    uint32_t wd[bits == 4 ? 4 : 8];
    {
      const uint4 q = *(const uint4*)(rec + l * 16);
      wd[0] = q.x; wd[1] = q.y; wd[2] = q.z; wd[3] = q.w;
      if constexpr (bits != 4) {
        const uint4 q1 = *(const uint4*)(rec + (64 + l) * 16);
        wd[4] = q1.x; wd[5] = q1.y; wd[6] = q1.z; wd[7] = q1.w;
      }
    }
    const uint16_t* sp = (const uint16_t*)(tile + dev_scale_off(fmt, KC, r, c));
    const uint16_t* mp = fmt_has_min(fmt) ? (const uint16_t*)(tile + dev_min_off(fmt, KC, r, c)) : nullptr;
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int blk = s >> 1;
      const float d = f16_to_f32(sp[blk]);
      const float m = fmt_has_min(fmt) ? f16_to_f32(mp[blk]) : 0.f;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        int code;
        if (bits == 4) code = (wd[s] >> (4 * dev_nib_pos(fmt, j))) & 15;
        else code = (wd[4 * (s >> 1) + 2 * (s & 1) + (j >> 2)] >> (8 * (j & 3))) & 0xff;
        v[j] = (LUT ? lut[code & 15] : hd_code_value(fmt, code)) * d + m;
      }
      *(uint4*)(rows + (w * TILE_N + r) * DQT_LD + 32 * s + 8 * g) =
          make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7]));
    }
  }
  __syncthreads();
  const int64_t n0 = tg * DQT_TILES * TILE_N, k0 = c * CHUNK_K;
  // each thread: two adjacent k (one 4-B LDS read per n) x 8 n -> two 16-B stores
#pragma unroll
  for (int p = 0; p < CHUNK_K / 2 * DQT_TILES * TILE_N / 8 / 256; p++) {
    const int v = tid + 256 * p;
    const int kk = (v >> 3) * 2, nl = (v & 7) * 8;
    const int64_t kg = k0 + kk, ng = n0 + nl;
    if (kg >= k || ng + 8 > n) continue;
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = *(const uint32_t*)(rows + (nl + i) * DQT_LD + kk);
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      lo[i] = __builtin_amdgcn_perm(a[2 * i + 1], a[2 * i], 0x05040100u);   // low halves: k = kk
      hi[i] = __builtin_amdgcn_perm(a[2 * i + 1], a[2 * i], 0x07060302u);   // high halves: k = kk + 1
    }
    *(uint4*)(out + (size_t)kg * n + ng) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    if (kg + 1 < k) *(uint4*)(out + (size_t)(kg + 1) * n + ng) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
  }
}

void launch_dequantize_device(bool bf16, int fmt, const uint8_t* blob, int64_t n, int64_t k,
                              uint16_t* out, hipStream_t st, bool transpose) {
  const int64_t KC = pad_to(k, CHUNK_K) / CHUNK_K;
  const int64_t NT = pad_to(n, TILE_N) / TILE_N;
  const int64_t nblk = NT * ((KC + DQ_CH - 1) / DQ_CH);
  dim3 grid((unsigned)nblk), gridt((unsigned)(((NT + DQT_TILES - 1) / DQT_TILES) * KC));
#define DQ_CASE(F)                                                                                       \
  case F:                                                                                                \
    if (transpose) {                                                                                     \
      if (bf16) hipLaunchKernelGGL((dequantize_tiled_tr_kernel<BF16, F>), gridt, dim3(256), 0, st, blob, n, k, out); \
      else hipLaunchKernelGGL((dequantize_tiled_tr_kernel<F16, F>), gridt, dim3(256), 0, st, blob, n, k, out);       \
    } else if (bf16) {                                                                                   \
      hipLaunchKernelGGL((dequantize_tiled_kernel<BF16, F>), grid, dim3(256), 0, st, blob, n, k, out); \
    } else {                                                                                             \
      hipLaunchKernelGGL((dequantize_tiled_kernel<F16, F>), grid, dim3(256), 0, st, blob, n, k, out);  \
    }                                                                                                    \
    break;
  switch (fmt) {
    DQ_CASE(FMT_SYM_INT4) DQ_CASE(FMT_ASYM_INT4) DQ_CASE(FMT_NF4) DQ_CASE(FMT_FP4) DQ_CASE(FMT_SYM_INT8)
    DQ_CASE(FMT_FP8E4) DQ_CASE(FMT_FP8E5) DQ_CASE(FMT_SYM_INT5) DQ_CASE(FMT_ASYM_INT5) DQ_CASE(FMT_NF3)
    DQ_CASE(FMT_FP6)
  }
#undef DQ_CASE
}

// ---- sum split-K partial slabs (+bias) -> T ----------------------------------
template <typename T>
__global__ void reduce_partials_kernel(const float* ws, int nsplit, const uint16_t* bias,
                                       uint16_t* out, int M, int N, int ldo) {
  const int64_t tot = (int64_t)M * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / N), n = (int)(i % N);
    float acc = 0.f;
    for (int s = 0; s < nsplit; s++) acc += ws[(size_t)s * tot + i];
    if (bias) acc += to_f32<T>(bias[n]);
    out[(size_t)m * ldo + n] = from_f32<T>(acc);
  }
}

void launch_reduce_partials(bool bf16, const float* ws, int nsplit, const uint16_t* bias,
                            uint16_t* out, int M, int N, int ldo, hipStream_t st) {
  const int64_t tot = (int64_t)M * N;
  const int blocks = (int)std::min<int64_t>((tot + 255) / 256, 2048);
  if (bf16) hipLaunchKernelGGL(reduce_partials_kernel<BF16>, dim3(blocks), dim3(256), 0, st, ws, nsplit, bias, out, M, N, ldo);
  else hipLaunchKernelGGL(reduce_partials_kernel<F16>, dim3(blocks), dim3(256), 0, st, ws, nsplit, bias, out, M, N, ldo);
}

// ---- MoE router: softmax / sigmoid + top-k (+renormalise) --------------------
// one wave per token row, E <= 512.  SC1: the logits were handed over by other
// workgroups of the same launch (sc1 loads).  ids_lds (optional) receives the
// chosen ids for a following in-workgroup align.
// nsp > 1: the logits are nsp partial sums, sp_stride floats apart.
template <bool SC1>
__device__ __forceinline__ void topk_row(const float* lrow, int E, int k, int renorm, int scoring, float* w_out,
                                         int32_t* id_out, int* ids_lds, int nsp = 1, size_t sp_stride = 0) {
  const int lane = threadIdx.x & 63;
  constexpr int PER = 8;
  float v[PER];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int e = lane + 64 * j;
    float x = -INFINITY;
    if (e < E) {
      x = 0.f;
      for (int sp = 0; sp < nsp; sp++) x += SC1 ? ld_sc1(lrow + sp * sp_stride + e) : lrow[sp * sp_stride + e];
    }
    v[j] = x;
    mx = fmaxf(mx, v[j]);
  }
  if (scoring == 0) {
    mx = wave_max(mx);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      v[j] = (lane + 64 * j) < E ? __expf(v[j] - mx) : 0.f;
      s += v[j];
    }
    s = wave_sum(s);
#pragma unroll
    for (int j = 0; j < PER; j++) v[j] /= s;
  } else {
#pragma unroll
    for (int j = 0; j < PER; j++) v[j] = (lane + 64 * j) < E ? 1.f / (1.f + __expf(-v[j])) : -1.f;
  }
  float tot = 0.f;
  float wsel = 0.f;                // lane i keeps the i-th chosen weight
  for (int i = 0; i < k; i++) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int e = lane + 64 * j;
      if (e < E && (v[j] > best || (v[j] == best && e < bi))) { best = v[j]; bi = e; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
#pragma unroll
    for (int j = 0; j < PER; j++)
      if (lane + 64 * j == bi) v[j] = -INFINITY;
    if (lane == i) {
      wsel = best;
      id_out[i] = bi;
      if (ids_lds) ids_lds[i] = bi;
    }
    tot += best;
  }
  if (lane < k) w_out[lane] = renorm ? wsel / tot : wsel;
}

__global__ void __launch_bounds__(64) moe_topk_kernel(const float* logits, int T, int E, int k,
                                                      int renorm, int scoring, float* topk_w,
                                                      int32_t* topk_ids) {
  const int t = blockIdx.x;
  topk_row<false>(logits + (size_t)t * E, E, k, renorm, scoring, topk_w + (size_t)t * k, topk_ids + (size_t)t * k,
                  nullptr);
}

// ---- fused decode router (T <= 16 tokens): logits = x Wr^T in f32, softmax /
// sigmoid top-k (+renormalise) and the per-expert pair lists of moe_align in
// ONE launch.  The last workgroup to finish
// (agent-scope counter, sc1 hand-off) runs top-k per token and the align.
// Workgroup = (expert, hidden slice of 2048): one 16-B chunk of the router
// row per thread, so every load is in flight at once; the last workgroup sums
// the slices' partial logits.
// Replaces router GEMM + f32 cast + moe_topk + moe_align (4 launches).
// top-k per token (one wave each) + per-local-expert pair lists, run by one
// workgroup of NT threads over logits lg [T, E] (SC1: handed over by other
// workgroups of the launch)
template <bool SC1, int NT>
__device__ __forceinline__ void route_tail(const MoeRouteArgs& a, const float* lg) {
  const int wave = threadIdx.x >> 6;
  __shared__ int ids_l[16 * 16];
  __shared__ int cnt[512], start[512];
  for (int t = wave; t < a.T; t += NT / 64)
    topk_row<SC1>(lg + (size_t)t * a.E, a.E, a.k, a.renorm, a.scoring, a.topk_w + (size_t)t * a.k,
                  a.topk_ids + (size_t)t * a.k, ids_l + t * a.k, a.nsp, (size_t)a.T * a.E);
  for (int i = threadIdx.x; i < a.El; i += NT) cnt[i] = 0;
  __syncthreads();
  const int P = a.T * a.k;
  for (int p = threadIdx.x; p < P; p += NT) {
    const int el = ids_l[p] - a.e0;
    if (el >= 0 && el < a.El) atomicAdd(&cnt[el], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < a.El; i++) {
      start[i] = acc;
      a.off[i] = acc;
      acc += cnt[i];
    }
    a.off[a.El] = acc;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += NT) {
    const int id = ids_l[p], el = id - a.e0;
    if (el < 0 || el >= a.El) continue;
    int r = 0;
    for (int q = 0; q < p; q++) r += ids_l[q] == id;
    a.rows[start[el] + r] = p;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) moe_route_kernel(const MoeRouteArgs a) {
  constexpr int TM = 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e = blockIdx.x, sp = blockIdx.y;
  __shared__ float red[4][TM];
  {
    float acc[TM];
#pragma unroll
    for (int t = 0; t < TM; t++) acc[t] = 0.f;
    const uint16_t* wrow = a.wr + (size_t)e * a.H;
    const int nc = a.H / 8;
    for (int c = sp * 256 + threadIdx.x; c < nc; c += 256 * a.nsp) {
      const uint4 wv = *(const uint4*)(wrow + 8 * c);
      const uint32_t ww[4] = {wv.x, wv.y, wv.z, wv.w};
      float wf[8];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        wf[2 * i] = to_f32<T>((uint16_t)(ww[i] & 0xffff));
        wf[2 * i + 1] = to_f32<T>((uint16_t)(ww[i] >> 16));
      }
#pragma unroll
      for (int t = 0; t < TM; t++) {
        if (t < a.T) {
          const uint4 xv = *(const uint4*)(a.x + (size_t)t * a.H + 8 * c);
          const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            acc[t] = __builtin_fmaf(wf[2 * i], to_f32<T>((uint16_t)(xw[i] & 0xffff)), acc[t]);
            acc[t] = __builtin_fmaf(wf[2 * i + 1], to_f32<T>((uint16_t)(xw[i] >> 16)), acc[t]);
          }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < TM; t++) {
      if (t < a.T) {
        const float v = wave_sum(acc[t]);
        if (lane == 0) red[wave][t] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x < a.T) {
      const int t = threadIdx.x;
      st_sc1(a.logits + ((size_t)sp * a.T + t) * a.E + e, red[0][t] + red[1][t] + red[2][t] + red[3][t]);
    }
  }
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // this wave's sc1 stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(a.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = prev == (int)(gridDim.x * gridDim.y) - 1;
    if (is_last) __hip_atomic_store(a.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!is_last) return;

  route_tail<true, 256>(a, a.logits);
}

void launch_moe_route(bool bf16, const MoeRouteArgs& a, hipStream_t st) {
  // (expert, hidden slice) workgroups: one 16-B chunk of the router row per thread
  const dim3 grid((unsigned)a.E, (unsigned)a.nsp);
  if (bf16) hipLaunchKernelGGL(moe_route_kernel<BF16>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(moe_route_kernel<F16>, grid, dim3(256), 0, st, a);
}

// ---- DeepSeek-V3 group-limited router (noaux_tc): sigmoid scores, + the
// e_score_correction_bias for the choice, groups ranked by the sum of their
// top-2 choice scores, top-k among the experts of the top `topk_group` groups,
// weights = un-biased scores (renormalised) * routed_scaling_factor.
// Reference: xe_addons.moe_group_topk (models/common.py:342-351,
// deepseek.py:274-290).  One wave per token; E <= 512, n_group <= 64.
__global__ void __launch_bounds__(64) moe_group_topk_kernel(const float* logits, const float* bias, int T, int E,
                                                            int k, int n_group, int topk_group, int renorm,
                                                            float scale, float* topk_w, int32_t* topk_ids) {
  const int t = blockIdx.x, lane = threadIdx.x;
  constexpr int PER = 8;
  __shared__ float sfc[512];
  __shared__ float gsc[64];
  __shared__ int gsel[64];
  float sc[PER], ch[PER];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int e = lane + 64 * j;
    const float l = e < E ? logits[(size_t)t * E + e] : 0.f;
    sc[j] = 1.f / (1.f + __expf(-l));
    ch[j] = e < E ? sc[j] + (bias ? bias[e] : 0.f) : -INFINITY;
    if (e < E) sfc[e] = ch[j];
  }
  __syncthreads();
  const int gs = E / n_group;
  if (lane < n_group) {
    float b1 = -INFINITY, b2 = -INFINITY;
    for (int i = 0; i < gs; i++) {
      const float v = sfc[lane * gs + i];
      if (v > b1) { b2 = b1; b1 = v; } else if (v > b2) { b2 = v; }
    }
    gsc[lane] = b1 + (gs > 1 ? b2 : 0.f);
    gsel[lane] = 0;
  }
  __syncthreads();
  if (lane == 0) {
    for (int i = 0; i < topk_group; i++) {
      int bi = -1;
      float best = -INFINITY;
      for (int g = 0; g < n_group; g++)
        if (!gsel[g] && (bi < 0 || gsc[g] > best)) { best = gsc[g]; bi = g; }
      if (bi >= 0) gsel[bi] = 1;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int e = lane + 64 * j;
    if (e < E && !gsel[e / gs]) ch[j] = -INFINITY;
  }
  float tot = 0.f;
  for (int i = 0; i < k; i++) {
    float best = -INFINITY, bw = 0.f;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER; j++) {
      const int e = lane + 64 * j;
      if (e < E && (ch[j] > best || (ch[j] == best && e < bi))) { best = ch[j]; bi = e; bw = sc[j]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      const float ow = __shfl_xor(bw, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; bw = ow; }
    }
#pragma unroll
    for (int j = 0; j < PER; j++)
      if (lane + 64 * j == bi) ch[j] = -INFINITY;
    if (lane == 0) {
      topk_w[(size_t)t * k + i] = bw;
      topk_ids[(size_t)t * k + i] = bi;
    }
    tot += bw;
  }
  if (lane == 0) {
    const float f = renorm ? scale / (tot + 1e-20f) : scale;
    for (int i = 0; i < k; i++) topk_w[(size_t)t * k + i] *= f;
  }
}

void launch_moe_group_topk(const float* logits, const float* bias, int T, int E, int k, int n_group, int topk_group,
                           int renorm, float scale, float* topk_w, int32_t* topk_ids, hipStream_t st) {
  hipLaunchKernelGGL(moe_group_topk_kernel, dim3(T), dim3(64), 0, st, logits, bias, T, E, k, n_group, topk_group,
                     renorm, scale, topk_w, topk_ids);
}

void launch_moe_topk(const float* logits, int T, int E, int k, int renorm, int scoring,
                     float* topk_w, int32_t* topk_ids, hipStream_t st) {
  hipLaunchKernelGGL(moe_topk_kernel, dim3(T), dim3(64), 0, st, logits, T, E, k, renorm, scoring,
                     topk_w, topk_ids);
}

// ---- MoE routing bookkeeping (device side, graph-capturable) ---------------
// ids [P] (P = T*k, row-major top-k) -> per-local-expert pair lists:
// off[e]..off[e+1] index rows[], rows sorted by (expert, pair id).  Experts
// outside [e0, e0+El) (other EP ranks) are skipped.
__global__ void __launch_bounds__(1024) moe_align_kernel(const int32_t* ids, int P, int e0, int El,
                                                         int32_t* off, int32_t* rows) {
  extern __shared__ int sh[];  // cnt[El] | start[El]
  int* cnt = sh;
  int* start = sh + El;
  for (int e = threadIdx.x; e < El; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const int e = ids[p] - e0;
    if (e >= 0 && e < El) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < El; e++) {
      start[e] = acc;
      off[e] = acc;
      acc += cnt[e];
    }
    off[El] = acc;
  }
  __syncthreads();
  // slot within the expert from an LDS cursor: O(P) (the within-expert order
  // is free -- every consumer indexes rows by pair id)
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const int e = ids[p] - e0;
    if (e < 0 || e >= El) continue;
    rows[atomicAdd(&start[e], 1)] = p;
  }
}

void launch_moe_align(const int32_t* ids, int P, int e0, int El, int32_t* off, int32_t* rows, hipStream_t st) {
  hipLaunchKernelGGL(moe_align_kernel, dim3(1), dim3(1024), (size_t)2 * El * sizeof(int), st, ids, P, e0, El,
                     off, rows);
}

// out[t, h] = sum_j w[t, j] * sum_s part[s, t*k + j, h] over local experts
template <typename T>
__global__ void moe_combine_kernel(const float* part, int ks, int P, const float* w, const int32_t* ids, int k,
                                   int e0, int El, uint16_t* out, int Tn, int H) {
  const int t = blockIdx.y;
  const int h = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (h >= H) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j = 0; j < k; j++) {
    const int p = t * k + j;
    const int e = ids[p] - e0;
    if (e < 0 || e >= El) continue;
    const float wj = w[p];
    for (int s = 0; s < ks; s++) {
      const float4 v = *(const float4*)(part + ((size_t)s * P + p) * H + h);
      acc.x += wj * v.x; acc.y += wj * v.y; acc.z += wj * v.z; acc.w += wj * v.w;
    }
  }
  *(uint2*)(out + (size_t)t * H + h) = make_uint2(pack2<T>(acc.x, acc.y), pack2<T>(acc.z, acc.w));
}

void launch_moe_combine(bool bf16, const float* part, int ks, int P, const float* w, const int32_t* ids, int k,
                        int e0, int El, uint16_t* out, int Tn, int H, hipStream_t st) {
  dim3 grid((unsigned)((H / 4 + 255) / 256), (unsigned)Tn);
  if (bf16) hipLaunchKernelGGL(moe_combine_kernel<BF16>, grid, dim3(256), 0, st, part, ks, P, w, ids, k, e0, El, out, Tn, H);
  else hipLaunchKernelGGL(moe_combine_kernel<F16>, grid, dim3(256), 0, st, part, ks, P, w, ids, k, e0, El, out, Tn, H);
}

// ---- act(gate) * up for two separate [.., I] tensors (the HF MLP form used in
// training) and its gradient, with HF's rounding: a = rnd(act(g)), y = rnd(a u);
// backward du = rnd(dy a), dg = rnd(rnd(dy u) act'(g)).  act: 0 silu, 1 gelu-tanh.
// 8 elements per thread, 16-B accesses.
template <typename T>
__global__ void __launch_bounds__(256) act_mul_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u,
                                                      const uint16_t* __restrict__ dy, uint16_t* __restrict__ y,
                                                      uint16_t* __restrict__ dg, uint16_t* __restrict__ du,
                                                      int64_t n8, int act) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  auto ld8 = [](const uint16_t* p, int64_t i, float* v) {
    const uint4 q = ((const uint4*)p)[i];
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int e = 0; e < 4; e++) { v[2 * e] = to_f32<T>(w[e] & 0xffff); v[2 * e + 1] = to_f32<T>(w[e] >> 16); }
  };
  auto st8 = [](uint16_t* p, int64_t i, const float* v) {
    ((uint4*)p)[i] = make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7]));
  };
  auto r = [](float v) { return to_f32<T>(from_f32<T>(v)); };
  float gv[8], uv[8];
  ld8(g, i, gv);
  ld8(u, i, uv);
  if (dy == nullptr) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; e++) o[e] = r(act == 0 ? silu_f(gv[e]) : gelu_tanh_f(gv[e])) * uv[e];
    st8(y, i, o);
    return;
  }
  float d[8], og[8], ou[8];
  ld8(dy, i, d);
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const float x = gv[e];
    float a, da;
    if (act == 0) {
      const float sg = 1.f / (1.f + __expf(-x));
      a = x * sg;
      da = sg * (1.f + x * (1.f - sg));
    } else {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      const float inner = k0 * (x + k1 * x * x * x);
      const float th = tanhf(inner);
      a = 0.5f * x * (1.f + th);
      da = 0.5f * (1.f + th) + 0.5f * x * (1.f - th * th) * k0 * (1.f + 3.f * k1 * x * x);
    }
    ou[e] = d[e] * r(a);
    og[e] = r(d[e] * uv[e]) * da;
  }
  st8(dg, i, og);
  st8(du, i, ou);
}

void launch_act_mul(bool bf16, const uint16_t* g, const uint16_t* u, const uint16_t* dy, uint16_t* y, uint16_t* dg,
                    uint16_t* du, int64_t n, int act, hipStream_t s) {
  const int64_t n8 = n / 8;
  if (n8 == 0) return;
  const dim3 grid((unsigned)((n8 + 255) / 256));
  if (bf16) hipLaunchKernelGGL(act_mul_kernel<BF16>, grid, dim3(256), 0, s, g, u, dy, y, dg, du, n8, act);
  else hipLaunchKernelGGL(act_mul_kernel<F16>, grid, dim3(256), 0, s, g, u, dy, y, dg, du, n8, act);
}

// ---- rotate-half RoPE on [B, H, T, D] activations (training / HF-forward path)
// out = x cos + rotate_half(x) sin with HF's bf16 rounding (each product, then
// the sum), x with any batch / head / token strides (the transposed q / k
// projection views) and D contiguous; cos / sin [Bc, T, D] (Bc = B or 1).
// bwd: the transposed rotation for the gradient, dx = g cos - rotate_half(g sin)
// (reference: the rotary wrappers of SRC/transformers/models/common.py and
// their xe_addons kernels; here also differentiated for QLoRA).
template <typename T>
__global__ void __launch_bounds__(256) rope_half_kernel(const uint16_t* __restrict__ x, int64_t sb, int64_t sh,
                                                        int64_t st, const uint16_t* __restrict__ cs,
                                                        const uint16_t* __restrict__ sn, int64_t csb,
                                                        uint16_t* __restrict__ out, int B, int H, int Tn, int D,
                                                        int bwd) {
  const int half = D / 2, per_row = half / 4;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / per_row;
  if (row >= (int64_t)B * H * Tn) return;
  const int j = (int)(gid % per_row) * 4;
  const int t = (int)(row % Tn), h = (int)((row / Tn) % H), b = (int)(row / ((int64_t)Tn * H));
  const uint16_t* xr = x + b * sb + h * sh + t * st;
  const size_t co = (size_t)b * csb + (size_t)t * D;
  auto ld4 = [](const uint16_t* p, float* v) {
    const uint2 u = *(const uint2*)p;
    v[0] = to_f32<T>(u.x & 0xffff); v[1] = to_f32<T>(u.x >> 16);
    v[2] = to_f32<T>(u.y & 0xffff); v[3] = to_f32<T>(u.y >> 16);
  };
  float x1[4], x2[4], c1[4], c2[4], s1[4], s2[4], o1[4], o2[4];
  ld4(xr + j, x1); ld4(xr + half + j, x2);
  ld4(cs + co + j, c1); ld4(cs + co + half + j, c2);
  ld4(sn + co + j, s1); ld4(sn + co + half + j, s2);
  auto r = [](float v) { return to_f32<T>(from_f32<T>(v)); };
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (!bwd) {
      o1[i] = r(x1[i] * c1[i]) + r(-x2[i] * s1[i]);
      o2[i] = r(x2[i] * c2[i]) + r(x1[i] * s2[i]);
    } else {
      o1[i] = r(x1[i] * c1[i]) + r(x2[i] * s2[i]);
      o2[i] = r(x2[i] * c2[i]) - r(x1[i] * s1[i]);
    }
  }
  uint16_t* orow = out + (size_t)row * D;
  *(uint2*)(orow + j) = make_uint2(pack2<T>(o1[0], o1[1]), pack2<T>(o1[2], o1[3]));
  *(uint2*)(orow + half + j) = make_uint2(pack2<T>(o2[0], o2[1]), pack2<T>(o2[2], o2[3]));
}

void launch_rope_half(bool bf16, const uint16_t* x, int64_t sb, int64_t sh, int64_t st, const uint16_t* cs,
                      const uint16_t* sn, int64_t csb, uint16_t* out, int B, int H, int Tn, int D, int bwd,
                      hipStream_t s) {
  const int64_t n = (int64_t)B * H * Tn * (D / 8);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (bf16) hipLaunchKernelGGL(rope_half_kernel<BF16>, grid, dim3(256), 0, s, x, sb, sh, st, cs, sn, csb, out, B, H, Tn, D, bwd);
  else hipLaunchKernelGGL(rope_half_kernel<F16>, grid, dim3(256), 0, s, x, sb, sh, st, cs, sn, csb, out, B, H, Tn, D, bwd);
}

// ---- low-bit embedding gather: canonical blob rows -> dense [T, k] --------------
// (reference xe_linear.dequantize_rows, SRC/transformers/embedding.py:213-224)
template <typename T>
__global__ void embedding_rows_kernel(const uint8_t* blob, int fmt, const int64_t* ids, int64_t n, int64_t k,
                                      uint16_t* out, int* err) {
  const int t = blockIdx.y;
  const int64_t kk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (kk >= k) return;
  int64_t row = ids[t];
  if (row < 0 || row >= n) {                       // out-of-vocabulary id: clamped, reported
    if (kk == 0) kerr(err, ERR_TOKEN);
    row = row < 0 ? 0 : n - 1;
  }
  const int bits = fmt_bits(fmt);
  const int64_t nb = k / QBLOCK;
  const uint8_t* codes = blob + row * (k * bits / 8);
  const uint16_t* scales = (const uint16_t*)(blob + canon_code_bytes(fmt, n, k));
  const uint16_t* mins = scales + canon_scale_elems(n, k);
  float v[2];
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const int64_t x = kk + e;
    const int64_t b = x / QBLOCK, j = x % QBLOCK;
    int code;
    if (bits == 4) {
      const uint8_t byte = codes[b * 32 + (j & 31)];
      code = j < 32 ? (byte & 15) : (byte >> 4);
    } else {
      code = codes[x];
    }
    const float d = f16_to_f32(scales[row * nb + b]);
    const float m = fmt_has_min(fmt) ? f16_to_f32(mins[row * nb + b]) : 0.f;
    v[e] = hd_code_value(fmt, code) * d + m;
  }
  *(uint32_t*)(out + (size_t)t * k + kk) = pack2<T>(v[0], v[1]);
}

void launch_embedding_rows(bool bf16, const uint8_t* blob, int fmt, const int64_t* ids, int T, int64_t n, int64_t k,
                           uint16_t* out, int* err, hipStream_t st) {
  dim3 grid((unsigned)((k / 2 + 255) / 256), (unsigned)T);
  if (bf16) hipLaunchKernelGGL(embedding_rows_kernel<BF16>, grid, dim3(256), 0, st, blob, fmt, ids, n, k, out, err);
  else hipLaunchKernelGGL(embedding_rows_kernel<F16>, grid, dim3(256), 0, st, blob, fmt, ids, n, k, out, err);
}

// ---- decode-step glue: greedy argmax + position / slot advance -------------------
// One workgroup per sequence: argmax over the vocabulary (if logits given),
// feeds the token back as the next input, advances the position and
// precomputes the next step's KV slot and key count -- replacing ~8 small
// framework kernels per graph-captured decode step.
//
// parts (instead of logits): the lm_head GEMV's per-wave argmax partials
// (lowbit_gemv5.cuh EPI_STORE + amax, {max, index bits} [nparts][B]): the
// vocabulary scan shrinks from V logits to nparts pairs, same tie rule
template <typename T>
__global__ void __launch_bounds__(1024) decode_advance_kernel(const uint16_t* logits, int V, int64_t* ids,
                                                              int64_t* next_ids, int64_t* pos,
                                                              const int32_t* block_tables, int max_blocks, int bs,
                                                              int64_t* slots, int32_t* seq_lens,
                                                              const int64_t* pos_offset, int* err,
                                                              const float2* parts, int nparts) {
  const int b = blockIdx.x, tid = threadIdx.x;
  if (parts) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    const int B = gridDim.x;
    for (int p0 = tid; p0 < nparts; p0 += 1024 * 4) {
      float2 q[4];
#pragma unroll
      for (int u = 0; u < 4; u++) q[u] = parts[(size_t)min(p0 + u * 1024, nparts - 1) * B + b];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (p0 + u * 1024 >= nparts) break;
        const int qi = __float_as_int(q[u].y);
        if (q[u].x > best || (q[u].x == best && qi < bi)) { best = q[u].x; bi = qi; }
      }
    }
    __shared__ float pv[16];
    __shared__ int pi[16];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if ((tid & 63) == 0) { pv[tid >> 6] = best; pi[tid >> 6] = bi; }
    __syncthreads();
    if (tid < 64) {
      best = tid < 16 ? pv[tid] : -INFINITY;
      bi = tid < 16 ? pi[tid] : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
      }
      if (tid == 0) {
        if (bi == 0x7fffffff) bi = 0;
        ids[b] = bi;
        next_ids[b] = bi;
      }
    }
  } else if (logits) {
    const uint16_t* row = logits + (size_t)b * V;
    float best = -INFINITY;
    int bi = 0x7fffffff;
    // 16-B vector loads, 8 in flight per thread before any compare
    const int nvec = ((V & 7) == 0 && (((uintptr_t)row) & 15) == 0) ? V / 8 : 0;
    for (int v0 = tid; v0 < nvec; v0 += 1024 * 8) {
      uint4 q[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int vi = min(v0 + u * 1024, nvec - 1);
        q[u] = ((const uint4*)row)[vi];
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int vi = v0 + u * 1024;
        if (vi >= nvec) break;
        const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const float x = to_f32<T>((uint16_t)(e & 1 ? w[e >> 1] >> 16 : w[e >> 1] & 0xffff));
          if (x > best) { best = x; bi = vi * 8 + e; }
        }
      }
    }
    for (int i = nvec * 8 + tid; i < V; i += 1024) {   // tail / unaligned rows
      const float x = to_f32<T>(row[i]);
      if (x > best) { best = x; bi = i; }
    }
    __shared__ float sv[16];
    __shared__ int si[16];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if ((tid & 63) == 0) { sv[tid >> 6] = best; si[tid >> 6] = bi; }
    __syncthreads();
    if (tid < 64) {
      best = tid < 16 ? sv[tid] : -INFINITY;
      bi = tid < 16 ? si[tid] : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
      }
      if (tid == 0) {
        if (bi == 0x7fffffff) bi = 0;            // all -inf / NaN row
        ids[b] = bi;
        next_ids[b] = bi;
      }
    }
  }
  if (tid == 0) {
    const int64_t p = pos[b] + 1;
    pos[b] = p;
    const int64_t ci = p - (pos_offset ? pos_offset[b] : 0);      // cache index
    if (ci < 0 || ci / bs >= max_blocks) {
      // past the sequence's block-table row: no slot (the KV append skips -1)
      kerr(err, ERR_SEQ_LEN);
      if (slots) slots[b] = -1;
    } else if (slots) {
      slots[b] = (int64_t)block_tables[(size_t)b * max_blocks + ci / bs] * bs + ci % bs;
    }
    if (seq_lens) seq_lens[b] = (int32_t)(ci + 1);
  }
}

void launch_decode_advance(bool bf16, const uint16_t* logits, int B, int V, int64_t* ids, int64_t* next_ids,
                           int64_t* pos, const int32_t* block_tables, int max_blocks, int bs, int64_t* slots,
                           int32_t* seq_lens, const int64_t* pos_offset, int* err, hipStream_t st,
                           const float* parts, int nparts) {
  const float2* pp = (const float2*)parts;
  if (bf16) hipLaunchKernelGGL(decode_advance_kernel<BF16>, dim3(B), dim3(1024), 0, st, logits, V, ids, next_ids, pos,
                               block_tables, max_blocks, bs, slots, seq_lens, pos_offset, err, pp, nparts);
  else hipLaunchKernelGGL(decode_advance_kernel<F16>, dim3(B), dim3(1024), 0, st, logits, V, ids, next_ids, pos,
                          block_tables, max_blocks, bs, slots, seq_lens, pos_offset, err, pp, nparts);
}

// ---- RWKV-4 WKV recurrence (reference xe_linear.rwkv_linear_attention_v4,
// models/rwkv4.py:96; HF rwkv_linear_attention_cpu semantics, f32 state in
// max-normalised form).  One thread per (batch, channel): the time loop is a
// true recurrence, channels are independent and coalesced across the wave.
__global__ void __launch_bounds__(256) rwkv4_wkv_kernel(const float* __restrict__ decay,
                                                        const float* __restrict__ first,
                                                        const float* __restrict__ k, const float* __restrict__ v,
                                                        float* __restrict__ out, float* num, float* den,
                                                        float* mx, int B, int T, int C) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * C) return;
  const int b = idx / C, c = idx % C;
  const float w = -__expf(decay[c]), u = first[c];
  float ns = num[idx], ds = den[idx], ms = mx[idx];
  const size_t base = (size_t)b * T * C + c;
  for (int t = 0; t < T; t++) {
    const float kt = k[base + (size_t)t * C], vt = v[base + (size_t)t * C];
    float mo = fmaxf(ms, kt + u);
    float e1 = __expf(ms - mo), e2 = __expf(kt + u - mo);
    out[base + (size_t)t * C] = (e1 * ns + e2 * vt) / (e1 * ds + e2);
    const float m2 = fmaxf(ms + w, kt);
    e1 = __expf(ms + w - m2);
    e2 = __expf(kt - m2);
    ns = e1 * ns + e2 * vt;
    ds = e1 * ds + e2;
    ms = m2;
  }
  num[idx] = ns;
  den[idx] = ds;
  mx[idx] = ms;
}

void launch_rwkv4_wkv(const float* decay, const float* first, const float* k, const float* v, float* out,
                      float* num, float* den, float* mx, int B, int T, int C, hipStream_t st) {
  const int n = B * C;
  hipLaunchKernelGGL(rwkv4_wkv_kernel, dim3((n + 255) / 256), dim3(256), 0, st, decay, first, k, v, out, num, den,
                     mx, B, T, C);
}

// RWKV-5 WKV (xe_linear.rwkv_linear_attention_v5, SRC/transformers/models/
// rwkv5.py:76-119): per (batch, head) an S x S f32 state, for every step
//   out_t[j] = sum_i r_t[i] (u[i] k_t[i] v_t[j] + s[i][j])
//   s[i][j]  = k_t[i] v_t[j] + w[i] s[i][j]            (w = exp(-exp(decay)))
// One workgroup of S threads per (batch, head): thread j owns state column j
// in registers (coalesced [i][j] rows in memory).  r / k / v of a chunk of
// RC steps are staged through LDS (coalesced loads, broadcast reads); the
// per-step scalar sum_i r u k is computed once per step by one lane while
// staging, so the inner loop is 2 FMAs + 1 MUL per key dim.
template <int S>
__global__ void __launch_bounds__(S) rwkv5_wkv_kernel(const float* __restrict__ w, const float* __restrict__ u,
                                                      const float* __restrict__ r, const float* __restrict__ k,
                                                      const float* __restrict__ v, float* __restrict__ out,
                                                      float* __restrict__ state, int T, int H) {
  constexpr int RC = 32;
  __shared__ float rs[RC][S], ks[RC][S], vs[RC][S], ws[S], us[S], ruk[RC];
  const int bh = blockIdx.x, h = bh % H, j = threadIdx.x;
  const int b = bh / H;
  float* st = state + (size_t)bh * S * S + j;
  float s[S];
#pragma unroll
  for (int i = 0; i < S; i++) s[i] = st[(size_t)i * S];
  ws[j] = w[h * S + j];
  us[j] = u[h * S + j];
  const size_t ld = (size_t)H * S;
  const size_t base = (size_t)b * T * ld + (size_t)h * S + j;
  for (int t0 = 0; t0 < T; t0 += RC) {
    const int nt = min(RC, T - t0);
    __syncthreads();
    for (int tt = 0; tt < nt; tt++) {
      const size_t o = base + (size_t)(t0 + tt) * ld;
      rs[tt][j] = r[o];
      ks[tt][j] = k[o];
      vs[tt][j] = v[o];
    }
    __syncthreads();
    // sum_i r u k per step: thread j reduces step j % RC over its slice of i
    // (S / RC threads per step), combined with shuffles
    {
      constexpr int PER = S / RC > 0 ? S / RC : 1;
      const int tt = j % RC, part = j / RC;
      float acc = 0.f;
      if (tt < nt)
        for (int i = part; i < S; i += PER) acc += rs[tt][i] * ks[tt][i] * us[i];
      for (int off = RC; off < S && off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
      if constexpr (S > 64) {
        // two waves: the second wave's partial sums are added through LDS
        __shared__ float half[RC];
        if (j >= 64 && j < 64 + RC) half[tt] = acc;
        __syncthreads();
        if (j < RC) ruk[tt] = acc + half[tt];
      } else {
        if (j < RC) ruk[tt] = acc;
      }
    }
    __syncthreads();
    for (int tt = 0; tt < nt; tt++) {
      const float vj = vs[tt][j];
      float o0 = vj * ruk[tt], o1 = 0.f;
#pragma unroll
      for (int i = 0; i < S; i += 2) {
        o0 = __builtin_fmaf(rs[tt][i], s[i], o0);
        o1 = __builtin_fmaf(rs[tt][i + 1], s[i + 1], o1);
        s[i] = __builtin_fmaf(ws[i], s[i], ks[tt][i] * vj);
        s[i + 1] = __builtin_fmaf(ws[i + 1], s[i + 1], ks[tt][i + 1] * vj);
      }
      out[base + (size_t)(t0 + tt) * ld] = o0 + o1;
    }
  }
#pragma unroll
  for (int i = 0; i < S; i++) st[(size_t)i * S] = s[i];
}

void launch_rwkv5_wkv(const float* w, const float* u, const float* r, const float* k, const float* v, float* out,
                      float* state, int B, int T, int H, int S, hipStream_t st) {
  const dim3 grid(B * H);
  if (S == 32) hipLaunchKernelGGL(rwkv5_wkv_kernel<32>, grid, dim3(32), 0, st, w, u, r, k, v, out, state, T, H);
  else if (S == 64) hipLaunchKernelGGL(rwkv5_wkv_kernel<64>, grid, dim3(64), 0, st, w, u, r, k, v, out, state, T, H);
  else hipLaunchKernelGGL(rwkv5_wkv_kernel<128>, grid, dim3(128), 0, st, w, u, r, k, v, out, state, T, H);
}

}  // namespace illm
