// Skinny GEMM (M <= 16 rows) over dense bf16 / fp16 weights: the decode
// projections of fp16 / bf16 models (FP16Linear / BF16Linear of the
// reference, SRC/transformers/low_bit_linear.py:758-948, whose XPU decode
// runs ESIMD skinny kernels) and the verify forward of self-speculative
// decoding (k + 1 rows).
//
// Pure weight streaming: W [N, K] is read exactly once.  A workgroup of 4
// waves owns 4 consecutive rows (one per wave); a lane loads 2 x 16 B of its
// row per step (2 loads in flight per lane, 2 KB per wave-step) and
// multiplies them against every activation row (L1/L2 resident); the row
// sums are wave reductions.  The bias is added in the epilogue.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

template <typename T>
__device__ __forceinline__ float dot8(const uint4& w, const uint4& x) {
  const uint32_t ws[4] = {w.x, w.y, w.z, w.w}, xs[4] = {x.x, x.y, x.z, x.w};
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; i++)
    s += to_f32<T>(ws[i] & 0xffff) * to_f32<T>(xs[i] & 0xffff) + to_f32<T>(ws[i] >> 16) * to_f32<T>(xs[i] >> 16);
  return s;
}

template <typename T, int MM>
__global__ void __launch_bounds__(256) dense_gemv_kernel(const uint16_t* __restrict__ x, int M, int64_t K,
                                                         const uint16_t* __restrict__ w, int64_t N,
                                                         const uint16_t* __restrict__ bias,
                                                         uint16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const uint16_t* wr = w + n * K;
  float acc[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) acc[m] = 0.f;
  int64_t k = (int64_t)lane * 8;
  // main loop: two 16-B weight loads per lane in flight
  for (; k + 64 * 8 < K; k += 2 * 64 * 8) {
    const uint4 w0 = *(const uint4*)(wr + k);
    const uint4 w1 = *(const uint4*)(wr + k + 64 * 8);
#pragma unroll
    for (int m = 0; m < MM; m++) {
      if (m < M) {
        const uint16_t* xr = x + (int64_t)m * K;
        acc[m] += dot8<T>(w0, *(const uint4*)(xr + k)) + dot8<T>(w1, *(const uint4*)(xr + k + 64 * 8));
      }
    }
  }
  for (; k < K; k += 64 * 8) {
    const uint4 w0 = *(const uint4*)(wr + k);
#pragma unroll
    for (int m = 0; m < MM; m++)
      if (m < M) acc[m] += dot8<T>(w0, *(const uint4*)(x + (int64_t)m * K + k));
  }
  const float b = bias != nullptr ? to_f32<T>(bias[n]) : 0.f;
#pragma unroll
  for (int m = 0; m < MM; m++) {
    if (m < M) {
      const float s = wave_sum(acc[m]);
      if (lane == 0) out[(int64_t)m * N + n] = from_f32<T>(s + b);
    }
  }
}

// act(x Wg^T) * (x Wu^T) for a gate/up weight in the 16-row tile interleave
// (rows 32 p .. + 15 gate, 32 p + 16 .. + 31 up: output column 16 p + j): one
// wave streams the gate and the up row of one output column, so the
// [M, 2I] projection, the de-interleave copies and the activation / product
// launches of the unfused path disappear.  Rounding follows that path: g and
// u rounded to T, act(g) rounded, the product rounded.  act: 0 SiLU, 1 GELU
// (tanh).
template <typename T, int MM>
__global__ void __launch_bounds__(256) dense_glu_kernel(const uint16_t* __restrict__ x, int M, int64_t K,
                                                        const uint16_t* __restrict__ w, int64_t I, int act,
                                                        uint16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= I) return;
  const int64_t rg = 32 * (i / 16) + (i % 16);
  const uint16_t* wg = w + rg * K;
  const uint16_t* wu = wg + 16 * K;
  float ag[MM], au[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) ag[m] = au[m] = 0.f;
  // each weight / activation element is widened once per step and shared by
  // the gate and up products of every row (the per-call conversions of two
  // dot8s per row made the 3-4-row verify VALU-bound)
  auto step = [&](const uint4& g0, const uint4& u0, int64_t k) {
    float gf[8], uf[8];
    const uint32_t gs[4] = {g0.x, g0.y, g0.z, g0.w}, us[4] = {u0.x, u0.y, u0.z, u0.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      gf[2 * j] = to_f32<T>(gs[j] & 0xffff), gf[2 * j + 1] = to_f32<T>(gs[j] >> 16);
      uf[2 * j] = to_f32<T>(us[j] & 0xffff), uf[2 * j + 1] = to_f32<T>(us[j] >> 16);
    }
#pragma unroll
    for (int m = 0; m < MM; m++) {
      if (m < M) {
        const uint4 xv = *(const uint4*)(x + (int64_t)m * K + k);
        const uint32_t xs[4] = {xv.x, xv.y, xv.z, xv.w};
        float sg = 0.f, su = 0.f;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const float x0 = to_f32<T>(xs[j] & 0xffff), x1 = to_f32<T>(xs[j] >> 16);
          sg += gf[2 * j] * x0 + gf[2 * j + 1] * x1;
          su += uf[2 * j] * x0 + uf[2 * j + 1] * x1;
        }
        ag[m] += sg;
        au[m] += su;
      }
    }
  };
  int64_t k = (int64_t)lane * 8;
  for (; k + 64 * 8 < K; k += 2 * 64 * 8) {         // two gate + two up loads per lane in flight
    const uint4 g0 = *(const uint4*)(wg + k), g1 = *(const uint4*)(wg + k + 64 * 8);
    const uint4 u0 = *(const uint4*)(wu + k), u1 = *(const uint4*)(wu + k + 64 * 8);
    step(g0, u0, k);
    step(g1, u1, k + 64 * 8);
  }
  for (; k < K; k += 64 * 8) step(*(const uint4*)(wg + k), *(const uint4*)(wu + k), k);
  auto rnd = [](float v) { return to_f32<T>(from_f32<T>(v)); };
#pragma unroll
  for (int m = 0; m < MM; m++) {
    if (m < M) {
      const float g = rnd(wave_sum(ag[m])), u = rnd(wave_sum(au[m]));
      float a;
      if (act == 0) {
        a = g / (1.f + __expf(-g));
      } else {
        const float c = 0.7978845608028654f * (g + 0.044715f * g * g * g);
        a = 0.5f * g * (1.f + tanhf(c));
      }
      if (lane == 0) out[(int64_t)m * I + i] = from_f32<T>(rnd(a) * u);
    }
  }
}

// ---- MFMA form (K % 64 == 0): one workgroup of DW waves per 16-row weight
// tile (GLU: per 16-row gate tile + its 16-row up tile), wave w over the K
// range [w K / DW, (w + 1) K / DW) in 64-deep steps.  The weight tile is the
// MFMA A operand straight from memory (lane: row lane % 16, 8 k at 8 (lane /
// 16) and 32 + 8 (lane / 16): 128 contiguous bytes per row per step), the
// <= 16 activation rows the B operand (absent rows zero): no per-element
// widening, so the 2-16-row verify / batched decode stays on the weight
// stream instead of the VALU (the dot8 form above converts every weight
// once per activation row).  Each output is its own MFMA column: a row's
// result does not depend on how many rows share the launch.  The DW partial
// tiles meet in LDS; wave 0 adds them in wave order and stores.
constexpr int DW = 8;

template <typename T, bool GLU>
__global__ void __launch_bounds__(DW * 64) dense_mfma_kernel(const uint16_t* __restrict__ x, int M, int64_t K,
                                                          const uint16_t* __restrict__ w, int64_t N,
                                                          const uint16_t* __restrict__ bias, int act,
                                                          uint16_t* __restrict__ out, int trans) {
  __shared__ f32x4 red[DW][GLU ? 2 : 1][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t t = blockIdx.x;                         // 16-row tile (GLU: tile pair)
  const int64_t row0 = GLU ? 32 * t : 16 * t;
  const int64_t steps = K / 64;
  const int64_t s0 = steps * wave / DW, s1 = steps * (wave + 1) / DW;
  const int64_t nr = min<int64_t>(row0 + r, GLU ? 2 * N - 1 : N - 1);   // clamp ragged tail rows
  const uint16_t* wg = w + nr * K + 8 * g;
  const uint16_t* wu = GLU ? wg + 16 * K : wg;
  const bool xon = r < M;
  const uint16_t* xr = x + (int64_t)(xon ? r : 0) * K + 8 * g;
  f32x4 ag = {0.f, 0.f, 0.f, 0.f}, au = {0.f, 0.f, 0.f, 0.f};
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  auto ld = [&](const uint16_t* p) { return *(const uint4*)p; };
  int64_t s = s0;
  // two 64-deep steps per iteration, the pair's weights requested first (a
  // 4-step form measured no faster, profiles/spec_bench_r5_*.jsonl)
  for (; s + 1 < s1; s += 2) {
    const int64_t k = s * 64;
    const uint4 a0 = ld(wg + k), a1 = ld(wg + k + 32), a2 = ld(wg + k + 64), a3 = ld(wg + k + 96);
    uint4 u0 = z4, u1 = z4, u2 = z4, u3 = z4;
    if constexpr (GLU) u0 = ld(wu + k), u1 = ld(wu + k + 32), u2 = ld(wu + k + 64), u3 = ld(wu + k + 96);
    const uint4 b0 = xon ? ld(xr + k) : z4, b1 = xon ? ld(xr + k + 32) : z4;
    const uint4 b2 = xon ? ld(xr + k + 64) : z4, b3 = xon ? ld(xr + k + 96) : z4;
    ag = mfma16<T>(a0, b0, ag);
    ag = mfma16<T>(a1, b1, ag);
    ag = mfma16<T>(a2, b2, ag);
    ag = mfma16<T>(a3, b3, ag);
    if constexpr (GLU) {
      au = mfma16<T>(u0, b0, au);
      au = mfma16<T>(u1, b1, au);
      au = mfma16<T>(u2, b2, au);
      au = mfma16<T>(u3, b3, au);
    }
  }
  if (s < s1) {
    const int64_t k = s * 64;
    const uint4 b0 = xon ? ld(xr + k) : z4, b1 = xon ? ld(xr + k + 32) : z4;
    ag = mfma16<T>(ld(wg + k), b0, ag);
    ag = mfma16<T>(ld(wg + k + 32), b1, ag);
    if constexpr (GLU) {
      au = mfma16<T>(ld(wu + k), b0, au);
      au = mfma16<T>(ld(wu + k + 32), b1, au);
    }
  }
  red[wave][0][lane] = ag;
  if constexpr (GLU) red[wave][1][lane] = au;
  __syncthreads();
  if (wave != 0) return;
  f32x4 sg = red[0][0][lane], su = GLU ? red[0][1][lane] : ag;
#pragma unroll
  for (int v = 1; v < DW; v++) {
    sg += red[v][0][lane];
    if constexpr (GLU) su += red[v][1][lane];
  }
  // lane holds outputs (n = 16 t + 4 g + i, m = r)
  const int m = r;
  if (m >= M) return;
  const int64_t n0 = 16 * t + 4 * g;
  auto rnd = [](float v) { return to_f32<T>(from_f32<T>(v)); };
  uint16_t o[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    float v;
    if constexpr (GLU) {
      const float gv = rnd(sg[i]), uv = rnd(su[i]);
      float a;
      if (act == 0) {
        a = gv / (1.f + __expf(-gv));
      } else {
        const float c = 0.7978845608028654f * (gv + 0.044715f * gv * gv * gv);
        a = 0.5f * gv * (1.f + tanhf(c));
      }
      v = rnd(a) * uv;
    } else {
      v = sg[i] + (bias != nullptr && n0 + i < N ? to_f32<T>(bias[n0 + i]) : 0.f);
    }
    o[i] = from_f32<T>(v);
  }
  if (trans) {                                     // out^T [N, M]: the skinny-GEMM caller's [tokens, r]
    for (int i = 0; i < 4 && n0 + i < N; i++) out[(n0 + i) * M + m] = o[i];
    return;
  }
  uint16_t* y = out + (int64_t)m * N + n0;
  if (n0 + 3 < N && (((int64_t)m * N + n0) & 3) == 0) {
    *(uint2*)y = make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
  } else {
    for (int i = 0; i < 4 && n0 + i < N; i++) y[i] = o[i];
  }
}

static bool dense_mfma_on() {
  static const int on = [] {
    const char* e = getenv("ILLM_DENSE_MFMA");
    return e ? atoi(e) : 1;
  }();
  return on != 0;
}

template <typename T>
static void dg_t(const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t N, const uint16_t* bias,
                 uint16_t* out, hipStream_t st, bool trans) {
  if (trans || (dense_mfma_on() && K % 64 == 0 && M <= 16)) {
    hipLaunchKernelGGL((dense_mfma_kernel<T, false>), dim3((unsigned)((N + 15) / 16)), dim3(DW * 64), 0, st, x, M, K,
                       w, N, bias, 0, out, trans ? 1 : 0);
    return;
  }
  const dim3 grid((unsigned)((N + 3) / 4));
#define DG(MMV) hipLaunchKernelGGL((dense_gemv_kernel<T, MMV>), grid, dim3(256), 0, st, x, M, K, w, N, bias, out)
  if (M <= 1) DG(1);
  else if (M <= 2) DG(2);
  else if (M <= 4) DG(4);
  else if (M <= 8) DG(8);
  else DG(16);
#undef DG
}

template <typename T>
static void dglu_t(const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t I, int act, uint16_t* out,
                   hipStream_t st) {
  if (dense_mfma_on() && K % 64 == 0 && M <= 16 && I % 16 == 0) {
    hipLaunchKernelGGL((dense_mfma_kernel<T, true>), dim3((unsigned)(I / 16)), dim3(DW * 64), 0, st, x, M, K, w, I,
                       nullptr, act, out, 0);
    return;
  }
  const dim3 grid((unsigned)((I + 3) / 4));
#define DG(MMV) hipLaunchKernelGGL((dense_glu_kernel<T, MMV>), grid, dim3(256), 0, st, x, M, K, w, I, act, out)
  if (M <= 1) DG(1);
  else if (M <= 2) DG(2);
  else if (M <= 4) DG(4);
  else if (M <= 8) DG(8);
  else DG(16);
#undef DG
}

void launch_dense_glu(bool bf16, const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t I, int act,
                      uint16_t* out, hipStream_t st) {
  if (bf16) dglu_t<BF16>(x, M, K, w, I, act, out, st);
  else dglu_t<F16>(x, M, K, w, I, act, out, st);
}

void launch_dense_gemv(bool bf16, const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t N,
                       const uint16_t* bias, uint16_t* out, hipStream_t st, bool trans_out) {
  if (bf16) dg_t<BF16>(x, M, K, w, N, bias, out, st, trans_out);
  else dg_t<F16>(x, M, K, w, N, bias, out, st, trans_out);
}

}  // namespace illm
