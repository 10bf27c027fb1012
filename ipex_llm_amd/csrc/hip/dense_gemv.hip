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

template <typename T>
static void dg_t(const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t N, const uint16_t* bias,
                 uint16_t* out, hipStream_t st) {
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
                       const uint16_t* bias, uint16_t* out, hipStream_t st) {
  if (bf16) dg_t<BF16>(x, M, K, w, N, bias, out, st);
  else dg_t<F16>(x, M, K, w, N, bias, out, st);
}

}  // namespace illm
