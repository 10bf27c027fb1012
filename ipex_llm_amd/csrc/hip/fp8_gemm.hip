// fp8 linear on gfx950 matrix cores: the torch_fp8_e4m3 / torch_fp8_e5m2
// qtypes' forward (reference ``xe_linear.run_linear_fp8`` after
// ``dynamic_scaled_fp8_quant``, SRC/transformers/low_bit_linear.py:168-178,
// 692-696).
//
//   y[m, n] = sx[m] * sw[n] * sum_k q(x)[m, k] * W8[n, k]  (+ bias[n])
//
// W8 is an fp8 weight (OCP e4m3fn or e5m2) with a per-tensor (reference) or
// per-output-channel f32 scale; q(x) is the activation quantized per token
// to e4m3 with sx = amax / 448 (fp8_act_quant_kernel).
//
// Prefill GEMM (fp8_gemm_kernel): 128 (m) x 128 (n) block of 4 waves (2 x 2,
// 64 x 64 each = 4 x 4 tiles of 16 x 16), K stepped 128 at a time with the
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 -- unit E8M0 scales (127):
// the row / column scales are applied once in the epilogue, so the MX form is
// used purely for its rate (2x the bf16 MFMA per clock; the unscaled
// 16x16x32 fp8 MFMA runs at the bf16 rate).  A lane's 32-byte fragment of a
// 16-row tile is row (lane & 15), k bytes 32 (lane >> 4) ... + 31 for the x
// tile and the weight tile alike (the same k map on both operands, so the
// instruction's internal k order does not matter); the C/D map is the
// dtype-independent 16x16 one (col = lane & 15, row = 4 (lane >> 4) + r).
// Tiles are staged global -> registers -> LDS one K-step ahead (double
// buffered), 144-B LDS rows (16 B of padding) keep the 16 rows of a
// fragment read off one bank group.
//
// Decode (M <= 16, fp8_gemv_kernel): one wave per output row streams the
// fp8 row 16 B per lane (v_cvt_pk_f32_fp8 / _bf8 decode) against bf16 x rows
// (L1/L2 resident): pure weight streaming, no activation quantization.
#include <hip/hip_runtime.h>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------- act quant
template <typename T>
__global__ void __launch_bounds__(256) fp8_act_quant_kernel(const uint16_t* __restrict__ x, int64_t K,
                                                            uint8_t* __restrict__ xq, float* __restrict__ sx) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const uint16_t* xr = x + row * K;
  float amax = 0.f;
  for (int64_t k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const uint4 v = *(const uint4*)(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++)
      amax = fmaxf(amax, fmaxf(fabsf(to_f32<T>(w[i] & 0xffff)), fabsf(to_f32<T>(w[i] >> 16))));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) sx[row] = s;
  uint8_t* qr = xq + row * K;
  for (int64_t k = threadIdx.x * 8; k < K; k += 256 * 8) {
    const uint4 v = *(const uint4*)(xr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const float a = fminf(fmaxf(to_f32<T>(w[2 * i] & 0xffff) * inv, -448.f), 448.f);
      const float b = fminf(fmaxf(to_f32<T>(w[2 * i] >> 16) * inv, -448.f), 448.f);
      const float c = fminf(fmaxf(to_f32<T>(w[2 * i + 1] & 0xffff) * inv, -448.f), 448.f);
      const float d = fminf(fmaxf(to_f32<T>(w[2 * i + 1] >> 16) * inv, -448.f), 448.f);
      int p = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
      p = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, p, true);
      o[i] = (uint32_t)p;
    }
    *(uint2*)(qr + k) = make_uint2(o[0], o[1]);
  }
}

// ----------------------------------------------------------------- GEMM
constexpr int F8_BM = 128, F8_BN = 128, F8_BK = 128, F8_LDS_ROW = F8_BK + 16;

template <typename T, int FMTB>
__global__ void __launch_bounds__(256) fp8_gemm_kernel(const Fp8GemmArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][2][F8_BM * F8_LDS_ROW];   // [buf][A|B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware order: consecutive block ids land on different XCDs, so give
  // the 8 m-blocks of one weight tile ids b, b + 8, ...: one XCD streams it
  const int nbn = a.N / F8_BN, nbm = (a.M + F8_BM - 1) / F8_BM;
  int bid = blockIdx.x, bn, bm;
  if (nbm >= 8 && (nbn * nbm) % 8 == 0) {
    const int xcd = bid & 7, slot = bid >> 3, per = nbn * nbm / 8;
    const int lin = xcd * per + slot;               // this XCD's contiguous share
    bn = lin / nbm;
    bm = lin % nbm;
  } else {
    bn = bid / nbm;
    bm = bid % nbm;
  }
  const int m0 = bm * F8_BM, n0 = bn * F8_BN;
  const int64_t K = a.K;
  const uint8_t* __restrict__ X = a.xq;
  const uint8_t* __restrict__ W = a.w;
  // staging: 4 x 16 B of the A tile and 4 of the B tile per thread per K step
  uint4 ra[4], rb[4];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = tid + 256 * q, r = i >> 3, c = i & 7;
      const int m = m0 + r;
      ra[q] = m < a.M ? *(const uint4*)(X + (int64_t)m * K + k0 + c * 16) : make_uint4(0, 0, 0, 0);
      rb[q] = *(const uint4*)(W + (int64_t)(n0 + r) * K + k0 + c * 16);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = tid + 256 * q, r = i >> 3, c = i & 7;
      *(uint4*)(&lds[buf][0][r * F8_LDS_ROW + c * 16]) = ra[q];
      *(uint4*)(&lds[buf][1][r * F8_LDS_ROW + c * 16]) = rb[q];
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (int)(K / F8_BK);
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = 32 * (lane >> 4);
  for (int kc = 0; kc < nk; kc++) {
    const int buf = kc & 1;
    if (kc + 1 < nk) load((int64_t)(kc + 1) * F8_BK);
    i32x8 fa[4], fb[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const uint8_t* pa = &lds[buf][0][(wm * 64 + t * 16 + fr) * F8_LDS_ROW + fk];
      const uint8_t* pb = &lds[buf][1][(wn * 64 + t * 16 + fr) * F8_LDS_ROW + fk];
      const uint4 a0 = *(const uint4*)pa, a1 = *(const uint4*)(pa + 16);
      const uint4 b0 = *(const uint4*)pb, b1 = *(const uint4*)(pb + 16);
      fa[t] = i32x8{(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
      fb[t] = i32x8{(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[i], fb[j], acc[i][j], 0, FMTB, 0, 127,
                                                                     0, 127);
    if (kc + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
  // epilogue: scales, bias, 16-bit store
  const int col = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int n = n0 + wn * 64 + j * 16 + col;
    const float swn = a.sw[a.sw_per_channel ? n : 0];
    const float bn_ = a.bias != nullptr ? to_f32<T>(a.bias[n]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int m = m0 + wm * 64 + i * 16 + rq + r;
        if (m < a.M) a.out[(int64_t)m * a.N + n] = from_f32<T>(acc[i][j][r] * a.sx[m] * swn + bn_);
      }
    }
  }
}

// ----------------------------------------------------------------- GEMV
template <int FMTB, bool HI>
__device__ __forceinline__ f32x2 f8pair(int v) {
  if constexpr (FMTB == 0) return __builtin_amdgcn_cvt_pk_f32_fp8(v, HI);
  else return __builtin_amdgcn_cvt_pk_f32_bf8(v, HI);
}

template <typename T, int FMTB, int MM>
__global__ void __launch_bounds__(256) fp8_gemv_kernel(const Fp8GemmArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= a.N) return;
  const int64_t K = a.K;
  const uint8_t* wr = a.w + n * K;
  float acc[MM];
#pragma unroll
  for (int m = 0; m < MM; m++) acc[m] = 0.f;
  for (int64_t k = lane * 16; k < K; k += 64 * 16) {
    const uint4 wv = *(const uint4*)(wr + k);
    const int wd[4] = {(int)wv.x, (int)wv.y, (int)wv.z, (int)wv.w};
    float wf[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const f32x2 lo = f8pair<FMTB, false>(wd[i]), hi = f8pair<FMTB, true>(wd[i]);
      wf[4 * i] = lo[0];
      wf[4 * i + 1] = lo[1];
      wf[4 * i + 2] = hi[0];
      wf[4 * i + 3] = hi[1];
    }
#pragma unroll
    for (int m = 0; m < MM; m++) {
      if (m < a.M) {
        const uint16_t* xr = a.x + (int64_t)m * K + k;
        const uint4 x0 = *(const uint4*)xr, x1 = *(const uint4*)(xr + 8);
        const uint32_t xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; i++)
          s += wf[2 * i] * to_f32<T>(xs[i] & 0xffff) + wf[2 * i + 1] * to_f32<T>(xs[i] >> 16);
        acc[m] += s;
      }
    }
  }
  const float swn = a.sw[a.sw_per_channel ? n : 0];
  const float bn_ = a.bias != nullptr ? to_f32<T>(a.bias[n]) : 0.f;
#pragma unroll
  for (int m = 0; m < MM; m++) {
    if (m < a.M) {
      const float s = wave_sum(acc[m]);
      if (lane == 0) a.out[(int64_t)m * a.N + n] = from_f32<T>(s * swn + bn_);
    }
  }
}

// ----------------------------------------------------------------- launchers
void launch_fp8_act_quant(bool bf16, const uint16_t* x, int64_t M, int64_t K, uint8_t* xq, float* sx,
                          hipStream_t st) {
  if (bf16) hipLaunchKernelGGL((fp8_act_quant_kernel<BF16>), dim3((unsigned)M), dim3(256), 0, st, x, K, xq, sx);
  else hipLaunchKernelGGL((fp8_act_quant_kernel<F16>), dim3((unsigned)M), dim3(256), 0, st, x, K, xq, sx);
}

template <typename T, int FMTB>
static void gemm_t(const Fp8GemmArgs& a, hipStream_t st) {
  const int blocks = (a.N / F8_BN) * ((a.M + F8_BM - 1) / F8_BM);
  hipLaunchKernelGGL((fp8_gemm_kernel<T, FMTB>), dim3(blocks), dim3(256), 0, st, a);
}

void launch_fp8_gemm(bool bf16, bool e5m2, const Fp8GemmArgs& a, hipStream_t st) {
  if (bf16) {
    if (e5m2) gemm_t<BF16, 1>(a, st); else gemm_t<BF16, 0>(a, st);
  } else {
    if (e5m2) gemm_t<F16, 1>(a, st); else gemm_t<F16, 0>(a, st);
  }
}

template <typename T, int FMTB>
static void gemv_t(const Fp8GemmArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.N + 3) / 4));
  if (a.M <= 1) hipLaunchKernelGGL((fp8_gemv_kernel<T, FMTB, 1>), grid, dim3(256), 0, st, a);
  else if (a.M <= 4) hipLaunchKernelGGL((fp8_gemv_kernel<T, FMTB, 4>), grid, dim3(256), 0, st, a);
  else if (a.M <= 8) hipLaunchKernelGGL((fp8_gemv_kernel<T, FMTB, 8>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((fp8_gemv_kernel<T, FMTB, 16>), grid, dim3(256), 0, st, a);
}

void launch_fp8_gemv(bool bf16, bool e5m2, const Fp8GemmArgs& a, hipStream_t st) {
  if (bf16) {
    if (e5m2) gemv_t<BF16, 1>(a, st); else gemv_t<BF16, 0>(a, st);
  } else {
    if (e5m2) gemv_t<F16, 1>(a, st); else gemv_t<F16, 0>(a, st);
  }
}

}  // namespace illm
