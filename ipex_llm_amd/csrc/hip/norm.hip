// Row normalisation kernels (RMSNorm / LayerNorm), with the residual add and
// the split-K partial reduction of the preceding low-bit GEMV fused in.
//
// Reference ops: xe_addons.rms_norm / xe_addons.layer_norm
// (SRC/transformers/models/common.py:184-216).  HF numerics are matched:
// normalise in f32, round to the activation dtype, then multiply by the
// weight and round again (LlamaRMSNorm.forward).
#include "illm_device.h"
#include "kernels.h"

namespace illm {

// 512 threads: a 4096-wide row is one 16-B vector per thread, so every
// partial-slab load of the row is in flight at once (latency, not bandwidth,
// bounds these small rows).
constexpr int NORM_THREADS = 512;

template <typename T>
__device__ __forceinline__ void load8(const uint16_t* p, float* v) {
  uint4 u = *(const uint4*)p;
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; i++) {
    v[2 * i] = to_f32<T>(w[i] & 0xffff);
    v[2 * i + 1] = to_f32<T>(w[i] >> 16);
  }
}
template <typename T>
__device__ __forceinline__ void store8(uint16_t* p, const float* v) {
  *(uint4*)p = make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                          pack2<T>(v[6], v[7]));
}
template <typename T>
__device__ __forceinline__ float rnd(float v) { return to_f32<T>(from_f32<T>(v)); }

// MAXV = max 8-element vectors per thread (H <= MAXV * 8 * 256)
template <typename T, int MAXV>
__global__ void __launch_bounds__(NORM_THREADS)
    add_rms_norm_kernel(const uint16_t* __restrict__ x, const float* __restrict__ partials,
                        int nsplit, uint16_t* __restrict__ residual, const uint16_t* __restrict__ w,
                        uint16_t* __restrict__ out, int H, float eps, int unit_offset,
                        int store_residual, int zero_partials, const int64_t* __restrict__ ids, int64_t vocab,
                        uint16_t* __restrict__ gather_out, float* zero, int zero_n, int* err) {
  __shared__ float red[NORM_THREADS / 64];
  const int row = blockIdx.x;
  const int M = gridDim.x;
  int64_t xrow = row;
  if (ids) {
    // embedding row of this token (an out-of-vocabulary id reads row 0 and is reported)
    xrow = ids[row];
    if ((uint64_t)xrow >= (uint64_t)vocab) {
      if (threadIdx.x == 0) kerr(err, ERR_TOKEN);
      xrow = 0;
    }
    if (zero && row == 0)
      for (int i = threadIdx.x; i < zero_n; i += NORM_THREADS) zero[i] = 0.f;
  }
  // the weight does not depend on the row: load it first so it is not a
  // dependent memory round trip behind the block reduction
  uint4 wraw[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    wraw[j] = c < H ? *(const uint4*)(w + c) : make_uint4(0, 0, 0, 0);
  }
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H) {
      float a[8];
      if (partials) {
        // sum the GEMV's split-K partial slabs, round like a standalone GEMV
        // (measured at batch 8: hoisting the residual load above this loop,
        // 5.09 -> 5.48 us, and unroll 8, were both slower than this form)
        for (int i = 0; i < 8; i++) a[i] = 0.f;
#pragma unroll 4
        for (int s = 0; s < nsplit; s++) {
          const float4* p = (const float4*)(partials + ((size_t)s * M + row) * H + c);
          float4 p0 = p[0], p1 = p[1];
          a[0] += p0.x; a[1] += p0.y; a[2] += p0.z; a[3] += p0.w;
          a[4] += p1.x; a[5] += p1.y; a[6] += p1.z; a[7] += p1.w;
        }
        for (int i = 0; i < 8; i++) a[i] = rnd<T>(a[i]);
        if (zero_partials) {
          float* z = (float*)partials + (size_t)row * H + c;
          ((float4*)z)[0] = make_float4(0.f, 0.f, 0.f, 0.f);
          ((float4*)z)[1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      } else {
        load8<T>(x + (size_t)xrow * H + c, a);
        if (gather_out) store8<T>(gather_out + (size_t)row * H + c, a);
      }
      if (residual) {
        float r[8];
        load8<T>(residual + (size_t)row * H + c, r);
        for (int i = 0; i < 8; i++) a[i] = rnd<T>(a[i] + r[i]);
        if (store_residual) store8<T>(residual + (size_t)row * H + c, a);
      }
      for (int i = 0; i < 8; i++) {
        v[j][i] = a[i];
        ss += a[i] * a[i];
      }
    }
  }
  ss = block_sum<NORM_THREADS>(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H) {
      float wv[8], o[8];
      const uint32_t wr[4] = {wraw[j].x, wraw[j].y, wraw[j].z, wraw[j].w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        wv[2 * i] = to_f32<T>((uint16_t)(wr[i] & 0xffff));
        wv[2 * i + 1] = to_f32<T>((uint16_t)(wr[i] >> 16));
      }
      for (int i = 0; i < 8; i++) {
        const float ww = unit_offset ? rnd<T>(1.f + wv[i]) : wv[i];
        o[i] = ww * rnd<T>(v[j][i] * inv);
      }
      store8<T>(out + (size_t)row * H + c, o);
    }
  }
}

template <typename T, int MAXV>
__global__ void __launch_bounds__(NORM_THREADS)
    layer_norm_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                      const uint16_t* __restrict__ b, uint16_t* __restrict__ out, int H, float eps) {
  __shared__ float red[NORM_THREADS / 64];
  const int row = blockIdx.x;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H) {
      load8<T>(x + (size_t)row * H + c, v[j]);
      for (int i = 0; i < 8; i++) s += v[j][i];
    }
  }
  const float mean = block_sum<NORM_THREADS>(s, red) / (float)H;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H)
      for (int i = 0; i < 8; i++) {
        const float d = v[j][i] - mean;
        q += d * d;
      }
  }
  __syncthreads();
  const float inv = rsqrtf(block_sum<NORM_THREADS>(q, red) / (float)H + eps);
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H) {
      float wv[8], bv[8], o[8];
      if (w) load8<T>(w + c, wv); else for (int i = 0; i < 8; i++) wv[i] = 1.f;
      if (b) load8<T>(b + c, bv); else for (int i = 0; i < 8; i++) bv[i] = 0.f;
      for (int i = 0; i < 8; i++) o[i] = (v[j][i] - mean) * inv * wv[i] + bv[i];
      store8<T>(out + (size_t)row * H + c, o);
    }
  }
}

template <typename T>
static void launch_add_rms(const NormArgs& a, hipStream_t st) {
  const int nv = (a.H / 8 + NORM_THREADS - 1) / NORM_THREADS;
#define L_RMS(MV)                                                                             \
  hipLaunchKernelGGL((add_rms_norm_kernel<T, MV>), dim3(a.M), dim3(NORM_THREADS), 0, st, a.x, \
                     a.partials, a.nsplit, a.residual, a.w, a.out, a.H, a.eps, a.unit_offset,  \
                     a.store_residual, a.zero_partials, a.ids, a.vocab, a.gather_out, a.zero,  \
                     a.zero_n, a.err)
  if (nv <= 1) L_RMS(1);
  else if (nv <= 2) L_RMS(2);
  else if (nv <= 4) L_RMS(4);
  else L_RMS(8);
#undef L_RMS
}

// ---- RMSNorm backward (training: QLoRA base models keep their norms frozen)
// dL/dx of out = w * rnd(x * r), r = rsqrt(mean(x^2) + eps), for the gradient g
// of out, matching the autograd graph of LlamaRMSNorm: gh = rnd(g * w) (the
// bf16 product), then in f32 dx = r gh - x r^3 mean(gh x).  One workgroup per
// row: x, g and w loaded once, two block reductions, one store.
template <typename T, int MAXV>
__global__ void __launch_bounds__(NORM_THREADS)
    rms_norm_bwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ g,
                        const uint16_t* __restrict__ w, uint16_t* __restrict__ dx, int H, float eps,
                        int unit_offset) {
  __shared__ float red[NORM_THREADS / 64];
  const int row = blockIdx.x;
  float xv[MAXV][8], gh[MAXV][8];
  float ss = 0.f, dot = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H) {
      float gv[8], wv[8];
      load8<T>(x + (size_t)row * H + c, xv[j]);
      load8<T>(g + (size_t)row * H + c, gv);
      load8<T>(w + c, wv);
      for (int i = 0; i < 8; i++) {
        const float ww = unit_offset ? rnd<T>(1.f + wv[i]) : wv[i];
        gh[j][i] = rnd<T>(gv[i] * ww);
        ss += xv[j][i] * xv[j][i];
        dot += gh[j][i] * xv[j][i];
      }
    }
  }
  ss = block_sum<NORM_THREADS>(ss, red);
  dot = block_sum<NORM_THREADS>(dot, red);
  const float r = rsqrtf(ss / (float)H + eps);
  const float k = r * r * r * dot / (float)H;
#pragma unroll
  for (int j = 0; j < MAXV; j++) {
    const int c = (threadIdx.x + j * NORM_THREADS) * 8;
    if (c < H) {
      float o[8];
      for (int i = 0; i < 8; i++) o[i] = r * gh[j][i] - k * xv[j][i];
      store8<T>(dx + (size_t)row * H + c, o);
    }
  }
}

void launch_rms_norm_bwd(bool bf16, const uint16_t* x, const uint16_t* g, const uint16_t* w, uint16_t* dx, int M,
                         int H, float eps, int unit_offset, hipStream_t st) {
  const int nv = (H / 8 + NORM_THREADS - 1) / NORM_THREADS;
#define L_BWD(TT, MV) \
  hipLaunchKernelGGL((rms_norm_bwd_kernel<TT, MV>), dim3(M), dim3(NORM_THREADS), 0, st, x, g, w, dx, H, eps, unit_offset)
  if (bf16) {
    if (nv <= 1) L_BWD(BF16, 1); else if (nv <= 2) L_BWD(BF16, 2); else if (nv <= 4) L_BWD(BF16, 4); else L_BWD(BF16, 8);
  } else {
    if (nv <= 1) L_BWD(F16, 1); else if (nv <= 2) L_BWD(F16, 2); else if (nv <= 4) L_BWD(F16, 4); else L_BWD(F16, 8);
  }
#undef L_BWD
}

void launch_add_rms_norm(bool bf16, const NormArgs& a, hipStream_t st) {
  if (bf16) launch_add_rms<BF16>(a, st); else launch_add_rms<F16>(a, st);
}

void launch_layer_norm(bool bf16, const uint16_t* x, const uint16_t* w, const uint16_t* b,
                       uint16_t* out, int M, int H, float eps, hipStream_t st) {
  const int nv = (H / 8 + NORM_THREADS - 1) / NORM_THREADS;
#define L_LN(TT, MV) \
  hipLaunchKernelGGL((layer_norm_kernel<TT, MV>), dim3(M), dim3(NORM_THREADS), 0, st, x, w, b, out, H, eps)
  if (bf16) {
    if (nv <= 1) L_LN(BF16, 1); else if (nv <= 2) L_LN(BF16, 2); else if (nv <= 4) L_LN(BF16, 4); else L_LN(BF16, 8);
  } else {
    if (nv <= 1) L_LN(F16, 1); else if (nv <= 2) L_LN(F16, 2); else if (nv <= 4) L_LN(F16, 4); else L_LN(F16, 8);
  }
#undef L_LN
}

}  // namespace illm
