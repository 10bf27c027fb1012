// Fused multi-tensor AdamW: ONE launch updates every parameter of a group.
//
// The reference trains with torch's AdamW through HF Trainer (one or more
// kernels per parameter tensor).  QLoRA has hundreds of small adapter
// tensors (2 per adapted linear x 7 linears x N layers), so per-tensor
// launches dominate the optimizer step.  Here a chunk table maps each
// workgroup to (tensor, 16 KiB-element chunk); each thread updates
// 4 elements with f32 math, reading/writing params in their own dtype
// (f32 or bf16) and keeping f32 moments.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

constexpr int ADAM_THREADS = 256;

__device__ __forceinline__ float ld(const void* p, int64_t i, int dt) {
  return dt == 0 ? ((const float*)p)[i] : bf16_to_f32(((const uint16_t*)p)[i]);
}
__device__ __forceinline__ void st(void* p, int64_t i, int dt, float v) {
  if (dt == 0) ((float*)p)[i] = v;
  else ((uint16_t*)p)[i] = f32_to_bf16(v);
}

__global__ void __launch_bounds__(ADAM_THREADS) fused_adamw_kernel(AdamWArgs a) {
  const int c = blockIdx.x;
  const int t = a.chunk_tensor[c];
  const int64_t start = a.chunk_start[c];
  const int64_t n = a.sizes[t];
  void* p = (void*)a.params[t];
  const void* g = (const void*)a.grads[t];
  float* m = (float*)a.exp_avg[t];
  float* v = (float*)a.exp_avg_sq[t];
  const int64_t end = min(n, start + (int64_t)a.chunk);
  float lr = a.lr, bc1 = a.bias_corr1, bc2 = a.bias_corr2;
  if (a.step_lr) {
    const float stp = a.step_lr[0];
    lr = a.step_lr[1];
    bc1 = 1.f - powf(a.beta1, stp);
    bc2 = 1.f - powf(a.beta2, stp);
  }
  for (int64_t i = start + threadIdx.x; i < end; i += ADAM_THREADS) {
    float gi = ld(g, i, a.grad_dtype) * a.grad_scale;
    float pi = ld(p, i, a.param_dtype);
    pi *= 1.f - lr * a.weight_decay;                  // decoupled weight decay
    const float mi = a.beta1 * m[i] + (1.f - a.beta1) * gi;
    const float vi = a.beta2 * v[i] + (1.f - a.beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi / bc2) + a.eps;
    pi -= lr * (mi / bc1) / denom;
    st(p, i, a.param_dtype, pi);
  }
}

void launch_fused_adamw(const AdamWArgs& a, int nchunks, hipStream_t st) {
  if (nchunks > 0) hipLaunchKernelGGL(fused_adamw_kernel, dim3(nchunks), dim3(ADAM_THREADS), 0, st, a);
}

}  // namespace illm
