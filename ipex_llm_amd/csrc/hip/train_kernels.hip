// Training kernels of the QLoRA step (reference recipe
// SRC/transformers/qlora.py + HF Trainer):
//   * fused softmax cross-entropy over an lm_head logits chunk: per row the
//     loss and, in place, the logits gradient (softmax - onehot) * scale --
//     the [tokens, vocab] f32 upcast + softmax + its backward of the HF loss
//     never exist (one read for the row max / sum, one read + write for the
//     gradient);
//   * skinny reductions over the token axis for the LoRA adapter gradients
//     (out[r, n] = sum_m a[m, r] * b[m, n], r <= 64): one pass over b.
#include <cstdlib>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

namespace {

// one workgroup (256 threads) per row; V % 8 == 0
template <typename T>
__global__ void __launch_bounds__(256) ce_fused_kernel(uint16_t* logits, int64_t ld, int V, const int64_t* labels,
                                                       int ignore_index, float scale, float* loss,
                                                       int write_grad) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  uint16_t* lr = logits + row * ld;
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < V;
  // pass 1: online max / sum of exp over the row (8 elements per thread step)
  float m = -INFINITY, s = 0.f;
  for (int k = threadIdx.x * 8; k < V; k += 256 * 8) {
    const uint4 v = *(const uint4*)(lr + k);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float x[8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      x[2 * j] = to_f32<T>(w[j] & 0xffff);
      x[2 * j + 1] = to_f32<T>(w[j] >> 16);
    }
    float tm = x[0];
#pragma unroll
    for (int j = 1; j < 8; j++) tm = fmaxf(tm, x[j]);
    const float mn = fmaxf(m, tm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) acc += __expf(x[j] - mn);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + acc;
    m = mn;
  }
  // wave reduction of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[w] = m; red[4 + w] = s; }
  __syncthreads();
  float M = red[0], S = red[4];
#pragma unroll
  for (int i = 1; i < 4; i++) {
    const float mn = fmaxf(M, red[i]);
    S = S * __expf(M - mn) + red[4 + i] * __expf(red[i] - mn);
    M = mn;
  }
  const float lse = M + __logf(S);
  if (threadIdx.x == 0) loss[row] = valid ? lse - to_f32<T>(lr[lab]) : 0.f;
  if (!write_grad) return;
  __syncthreads();                       // the label logit was read before any gradient is written
  // pass 2: gradient (softmax - onehot) * scale in place (0 for ignored rows)
  const float sc = valid ? scale : 0.f;
  for (int k = threadIdx.x * 8; k < V; k += 256 * 8) {
    const uint4 v = *(const uint4*)(lr + k);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      float a0 = __expf(to_f32<T>(wv[j] & 0xffff) - lse), a1 = __expf(to_f32<T>(wv[j] >> 16) - lse);
      if (k + 2 * j == lab) a0 -= 1.f;
      if (k + 2 * j + 1 == lab) a1 -= 1.f;
      o[j] = pack2<T>(a0 * sc, a1 * sc);
    }
    *(uint4*)(lr + k) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// out[r, n] (+)= alpha * sum_m a[m, r] * b[m, n]: a f32 [M, rr] (rr <= R <=
// 64), b 16-bit [M, ldb]; each workgroup owns 64 * COLS columns (COLS per
// thread: 16-B loads at R <= 16) and a slice of rows, f32 atomics into out
// (zeroed by the caller)
template <typename T, int R, int COLS>
__global__ void __launch_bounds__(64) skinny_tn_kernel(const float* a, int rr, const uint16_t* b, int64_t ldb, int M,
                                                       int N, int rows_per, float alpha, float* out) {
  __shared__ float as[64 * R];
  const int n = (blockIdx.x * 64 + threadIdx.x) * COLS;
  const int m0 = blockIdx.y * rows_per, m1 = min(M, m0 + rows_per);
  float acc[R][COLS];
#pragma unroll
  for (int r = 0; r < R; r++)
#pragma unroll
    for (int j = 0; j < COLS; j++) acc[r][j] = 0.f;
  for (int mb = m0; mb < m1; mb += 64) {
    const int cnt = min(64, m1 - mb);
    __syncthreads();
    for (int i = threadIdx.x; i < cnt * R; i += 64) {
      const int mi = i / R, r = i % R;
      as[i] = r < rr ? a[(size_t)(mb + mi) * rr + r] : 0.f;
    }
    __syncthreads();
    if (n < N) {
      for (int i = 0; i < cnt; i++) {
        const uint16_t* bp = b + (size_t)(mb + i) * ldb + n;
        float x[COLS];
        if constexpr (COLS == 8) {
          const uint4 v = *(const uint4*)bp;
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int j = 0; j < 4; j++) { x[2 * j] = to_f32<T>(w[j] & 0xffff); x[2 * j + 1] = to_f32<T>(w[j] >> 16); }
        } else if constexpr (COLS == 4) {
          const uint2 v = *(const uint2*)bp;
          x[0] = to_f32<T>(v.x & 0xffff); x[1] = to_f32<T>(v.x >> 16);
          x[2] = to_f32<T>(v.y & 0xffff); x[3] = to_f32<T>(v.y >> 16);
        } else {
          const uint32_t v = *(const uint32_t*)bp;
          x[0] = to_f32<T>(v & 0xffff); x[1] = to_f32<T>(v >> 16);
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
          const float av = as[i * R + r];
#pragma unroll
          for (int j = 0; j < COLS; j++) acc[r][j] = fmaf(av, x[j], acc[r][j]);
        }
      }
    }
  }
  if (n >= N) return;
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (r >= rr) break;
#pragma unroll
    for (int j = 0; j < COLS; j++) atomicAdd(out + (size_t)r * N + n + j, alpha * acc[r][j]);
  }
}

template <typename T, int R, int COLS>
void launch_tn(const float* a, int rr, const uint16_t* b, int64_t ldb, int M, int N, float alpha, float* out,
               hipStream_t st) {
  const int cols = (N + 64 * COLS - 1) / (64 * COLS);
  // enough row slices for ~2 workgroups per CU, >= 64 rows each
  int slices = max(1, min((M + 63) / 64, 512 / max(1, cols)));
  const int rows_per = ((M + slices - 1) / slices + 63) / 64 * 64;
  slices = (M + rows_per - 1) / rows_per;
  hipLaunchKernelGGL((skinny_tn_kernel<T, R, COLS>), dim3((unsigned)cols, (unsigned)slices), dim3(64), 0, st, a, rr,
                     b, ldb, M, N, rows_per, alpha, out);
}

}  // namespace

void launch_ce_fused(bool bf16, uint16_t* logits, int64_t rows, int64_t ld, int V, const int64_t* labels,
                     int ignore_index, float scale, float* loss, bool write_grad, hipStream_t st) {
  if (rows <= 0) return;
  if (bf16)
    hipLaunchKernelGGL(ce_fused_kernel<BF16>, dim3((unsigned)rows), dim3(256), 0, st, logits, ld, V, labels,
                       ignore_index, scale, loss, write_grad ? 1 : 0);
  else
    hipLaunchKernelGGL(ce_fused_kernel<F16>, dim3((unsigned)rows), dim3(256), 0, st, logits, ld, V, labels,
                       ignore_index, scale, loss, write_grad ? 1 : 0);
}

void launch_skinny_tn(bool bf16, const float* a, int R, const uint16_t* b, int64_t ldb, int M, int N, float alpha,
                      float* out, hipStream_t st) {
#define ILLM_TN(RR, CC)                                                          \
  if (R <= RR) {                                                                 \
    if (bf16) launch_tn<BF16, RR, CC>(a, R, b, ldb, M, N, alpha, out, st);       \
    else launch_tn<F16, RR, CC>(a, R, b, ldb, M, N, alpha, out, st);             \
    return;                                                                      \
  }
  ILLM_TN(8, 8)
  ILLM_TN(16, 8)
  ILLM_TN(32, 4)
  ILLM_TN(64, 2)
#undef ILLM_TN
}

}  // namespace illm
