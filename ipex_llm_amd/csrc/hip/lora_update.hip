// Low-rank accumulate C[M, N] += alpha * A[M, r] B[N, r]^T (r <= 64) on the
// matrix cores: the LoRA term of the QLoRA linear (y += s (x A^T) B^T) and of
// its grad_x (gx += (s g B) A).  Reference: LoraLowBitLinear.forward
// (SRC/transformers/qlora.py:114-143), which adds the adapter output as a
// separate GEMM + add.
//
// Why a kernel of its own: with K = r (8-64) the library GEMM runs a
// 256 x 128 x 32 macro-tile at ~0.4 TB/s of C traffic (MI355X, QLoRA step:
// 93 us for a [4096, 4096] bf16 C, profiles/qlora_llama3_8b_r4_final_rocprof.txt);
// the update is a pure read-modify-write of C.
//
// MI355X design: one wave per 16 rows x (16 x NT) columns.  D^T = B A^T on
// v_mfma_f32_16x16x32: the A operand is B's row n (r contiguous bf16 of one
// adapter row, 16 B per lane), the B operand is A's row m; the result lane
// holds C[m][n .. n + 3] -- four consecutive columns of one row -- so C is
// read and written with 8-B vector accesses in its natural layout.  Every C
// load of the wave's strip is issued before the first MFMA (one memory
// latency per wave), k > r lanes feed zeros, fp32 math, one rounding.
#include "illm_device.h"
#include "kernels.h"

namespace illm {

namespace {

constexpr int LU_NT = 16;      // 16-column tiles per wave (256 columns)

template <typename T>
__global__ void __launch_bounds__(256) lora_update_kernel(uint16_t* C, int64_t ldc, const uint16_t* A, int64_t lda,
                                                          const uint16_t* Bm, int64_t ldb, int M, int N, int r,
                                                          float alpha) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int m0 = blockIdx.y * 16;
  const int n_strip = (blockIdx.x * 4 + wave) * (16 * LU_NT);
  if (n_strip >= N) return;
  const int m = m0 + c16;                    // this lane's row (B operand / output row)
  const int mc = min(m, M - 1);
  // A fragments (row m, k = 8 g .. + 7 of each 32-chunk); k >= r -> 0
  uint4 af[2];
#pragma unroll
  for (int kc = 0; kc < 2; kc++) {
    const int k = kc * 32 + 8 * g;
    af[kc] = k < r ? *(const uint4*)(A + (size_t)mc * lda + k) : make_uint4(0, 0, 0, 0);
  }
  const int nkc = r > 32 ? 2 : 1;
  // C strip: lane holds C[m][n0 + 4 g .. + 3] of each tile
  uint2 cv[LU_NT];
#pragma unroll
  for (int t = 0; t < LU_NT; t++) {
    const int n = n_strip + t * 16 + 4 * g;
    cv[t] = (m < M && n < N) ? *(const uint2*)(C + (size_t)m * ldc + n) : make_uint2(0, 0);
  }
#pragma unroll
  for (int t = 0; t < LU_NT; t++) {
    const int nb = n_strip + t * 16;
    if (nb >= N) break;
    const int nr = min(nb + c16, N - 1);     // this lane's adapter row (A operand)
    f32x4 p = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < nkc; kc++) {
      const int k = kc * 32 + 8 * g;
      const uint4 bf = k < r ? *(const uint4*)(Bm + (size_t)nr * ldb + k) : make_uint4(0, 0, 0, 0);
      p = mfma16<T>(bf, af[kc], p);
    }
    const int n = nb + 4 * g;
    if (m < M && n < N) {
      const uint2 c = cv[t];
      const float o0 = to_f32<T>(c.x & 0xffff) + alpha * p[0], o1 = to_f32<T>(c.x >> 16) + alpha * p[1];
      const float o2 = to_f32<T>(c.y & 0xffff) + alpha * p[2], o3 = to_f32<T>(c.y >> 16) + alpha * p[3];
      *(uint2*)(C + (size_t)m * ldc + n) = make_uint2(pack2<T>(o0, o1), pack2<T>(o2, o3));
    }
  }
}

}  // namespace

void launch_lora_update(bool bf16, uint16_t* C, int64_t ldc, const uint16_t* A, int64_t lda, const uint16_t* B,
                        int64_t ldb, int M, int N, int r, float alpha, hipStream_t st) {
  const int strips = (N + 16 * LU_NT - 1) / (16 * LU_NT);
  dim3 grid((unsigned)((strips + 3) / 4), (unsigned)((M + 15) / 16));
  if (bf16)
    hipLaunchKernelGGL(lora_update_kernel<BF16>, grid, dim3(256), 0, st, C, ldc, A, lda, B, ldb, M, N, r, alpha);
  else
    hipLaunchKernelGGL(lora_update_kernel<F16>, grid, dim3(256), 0, st, C, ldc, A, lda, B, ldb, M, N, r, alpha);
}

}  // namespace illm
