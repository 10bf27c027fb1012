// Host-callable launchers of the training attention kernels (train_attn.hip).
// Kept out of kernels.h so that edits here rebuild only their users.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace illm {

// q [B, Hq, T, D], k / v [B, Hkv, T, D] with element strides (D contiguous);
// out [B, T, Hq, D] contiguous; lse / delta [B, Hq, T] f32 (log2 domain);
// dout (grad of out) and o with strides; dq [B, Hq, T, D], dk / dv
// [B, Hkv, T, D] contiguous.  T % 64 == 0, D in {64, 128}.
struct TrainAttnArgs {
  const uint16_t* q;
  int64_t qsb, qsh, qst;
  const uint16_t* k;
  int64_t ksb, ksh, kst;
  const uint16_t* v;
  int64_t vsb, vsh, vst;
  uint16_t* out;
  const uint16_t* o;
  int64_t osb, osh, ost;
  const uint16_t* dout;
  int64_t dsb, dsh, dst;
  float* lse;
  float* delta;
  uint16_t* dq;
  uint16_t* dk;
  uint16_t* dv;
  int B, T, Hq, Hkv, D;
  float scale;
  int causal;
};
void launch_train_attn_fwd(bool bf16, const TrainAttnArgs& a, hipStream_t st);
// x_to_f16_rowscale + the LoRA down-projection of each row (gemm_mfma.hip):
// y (f16, may be null) / rs as launch_x_to_f16_rowscale; xa [M, rp] bf16 =
// alpha * x la^T for r < R (la [R, K] bf16), zero-padded to rp (R <= 64, rp % 32 == 0)
void launch_x_rowscale_lora(bool bf16, const uint16_t* x, int64_t M, int64_t ldx, int K, uint16_t* y, float* rs,
                            const uint16_t* la, int R, float alpha, uint16_t* xa, int rp, hipStream_t st);
void launch_train_attn_bwd(bool bf16, const TrainAttnArgs& a, hipStream_t st);
// C[M, N] += alpha * A[M, r] B[N, r]^T (lora_update.hip); 16-bit, r % 8 == 0,
// r <= 64, N % 4 == 0, rows of A / B 16-B aligned
void launch_lora_update(bool bf16, uint16_t* C, int64_t ldc, const uint16_t* A, int64_t lda, const uint16_t* B,
                        int64_t ldb, int M, int N, int r, float alpha, hipStream_t st);
// out[r, n] += alpha * sum_m a[m, r] b[m, n] (f32 out, zeroed by the caller; trans:
// out is [N, r]);
// 16-bit a [M, r] / b [M, N], r <= 64, r % 8 == 0, N % 8 == 0, rows 16-B aligned
void launch_lora_tn(bool bf16, const uint16_t* a, int64_t lda, int r, const uint16_t* b, int64_t ldb, int M, int N,
                    float alpha, float* out, bool trans, hipStream_t st);

}  // namespace illm
