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
// holds four D^T rows of one column m.  The adapter rows fed to the four
// tiles of a 64-column block are permuted (tile t, operand row j ->
// column 16 (j / 4) + 4 t + j % 4) so that a lane ends up owning 16
// CONSECUTIVE columns of its row m: C moves as two 16-B accesses per lane per
// block and each row segment a wave touches is a whole 128-B line (the
// unpermuted layout split rows into 32-B pieces and ran at ~3 TB/s).  Every C
// load of the wave's strip is issued before the first MFMA (one memory
// latency per wave), k > r lanes feed zeros, fp32 math, one rounding.
#include <algorithm>
#include <cstdlib>

#include "illm_device.h"
#include "kernels.h"

namespace illm {

namespace {

constexpr int LU_NB = 4;       // 64-column blocks per wave (256 columns)

template <typename T>
__global__ void __launch_bounds__(256) lora_update_kernel(uint16_t* C, int64_t ldc, const uint16_t* A, int64_t lda,
                                                          const uint16_t* Bm, int64_t ldb, int M, int N, int r,
                                                          float alpha) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int m0 = blockIdx.y * 16;
  const int n_strip = (blockIdx.x * 4 + wave) * (64 * LU_NB);
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
  // C strip: lane holds C[m][nb + 16 g .. + 15] of each 64-column block (two 16-B halves)
  uint4 cv[2 * LU_NB];
#pragma unroll
  for (int b = 0; b < LU_NB; b++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int n = n_strip + 64 * b + 16 * g + 8 * h;
      cv[2 * b + h] = (m < M && n < N) ? *(const uint4*)(C + (size_t)m * ldc + n) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
  for (int b = 0; b < LU_NB; b++) {
    const int nb = n_strip + 64 * b;
    if (nb >= N) break;
    f32x4 p[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
      // operand row j = c16 of tile t -> column nb + 16 (j / 4) + 4 t + j % 4
      const int nr = min(nb + 16 * (c16 >> 2) + 4 * t + (c16 & 3), N - 1);
      p[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int kc = 0; kc < nkc; kc++) {
        const int k = kc * 32 + 8 * g;
        const uint4 bf = k < r ? *(const uint4*)(Bm + (size_t)nr * ldb + k) : make_uint4(0, 0, 0, 0);
        p[t] = mfma16<T>(bf, af[kc], p[t]);
      }
    }
    // lane: p[t][i] = D[m][nb + 16 g + 4 t + i]
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int n = nb + 16 * g + 8 * h;
      if (m < M && n < N) {
        const uint4 c = cv[2 * b + h];
        const f32x4 &pa = p[2 * h], &pb = p[2 * h + 1];
        uint4 o;
        o.x = pack2<T>(to_f32<T>(c.x & 0xffff) + alpha * pa[0], to_f32<T>(c.x >> 16) + alpha * pa[1]);
        o.y = pack2<T>(to_f32<T>(c.y & 0xffff) + alpha * pa[2], to_f32<T>(c.y >> 16) + alpha * pa[3]);
        o.z = pack2<T>(to_f32<T>(c.z & 0xffff) + alpha * pb[0], to_f32<T>(c.z >> 16) + alpha * pb[1]);
        o.w = pack2<T>(to_f32<T>(c.w & 0xffff) + alpha * pb[2], to_f32<T>(c.w >> 16) + alpha * pb[3]);
        *(uint4*)(C + (size_t)m * ldc + n) = o;
      }
    }
  }
}

// ---- token-axis reduction out[r, n] += alpha * sum_m a[m, r] b[m, n] ------------
// (the LoRA weight gradients dA = gxa^T x, dB^T = xa^T g over the M tokens).
// A workgroup (4 waves) owns 64 columns of b and a slice of the rows; 64-row
// tiles of b ([m][n], 128-B rows) and a ([m][r], zero-padded to 64 columns)
// go to LDS in the XOR-swizzled pf_off layout and BOTH MFMA operands come
// back by ds_read_b64_tr_b16 transposed reads (k = token axis): the same
// read pattern on both tiles gives both fragments the same token order, so
// D[r][n] = sum_m a^T[r][m] b[m][n] needs no register transposes.  Partial
// sums of the row slices meet in f32 atomics.
constexpr int TN_RB = 64;       // rows per LDS stage

template <typename T>
__global__ void __launch_bounds__(256) lora_tn_kernel(const uint16_t* a, int64_t lda, int r, const uint16_t* b,
                                                      int64_t ldb, int M, int N, int rows_per, float alpha,
                                                      float* out, bool trans) {
  __shared__ __attribute__((aligned(16))) uint16_t bt[TN_RB * 64];
  __shared__ __attribute__((aligned(16))) uint16_t at[TN_RB * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = blockIdx.x * 64;
  const int m_lo = blockIdx.y * rows_per, m_hi = min(M, m_lo + rows_per);
  const int nrt = (r + 15) / 16;
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int mb = m_lo; mb < m_hi; mb += TN_RB) {
    // stage 64 rows: thread -> (row tid / 4, 16-B chunks 2 (tid & 3), +1) of b and of a
    {
      const int row = tid >> 2, c0 = 2 * (tid & 3);
      const int m = mb + row;
      const bool ok = m < m_hi;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int c = c0 + j;
        const int n = n0 + 8 * c;
        uint4 vb = make_uint4(0, 0, 0, 0), va = make_uint4(0, 0, 0, 0);
        if (ok && n < N) vb = *(const uint4*)(b + (size_t)m * ldb + n);
        if (ok && 8 * c < r) va = *(const uint4*)(a + (size_t)m * lda + 8 * c);
        *(uint4*)(bt + pf_off<64>(row, c)) = vb;
        *(uint4*)(at + pf_off<64>(row, c)) = va;
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      const int qq = r16 >> 2, pp = r16 & 3;
      const int row0 = 16 * (2 * kk) + 4 * g + qq, row1 = row0 + 16;
      const int colb = 16 * wave + 4 * pp;
      const uint2 b0 = ds_read_tr16(bt + pf_off<64>(row0, colb >> 3) + (colb & 7));
      const uint2 b1 = ds_read_tr16(bt + pf_off<64>(row1, colb >> 3) + (colb & 7));
      const uint4 bf = make_uint4(b0.x, b0.y, b1.x, b1.y);
#pragma unroll
      for (int rt = 0; rt < 4; rt++) {
        if (rt >= nrt) break;
        const int cola = 16 * rt + 4 * pp;
        const uint2 a0 = ds_read_tr16(at + pf_off<64>(row0, cola >> 3) + (cola & 7));
        const uint2 a1 = ds_read_tr16(at + pf_off<64>(row1, cola >> 3) + (cola & 7));
        acc[rt] = mfma16<T>(make_uint4(a0.x, a0.y, a1.x, a1.y), bf, acc[rt]);
      }
    }
    __syncthreads();
  }
  // lane holds D[r = 16 rt + 4 g + i][n = n0 + 16 wave + r16]
  const int n = n0 + 16 * wave + r16;
  if (n >= N) return;
#pragma unroll
  for (int rt = 0; rt < 4; rt++) {
    if (rt >= nrt) break;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int rr = 16 * rt + 4 * g + i;
      // trans: out is [N, r] (the layout of a LoRA B gradient), else [r, N]
      if (rr < r) atomicAdd(out + (trans ? (size_t)n * r + rr : (size_t)rr * N + n), alpha * acc[rt][i]);
    }
  }
}

}  // namespace

void launch_lora_tn(bool bf16, const uint16_t* a, int64_t lda, int r, const uint16_t* b, int64_t ldb, int M, int N,
                    float alpha, float* out, bool trans, hipStream_t st) {
  const int nb = (N + 63) / 64;
  // row slices of >= min_rows (every slice ends in r x 64 f32 atomics per
  // workgroup), up to ~wg_target workgroups; ILLM_LORA_TN_ROWS / _WGS for sweeps
  static const int min_rows = getenv("ILLM_LORA_TN_ROWS") ? atoi(getenv("ILLM_LORA_TN_ROWS")) : 256;
  static const int wg_target = getenv("ILLM_LORA_TN_WGS") ? atoi(getenv("ILLM_LORA_TN_WGS")) : 2048;
  int splits = std::max(1, std::min((M + min_rows - 1) / std::max(TN_RB, min_rows), wg_target / std::max(1, nb)));
  const int rows_per = ((M + splits - 1) / splits + TN_RB - 1) / TN_RB * TN_RB;
  splits = (M + rows_per - 1) / rows_per;
  dim3 grid((unsigned)nb, (unsigned)splits);
  if (bf16)
    hipLaunchKernelGGL(lora_tn_kernel<BF16>, grid, dim3(256), 0, st, a, lda, r, b, ldb, M, N, rows_per, alpha, out,
                       trans);
  else
    hipLaunchKernelGGL(lora_tn_kernel<F16>, grid, dim3(256), 0, st, a, lda, r, b, ldb, M, N, rows_per, alpha, out,
                       trans);
}

void launch_lora_update(bool bf16, uint16_t* C, int64_t ldc, const uint16_t* A, int64_t lda, const uint16_t* B,
                        int64_t ldb, int M, int N, int r, float alpha, hipStream_t st) {
  const int strips = (N + 64 * LU_NB - 1) / (64 * LU_NB);
  dim3 grid((unsigned)((strips + 3) / 4), (unsigned)((M + 15) / 16));
  if (bf16)
    hipLaunchKernelGGL(lora_update_kernel<BF16>, grid, dim3(256), 0, st, C, ldc, A, lda, B, ldb, M, N, r, alpha);
  else
    hipLaunchKernelGGL(lora_update_kernel<F16>, grid, dim3(256), 0, st, C, ldc, A, lda, B, ldb, M, N, r, alpha);
}

}  // namespace illm
