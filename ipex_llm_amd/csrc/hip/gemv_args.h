// Host/device-shared argument block and enums of the low-bit GEMV
// (lowbit_gemv.cuh).  No device code: included by the torch op wrappers.
#pragma once
#include <stdint.h>

#include "../common/formats.h"

namespace illm {

// EPI_ATOMIC: f32 atomic adds into a zero-initialised [M][N] accumulator (the
// consumer reads ONE slab and re-zeroes it), so split-K needs no slab reduce
enum GemvEpi : int { EPI_STORE = 0, EPI_PARTIAL = 1, EPI_GLU = 2, EPI_ATOMIC = 3 };
enum DecKind : int {
  DK_INT4S = 0,  // sym_int4 / woq_int4
  DK_INT4A = 1,  // asym_int4
  DK_LUT4 = 2,   // nf4 / nf3 (LDS pair table)
  DK_FP4 = 3,    // fp4 e2m1 (hardware converter)
  DK_INT8S = 4,  // sym_int8 / sym_int5 (signed byte)
  DK_INT8A = 5,  // asym_int5 (unsigned byte + min)
  DK_FP8E4 = 6,  // fp8_e4m3 / fp6 (e3m2 grid stored as e4m3)
  DK_FP8E5 = 7,  // fp8_e5m2
};

// constexpr functions are implicitly host+device under clang HIP
constexpr int dk_bits(int dk) { return dk <= DK_FP4 ? 4 : 8; }
constexpr bool dk_has_min(int dk) { return dk == DK_INT4A || dk == DK_INT8A; }
// code bytes of one (tile, chunk) and bytes of one tile region (formats.h)
constexpr int dk_code_chunk(int dk) { return dk_bits(dk) * 256; }
constexpr int64_t dk_tile_bytes(int dk, int64_t KC) {
  return KC * dk_code_chunk(dk) + 16 * KC * 4 * (dk_has_min(dk) ? 2 : 1);
}
constexpr bool dk_needx(int dk) {
  return dk == DK_INT4S || dk == DK_INT4A || dk == DK_INT8S || dk == DK_INT8A;
}
inline int fmt_to_dk(int fmt) {
  switch (fmt) {
    case FMT_SYM_INT4: return DK_INT4S;
    case FMT_ASYM_INT4: return DK_INT4A;
    case FMT_NF4: case FMT_NF3: return DK_LUT4;
    case FMT_FP4: return DK_FP4;
    case FMT_SYM_INT8: case FMT_SYM_INT5: return DK_INT8S;
    case FMT_ASYM_INT5: return DK_INT8A;
    case FMT_FP8E4: case FMT_FP6: return DK_FP8E4;
    case FMT_FP8E5: return DK_FP8E5;
  }
  return -1;
}

struct GemvArgs {
  const uint16_t* x;  // [M, ldx] activations (bf16/f16 bits)
  int M, K, ldx;
  const uint8_t* w;        // device blob: (tile, chunk) records (formats.h)
  int N, KC;               // logical out features, K chunks (Kp / 128)
  void* out;               // EPI_STORE/GLU: T [M, ldo]; EPI_PARTIAL: f32 [ks][M][N]
  int ldo;
  const uint16_t* bias;    // T [N] or null (EPI_STORE only)
  int act;                 // EPI_GLU: 0 = silu, 1 = gelu(tanh)
  int lut_fmt;             // DK_LUT4: FMT_NF4 / FMT_NF3
  // grouped (MoE) launch: blockIdx.z = expert; null for a plain GEMV
  const int32_t* moe_off;  // [E + 1] pair offsets per expert
  const int32_t* moe_rows; // [P] pair ids sorted by expert
  int moe_xdiv;            // x row of pair p = p / moe_xdiv
  // grouped EPI_ATOMIC: pair p adds moe_w[p] * y into output row p / moe_odiv
  // (the routing-weighted combine of the down projection; null = row p)
  const float* moe_w;
  int moe_odiv;
  int64_t w_stride;        // bytes between experts' weight blobs
  int waves;               // v4: waves per workgroup (4 or 8; 0 = 4)
  int cpk;                 // v4: chunks per split-K slice (multiple of 4 enables quad scale loads; 0 = derive)
  // v4 GLU-input prologue: x[m, k] = act(sum_s P[s, m, g(k)]) * sum_s P[s, m, u(k)] from the
  // gate/up GEMV's split-K slabs P [xpart_ns, M, 2K] (16-row tile-interleaved gate/up columns)
  const float* xpart;
  int xpart_ns;
  // v5 int4 decode constants (set by the launcher): packed-pair nibble mask
  // and magic exponent; runtime values so hipcc emits one v_and_or_b32
  uint32_t nib_mask, nib_magic;
  int nw;                  // v5 waves per workgroup (4 or 8)
  // v5 attention-combine prologue (o_proj over flash-decoding partials): x[m, h*D + d] =
  // sum_s w_s po[b, h, t, s, d] / L with m = b*Tq + t, split weights from pml and seq_lens
  const float* apo;        // [B, Hq, Tq, ans, D] f32 or null
  const float* aml;        // [B, Hq, Tq, ans, 2] (max, sum)
  const int32_t* alens;    // [B] keys per sequence (valid splits = ceil(len / 64))
  int ans, aD, aHq, aTq;
  // v5 residual-add + RMSNorm prologue (decode, M <= 16): the input row is
  // x = w * rms_norm(h), h = round(round(nacc) + nres), computed per workgroup
  // over the full row (sum of squares) and staged for its K slice; workgroup
  // (0, 0) writes h to nres_out (the caller ping-pongs residual buffers).
  const float* nacc;       // [M, K] f32 atomic accumulator of the previous projection
  const uint16_t* nres;    // [M, K] residual in
  uint16_t* nres_out;      // [M, K] residual out
  const uint16_t* nweight; // [K] norm weight
  float neps;
  int nunit;               // weight is stored as (w - 1) (gemma-style unit offset)
  // workgroup (0, 0) zeroes nzero[0:nzero_n] on entry: an atomic accumulator
  // whose readers all finished before this launch (stream order)
  float* nzero;
  int nzero_n;
  int pf8;                 // v5: request a <= 8-chunk split-K slice in one go (ILLM_GEMV5_PF8)
  // deferred RMSNorm (ndefer = 1, with the nacc/nres/nweight inputs above):
  // each workgroup stages x' = w * h for its own K slice only (no full-row
  // pass); the per-row sum of squares of h goes to nss [M] (split-K: the
  // workgroups of grid column 0 add their slice with one atomic per row) and
  // the consumer applies rsqrt(ss / K + eps), which commutes with the
  // projection.  GLU launches (full K per workgroup) apply it themselves.
  int ndefer;
  float* nss;
  // glu-in prologue of a deferred-norm gate/up accumulator: its rows are
  // scaled by rsqrt(xpss[m] / xpss_n + xpss_eps) before the activation
  const float* xpss;
  int xpss_n;
  float xpss_eps;
  // NeoX RoPE applied to the split-K partial sums before the atomic add
  // (rotation is linear, so the accumulator ends up holding rotated q / k):
  // output columns [0, rcols) are heads of rD dims, rotated at position
  // rpos[m] with the f32 (cos, sin) table rcs [max_pos][rD / 2][2]; needs
  // head-aligned workgroup column blocks (TG * TPW * 16 a multiple of rD)
  const float* rcs;
  const int64_t* rpos;
  int rcols, rD;
  int* err;                // kernel error word: set by the dispatcher in ILLM_DEVICE_DEBUG builds
  // EPI_STORE (v5, plain): greedy-decode argmax partials of the stored (T-rounded)
  // outputs: wave (blockIdx.x * TG + tile group) writes {max, index as int bits}
  // of its columns for every row m to amax[part * M + m] (first index on ties)
  float2* amax;
  // EPI_ATOMIC norm-out (decode o_proj -> gate/up, no standalone norm launch):
  // the last of the gridDim.y split-K workgroups of column block blockIdx.x
  // (ticket lctr[blockIdx.x], reset by that workgroup) reads the block's
  // finished sums back (sc1), forms h = rnd(rnd(acc) + lres) exactly as
  // add_rms_norm rounds it, writes lres_out = h and the deferred-norm input
  // lxo = rnd(w * h), re-zeroes its slice of the accumulator and adds the
  // rows' sums of squares of h to lss [M]; the GLU GEMV applies
  // rsqrt(lss / N + eps) in its epilogue (xpss below)
  int* lctr;
  const uint16_t* lres;
  uint16_t* lres_out;
  const uint16_t* lnw;
  uint16_t* lxo;
  float* lss;
  int lunit;
};

}  // namespace illm
