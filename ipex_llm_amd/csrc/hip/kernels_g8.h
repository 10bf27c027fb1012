// Host-callable launcher of the 8-phase 256x256 bf16 GEMM (gemm_8p.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace illm {

struct G8Args {
  const uint16_t* x;      // [M, ldx] bf16
  const uint16_t* w;      // [N, ldw] bf16
  const uint16_t* bias;   // [N] bf16 or null
  void* out;              // [M, ldo] bf16 or f32
  int M, N, K;            // K % 64 == 0
  int ldx, ldw, ldo;
  int out_f32;
  uint32_t x_bytes, w_bytes;   // buffer extents (reads past them return 0)
  int w_fmt;              // -1: dense bf16 w; else a low-bit device-blob format (gemm8p_supports)
  int lut_fmt;            // LUT formats: the code table (FMT_NF4 / FMT_NF3)
  int glu, act;           // glu: w rows are 16-row gate/up tile pairs, out [M, N/2] = act(gate) * up
  // fp8 (w_fmt == G8_FP8): x = e4m3 bytes [M, ldx], w = e4m3 / e5m2 bytes [N, ldw],
  // y = sx[m] * sw[n] * (xq . wq) (+ bias), 16-bit out (bf16, or f16 if out_f16)
  const float* sx;
  const float* sw;
  int sw_per_channel, w_e5m2, out_f16;
  // split-K (dense bf16 only): ksplit > 1 workgroups per output tile, each
  // over a K-tile range, store f32 partials into slab ks of ws [ksplit, M, N]
  // (no zeroing, no atomics); launch_gemm8p_finish sums the slabs, applies
  // bias / GLU and rounds
  int ksplit;
  float* ws;
  int gm;                 // m-blocks per rasterization group (0: 4)
  int accum;              // dense, no GLU: out += x w^T instead of out = (bf16: one rounding of old + sum)
};
constexpr int G8_FP8 = -2;

void launch_gemm8p(const G8Args& a, hipStream_t st);
// out = round(ws (+ bias)) or GLU over ws: the split-K epilogue
void launch_gemm8p_finish(const G8Args& a, hipStream_t st);
// split-K factor for a grid of fewer 256 x 256 tiles than half the CUs (each
// split >= 8 K-tiles; 1 = no split)
int gemm8p_auto_split(int64_t M, int64_t N, int64_t ktiles);
bool gemm8p_supports(int fmt);

}  // namespace illm
