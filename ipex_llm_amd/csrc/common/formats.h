// Low-bit weight formats shared by the C++ host library (quantizers, CPU
// GEMM, repacker) and the HIP kernels.
//
// Canonical ("planar") blob for a weight W[N, K]  (checkpoint / CPU layout)
//   codes : N rows x (K * bits / 8) bytes.  4-bit: inside each 64-element
//           block byte j holds code[j] (low nibble) and code[j+32] (high).
//           8-bit: byte j holds code[j].
//   scales: N x K/64 fp16, row-major
//   mins  : N x K/64 fp16 (asym formats only)
//
// Device ("tiled") blob, MI355X gfx950 MFMA fragment order.  N is padded to
// a multiple of 16 rows, K to a multiple of 128.  Tile t = n/16, chunk
// c = k/128, KC = Kp/128.  Every tile owns one contiguous region of
// dev_tile_bytes(f, KC) bytes (tiles in order, +16 B tail pad):
//   [codes of chunks 0..KC-1][scales [KC][16 rows][2 blocks] fp16][mins, asym]
// One wave64 streams one chunk with one global_load_dwordx4 per lane per
// KiB of codes:
//   lane l: A-operand row r = l & 15, k-group g = l >> 4
//   4-bit: 16 B at T + c*1024 + l*16; dword s (0..3) = k-step s, holds
//          the 8 codes k = 128c + 32s + 8g + j; nibble position p holds
//          element j = dev_nib_pos (so (u >> 4q) & 0x000F000F yields the
//          packed pair (2q, 2q+1) of the A fragment).
//   8-bit: 32 B per lane, two 16-B halves h at T + c*2048 + (h*64 + l)*16;
//          half h holds k-steps 2h, 2h+1, each as 8 bytes in element order.
//   scales: one dword (blk0 | blk1 << 16) per (row, chunk), chunk-major
//          ([KC][16 rows], dev_scale_off): the 4 MFMA C-fragment rows
//          4g..4g+3 of a chunk are one 16-B load, so the decode GEMV applies
//          block scales on the accumulator side; mins follow the same
//          layout (asym only).
#pragma once
#include <stdint.h>

namespace illm {

enum Fmt : int {
  FMT_SYM_INT4 = 0,
  FMT_ASYM_INT4 = 1,
  FMT_NF4 = 2,
  FMT_FP4 = 3,
  FMT_SYM_INT8 = 4,
  FMT_FP8E4 = 5,
  FMT_FP8E5 = 6,
  FMT_SYM_INT5 = 7,
  FMT_ASYM_INT5 = 8,
  FMT_NF3 = 9,
  FMT_FP6 = 10,
  FMT_COUNT = 11,
};

constexpr int QBLOCK = 64;      // elements per scale block
constexpr int TILE_N = 16;      // rows per device tile
constexpr int CHUNK_K = 128;    // K per device chunk

constexpr int fmt_bits(int f) {
  switch (f) {
    case FMT_SYM_INT4: case FMT_ASYM_INT4: case FMT_NF4: case FMT_FP4: case FMT_NF3:
      return 4;
    default:
      return 8;
  }
}
constexpr bool fmt_has_min(int f) { return f == FMT_ASYM_INT4 || f == FMT_ASYM_INT5; }

// nibble position p -> fragment element j
constexpr int perm4(int p) { return p < 4 ? 2 * p : 2 * (p - 4) + 1; }
// fragment element j -> nibble position p
constexpr int iperm4(int j) { return (j & 1) ? 4 + (j >> 1) : (j >> 1); }
// Device nibble position of fragment element j inside a code dword: integer
// 4-bit formats use the magic-number decode order (perm4); LUT formats
// (nf4/fp4/nf3) keep natural order so byte b = elements (2b, 2b+1) feeds
// v_cvt_scalef32_pk_*_fp4 / a 256-entry pair table directly.
constexpr int dev_nib_pos(int f, int j) {
  return (f == 0 || f == 1) ? iperm4(j) : j;
}

static const float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
    0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
    0.7229568362236023f, 1.0f};
static const float kNF3[16] = {-1.0f, -0.5350227355957031f, -0.2469314038753510f, 0.0f,
                               0.1833375245332718f, 0.3819939494132996f,
                               0.6229856610298157f, 1.0f, 0, 0, 0, 0, 0, 0, 0, 0};
static const float kFP4[16] = {0.0f, 0.5f, 1.0f, 1.5f, 2.0f, 3.0f, 4.0f, 6.0f,
                               -0.0f, -0.5f, -1.0f, -1.5f, -2.0f, -3.0f, -4.0f, -6.0f};

// Byte sizes of the planes.
constexpr int64_t canon_code_bytes(int f, int64_t n, int64_t k) { return n * k * fmt_bits(f) / 8; }
constexpr int64_t canon_scale_elems(int64_t n, int64_t k) { return n * (k / QBLOCK); }
constexpr int64_t pad_to(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
// Device tile region (see the layout comment above).
constexpr int64_t dev_code_chunk(int f) { return fmt_bits(f) == 4 ? 1024 : 2048; }
constexpr int64_t dev_tile_bytes(int f, int64_t KC) {
  return KC * dev_code_chunk(f) + TILE_N * KC * 4 * (fmt_has_min(f) ? 2 : 1);
}
// byte offset (within a tile region) of the scale dword of (row r, chunk c)
constexpr int64_t dev_scale_off(int f, int64_t KC, int r, int64_t c) {
  return KC * dev_code_chunk(f) + (c * TILE_N + r) * 4;
}
// byte offset of the min dword of (row r, chunk c) (asym formats)
constexpr int64_t dev_min_off(int f, int64_t KC, int r, int64_t c) {
  return dev_scale_off(f, KC, r, c) + (int64_t)TILE_N * KC * 4;
}
constexpr int64_t canon_total_bytes(int f, int64_t n, int64_t k) {
  return canon_code_bytes(f, n, k) + canon_scale_elems(n, k) * 2 * (fmt_has_min(f) ? 2 : 1);
}
constexpr int64_t dev_total_bytes(int f, int64_t n, int64_t k) {
  return pad_to(n, TILE_N) / TILE_N * dev_tile_bytes(f, pad_to(k, CHUNK_K) / CHUNK_K) + 16;
}

}  // namespace illm
