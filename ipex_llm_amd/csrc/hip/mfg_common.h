// Device helpers shared by the MFMA GEMM engine kernels (gemm_mfma.hip,
// gemm_mfma_nn.hip).
#pragma once
#include <stdint.h>

#include "illm_device.h"

namespace illm {
namespace mfg {

// 16-B LDS-DMA (buffer_load_dwordx4 ... lds) through a raw buffer descriptor
// on `base`: bytes past `bytes` read as zero.  A device function, not inline
// in the kernels' lambdas: a lambda that names __amdgpu_buffer_rsrc_t makes
// hipcc silently drop the kernel's host stub.
__device__ __forceinline__ void buf_lds16(const void* base, uint32_t bytes, uint16_t* lds, uint32_t voff, int soff) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// XCD-aware bijective block remap: blocks sharing id % 8 (one XCD / L2) get
// consecutive indices of a grid of `total` blocks
__device__ __forceinline__ int xcd_remap(int id, int total) {
  const int xcd = id & 7, q8 = total >> 3, r8 = total & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (id >> 3);
}

// row swizzle of the [n][256] transposed-read weight image (NN kernels):
// 16-B chunk c of row n lives at chunk c ^ nn_swz(n), so the
// ds_read_b64_tr_b16 reads of rows {0..3, 8..11} (one 32-lane half) and the
// 16-B decode writes of 8 consecutive rows are bank-conflict free
__device__ __forceinline__ int nn_swz(int n) {
  return ((((n & 3) | ((n >> 1) & 4)) << 1) | ((n >> 2) & 1));
}

}  // namespace mfg
}  // namespace illm
