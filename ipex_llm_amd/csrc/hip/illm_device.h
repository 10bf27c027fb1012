// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
// Wave64 everywhere: lane = threadIdx.x & 63.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../common/formats.h"

namespace illm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// dtype tags: activations travel as raw 16-bit patterns
struct BF16 {};
struct F16 {};

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // round-to-nearest-even; NaN stays NaN (hipcc lowers the cast to v_cvt_pk_bf16_f32)
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float f16_to_f32(uint16_t v) {
  return (float)__builtin_bit_cast(_Float16, v);
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}

template <typename T> __device__ __forceinline__ float to_f32(uint16_t v);
template <> __device__ __forceinline__ float to_f32<BF16>(uint16_t v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float to_f32<F16>(uint16_t v) { return f16_to_f32(v); }
template <typename T> __device__ __forceinline__ uint16_t from_f32(float f);
template <> __device__ __forceinline__ uint16_t from_f32<BF16>(float f) { return f32_to_bf16(f); }
template <> __device__ __forceinline__ uint16_t from_f32<F16>(float f) { return f32_to_f16(f); }

// pack two f32 into one dword of two 16-bit values (lo = a)
template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b);
// (one vector conversion: a single v_cvt_pk_bf16_f32 / v_cvt_pkrtz-free
// v_cvt_f16 pair instead of two scalar converts + shift + or)
typedef float illm_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 illm_bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 illm_f16x2 __attribute__((ext_vector_type(2)));
template <> __device__ __forceinline__ uint32_t pack2<BF16>(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((illm_f32x2){a, b}, illm_bf16x2));
}
template <> __device__ __forceinline__ uint32_t pack2<F16>(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((illm_f32x2){a, b}, illm_f16x2));
}

// 16x16x32 MFMA on raw 16-byte fragments
template <typename T>
__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mfma16<BF16>(const uint4& a, const uint4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mfma16<F16>(const uint4& a, const uint4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// [row][D] 16-bit tile in LDS with a 16-byte XOR swizzle: chunk c of row r
// lives at chunk c ^ (r & 15) (D >= 128: 16 chunks per row; D = 64: r & 7),
// so both row-wise b128 reads and the transposed reads below are conflict-free
template <int D>
__device__ __forceinline__ int pf_off(int r, int c) {
  constexpr int CH = D / 8;            // 16-B chunks per row
  constexpr int MSK = CH >= 16 ? 15 : CH - 1;
  return r * D + ((c ^ (r & MSK)) * 8);
}

// gfx950 ds_read_b64_tr_b16: transposed read of a 16-bit tile (the MFMA A/B
// fragment of a row-major [k][n] tile read along k)
__device__ __forceinline__ uint2 ds_read_tr16(const uint16_t* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  const s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
  return __builtin_bit_cast(uint2, v);
}

// write-through (sc1) stores / L1-bypassing (sc1) loads of data handed to
// the last-arriving workgroup of a launch: the MI355X hand-off form "sc1
// stores, s_waitcnt vmcnt(0), one agent-scope atomic add per workgroup, sc1
// loads by the workgroup whose add came last" (no __threadfence / L2
// write-back on the critical path)
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B / 8-B forms of the same hand-off (a scalarised 4-B sc1 store per
// element is several times slower per byte): buffer_store/load_dwordx4 with
// the sc1 bit (aux 16) through a raw buffer descriptor on `base`
// (gfx9 word 3 = 0x00020000), and 8-B agent-scope atomic stores / loads
typedef unsigned int illm_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_sc1(float* base, size_t elem, float4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(illm_u32x4, v), r, (int)(elem * 4), 0, 16);
}
__device__ __forceinline__ float4 ld16_sc1(const float* base, size_t elem) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 4), 0, 16));
}
__device__ __forceinline__ void st8_sc1(float* p, float a, float b) {
  const unsigned long long v = (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
  __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld8_sc1(const float* p) {
  const unsigned long long v = __hip_atomic_load((const unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)));
}

// Kernel error word (SURVEY §5.2 bounds checks): a kernel that finds an
// out-of-range index from device data (block table entry, cache slot, expert
// id) skips the access and ORs a code here; the host reads it with
// ops.check_kernel_errors() (ILLM_CHECK_KERNELS=1: after every engine step).
// The bad access never happens, so a corrupt table is an error, not a fault.
enum KernelErr : int { ERR_BLOCK_ID = 1, ERR_SLOT = 2, ERR_EXPERT = 4, ERR_SEQ_LEN = 8, ERR_TOKEN = 16,
                       ERR_GEOMETRY = 32, ERR_PEER = 64 };
__device__ __forceinline__ void kerr(int* err, int code) {
  if (err != nullptr) atomicOr(err, code);
}

// Debug build (python -m ipex_llm_amd._build --debug -> _C_debug.so, loaded
// with IPEX_LLM_AMD_LIB=_C_debug.so): ILLM_DCHECK adds launch-geometry and
// host-contract checks to the hot kernels (grid covers every output tile and
// K chunk, MoE pair offsets monotonic, ...).  A failed check prints the kernel
// site once per workgroup, ORs the code into the error word and makes the
// caller skip the work; the release build compiles the checks out entirely.
#ifndef ILLM_DEVICE_DEBUG
#define ILLM_DEVICE_DEBUG 0
#endif
#if ILLM_DEVICE_DEBUG
#define ILLM_DCHECK_FAILS(ok, err, code)                                                              \
  ([&]() -> bool {                                                                                    \
    if (ok) return false;                                                                             \
    if (threadIdx.x == 0) {                                                                           \
      printf("[illm device check] %s:%d: %s failed (block %u,%u,%u)\n", __FILE__, __LINE__, #ok,       \
             blockIdx.x, blockIdx.y, blockIdx.z);                                                     \
      kerr((err), (code));                                                                            \
    }                                                                                                 \
    return true;                                                                                      \
  }())
#else
#define ILLM_DCHECK_FAILS(ok, err, code) false
#endif
__device__ __forceinline__ bool bad_block(int blk, int num_blocks) {
  return num_blocks > 0 && (unsigned)blk >= (unsigned)num_blocks;
}

// wave-level reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-level sum for blockDim.x == NT (multiple of 64); smem >= NT/64 floats
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* smem) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  __syncthreads();
  if (l == 0) smem[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) t += smem[i];
  return t;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

}  // namespace illm

#define ILLM_CHECK_LAUNCH() (void)hipGetLastError()
