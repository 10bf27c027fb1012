// C API of the host low-bit library (csrc/cpu/quant.cpp).
#pragma once
#include <stdint.h>

extern "C" {
int illm_fmt_bits(int fmt);
void illm_quantize(int fmt, const float* src, int64_t n, int64_t k, const float* imatrix,
                   int scale_search, uint8_t* codes, uint16_t* scales, uint16_t* mins);
void illm_dequantize(int fmt, const uint8_t* codes, const uint16_t* scales, const uint16_t* mins,
                     int64_t n, int64_t k, float* dst);
void illm_repack_to_device(int fmt, const uint8_t* codes, const uint16_t* scales,
                           const uint16_t* mins, int64_t n, int64_t k, uint8_t* dev);
void illm_repack_from_device(int fmt, const uint8_t* dev, int64_t n, int64_t k, uint8_t* codes,
                             uint16_t* scales, uint16_t* mins);
void illm_cpu_gemm(int fmt, const float* x, int64_t m, const uint8_t* codes,
                   const uint16_t* scales, const uint16_t* mins, int64_t n, int64_t k, float* y);
void illm_f32_to_fp8(const float* src, int64_t n, int e5m2, uint8_t* dst);
// gemm_q4.cpp: int8-activation integer-dot path for sym_int4 / asym_int4
// (isa: 0 = auto, 1 = AVX2, 2 = AVX-512 VNNI)
int illm_cpu_q4_supported(int fmt);
// kquant.cpp: GGUF k-quant super-block formats (fmt 11..14, common/kquant.h)
int64_t illm_kq_total_bytes(int fmt, int64_t n, int64_t k);
void illm_kq_quantize(int fmt, const float* src, int64_t n, int64_t k, const float* imatrix, uint8_t* dst);
void illm_kq_dequantize(int fmt, const uint8_t* src, int64_t n, int64_t k, float* dst);
void illm_kq_gemm(int fmt, const float* x, int64_t m, const uint8_t* w, int64_t n, int64_t k, float* y);
// gemm_kq.cpp: integer-dot GEMV / GEMM straight from the super-blocks (isa: 0 auto, 1 AVX2, 2 AVX-512 VNNI)
void illm_kq_gemm_int(int fmt, const float* x, int64_t m, const uint8_t* w, int64_t n, int64_t k, float* y,
                      int isa);
void illm_cpu_gemm_q4(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                      const uint16_t* mins, int64_t n, int64_t k, float* y, int isa);
int illm_cpu_i8_supported(int fmt);
int illm_cpu_lut_supported(int fmt);
void illm_cpu_gemm_i8(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                      const uint16_t* mins, int64_t n, int64_t k, float* y, int isa);
void illm_cpu_gemm_lut(int fmt, const float* x, int64_t m, const uint8_t* codes, const uint16_t* scales,
                       int64_t n, int64_t k, float* y, int isa);
}
