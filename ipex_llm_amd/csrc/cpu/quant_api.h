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
}
