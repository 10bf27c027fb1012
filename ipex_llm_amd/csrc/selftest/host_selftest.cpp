// Host self-test driver for the C++ low-bit library, built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_sanitizers.py
// (sanitizers on host code; GPU kernels are checked by their own
// numerics tests).  Randomised shapes exercise every format's quantizer,
// dequantizer, device-layout repack round trip and both CPU GEMM paths.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "../common/formats.h"
#include "../cpu/quant_api.h"

using namespace illm;

static int fails = 0;
#define CHECK(c, ...)                           \
  do {                                          \
    if (!(c)) {                                 \
      fprintf(stderr, "FAIL: " __VA_ARGS__);    \
      fprintf(stderr, "\n");                    \
      fails++;                                  \
    }                                           \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 24;
  std::mt19937 rng(1234);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int fmts[] = {FMT_SYM_INT4, FMT_ASYM_INT4, FMT_NF4, FMT_FP4, FMT_SYM_INT8, FMT_FP8E4, FMT_FP8E5,
                      FMT_SYM_INT5, FMT_ASYM_INT5, FMT_NF3, FMT_FP6};
  for (int it = 0; it < iters; it++) {
    const int fmt = fmts[it % 11];
    const int64_t n = 16 * (1 + rng() % 5) + (it % 3 == 0 ? 7 : 0);   // ragged last tile
    const int64_t k = 64 * (1 + rng() % 6);
    const int64_t m = 1 + rng() % 9;
    const int bits = illm_fmt_bits(fmt);
    std::vector<float> w(n * k), x(m * k), deq(n * k), y(m * n), yref(m * n);
    for (auto& v : w) v = nd(rng) * 0.05f;
    for (auto& v : x) v = nd(rng);
    const int64_t nb = k / 64;
    std::vector<uint8_t> codes(n * k * bits / 8);
    std::vector<uint16_t> scales(n * nb), mins(n * nb);
    const bool hm = fmt == FMT_ASYM_INT4 || fmt == FMT_ASYM_INT5;
    illm_quantize(fmt, w.data(), n, k, nullptr, it & 1, codes.data(), scales.data(), hm ? mins.data() : nullptr);
    illm_dequantize(fmt, codes.data(), scales.data(), hm ? mins.data() : nullptr, n, k, deq.data());
    double err = 0, ref = 0;
    for (int64_t i = 0; i < n * k; i++) {
      err += (deq[i] - w[i]) * (double)(deq[i] - w[i]);
      ref += (double)w[i] * w[i];
    }
    CHECK(sqrt(err / ref) < (bits >= 8 ? 0.08 : 0.3), "fmt %d quant error %.3f", fmt, sqrt(err / ref));
    // device-layout repack round trip must be exact
    const int64_t devbytes = dev_total_bytes(fmt, n, k);
    std::vector<uint8_t> dev(devbytes);
    illm_repack_to_device(fmt, codes.data(), scales.data(), hm ? mins.data() : nullptr, n, k, dev.data());
    std::vector<uint8_t> codes2(codes.size());
    std::vector<uint16_t> scales2(scales.size()), mins2(mins.size());
    illm_repack_from_device(fmt, dev.data(), n, k, codes2.data(), scales2.data(), hm ? mins2.data() : nullptr);
    CHECK(codes2 == codes && scales2 == scales && (!hm || mins2 == mins), "fmt %d repack round trip", fmt);
    // CPU GEMMs vs the dequantized weight
    for (int64_t i = 0; i < m; i++)
      for (int64_t r = 0; r < n; r++) {
        double s = 0;
        for (int64_t j = 0; j < k; j++) s += (double)x[i * k + j] * deq[r * k + j];
        yref[i * n + r] = (float)s;
      }
    illm_cpu_gemm(fmt, x.data(), m, codes.data(), scales.data(), hm ? mins.data() : nullptr, n, k, y.data());
    double e1 = 0, r1 = 0;
    for (int64_t i = 0; i < m * n; i++) {
      e1 += (y[i] - yref[i]) * (double)(y[i] - yref[i]);
      r1 += (double)yref[i] * yref[i];
    }
    CHECK(sqrt(e1 / r1) < 1e-4, "fmt %d cpu gemm rel %.2e", fmt, sqrt(e1 / r1));
    if (illm_cpu_q4_supported(fmt)) {
      for (int isa = 1; isa <= 2; isa++) {
        if (isa == 2 && !__builtin_cpu_supports("avx512vnni")) continue;
        illm_cpu_gemm_q4(fmt, x.data(), m, codes.data(), scales.data(), hm ? mins.data() : nullptr, n, k, y.data(),
                         isa);
        double e2 = 0;
        for (int64_t i = 0; i < m * n; i++) e2 += (y[i] - yref[i]) * (double)(y[i] - yref[i]);
        CHECK(sqrt(e2 / r1) < 2e-2, "fmt %d q4 gemm isa %d rel %.2e", fmt, isa, sqrt(e2 / r1));
      }
    }
  }
  printf("selftest: %d iterations, %d failures\n", iters, fails);
  return fails ? 1 : 0;
}
