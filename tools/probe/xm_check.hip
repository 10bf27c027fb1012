// Correctness check of the decode GEMV XM instantiations (round 6, run with
// ILLM_GEMV5_XM_RT=2) against the
// generic kernels on the SAME random inputs: sym_int4 codes random bytes,
// scales random f16 in [2^-7, 2^-4), x random bf16 in (-1, 1).  The XM form
// only changes how x reaches LDS, so outputs must match the generic kernel
// (launch5_epi, which bypasses launch5_xm) to f32 rounding.  Every config runs
// three times (non-determinism shows as a mismatch between repeats).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <random>
#include <vector>

// staged x (first 4096 elements of row 0) and block sums of workgroup 0, after the staging barrier
__device__ uint16_t g_xs[4096];
__device__ float g_sx[256];
#ifdef XMC_DUMP
#define ILLM_GEMV5_DUMP()                                                                   \
  do {                                                                                      \
    if (blk.x == 0 && blk.y == 0) {                                                         \
      for (int i = threadIdx.x; i < min(kw, 4096); i += NW * 64) g_xs[i] = xs[i];           \
      for (int i = threadIdx.x; i < min(4 * (c1 - c0), 256); i += NW * 64) g_sx[i] = ((float*)sxs)[i]; \
    }                                                                                       \
  } while (0)
#endif
#include "../../ipex_llm_amd/csrc/hip/lowbit_gemv5.cuh"

using namespace illm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static uint16_t f2bf(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }
static float bf2f(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }

int main() {
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> ux(-1.f, 1.f), us(1.f / 128, 1.f / 16);
  float* acc;
  uint16_t *x, *y;
  uint8_t* w;
  CK(hipMalloc(&acc, 16 * 32768 * 4));
  CK(hipMalloc(&x, 16 * 16384 * 2));
  CK(hipMalloc(&y, 16 * 32768 * 2));
  // XMC_MODE: 0 all random; 1 random x, uniform weights; 2 uniform x, random codes,
  // uniform scales; 3 uniform x and codes, random scales
  const int mode = getenv("XMC_MODE") ? atoi(getenv("XMC_MODE")) : 0;
  {
    std::vector<uint16_t> xh(16 * 16384);
    for (auto& v : xh) v = (mode == 0 || mode == 1) ? f2bf(ux(rng)) : f2bf(0.25f);
    CK(hipMemcpy(x, xh.data(), xh.size() * 2, hipMemcpyHostToDevice));
  }
  int fails = 0;
  for (int glu = 0; glu < 2; glu++)
    for (int K : {1024, 2048, 4096, 14336})
      for (int M : {1, 2, 5, 8})
        for (int ks : {1, 2, 4, 8}) {
          if (glu && (ks != 1 || K == 14336)) continue;
          const int N = glu ? 2048 : 1024, NT = (N * (glu ? 2 : 1) + 15) / 16, KC = K / 128;
          const size_t TB = (size_t)KC * 1088, wb = (size_t)NT * TB;
          CK(hipMalloc(&w, wb));
          {
            std::vector<uint8_t> wh(wb);
            for (int t = 0; t < NT; t++) {
              uint8_t* tb = wh.data() + (size_t)t * TB;
              for (size_t i = 0; i < (size_t)KC * 1024; i++) tb[i] = (mode == 0 || mode == 2) ? (uint8_t)rng() : 0x5a;
              uint16_t* sc = (uint16_t*)(tb + (size_t)KC * 1024);
              for (int i = 0; i < KC * 32; i++) {
                _Float16 h = (_Float16)((mode == 0 || mode == 3) ? us(rng) : 0.03125f);
                memcpy(&sc[i], &h, 2);
              }
            }
            CK(hipMemcpy(w, wh.data(), wb, hipMemcpyHostToDevice));
          }
          GemvArgs a{};
          a.M = M; a.K = K; a.ldx = K; a.KC = KC; a.lut_fmt = FMT_SYM_INT4; a.x = x; a.w = w; a.N = N;
          a.nib_mask = 0x000F000Fu; a.nib_magic = Raw<BF16>::k4;
          int kw, epi; unsigned gx, gy; size_t sh;
          if (glu) {
            kw = 2; a.nw = M <= 2 ? 4 : 8;
            gx = (NT / 2 + a.nw / kw - 1) / (a.nw / kw); gy = 1; sh = gemv5_shmem(M, KC);
            a.out = y; a.ldo = N; epi = EPI_GLU;
          } else {
            kw = 1; a.nw = M >= 4 ? 8 : 4;
            const int cpk = (KC + ks - 1) / ks;
            a.cpk = cpk; gx = (NT + a.nw - 1) / a.nw; gy = (KC + cpk - 1) / cpk; sh = gemv5_shmem(M, cpk);
            a.out = acc; a.ldo = N; epi = EPI_ATOMIC;
          }
          const size_t nout = (size_t)M * N;
          std::vector<float> out[4];
          for (int run = 0; run < 4; run++) {   // run 0: generic; 1..3: launch_gemv5_dk (XM where it applies)
            if (!glu) CK(hipMemset(acc, 0, nout * 4));
            if (run == 0) {
              if (kw == 2 && a.nw == 8) launch5_epi<DK_INT4S, BF16, 2, false, 8>(epi, dim3(gx, gy), sh, a, 0);
              else if (kw == 2) launch5_epi<DK_INT4S, BF16, 2, false, 4>(epi, dim3(gx, gy), sh, a, 0);
              else if (a.nw == 8) launch5_epi<DK_INT4S, BF16, 1, false, 8>(epi, dim3(gx, gy), sh, a, 0);
              else launch5_epi<DK_INT4S, BF16, 1, false, 4>(epi, dim3(gx, gy), sh, a, 0);
            } else {
              launch_gemv5_dk<DK_INT4S>(true, kw, epi, dim3(gx, gy), sh, a, 0);
            }
            CK(hipDeviceSynchronize());
            if (glu && M == 1) {
              std::vector<uint16_t> xs(4096), xh(K);
              std::vector<float> sx(256);
              CK(hipMemcpyFromSymbol(xs.data(), HIP_SYMBOL(g_xs), 8192, 0, hipMemcpyDeviceToHost));
              CK(hipMemcpyFromSymbol(sx.data(), HIP_SYMBOL(g_sx), 1024, 0, hipMemcpyDeviceToHost));
              CK(hipMemcpy(xh.data(), x, K * 2, hipMemcpyDeviceToHost));
              int badx = 0, bads = 0;
              for (int i = 0; i < std::min(K, 4096); i++) badx += xs[i] != xh[i];
              for (int c = 0; c < std::min(KC, 64); c++)
                for (int b = 0; b < 2; b++) {
                  float ref = 0;
                  for (int i = 0; i < 64; i++) ref += bf2f(xh[c * 128 + b * 64 + i]);
                  bads += std::fabs(sx[c * 4 + 2 + b] - ref) > 1e-3f * (1 + std::fabs(ref));
                }
              printf("   run %d: staged x mismatches %d, block sums off %d\n", run, badx, bads);
            }
            out[run].resize(nout);
            if (glu) {
              std::vector<uint16_t> h(nout);
              CK(hipMemcpy(h.data(), y, nout * 2, hipMemcpyDeviceToHost));
              for (size_t i = 0; i < nout; i++) out[run][i] = bf2f(h[i]);
            } else {
              CK(hipMemcpy(out[run].data(), acc, nout * 4, hipMemcpyDeviceToHost));
            }
          }
          double nr = 0, worst = 0;
          size_t nonfin = 0;
          for (size_t i = 0; i < nout; i++) nr += (double)out[0][i] * out[0][i];
          nr = std::sqrt(nr / nout) + 1e-30;
          for (int run = 1; run < 4; run++)
            for (size_t i = 0; i < nout; i++) {
              if (!std::isfinite(out[run][i])) nonfin++;
              else worst = std::max(worst, std::fabs((double)out[run][i] - out[0][i]) / nr);
            }
          const bool bad = nonfin || worst > (glu ? 2e-2 : 1e-4);
          if (bad) {   // where: rows, 16-column tiles (first 16), and whether the repeats agree
            std::vector<int> rows(M, 0), tiles;
            for (size_t i = 0; i < nout; i++) {
              const float v = out[1][i];
              if (!std::isfinite(v) || std::fabs((double)v - out[0][i]) / nr > (glu ? 2e-2 : 1e-4)) {
                rows[i / N]++;
                const int tl = (int)(i % N) / 16;
                if (tiles.size() < 16 && (tiles.empty() || tiles.back() != tl)) tiles.push_back(tl);
              }
            }
            size_t rep = 0;
            for (size_t i = 0; i < nout; i++) rep += memcmp(&out[1][i], &out[2][i], 4) != 0;
            printf("   bad per row:");
            for (int m = 0; m < M; m++) printf(" %d", rows[m]);
            printf("  tiles:");
            for (int t : tiles) printf(" %d", t);
            printf("  run1!=run2: %zu\n", rep);
          }
          fails += bad;
          printf("%s K=%d M=%d ks=%d rms=%.3g worst=%.2e nonfinite=%zu%s\n", glu ? "glu" : "accum", K, M, ks, nr, worst,
                 nonfin, bad ? "  FAIL" : "");
          fflush(stdout);
          CK(hipFree(w));
        }
  printf("fails=%d\n", fails);
  return 0;
}
