// Decode GEMV time breakdown on MI355X: the production v5 kernel
// (csrc/hip/lowbit_gemv5.cuh) at the Llama-3-8B decode shapes, launched with
// the geometry ops_hip.cpp's plan5 picks, hipGraph-replayed over rotating
// weight copies (cold in the MALL), next to a pure weight-streaming kernel
// of the same bytes.  Build with -DILLM_GEMV5_ABL=<bits> to drop parts of
// the kernel (lowbit_gemv5.cuh: 1 dequant/MFMA, 2 prologue, 4 epilogue).
// Weights are random bytes: timing only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#ifdef PROBE_STAMPS
// per-workgroup timeline of the last launch (PROBE_MODE=s): wall clock at the
// kernel's hook points (lowbit_gemv5.cuh ILLM_GEMV5_STAMP: 0 entry, 1 x staged,
// 2 chunks computed, 3 epilogue issued)
__device__ unsigned long long g_stamps[65536 * 4];
#define ILLM_GEMV5_STAMP(i)                                                                              \
  do {                                                                                                   \
    if (threadIdx.x == 0) g_stamps[((size_t)(blk.z * blk.gy + blk.y) * blk.gx + blk.x) * 4 + (i)] = wall_clock64(); \
  } while (0)
#endif
#include "../../ipex_llm_amd/csrc/hip/lowbit_gemv5.cuh"

using namespace illm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static size_t shmem5(int rows, int cpk) { return gemv5_shmem(rows, cpk); }

struct Shape { const char* name; int N, K; bool glu; };

int main(int argc, char** argv) {
  const Shape shapes[] = {{"qkv", 6144, 4096, false}, {"o", 4096, 4096, false},
                          {"gate_up", 28672, 4096, true}, {"down", 4096, 14336, false},
                          {"gate_up_acc", 28672, 4096, false}};
  const int Ms[] = {1, 8};
  float *nacc, *accout, *ssbuf;
  uint16_t *x, *res, *res2, *nw, *yout;
  CK(hipMalloc(&nacc, 16 * 16384 * 4));
  CK(hipMalloc(&ssbuf, 64 * 4));
  CK(hipMemset(ssbuf, 0, 64 * 4));
  CK(hipMalloc(&accout, 16 * 32768 * 4));
  CK(hipMalloc(&x, 16 * 16384 * 2));
  CK(hipMalloc(&res, 16 * 16384 * 2));
  CK(hipMalloc(&res2, 16 * 16384 * 2));
  CK(hipMalloc(&nw, 16384 * 2));
  CK(hipMalloc(&yout, 16 * 32768 * 2));
  CK(hipMemset(nacc, 0, 16 * 16384 * 4));
  CK(hipMemset(accout, 0, 16 * 32768 * 4));
  CK(hipMemset(x, 0x3c, 16 * 16384 * 2));
  CK(hipMemset(res, 0x3c, 16 * 16384 * 2));
  CK(hipMemset(nw, 0x3f, 16384 * 2));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // sweep: (shape, M, normin, kw, nw, ks); 0 = the production plan5 value
  struct Cfg { int shape, M, normin, kw, nw, ks; };
  std::vector<Cfg> cfgs;
  const char* mode = getenv("PROBE_MODE");
  if (mode && mode[0] == 'a') {
    // ablation builds: production geometry, plain / deferred input
    for (int M : {1, 8})
      for (int sh : {0, 1, 2, 3, 4})
        for (int ni = 0; ni < 3; ni += 2) cfgs.push_back({sh, M, ni, 0, 0, 0});
  } else if (mode && mode[0] == 's') {
    // timelines (PROBE_STAMPS build): production geometry, plain and deferred input
    for (int M : {1, 8}) {
      cfgs.push_back({0, M, 0, 0, 0, 0});
      cfgs.push_back({0, M, 2, 0, 0, 0});
      cfgs.push_back({1, M, 0, 0, 0, 0});
      cfgs.push_back({2, M, 0, 0, 0, 0});
      cfgs.push_back({3, M, 0, 0, 0, 0});
    }
  } else if (mode && mode[0] == 'd') {
    // deferred vs full-row norm-in vs plain input, production geometry
    for (int M : {1, 2, 4, 8}) {
      for (int ni = 0; ni < 3; ni++) {
        cfgs.push_back({0, M, ni, 0, 0, 0});
        cfgs.push_back({2, M, ni, 0, 0, 0});
        cfgs.push_back({4, M, ni, 0, 0, 0});
      }
      cfgs.push_back({1, M, 0, 0, 0, 0});
      cfgs.push_back({3, M, 0, 0, 0, 0});
    }
  } else {
  for (int M : Ms) {
    cfgs.push_back({0, M, 0, 0, 0, 0});
    cfgs.push_back({0, M, 1, 0, 0, 0});
    for (int ks : {2, 4, 8}) for (int nwv : {4, 8}) cfgs.push_back({0, M, 0, 1, nwv, ks});
    cfgs.push_back({1, M, 0, 0, 0, 0});
    for (int ks : {2, 4, 8}) for (int nwv : {4, 8}) cfgs.push_back({1, M, 0, 1, nwv, ks});
    cfgs.push_back({2, M, 0, 0, 0, 0});
    cfgs.push_back({2, M, 1, 0, 0, 0});
    for (int kwv : {1, 2, 4}) for (int nwv : {4, 8}) cfgs.push_back({2, M, 0, kwv, nwv, 0});
    cfgs.push_back({3, M, 0, 0, 0, 0});
    for (int ks : {4, 7, 8, 14, 16}) for (int nwv : {4, 8}) cfgs.push_back({3, M, 0, 1, nwv, ks});
  }
  }
  int cur_shape = -1;
  uint8_t* wbuf = nullptr;
  size_t wb = 0;
  int copies = 0;
  for (const Cfg& c : cfgs) {
    const Shape& s = shapes[c.shape];
    if (c.shape != cur_shape) {
      if (wbuf) CK(hipFree(wbuf));
      wb = (size_t)dev_total_bytes(FMT_SYM_INT4, s.N, s.K);
      copies = std::max(2, (int)(700e6 / wb));
      CK(hipMalloc(&wbuf, wb * copies));
      CK(hipMemset(wbuf, 0x5a, wb * copies));
      cur_shape = c.shape;
    }
    const int NT = (s.N + 15) / 16, KC = (s.K + 127) / 128;
    const int M = c.M, normin = c.normin;
    if (normin && s.K != 4096) continue;
    {
      {
        GemvArgs a{};
        a.M = M; a.K = s.K; a.ldx = s.K; a.KC = KC; a.lut_fmt = FMT_SYM_INT4;
        int kw, nwv, epi;
        unsigned gx, gy;
        size_t sh;
        if (s.glu) {
          kw = 2;
          nwv = M <= 2 ? 4 : 8;
          while (kw > 1 && KC / kw < 4) kw /= 2;
          if (c.kw) kw = c.kw;
          if (c.nw) nwv = c.nw;
          const int groups = NT / 2;
          gx = (groups + nwv / kw - 1) / (nwv / kw);
          gy = 1;
          sh = shmem5(M, KC);
          a.N = s.N / 2; a.out = yout; a.ldo = s.N / 2; epi = EPI_GLU;
        } else {
          kw = 1;
          nwv = (M >= 4 || NT <= 256) ? 8 : 4;
          const int target = KC >= 64 ? 7 : 4;
          int ks = std::min(32, std::max(1, (KC + target - 1) / target));
          while (ks > 1 && NT * ks > 4096) ks /= 2;
          while (shmem5(M, (KC + ks - 1) / ks) > 65536 && ks < KC) ks *= 2;
          if (c.ks) ks = c.ks;
          if (c.nw) nwv = c.nw;
          const int cpk = (KC + ks - 1) / ks;
          ks = (KC + cpk - 1) / cpk;
          a.cpk = cpk;
          gx = (NT + nwv - 1) / nwv;
          gy = ks;
          sh = shmem5(M, cpk);
          a.N = s.N; a.out = accout; a.ldo = s.N; epi = EPI_ATOMIC;
        }
        a.nw = nwv;
        if (normin) {
          a.nacc = nacc; a.nres = res; a.nres_out = res2; a.nweight = nw; a.neps = 1e-5f;
          if (normin == 2) { a.ndefer = 1; a.nss = ssbuf; }
        } else {
          a.x = x;
        }
        auto launch = [&](int i) {
          GemvArgs b = a;
          b.w = wbuf + (size_t)(i % copies) * wb;
          launch_gemv5_dk<DK_INT4S>(true, kw, epi, dim3(gx, gy), sh, b, st);
        };
        for (int i = 0; i < copies; i++) launch(i);
        CK(hipStreamSynchronize(st));
        const int reps = 4 * copies;
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int i = 0; i < reps; i++) launch(i);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("{\"abl\":%d,\"minw\":%d,\"op\":\"%s\",\"M\":%d,\"normin\":%d,\"grid\":[%u,%u],\"nw\":%d,\"kw\":%d,"
               "\"us\":%.2f,\"TBps\":%.2f}\n", ILLM_GEMV5_ABL, ILLM_GEMV5_MINW, s.name, M, normin, gx, gy, nwv, kw, us,
               wb / us / 1e6);
        fflush(stdout);
        if (s.glu) {
          // uniform inputs (every weight byte 0x5a, every x 0x3c3c): every
          // output element must be the same finite value
          std::vector<uint16_t> yh((size_t)M * (s.N / 2));
          CK(hipMemcpy(yh.data(), yout, yh.size() * 2, hipMemcpyDeviceToHost));
          size_t bad = 0;
          for (size_t i = 0; i < yh.size(); i++) bad += yh[i] != yh[0] || (yh[i] & 0x7f80) == 0x7f80;
          printf("{\"check\":\"%s\",\"M\":%d,\"first\":\"0x%04x\",\"mismatch\":%zu,\"of\":%zu}\n", s.name, M, yh[0],
                 bad, yh.size());
        }
#ifdef PROBE_STAMPS
        {
          const int nwg = (int)(gx * gy);
          std::vector<unsigned long long> st4((size_t)nwg * 4);
          CK(hipMemcpyFromSymbol(st4.data(), HIP_SYMBOL(g_stamps), st4.size() * 8, 0, hipMemcpyDeviceToHost));
          int khz = 0;
          CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
          const double tick_us = 1e3 / (double)khz;
          unsigned long long t0 = ~0ull, tend = 0;
          for (int b = 0; b < nwg; b++) { t0 = std::min(t0, st4[b * 4]); tend = std::max(tend, st4[b * 4 + 3]); }
          std::vector<double> d[4];
          for (int b = 0; b < nwg; b++) {
            d[0].push_back((st4[b * 4] - t0) * tick_us);
            for (int j = 1; j < 4; j++) d[j].push_back(((long long)st4[b * 4 + j] - (long long)st4[b * 4 + j - 1]) * tick_us);
          }
          auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };
          printf("{\"timeline\":\"%s\",\"M\":%d,\"normin\":%d,\"wgs\":%d,\"span_us\":%.2f,"
                 "\"start_p50\":%.2f,\"start_max\":%.2f,\"stage_p50\":%.2f,\"stage_p90\":%.2f,"
                 "\"compute_p50\":%.2f,\"compute_p90\":%.2f,\"epi_p50\":%.2f,\"epi_p90\":%.2f}\n",
                 s.name, M, normin, nwg, (tend - t0) * tick_us, pct(d[0], 0.5), pct(d[0], 1.0), pct(d[1], 0.5),
                 pct(d[1], 0.9), pct(d[2], 0.5), pct(d[2], 0.9), pct(d[3], 0.5), pct(d[3], 0.9));
          fflush(stdout);
        }
#endif
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
    }
  }
  if (wbuf) CK(hipFree(wbuf));
  return 0;
}
