// Read-bandwidth probe: what a wave64 streaming 1 KiB chunks (the GEMV's
// weight access pattern) achieves on this MI355X, vs grid size / depth.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int PF>
__global__ void __launch_bounds__(256) stream_k(const uint4* __restrict__ p, size_t chunks_per_wave, float* out) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint4* base = p + wave * chunks_per_wave * 64 + lane;
  uint32_t acc = 0;
  uint4 r[PF];
#pragma unroll
  for (int u = 0; u < PF; u++) r[u] = base[u * 64];
  size_t c = 0;
  for (; c + 2 * PF <= chunks_per_wave; c += PF) {
#pragma unroll
    for (int u = 0; u < PF; u++) {
      acc ^= r[u].x + r[u].y * 3 + r[u].z * 5 + r[u].w * 7;
      r[u] = base[(c + u + PF) * 64];
    }
  }
  for (int u = 0; u < PF; u++) acc ^= r[u].x + r[u].y;
  if (acc == 0x12345678u) out[wave] = (float)acc;
}

int main() {
  const size_t bytes = 2ull << 30;
  uint4* buf;
  float* out;
  hipMalloc(&buf, bytes);
  hipMalloc(&out, 1 << 24);
  hipMemset(buf, 1, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t total_chunks = bytes / 1024;
  for (int cpw : {8, 16, 32, 64, 128}) {
    size_t waves = total_chunks / cpw;
    size_t wgs = waves / 4;
    for (int pf : {2, 4, 8}) {
      auto launch = [&]() {
        if (pf == 2) hipLaunchKernelGGL(stream_k<2>, dim3(wgs), dim3(256), 0, 0, buf, (size_t)cpw, out);
        if (pf == 4) hipLaunchKernelGGL(stream_k<4>, dim3(wgs), dim3(256), 0, 0, buf, (size_t)cpw, out);
        if (pf == 8) hipLaunchKernelGGL(stream_k<8>, dim3(wgs), dim3(256), 0, 0, buf, (size_t)cpw, out);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int i = 0; i < 10; i++) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("chunks/wave %4d  PF %d  wgs %7zu  %.2f TB/s\n", cpw, pf, wgs, bytes * 10 / (ms * 1e-3) / 1e12);
    }
  }
  // GEMV-sized working sets rotated over a 1.5 GB window (defeats the MALL)
  for (size_t ws : {8ull << 20, 14ull << 20, 33ull << 20, 64ull << 20}) {
    const int nbuf = (int)((1536ull << 20) / ws);
    for (int cpw : {4, 8, 32}) {
      size_t waves = ws / 1024 / cpw, wgs = waves / 4;
      auto launch = [&](int i) {
        const uint4* p = (const uint4*)((const char*)buf + (size_t)(i % nbuf) * ws);
        hipLaunchKernelGGL(stream_k<4>, dim3(wgs), dim3(256), 0, 0, p, (size_t)cpw, out);
      };
      for (int i = 0; i < nbuf; i++) launch(i);
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int i = 0; i < 4 * nbuf; i++) launch(i);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double us = ms * 1e3 / (4 * nbuf);
      printf("ws %5zu MB  chunks/wave %3d  wgs %6zu  %.2f us  %.2f TB/s\n", ws >> 20, cpw, wgs, us, ws / (us * 1e-6) / 1e12);
    }
  }
  return 0;
}
