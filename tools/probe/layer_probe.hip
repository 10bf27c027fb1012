// Decode-layer streaming floor on MI355X: what a chain of pure weight-
// streaming kernels with the byte counts of one Llama-3-8B int4 layer costs
// (qkv 13.4 MB, attention ~4 MB over 128 workgroups, o 8.9 MB, gate/up
// 62.4 MB, down 31.2 MB), over 32 distinct layers (no MALL reuse across
// replays), and how much of it a MALL prefetch issued by idle workgroups of
// the attention launch buys back.  Prints us per layer per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// each wave streams `cpw` 1 KiB chunks (16 B per lane), PF in flight
template <int PF, bool NT>
__global__ void __launch_bounds__(256) stream_k(const u32x4* __restrict__ p, int cpw, size_t nchunks, uint32_t* sink) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const size_t c0 = wave * cpw;
  if (c0 >= nchunks) return;
  const int n = (int)((c0 + cpw <= nchunks) ? cpw : nchunks - c0);
  const u32x4* base = p + c0 * 64 + lane;
  uint32_t acc = 0;
  u32x4 r[PF];
#pragma unroll
  for (int u = 0; u < PF; u++) r[u] = ld<NT>(base + (size_t)min(u, n - 1) * 64);
  for (int c = 0; c < n; c += PF) {
#pragma unroll
    for (int u = 0; u < PF; u++) {
      if (c + u < n) acc ^= r[u].x + r[u].y * 3 + r[u].z * 5 + r[u].w * 7;
      r[u] = ld<NT>(base + (size_t)min(c + u + PF, n - 1) * 64);
    }
  }
  if (acc == 0x12345678u) sink[wave & 1023] = acc;
}

// "attention": 128 workgroups of one wave read 32 KB each; workgroups past
// 128 (when pf_bytes > 0) read the NEXT kernels' weights with default policy
// so they land in the MALL
__global__ void __launch_bounds__(64) attn_like(const u32x4* __restrict__ kv, const u32x4* __restrict__ pf,
                                                size_t pf_chunks, int pf_wgs, uint32_t* sink) {
  const int lane = threadIdx.x;
  uint32_t acc = 0;
  if (blockIdx.x < 128) {
    const u32x4* b = kv + (size_t)blockIdx.x * 32 * 64 + lane;
    // dependent-ish: 32 chunks, 4 in flight, plus some ALU per chunk
    for (int c = 0; c < 32; c += 4) {
      u32x4 r0 = b[(c + 0) * 64], r1 = b[(c + 1) * 64], r2 = b[(c + 2) * 64], r3 = b[(c + 3) * 64];
      acc ^= r0.x + r1.y + r2.z + r3.w;
      for (int i = 0; i < 64; i++) acc = acc * 1664525u + 1013904223u;
    }
  } else {
    const int w = blockIdx.x - 128;
    const size_t per = (pf_chunks + pf_wgs - 1) / pf_wgs;
    const size_t s = (size_t)w * per, e = min(pf_chunks, s + per);
    for (size_t c = s; c < e; c += 8) {
      u32x4 r[8];
#pragma unroll
      for (int u = 0; u < 8; u++) r[u] = pf[(min(c + u, e - 1)) * 64 + lane];
#pragma unroll
      for (int u = 0; u < 8; u++) acc ^= r[u].x;
    }
  }
  if (acc == 0x12345678u) sink[blockIdx.x & 1023] = acc;
}


// ---------------------------------------------------------------- fused
// producer WGs signal a counter after their loads; consumer WGs issue their
// own loads FIRST (prefetch), then wait for the counter, then "consume".
#ifndef SLEEP
#define SLEEP 8
#endif
__device__ __forceinline__ void signal_ctr(int* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // arrivals sharded over 64 counters (one 128-B line each): same-address
  // atomics serialise at ~12 ns each
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(ctr + 32 * (blockIdx.x & 63), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wait_ctr(const int* ctr, int target, int* err) {
  if (threadIdx.x < 64) {
    int spins = 0;
    while (true) {
      int v = __hip_atomic_load(ctr + 32 * threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (v >= target) break;
      __builtin_amdgcn_s_sleep(SLEEP);
      if (++spins > (1 << 22)) { if (threadIdx.x == 0) atomicExch(err, 1); break; }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// one wave streams `cpw` chunks of p starting at chunk c0 (all loads in flight)
template <int CPW>
__device__ __forceinline__ uint32_t stream_item(const u32x4* p, size_t c0, size_t nchunks) {
  const int lane = threadIdx.x & 63;
  u32x4 r[CPW];
#pragma unroll
  for (int u = 0; u < CPW; u++) r[u] = __builtin_nontemporal_load(p + min(c0 + u, nchunks - 1) * 64 + lane);
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < CPW; u++) acc ^= r[u].x + r[u].y * 3 + r[u].z * 5 + r[u].w * 7;
  return acc;
}

// K1: [nq qkv WGs][na attention WGs][no o_proj WGs]
template <int CPW>
__global__ void __launch_bounds__(256) fused_attn_block(const u32x4* qkv, size_t qc, const u32x4* kv, const u32x4* o,
                                                        size_t oc, int nq, int na, int* ctr, int* ctr_other,
                                                        uint32_t* sink, int* err) {
  const int b = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (b == 0) for (int i = threadIdx.x; i < 4096; i += 256) ctr_other[i] = 0;
  uint32_t acc = 0;
  if (b < nq) {
    acc = stream_item<CPW>(qkv, ((size_t)b * 4 + wave) * CPW, qc);
    signal_ctr(&ctr[0]);
  } else if (b < nq + na) {
    // attention-like: prefetch this WG's 4 splits (32 KB / wave), wait for qkv
    const u32x4* bp = kv + ((size_t)(b - nq) * 4 + wave) * 32 * 64 + lane;
    u32x4 r[8];
    for (int c = 0; c < 32; c += 8) {
#pragma unroll
      for (int u = 0; u < 8; u++) r[u] = bp[(c + u) * 64];
#pragma unroll
      for (int u = 0; u < 8; u++) acc ^= r[u].x;
    }
    wait_ctr(&ctr[0], nq, err);
    for (int i = 0; i < 256; i++) acc = acc * 1664525u + 1013904223u;   // softmax/PV stand-in
    signal_ctr(&ctr[2048]);
  } else {
    const size_t c0 = ((size_t)(b - nq - na) * 4 + wave) * CPW;
    u32x4 r[CPW];
#pragma unroll
    for (int u = 0; u < CPW; u++) r[u] = __builtin_nontemporal_load(o + min(c0 + u, oc - 1) * 64 + lane);
    wait_ctr(&ctr[2048], na, err);
#pragma unroll
    for (int u = 0; u < CPW; u++) acc ^= r[u].x + r[u].y * 3 + r[u].z * 5 + r[u].w * 7;
  }
  if (acc == 0x12345678u) sink[b & 1023] = acc;
}

// K2: [ng gate/up WGs][nd down WGs]
template <int CPW>
__global__ void __launch_bounds__(256) fused_mlp_block(const u32x4* gu, size_t gc, const u32x4* dn, size_t dc, int ng,
                                                       int* ctr, int* ctr_other, uint32_t* sink, int* err) {
  const int b = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (b == 0) for (int i = threadIdx.x; i < 4096; i += 256) ctr_other[i] = 0;
  uint32_t acc = 0;
  if (b < ng) {
    acc = stream_item<CPW>(gu, ((size_t)b * 4 + wave) * CPW, gc);
    signal_ctr(&ctr[0]);
  } else {
    const size_t c0 = ((size_t)(b - ng) * 4 + wave) * CPW;
    u32x4 r[CPW];
#pragma unroll
    for (int u = 0; u < CPW; u++) r[u] = __builtin_nontemporal_load(dn + min(c0 + u, dc - 1) * 64 + lane);
    wait_ctr(&ctr[0], ng, err);
#pragma unroll
    for (int u = 0; u < CPW; u++) acc ^= r[u].x + r[u].y * 3 + r[u].z * 5 + r[u].w * 7;
  }
  if (acc == 0x12345678u) sink[b & 1023] = acc;
}

int main(int argc, char** argv) {
  const size_t MB = 1000000;
  const size_t sz[4] = {13421772, 8912896, 62390272, 31195136};  // qkv, o, gate_up, down (int4 + scales)
  size_t layer = 0;
  for (size_t s : sz) layer += (s + 1023) / 1024 * 1024;
  const int L = 32;
  const size_t kvb = 128 * 32 * 1024;
  char* buf;
  uint32_t* sink;
  if (hipMalloc(&buf, layer * L + kvb * L) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&sink, 4096 * 4);
  hipMemset(buf, 1, layer * L + kvb * L);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto chunks = [](size_t s) { return (s + 1023) / 1024; };

  // variant: cpw chunks per wave, nt loads, prefetch mode (0 none, 1 o only, 2 o + gate/up)
  auto run = [&](int cpw, bool nt, int pfmode, int reps, bool attn) -> double {
    auto one_layer = [&](int l) {
      char* lb = buf + (size_t)l * layer;
      size_t off[4];
      size_t o = 0;
      for (int i = 0; i < 4; i++) { off[i] = o; o += chunks(sz[i]) * 1024; }
      auto launch = [&](int i) {
        const size_t nc = chunks(sz[i]);
        const size_t waves = (nc + cpw - 1) / cpw;
        const unsigned wgs = (unsigned)((waves + 3) / 4);
        const u32x4* p = (const u32x4*)(lb + off[i]);
        if (nt) hipLaunchKernelGGL((stream_k<4, true>), dim3(wgs), dim3(256), 0, 0, p, cpw, nc, sink);
        else hipLaunchKernelGGL((stream_k<4, false>), dim3(wgs), dim3(256), 0, 0, p, cpw, nc, sink);
      };
      launch(0);
      if (attn) {
        const u32x4* kv = (const u32x4*)(buf + layer * L + (size_t)l * kvb);
        size_t pfc = pfmode == 0 ? 0 : (pfmode == 1 ? chunks(sz[1]) : chunks(sz[1]) + chunks(sz[2]));
        int pfw = pfmode == 0 ? 0 : 384;
        hipLaunchKernelGGL(attn_like, dim3(128 + pfw), dim3(64), 0, 0, kv, (const u32x4*)(lb + off[1]), pfc, pfw, sink);
      }
      launch(1);
      launch(2);
      launch(3);
    };
    for (int l = 0; l < L; l++) one_layer(l);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < reps; r++)
      for (int l = 0; l < L; l++) one_layer(l);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3 / (reps * L);
  };

  // single-kernel floors per size (cold: rotate over the 32 layers)
  for (int i = 0; i < 4; i++) {
    for (int cpw : {2, 4, 8, 16}) {
      for (int nt = 0; nt < 2; nt++) {
        const size_t nc = chunks(sz[i]);
        const unsigned wgs = (unsigned)(((nc + cpw - 1) / cpw + 3) / 4);
        auto launch = [&](int l) {
          size_t o = 0;
          for (int j = 0; j < i; j++) o += chunks(sz[j]) * 1024;
          const u32x4* p = (const u32x4*)(buf + (size_t)l * layer + o);
          if (nt) hipLaunchKernelGGL((stream_k<4, true>), dim3(wgs), dim3(256), 0, 0, p, cpw, nc, sink);
          else hipLaunchKernelGGL((stream_k<4, false>), dim3(wgs), dim3(256), 0, 0, p, cpw, nc, sink);
        };
        for (int l = 0; l < L; l++) launch(l);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 8; r++)
          for (int l = 0; l < L; l++) launch(l);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / (8 * L);
        // warm: same buffer back to back (MALL resident)
        for (int r = 0; r < 4; r++) launch(0);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 64; r++) launch(0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        const double usw = ms * 1e3 / 64;
        printf("{\"kind\":\"single\",\"MB\":%.1f,\"cpw\":%d,\"nt\":%d,\"wgs\":%u,\"cold_us\":%.2f,\"cold_TBps\":%.2f,"
               "\"warm_us\":%.2f,\"warm_TBps\":%.2f}\n",
               sz[i] / 1e6, cpw, nt, wgs, us, sz[i] / us / 1e6, usw, sz[i] / usw / 1e6);
      }
    }
  }
  // empty-kernel boundary
  {
    auto launch = [&]() { hipLaunchKernelGGL((stream_k<4, true>), dim3(256), dim3(256), 0, 0, (const u32x4*)buf, 1, 0, sink); };
    for (int r = 0; r < 16; r++) launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 1000; r++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("{\"kind\":\"empty\",\"us\":%.2f}\n", ms);
  }
  // whole layer chains
  for (int cpw : {4, 8}) {
    for (int nt = 0; nt < 2; nt++) {
      const double base = run(cpw, nt, 0, 4, false);
      const double att = run(cpw, nt, 0, 4, true);
      const double pf1 = run(cpw, nt, 1, 4, true);
      const double pf2 = run(cpw, nt, 2, 4, true);
      printf("{\"kind\":\"layer\",\"cpw\":%d,\"nt\":%d,\"gemv_only_us\":%.2f,\"with_attn_us\":%.2f,"
             "\"attn_pf_o_us\":%.2f,\"attn_pf_o_gu_us\":%.2f,\"bytes_MB\":%.1f}\n",
             cpw, nt, base, att, pf1, pf2, layer / 1e6);
    }
  }
  // fused: 2 launches per layer (producer/consumer roles, consumer prefetch)
  {
    int *ctr, *err;
    hipMalloc(&ctr, 8192 * sizeof(int));
    hipMalloc(&err, sizeof(int));
    hipMemset(ctr, 0, 8192 * sizeof(int));
    hipMemset(err, 0, sizeof(int));
    constexpr int CPW = 8;
    auto fused_layer = [&](int l) {
      char* lb = buf + (size_t)l * layer;
      size_t off[4];
      size_t o = 0;
      for (int i = 0; i < 4; i++) { off[i] = o; o += chunks(sz[i]) * 1024; }
      const size_t qc = chunks(sz[0]), oc = chunks(sz[1]), gc = chunks(sz[2]), dc = chunks(sz[3]);
      const int nq = (int)((qc + 4 * CPW - 1) / (4 * CPW)), na = 32, no = (int)((oc + 4 * CPW - 1) / (4 * CPW));
      const int ng = (int)((gc + 4 * CPW - 1) / (4 * CPW)), nd = (int)((dc + 4 * CPW - 1) / (4 * CPW));
      const u32x4* kv = (const u32x4*)(buf + layer * L + (size_t)l * kvb);
      hipLaunchKernelGGL((fused_attn_block<CPW>), dim3(nq + na + no), dim3(256), 0, 0, (const u32x4*)(lb + off[0]), qc,
                         kv, (const u32x4*)(lb + off[1]), oc, nq, na, ctr, ctr + 4096, sink, err);
      hipLaunchKernelGGL((fused_mlp_block<CPW>), dim3(ng + nd), dim3(256), 0, 0, (const u32x4*)(lb + off[2]), gc,
                         (const u32x4*)(lb + off[3]), dc, ng, ctr + 4096, ctr, sink, err);
    };
    for (int l = 0; l < L; l++) fused_layer(l);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 4; r++)
      for (int l = 0; l < L; l++) fused_layer(l);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    int herr = 0;
    hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost);
    printf("{\"kind\":\"fused_layer\",\"us\":%.2f,\"err\":%d}\n", ms * 1e3 / (4 * L), herr);
    // same in a hipGraph (launch overhead of the real decode step)
    hipStream_t st;
    hipStreamCreate(&st);
    hipGraph_t gr;
    hipGraphExec_t ge;
    auto cap = [&](bool fused) {
      hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
      for (int l = 0; l < L; l++) {
        char* lb = buf + (size_t)l * layer;
        size_t off[4];
        size_t o = 0;
        for (int i = 0; i < 4; i++) { off[i] = o; o += chunks(sz[i]) * 1024; }
        const size_t qc = chunks(sz[0]), oc = chunks(sz[1]), gc = chunks(sz[2]), dc = chunks(sz[3]);
        if (fused) {
          const int nq = (int)((qc + 4 * CPW - 1) / (4 * CPW)), na = 32, no = (int)((oc + 4 * CPW - 1) / (4 * CPW));
          const int ng = (int)((gc + 4 * CPW - 1) / (4 * CPW)), nd = (int)((dc + 4 * CPW - 1) / (4 * CPW));
          const u32x4* kv = (const u32x4*)(buf + layer * L + (size_t)l * kvb);
          hipLaunchKernelGGL((fused_attn_block<CPW>), dim3(nq + na + no), dim3(256), 0, st, (const u32x4*)(lb + off[0]),
                             qc, kv, (const u32x4*)(lb + off[1]), oc, nq, na, ctr, ctr + 4096, sink, err);
          hipLaunchKernelGGL((fused_mlp_block<CPW>), dim3(ng + nd), dim3(256), 0, st, (const u32x4*)(lb + off[2]), gc,
                             (const u32x4*)(lb + off[3]), dc, ng, ctr + 4096, ctr, sink, err);
        } else {
          for (int i = 0; i < 4; i++) {
            const size_t nc = chunks(sz[i]);
            const unsigned wgs = (unsigned)(((nc + 7) / 8 + 3) / 4);
            hipLaunchKernelGGL((stream_k<4, true>), dim3(wgs), dim3(256), 0, st, (const u32x4*)(lb + off[i]), 8, nc, sink);
            if (i == 0) {
              const u32x4* kv = (const u32x4*)(buf + layer * L + (size_t)l * kvb);
              hipLaunchKernelGGL(attn_like, dim3(128), dim3(64), 0, st, kv, (const u32x4*)(lb + off[1]), 0, 0, sink);
            }
          }
        }
      }
      hipStreamEndCapture(st, &gr);
      hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
      hipGraphLaunch(ge, st);
      hipStreamSynchronize(st);
      hipEventRecord(a, st);
      for (int r = 0; r < 4; r++) hipGraphLaunch(ge, st);
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      float ms2;
      hipEventElapsedTime(&ms2, a, b);
      hipGraphExecDestroy(ge);
      hipGraphDestroy(gr);
      return ms2 * 1e3 / (4 * L);
    };
    const double g5 = cap(false), g2 = cap(true);
    hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost);
    printf("{\"kind\":\"graph_layer\",\"launches5_us\":%.2f,\"fused2_us\":%.2f,\"err\":%d}\n", g5, g2, herr);
  }
  return 0;
}
