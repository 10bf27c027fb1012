// Flash attention for training: forward with the row log-sum-exp, and the
// backward as two kernels (dK / dV per key block, dQ per query block), causal
// or full, GQA.  Replaces the AOTriton SDPA kernels (attn_fwd,
// bwd_kernel_dk_dv, bwd_kernel_dq) of the HF forward in the QLoRA step
// (reference recipe: SRC/transformers/qlora.py + the HF Llama attention;
// SURVEY §3.5).
//
// MI355X design (gfx950, wave64, v_mfma_f32_16x16x32 bf16/f16; the prefill
// kernel attn_prefill.hip is the forward's template):
//   * forward / dQ: workgroup = 4 waves = 64 query rows of one head; K / V
//     tiles of 64 keys staged in LDS as XOR-swizzled [key][D] rows, next tile
//     in flight; S^T = K Q^T puts the 16 scores of one query row on a lane,
//     so the softmax statistics are register reductions; P V and dS K take
//     their A operand (V^T / K^T) from ds_read_b64_tr_b16 transposed reads of
//     the row-major tile in the key order of the C layout, and their B operand
//     is the lane's own P^T / dS^T converted to 16-bit (no lane movement);
//   * dK / dV: workgroup = 4 waves = 64 keys of one kv head (16 per wave, K and
//     V fragments in registers); it sweeps the group's query heads x 64-row
//     query blocks with Q / dO tiles in LDS: S = Q K^T and dP = dO V^T put the
//     key on the lane, so P^T / dS^T ARE the A operands of dV += P^T dO and
//     dK += dS^T Q (B operands = transposed reads of the dO / Q tiles); dK and
//     dV stay in registers for the whole sweep -- no cross-workgroup sums, no
//     atomics, deterministic;
//   * P = exp2(S * scale * log2 e - LSE2) from the forward's log2-domain
//     log-sum-exp (no max / sum pass in backward); delta = rowsum(dO * O)
//     precomputed once per row.
#include <cstdlib>

#include "illm_device.h"
#include "kernels_train.h"

namespace illm {

namespace {

constexpr int FA_KT = 64;   // keys per tile
constexpr int FA_QB = 64;   // query rows per workgroup (forward / dQ)

// ---- LDS-DMA tile staging ------------------------------------------------------
// A [64 rows][D] 16-bit tile of a row-strided tensor goes straight to LDS
// (buffer_load_dwordx4 ... lds: 1 KB per wave instruction, lane-linear
// destination), swizzled on the SOURCE side into the pf_off layout: the lane
// writing physical chunk p of row r fetches logical chunk p ^ (r & MSK).  No
// register staging (the register form spilled to scratch and waited on its
// own loads), the next tile in flight across the compute of the current one.
// Issued from inline asm so hipcc does not drain vmcnt before the LDS reads.
typedef int32_t ta_rsrc __attribute__((ext_vector_type(4)));

__device__ __forceinline__ ta_rsrc ta_make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = (uint64_t)(uintptr_t)base;
  return ta_rsrc{(int32_t)(uint32_t)p, (int32_t)((uint32_t)(p >> 32) & 0xffffu), (int32_t)bytes, 0x00020000};
}

__device__ __forceinline__ uint32_t ta_lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p);
}

// rows row0 .. row0 + 63 (clamped to nrows - 1) of a tensor with row stride
// `rstride` elements -> LDS tile at byte address `lds` (wave-uniform)
template <int D>
__device__ __forceinline__ void ta_stage(const ta_rsrc& rs, uint32_t lds, int row0, int64_t rstride, int nrows,
                                         int wave, int lane) {
  constexpr int CH = D / 8, MSK = CH >= 16 ? 15 : CH - 1;
  constexpr int RPI = 64 / CH;                    // rows per wave instruction
  constexpr int NI = 64 / RPI / 4;                // instructions per wave (4 waves)
#pragma unroll
  for (int i = 0; i < NI; i++) {
    const int idx = wave * NI + i;
    const int r = idx * RPI + lane / CH, pch = lane % CH;
    const int srow = min(row0 + r, nrows - 1);
    const uint32_t voff = (uint32_t)((int64_t)srow * rstride * 2) + (uint32_t)((pch ^ (r & MSK)) * 16);
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds + (uint32_t)(idx * RPI * D * 2));   // wave-uniform
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(m0), "v"(voff), "s"(rs), "s"(0) : "memory", "m0");
  }
}

__device__ __forceinline__ void ta_wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- forward (with_dq = false) and dQ (with_dq = true) --------------------
template <typename T, int D, bool BWD>
__global__ void __launch_bounds__(256) fa_q_kernel(const TrainAttnArgs a) {
  constexpr int KSTEP = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) uint16_t ks[2][FA_KT * D];
  __shared__ __attribute__((aligned(16))) uint16_t vs[2][FA_KT * D];
  const int nqb = gridDim.x;
  const int qb = a.causal ? nqb - 1 - blockIdx.x : blockIdx.x;     // causal: heaviest blocks first
  const int h = blockIdx.y, b = blockIdx.z;
  const int kvh = h / (a.Hq / a.Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // the forward also takes ragged T (encoders, inference): rows >= T load
  // row T - 1 and store nothing, keys >= T are masked (backward: T % 64 == 0)
  const int qrow = qb * FA_QB + wave * 16 + r16;
  const int qld = min(qrow, a.T - 1);
  const int kend = a.causal ? min((qb + 1) * FA_QB, a.T) : a.T;
  const int ntile = (kend + FA_KT - 1) / FA_KT;

  // Q (and dO) fragments: B operands of S^T = K Q^T (dP^T = V dO^T)
  uint4 qf[KSTEP], df[BWD ? KSTEP : 1];
  {
    const uint16_t* qp = a.q + (size_t)b * a.qsb + (size_t)h * a.qsh + (size_t)qld * a.qst;
#pragma unroll
    for (int s = 0; s < KSTEP; s++) qf[s] = *(const uint4*)(qp + 32 * s + 8 * g);
    if constexpr (BWD) {
      const uint16_t* dp = a.dout + (size_t)b * a.dsb + (size_t)h * a.dsh + (size_t)qrow * a.dst;
#pragma unroll
      for (int s = 0; s < KSTEP; s++) df[s] = *(const uint4*)(dp + 32 * s + 8 * g);
    }
  }
  float lse2 = 0.f, delta = 0.f;
  if constexpr (BWD) {
    const size_t ri = ((size_t)b * a.Hq + h) * a.T + qrow;
    lse2 = a.lse[ri];
    delta = a.delta[ri];
  }

  const uint16_t* kbase = a.k + (size_t)b * a.ksb + (size_t)kvh * a.ksh;
  const uint16_t* vbase = a.v + (size_t)b * a.vsb + (size_t)kvh * a.vsh;
  const ta_rsrc rk = ta_make_rsrc(kbase, (uint32_t)(((int64_t)(a.T - 1) * a.kst + D) * 2));
  const ta_rsrc rv = ta_make_rsrc(vbase, (uint32_t)(((int64_t)(a.T - 1) * a.vst + D) * 2));
  const uint32_t ks_l = ta_lds_addr(ks), vs_l = ta_lds_addr(vs);
  constexpr uint32_t TILE_B = FA_KT * D * 2;
  auto stage = [&](int t, int buf) {
    ta_stage<D>(rk, ks_l + buf * TILE_B, t * FA_KT, a.kst, a.T, wave, lane);
    ta_stage<D>(rv, vs_l + buf * TILE_B, t * FA_KT, a.vst, a.T, wave, lane);
  };

  f32x4 o[DT];                                 // forward: O^T; backward: dQ^T
#pragma unroll
  for (int d = 0; d < DT; d++) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow = -INFINITY, lpart = 0.f;
  constexpr float kLog2e = 1.4426950408889634f;
  const float sc2 = a.scale * kLog2e;

  stage(0, 0);
  // the Q / dO fragments (and LSE / delta) are consumed here, so hipcc's own
  // vmcnt waits for them sit before the loop, not at its head where they
  // would also drain the next tile's DMA every iteration
#pragma unroll
  for (int s2 = 0; s2 < KSTEP; s2++) {
    asm volatile("" :: "v"(qf[s2].x), "v"(qf[s2].y), "v"(qf[s2].z), "v"(qf[s2].w));
    if constexpr (BWD) asm volatile("" :: "v"(df[s2].x), "v"(df[s2].y), "v"(df[s2].z), "v"(df[s2].w));
  }
  if constexpr (BWD) asm volatile("" :: "v"(lse2), "v"(delta));
  ta_wait_vm0();
  __syncthreads();
  for (int t = 0; t < ntile; t++) {
    const int buf = t & 1;
    if (t + 1 < ntile) stage(t + 1, buf ^ 1);   // buffer last read in iteration t - 1
    const int kt0 = t * FA_KT;
    const uint16_t* kb_ = ks[buf];
    const uint16_t* vb_ = vs[buf];
    const bool full = (!a.causal || kt0 + FA_KT - 1 <= qb * FA_QB) && kt0 + FA_KT <= a.T;

    // ---- S^T = K Q^T (and dP^T = V dO^T): lane holds keys 16 kb + 4 g + i of query qrow
    f32x4 st[4], dp[BWD ? 4 : 1];
#pragma unroll
    for (int kb = 0; kb < 4; kb++) {
      st[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (BWD) dp[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSTEP; s++) {
        const uint4 kf = *(const uint4*)(kb_ + pf_off<D>(16 * kb + r16, 4 * s + g));
        st[kb] = mfma16<T>(kf, qf[s], st[kb]);
        if constexpr (BWD) {
          const uint4 vf = *(const uint4*)(vb_ + pf_off<D>(16 * kb + r16, 4 * s + g));
          dp[kb] = mfma16<T>(vf, df[s], dp[kb]);
        }
      }
    }
    uint32_t pk[4][2];                         // forward: P^T; backward: dS^T (16-bit pairs)
    if constexpr (!BWD) {
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float v = st[kb][i] * sc2;
          const int key = kt0 + 16 * kb + 4 * g + i;
          if (!full && ((a.causal && key > qrow) || key >= a.T)) v = -INFINITY;
          st[kb][i] = v;
        }
      float tmax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) tmax = fmaxf(tmax, st[kb][i]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(mrow, tmax);
      const float alpha = mnew == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(mrow - mnew);
      const float msafe = mnew == -INFINITY ? 0.f : mnew;
      mrow = mnew;
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
        lpart *= alpha;
#pragma unroll
        for (int d = 0; d < DT; d++) { o[d][0] *= alpha; o[d][1] *= alpha; o[d][2] *= alpha; o[d][3] *= alpha; }
      }
#pragma unroll
      for (int kb = 0; kb < 4; kb++) {
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          p[i] = __builtin_amdgcn_exp2f(st[kb][i] - msafe);
          lpart += p[i];
        }
        pk[kb][0] = pack2<T>(p[0], p[1]);
        pk[kb][1] = pack2<T>(p[2], p[3]);
      }
    } else {
      // P^T = exp2(S^T * scale * log2 e - LSE2); dS^T = P^T (dP^T - delta)
#pragma unroll
      for (int kb = 0; kb < 4; kb++) {
        float ds[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          float p = __builtin_amdgcn_exp2f(st[kb][i] * sc2 - lse2);
          if (!full && kt0 + 16 * kb + 4 * g + i > qrow) p = 0.f;
          ds[i] = p * (dp[kb][i] - delta);
        }
        pk[kb][0] = pack2<T>(ds[0], ds[1]);
        pk[kb][1] = pack2<T>(ds[2], ds[3]);
      }
    }
    // ---- O^T += V^T P^T  /  dQ^T += K^T dS^T (two 32-key steps)
    const uint16_t* tb = BWD ? kb_ : vb_;
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      const int qq = r16 >> 2, pp = r16 & 3;
      const int row0 = 16 * (2 * kk) + 4 * g + qq, row1 = row0 + 16;
#pragma unroll
      for (int d = 0; d < DT; d++) {
        const int col = 16 * d + 4 * pp;
        const uint2 v0 = ds_read_tr16(tb + pf_off<D>(row0, col >> 3) + (col & 7));
        const uint2 v1 = ds_read_tr16(tb + pf_off<D>(row1, col >> 3) + (col & 7));
        const uint4 va = make_uint4(v0.x, v0.y, v1.x, v1.y);
        const uint4 pb = make_uint4(pk[2 * kk][0], pk[2 * kk][1], pk[2 * kk + 1][0], pk[2 * kk + 1][1]);
        o[d] = mfma16<T>(va, pb, o[d]);
      }
    }
    ta_wait_vm0();                               // tile t + 1 landed (this wave's pieces)
    __syncthreads();
  }

  // ---- store: lane holds O^T / dQ^T [16 d + 4 g + i][row qrow]
  if constexpr (!BWD) {
    float l = lpart;
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    if (qrow >= a.T) return;
    uint16_t* op = a.out + ((size_t)(b * a.T + qrow) * a.Hq + h) * D;
#pragma unroll
    for (int d = 0; d < DT; d++)
      *(uint2*)(op + 16 * d + 4 * g) = make_uint2(pack2<T>(o[d][0] * inv, o[d][1] * inv),
                                                  pack2<T>(o[d][2] * inv, o[d][3] * inv));
    if (g == 0) a.lse[((size_t)b * a.Hq + h) * a.T + qrow] = l > 0.f ? mrow + __log2f(l) : INFINITY;
  } else {
    const float s = a.scale;
    uint16_t* op = a.dq + (((size_t)b * a.Hq + h) * a.T + qrow) * D;
#pragma unroll
    for (int d = 0; d < DT; d++)
      *(uint2*)(op + 16 * d + 4 * g) = make_uint2(pack2<T>(o[d][0] * s, o[d][1] * s),
                                                  pack2<T>(o[d][2] * s, o[d][3] * s));
  }
}

// ---- dK / dV -----------------------------------------------------------------
template <typename T, int D>
__global__ void __launch_bounds__(256) fa_dkdv_kernel(const TrainAttnArgs a) {
  constexpr int KSTEP = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) uint16_t qs[2][FA_QB * D];
  __shared__ __attribute__((aligned(16))) uint16_t os[2][FA_QB * D];   // dO tile
  __shared__ float ls[2][2 * FA_QB];                                   // LSE2, delta of the tile's rows
  const int nkb = gridDim.x;
  const int kb = blockIdx.x;                                           // key block (light ones last: causal)
  const int kvh = blockIdx.y, b = blockIdx.z;
  const int G = a.Hq / a.Hkv;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int key = kb * FA_KT + wave * 16 + r16;                        // this lane's key (B operand column)
  (void)nkb;
  // K / V fragments: B operands of S = Q K^T and dP = dO V^T
  uint4 kf[KSTEP], vf[KSTEP];
  {
    const uint16_t* kp = a.k + (size_t)b * a.ksb + (size_t)kvh * a.ksh + (size_t)key * a.kst;
    const uint16_t* vp = a.v + (size_t)b * a.vsb + (size_t)kvh * a.vsh + (size_t)key * a.vst;
#pragma unroll
    for (int s = 0; s < KSTEP; s++) {
      kf[s] = *(const uint4*)(kp + 32 * s + 8 * g);
      vf[s] = *(const uint4*)(vp + 32 * s + 8 * g);
    }
  }
  const int qb0 = a.causal ? kb : 0;                                   // first query block that sees these keys
  const int nqb = a.T / FA_QB - qb0;
  const int nwork = G * nqb;                                           // (head, query block) pairs
  float lreg = 0.f;
  const uint32_t qs_l = ta_lds_addr(qs), os_l = ta_lds_addr(os);
  constexpr uint32_t TILE_B = FA_QB * D * 2;
  auto load_tile = [&](int w, int buf) {
    const int hh = kvh * G + w / nqb, qb = qb0 + w % nqb;
    const uint16_t* qp = a.q + (size_t)b * a.qsb + (size_t)hh * a.qsh;
    const uint16_t* dp = a.dout + (size_t)b * a.dsb + (size_t)hh * a.dsh;
    ta_stage<D>(ta_make_rsrc(qp, (uint32_t)(((int64_t)(a.T - 1) * a.qst + D) * 2)), qs_l + buf * TILE_B,
                qb * FA_QB, a.qst, a.T, wave, lane);
    ta_stage<D>(ta_make_rsrc(dp, (uint32_t)(((int64_t)(a.T - 1) * a.dst + D) * 2)), os_l + buf * TILE_B,
                qb * FA_QB, a.dst, a.T, wave, lane);
    if (tid < 2 * FA_QB) {
      const size_t ri = ((size_t)b * a.Hq + hh) * a.T + qb * FA_QB + (tid & (FA_QB - 1));
      lreg = tid < FA_QB ? a.lse[ri] : a.delta[ri];
    }
  };
  auto store_tile = [&](int buf) {
    if (tid < 2 * FA_QB) ls[buf][tid] = lreg;
  };

  f32x4 dk[DT], dv[DT];                       // lane holds dK / dV [key 4 g + i of the wave][d 16 dt + r16]
#pragma unroll
  for (int d = 0; d < DT; d++) { dk[d] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[d] = f32x4{0.f, 0.f, 0.f, 0.f}; }
  constexpr float kLog2e = 1.4426950408889634f;
  const float sc2 = a.scale * kLog2e;

  if (nwork > 0) {
    load_tile(0, 0);
    ta_wait_vm0();
    store_tile(0);
  }
  __syncthreads();
  for (int w = 0; w < nwork; w++) {
    const int buf = w & 1;
    if (w + 1 < nwork) load_tile(w + 1, buf ^ 1);
    const int qb = qb0 + w % nqb;
    const bool diag = a.causal && qb == kb;
    const uint16_t* qb_ = qs[buf];
    const uint16_t* ob_ = os[buf];
    // ---- S = Q K^T, dP = dO V^T: lane holds query rows 16 qt + 4 g + i for key `key`
    uint32_t pk[4][2], dk16[4][2];
#pragma unroll
    for (int qt = 0; qt < 4; qt++) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f}, p = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < KSTEP; ss++) {
        const uint4 qa = *(const uint4*)(qb_ + pf_off<D>(16 * qt + r16, 4 * ss + g));
        const uint4 oa = *(const uint4*)(ob_ + pf_off<D>(16 * qt + r16, 4 * ss + g));
        s = mfma16<T>(qa, kf[ss], s);
        p = mfma16<T>(oa, vf[ss], p);
      }
      float pv[4], dsv[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int qr = 16 * qt + 4 * g + i;                           // row within the tile
        float pr = __builtin_amdgcn_exp2f(s[i] * sc2 - ls[buf][qr]);
        if (diag && wave * 16 + r16 > qr) pr = 0.f;                    // key > query (same block offsets)
        pv[i] = pr;
        dsv[i] = pr * (p[i] - ls[buf][FA_QB + qr]);
      }
      pk[qt][0] = pack2<T>(pv[0], pv[1]);
      pk[qt][1] = pack2<T>(pv[2], pv[3]);
      dk16[qt][0] = pack2<T>(dsv[0], dsv[1]);
      dk16[qt][1] = pack2<T>(dsv[2], dsv[3]);
    }
    // ---- dV += P^T dO, dK += dS^T Q over two 32-row query steps
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      const int qq = r16 >> 2, pp = r16 & 3;
      const int row0 = 16 * (2 * kk) + 4 * g + qq, row1 = row0 + 16;
      const uint4 pa = make_uint4(pk[2 * kk][0], pk[2 * kk][1], pk[2 * kk + 1][0], pk[2 * kk + 1][1]);
      const uint4 da = make_uint4(dk16[2 * kk][0], dk16[2 * kk][1], dk16[2 * kk + 1][0], dk16[2 * kk + 1][1]);
#pragma unroll
      for (int d = 0; d < DT; d++) {
        const int col = 16 * d + 4 * pp;
        const uint2 o0 = ds_read_tr16(ob_ + pf_off<D>(row0, col >> 3) + (col & 7));
        const uint2 o1 = ds_read_tr16(ob_ + pf_off<D>(row1, col >> 3) + (col & 7));
        const uint2 q0 = ds_read_tr16(qb_ + pf_off<D>(row0, col >> 3) + (col & 7));
        const uint2 q1 = ds_read_tr16(qb_ + pf_off<D>(row1, col >> 3) + (col & 7));
        dv[d] = mfma16<T>(pa, make_uint4(o0.x, o0.y, o1.x, o1.y), dv[d]);
        dk[d] = mfma16<T>(da, make_uint4(q0.x, q0.y, q1.x, q1.y), dk[d]);
      }
    }
    ta_wait_vm0();                               // Q / dO tiles and the LSE / delta row of w + 1
    if (w + 1 < nwork) store_tile(buf ^ 1);
    __syncthreads();
  }
  // ---- store dK (scaled) / dV: [B, Hkv, T, D] contiguous
  const int k0 = kb * FA_KT + wave * 16 + 4 * g;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint16_t* kp = a.dk + (((size_t)b * a.Hkv + kvh) * a.T + k0 + i) * D + r16;
    uint16_t* vp = a.dv + (((size_t)b * a.Hkv + kvh) * a.T + k0 + i) * D + r16;
#pragma unroll
    for (int d = 0; d < DT; d++) {
      kp[16 * d] = from_f32<T>(dk[d][i] * a.scale);
      vp[16 * d] = from_f32<T>(dv[d][i]);
    }
  }
}

// delta[b, h, t] = sum_d dO * O  (O / dO [B, T, Hq, D] contiguous rows); one wave per row
template <typename T, int D>
__global__ void __launch_bounds__(256) fa_delta_kernel(const TrainAttnArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);                 // over B * T * Hq
  const int lane = threadIdx.x & 63;
  if (row >= a.B * a.T * a.Hq) return;
  const int h = row % a.Hq, bt = row / a.Hq, t = bt % a.T, b = bt / a.T;
  const uint16_t* op = a.o + (size_t)b * a.osb + (size_t)h * a.osh + (size_t)t * a.ost;
  const uint16_t* dp = a.dout + (size_t)b * a.dsb + (size_t)h * a.dsh + (size_t)t * a.dst;
  float s = 0.f;
  for (int d = lane * 2; d < D; d += 128) {
    const uint32_t ov = *(const uint32_t*)(op + d), dv = *(const uint32_t*)(dp + d);
    s += to_f32<T>(ov & 0xffff) * to_f32<T>(dv & 0xffff) + to_f32<T>(ov >> 16) * to_f32<T>(dv >> 16);
  }
  s = wave_sum(s);
  if (lane == 0) a.delta[((size_t)b * a.Hq + h) * a.T + t] = s;
}

template <typename T, int D>
void launch_fwd_d(const TrainAttnArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((fa_q_kernel<T, D, false>), dim3((a.T + FA_QB - 1) / FA_QB, a.Hq, a.B), dim3(256), 0, st, a);
}

template <typename T, int D>
void launch_bwd_d(const TrainAttnArgs& a, hipStream_t st) {
  const int rows = a.B * a.T * a.Hq;
  hipLaunchKernelGGL((fa_delta_kernel<T, D>), dim3((rows + 3) / 4), dim3(256), 0, st, a);
  hipLaunchKernelGGL((fa_dkdv_kernel<T, D>), dim3(a.T / FA_KT, a.Hkv, a.B), dim3(256), 0, st, a);
  hipLaunchKernelGGL((fa_q_kernel<T, D, true>), dim3(a.T / FA_QB, a.Hq, a.B), dim3(256), 0, st, a);
}

}  // namespace

void launch_train_attn_fwd(bool bf16, const TrainAttnArgs& a, hipStream_t st) {
  if (bf16) { if (a.D == 64) launch_fwd_d<BF16, 64>(a, st); else launch_fwd_d<BF16, 128>(a, st); }
  else { if (a.D == 64) launch_fwd_d<F16, 64>(a, st); else launch_fwd_d<F16, 128>(a, st); }
}

void launch_train_attn_bwd(bool bf16, const TrainAttnArgs& a, hipStream_t st) {
  if (bf16) { if (a.D == 64) launch_bwd_d<BF16, 64>(a, st); else launch_bwd_d<BF16, 128>(a, st); }
  else { if (a.D == 64) launch_bwd_d<F16, 64>(a, st); else launch_bwd_d<F16, 128>(a, st); }
}

}  // namespace illm
