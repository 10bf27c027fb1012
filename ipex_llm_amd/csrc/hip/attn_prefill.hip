// Prefill / long-query attention straight over the paged KV cache
// (flash-attention forward, causal, GQA).
//
// Reference ops: xe_addons.sdp_causal / sdp_fp8_causal / sdp_non_causal
// (SRC/transformers/models/common.py:271-286), gemma2_sdp_causal (softcap,
// sliding window; models/gemma2.py:133-155) and the vLLM-XPU context
// (chunked-prefill) attention (VLLM_PATCH csrc/xpu).  Used for prefill,
// chunked prefill over a cached prefix and speculative / lookup verification
// (query chunks too wide for the decode kernel).
//
// MI355X design (gfx950, wave64, v_mfma_f32_16x16x32 bf16/f16):
//   * workgroup = 4 waves = 64 query rows of one head; wave w owns rows
//     16w..16w+15.  Causal q-blocks are issued heaviest first;
//   * K/V tiles of 64 keys are read once per workgroup straight from the
//     paged cache (a 64-key tile never crosses a cache block, bs % 64 == 0),
//     the next tile's loads in flight while the current one is computed,
//     and staged in LDS as [key][D] rows with a 16-byte XOR swizzle;
//   * swapped QK^T: S^T = K Q^T (A = K rows from LDS by ds_read_b128, B = the
//     wave's Q rows kept in registers), so a lane holds 16 scores of ONE query
//     row: the online-softmax row max / sum is a register reduction plus two
//     shuffles;
//   * P V as O^T = V^T P^T: the B operand (P^T) is the lane's own scores
//     converted to 16-bit (key order of the C layout, no lane movement), the
//     A operand (V^T) comes from ds_read_b64_tr_b16 transposed reads of the
//     row-major V tile in exactly that key order;
//   * fp8 KV caches are converted to 16-bit while the tile is staged.
#include <cstdlib>

#include "../common/quant_block.h"
#include "illm_device.h"
#include "kernels.h"

namespace illm {

constexpr int PF_KT = 64;      // keys per tile
constexpr int PF_QB = 64;      // query rows per workgroup

template <typename T, int KVF>
__device__ __forceinline__ uint4 pf_load8(const uint8_t* p, float scale) {
  if constexpr (KVF == 0) {
    return *(const uint4*)p;
  } else {
    const uint2 u = *(const uint2*)p;
    float v[8];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t w = i ? u.y : u.x;
      auto f0 = KVF == 1 ? __builtin_amdgcn_cvt_pk_f32_bf8(w, false) : __builtin_amdgcn_cvt_pk_f32_fp8(w, false);
      auto f1 = KVF == 1 ? __builtin_amdgcn_cvt_pk_f32_bf8(w, true) : __builtin_amdgcn_cvt_pk_f32_fp8(w, true);
      v[4 * i + 0] = f0[0] * scale;
      v[4 * i + 1] = f0[1] * scale;
      v[4 * i + 2] = f1[0] * scale;
      v[4 * i + 3] = f1[1] * scale;
    }
    return make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7]));
  }
}

// HP = query heads per wave that share one kv head (GQA): every K fragment
// read from LDS and every transposed V read feeds HP MFMAs.
template <typename T, int D, int KVF, int HP, bool SOFTCAP>
__global__ void __launch_bounds__(256) attn_prefill_kernel(const AttnPrefillArgs a) {
  constexpr int EB = KVF == 0 ? 2 : 1;            // cache bytes per element
  constexpr int KSTEP = D / 32;                   // MFMA k-steps over the head dim (QK^T)
  constexpr int DT = D / 16;                      // 16-wide d tiles of O^T
  constexpr int UPT = PF_KT * D / 8 / 256;        // 8-element staging units per thread per tile
  // double-buffered K / V tiles: the next tile is written while the current
  // one is read, one workgroup barrier per tile
  __shared__ __attribute__((aligned(16))) uint16_t ks[2][PF_KT * D];
  __shared__ __attribute__((aligned(16))) uint16_t vs[2][PF_KT * D];

  // causal work per query block grows with its index.  Block order: heaviest
  // query blocks of every (head, batch) first (longest-processing-time first
  // for the dynamic dispatch); when the whole grid is resident at once (<= 2
  // workgroups per CU: 64 KiB of LDS each) the second half runs the light
  // blocks in ascending order instead, so workgroups i and i + grid/2 (one CU)
  // pair up to the same total (T = 1024: every CU 17 tiles instead of up to 32)
  const int nqb = gridDim.x, nother = gridDim.y * gridDim.z;
  const int lin = blockIdx.x + nqb * (blockIdx.y + gridDim.y * blockIdx.z);
  const int rank = lin / nother, other = lin % nother;
  const int half = (nqb + 1) / 2;
  const int qb = (nqb * nother <= 512 && rank >= half) ? rank - half : nqb - 1 - rank;
  const int h0 = (other % gridDim.y) * HP, b = other / gridDim.y;
  const int kvh = h0 / (a.Hq / a.Hkv);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int L = a.seq_lens[b];
  const int Tq = a.Tq;
  const int p0 = L - Tq;                          // position of query row 0
  const int qrow = qb * PF_QB + wave * 16 + r16;  // this lane's query row (B operand column)
  const int qpos = p0 + min(qrow, Tq - 1);

  // key range of the workgroup
  const int wg_q0 = p0 + qb * PF_QB;
  const int wg_q_last = min(Tq - 1, qb * PF_QB + PF_QB - 1);
  const int kend = min(L, p0 + wg_q_last + 1);
  int kbeg = 0;
  if (a.sliding_window > 0) kbeg = max(0, wg_q0 - a.sliding_window + 1) & ~(PF_KT - 1);
  const int ntile = kend > kbeg ? (kend - kbeg + PF_KT - 1) / PF_KT : 0;

  // Q fragments (B operand of S^T = K Q^T): row qrow, dims 32 s + 8 g .. + 7
  uint4 qf[HP][KSTEP];
#pragma unroll
  for (int j = 0; j < HP; j++) {
    const uint16_t* qp = a.q + ((size_t)(b * Tq + min(qrow, Tq - 1)) * a.Hq + h0 + j) * D;
#pragma unroll
    for (int s = 0; s < KSTEP; s++) qf[j][s] = *(const uint4*)(qp + 32 * s + 8 * g);
  }

  // staging: unit u = tid + 256 j covers key u / (D / 8), chunk u % (D / 8)
  auto tile_src = [&](int t, const uint8_t* cache) -> const uint8_t* {
    const int k0 = kbeg + t * PF_KT;
    int blk = a.block_tables[(size_t)b * a.max_blocks + k0 / a.bs];
    if (bad_block(blk, a.num_blocks)) {                  // read block 0 instead, report
      kerr(a.err, ERR_BLOCK_ID);
      blk = 0;
    }
    return cache + (((size_t)blk * a.Hkv + kvh) * a.bs + (k0 % a.bs)) * D * EB;
  };
  uint4 kreg[UPT], vreg[UPT];
  auto load_tile = [&](int t) {
    const uint8_t* kp = tile_src(t, a.k_cache);
    const uint8_t* vp = tile_src(t, a.v_cache);
    const int k0 = kbeg + t * PF_KT;
#pragma unroll
    for (int j = 0; j < UPT; j++) {
      const int u = tid + 256 * j;
      const int r = u / (D / 8), c = u % (D / 8);
      kreg[j] = pf_load8<T, KVF>(kp + ((size_t)r * D + c * 8) * EB, a.k_scale);
      vreg[j] = pf_load8<T, KVF>(vp + ((size_t)r * D + c * 8) * EB, a.v_scale);
      // slots past the sequence end hold stale bytes (possibly NaN patterns):
      // p = 0 times NaN would still poison the P V product, so zero them
      if (k0 + r >= L) kreg[j] = vreg[j] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < UPT; j++) {
      const int u = tid + 256 * j;
      const int r = u / (D / 8), c = u % (D / 8);
      *(uint4*)(ks[buf] + pf_off<D>(r, c)) = kreg[j];
      *(uint4*)(vs[buf] + pf_off<D>(r, c)) = vreg[j];
    }
  };

  f32x4 o[HP][DT];
#pragma unroll
  for (int j = 0; j < HP; j++)
#pragma unroll
    for (int d = 0; d < DT; d++) o[j][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[HP], lpart[HP];
#pragma unroll
  for (int j = 0; j < HP; j++) { mrow[j] = -INFINITY; lpart[j] = 0.f; }
  const float sc = a.scale;
  constexpr float kLog2e = 1.4426950408889634f;
  const float sc2 = a.scale * kLog2e;

  if (ntile > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  for (int t = 0; t < ntile; t++) {
    const int buf = t & 1;
    if (t + 1 < ntile) load_tile(t + 1);          // next tile in flight during the compute
    const int kt0 = kbeg + t * PF_KT;
    const uint16_t* kb_ = ks[buf];
    const uint16_t* vb_ = vs[buf];
    // tiles wholly below every query row of the workgroup need no mask
    const bool full = kt0 + PF_KT - 1 <= wg_q0 && kt0 + PF_KT <= L && a.sliding_window <= 0;

    // ---- S^T = K Q^T : lane holds keys 16 kb + 4 g + i of query row r16
    f32x4 st[HP][4];
#pragma unroll
    for (int kb = 0; kb < 4; kb++) {
#pragma unroll
      for (int j = 0; j < HP; j++) st[j][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSTEP; s++) {
        const uint4 kf = *(const uint4*)(kb_ + pf_off<D>(16 * kb + r16, 4 * s + g));
#pragma unroll
        for (int j = 0; j < HP; j++) st[j][kb] = mfma16<T>(kf, qf[j][s], st[j][kb]);
      }
    }
    // ---- scale, soft-cap, causal / window / length mask, online softmax
    uint32_t pk[HP][4][2];                         // P^T fragments, 16-bit pairs
#pragma unroll
    for (int j = 0; j < HP; j++) {
      // soft-cap is a template flag and the mask one uniform branch per tile:
      // a per-score branch (tanhf's own control flow inlined 16 times) split
      // the tile loop into ~100 basic blocks, so no MFMA / VALU interleaving
      // across them (rocprofv3: 3 SALU and 10 VALU per MFMA)
#pragma unroll
      for (int kb = 0; kb < 4; kb++) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
          // scores in the exp2 domain (scale * log2 e folded in): p = exp2(v - m)
          float v;
          if constexpr (SOFTCAP) v = a.softcap * tanhf(st[j][kb][i] * sc / a.softcap) * kLog2e;
          else v = st[j][kb][i] * sc2;
          st[j][kb][i] = v;
        }
      }
      if (!full) {
        const int win = a.sliding_window > 0 ? qpos - a.sliding_window : -1;
#pragma unroll
        for (int kb = 0; kb < 4; kb++) {
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int key = kt0 + 16 * kb + 4 * g + i;
            const bool ok = key <= qpos && key < L && key > win;
            st[j][kb][i] = ok ? st[j][kb][i] : -INFINITY;
          }
        }
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 4; kb++)
#pragma unroll
        for (int i = 0; i < 4; i++) tmax = fmaxf(tmax, st[j][kb][i]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(mrow[j], tmax);
      // nothing seen yet (mrow = -inf): exp2(-inf) = 0 clears the empty O; a row
      // still fully masked keeps alpha 1 and a finite max of 0 for the exp2 below
      const float alpha = mnew == -INFINITY ? 1.f : __builtin_amdgcn_exp2f(mrow[j] - mnew);
      const float msafe = mnew == -INFINITY ? 0.f : mnew;
      mrow[j] = mnew;
      // O rescale only when some row max of the wave moved (wave-uniform)
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {
        lpart[j] *= alpha;
#pragma unroll
        for (int d = 0; d < DT; d++) {
          o[j][d][0] *= alpha; o[j][d][1] *= alpha; o[j][d][2] *= alpha; o[j][d][3] *= alpha;
        }
      }
#pragma unroll
      for (int kb = 0; kb < 4; kb++) {
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          p[i] = __builtin_amdgcn_exp2f(st[j][kb][i] - msafe);      // masked: exp2(-inf) = 0
          lpart[j] += p[i];
        }
        pk[j][kb][0] = pack2<T>(p[0], p[1]);
        pk[j][kb][1] = pack2<T>(p[2], p[3]);
      }
    }
    // ---- O^T += V^T P^T over two 32-key steps (key blocks 2 ks, 2 ks + 1)
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
      // lane 4q + p of the 16-lane group g addresses row 16 kb + 4 g + q, columns 16 dt + 4 p
      const int qq = r16 >> 2, pp = r16 & 3;
      const int row0 = 16 * (2 * kk) + 4 * g + qq, row1 = row0 + 16;
#pragma unroll
      for (int d = 0; d < DT; d++) {
        const int col = 16 * d + 4 * pp;                     // element column; chunk col / 8
        const uint2 v0 = ds_read_tr16(vb_ + pf_off<D>(row0, col >> 3) + (col & 7));
        const uint2 v1 = ds_read_tr16(vb_ + pf_off<D>(row1, col >> 3) + (col & 7));
        const uint4 va = make_uint4(v0.x, v0.y, v1.x, v1.y);
#pragma unroll
        for (int j = 0; j < HP; j++) {
          const uint4 pb = make_uint4(pk[j][2 * kk][0], pk[j][2 * kk][1], pk[j][2 * kk + 1][0], pk[j][2 * kk + 1][1]);
          o[j][d] = mfma16<T>(va, pb, o[j][d]);
        }
      }
    }
    if (t + 1 < ntile) store_tile(buf ^ 1);       // read last during tile t - 1: free since the barrier
    __syncthreads();
  }

  // ---- normalise and store: lane holds O^T[16 d + 4 g + i][row r16]
#pragma unroll
  for (int j = 0; j < HP; j++) {
    float l = lpart[j];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (qrow >= Tq) continue;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = a.out + ((size_t)(b * Tq + qrow) * a.Hq + h0 + j) * D;
#pragma unroll
    for (int d = 0; d < DT; d++) {
      *(uint2*)(op + 16 * d + 4 * g) = make_uint2(pack2<T>(o[j][d][0] * inv, o[j][d][1] * inv),
                                                  pack2<T>(o[j][d][2] * inv, o[j][d][3] * inv));
    }
  }
}

template <typename T, int D, int HP, bool SC>
static void launch_pf_sc(const AttnPrefillArgs& a, hipStream_t st) {
  dim3 grid((a.Tq + PF_QB - 1) / PF_QB, a.Hq / HP, a.B);
  if (a.kv_fp8 == 1) hipLaunchKernelGGL((attn_prefill_kernel<T, D, 1, HP, SC>), grid, dim3(256), 0, st, a);
  else if (a.kv_fp8 == 2) hipLaunchKernelGGL((attn_prefill_kernel<T, D, 2, HP, SC>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((attn_prefill_kernel<T, D, 0, HP, SC>), grid, dim3(256), 0, st, a);
}

template <typename T, int D, int HP>
static void launch_pf_hp(const AttnPrefillArgs& a, hipStream_t st) {
  if (a.softcap > 0.f) launch_pf_sc<T, D, HP, true>(a, st);
  else launch_pf_sc<T, D, HP, false>(a, st);
}

template <typename T, int D>
static void launch_pf_d(const AttnPrefillArgs& a, hipStream_t st) {
  // HP = 2: two query heads of one kv head per wave, so every K fragment and
  // transposed V read from LDS feeds two MFMAs (even GQA group).  It halves
  // the grid, so it is taken when the halved grid still covers the chip
  // twice (2 workgroups per CU).  Measured on MI355X (Llama-3-8B heads):
  // T = 4096 266 -> 212 us, B = 8 x 1024 164 -> 120 us, T = 16 K 3.42 ->
  // 2.46 ms (895 TFLOP/s); T = 1024 (256 workgroups) 30.3 -> 37.3 us, so HP = 1
  // there.  ILLM_PREFILL_HP=1/2 forces either.
  static const int hp_env = getenv("ILLM_PREFILL_HP") ? atoi(getenv("ILLM_PREFILL_HP")) : 0;
  const bool even = (a.Hq / a.Hkv) % 2 == 0;
  const long wg2 = (long)((a.Tq + PF_QB - 1) / PF_QB) * (a.Hq / 2) * a.B;
  const bool hp2 = even && (hp_env == 2 || (hp_env == 0 && wg2 >= 512));
  if (hp2) launch_pf_hp<T, D, 2>(a, st);
  else launch_pf_hp<T, D, 1>(a, st);
}

template <typename T>
static void launch_pf_t(const AttnPrefillArgs& a, hipStream_t st) {
  if (a.D == 64) launch_pf_d<T, 64>(a, st);
  else launch_pf_d<T, 128>(a, st);
}

void launch_attn_prefill(bool bf16, const AttnPrefillArgs& a, hipStream_t st) {
  if (bf16) launch_pf_t<BF16>(a, st); else launch_pf_t<F16>(a, st);
}

}  // namespace illm
