// Decode attention v3: multi-wave flash-decoding splits (included by attention.cuh).
//
// Reference ops: xe_addons.sdp (decode, q_len <= 32, native GQA;
// models/common.py:250-286) and the vLLM-XPU paged_attention_v2 GQA kernels
// (VLLM_PATCH:3380-3460); the fused RoPE + KV append replaces
// rotary_half_inplaced + the KV-cache write of models/llama.py:155-166.
//
// Why a v3 (MI355X, Llama-3-8B, 1 K keys; profiles/decode_trace_b{1,8}_r4.txt):
// v2 runs one wave per 64-key split.  At batch 8 that is 1088 one-wave
// workgroups = 4.25 waves per CU; each wave requests its K rows, computes
// Q K^T, and only then its V rows (a second memory round trip), so the
// 33.5 MB of KV streamed at 1.66 TB/s (15.4 us) plus a 4.8 us combine launch.
// v3:
//   * one wave per 32 keys and NW (2, 4, 8) waves per workgroup (split = 32 NW
//     keys): every K AND V byte of the wave is requested before any math
//     (16 KB per wave at D = 128, 64 VGPRs), so a CU has 9+ waves x 16 KB in
//     flight in ONE round trip;
//   * the sequence length and the wave's block-table entry are loaded
//     together (the table index is clamped, the entry is used only by waves
//     that hold keys), one dependent step less than v2;
//   * the NW waves merge max / sum / P V in LDS: one (o, m, l) partial per
//     workgroup (a quarter / eighth of v2's), and workgroups past the sequence
//     write an empty (m = -inf) partial, so the merge needs no sequence length;
//   * the merge of a (batch, kv head) is done either by a small combine launch
//     (one memory round trip: every split's partial of a row is in flight at
//     once) or, with v3_counters, by the last-arriving workgroup of that
//     (batch, kv head) with all its NW waves (write-through partials + one
//     agent-scope atomic ticket, the MI355X hand-off form of illm_device.h).
// Row r of the P V MFMA depends only on row r of P, and each split's
// reductions run in a fixed key order: a multi-row verify (speculative decoding)
// reduces every row exactly like one-token decoding with the same NW.
#pragma once

namespace illm {

constexpr int V3_KPW = 32;   // keys per wave
// waves per SIMD the register allocation must leave room for (hipcc
// -DILLM_ATTN_V3_MINW=n forces one value): per mode, the most that compiles
// without scratch spills -- q from memory 4 (118 VGPRs), pre-rotated fused
// RoPE 3 (156), RoPE applied here 2.  At the default (1) hipcc took 188-276
// VGPRs: 1-2 waves per SIMD, so the 576 four-wave workgroups of batch 8 ran in
// more than one round over the 256 CUs
#ifdef ILLM_ATTN_V3_MINW
#define ILLM_V3_MINW(RQ) ILLM_ATTN_V3_MINW
#else
#define ILLM_V3_MINW(RQ) ((RQ) == 1 ? 2 : (RQ) == 2 ? 3 : 4)
#endif

// q / k / v of the new token from the qkv GEMV's f32 accumulator (fused
// RoPE decode, Tq == 1): see attn_decode_v2_kernel (attention.cuh) for the
// rounding contract; lane (r16, g) gets dims 32 s + 8 g + j, s < KSTEP.
// Loads and math are split: the kernel issues every accumulator / bias /
// cos-sin load of the wave (load(), load_cs(), vload()) right behind its K / V
// loads, straight-line, and only then does the math, so the fused-RoPE path
// waits once, for the K / V round trip (the previous per-column load-use chain
// behind a bias branch added one round trip per k-step after the K / V rows
// arrived: 18.5 vs 14.1 us at batch 8, profiles/attn_dec_v3_r5.jsonl).
// PRE: the qkv GEMV epilogue already rotated q / k and there is no bias (the
// decoder's Llama path): no cos / sin, no bias registers.
template <typename T, int D, bool PRE>
struct V3Rope {
  static constexpr int KSTEP = D / 32;
  static constexpr int HS = KSTEP / 2;
  struct Raw {            // the lane's KSTEP x 8 accumulator columns (+ bias)
    float4 f[KSTEP][2];
    uint4 bb[KSTEP];
  };
  struct CS {             // cos / sin of the lane's rotated dims (fast path)
    float4 q[HS][4];
  };
  const AttnDecodeArgs a;   // by value: a reference member made hipcc copy the kernel arguments to scratch
  int b, g;
  float ss;
  int64_t rpos;
  __device__ V3Rope(const AttnDecodeArgs& a_, int b_, int g_, bool on) : a(a_), b(b_), g(g_) {
    ss = on && a.rq_ss ? a.rq_ss[b] : 0.f;
    rpos = on && !PRE ? a.rq_pos[b] : 0;
  }
  __device__ float rs() const { return a.rq_ss ? rsqrtf(ss / (float)a.rq_ss_n + a.rq_ss_eps) : 1.f; }
  __device__ bool fast_rot() const { return !PRE && a.rq_rot == D && !a.rq_interleaved; }
  __device__ static float rnd(float v) { return to_f32<T>(from_f32<T>(v)); }
  // issue the loads of columns col0 + 32 s + 8 g .. + 8 (straight-line: the
  // bias is read unconditionally from a valid address and selected away)
  __device__ void load(int col0, Raw& r) const {
    const float* p = a.rq_part + (size_t)b * a.rq_ld + col0 + 8 * g;
    const bool hb = a.rq_bias != nullptr;
    const uint16_t* bp = hb ? a.rq_bias + col0 + 8 * g : (const uint16_t*)p;
#pragma unroll
    for (int s = 0; s < KSTEP; s++) {
      r.f[s][0] = *(const float4*)(p + 32 * s);
      r.f[s][1] = *(const float4*)(p + 32 * s + 4);
      if constexpr (!PRE) r.bb[s] = *(const uint4*)(bp + (hb ? 32 * s : 64 * s));
    }
  }
  __device__ void load_cs(CS& c) const {
    if (!fast_rot() || a.rq_prerot) return;
    const float4* csp = (const float4*)a.rq_cos_sin + (size_t)rpos * (D / 4);
#pragma unroll
    for (int s = 0; s < HS; s++)
#pragma unroll
      for (int e = 0; e < 4; e++) c.q[s][e] = csp[(32 * s + 8 * g) / 2 + e];
  }
  // the 8 columns at col .. col + 8 (value-row layout), loads only
  __device__ void vload(int col, float4& f0, float4& f1, uint4& u) const {
    const float* p = a.rq_part + (size_t)b * a.rq_ld + col;
    f0 = *(const float4*)p;
    f1 = *(const float4*)(p + 4);
    if constexpr (!PRE) u = *(const uint4*)(a.rq_bias ? a.rq_bias + col : (const uint16_t*)p);
  }
  __device__ void vals8(const float4& f0, const float4& f1, const uint4& u, float rsv, float* v) const {
    float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!PRE && a.rq_bias) {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; e++) {
        bb[2 * e] = to_f32<T>((uint16_t)(w[e] & 0xffff));
        bb[2 * e + 1] = to_f32<T>((uint16_t)(w[e] >> 16));
      }
    }
    const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = rnd(bb[j] + rsv * f[j]);
  }
  __device__ void vals(const Raw& r, float (&v)[KSTEP][8]) const {
    const float rsv = rs();
#pragma unroll
    for (int s = 0; s < KSTEP; s++) vals8(r.f[s][0], r.f[s][1], r.bb[s], rsv, v[s]);
  }
  // general rotary (partial / interleaved): per-element reads, not the hot path
  __device__ float raw1(int col) const {
    float s = a.rq_bias ? to_f32<T>(a.rq_bias[col]) : 0.f;
    s += rs() * a.rq_part[(size_t)b * a.rq_ld + col];
    return rnd(s);
  }
  __device__ float rot1(int col0, int d) const {
    const int half = a.rq_rot / 2;
    if (d >= a.rq_rot) return raw1(col0 + d);
    int i, d0, d1;
    bool first;
    if (a.rq_interleaved) { i = d >> 1; d0 = 2 * i; d1 = d0 + 1; first = (d & 1) == 0; }
    else { first = d < half; i = first ? d : d - half; d0 = i; d1 = i + half; }
    const float2 cs = ((const float2*)a.rq_cos_sin)[(size_t)rpos * half + i];
    const float c = rnd(cs.x), sn = rnd(cs.y);
    const float x0 = raw1(col0 + d0), x1 = raw1(col0 + d1);
    return first ? rnd(x0 * c) - rnd(x1 * sn) : rnd(x1 * c) + rnd(x0 * sn);
  }
  // rotated (q: scaled by scale_out) fragments of the head at column col0
  // from its values v (the lane's dims 32 s + 8 g + j)
  __device__ void frags(int col0, const float (&v)[KSTEP][8], const CS& c, float scale_out, uint4* outf) const {
    if (PRE || a.rq_prerot) {
#pragma unroll
      for (int s = 0; s < KSTEP; s++) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; j++) w[j] = pack2<T>(v[s][2 * j] * scale_out, v[s][2 * j + 1] * scale_out);
        outf[s] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    } else if (fast_rot()) {
#pragma unroll
      for (int s = 0; s < HS; s++) {
        float cc[8], sn[8];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const float4 q = c.q[s][e];
          cc[2 * e] = rnd(q.x); sn[2 * e] = rnd(q.y); cc[2 * e + 1] = rnd(q.z); sn[2 * e + 1] = rnd(q.w);
        }
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          float r0[2], r1[2];
#pragma unroll
          for (int t = 0; t < 2; t++) {
            const int j = 2 * e + t;
            const float x0 = v[s][j], x1 = v[s + HS][j];
            r0[t] = (rnd(x0 * cc[j]) - rnd(x1 * sn[j])) * scale_out;
            r1[t] = (rnd(x1 * cc[j]) + rnd(x0 * sn[j])) * scale_out;
          }
          lo[e] = pack2<T>(r0[0], r0[1]);
          hi[e] = pack2<T>(r1[0], r1[1]);
        }
        outf[s] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
        outf[s + HS] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KSTEP; s++) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
          w[j] = pack2<T>(rot1(col0, 32 * s + 8 * g + 2 * j) * scale_out, rot1(col0, 32 * s + 8 * g + 2 * j + 1) * scale_out);
        outf[s] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
};

// merge the ns split partials of every query row of (b, kv head kvh):
// thread -> (row, 16-B quad of D); all of a row's (m, l) and o quads of a
// 16-split chunk are requested before any is used (one memory round trip for
// ns <= 16), later chunks rescale online.  SC1: handed over inside the launch.
template <typename T, bool SC1>
__device__ __forceinline__ void v3_combine(const AttnDecodeArgs& a, int b, int kvh, int ns, int tid, int nthr) {
  constexpr int CH = 16;
  const int group = a.Hq / a.Hkv, R = group * a.Tq, Q = a.D / 4;
  for (int idx = tid; idx < R * Q; idx += nthr) {
    const int r = idx / Q, q = idx % Q;
    const int t = r / group, h = kvh * group + r % group;
    const size_t row0 = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit;
    float M = -INFINITY, L = 0.f;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s0 = 0; s0 < ns; s0 += CH) {
      float2 ml[CH];
      float4 pv[CH];
#pragma unroll
      for (int j = 0; j < CH; j++) {
        const size_t s = row0 + min(s0 + j, ns - 1);
        if constexpr (SC1) {
          ml[j] = ld8_sc1(a.part_ml + s * 2);
          pv[j] = ld16_sc1(a.part_o, s * a.D + 4 * q);
        } else {
          ml[j] = *(const float2*)(a.part_ml + s * 2);
          pv[j] = *(const float4*)(a.part_o + s * a.D + 4 * q);
        }
      }
      float mc = -INFINITY;
#pragma unroll
      for (int j = 0; j < CH; j++)
        if (s0 + j < ns) mc = fmaxf(mc, ml[j].x);
      const float Mn = fmaxf(M, mc);
      if (Mn == -INFINITY) continue;                 // nothing visible yet
      const float f = M == -INFINITY ? 0.f : __expf(M - Mn);
      L *= f; o.x *= f; o.y *= f; o.z *= f; o.w *= f;
#pragma unroll
      for (int j = 0; j < CH; j++) {
        // an empty split's o is unwritten: select, never multiply
        const bool on = s0 + j < ns && ml[j].x != -INFINITY;
        const float w = on ? __expf(ml[j].x - Mn) : 0.f;
        L += on ? w * ml[j].y : 0.f;
        o.x += on ? w * pv[j].x : 0.f; o.y += on ? w * pv[j].y : 0.f;
        o.z += on ? w * pv[j].z : 0.f; o.w += on ? w * pv[j].w : 0.f;
      }
      M = Mn;
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    uint16_t* out = a.out + (((size_t)b * a.Tq + t) * a.Hq + h) * a.D + 4 * q;
    *(uint2*)out = make_uint2(pack2<T>(o.x * inv, o.y * inv), pack2<T>(o.z * inv, o.w * inv));
  }
  if (a.rq_part != nullptr) {
    // fused-RoPE decode: every split of (b, kvh) has read its q / k / v columns
    // of the qkv accumulator: re-zero them for the next layer's atomic GEMV
    float* prow = (float*)a.rq_part + (size_t)b * a.rq_ld;
    const int D = a.D;
    for (int i = tid * 4; i < (group + 2) * D; i += nthr * 4) {
      const int hh = i / D, d = i % D;
      const int col = hh < group ? (kvh * group + hh) * D : (a.Hq + (hh - group) * a.Hkv + kvh) * D;
      *(float4*)(prow + col + d) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) attn_combine_v3_kernel(const AttnDecodeArgs a, int ns) {
  v3_combine<T, false>(a, blockIdx.y, blockIdx.x, ns, threadIdx.x, 256);
}

// LDS of one v3 workgroup
template <int D, int NW, int RQ>
struct V3Smem {
  __attribute__((aligned(16))) uint16_t vl[V3_KPW * NW * D];   // V tile; then the P V reduction
  __attribute__((aligned(16))) float knew[RQ != 0 ? NW : 1][D];  // the new k row (fused RoPE)
  float smx[NW][16], sml[NW][16];
  int s_last;
};

// one (split, kv head, batch row) workgroup of NW waves; nsg = splits in the
// grid; RQ: q/k/v from the qkv accumulator (Tq == 1): 1 RoPE applied here
// (+ bias), 2 pre-rotated by the qkv GEMV and bias-free
template <typename T, int D, int NW, int RQ, bool FUSE>
__device__ __forceinline__ void attn_v3_body(const AttnDecodeArgs& a, int split, int kvh, int b, int nsg,
                                             V3Smem<D, NW, RQ>& sm) {
  constexpr int KSTEP = D / 32;     // MFMA k-steps over the head dim
  constexpr int DT = D / 16;        // 16-dim output tiles
  constexpr int VU = D / 8;         // 16-B chunks per key row
  constexpr int KPJ = 64 / VU;      // keys per V staging instruction
  constexpr int VJ = V3_KPW / KPJ;  // V staging loads per lane
  constexpr int SK = V3_KPW * NW;   // keys per workgroup split
  static_assert(D == 64 || D == 128, "v3: head_dim 64 / 128");
  static_assert(RQ == 0 || D == 128, "v3: fused RoPE needs head_dim 128");
  const int lane = threadIdx.x & 63, r16 = lane & 15, g = lane >> 4;
  const int wv = threadIdx.x >> 6;
  const int group = a.Hq / a.Hkv;
  const int R = group * a.Tq;
  const int k0 = split * SK, kw0 = k0 + V3_KPW * wv;

  auto& smx = sm.smx;
  auto& sml = sm.sml;
  auto& knew = sm.knew;
  uint16_t* vl = sm.vl;

  // ---- sequence length and this wave's block-table entry, in flight together
  // (fused RoPE: with the row's rms scale, position and the wave's q columns)
  int len = a.seq_lens[b];
  const int blk = a.block_tables[(size_t)b * a.max_blocks + min(kw0 / a.bs, a.max_blocks - 1)];
  const int row = r16 < R ? r16 : 0;
  const int t = row / group, h = kvh * group + row % group;
  const V3Rope<T, D, RQ == 2> rp(a, b, g, RQ != 0);
  typename V3Rope<T, D, RQ == 2>::Raw qraw;
  uint4 qpl[KSTEP];
  if constexpr (RQ == 0) {
    const uint16_t* qr = a.q + (((size_t)b * a.Tq + t) * a.Hq + h) * D;
#pragma unroll
    for (int s = 0; s < KSTEP; s++) qpl[s] = *(const uint4*)(qr + 32 * s + 8 * g);
  }
  // coverage is the caller's nominal split grid (nsplit x SPLIT keys), which
  // the rounded-up v3 grid can exceed: keys past it are reported, not read
  if ((int64_t)len > (int64_t)a.max_blocks * a.bs || (int64_t)a.nsplit * SPLIT < len) {
    if (split == 0 && threadIdx.x == 0) kerr(a.err, ERR_SEQ_LEN);
    len = min(min(len, a.max_blocks * a.bs), a.nsplit * SPLIT);
  }
  const size_t prow = (((size_t)b * a.Hq + h) * a.Tq + t) * a.nsplit + split;

  if (k0 >= len) {
    // past the sequence: an empty partial (the merge skips it by its m)
    if (wv == 0 && g == 0 && r16 < R) {
      if constexpr (FUSE) st8_sc1(a.part_ml + prow * 2, -INFINITY, 0.f);
      else *(float2*)(a.part_ml + prow * 2) = make_float2(-INFINITY, 0.f);
    }
  } else {
    const int nkw = kw0 < len ? min(V3_KPW, len - kw0) : 0;
    const bool blk_bad = nkw > 0 && bad_block(blk, a.num_blocks);
    if (blk_bad && lane == 0) kerr(a.err, ERR_BLOCK_ID);
    const bool ld_on = nkw > 0 && !blk_bad;            // wave-uniform
    const int nvis = ld_on ? nkw : 0;
    const size_t base = ld_on ? (((size_t)blk * a.Hkv + kvh) * a.bs + (kw0 % a.bs)) * D : 0;
    const uint16_t* kb = (const uint16_t*)a.k_cache + base;
    const uint16_t* vb = (const uint16_t*)a.v_cache + base;

    // ---- every K and V load of the wave
    uint4 kf[2][KSTEP], vm[VJ];
    if (ld_on) {
#pragma unroll
      for (int kt = 0; kt < 2; kt++) {
        const int kk = min(kt * 16 + r16, nkw - 1);
#pragma unroll
        for (int s = 0; s < KSTEP; s++) kf[kt][s] = *(const uint4*)(kb + (size_t)kk * D + 32 * s + 8 * g);
      }
#pragma unroll
      for (int j = 0; j < VJ; j++) {
        const int kk = min(j * KPJ + lane / VU, nkw - 1);
        vm[j] = *(const uint4*)(vb + (size_t)kk * D + 8 * (lane % VU));
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < 2; kt++)
#pragma unroll
        for (int s = 0; s < KSTEP; s++) kf[kt][s] = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < VJ; j++) vm[j] = make_uint4(0, 0, 0, 0);
    }

    // fused RoPE: the wave's q columns, cos / sin and (the wave holding the
    // new key, position len - 1) the new k / v rows' columns in value-row
    // layout (lane: 8 dims at d0), requested right behind the K / V rows
    const bool holds_new = RQ != 0 && ld_on && kw0 + nkw == len;   // wave-uniform
    const int d0 = 8 * (lane % VU);
    typename V3Rope<T, D, RQ == 2>::CS cs;
    float4 kn0, kn1, vn0, vn1;
    uint4 knb, vnb;
    if constexpr (RQ != 0) {
      rp.load(h * D, qraw);
      rp.load_cs(cs);
      if (holds_new) {
        rp.vload((a.Hq + kvh) * D + d0, kn0, kn1, knb);
        rp.vload((a.Hq + a.Hkv + kvh) * D + d0, vn0, vn1, vnb);
      }
    }

    // ---- q fragments (lane: row r16, dims 32 s + 8 g .. + 8)
    uint4 qf[KSTEP];
    if constexpr (RQ != 0) {
      {
        float v[KSTEP][8];
        rp.vals(qraw, v);
        rp.frags(h * D, v, cs, a.rq_qscale, qf);
      }
      if (r16 >= R)
#pragma unroll
        for (int s = 0; s < KSTEP; s++) qf[s] = make_uint4(0, 0, 0, 0);
      if (holds_new) {
        // k / v from the accumulator replace the not-yet-written cache row in
        // registers and are appended to the cache for later steps; the k row
        // goes through the wave's LDS row to the MFMA layout (lane (kn & 15, g))
        const int kn = nkw - 1;
        const float rsv = rp.rs();
        const size_t crow = (((size_t)blk * a.Hkv + kvh) * a.bs + (size_t)((len - 1) % a.bs)) * D;
        if (lane < VU) {
          float kv[8];
          rp.vals8(kn0, kn1, knb, rsv, kv);
          *(float4*)&knew[wv][d0] = make_float4(kv[0], kv[1], kv[2], kv[3]);
          *(float4*)&knew[wv][d0 + 4] = make_float4(kv[4], kv[5], kv[6], kv[7]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (r16 == (kn & 15)) {
          float kv[KSTEP][8];
#pragma unroll
          for (int s = 0; s < KSTEP; s++) {
            const float4 u0 = *(const float4*)&knew[wv][32 * s + 8 * g];
            const float4 u1 = *(const float4*)&knew[wv][32 * s + 8 * g + 4];
            kv[s][0] = u0.x; kv[s][1] = u0.y; kv[s][2] = u0.z; kv[s][3] = u0.w;
            kv[s][4] = u1.x; kv[s][5] = u1.y; kv[s][6] = u1.z; kv[s][7] = u1.w;
          }
          uint4 kq[KSTEP];
          rp.frags((a.Hq + kvh) * D, kv, cs, 1.f, kq);
#pragma unroll
          for (int kt = 0; kt < 2; kt++)
            if (kt == (kn >> 4))
#pragma unroll
              for (int s = 0; s < KSTEP; s++) kf[kt][s] = kq[s];
#pragma unroll
          for (int s = 0; s < KSTEP; s++) *(uint4*)((uint16_t*)a.k_cache + crow + 32 * s + 8 * g) = kq[s];
        }
        if (lane / VU == kn % KPJ) {
          float vv[8];
          rp.vals8(vn0, vn1, vnb, rsv, vv);
          const uint4 vq = make_uint4(pack2<T>(vv[0], vv[1]), pack2<T>(vv[2], vv[3]), pack2<T>(vv[4], vv[5]),
                                      pack2<T>(vv[6], vv[7]));
#pragma unroll
          for (int j = 0; j < VJ; j++)
            if (j == kn / KPJ) vm[j] = vq;
          *(uint4*)((uint16_t*)a.v_cache + crow + d0) = vq;
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < KSTEP; s++) qf[s] = r16 < R ? qpl[s] : make_uint4(0, 0, 0, 0);
    }

    // ---- S^T tiles: lane holds (key = 16 kt + 4 g + i, row = r16)
    f32x4 st[2];
#pragma unroll
    for (int kt = 0; kt < 2; kt++) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSTEP; s++) acc = mfma16<T>(kf[kt][s], qf[s], acc);
      st[kt] = acc;
    }
    const int qpos = len - a.Tq + t;
#pragma unroll
    for (int kt = 0; kt < 2; kt++)
#pragma unroll
      for (int i = 0; i < 4; i++) st[kt][i] *= a.scale;
    if (a.softcap > 0.f) {
#pragma unroll
      for (int kt = 0; kt < 2; kt++)
#pragma unroll
        for (int i = 0; i < 4; i++) st[kt][i] = a.softcap * tanhf(st[kt][i] / a.softcap);
    }
    if (a.alibi) {
      const float slope = r16 < R ? a.alibi[h] : 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; kt++)
#pragma unroll
        for (int i = 0; i < 4; i++) st[kt][i] += slope * (float)(kw0 + kt * 16 + 4 * g + i);
    }
    const int win = a.sliding_window > 0 ? qpos - a.sliding_window : -1;
    const int klim = min(nvis, qpos - kw0 + 1);           // keys kk < klim are visible
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; kt++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int kk = kt * 16 + 4 * g + i;
        const bool ok = r16 < R && kk < klim && kw0 + kk > win;
        st[kt][i] = ok ? st[kt][i] : -INFINITY;
        m = fmaxf(m, st[kt][i]);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    if constexpr (NW > 1) {
      if (g == 0) smx[wv][r16] = m;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < NW; w++) m = fmaxf(m, smx[w][r16]);
    }
    // ---- P (T precision, as the MFMA consumes it) and the wave's V rows in LDS
    float l = 0.f;
    uint32_t pk[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; kt++) {
      float p[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        p[i] = m == -INFINITY ? 0.f : __expf(st[kt][i] - m);
        l += p[i];
      }
      pk[kt][0] = pack2<T>(p[0], p[1]);
      pk[kt][1] = pack2<T>(p[2], p[3]);
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
#pragma unroll
    for (int j = 0; j < VJ; j++) *(uint4*)(vl + pf_off<D>(V3_KPW * wv + j * KPJ + lane / VU, lane % VU)) = vm[j];
    if constexpr (NW > 1) {
      if (g == 0) sml[wv][r16] = l;
    }
    // ---- O^T = V^T P^T over the wave's own 32 keys (its own LDS rows: no barrier)
    f32x4 o[DT];
#pragma unroll
    for (int d = 0; d < DT; d++) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      const int qq = r16 >> 2, pp = r16 & 3;
      const int row0 = V3_KPW * wv + 4 * g + qq, row1 = row0 + 16;
      const uint4 pb = make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
#pragma unroll
      for (int d = 0; d < DT; d++) {
        const int col = 16 * d + 4 * pp;
        const uint2 v0 = ds_read_tr16(vl + pf_off<D>(row0, col >> 3) + (col & 7));
        const uint2 v1 = ds_read_tr16(vl + pf_off<D>(row1, col >> 3) + (col & 7));
        o[d] = mfma16<T>(make_uint4(v0.x, v0.y, v1.x, v1.y), pb, o[d]);
      }
    }
    float* ob = (float*)vl;          // [NW][DT][64] float4: wave w's rows of vl (its own V rows, now read)
    if constexpr (NW > 1) {
#pragma unroll
      for (int d = 0; d < DT; d++)
        *(float4*)(ob + ((size_t)(wv * DT + d) * 64 + lane) * 4) = make_float4(o[d][0], o[d][1], o[d][2], o[d][3]);
      __syncthreads();
      l = 0.f;
#pragma unroll
      for (int w = 0; w < NW; w++) l += sml[w][r16];
    }
    // ---- the workgroup's partial: wave w writes output tiles w, w + NW, ...
    if (r16 < R) {
      float* po = a.part_o + prow * D + 4 * g;
#pragma unroll
      for (int d = 0; d < DT; d++) {
        if (NW > 1 && d % NW != wv) continue;
        float4 s4 = make_float4(o[d][0], o[d][1], o[d][2], o[d][3]);
        if constexpr (NW > 1) {
          s4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int w = 0; w < NW; w++) {
            const float4 u = *(const float4*)(ob + ((size_t)(w * DT + d) * 64 + lane) * 4);
            s4.x += u.x; s4.y += u.y; s4.z += u.z; s4.w += u.w;
          }
        }
        if constexpr (FUSE) st16_sc1(a.part_o, (size_t)(po - a.part_o) + 16 * d, s4);
        else *(float4*)(po + 16 * d) = s4;
      }
      if (wv == 0 && g == 0) {
        if constexpr (FUSE) st8_sc1(a.part_ml + prow * 2, m, l);
        else *(float2*)(a.part_ml + prow * 2) = make_float2(m, l);
      }
    }
  }
  if constexpr (FUSE) {
    // ---- the last workgroup of (b, kvh) to arrive merges every split
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's write-through stores are done
    __syncthreads();
    if (threadIdx.x == 0) {
      int* ctr = a.v3_counters + (size_t)b * a.Hkv + kvh;
      const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sm.s_last = prev == nsg - 1;
      if (sm.s_last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!sm.s_last) return;
    v3_combine<T, true>(a, b, kvh, nsg, threadIdx.x, NW * 64);
  }
}

template <typename T, int D, int NW, int RQ, bool FUSE>
__global__ void __launch_bounds__(64 * NW, ILLM_V3_MINW(RQ)) attn_decode_v3_kernel(const AttnDecodeArgs a) {
  __shared__ V3Smem<D, NW, RQ> sm;
  attn_v3_body<T, D, NW, RQ, FUSE>(a, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, sm);
}

// waves per workgroup: the most (>= 4) that still leaves >= ~2 workgroups per CU
// (a function of the batch, kv heads and split grid only, so a multi-row
// verify picks the same NW as one-token decoding of the same batch);
// ILLM_ATTN_V3_NW forces it
inline int v3_pick_nw(const AttnDecodeArgs& a) {
  static const int env = getenv("ILLM_ATTN_V3_NW") ? atoi(getenv("ILLM_ATTN_V3_NW")) : 0;
  if (env == 2 || env == 4 || env == 8) return env;   // >= 2: the partial arrays hold nsplit 64-key splits
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const long keys = (long)a.nsplit * SPLIT;
  for (int nw = 8; nw >= 4; nw >>= 1) {
    const long wgs = (long)a.B * a.Hkv * ((keys + V3_KPW * nw - 1) / (V3_KPW * nw));
    if (wgs >= 2L * cus) return nw;
  }
  // small grids: 4 waves (128-key splits) measured fastest at batch 1 and 8
  // (tools/bench_attn_dec.py, profiles/attn_dec_v3_r5.jsonl)
  return 4;
}

template <typename T, int D, int NW, int RQ>
static void launch_v3_nw(const AttnDecodeArgs& a, hipStream_t st) {
  const int ns = (a.nsplit * SPLIT + V3_KPW * NW - 1) / (V3_KPW * NW);
  dim3 grid(ns, a.Hkv, a.B);
  if (a.v3_counters != nullptr) {
    hipLaunchKernelGGL((attn_decode_v3_kernel<T, D, NW, RQ, true>), grid, dim3(64 * NW), 0, st, a);
  } else {
    hipLaunchKernelGGL((attn_decode_v3_kernel<T, D, NW, RQ, false>), grid, dim3(64 * NW), 0, st, a);
    hipLaunchKernelGGL((attn_combine_v3_kernel<T>), dim3(a.Hkv, a.B), dim3(256), 0, st, a, ns);
  }
}

template <typename T, int D, int RQ>
static void launch_v3(const AttnDecodeArgs& a, hipStream_t st) {
  switch (v3_pick_nw(a)) {
    case 1: return launch_v3_nw<T, D, 1, RQ>(a, st);
    case 2: return launch_v3_nw<T, D, 2, RQ>(a, st);
    case 4: return launch_v3_nw<T, D, 4, RQ>(a, st);
    default: return launch_v3_nw<T, D, 8, RQ>(a, st);
  }
}

// v3 serves the 16-bit-KV, combined (not split-only) decode of head dim 64 /
// 128 with <= 16 rows per kv head; ILLM_ATTN_V3=0 keeps v2 everywhere
inline bool v3_ok(const AttnDecodeArgs& a, int D) {
  static const bool on = !(getenv("ILLM_ATTN_V3") && atoi(getenv("ILLM_ATTN_V3")) == 0);
  const int R = (a.Hq / a.Hkv) * a.Tq;
  return on && a.kv_fp8 == 0 && !a.no_combine && R <= 16 && (D == 128 || (D == 64 && a.rq_part == nullptr)) &&
         a.counters == nullptr;
}

}  // namespace illm
