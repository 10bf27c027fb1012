// Host-callable launchers of the gfx950 kernels.  Implemented in the .hip
// files of this directory; called from the torch op wrappers
// (csrc/torch/ops_hip.cpp).  Pure HIP API: no torch headers here, so the
// kernel translation units compile in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace illm {

}  // namespace illm
#include "gemv_args.h"
namespace illm {

// ---- low-bit GEMV / skinny GEMM (lowbit_gemv.cuh) -------------------------
// dk = decoder kind (fmt_to_dk), mt = ceil(M/16) in {1,2,4}
template <int DK>
void launch_gemv_dk(bool bf16, int mt, int epi, dim3 grid, const GemvArgs& a, hipStream_t st);
// v5 (M <= 16, lowbit_gemv5.cuh): workgroup = 4 waves = (4 / kw) tile groups
// x kw k-parts; grid = (ceil(groups / (4 / kw)), ksplit[, experts]),
// shmem = gemv5_shmem(rows, chunks per split) <= 159 KiB
template <int DK>
void launch_gemv5_dk(bool bf16, int kw, int epi, dim3 grid, size_t shmem, const GemvArgs& a, hipStream_t st);
constexpr int gemv5_x_ld_h(int kw) { return (kw + 511) / 512 * 512 + 8; }   // == gemv5_x_ld
constexpr size_t gemv5_attn_shmem_h(int rows, int cpk, int D, int ns) {
  return (size_t)rows * ((cpk * 128 + D - 1) / D + 1) * (ns + 1) * 4;
}
constexpr size_t gemv5_shmem_h(int rows, int cpk) {
  return ((size_t)rows * gemv5_x_ld_h(cpk * 128) * 2 + 15) / 16 * 16 + (size_t)rows * cpk * 16 + 8 * 2 * 64 * 16;
}

// ---- prefill low-bit GEMM (gemm.hip): out[M, N] = x[M, K] @ W^T (+ bias), f16 MFMA
struct GemmArgs {
  const uint16_t* x;       // [M, ldx] T
  int M, K, ldx;
  const uint8_t* w;        // tiled device blob
  int N, KC;
  const uint16_t* bias;    // T [N] or null
  uint16_t* out;           // [M, ldo] T
  int ldo;
  int lut_fmt;
  int glu;                 // 1: tile-interleaved gate/up weight, out = act(gate) * up [M, N / 2]
  int act;                 // 0 = silu, 1 = gelu(tanh)
  int x_f16;               // 1: x already holds f16 copies of the bf16 activations
  const float* rs;         // per x-row power-of-two scale (launch_x_to_f16_rowscale), null = 1:
                           // x rows are normalised into f16 range, the epilogue multiplies rs back
  // grouped (MoE, "FlashMoE") launch: (token, expert) pairs sorted by expert
  // (moe_align); blockIdx.x walks (expert, m-block) over every local expert's
  // pairs, weights of expert e at w + e * w_stride.  M = number of pairs.
  const int32_t* moe_off;  // [El + 1] pair offsets per local expert (device), null = plain GEMM
  const int32_t* moe_rows; // [P] pair ids sorted by expert
  int moe_el;              // local experts
  int moe_xdiv;            // gathered x row = pair id / moe_xdiv (x_sorted == 0)
  int moe_x_sorted;        // 1: x row = sorted position (the previous grouped GEMM's output)
  int moe_out_sorted;      // 1: out row = sorted position; 0: out row = pair id
  int64_t w_stride;        // bytes between experts' blobs
  int out_f32;             // 1: out is f32 [rows, ldo] (pre-combine partials)
};
void launch_lowbit_gemm(bool bf16, int fmt, const GemmArgs& a, hipStream_t st);
// bf16 -> f16 with saturation at +-65504 (the GEMM's MFMA input type), n % 8 == 0
void launch_bf16_to_f16_sat(const uint16_t* x, uint16_t* y, int64_t n, hipStream_t st);

// per-row power-of-two normalisation to f16: y = x * 2^s_m (row max in [2^14, 2^15)), rs[m] = 2^-s_m
void launch_x_to_f16_rowscale(bool bf16, const uint16_t* x, int64_t M, int64_t ldx, int K, uint16_t* y, float* rs,
                              hipStream_t st);

// ---- training kernels (train_kernels.hip) ------------------------------------
// fused CE over logits [rows, ld] (V % 8 == 0): loss[row] = lse - x[label] (0 when
// ignored); write_grad: logits := (softmax - onehot) * scale in place (0 rows if ignored)
void launch_ce_fused(bool bf16, uint16_t* logits, int64_t rows, int64_t ld, int V, const int64_t* labels,
                     int ignore_index, float scale, float* loss, bool write_grad, hipStream_t st);
// out[r, n] += alpha * sum_m a[m, r] * b[m, n]  (a f32 [M, R], R <= 64; b 16-bit [M, ldb]; N % 8 == 0)
void launch_skinny_tn(bool bf16, const float* a, int R, const uint16_t* b, int64_t ldb, int M, int N, float alpha,
                      float* out, hipStream_t st);

// ---- k-quant decoders (kquant.hip): GGUF q4_K / q5_K / q6_K / q2_K blocks ---
void launch_kq_dequant(int fmt, bool bf16, const uint8_t* w, int64_t n, int64_t k, uint16_t* out, hipStream_t st);
void launch_kq_gemv(int fmt, bool bf16, const uint16_t* x, int M, int64_t K, const uint8_t* w, int64_t N,
                    uint16_t* out, hipStream_t st);

// ---- dense bf16/f16 skinny GEMM (dense_gemv.hip): M <= 16, K % 8 == 0 ----
// act(x Wg^T) * (x Wu^T), W = 16-row tile-interleaved gate/up [2I, K], M <= 16
void launch_dense_glu(bool bf16, const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t I, int act,
                      uint16_t* out, hipStream_t st);
void launch_dense_gemv(bool bf16, const uint16_t* x, int M, int64_t K, const uint16_t* w, int64_t N,
                       const uint16_t* bias, uint16_t* out, hipStream_t st, bool trans_out = false);

// ---- fp8 linear (fp8_gemm.hip): torch_fp8 qtypes on the f8f6f4 MFMA --------
struct Fp8GemmArgs {
  const uint8_t* xq;       // [M, K] e4m3 activations (GEMM)
  const float* sx;         // [M] activation scales (GEMM)
  const uint16_t* x;       // [M, K] bf16/f16 activations (GEMV)
  const uint8_t* w;        // [N, K] fp8 weight
  const float* sw;         // [1] or [N] weight scale
  int sw_per_channel;
  const uint16_t* bias;    // [N] or null
  uint16_t* out;           // [M, N]
  int M, N;
  int64_t K;
};
// per-token e4m3 quantization: xq = sat(x / sx), sx = amax / 448 (K % 8 == 0)
void launch_fp8_act_quant(bool bf16, const uint16_t* x, int64_t M, int64_t K, uint8_t* xq, float* sx,
                          hipStream_t st);
// N % 128 == 0, K % 128 == 0
void launch_fp8_gemm(bool bf16, bool e5m2, const Fp8GemmArgs& a, hipStream_t st);
// M <= 16, K % 16 == 0
void launch_fp8_gemv(bool bf16, bool e5m2, const Fp8GemmArgs& a, hipStream_t st);

// ---- norms (norm.hip) ------------------------------------------------------
struct NormArgs {
  const uint16_t* x;       // [M, H] input (ignored when partials != null)
  const float* partials;   // [nsplit, M, H] f32 GEMV partial slabs or null
  int nsplit;
  uint16_t* residual;      // [M, H] residual stream (in/out) or null
  const uint16_t* w;       // [H]
  uint16_t* out;           // [M, H]
  int M, H;
  float eps;
  int unit_offset;         // gemma: x * (1 + w)
  int store_residual;
  int zero_partials;       // re-zero the (atomic-accumulated) partial slab after reading it
  // embedding gather (decode step entry): row m of the input is x[ids[m]] of
  // the [vocab, H] table, written unnormalised to gather_out (the residual
  // stream) next to the normalised out; block 0 also zeroes zero[0:zero_n]
  const int64_t* ids;
  int64_t vocab;
  uint16_t* gather_out;
  float* zero;
  int zero_n;
  int* err;
};
void launch_add_rms_norm(bool bf16, const NormArgs& a, hipStream_t st);
void launch_rms_norm_bwd(bool bf16, const uint16_t* x, const uint16_t* g, const uint16_t* w, uint16_t* dx, int M,
                         int H, float eps, int unit_offset, hipStream_t st);
void launch_layer_norm(bool bf16, const uint16_t* x, const uint16_t* w, const uint16_t* b,
                       uint16_t* out, int M, int H, float eps, hipStream_t st);

// ---- rotary embedding + KV-cache append (rope_kv.hip) --------------------
struct RopeKVArgs {
  const uint16_t* qkv;     // [T, (Hq + 2 Hkv) * D] fused projection output
  int ld_qkv;
  uint16_t* q_out;         // [T, Hq, D]
  uint8_t* k_cache;        // paged cache [nblocks, Hkv, bs, D] (elem = kv_bytes)
  uint8_t* v_cache;
  const int64_t* slots;    // [T] cache slot = block * bs + offset; <0 = skip
  const int64_t* pos;      // [T] rotary position
  const float* inv_freq;   // [rot_dim / 2]  (used when cos_sin is null)
  const float* cos_sin;    // [max_pos, rot_dim / 2, 2] precomputed f32 table or null
  const uint16_t* q_norm;  // [D] per-head RMSNorm weight (qwen3) or null
  const uint16_t* k_norm;
  float norm_eps;
  float attn_scale_q;      // multiply q by this (1.0 = none)
  int T, Hq, Hkv, D, rot_dim, bs;
  int interleaved;         // 0 = rotate_half (NeoX/llama), 1 = pairwise (GPT-J/GLM)
  int kv_fp8;              // 0 = same dtype as activations, 1 = fp8 e5m2, 2 = fp8 e4m3
  float k_scale, v_scale;  // fp8 KV scales (value = code * scale)
  // fused split-K reduction of the QKV GEMV: qkv = sum_s part[s] (+ bias)
  const float* part;       // [nsplit, T, ld_qkv] f32 or null (then qkv is read)
  int nsplit;
  int zero_part;            // re-zero part (atomic accumulator, nsplit == 1) after use
  const uint16_t* bias;    // [ld_qkv] or null
  // device-side slots (slots == null): slot = block_tables[t / tq][pos / bs] * bs + pos % bs
  const int32_t* block_tables;
  int max_blocks, tq;
  const int64_t* pos_offset;   // [B] (cache index = pos - offset) or null
  int num_blocks;              // cache blocks (bounds check of slots / block ids)
  int* err;                    // kernel error word (illm_device.h kerr) or null
  // deferred RMSNorm of the projection input (lowbit_gemv5.cuh ndefer): the
  // accumulator row t is scaled by rsqrt(pss[t] / pss_n + pss_eps) before the bias
  const float* pss;
  int pss_n;
  float pss_eps;
};
void launch_rope_kv(bool bf16, const RopeKVArgs& a, hipStream_t st);

// ---- decode / short-query attention (attention.hip) -----------------------
struct AttnDecodeArgs {
  const uint16_t* q;        // [B, Tq, Hq, D]
  const uint8_t* k_cache;   // [nblocks, Hkv, bs, D]
  const uint8_t* v_cache;
  const int32_t* block_tables;  // [B, max_blocks]
  const int32_t* seq_lens;      // [B] total keys incl. the Tq new ones
  int max_blocks;
  int* counters;                // [B * Hkv] zeroed arrival counters (fused combine) or null
  float* part_o;            // [B, Hq, Tq, nsplit, D]
  float* part_ml;           // [B, Hq, Tq, nsplit, 2]
  uint16_t* out;            // [B, Tq, Hq, D]
  int B, Tq, Hq, Hkv, D, bs, nsplit;
  float scale, softcap;     // softcap > 0: gemma2 tanh soft-capping
  int sliding_window;       // > 0: attend to the last W keys only
  int kv_fp8;
  float k_scale, v_scale;
  const float* alibi;       // [Hq] slopes or null
  int no_combine;           // leave the split partials for the consumer (o_proj GEMV prologue)
  // fused RoPE + KV append (decode, Tq == 1, bf16/f16 KV, D >= 128): q / k / v
  // come straight from the qkv GEMV's atomic accumulator rq_part [B, rq_ld]
  // (+ rq_bias), q/k rotated in registers; the split holding the new key
  // uses it from registers and writes it to the cache (no rope_kv launch)
  const float* rq_part;
  const float* rq_ss;       // deferred RMSNorm: row b of rq_part scaled by rsqrt(rq_ss[b] / rq_ss_n + rq_ss_eps)
  int rq_ss_n;
  float rq_ss_eps;
  const uint16_t* rq_bias;
  const float* rq_cos_sin;  // [max_pos, rot / 2, 2]
  const int64_t* rq_pos;    // [B] rotary positions
  int rq_ld, rq_rot, rq_interleaved;
  float rq_qscale;
  int rq_prerot;            // rq_part already holds rotated q / k (RoPE in the qkv GEMV epilogue)
  int num_blocks;           // cache blocks: block-table entries are bounds-checked
  int* err;                 // kernel error word or null
  // v3 (attn_dec_v3.cuh): zeroed [B * Hkv] arrival counters for its in-kernel
  // combine (null: separate combine launch)
  int* v3_counters;
};
void launch_attn_decode(bool bf16, const AttnDecodeArgs& a, hipStream_t st);

// ---- prefill / long-query attention over the paged cache (attn_prefill.hip)
struct AttnPrefillArgs {
  const uint16_t* q;            // [B * Tq, Hq, D] (sequence-major tokens)
  const uint8_t* k_cache;       // [nblocks, Hkv, bs, D] (bf16/f16 or fp8 bytes)
  const uint8_t* v_cache;
  const int32_t* block_tables;  // [B, max_blocks]
  const int32_t* seq_lens;      // [B] keys incl. the Tq new ones (query t sits at L - Tq + t)
  uint16_t* out;                // [B * Tq, Hq, D]
  int B, Tq, Hq, Hkv, D, bs, max_blocks;
  float scale, softcap;
  int sliding_window;
  int kv_fp8;                   // 0 = 16-bit cache, 1 = e5m2, 2 = e4m3
  float k_scale, v_scale;
  int num_blocks;
  int* err;
};
void launch_attn_prefill(bool bf16, const AttnPrefillArgs& a, hipStream_t st);

// ---- elementwise & misc (misc.hip) ------------------------------------------
void launch_rwkv4_wkv(const float* decay, const float* first, const float* k, const float* v, float* out,
                      float* num, float* den, float* mx, int B, int T, int C, hipStream_t st);
void launch_rwkv5_wkv(const float* w, const float* u, const float* r, const float* k, const float* v, float* out,
                      float* state, int B, int T, int H, int S, hipStream_t st);
void launch_softmax_rows(bool bf16, uint16_t* x, int64_t rows, int L, hipStream_t st);
// read nbytes (16-B granules) from p on `wgs` workgroups and drop them: an
// Infinity-Cache warm-up for the next reader (csrc/hip/prefetch.hip)
void launch_l3_prefetch(const void* p, size_t nbytes, int wgs, unsigned* sink, hipStream_t st);
void launch_glu(bool bf16, const uint16_t* gu, int ld, uint16_t* out, int M, int I, int act, int tile,
                hipStream_t st);
void launch_quantize_device(int fmt, int in_kind, const void* w, int64_t n, int64_t k,
                            uint8_t* blob, int search, hipStream_t st);
// transpose: out is [k, n] (n % 8 == 0) instead of [n, k]
void launch_dequantize_device(bool bf16, int fmt, const uint8_t* blob, int64_t n, int64_t k,
                              uint16_t* out, hipStream_t st, bool transpose = false);
void launch_reduce_partials(bool bf16, const float* ws, int nsplit, const uint16_t* bias,
                            uint16_t* out, int M, int N, int ldo, hipStream_t st);
void launch_moe_topk(const float* logits, int T, int E, int k, int renorm, int scoring,
                     float* topk_w, int32_t* topk_ids, hipStream_t st);

void launch_moe_group_topk(const float* logits, const float* bias, int T, int E, int k, int n_group, int topk_group,
                           int renorm, float scale, float* topk_w, int32_t* topk_ids, hipStream_t st);

void launch_moe_align(const int32_t* ids, int P, int e0, int El, int32_t* off, int32_t* rows, hipStream_t st);

// fused decode router: logits, top-k and per-expert pair lists in one launch
struct MoeRouteArgs {
  const uint16_t* x;      // [T, H] activations
  const uint16_t* wr;     // [E, H] router weight (same 16-bit type)
  int T, H, E, k, renorm, scoring, e0, El;
  int nsp;                // hidden slices (workgroups per expert)
  float* logits;          // [nsp, T, E] f32 scratch (partial sums)
  int* counter;           // zero on entry, left zero (last workgroup resets it)
  float* topk_w;          // [T, k]
  int32_t* topk_ids;      // [T, k]
  int32_t* off;           // [El + 1]
  int32_t* rows;          // [T * k]
};
void launch_moe_route(bool bf16, const MoeRouteArgs& a, hipStream_t st);
void launch_moe_combine(bool bf16, const float* part, int ks, int P, const float* w, const int32_t* ids, int k,
                        int e0, int El, uint16_t* out, int Tn, int H, hipStream_t st);

void launch_act_mul(bool bf16, const uint16_t* g, const uint16_t* u, const uint16_t* dy, uint16_t* y, uint16_t* dg,
                    uint16_t* du, int64_t n, int act, hipStream_t s);
void launch_rope_half(bool bf16, const uint16_t* x, int64_t sb, int64_t sh, int64_t st, const uint16_t* cs,
                      const uint16_t* sn, int64_t csb, uint16_t* out, int B, int H, int Tn, int D, int bwd,
                      hipStream_t s);
void launch_embedding_rows(bool bf16, const uint8_t* blob, int fmt, const int64_t* ids, int T, int64_t n, int64_t k,
                           uint16_t* out, int* err, hipStream_t st);

void launch_decode_advance(bool bf16, const uint16_t* logits, int B, int V, int64_t* ids, int64_t* next_ids,
                           int64_t* pos, const int32_t* block_tables, int max_blocks, int bs, int64_t* slots,
                           int32_t* seq_lens, const int64_t* pos_offset, int* err, hipStream_t st,
                           const float* parts = nullptr, int nparts = 0);

// ---- one-shot / two-shot xGMI peer all-reduce (allreduce.hip) -------------
constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 64;
constexpr int AR_THREADS = 512;
// signal area: uint32 [2 phase][2 parity][AR_MAX_BLOCKS][AR_MAX_RANKS] = 8 KiB
constexpr int64_t AR_SIGNAL_BYTES = 8192;
// peer buffer: [signal | data parity 0 | data parity 1 | result parity 0 | result parity 1],
// each data / result half `cap` bytes (the result halves are used by the two-shot form)
enum ArDtype : int { AR_BF16 = 0, AR_F16 = 1, AR_F32 = 2 };

struct AllReduceArgs {
  uint8_t* bufs[AR_MAX_RANKS];  // every rank's buffer base (mapped), own included
  int rank, world;
  const uint4* in;
  uint4* out;
  int64_t nvec;                 // 16-B vectors in the message
  int64_t cap;                  // bytes per data half
  uint32_t* counter;            // [AR_MAX_BLOCKS] local epochs
  int* err;                     // the communicator's flag (CustomAllReduce.check)
  int* kerr;                    // the device kernel error word (ERR_PEER)
  int dtype;                    // ArDtype
  int two_shot;                 // reduce-scatter + all-gather through the result halves
  int64_t inner;                // all-gather: 16-B vectors per row of a rank's slice
};

void launch_custom_all_reduce(const AllReduceArgs& a, hipStream_t st);
// out [rows, W * inner] <- every rank's in [rows, inner] (16-B vectors): the
// vocab-parallel logits gather, same buffers / epochs as the all-reduce
void launch_custom_all_gather(const AllReduceArgs& a, hipStream_t st);
int custom_all_reduce_blocks(int64_t nvec);

// ---- fused multi-tensor AdamW (optim.hip) ----------------------------------
struct AdamWArgs {
  const int64_t* params;       // device pointer tables, one entry per tensor
  const int64_t* grads;
  const int64_t* exp_avg;      // f32 moments
  const int64_t* exp_avg_sq;
  const int64_t* sizes;        // elements per tensor
  const int32_t* chunk_tensor; // [nchunks] tensor of each chunk
  const int64_t* chunk_start;  // [nchunks] first element of each chunk
  int chunk;                   // elements per chunk
  float lr, beta1, beta2, eps, weight_decay, bias_corr1, bias_corr2, grad_scale;
  int param_dtype, grad_dtype; // 0 = f32, 1 = bf16
  // capturable form: f32 {step, lr} read on the device (bias corrections
  // derived in-kernel), so a hipGraph-replayed optimizer step advances them
  const float* step_lr;        // nullptr: use lr / bias_corr1 / bias_corr2 above
};
void launch_fused_adamw(const AdamWArgs& a, int nchunks, hipStream_t st);

}  // namespace illm
