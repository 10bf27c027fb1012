// GPU (HIP, gfx950) implementations of the ipex_llm_amd ops.  Thin shape
// checking + launch on torch's current HIP stream (so everything is
// capturable in a hipGraph via torch.cuda.graph).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include <map>

#include "../common/formats.h"
#include "../hip/kernels.h"
#include "../hip/gemv_args.h"

using at::Tensor;

namespace {

int* kernel_err(const c10::Device& dev);       // per-device kernel error word (defined below)

// decode combine scratch: the wide combine holds up to 4096 split weights in
// LDS (attention.cuh CW_MAXS), the one-wave combine 1024 (used for D % 4 != 0)
constexpr int64_t kMaxDecodeSplits = 4096;

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }
inline bool is_bf16(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf,
              "activations must be bf16 or fp16, got ", t.scalar_type());
  return t.scalar_type() == at::kBFloat16;
}
inline const uint16_t* p16(const Tensor& t) { return (const uint16_t*)t.data_ptr(); }
inline uint16_t* m16(Tensor& t) { return (uint16_t*)t.data_ptr(); }
template <typename O>
inline const uint16_t* p16o(const O& t) {
  return (t.has_value() && t->defined()) ? (const uint16_t*)t->data_ptr() : nullptr;
}

Tensor quantize_device(const Tensor& w, int64_t fmt, bool scale_search) {
  TORCH_CHECK(w.is_cuda() && w.dim() == 2, "quantize_device expects a 2-D GPU tensor");
  c10::DeviceGuard g(w.device());
  const int64_t n = w.size(0), k = w.size(1);
  TORCH_CHECK(k % illm::QBLOCK == 0, "in_features must be a multiple of 64");
  Tensor wc = w.contiguous();
  int kind = 0;
  if (wc.scalar_type() == at::kBFloat16) kind = 1;
  else if (wc.scalar_type() == at::kHalf) kind = 2;
  else wc = wc.to(at::kFloat);
  Tensor blob = at::empty({illm::dev_total_bytes((int)fmt, n, k)}, wc.options().dtype(at::kByte));
  illm::launch_quantize_device((int)fmt, kind, wc.data_ptr(), n, k, blob.data_ptr<uint8_t>(),
                               scale_search ? 1 : 0, cur_stream());
  return blob;
}

// transpose: W^T [k, n] (the operand of grad_x = g W on the NT GEMM)
Tensor dequantize_device(const Tensor& blob, int64_t fmt, int64_t n, int64_t k, at::ScalarType dt, bool transpose) {
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf, "dequantize_device: bf16/fp16 output");
  TORCH_CHECK(!transpose || n % 8 == 0, "dequantize_device: transposed output needs n % 8 == 0");
  c10::DeviceGuard g(blob.device());
  Tensor out = transpose ? at::empty({k, n}, blob.options().dtype(dt)) : at::empty({n, k}, blob.options().dtype(dt));
  illm::launch_dequantize_device(dt == at::kBFloat16, (int)fmt, blob.data_ptr<uint8_t>(), n, k,
                                 m16(out), cur_stream(), transpose);
  return out;
}

#define ILLM_DK_SWITCH(fmt, CALL)                                           \
  switch (illm::fmt_to_dk(fmt)) {                                            \
    case illm::DK_INT4S: { constexpr int DKV = illm::DK_INT4S; CALL; } break; \
    case illm::DK_INT4A: { constexpr int DKV = illm::DK_INT4A; CALL; } break; \
    case illm::DK_LUT4: { constexpr int DKV = illm::DK_LUT4; CALL; } break;   \
    case illm::DK_FP4: { constexpr int DKV = illm::DK_FP4; CALL; } break;     \
    case illm::DK_INT8S: { constexpr int DKV = illm::DK_INT8S; CALL; } break; \
    case illm::DK_INT8A: { constexpr int DKV = illm::DK_INT8A; CALL; } break; \
    case illm::DK_FP8E4: { constexpr int DKV = illm::DK_FP8E4; CALL; } break; \
    case illm::DK_FP8E5: { constexpr int DKV = illm::DK_FP8E5; CALL; } break; \
    default: TORCH_CHECK(false, "gemv: unsupported fmt ", fmt);              \
  }

void launch_gemv_any(int fmt, bool bf16, int mt, int epi, dim3 grid, const illm::GemvArgs& a) {
  hipStream_t st = cur_stream();
  ILLM_DK_SWITCH(fmt, illm::launch_gemv_dk<DKV>(bf16, mt, epi, grid, a, st));
}
int* kernel_err(const c10::Device& dev);
void launch_gemv5_any(int fmt, bool bf16, int kw, int epi, dim3 grid, size_t shmem, const illm::GemvArgs& a0) {
  hipStream_t st = cur_stream();
  static const int pf8 = getenv("ILLM_GEMV5_PF8") ? atoi(getenv("ILLM_GEMV5_PF8")) : 0;
  illm::GemvArgs a = a0;
  a.pf8 = pf8;
#if ILLM_DEVICE_DEBUG
  int dev = 0;
  (void)hipGetDevice(&dev);
  a.err = kernel_err(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)dev));
#endif
  ILLM_DK_SWITCH(fmt, illm::launch_gemv5_dk<DKV>(bf16, kw, epi, grid, shmem, a, st));
}

constexpr size_t kMaxLds = 159 * 1024;

// v1 (M > 16): split K over workgroups until there are >= 768 of them
int64_t auto_ksplit(int64_t NT, int64_t KC) {
  int64_t ks = 1;
  while (NT * ks < 768 && KC >= 4 * 2 * (ks * 2)) ks *= 2;
  return ks;
}

// v5 geometry (M <= 16): each of `groups` tile groups (a tile, or a gate/up
// tile pair for GLU) is streamed by kw waves of one workgroup (in-LDS
// reduction) and, when allowed, by ks workgroups (f32 split-K slabs).
// Measured on MI355X (tools/gemv_sweep5.sh, Llama-3-8B shapes): the x slice
// is staged once per workgroup, so kw > 1 (fewer tiles per workgroup) only
// pays for the unsplittable GLU at M <= 2; split-K workgroups of ~8 chunks
// (M <= 2) / ~4 chunks (M > 2) are fastest for the slab-output projections.
// ILLM_GEMV5_KW / ILLM_GEMV5_KS / ILLM_GEMV5_NW override (sweeps).
struct Plan5 {
  int kw;
  int64_t ks, cpk;
  size_t shmem;
  unsigned gx;
  int nw;
};
Plan5 plan5(int64_t rows, int64_t groups, int64_t KC, bool can_split, int64_t ks_req = 0, bool atomic = false) {
  static const int kw_env = getenv("ILLM_GEMV5_KW") ? atoi(getenv("ILLM_GEMV5_KW")) : 0;
  static const int ks_env = getenv("ILLM_GEMV5_KS") ? atoi(getenv("ILLM_GEMV5_KS")) : 0;
  static const int nw_env = getenv("ILLM_GEMV5_NW") ? atoi(getenv("ILLM_GEMV5_NW")) : 0;
  Plan5 p{1, 1, KC, 0, 0, 4};  // kw, ks, cpk, shmem, gx, nw
  if (!can_split) {
    // GLU: 2-way K split inside the workgroup; M <= 2 -> 4-wave groups (2 tile
    // pairs), larger M -> 8-wave groups (x staged once per 4 pairs).  MI355X
    // (profiles/gemv5_geometry_sweep_r3.jsonl, Llama-3-8B gate/up, M = 1):
    // 448 x 4-wave groups 17.1 us vs 896 x (4-way split, 1 pair) 20.7 us --
    // the 896-group grid needed two residency rounds at 2 waves per SIMD
    p.kw = 2;
    p.nw = rows <= 2 ? 4 : 8;
    while (p.kw > 1 && KC / p.kw < 4) p.kw /= 2;
  } else if (ks_req > 0) {
    p.ks = ks_req;
  } else {
    // 8-wave groups: x slice shared by 8 tiles (down M=16: 10.8 vs 15.7 us);
    // also for the narrow (<= 256-tile) outputs at M = 1 (o 4.85 vs 4.92 us)
    p.nw = (rows >= 4 || groups <= 256) ? 8 : 4;
    // ~4-chunk slices for K <= 8K, ~7 for the wide-K down projection: qkv
    // M = 1 5.75 vs 6.16 us (8 x 4 chunks vs 4 x 8), down M = 1 7.6 vs 10.9 us
    // (16 x 7 vs 14 x 8), M = 8 9.6 vs 11.1 us (same sweep)
    const int64_t target = KC >= 64 ? 7 : 4;
    p.ks = std::min<int64_t>(atomic ? 32 : 16, std::max<int64_t>(1, (KC + target - 1) / target));
    // wide outputs (lm_head: 8016 tiles) already fill the chip: slabs only cost
    while (p.ks > 1 && groups * p.ks > 4096) p.ks /= 2;
    while (illm::gemv5_shmem_h((int)rows, (int)((KC + p.ks - 1) / p.ks)) > 65536 && p.ks < KC) p.ks *= 2;
  }
  if (kw_env) p.kw = kw_env;
  if (ks_env && can_split) p.ks = ks_env;
  p.ks = std::max<int64_t>(1, std::min<int64_t>(p.ks, KC));
  p.cpk = (KC + p.ks - 1) / p.ks;
  p.ks = (KC + p.cpk - 1) / p.cpk;
  p.shmem = illm::gemv5_shmem_h((int)rows, (int)p.cpk);
  if (nw_env) p.nw = nw_env;
  const int64_t per_wg = p.nw / p.kw;
  p.gx = (unsigned)((groups + per_wg - 1) / per_wg);
  return p;
}

// RoPE epilogue: 8-wave groups of one tile each = 128-column, head-aligned blocks
Plan5 plan5_rope(Plan5 p, int64_t NT, int64_t rows) {
  p.kw = 1;
  p.nw = 8;
  p.gx = (unsigned)((NT + 7) / 8);
  return p;
}

Tensor gemv(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k,
            const c10::optional<Tensor>& bias, int64_t epi, int64_t ksplit, int64_t act) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda(), "gemv: GPU tensors expected");
  TORCH_CHECK(x.size(-1) == k, "gemv: x last dim ", x.size(-1), " != in_features ", k);
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(M >= 1 && M <= 64, "gemv handles 1..64 rows, got ", M);
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv: weight blob too small");
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  // M <= 16 runs v5 (ILLM_GEMV_V1=1 forces the general kernel, for A/B tests)
  const bool small = M <= 16 && getenv("ILLM_GEMV_V1") == nullptr;

  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.act = (int)act;
  a.lut_fmt = (int)fmt;
  a.bias = nullptr;
  auto out_shape = xc.sizes().vec();
  if (epi == illm::EPI_GLU) {
    TORCH_CHECK(n % 32 == 0, "GLU weights must have a multiple of 32 rows");
    out_shape.back() = n / 2;
    Tensor out = at::empty(out_shape, xc.options());
    a.N = (int)(n / 2);
    a.out = out.data_ptr();
    a.ldo = (int)(n / 2);
    const Plan5 p = plan5(M, NT / 2, KC, false);
    if (small && p.shmem <= kMaxLds)
      a.nw = p.nw, launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_GLU, dim3(p.gx, 1), p.shmem, a);
    else
      launch_gemv_any((int)fmt, bf16, mt, illm::EPI_GLU, dim3((unsigned)(NT / 2), 1), a);
    return out;
  }
  a.N = (int)n;
  Plan5 p5{};
  bool use5 = false;
  if (small) {
    p5 = plan5(M, NT, KC, true, ksplit);
    use5 = p5.shmem <= kMaxLds;
  }
  if (use5) {
    ksplit = p5.ks;
    a.cpk = (int)p5.cpk;
    a.nw = p5.nw;
  } else {
    if (ksplit <= 0) ksplit = auto_ksplit(NT, KC);
    ksplit = std::min<int64_t>(ksplit, KC);
  }
  auto launch = [&](int e) {
    if (use5) launch_gemv5_any((int)fmt, bf16, p5.kw, e, dim3(p5.gx, (unsigned)ksplit), p5.shmem, a);
    else launch_gemv_any((int)fmt, bf16, mt, e, dim3((unsigned)NT, (unsigned)ksplit), a);
  };
  if (epi == illm::EPI_PARTIAL || ksplit > 1) {
    Tensor ws = at::empty({ksplit, M, n}, xc.options().dtype(at::kFloat));
    a.out = ws.data_ptr();
    a.ldo = (int)n;
    launch(illm::EPI_PARTIAL);
    if (epi == illm::EPI_PARTIAL) return ws;
    out_shape.back() = n;
    Tensor out = at::empty(out_shape, xc.options());
    illm::launch_reduce_partials(bf16, ws.data_ptr<float>(), (int)ksplit, p16o(bias), m16(out), (int)M,
                                 (int)n, (int)n, cur_stream());
    return out;
  }
  out_shape.back() = n;
  Tensor out = at::empty(out_shape, xc.options());
  a.out = out.data_ptr();
  a.ldo = (int)n;
  a.bias = p16o(bias);
  launch(illm::EPI_STORE);
  return out;
}

// greedy decode head: the v5 GEMV stores the logits (T) and every wave writes
// the argmax {max, index} of its columns per row (parts [nparts, M, 2] f32),
// which decode_advance reduces instead of re-reading the [M, V] logits.
// Split-K 1 (the stored values are final); M <= 16.
std::tuple<Tensor, Tensor> gemv_argmax(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k,
                                       const c10::optional<Tensor>& bias) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && x.size(-1) == k, "gemv_argmax: GPU x [M, k]");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(M >= 1 && M <= 16, "gemv_argmax: 1..16 rows");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_argmax: weight blob too small");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  Plan5 p = plan5(M, NT, KC, true, 1);
  // the full-K x slice (M x K bf16) is staged once per workgroup: larger M
  // shares it among 8 tiles (one workgroup per CU fits at M = 8, K = 4096)
  static const int nw_env = getenv("ILLM_ARGMAX_NW") ? atoi(getenv("ILLM_ARGMAX_NW")) : 0;
  p.nw = nw_env == 4 || nw_env == 8 ? nw_env : (M > 2 ? 8 : 4);
  p.gx = (unsigned)((NT + p.nw - 1) / p.nw);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_argmax: x slice exceeds LDS");
  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.lut_fmt = (int)fmt;
  a.N = (int)n;
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  auto out_shape = xc.sizes().vec();
  out_shape.back() = n;
  Tensor out = at::empty(out_shape, xc.options());
  a.out = out.data_ptr();
  a.ldo = (int)n;
  a.bias = p16o(bias);
  const int64_t tg = p.nw / p.kw;
  const int64_t nparts = NT;                        // TPW = 1: one part per 16-column tile
  TORCH_CHECK((int64_t)p.gx * tg >= nparts, "gemv_argmax: geometry");
  Tensor parts = at::empty({nparts, M, 2}, xc.options().dtype(at::kFloat));
  a.amax = (float2*)parts.data_ptr<float>();
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_STORE, dim3(p.gx, 1), p.shmem, a);
  return {out, parts};
}

// prefill-size low-bit GEMM: MFMA with in-register dequant of the tiled weight
Tensor gemm(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, const c10::optional<Tensor>& bias) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda(), "gemm: GPU tensors expected");
  TORCH_CHECK(x.size(-1) == k, "gemm: x last dim ", x.size(-1), " != in_features ", k);
  TORCH_CHECK(k % 8 == 0, "gemm: in_features must be a multiple of 8");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemm: weight blob too small");
  auto shape = xc.sizes().vec();
  shape.back() = n;
  Tensor out = at::empty(shape, xc.options());
  if (M == 0) return out;
  illm::GemmArgs a{};
  // bf16 activations -> f16 once per call (the MFMA input type of the decoded weights)
  Tensor xh, xrs;
  if (bf16) {   // per-row power-of-two normalisation into f16 range (no saturation)
    const int64_t xr = xc.numel() / k;
    xh = at::empty(xc.sizes(), xc.options().dtype(at::kHalf));
    xrs = at::empty({xr}, xc.options().dtype(at::kFloat));
    illm::launch_x_to_f16_rowscale(true, p16(xc), xr, k, (int)k, m16(xh), xrs.data_ptr<float>(), cur_stream());
    a.x_f16 = 1;
    a.rs = xrs.data_ptr<float>();
  }
  a.x = bf16 ? p16(xh) : p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.N = (int)n;
  a.KC = (int)(illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K);
  a.bias = p16o(bias);
  a.out = m16(out);
  a.ldo = (int)n;
  a.lut_fmt = (int)fmt;
  illm::launch_lowbit_gemm(bf16, (int)fmt, a, cur_stream());
  return out;
}

// prefill GEMM over a tile-interleaved gate/up weight with the activation
// fused into the epilogue: returns act(x Wg^T) * (x Wu^T) [M, n / 2]
Tensor gemm_glu(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t act) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda(), "gemm_glu: GPU tensors expected");
  TORCH_CHECK(x.size(-1) == k && k % 8 == 0 && n % 32 == 0, "gemm_glu: shapes");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemm_glu: weight blob too small");
  auto shape = xc.sizes().vec();
  shape.back() = n / 2;
  Tensor out = at::empty(shape, xc.options());
  if (M == 0) return out;
  illm::GemmArgs a{};
  // bf16 activations -> f16 once per call (the MFMA input type of the decoded weights)
  Tensor xh, xrs;
  if (bf16) {   // per-row power-of-two normalisation into f16 range (no saturation)
    const int64_t xr = xc.numel() / k;
    xh = at::empty(xc.sizes(), xc.options().dtype(at::kHalf));
    xrs = at::empty({xr}, xc.options().dtype(at::kFloat));
    illm::launch_x_to_f16_rowscale(true, p16(xc), xr, k, (int)k, m16(xh), xrs.data_ptr<float>(), cur_stream());
    a.x_f16 = 1;
    a.rs = xrs.data_ptr<float>();
  }
  a.x = bf16 ? p16(xh) : p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.N = (int)n;
  a.KC = (int)(illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K);
  a.bias = nullptr;
  a.out = m16(out);
  a.ldo = (int)(n / 2);
  a.lut_fmt = (int)fmt;
  a.glu = 1;
  a.act = (int)act;
  illm::launch_lowbit_gemm(bf16, (int)fmt, a, cur_stream());
  return out;
}

// grouped ("FlashMoE") prefill GEMM over (token, expert) pairs sorted by
// expert (moe_align): ONE launch per projection for every local expert, the
// weights of expert e dequantized in registers from blob[e].  x rows are
// gathered by pair id / xdiv (x_sorted = false: the tokens) or taken in sorted
// order (x_sorted: the previous grouped GEMM's output); out rows are the
// sorted position (out_sorted) or the pair id.  Reference: the vLLM-XPU
// fused_moe over ipex-llm low-bit experts (vllm_for_multi_arc.patch:5933-6116)
// and the per-expert loops of models/qwen3_moe.py:70-105.
Tensor moe_gemm(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, const Tensor& off,
                const Tensor& rows, int64_t xdiv, bool x_sorted, bool out_sorted, bool glu, int64_t act,
                bool out_f32) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && off.is_cuda() && rows.is_cuda(), "moe_gemm: GPU tensors expected");
  TORCH_CHECK(blob.dim() == 2 && blob.scalar_type() == at::kByte, "moe_gemm: blob must be uint8 [E, bytes]");
  TORCH_CHECK(off.scalar_type() == at::kInt && rows.scalar_type() == at::kInt, "moe_gemm: int32 off / rows");
  TORCH_CHECK(x.size(-1) == k && k % 8 == 0, "moe_gemm: x last dim != in_features");
  TORCH_CHECK(!glu || n % 32 == 0, "moe_gemm: GLU weights need a multiple of 32 rows");
  const int64_t El = off.numel() - 1, P = rows.numel();
  TORCH_CHECK(El >= 1 && El <= 4096 && blob.size(0) == El, "moe_gemm: blob experts != off");
  TORCH_CHECK(blob.size(1) >= illm::dev_total_bytes((int)fmt, n, k), "moe_gemm: weight blob too small");
  TORCH_CHECK(xdiv >= 1, "moe_gemm: xdiv >= 1");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous().view({-1, k});
  TORCH_CHECK(!x_sorted || xc.size(0) >= P, "moe_gemm: sorted x needs a row per pair");
  const int64_t nout = glu ? n / 2 : n;
  Tensor out = at::empty({P, nout}, xc.options().dtype(out_f32 ? at::kFloat : xc.scalar_type()));
  if (P == 0) return out;
  illm::GemmArgs a{};
  Tensor xh, xrs;
  if (bf16) {   // per-row power-of-two normalisation into f16 range (no saturation)
    const int64_t xr = xc.numel() / k;
    xh = at::empty(xc.sizes(), xc.options().dtype(at::kHalf));
    xrs = at::empty({xr}, xc.options().dtype(at::kFloat));
    illm::launch_x_to_f16_rowscale(true, p16(xc), xr, k, (int)k, m16(xh), xrs.data_ptr<float>(), cur_stream());
    a.x_f16 = 1;
    a.rs = xrs.data_ptr<float>();
  }
  a.x = bf16 ? p16(xh) : p16(xc);
  a.M = (int)P;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.N = (int)n;
  a.KC = (int)(illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K);
  a.out = (uint16_t*)out.data_ptr();
  a.ldo = (int)nout;
  a.lut_fmt = (int)fmt;
  a.glu = glu ? 1 : 0;
  a.act = (int)act;
  a.moe_off = off.data_ptr<int32_t>();
  a.moe_rows = rows.data_ptr<int32_t>();
  a.moe_el = (int)El;
  a.moe_xdiv = (int)xdiv;
  a.moe_x_sorted = x_sorted ? 1 : 0;
  a.moe_out_sorted = out_sorted ? 1 : 0;
  a.w_stride = blob.size(1);
  a.out_f32 = out_f32 ? 1 : 0;
  TORCH_CHECK(!(glu && out_f32), "moe_gemm: the GLU epilogue writes activations (no f32 out)");
  illm::launch_lowbit_gemm(bf16, (int)fmt, a, cur_stream());
  return out;
}

// RWKV-4 WKV over [B, T, C] (f32 compute); num/den/max [B, C] f32 states updated in place
Tensor rwkv_wkv4(const Tensor& time_decay, const Tensor& time_first, const Tensor& k, const Tensor& v, Tensor& num,
                 Tensor& den, Tensor& mx) {
  TORCH_CHECK(k.is_cuda() && k.dim() == 3 && v.sizes() == k.sizes(), "rwkv_wkv4: k, v [B, T, C] on the GPU");
  c10::DeviceGuard g(k.device());
  const int64_t B = k.size(0), T = k.size(1), C = k.size(2);
  for (const Tensor* s : {&num, &den, &mx})
    TORCH_CHECK(s->scalar_type() == at::kFloat && s->is_contiguous() && s->numel() == B * C,
                "rwkv_wkv4: states must be contiguous f32 [B, C]");
  Tensor kf = k.to(at::kFloat).contiguous(), vf = v.to(at::kFloat).contiguous();
  Tensor w = time_decay.to(at::kFloat).contiguous(), u = time_first.to(at::kFloat).contiguous();
  TORCH_CHECK(w.numel() == C && u.numel() == C, "rwkv_wkv4: time_decay / time_first [C]");
  Tensor out = at::empty_like(kf);
  if (B * C > 0 && T > 0)
    illm::launch_rwkv4_wkv(w.data_ptr<float>(), u.data_ptr<float>(), kf.data_ptr<float>(), vf.data_ptr<float>(),
                           out.data_ptr<float>(), num.data_ptr<float>(), den.data_ptr<float>(), mx.data_ptr<float>(),
                           (int)B, (int)T, (int)C, cur_stream());
  return out.to(k.scalar_type());
}

// RWKV-5 WKV over r/k/v [B, T, H, S] (f32 compute); w = exp(-exp(time_decay)),
// u = time_first, both [H, S]; state [B, H, S, S] f32 updated in place
Tensor rwkv_wkv5(const Tensor& w, const Tensor& u, const Tensor& r, const Tensor& k, const Tensor& v, Tensor& state) {
  TORCH_CHECK(k.is_cuda() && k.dim() == 4 && r.sizes() == k.sizes() && v.sizes() == k.sizes(),
              "rwkv_wkv5: r, k, v [B, T, H, S] on the GPU");
  c10::DeviceGuard g(k.device());
  const int64_t B = k.size(0), T = k.size(1), H = k.size(2), S = k.size(3);
  TORCH_CHECK(S == 32 || S == 64 || S == 128, "rwkv_wkv5: head size must be 32, 64 or 128");
  TORCH_CHECK(state.scalar_type() == at::kFloat && state.is_contiguous() && state.dim() == 4 &&
                  state.size(0) == B && state.size(1) == H && state.size(2) == S && state.size(3) == S,
              "rwkv_wkv5: state must be contiguous f32 [B, H, S, S]");
  Tensor rf = r.to(at::kFloat).contiguous(), kf = k.to(at::kFloat).contiguous(), vf = v.to(at::kFloat).contiguous();
  Tensor wf = w.to(at::kFloat).contiguous(), uf = u.to(at::kFloat).contiguous();
  TORCH_CHECK(wf.numel() == H * S && uf.numel() == H * S, "rwkv_wkv5: w / u [H, S]");
  Tensor out = at::empty_like(kf);
  if (B * H > 0 && T > 0)
    illm::launch_rwkv5_wkv(wf.data_ptr<float>(), uf.data_ptr<float>(), rf.data_ptr<float>(), kf.data_ptr<float>(),
                           vf.data_ptr<float>(), out.data_ptr<float>(), state.data_ptr<float>(), (int)B, (int)T,
                           (int)H, (int)S, cur_stream());
  return out;
}

// split-K GEMV accumulated with f32 atomics into acc [M, n] (zero on entry;
// the consumer -- add_rms_norm / rope_kv_fused with zero_*=True -- reads the
// single slab and re-zeroes it, so no ks-slab reduction is ever needed)
// RoPE in the atomic GEMV epilogue (GemvArgs rcs): cos/sin table f32
// [max_pos, D / 2, 2], positions int64 [M]; the plan must give head-aligned
// 8-wave column blocks (128 columns: D in {64, 128})
static bool set_rope(illm::GemvArgs& a, const c10::optional<Tensor>& cs, const c10::optional<Tensor>& pos,
                     int64_t cols, int64_t D, int64_t M) {
  if (!cs.has_value() || !cs->defined()) return false;
  TORCH_CHECK(cs->is_cuda() && cs->scalar_type() == at::kFloat && cs->is_contiguous() && cs->dim() == 3 &&
                  cs->size(1) * 2 == D && (D == 64 || D == 128),
              "gemv rope: f32 cos/sin table [max_pos, D/2, 2] with D in {64, 128}");
  TORCH_CHECK(pos.has_value() && pos->defined() && pos->scalar_type() == at::kLong && pos->numel() >= M,
              "gemv rope: int64 positions [M]");
  TORCH_CHECK(cols % D == 0 && cols <= a.N, "gemv rope: rotated columns must be whole heads");
  a.rcs = cs->data_ptr<float>();
  a.rpos = pos->data_ptr<int64_t>();
  a.rcols = (int)cols;
  a.rD = (int)D;
  return true;
}

static void set_zero(illm::GemvArgs& a, const c10::optional<Tensor>& zero) {
  if (zero.has_value() && zero->defined()) {
    TORCH_CHECK(zero->is_cuda() && zero->scalar_type() == at::kFloat && zero->is_contiguous() &&
                    zero->numel() % 4 == 0, "zero: contiguous f32 buffer with a multiple of 4 elements");
    a.nzero = zero->data_ptr<float>();
    a.nzero_n = (int)zero->numel();
  }
}

// Decode projection whose input is rms_norm(residual + acc_in) * w, computed in
// the GEMV prologue (no standalone norm launch).  acc_in: the previous
// projection's atomic accumulator [M, k] f32 (read only; the caller zeroes it
// through a later launch's `zero`), residual -> res_out (= residual + acc_in,
// written once).  epi: EPI_ATOMIC (out = acc_out [M, n] f32, zero on entry) or
// EPI_GLU (returns act(gate) * up [M, n / 2] in dt).
Tensor gemv_norm_in(const Tensor& acc_in, const Tensor& residual, Tensor& res_out, const Tensor& norm_w, double eps,
                    bool unit_offset, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t epi,
                    int64_t act, const c10::optional<Tensor>& acc_out, const c10::optional<Tensor>& zero,
                    const c10::optional<Tensor>& ss, const c10::optional<Tensor>& rope_cs,
                    const c10::optional<Tensor>& rope_pos, int64_t rope_cols, int64_t rope_d) {
  TORCH_CHECK(acc_in.is_cuda() && blob.is_cuda() && residual.is_cuda(), "gemv_norm_in: GPU tensors expected");
  c10::DeviceGuard g(acc_in.device());
  const bool bf16 = is_bf16(residual);
  const int64_t M = residual.numel() / k;
  TORCH_CHECK(M >= 1 && M <= 16, "gemv_norm_in handles 1..16 rows, got ", M);
  TORCH_CHECK(k % 8 == 0 && norm_w.numel() == k && residual.is_contiguous() && res_out.is_contiguous() &&
                  res_out.numel() == M * k && residual.scalar_type() == res_out.scalar_type() &&
                  norm_w.scalar_type() == residual.scalar_type(),
              "gemv_norm_in: residual/res_out [M, k] and norm weight [k] of one 16-bit dtype");
  TORCH_CHECK(acc_in.scalar_type() == at::kFloat && acc_in.is_contiguous() && acc_in.numel() == M * k,
              "gemv_norm_in: acc_in must be contiguous f32 [M, k]");
  TORCH_CHECK(res_out.data_ptr() != residual.data_ptr(), "gemv_norm_in: res_out must not alias residual");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_norm_in: weight blob too small");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  illm::GemvArgs a{};
  a.x = nullptr;
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.act = (int)act;
  a.lut_fmt = (int)fmt;
  a.nacc = acc_in.data_ptr<float>();
  a.nres = p16(residual);
  a.nres_out = m16(res_out);
  a.nweight = p16(norm_w);
  a.neps = (float)eps;
  a.nunit = unit_offset ? 1 : 0;
  set_zero(a, zero);
  if (ss.has_value() && ss->defined()) {
    // deferred norm: the row scales are applied by the consumer (split-K
    // atomic output: ss [M] f32 zeroed on entry gets the sum of squares) or
    // by the GLU epilogue itself
    TORCH_CHECK(ss->is_cuda() && ss->scalar_type() == at::kFloat && ss->is_contiguous() && ss->numel() >= M,
                "gemv_norm_in: ss must be contiguous f32 [>= M]");
    a.ndefer = 1;
    a.nss = ss->data_ptr<float>();
  }
  if (epi == illm::EPI_GLU) {
    TORCH_CHECK(n % 32 == 0, "GLU weights must have a multiple of 32 rows");
    Tensor out = at::empty({M, n / 2}, residual.options());
    a.N = (int)(n / 2);
    a.out = out.data_ptr();
    a.ldo = (int)(n / 2);
    const Plan5 p = plan5(M, NT / 2, KC, false);
    TORCH_CHECK(p.shmem <= kMaxLds, "gemv_norm_in: K slice too large for LDS");
    a.nw = p.nw;
    launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_GLU, dim3(p.gx, 1), p.shmem, a);
    return out;
  }
  TORCH_CHECK(epi == illm::EPI_ATOMIC && acc_out.has_value() && acc_out->defined() &&
                  acc_out->scalar_type() == at::kFloat && acc_out->is_contiguous() && acc_out->numel() == M * n,
              "gemv_norm_in: EPI_ATOMIC needs acc_out, contiguous f32 [M, n]");
  a.N = (int)n;
  a.out = acc_out->data_ptr();
  a.ldo = (int)n;
  const bool rope = set_rope(a, rope_cs, rope_pos, rope_cols, rope_d, M);
  Plan5 p = plan5(M, NT, KC, true, 0, true);
  if (rope) p = plan5_rope(p, NT, M);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_norm_in: K slice too large for LDS");
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_ATOMIC, dim3(p.gx, (unsigned)p.ks), p.shmem, a);
  return *acc_out;
}

void gemv_accum(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, Tensor& acc,
                int64_t ksplit, const c10::optional<Tensor>& zero, const c10::optional<Tensor>& rope_cs,
                const c10::optional<Tensor>& rope_pos, int64_t rope_cols, int64_t rope_d) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && acc.is_cuda(), "gemv_accum: GPU tensors expected");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(M >= 1 && M <= 16, "gemv_accum handles 1..16 rows, got ", M);
  TORCH_CHECK(acc.scalar_type() == at::kFloat && acc.is_contiguous() && acc.numel() == M * n,
              "gemv_accum: acc must be contiguous f32 [M, n]");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_accum: weight blob too small");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.lut_fmt = (int)fmt;
  a.N = (int)n;
  a.out = acc.data_ptr();
  a.ldo = (int)n;
  const bool rope = set_rope(a, rope_cs, rope_pos, rope_cols, rope_d, M);
  Plan5 p = plan5(M, NT, KC, true, ksplit, true);
  if (rope) p = plan5_rope(p, NT, M);
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  set_zero(a, zero);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_accum: K slice too large for LDS");
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_ATOMIC, dim3(p.gx, (unsigned)p.ks), p.shmem, a);
}

// gemv_accum whose last-arriving split-K workgroup per column block also does
// the residual add and the deferred RMSNorm staging of the next GEMV's input
// (lowbit_gemv5.cuh gemv5_norm_out): res_out = rnd(rnd(acc) + residual),
// xo = rnd(w * res_out), ss[m] += sum of res_out[m]^2, acc re-zeroed.
// ctr: int32 [>= column blocks], zero on the first call (self-resetting).
void gemv_accum_norm(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, Tensor& acc,
                     Tensor& ctr, const Tensor& residual, Tensor& res_out, const Tensor& norm_w, bool unit_offset,
                     Tensor& xo, Tensor& ss, const c10::optional<Tensor>& zero) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && acc.is_cuda(), "gemv_accum_norm: GPU tensors expected");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(M >= 1 && M <= 16, "gemv_accum_norm handles 1..16 rows, got ", M);
  TORCH_CHECK(n % 4 == 0, "gemv_accum_norm: n must be a multiple of 4");
  TORCH_CHECK(acc.scalar_type() == at::kFloat && acc.is_contiguous() && acc.numel() == M * n,
              "gemv_accum_norm: acc must be contiguous f32 [M, n]");
  TORCH_CHECK(residual.is_contiguous() && res_out.is_contiguous() && xo.is_contiguous() &&
                  residual.numel() == M * n && res_out.numel() == M * n && xo.numel() == M * n &&
                  residual.scalar_type() == x.scalar_type() && res_out.scalar_type() == x.scalar_type() &&
                  xo.scalar_type() == x.scalar_type() && norm_w.scalar_type() == x.scalar_type() &&
                  norm_w.numel() == n && norm_w.is_contiguous(),
              "gemv_accum_norm: residual / res_out / xo [M, n] and norm weight [n] in x's dtype");
  TORCH_CHECK(res_out.data_ptr() != residual.data_ptr(), "gemv_accum_norm: res_out must not alias residual");
  TORCH_CHECK(ss.scalar_type() == at::kFloat && ss.is_contiguous() && ss.numel() >= M, "gemv_accum_norm: ss f32 [>= M]");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_accum_norm: weight blob too small");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.lut_fmt = (int)fmt;
  a.N = (int)n;
  a.out = acc.data_ptr();
  a.ldo = (int)n;
  Plan5 p = plan5(M, NT, KC, true, 0, true);
  p.kw = 1;                                   // column blocks of nw tiles: 64 / 128 columns
  p.gx = (unsigned)((NT + p.nw - 1) / p.nw);
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  set_zero(a, zero);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_accum_norm: K slice too large for LDS");
  TORCH_CHECK(ctr.scalar_type() == at::kInt && ctr.is_contiguous() && ctr.numel() >= (int64_t)p.gx,
              "gemv_accum_norm: ctr int32 [>= ", p.gx, "]");
  a.lctr = ctr.data_ptr<int>();
  a.lres = p16(residual);
  a.lres_out = m16(res_out);
  a.lnw = p16(norm_w);
  a.lxo = m16(xo);
  a.lss = ss.data_ptr<float>();
  a.lunit = unit_offset ? 1 : 0;
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_ATOMIC, dim3(p.gx, (unsigned)p.ks), p.shmem, a);
}

// gate/up GLU GEMV over a deferred-norm input (gemv_accum_norm's xo): the row
// scale rsqrt(ss[m] / ss_n + eps) is applied to gate and up before the activation
Tensor gemv_glu_ss(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t act,
                   const Tensor& ss, int64_t ss_n, double eps) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && x.size(-1) == k, "gemv_glu_ss: GPU x [M, k]");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  TORCH_CHECK(M >= 1 && M <= 16 && n % 32 == 0, "gemv_glu_ss: 1..16 rows, n a multiple of 32");
  TORCH_CHECK(ss.is_cuda() && ss.scalar_type() == at::kFloat && ss.numel() >= M, "gemv_glu_ss: ss f32 [>= M]");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_glu_ss: weight blob too small");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.act = (int)act;
  a.lut_fmt = (int)fmt;
  a.xpss = ss.data_ptr<float>();
  a.xpss_n = (int)ss_n;
  a.xpss_eps = (float)eps;
  Tensor out = at::empty({M, n / 2}, xc.options());
  a.N = (int)(n / 2);
  a.out = out.data_ptr();
  a.ldo = (int)(n / 2);
  const Plan5 p = plan5(M, NT / 2, KC, false);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_glu_ss: x slice exceeds LDS");
  a.nw = p.nw;
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_GLU, dim3(p.gx, 1), p.shmem, a);
  return out;
}

// down-projection GEMV whose input is act(gate) * up computed on the fly from
// the gate/up GEMV's split-K slabs or atomic accumulator (saves the GLU
// epilogue's unsplittable launch and one [M, I] round trip); returns f32
// partial slabs [ks, M, n], or accumulates atomically into ``acc`` [M, n].
Tensor gemv_glu_in(const Tensor& part, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t act,
                   int64_t ksplit, at::ScalarType dt, const c10::optional<Tensor>& acc,
                   const c10::optional<Tensor>& zero, const c10::optional<Tensor>& xss, int64_t xss_n,
                   double xss_eps) {
  TORCH_CHECK(part.is_cuda() && blob.is_cuda() && part.dim() == 3 && part.scalar_type() == at::kFloat &&
              part.is_contiguous(), "gemv_glu_in: part must be contiguous f32 [ns, M, 2k] on the GPU");
  TORCH_CHECK(part.size(2) == 2 * k && k % 16 == 0, "gemv_glu_in: part width must be 2 * k");
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf, "gemv_glu_in: bf16/fp16 activations");
  c10::DeviceGuard g(part.device());
  const bool bf16 = dt == at::kBFloat16;
  const int64_t M = part.size(1);
  TORCH_CHECK(M >= 1 && M <= 16, "gemv_glu_in handles 1..16 rows");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_glu_in: weight blob too small");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  illm::GemvArgs a{};
  a.x = nullptr;
  a.xpart = part.data_ptr<float>();
  a.xpart_ns = (int)part.size(0);
  if (xss.has_value() && xss->defined()) {
    TORCH_CHECK(xss->is_cuda() && xss->scalar_type() == at::kFloat && xss_n > 0,
                "gemv_glu_in: xss must be f32 [M] with xss_n > 0");
    a.xpss = xss->data_ptr<float>();
    a.xpss_n = (int)xss_n;
    a.xpss_eps = (float)xss_eps;
  }
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.act = (int)act;
  a.lut_fmt = (int)fmt;
  a.N = (int)n;
  const bool atomic = acc.has_value() && acc->defined();
  const Plan5 p = plan5(M, NT, KC, true, ksplit, atomic);
  ksplit = p.ks;
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  set_zero(a, zero);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_glu_in: K slice too large for LDS");
  if (atomic) {
    TORCH_CHECK(acc->scalar_type() == at::kFloat && acc->is_contiguous() && acc->numel() == M * n,
                "gemv_glu_in: acc must be contiguous f32 [M, n]");
    a.out = acc->data_ptr();
    a.ldo = (int)n;
    launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_ATOMIC, dim3(p.gx, (unsigned)ksplit), p.shmem, a);
    return *acc;
  }
  Tensor ws = at::empty({ksplit, M, n}, part.options());
  a.out = ws.data_ptr();
  a.ldo = (int)n;
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_PARTIAL, dim3(p.gx, (unsigned)ksplit), p.shmem, a);
  return ws;
}

Tensor add_rms_norm(const c10::optional<Tensor>& x, const c10::optional<Tensor>& partials,
                    const c10::optional<Tensor>& residual, const Tensor& w, double eps,
                    bool unit_offset, bool store_residual, bool zero_partials) {
  c10::DeviceGuard g(w.device());
  const bool bf16 = is_bf16(w);
  const int64_t H = w.numel();
  TORCH_CHECK(H % 8 == 0 && H <= 8 * 256 * 8, "rms_norm hidden size must be a multiple of 8 and <= 16384");
  illm::NormArgs a{};
  int64_t M;
  std::vector<int64_t> shape;
  if (partials.has_value() && partials->defined()) {
    TORCH_CHECK(partials->dim() == 3 && partials->size(2) == H, "partials must be [ks, M, H]");
    a.partials = partials->data_ptr<float>();
    a.nsplit = (int)partials->size(0);
    M = partials->size(1);
    shape = {M, H};
    if (residual.has_value() && residual->defined()) shape = residual->sizes().vec();
  } else {
    TORCH_CHECK(x.has_value() && x->defined(), "add_rms_norm needs x or partials");
    TORCH_CHECK(x->is_contiguous(), "x must be contiguous");
    a.x = p16(*x);
    M = x->numel() / H;
    shape = x->sizes().vec();
  }
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->is_contiguous() && residual->numel() == M * H, "residual shape mismatch");
    a.residual = (uint16_t*)residual->data_ptr();
  }
  Tensor out = at::empty(shape, w.options());
  a.w = p16(w);
  a.out = m16(out);
  a.M = (int)M;
  a.H = (int)H;
  a.eps = (float)eps;
  a.unit_offset = unit_offset;
  a.store_residual = store_residual;
  a.zero_partials = zero_partials && a.partials != nullptr;
  if (M > 0) illm::launch_add_rms_norm(bf16, a, cur_stream());
  return out;
}

// decode-step entry: embedding gather + RMSNorm of the first layer in one
// launch (the gathered rows are the residual stream), optionally zeroing an
// f32 buffer (the step's deferred-norm sums of squares): replaces the
// embedding gather, the Fill and the first norm launch
std::tuple<Tensor, Tensor> embed_rms_norm(const Tensor& ids, const Tensor& table, const Tensor& w, double eps,
                                          bool unit_offset, const c10::optional<Tensor>& zero) {
  c10::DeviceGuard g(w.device());
  const bool bf16 = is_bf16(w);
  const int64_t H = w.numel();
  TORCH_CHECK(H % 8 == 0 && H <= 8 * 256 * 8, "embed_rms_norm: hidden size must be a multiple of 8, <= 16384");
  TORCH_CHECK(table.dim() == 2 && table.size(1) == H && table.is_contiguous() &&
                  table.scalar_type() == w.scalar_type(), "embed_rms_norm: table [V, H] in the weight dtype");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous() && ids.is_cuda(), "embed_rms_norm: int64 ids");
  const int64_t M = ids.numel();
  Tensor res = at::empty({M, H}, w.options());
  Tensor out = at::empty({M, H}, w.options());
  illm::NormArgs a{};
  a.x = p16(table);
  a.w = p16(w);
  a.out = m16(out);
  a.M = (int)M;
  a.H = (int)H;
  a.eps = (float)eps;
  a.unit_offset = unit_offset;
  a.ids = ids.data_ptr<int64_t>();
  a.vocab = table.size(0);
  a.gather_out = m16(res);
  a.err = kernel_err(w.device());
  if (zero.has_value() && zero->defined()) {
    TORCH_CHECK(zero->scalar_type() == at::kFloat && zero->is_contiguous() && zero->is_cuda(), "zero: f32");
    a.zero = zero->data_ptr<float>();
    a.zero_n = (int)zero->numel();
  }
  if (M > 0) illm::launch_add_rms_norm(bf16, a, cur_stream());
  return {res, out};
}

// act(gate) * up (dy undefined) or its gradient (dgate, dup) for contiguous same-shape tensors
std::vector<Tensor> act_mul(const Tensor& g, const Tensor& u, const c10::optional<Tensor>& dy, int64_t act) {
  c10::DeviceGuard dg_(g.device());
  TORCH_CHECK(g.is_contiguous() && u.is_contiguous() && g.sizes() == u.sizes() && g.scalar_type() == u.scalar_type() &&
                  (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kHalf) && g.numel() % 8 == 0,
              "act_mul: contiguous bf16/f16 gate and up of one shape, numel % 8 == 0");
  const bool bf16 = is_bf16(g);
  if (!(dy.has_value() && dy->defined())) {
    Tensor y = at::empty_like(g);
    illm::launch_act_mul(bf16, p16(g), p16(u), nullptr, m16(y), nullptr, nullptr, g.numel(), (int)act, cur_stream());
    return {y};
  }
  TORCH_CHECK(dy->is_contiguous() && dy->sizes() == g.sizes() && dy->scalar_type() == g.scalar_type(),
              "act_mul: dy like gate");
  Tensor dgt = at::empty_like(g), dut = at::empty_like(u);
  illm::launch_act_mul(bf16, p16(g), p16(u), p16(*dy), nullptr, m16(dgt), m16(dut), g.numel(), (int)act,
                       cur_stream());
  return {dgt, dut};
}

// rotate-half RoPE of a [B, H, T, D] view (D contiguous) -> contiguous [B, H, T, D]
Tensor rope_half(const Tensor& x, const Tensor& cos, const Tensor& sin, bool bwd) {
  c10::DeviceGuard dg(x.device());
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "rope_half: x [B, H, T, D] with contiguous D");
  const int64_t B = x.size(0), H = x.size(1), Tn = x.size(2), D = x.size(3);
  TORCH_CHECK(D % 8 == 0, "rope_half: head dim multiple of 8");
  TORCH_CHECK(cos.dim() == 3 && cos.is_contiguous() && sin.is_contiguous() && cos.sizes() == sin.sizes() &&
                  cos.size(1) == Tn && cos.size(2) == D && (cos.size(0) == B || cos.size(0) == 1),
              "rope_half: cos / sin [B or 1, T, D] contiguous");
  TORCH_CHECK(x.scalar_type() == cos.scalar_type() && x.scalar_type() == sin.scalar_type() &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "rope_half: bf16/f16 x, cos, sin");
  TORCH_CHECK(x.stride(0) % 4 == 0 && x.stride(1) % 4 == 0 && x.stride(2) % 4 == 0, "rope_half: 8-B aligned rows");
  Tensor out = at::empty({B, H, Tn, D}, x.options());
  if (out.numel() > 0)
    illm::launch_rope_half(is_bf16(x), (const uint16_t*)x.data_ptr(), x.stride(0), x.stride(1), x.stride(2),
                           p16(cos), p16(sin), cos.size(0) == 1 ? 0 : Tn * D, m16(out), (int)B, (int)H, (int)Tn,
                           (int)D, bwd ? 1 : 0, cur_stream());
  return out;
}

// gradient of rms_norm(x) * w w.r.t. x (frozen w), HF rounding
Tensor rms_norm_bwd(const Tensor& x, const Tensor& g, const Tensor& w, double eps, bool unit_offset) {
  c10::DeviceGuard dg(x.device());
  const int64_t H = w.numel();
  TORCH_CHECK(x.is_contiguous() && g.is_contiguous() && x.numel() == g.numel() && x.numel() % H == 0,
              "rms_norm_bwd: contiguous x and grad of one shape");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && g.scalar_type() == w.scalar_type() &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "rms_norm_bwd: bf16/f16 x, grad and weight");
  TORCH_CHECK(H % 8 == 0 && H <= 8 * 512 * 8, "rms_norm_bwd: hidden size multiple of 8, <= 32768");
  Tensor dx = at::empty_like(x);
  const int64_t M = x.numel() / H;
  if (M > 0)
    illm::launch_rms_norm_bwd(is_bf16(x), p16(x), p16(g), p16(w), m16(dx), (int)M, (int)H, (float)eps, unit_offset,
                              cur_stream());
  return dx;
}

Tensor layer_norm(const Tensor& x, const c10::optional<Tensor>& w, const c10::optional<Tensor>& b,
                  double eps) {
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  const int64_t H = xc.size(-1), M = xc.numel() / H;
  TORCH_CHECK(H % 8 == 0 && H <= 16384, "layer_norm hidden size must be a multiple of 8");
  Tensor out = at::empty_like(xc);
  if (M > 0) illm::launch_layer_norm(bf16, p16(xc), p16o(w), p16o(b), m16(out), (int)M, (int)H, (float)eps, cur_stream());
  return out;
}

void rope_kv(const Tensor& qkv, Tensor& q_out, Tensor& k_cache, Tensor& v_cache, const Tensor& slots,
             const Tensor& pos, const Tensor& inv_freq, const c10::optional<Tensor>& q_norm,
             const c10::optional<Tensor>& k_norm, double norm_eps, double q_scale, int64_t Hq,
             int64_t Hkv, int64_t D, int64_t rot_dim, bool interleaved, int64_t kv_fp8,
             double k_scale, double v_scale) {
  c10::DeviceGuard g(qkv.device());
  const bool bf16 = is_bf16(qkv);
  TORCH_CHECK(qkv.stride(-1) == 1, "qkv last dim must be contiguous");
  const int64_t T = qkv.numel() / qkv.size(-1);
  TORCH_CHECK(slots.scalar_type() == at::kLong && pos.scalar_type() == at::kLong, "slots/pos int64");
  TORCH_CHECK(inv_freq.scalar_type() == at::kFloat, "inv_freq must be f32");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D, "k_cache must be [nblocks, Hkv, bs, D]");
  illm::RopeKVArgs a{};
  a.qkv = p16(qkv);
  a.ld_qkv = (int)qkv.size(-1);
  a.q_out = m16(q_out);
  a.k_cache = (uint8_t*)k_cache.data_ptr();
  a.v_cache = (uint8_t*)v_cache.data_ptr();
  a.slots = slots.data_ptr<int64_t>();
  a.pos = pos.data_ptr<int64_t>();
  if (inv_freq.dim() == 3) {
    TORCH_CHECK(inv_freq.size(1) == rot_dim / 2 && inv_freq.size(2) == 2, "cos_sin table must be [P, rot/2, 2]");
    a.cos_sin = inv_freq.data_ptr<float>();
  } else {
    a.inv_freq = inv_freq.data_ptr<float>();
  }
  a.q_norm = p16o(q_norm);
  a.k_norm = p16o(k_norm);
  a.norm_eps = (float)norm_eps;
  a.attn_scale_q = (float)q_scale;
  a.T = (int)T;
  a.Hq = (int)Hq;
  a.Hkv = (int)Hkv;
  a.D = (int)D;
  a.rot_dim = (int)rot_dim;
  a.bs = (int)k_cache.size(2);
  a.interleaved = interleaved;
  a.kv_fp8 = (int)kv_fp8;
  a.k_scale = (float)k_scale;
  a.v_scale = (float)v_scale;
  a.num_blocks = (int)k_cache.size(0);
  a.err = kernel_err(qkv.device());
  if (T > 0) illm::launch_rope_kv(bf16, a, cur_stream());
}

// Zeroed per-device arrival counters for the fused attention combine.  The
// buffer is allocated once (outside any graph capture: the first eager call
// of a shape allocates it) and every merging block resets its counter, so the
// same pointer is valid across hipGraph replays.
// in-kernel merge of the split partials by the last-arriving split of each
// (batch, kv head), handed over with write-through stores + one agent-scope
// atomic (no combine launch).  Opt-in (ILLM_ATTN_FUSED_COMBINE=1): correct,
// but ONE wave merging R rows x D dims over all splits is a serial tail longer
// than the parallel combine launch it replaces (MI355X, Llama-3-8B, L = 1024:
// batch 1 1.988 -> 2.158 ms/token, batch 8 2.407 -> 2.725 ms/step).
static bool fused_combine_on() {
  static const bool on = [] {
    const char* e = getenv("ILLM_ATTN_FUSED_COMBINE");
    return e != nullptr && atoi(e) != 0;
  }();
  return on;
}

// Per-device kernel error word (illm_device.h kerr): allocated on first use
// (outside graph capture, like the combine counters), read and reset by the
// kernel_errors op (ops.check_kernel_errors).
static at::Tensor& kernel_err_buf(const c10::Device& dev) {
  static std::map<int, at::Tensor> bufs;
  auto it = bufs.find(dev.index());
  if (it == bufs.end())
    it = bufs.emplace(dev.index(), at::zeros({4}, at::TensorOptions().dtype(at::kInt).device(dev))).first;
  return it->second;
}
int* kernel_err(const c10::Device& dev) { return kernel_err_buf(dev).data_ptr<int>(); }

Tensor kernel_errors(const Tensor& like, bool reset) {
  c10::DeviceGuard g(like.device());
  at::Tensor& b = kernel_err_buf(like.device());
  Tensor out = b.clone();
  if (reset) b.zero_();
  return out;
}

// v3 decode attention (attn_dec_v3.cuh): the last-arriving split workgroup of
// each (batch, kv head) merges the partials in-kernel (its own counter buffer:
// the v2 fused combine keeps ILLM_ATTN_FUSED_COMBINE).  Default on: MI355X,
// Llama-3-8B at 1 K keys, per layer from cold caches (profiles/attn_dec_v3_r5.jsonl):
// batch 1 9.42 vs 10.29 us with the combine launch, batch 8 18.50 vs 18.57;
// ILLM_ATTN_V3_FUSE=0 keeps the combine launch
static bool v3_fuse_on() {
  static const bool on = [] {
    const char* e = getenv("ILLM_ATTN_V3_FUSE");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}
int* attn_counters(const c10::Device& dev, int64_t n);
static int* v3_counters(const c10::Device& dev, int64_t n) {
  static std::vector<Tensor> bufs(64);
  const int idx = dev.index() < 0 ? 0 : dev.index();
  constexpr int64_t kCap = 1 << 16;
  if (n > kCap) return nullptr;
  if (!bufs[idx].defined()) bufs[idx] = at::zeros({kCap}, at::TensorOptions().device(dev).dtype(at::kInt));
  return bufs[idx].data_ptr<int>();
}

int* attn_counters(const c10::Device& dev, int64_t n) {
  static std::vector<Tensor> bufs(64);
  const int idx = dev.index() < 0 ? 0 : dev.index();
  constexpr int64_t kCap = 1 << 16;
  if (n > kCap) return nullptr;
  if (!bufs[idx].defined()) {
    bufs[idx] = at::zeros({kCap}, at::TensorOptions().device(dev).dtype(at::kInt));
  }
  return bufs[idx].data_ptr<int>();
}

void rope_kv_fused(const Tensor& part, const c10::optional<Tensor>& bias, Tensor& q_out, Tensor& k_cache,
                   Tensor& v_cache, const Tensor& pos, const Tensor& block_tables, int64_t tq, const Tensor& inv_freq,
                   const c10::optional<Tensor>& q_norm, const c10::optional<Tensor>& k_norm, double norm_eps,
                   double q_scale, int64_t Hq, int64_t Hkv, int64_t D, int64_t rot_dim, bool interleaved,
                   int64_t kv_fp8, double k_scale, double v_scale, const c10::optional<Tensor>& pos_offset,
                   bool zero_part, const c10::optional<Tensor>& pss, int64_t pss_n, double pss_eps) {
  c10::DeviceGuard g(part.device());
  const bool bf16 = is_bf16(q_out);
  TORCH_CHECK(part.dim() == 3 && part.scalar_type() == at::kFloat && part.is_contiguous(),
              "rope_kv_fused: part must be contiguous f32 [ks, T, N]");
  TORCH_CHECK(part.size(2) == (Hq + 2 * Hkv) * D, "rope_kv_fused: N != (Hq + 2 Hkv) * D");
  TORCH_CHECK(pos.scalar_type() == at::kLong && block_tables.scalar_type() == at::kInt, "pos int64, block_tables int32");
  TORCH_CHECK(inv_freq.scalar_type() == at::kFloat, "inv_freq / cos_sin must be f32");
  illm::RopeKVArgs a{};
  a.part = part.data_ptr<float>();
  a.nsplit = (int)part.size(0);
  a.zero_part = zero_part ? 1 : 0;
  TORCH_CHECK(!zero_part || a.nsplit == 1, "rope_kv_fused: zero_part needs a single accumulator slab");
  a.bias = p16o(bias);
  a.ld_qkv = (int)part.size(2);
  a.q_out = m16(q_out);
  a.k_cache = (uint8_t*)k_cache.data_ptr();
  a.v_cache = (uint8_t*)v_cache.data_ptr();
  a.slots = nullptr;
  a.block_tables = block_tables.data_ptr<int32_t>();
  a.max_blocks = (int)block_tables.size(1);
  a.tq = (int)tq;
  a.pos_offset = (pos_offset.has_value() && pos_offset->defined()) ? pos_offset->data_ptr<int64_t>() : nullptr;
  a.pos = pos.data_ptr<int64_t>();
  if (inv_freq.dim() == 3) a.cos_sin = inv_freq.data_ptr<float>();
  else a.inv_freq = inv_freq.data_ptr<float>();
  a.q_norm = p16o(q_norm);
  a.k_norm = p16o(k_norm);
  a.norm_eps = (float)norm_eps;
  a.attn_scale_q = (float)q_scale;
  a.T = (int)part.size(1);
  a.Hq = (int)Hq;
  a.Hkv = (int)Hkv;
  a.D = (int)D;
  a.rot_dim = (int)rot_dim;
  a.bs = (int)k_cache.size(2);
  a.interleaved = interleaved;
  a.kv_fp8 = (int)kv_fp8;
  a.k_scale = (float)k_scale;
  a.v_scale = (float)v_scale;
  a.num_blocks = (int)k_cache.size(0);
  a.err = kernel_err(part.device());
  if (pss.has_value() && pss->defined()) {
    TORCH_CHECK(pss->is_cuda() && pss->scalar_type() == at::kFloat && pss->numel() >= a.T && pss_n > 0,
                "rope_kv_fused: pss must be f32 [T] with pss_n > 0");
    a.pss = pss->data_ptr<float>();
    a.pss_n = (int)pss_n;
    a.pss_eps = (float)pss_eps;
  }
  if (a.T > 0) illm::launch_rope_kv(bf16, a, cur_stream());
}

static std::tuple<Tensor, Tensor, Tensor> attn_decode_impl(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                   const Tensor& seq_lens, int64_t nsplit, double scale, double softcap, int64_t window,
                   int64_t kv_fp8, double k_scale, double v_scale, const c10::optional<Tensor>& alibi,
                   bool no_combine) {
  c10::DeviceGuard g(q.device());
  const bool bf16 = is_bf16(q);
  TORCH_CHECK(q.dim() == 4 && q.is_contiguous(), "q must be contiguous [B, Tq, Hq, D]");
  const int64_t B = q.size(0), Tq = q.size(1), Hq = q.size(2), D = q.size(3);
  const int64_t Hkv = k_cache.size(1), bs = k_cache.size(2);
  TORCH_CHECK(Hq % Hkv == 0 && (Hq / Hkv) * Tq <= 16, "attn_decode: (Hq/Hkv)*Tq must be <= 16");
  TORCH_CHECK(bs % 64 == 0, "KV block size must be a multiple of 64");
  TORCH_CHECK(D == 64 || D == 80 || D == 96 || D == 128 || D == 256, "unsupported head_dim ", D);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_lens.scalar_type() == at::kInt, "int32 tables");
  illm::AttnDecodeArgs a{};
  Tensor po = at::empty({B, Hq, Tq, nsplit, D}, q.options().dtype(at::kFloat));
  Tensor pml = at::empty({B, Hq, Tq, nsplit, 2}, q.options().dtype(at::kFloat));
  Tensor out = at::empty_like(q);
  a.q = p16(q);
  a.k_cache = (const uint8_t*)k_cache.data_ptr();
  a.v_cache = (const uint8_t*)v_cache.data_ptr();
  a.block_tables = block_tables.data_ptr<int32_t>();
  a.seq_lens = seq_lens.data_ptr<int32_t>();
  a.max_blocks = (int)block_tables.size(1);
  a.num_blocks = (int)k_cache.size(0);
  a.err = kernel_err(k_cache.device());
  a.part_o = po.data_ptr<float>();
  a.part_ml = pml.data_ptr<float>();
  a.out = m16(out);
  a.B = (int)B;
  a.Tq = (int)Tq;
  a.Hq = (int)Hq;
  a.Hkv = (int)Hkv;
  a.D = (int)D;
  a.bs = (int)bs;
  TORCH_CHECK(nsplit >= 1 && nsplit <= kMaxDecodeSplits && (nsplit <= 1024 || D % 4 == 0),
              "attn_decode: nsplit must be 1..", kMaxDecodeSplits, " (1..1024 when D % 4 != 0; combine LDS), got ", nsplit);
  a.nsplit = (int)nsplit;
  a.scale = (float)scale;
  a.softcap = (float)softcap;
  a.sliding_window = (int)window;
  a.kv_fp8 = (int)kv_fp8;
  a.k_scale = (float)k_scale;
  a.v_scale = (float)v_scale;
  if (alibi.has_value() && alibi->defined())
    TORCH_CHECK(alibi->is_cuda() && alibi->is_contiguous() && alibi->numel() == Hq,
                "attn_decode: alibi must be a contiguous f32 [Hq] device tensor");
  a.alibi = (alibi.has_value() && alibi->defined()) ? alibi->data_ptr<float>() : nullptr;
  a.counters = fused_combine_on() ? attn_counters(q.device(), B * Hkv) : nullptr;
  a.v3_counters = !no_combine && v3_fuse_on() ? v3_counters(q.device(), B * Hkv) : nullptr;
  a.no_combine = no_combine ? 1 : 0;
  illm::launch_attn_decode(bf16, a, cur_stream());
  return {out, po, pml};
}

// decode attention with RoPE + KV append fused in (Tq == 1): q/k/v of the new
// token come from the qkv GEMV's atomic accumulator part [B, ld] (+ bias); no
// rope_kv launch.  The combine launch re-zeroes the accumulator (part is
// written: zero for the next atomic GEMV).
static std::tuple<Tensor, Tensor, Tensor> attn_decode_rope_impl(
    const Tensor& part, const c10::optional<Tensor>& bias, const Tensor& cos_sin, const Tensor& pos, Tensor& k_cache,
    Tensor& v_cache, const Tensor& block_tables, const Tensor& seq_lens, int64_t nsplit, double scale, double softcap,
    int64_t window, int64_t Hq, int64_t rot_dim, bool interleaved, double q_scale, at::ScalarType dt, bool no_combine,
    const c10::optional<Tensor>& pss, int64_t pss_n, double pss_eps, bool prerot) {
  c10::DeviceGuard g(part.device());
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf, "attn_decode_rope: bf16/fp16 activations");
  TORCH_CHECK(k_cache.scalar_type() == dt && v_cache.scalar_type() == dt, "attn_decode_rope: 16-bit KV cache");
  TORCH_CHECK(part.is_cuda() && part.dim() == 2 && part.scalar_type() == at::kFloat && part.is_contiguous(),
              "attn_decode_rope: part must be contiguous f32 [B, ld]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.dim() == 3,
              "attn_decode_rope: f32 cos/sin table [max_pos, rot/2, 2]");
  TORCH_CHECK(pos.scalar_type() == at::kLong && block_tables.scalar_type() == at::kInt &&
                  seq_lens.scalar_type() == at::kInt, "attn_decode_rope: int64 positions, int32 tables");
  const int64_t B = part.size(0), Hkv = k_cache.size(1), bs = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(part.size(1) == (Hq + 2 * Hkv) * D, "attn_decode_rope: part width != (Hq + 2 Hkv) * D");
  TORCH_CHECK((D == 128 && Hq / Hkv <= 16) || (D == 256 && Hq / Hkv <= 8), "attn_decode_rope: head_dim/group");
  TORCH_CHECK(Hq % Hkv == 0 && bs % 64 == 0 && rot_dim <= D && rot_dim % 2 == 0 && cos_sin.size(1) == rot_dim / 2,
              "attn_decode_rope: geometry");
  illm::AttnDecodeArgs a{};
  Tensor po = at::empty({B, Hq, 1, nsplit, D}, part.options());
  Tensor pml = at::empty({B, Hq, 1, nsplit, 2}, part.options());
  Tensor out = at::empty({B, 1, Hq, D}, part.options().dtype(dt));
  a.q = nullptr;
  a.k_cache = (const uint8_t*)k_cache.data_ptr();
  a.v_cache = (const uint8_t*)v_cache.data_ptr();
  a.block_tables = block_tables.data_ptr<int32_t>();
  a.seq_lens = seq_lens.data_ptr<int32_t>();
  a.max_blocks = (int)block_tables.size(1);
  a.num_blocks = (int)k_cache.size(0);
  a.err = kernel_err(k_cache.device());
  a.part_o = po.data_ptr<float>();
  a.part_ml = pml.data_ptr<float>();
  a.out = m16(out);
  a.B = (int)B;
  a.Tq = 1;
  a.Hq = (int)Hq;
  a.Hkv = (int)Hkv;
  a.D = (int)D;
  a.bs = (int)bs;
  TORCH_CHECK(nsplit >= 1 && nsplit <= kMaxDecodeSplits && (nsplit <= 1024 || D % 4 == 0),
              "attn_decode: nsplit must be 1..", kMaxDecodeSplits, " (1..1024 when D % 4 != 0; combine LDS), got ", nsplit);
  a.nsplit = (int)nsplit;
  a.scale = (float)scale;
  a.softcap = (float)softcap;
  a.sliding_window = (int)window;
  a.kv_fp8 = 0;
  a.k_scale = a.v_scale = 1.f;
  // the merging split (fused combine) or the combine launch re-zeroes the
  // accumulator; split-only (no_combine): the consumer merges and a later
  // launch zeroes it
  a.counters = !no_combine && fused_combine_on() ? attn_counters(part.device(), B * Hkv) : nullptr;
  a.v3_counters = !no_combine && v3_fuse_on() ? v3_counters(part.device(), B * Hkv) : nullptr;
  a.no_combine = no_combine ? 1 : 0;
  a.rq_part = part.data_ptr<float>();
  a.rq_bias = p16o(bias);
  a.rq_cos_sin = cos_sin.data_ptr<float>();
  a.rq_pos = pos.data_ptr<int64_t>();
  a.rq_ld = (int)part.size(1);
  a.rq_rot = (int)rot_dim;
  a.rq_interleaved = interleaved ? 1 : 0;
  a.rq_qscale = (float)q_scale;
  a.rq_prerot = prerot ? 1 : 0;
  TORCH_CHECK(!prerot || (rot_dim == D && !interleaved), "attn_decode_rope: prerot needs full-width NeoX RoPE");
  if (pss.has_value() && pss->defined()) {
    TORCH_CHECK(pss->is_cuda() && pss->scalar_type() == at::kFloat && pss->numel() >= B && pss_n > 0,
                "attn_decode_rope: pss must be f32 [B] with pss_n > 0");
    a.rq_ss = pss->data_ptr<float>();
    a.rq_ss_n = (int)pss_n;
    a.rq_ss_eps = (float)pss_eps;
  }
  illm::launch_attn_decode(dt == at::kBFloat16, a, cur_stream());
  return {out, po, pml};
}


Tensor attn_decode_rope(const Tensor& part, const c10::optional<Tensor>& bias, const Tensor& cos_sin,
                        const Tensor& pos, Tensor& k_cache, Tensor& v_cache, const Tensor& block_tables,
                        const Tensor& seq_lens, int64_t nsplit, double scale, double softcap, int64_t window,
                        int64_t Hq, int64_t rot_dim, bool interleaved, double q_scale, at::ScalarType dt,
                        const c10::optional<Tensor>& pss, int64_t pss_n, double pss_eps, bool prerot) {
  return std::get<0>(attn_decode_rope_impl(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit,
                                           scale, softcap, window, Hq, rot_dim, interleaved, q_scale, dt, false, pss,
                                           pss_n, pss_eps, prerot));
}

// fused-RoPE split attention without the combine: (o, m, l) partials for the
// o_proj GEMV's merging prologue (gemv_attn); the qkv accumulator is NOT
// re-zeroed here (the caller hands it to a later launch's zeroing)
std::tuple<Tensor, Tensor> attn_decode_rope_split(const Tensor& part, const c10::optional<Tensor>& bias,
                                                  const Tensor& cos_sin, const Tensor& pos, Tensor& k_cache,
                                                  Tensor& v_cache, const Tensor& block_tables, const Tensor& seq_lens,
                                                  int64_t nsplit, double scale, double softcap, int64_t window,
                                                  int64_t Hq, int64_t rot_dim, bool interleaved, double q_scale,
                                                  at::ScalarType dt, const c10::optional<Tensor>& pss,
                                                  int64_t pss_n, double pss_eps, bool prerot) {
  auto r = attn_decode_rope_impl(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit, scale,
                                 softcap, window, Hq, rot_dim, interleaved, q_scale, dt, true, pss, pss_n, pss_eps,
                                 prerot);
  return {std::get<1>(r), std::get<2>(r)};
}

Tensor attn_decode(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                   const Tensor& seq_lens, int64_t nsplit, double scale, double softcap, int64_t window,
                   int64_t kv_fp8, double k_scale, double v_scale, const c10::optional<Tensor>& alibi) {
  return std::get<0>(attn_decode_impl(q, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap, window,
                                      kv_fp8, k_scale, v_scale, alibi, false));
}

// prefill / long-query attention straight over the paged cache (attn_prefill.hip):
// q [B * Tq, Hq, D] -> out [B * Tq, Hq, D]; query t of sequence b sits at
// position seq_lens[b] - Tq + t (causal against everything before it)
Tensor attn_prefill(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache, const Tensor& block_tables,
                    const Tensor& seq_lens, int64_t Tq, double scale, double softcap, int64_t window,
                    int64_t kv_fp8, double k_scale, double v_scale) {
  c10::DeviceGuard g(q.device());
  TORCH_CHECK(q.dim() == 3 && q.is_contiguous(), "attn_prefill: q must be contiguous [B*Tq, Hq, D]");
  const bool bf16 = is_bf16(q);
  const int64_t Hq = q.size(1), D = q.size(2), Hkv = k_cache.size(1), bs = k_cache.size(2);
  const int64_t B = block_tables.size(0);
  TORCH_CHECK(Tq >= 1 && q.size(0) == B * Tq, "attn_prefill: q rows != B * Tq");
  TORCH_CHECK(D == 64 || D == 128, "attn_prefill: head_dim 64 or 128");
  TORCH_CHECK(k_cache.size(3) == D && v_cache.sizes() == k_cache.sizes(), "attn_prefill: cache shape");
  TORCH_CHECK(Hq % Hkv == 0 && bs % 64 == 0, "attn_prefill: GQA ratio / block size (multiple of 64)");
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && seq_lens.scalar_type() == at::kInt &&
                  seq_lens.numel() == B && block_tables.is_contiguous() && seq_lens.is_cuda(),
              "attn_prefill: int32 device tables");
  TORCH_CHECK(kv_fp8 != 0 || k_cache.scalar_type() == q.scalar_type(), "attn_prefill: KV dtype != q dtype");
  Tensor out = at::empty_like(q);
  illm::AttnPrefillArgs a{};
  a.q = p16(q);
  a.k_cache = (const uint8_t*)k_cache.data_ptr();
  a.v_cache = (const uint8_t*)v_cache.data_ptr();
  a.block_tables = block_tables.data_ptr<int32_t>();
  a.seq_lens = seq_lens.data_ptr<int32_t>();
  a.out = m16(out);
  a.B = (int)B;
  a.Tq = (int)Tq;
  a.Hq = (int)Hq;
  a.Hkv = (int)Hkv;
  a.D = (int)D;
  a.bs = (int)bs;
  a.max_blocks = (int)block_tables.size(1);
  a.num_blocks = (int)k_cache.size(0);
  a.err = kernel_err(k_cache.device());
  a.scale = (float)scale;
  a.softcap = (float)softcap;
  a.sliding_window = (int)window;
  a.kv_fp8 = (int)kv_fp8;
  a.k_scale = (float)k_scale;
  a.v_scale = (float)v_scale;
  if (B > 0) illm::launch_attn_prefill(bf16, a, cur_stream());
  return out;
}

// split kernel only: the (o, m, l) partials [B, Hq, Tq, nsplit, D] / [.., 2] are merged by the
// o_proj GEMV's prologue (gemv_attn), which saves the combine launch
std::tuple<Tensor, Tensor> attn_decode_split(const Tensor& q, const Tensor& k_cache, const Tensor& v_cache,
                                             const Tensor& block_tables, const Tensor& seq_lens, int64_t nsplit,
                                             double scale, double softcap, int64_t window, int64_t kv_fp8,
                                             double k_scale, double v_scale, const c10::optional<Tensor>& alibi) {
  auto r = attn_decode_impl(q, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap, window, kv_fp8,
                            k_scale, v_scale, alibi, true);
  return {std::get<1>(r), std::get<2>(r)};
}

// o_proj GEMV whose input rows are combined from the flash-decoding partials in
// its prologue.  acc given: f32 atomics into acc [T, n] (returned); else f32
// split-K slabs [ks, T, n].
Tensor gemv_attn(const Tensor& po, const Tensor& pml, const Tensor& seq_lens, const Tensor& blob, int64_t fmt,
                 int64_t n, int64_t k, const c10::optional<Tensor>& acc, int64_t ksplit, at::ScalarType dt,
                 const c10::optional<Tensor>& zero, int64_t nw) {
  TORCH_CHECK(po.is_cuda() && po.dim() == 5 && po.scalar_type() == at::kFloat && po.is_contiguous(),
              "gemv_attn: po must be f32 [B, Hq, Tq, ns, D]");
  c10::DeviceGuard g(po.device());
  const int64_t B = po.size(0), Hq = po.size(1), Tq = po.size(2), ns = po.size(3), D = po.size(4);
  const int64_t M = B * Tq;
  TORCH_CHECK(Hq * D == k && D % 8 == 0, "gemv_attn: Hq * D must equal in_features");
  TORCH_CHECK(M >= 1 && M <= 16, "gemv_attn handles 1..16 rows");
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf, "gemv_attn: bf16/fp16 activations");
  TORCH_CHECK(blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemv_attn: weight blob too small");
  const bool bf16 = dt == at::kBFloat16;
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  illm::GemvArgs a{};
  a.apo = po.data_ptr<float>();
  a.aml = pml.data_ptr<float>();
  a.alens = seq_lens.data_ptr<int32_t>();
  a.ans = (int)ns;
  a.aD = (int)D;
  a.aHq = (int)Hq;
  a.aTq = (int)Tq;
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.lut_fmt = (int)fmt;
  a.N = (int)n;
  const bool atomic = acc.has_value() && acc->defined();
  Plan5 p = plan5(M, NT, KC, true, ksplit, atomic);
  if (nw == 4 || nw == 8) {            // workgroup size: 8 waves halve the per-head re-reads of the partials
    p.nw = (int)nw;
    p.gx = (unsigned)((NT + (p.nw / p.kw) - 1) / (p.nw / p.kw));
  }
  p.shmem += illm::gemv5_attn_shmem_h((int)M, (int)p.cpk, (int)D, (int)ns);
  TORCH_CHECK(p.shmem <= kMaxLds, "gemv_attn: LDS plan too large (too many attention splits)");
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  Tensor out;
  if (atomic) {
    TORCH_CHECK(acc->scalar_type() == at::kFloat && acc->is_contiguous() && acc->numel() == M * n,
                "gemv_attn: acc must be contiguous f32 [T, n]");
    a.out = acc->data_ptr();
    out = *acc;
  } else {
    out = at::empty({p.ks, M, n}, po.options());
    a.out = out.data_ptr();
  }
  if (zero.has_value() && zero->defined()) {
    TORCH_CHECK(zero->scalar_type() == at::kFloat && zero->is_contiguous() && zero->numel() % 4 == 0,
                "gemv_attn: zero must be contiguous f32 (numel % 4 == 0)");
    a.nzero = zero->data_ptr<float>();
    a.nzero_n = (int)zero->numel();
  }
  a.ldo = (int)n;
  launch_gemv5_any((int)fmt, bf16, p.kw, atomic ? illm::EPI_ATOMIC : illm::EPI_PARTIAL, dim3(p.gx, (unsigned)p.ks),
                   p.shmem, a);
  return out;
}


Tensor glu(const Tensor& gu, int64_t act, int64_t tile) {
  c10::DeviceGuard g(gu.device());
  const bool bf16 = is_bf16(gu);
  Tensor x = gu.contiguous();
  const int64_t I2 = x.size(-1), M = x.numel() / I2, I = I2 / 2;
  TORCH_CHECK(I % 8 == 0 && (tile == 0 || (tile % 8 == 0 && I % tile == 0)),
              "glu: intermediate size must be a multiple of 8 (and of the interleave tile)");
  auto shape = x.sizes().vec();
  shape.back() = I;
  Tensor out = at::empty(shape, x.options());
  if (M > 0) illm::launch_glu(bf16, p16(x), (int)I2, m16(out), (int)M, (int)I, (int)act, (int)tile, cur_stream());
  return out;
}

void attn_softmax_(const Tensor& x) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf),
              "attn_softmax_: contiguous bf16/fp16 GPU tensor expected");
  TORCH_CHECK(x.dim() >= 1 && x.size(-1) > 0 && x.size(-1) < (1LL << 31), "attn_softmax_: bad row length");
  const int64_t L = x.size(-1), rows = x.numel() / L;
  TORCH_CHECK((rows + 3) / 4 < (1LL << 31), "attn_softmax_: too many rows");
  if (rows > 0) illm::launch_softmax_rows(is_bf16(x), (uint16_t*)x.data_ptr(), rows, (int)L, cur_stream());
}

Tensor reduce_partials(const Tensor& ws, const c10::optional<Tensor>& bias, at::ScalarType dt) {
  c10::DeviceGuard g(ws.device());
  const int64_t ks = ws.size(0), M = ws.size(1), N = ws.size(2);
  Tensor out = at::empty({M, N}, ws.options().dtype(dt));
  illm::launch_reduce_partials(dt == at::kBFloat16, ws.data_ptr<float>(), (int)ks, p16o(bias), m16(out),
                               (int)M, (int)N, (int)N, cur_stream());
  return out;
}

std::tuple<Tensor, Tensor> moe_group_topk(const Tensor& logits, const c10::optional<Tensor>& bias, int64_t k,
                                          int64_t n_group, int64_t topk_group, bool renorm, double scale) {
  c10::DeviceGuard g(logits.device());
  Tensor l = logits.to(at::kFloat).contiguous();
  const int64_t E = l.size(-1), T = l.numel() / E;
  TORCH_CHECK(E <= 512 && k <= E && n_group >= 1 && n_group <= 64 && E % n_group == 0 && topk_group <= n_group,
              "moe_group_topk: E <= 512, n_group <= 64 dividing E");
  Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(b.numel() == E && b.is_cuda(), "moe_group_topk: bias [E] on the GPU");
  }
  Tensor w = at::empty({T, k}, l.options());
  Tensor ids = at::empty({T, k}, l.options().dtype(at::kInt));
  if (T > 0)
    illm::launch_moe_group_topk(l.data_ptr<float>(), b.defined() ? b.data_ptr<float>() : nullptr, (int)T, (int)E,
                                (int)k, (int)n_group, (int)topk_group, renorm ? 1 : 0, (float)scale,
                                w.data_ptr<float>(), ids.data_ptr<int32_t>(), cur_stream());
  return {w, ids};
}

std::tuple<Tensor, Tensor> moe_topk(const Tensor& logits, int64_t k, bool renorm, int64_t scoring) {
  c10::DeviceGuard g(logits.device());
  Tensor l = logits.to(at::kFloat).contiguous();
  const int64_t E = l.size(-1), T = l.numel() / E;
  TORCH_CHECK(E <= 512 && k <= E && k <= 64, "moe_topk: E <= 512, k <= 64");
  Tensor w = at::empty({T, k}, l.options());
  Tensor ids = at::empty({T, k}, l.options().dtype(at::kInt));
  if (T > 0) illm::launch_moe_topk(l.data_ptr<float>(), (int)T, (int)E, (int)k, renorm, (int)scoring,
                                   w.data_ptr<float>(), ids.data_ptr<int32_t>(), cur_stream());
  return {w, ids};
}

std::tuple<Tensor, Tensor> moe_align(const Tensor& ids, int64_t e0, int64_t num_local) {
  c10::DeviceGuard g(ids.device());
  Tensor idc = ids.to(at::kInt).contiguous();
  const int64_t P = idc.numel();
  TORCH_CHECK(num_local >= 1 && num_local <= 4096, "moe_align: 1..4096 local experts");
  Tensor off = at::empty({num_local + 1}, idc.options());
  Tensor rows = at::empty({std::max<int64_t>(P, 1)}, idc.options());
  illm::launch_moe_align(idc.data_ptr<int32_t>(), (int)P, (int)e0, (int)num_local, off.data_ptr<int32_t>(),
                         rows.data_ptr<int32_t>(), cur_stream());
  return {off, rows};
}

// Grouped low-bit GEMV over experts (decode MoE, <= 16 tokens):
//   epi GLU:     x [T, k] (pair p reads row p / xdiv)  -> [npairs, n/2]
//   epi PARTIAL: x [npairs, k]                         -> f32 [ks, npairs, n]
Tensor moe_gemv(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, const Tensor& off,
                const Tensor& rows, int64_t xdiv, int64_t npairs, int64_t epi, int64_t ksplit, int64_t act) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && blob.dim() == 2, "moe_gemv: GPU x and [E, bytes] blob");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  TORCH_CHECK(xc.size(-1) == k, "moe_gemv: x last dim != k");
  const int64_t rows_x = xc.numel() / k;
  TORCH_CHECK(blob.size(1) >= illm::dev_total_bytes((int)fmt, n, k), "moe_gemv: expert blob too small");
  const int64_t E = blob.size(0);
  TORCH_CHECK(off.numel() == E + 1, "moe_gemv: off must have E+1 entries");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  // rows per expert <= tokens routed in this step (each token picks an expert once)
  const int64_t Mmax = std::min<int64_t>(16, epi == illm::EPI_GLU ? rows_x : npairs);
  TORCH_CHECK(epi != illm::EPI_GLU || rows_x <= 16, "moe_gemv: the decode path handles <= 16 tokens");
  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)npairs;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.act = (int)act;
  a.lut_fmt = (int)fmt;
  a.moe_off = off.data_ptr<int32_t>();
  a.moe_rows = rows.data_ptr<int32_t>();
  a.moe_xdiv = (int)std::max<int64_t>(1, xdiv);
  a.w_stride = blob.size(1);
  if (epi == illm::EPI_GLU) {
    TORCH_CHECK(n % 32 == 0, "GLU expert weights need a multiple of 32 rows");
    Tensor out = at::empty({npairs, n / 2}, xc.options());
    a.N = (int)(n / 2);
    a.out = out.data_ptr();
    a.ldo = (int)(n / 2);
    const Plan5 p = plan5(Mmax, NT / 2, KC, false);
    TORCH_CHECK(p.shmem <= kMaxLds, "moe_gemv: hidden size too large for the LDS-staged GLU path");
    a.nw = p.nw;
    launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_GLU, dim3(p.gx, 1, (unsigned)E), p.shmem, a);
    return out;
  }
  a.N = (int)n;
  const Plan5 p = plan5(Mmax, NT, KC, true, ksplit);
  ksplit = p.ks;
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  TORCH_CHECK(p.shmem <= kMaxLds, "moe_gemv: K slice too large for LDS");
  Tensor ws = at::empty({ksplit, npairs, n}, xc.options().dtype(at::kFloat));
  a.out = ws.data_ptr();
  a.ldo = (int)n;
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_PARTIAL, dim3(p.gx, (unsigned)ksplit, (unsigned)E), p.shmem, a);
  return ws;
}

// grouped down projection over expert pairs with the routing-weighted combine
// in the epilogue: acc[p / topk, :] += w[p] * (x[p] @ W_e^T) by f32 atomics
// (acc zero on entry; its consumer, add_rms_norm, reads and re-zeroes it)
void moe_gemv_accum(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, const Tensor& off,
                    const Tensor& rows, const Tensor& acc, const Tensor& w, int64_t topk, int64_t ksplit) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && blob.dim() == 2, "moe_gemv_accum: GPU x and [E, bytes] blob");
  c10::DeviceGuard g(x.device());
  const bool bf16 = is_bf16(x);
  Tensor xc = x.contiguous();
  TORCH_CHECK(xc.dim() == 2 && xc.size(1) == k, "moe_gemv_accum: x must be [pairs, k]");
  const int64_t P = xc.size(0);
  TORCH_CHECK(topk >= 1 && P % topk == 0, "moe_gemv_accum: pairs must be tokens * topk");
  TORCH_CHECK(acc.scalar_type() == at::kFloat && acc.is_contiguous() && acc.numel() == (P / topk) * n,
              "moe_gemv_accum: acc must be contiguous f32 [tokens, n]");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == P,
              "moe_gemv_accum: w must be contiguous f32 [tokens, topk]");
  TORCH_CHECK(blob.size(1) >= illm::dev_total_bytes((int)fmt, n, k), "moe_gemv_accum: expert blob too small");
  const int64_t E = blob.size(0);
  TORCH_CHECK(off.numel() == E + 1 && off.scalar_type() == at::kInt && rows.scalar_type() == at::kInt,
              "moe_gemv_accum: off int32 [E+1], rows int32");
  const int64_t NT = illm::pad_to(n, illm::TILE_N) / illm::TILE_N;
  const int64_t KC = illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K;
  const int64_t Mmax = std::min<int64_t>(16, P);
  illm::GemvArgs a{};
  a.x = p16(xc);
  a.M = (int)P;
  a.K = (int)k;
  a.ldx = (int)k;
  a.w = blob.data_ptr<uint8_t>();
  a.KC = (int)KC;
  a.lut_fmt = (int)fmt;
  a.moe_off = off.data_ptr<int32_t>();
  a.moe_rows = rows.data_ptr<int32_t>();
  a.moe_xdiv = 1;
  a.moe_w = w.data_ptr<float>();
  a.moe_odiv = (int)topk;
  a.w_stride = blob.size(1);
  a.N = (int)n;
  a.out = acc.data_ptr();
  a.ldo = (int)n;
  const Plan5 p = plan5(Mmax, NT, KC, true, ksplit, true);
  a.cpk = (int)p.cpk;
  a.nw = p.nw;
  TORCH_CHECK(p.shmem <= kMaxLds, "moe_gemv_accum: K slice too large for LDS");
  launch_gemv5_any((int)fmt, bf16, p.kw, illm::EPI_ATOMIC, dim3(p.gx, (unsigned)p.ks, (unsigned)E), p.shmem, a);
}

// fused decode router (<= 16 tokens): logits, top-k and pair lists in one launch
std::tuple<Tensor, Tensor, Tensor, Tensor> moe_route(const Tensor& x, const Tensor& wr, int64_t k, bool renorm,
                                                     int64_t scoring, int64_t e0, int64_t num_local,
                                                     const Tensor& counter) {
  TORCH_CHECK(x.is_cuda() && wr.is_cuda() && counter.is_cuda(), "moe_route: GPU tensors expected");
  c10::DeviceGuard g(x.device());
  Tensor xc = x.contiguous(), wc = wr.contiguous();
  TORCH_CHECK(xc.dim() == 2 && wc.dim() == 2 && xc.size(1) == wc.size(1), "moe_route: x [T, H], router [E, H]");
  TORCH_CHECK(xc.scalar_type() == wc.scalar_type() && (is_bf16(xc) || xc.scalar_type() == at::kHalf),
              "moe_route: x and router must share one 16-bit dtype");
  const int64_t T = xc.size(0), H = xc.size(1), E = wc.size(0);
  TORCH_CHECK(T >= 1 && T <= 16, "moe_route: 1..16 tokens");
  TORCH_CHECK(H % 8 == 0, "moe_route: hidden % 8");
  TORCH_CHECK(E <= 512 && k >= 1 && k <= 16 && k <= E, "moe_route: E <= 512, 1 <= k <= 16");
  TORCH_CHECK(num_local >= 1 && num_local <= 512 && e0 >= 0, "moe_route: 1..512 local experts");
  TORCH_CHECK(counter.scalar_type() == at::kInt && counter.numel() >= 1, "moe_route: int32 counter");
  auto f32 = xc.options().dtype(at::kFloat);
  auto i32 = xc.options().dtype(at::kInt);
  const int64_t nsp = std::max<int64_t>(1, (H / 8 + 255) / 256);   // 256 16-B chunks per workgroup
  Tensor logits = at::empty({nsp, T, E}, f32);
  Tensor w = at::empty({T, k}, f32);
  Tensor ids = at::empty({T, k}, i32);
  Tensor off = at::empty({num_local + 1}, i32);
  Tensor rows = at::empty({T * k}, i32);
  illm::MoeRouteArgs a{};
  a.x = p16(xc);
  a.wr = p16(wc);
  a.T = (int)T; a.H = (int)H; a.E = (int)E; a.k = (int)k;
  a.renorm = renorm ? 1 : 0; a.scoring = (int)scoring; a.e0 = (int)e0; a.El = (int)num_local;
  a.nsp = (int)nsp;
  a.logits = logits.data_ptr<float>();
  a.counter = counter.data_ptr<int32_t>();
  a.topk_w = w.data_ptr<float>();
  a.topk_ids = ids.data_ptr<int32_t>();
  a.off = off.data_ptr<int32_t>();
  a.rows = rows.data_ptr<int32_t>();
  illm::launch_moe_route(is_bf16(xc), a, cur_stream());
  return {w, ids, off, rows};
}

Tensor moe_combine(const Tensor& part, const Tensor& w, const Tensor& ids, int64_t e0, int64_t num_local,
                   at::ScalarType dt) {
  c10::DeviceGuard g(part.device());
  TORCH_CHECK(part.dim() == 3 && part.scalar_type() == at::kFloat, "moe_combine: part f32 [ks, P, H]");
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf, "moe_combine: bf16/fp16 out");
  const int64_t ks = part.size(0), P = part.size(1), H = part.size(2);
  TORCH_CHECK(H % 4 == 0, "moe_combine: hidden % 4");
  Tensor wc = w.to(at::kFloat).contiguous(), ic = ids.to(at::kInt).contiguous();
  const int64_t k = wc.size(-1), Tn = wc.numel() / k;
  TORCH_CHECK(Tn * k == P, "moe_combine: P != T * k");
  Tensor out = at::empty({Tn, H}, part.options().dtype(dt));
  illm::launch_moe_combine(dt == at::kBFloat16, part.data_ptr<float>(), (int)ks, (int)P, wc.data_ptr<float>(),
                           ic.data_ptr<int32_t>(), (int)k, (int)e0, (int)num_local, m16(out), (int)Tn, (int)H,
                           cur_stream());
  return out;
}

Tensor embedding_lowbit(const Tensor& blob, int64_t fmt, int64_t n, int64_t k, const Tensor& ids,
                        at::ScalarType dt) {
  c10::DeviceGuard g(blob.device());
  TORCH_CHECK(k % 64 == 0, "embedding_lowbit: hidden % 64");
  TORCH_CHECK(blob.numel() >= illm::canon_total_bytes((int)fmt, n, k), "embedding_lowbit: blob too small");
  Tensor idc = ids.to(at::kLong).contiguous();
  auto shape = idc.sizes().vec();
  shape.push_back(k);
  Tensor out = at::empty(shape, blob.options().dtype(dt));
  const int64_t T = idc.numel();
  if (T > 0)
    illm::launch_embedding_rows(dt == at::kBFloat16, blob.data_ptr<uint8_t>(), (int)fmt, idc.data_ptr<int64_t>(),
                                (int)T, n, k, m16(out), kernel_err(blob.device()), cur_stream());
  return out;
}

// logits: [B, V] bf16/f16 or undefined (sampling done by the host: only advance)
void decode_advance(const c10::optional<Tensor>& logits, Tensor& ids, Tensor& next_ids, Tensor& pos,
                    const Tensor& block_tables, int64_t bs, Tensor& slots, Tensor& seq_lens,
                    const c10::optional<Tensor>& pos_offset, const c10::optional<Tensor>& parts) {
  c10::DeviceGuard g(pos.device());
  const int64_t B = pos.numel();
  TORCH_CHECK(pos.scalar_type() == at::kLong && ids.scalar_type() == at::kLong && slots.scalar_type() == at::kLong &&
              seq_lens.scalar_type() == at::kInt && block_tables.scalar_type() == at::kInt, "decode_advance dtypes");
  const bool has = logits.has_value() && logits->defined();
  const bool hp = parts.has_value() && parts->defined();
  TORCH_CHECK(!hp || (parts->dim() == 3 && parts->size(1) == B && parts->size(2) == 2 &&
                      parts->scalar_type() == at::kFloat && parts->is_contiguous()),
              "decode_advance: parts must be f32 [nparts, B, 2]");
  bool bf16 = true;
  int V = 0;
  if (has) {
    bf16 = is_bf16(*logits);
    TORCH_CHECK(logits->is_contiguous() && logits->size(0) == B, "decode_advance: logits [B, V]");
    V = (int)logits->size(-1);
  }
  illm::launch_decode_advance(bf16, has ? p16(*logits) : nullptr, (int)B, V, ids.data_ptr<int64_t>(),
                              next_ids.data_ptr<int64_t>(), pos.data_ptr<int64_t>(), block_tables.data_ptr<int32_t>(),
                              (int)block_tables.size(1), (int)bs, slots.data_ptr<int64_t>(),
                              seq_lens.data_ptr<int32_t>(),
                              (pos_offset.has_value() && pos_offset->defined()) ? pos_offset->data_ptr<int64_t>() : nullptr,
                              kernel_err(pos.device()), cur_stream(), hp ? parts->data_ptr<float>() : nullptr,
                              hp ? (int)parts->size(0) : 0);
}

// stream bytes [offset, offset + nbytes) of t's storage through the caches
// (Infinity-Cache warm-up for the next reader); nbytes < 0 -> to the end
void l3_prefetch(const Tensor& t, int64_t offset, int64_t nbytes, int64_t wgs) {
  TORCH_CHECK(t.is_cuda(), "l3_prefetch: GPU tensor");
  const int64_t total = (int64_t)(t.numel() * t.element_size());
  TORCH_CHECK(offset >= 0 && offset <= total, "l3_prefetch: offset out of range");
  if (nbytes < 0 || offset + nbytes > total) nbytes = total - offset;
  const char* p = (const char*)t.data_ptr() + offset;
  // 16-B granules from the first aligned address inside the range
  const int64_t lead = (int64_t)((16 - ((uintptr_t)p & 15)) & 15);
  if (nbytes <= lead) return;
  c10::DeviceGuard g(t.device());
  // the kernel's write-only sink (its loads must be consumed): one per device,
  // made on first use outside capture like the error word
  static std::map<int, at::Tensor> sinks;
  auto it = sinks.find(t.device().index());
  if (it == sinks.end())
    it = sinks.emplace(t.device().index(), at::empty({64}, t.options().dtype(at::kInt))).first;
  illm::launch_l3_prefetch(p + lead, (size_t)(nbytes - lead), (int)wgs, (unsigned*)it->second.data_ptr<int>(),
                           cur_stream());
}

}  // namespace

// the device error word for the other binding units (ops_dist.cpp)
int* illm_kernel_err(const c10::Device& dev) { return kernel_err(dev); }

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("gemv_glu_in", &gemv_glu_in);
  m.impl("decode_advance", &decode_advance);
  m.impl("gemv_argmax", &gemv_argmax);
  m.impl("embed_rms_norm", &embed_rms_norm);
  m.impl("l3_prefetch", &l3_prefetch);
  m.impl("rope_kv_fused", &rope_kv_fused);
  m.impl("embedding_lowbit", &embedding_lowbit);
  m.impl("moe_align", &moe_align);
  m.impl("moe_gemv", &moe_gemv);
  m.impl("moe_combine", &moe_combine);
  m.impl("moe_gemv_accum", &moe_gemv_accum);
  m.impl("moe_route", &moe_route);
  m.impl("quantize_device", &quantize_device);
  m.impl("dequantize_device", &dequantize_device);
  m.impl("gemv", &gemv);
  m.impl("gemv_accum", &gemv_accum);
  m.impl("gemv_accum_norm", &gemv_accum_norm);
  m.impl("gemv_glu_ss", &gemv_glu_ss);
  m.impl("gemv_norm_in", &gemv_norm_in);
  m.impl("gemm_glu", &gemm_glu);
  m.impl("moe_gemm", &moe_gemm);
  m.impl("rwkv_wkv4", &rwkv_wkv4);
  m.impl("rwkv_wkv5", &rwkv_wkv5);
  m.impl("attn_decode_rope", &attn_decode_rope);
  m.impl("attn_decode_rope_split", &attn_decode_rope_split);
  m.impl("gemm", &gemm);
  m.impl("attn_decode_split", &attn_decode_split);
  m.impl("attn_prefill", &attn_prefill);
  m.impl("moe_group_topk", &moe_group_topk);
  m.impl("gemv_attn", &gemv_attn);
  m.impl("add_rms_norm", &add_rms_norm);
  m.impl("rms_norm_bwd", &rms_norm_bwd);
  m.impl("rope_half", &rope_half);
  m.impl("act_mul", &act_mul);
  m.impl("layer_norm", &layer_norm);
  m.impl("kernel_errors", &kernel_errors);
  m.impl("rope_kv", &rope_kv);
  m.impl("attn_decode", &attn_decode);
  m.impl("glu", &glu);
  m.impl("attn_softmax_", &attn_softmax_);
  m.impl("reduce_partials", &reduce_partials);
  m.impl("moe_topk", &moe_topk);
}
