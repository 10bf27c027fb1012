// torch.library ops of the MFMA GEMM engine (csrc/hip/gemm_mfma.hip):
// prefill / training GEMMs over low-bit tiled blobs or dense 16-bit weights.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "../common/formats.h"
#include "../hip/kernels.h"
#include "../hip/kernels_train.h"
#include "../hip/kernels_g8.h"

using at::Tensor;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// geometry: 256 x 256 blocks while they fill the 256 CUs, else 256 x 128,
// then split-K over even step counts until ~1 wave of blocks
struct MfgPlan {
  int tile, ksplit, sps;
};
MfgPlan mfg_plan(int64_t M, int64_t N, int64_t K, int64_t tile_req, int64_t ks_req, bool glu) {
  static const int tile_env = getenv("ILLM_MFG_TILE") ? atoi(getenv("ILLM_MFG_TILE")) : -1;
  static const int ks_env = getenv("ILLM_MFG_KSPLIT") ? atoi(getenv("ILLM_MFG_KSPLIT")) : 0;
  const int T = (int)(K / 64);
  MfgPlan p{illm::MFG_TILE_256x256, 1, T};
  auto blocks = [&](int tile) {
    return ((N + illm::mfg_block_n(tile) - 1) / illm::mfg_block_n(tile)) *
           ((M + illm::mfg_block_m(tile) - 1) / illm::mfg_block_m(tile));
  };
  if (tile_req >= 0) p.tile = (int)tile_req;
  else if (tile_env >= 0) p.tile = tile_env;
  else if (blocks(illm::MFG_TILE_256x256) < 256) p.tile = illm::MFG_TILE_256x128;
  int ks = (int)(ks_req > 0 ? ks_req : ks_env);
  if (ks <= 0) {
    ks = 1;
    if (!glu)
      while (blocks(p.tile) * ks * 2 <= 320 && T / (ks * 2) >= 8) ks *= 2;
  }
  if (glu) ks = 1;
  p.sps = ((T + ks - 1) / ks + 1) / 2 * 2;
  p.ksplit = (T + p.sps - 1) / p.sps;
  return p;
}

// out[..., N] = x[..., K] . W^T (+ bias).  fmt >= 0: w = tiled low-bit blob
// (bf16 activations normalised per row to f16 for the f16 MFMA); fmt < 0: w =
// dense [N, K] bf16 / f16 (x converted to w's dtype if needed).  glu: the
// tile-interleaved gate/up weight, out = act(gate) * up [..., N / 2].
Tensor mfgemm(const Tensor& x, const Tensor& w, int64_t fmt, int64_t n, int64_t k, const c10::optional<Tensor>& bias,
              bool glu, int64_t act, int64_t tile, int64_t ksplit) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda(), "mfgemm: GPU tensors expected");
  TORCH_CHECK(x.size(-1) == k, "mfgemm: x last dim ", x.size(-1), " != in_features ", k);
  TORCH_CHECK(k % 128 == 0, "mfgemm: in_features must be a multiple of 128");
  TORCH_CHECK(n % 16 == 0 && (!glu || n % 32 == 0), "mfgemm: out_features must be a multiple of 16 (32 for glu)");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "mfgemm: bf16/fp16 activations");
  c10::DeviceGuard g(x.device());
  const bool out_bf16 = x.scalar_type() == at::kBFloat16;
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k;
  auto shape = xc.sizes().vec();
  shape.back() = glu ? n / 2 : n;
  Tensor out = at::empty(shape, xc.options());
  if (M == 0) return out;
  const bool dense = fmt < 0;
  illm::MfgArgs a{};
  Tensor xm, rs;
  bool dense_bf16 = false;
  if (dense) {
    TORCH_CHECK(w.dim() == 2 && w.size(0) == n && w.size(1) == k && w.is_contiguous(), "mfgemm: dense w [n, k]");
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kHalf, "mfgemm: dense w bf16/fp16");
    dense_bf16 = w.scalar_type() == at::kBFloat16;
    xm = xc.scalar_type() == w.scalar_type() ? xc : xc.to(w.scalar_type());
    TORCH_CHECK((n + 256) * k * 2 < (int64_t)UINT32_MAX, "mfgemm: dense weight too large for one buffer descriptor");
    a.w_bytes = (uint32_t)(n * k * 2);
    a.ldw = (int)k;
  } else {
    TORCH_CHECK(w.scalar_type() == at::kByte, "mfgemm: low-bit blob must be uint8");
    TORCH_CHECK(w.numel() >= illm::dev_total_bytes((int)fmt, n, k), "mfgemm: weight blob too small");
    if (out_bf16) {
      xm = at::empty({M, k}, xc.options().dtype(at::kHalf));
      rs = at::empty({M}, xc.options().dtype(at::kFloat));
      illm::launch_x_to_f16_rowscale(true, (const uint16_t*)xc.data_ptr(), M, k, (int)k, (uint16_t*)xm.data_ptr(),
                                     rs.data_ptr<float>(), cur_stream());
      a.rs = rs.data_ptr<float>();
    } else {
      xm = xc;
    }
  }
  TORCH_CHECK((M + 256) * k * 2 < (int64_t)UINT32_MAX, "mfgemm: activations too large for one buffer descriptor");
  a.x = (const uint16_t*)xm.data_ptr();
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.x_bytes = (uint32_t)(M * k * 2);
  a.w = (const uint8_t*)w.data_ptr();
  a.N = (int)n;
  a.KC = (int)(illm::pad_to(k, illm::CHUNK_K) / illm::CHUNK_K);
  a.glu = glu ? 1 : 0;
  a.act = (int)act;
  a.lut_fmt = (int)fmt;
  a.out_bf16 = out_bf16 ? 1 : 0;
  const Tensor* bp = (bias.has_value() && bias->defined()) ? &*bias : nullptr;
  Tensor bconv;
  if (bp != nullptr) {
    TORCH_CHECK(!glu, "mfgemm: bias with glu is not supported");
    TORCH_CHECK(bp->numel() == n, "mfgemm: bias size");
    bconv = bp->contiguous();
    if (bconv.scalar_type() != at::kBFloat16 && bconv.scalar_type() != at::kHalf) bconv = bconv.to(xc.scalar_type());
  }
  const MfgPlan p = mfg_plan(M, n, k, tile, ksplit, glu);
  a.sps = p.sps;
  if (p.ksplit > 1) {
    Tensor ws = at::empty({p.ksplit, M, n}, xc.options().dtype(at::kFloat));
    a.out = ws.data_ptr();
    a.out_f32 = 1;
    a.ldo = (int)n;
    a.slab = M * n;
    illm::launch_mfgemm((int)fmt, dense_bf16, p.tile, a, p.ksplit, cur_stream());
    Tensor b16;
    if (bp != nullptr) b16 = bconv.scalar_type() == xc.scalar_type() ? bconv : bconv.to(xc.scalar_type());
    illm::launch_reduce_partials(out_bf16, ws.data_ptr<float>(), p.ksplit,
                                 bp != nullptr ? (const uint16_t*)b16.data_ptr() : nullptr, (uint16_t*)out.data_ptr(),
                                 (int)M, (int)n, (int)n, cur_stream());
    return out;
  }
  a.out = out.data_ptr();
  a.ldo = (int)(glu ? n / 2 : n);
  if (bp != nullptr) {
    a.bias = (const uint16_t*)bconv.data_ptr();
    a.bias_bf16 = bconv.scalar_type() == at::kBFloat16 ? 1 : 0;
  }
  illm::launch_mfgemm((int)fmt, dense_bf16, p.tile, a, 1, cur_stream());
  return out;
}

// grad_x of a linear with weight W [n, k]: out[..., k] = g[..., n] . W.  fmt >=
// 0: W = tiled low-bit blob (g normalised per row to f16); fmt < 0: dense W.
Tensor mfgemm_nn(const Tensor& g, const Tensor& w, int64_t fmt, int64_t n, int64_t k, int64_t tile, int64_t ksplit) {
  TORCH_CHECK(g.is_cuda() && w.is_cuda(), "mfgemm_nn: GPU tensors expected");
  TORCH_CHECK(g.size(-1) == n, "mfgemm_nn: g last dim ", g.size(-1), " != out_features ", n);
  TORCH_CHECK(n % 128 == 0, "mfgemm_nn: out_features must be a multiple of 128");
  TORCH_CHECK(k % (fmt < 0 ? 128 : 256) == 0, "mfgemm_nn: in_features must be a multiple of 256 (128 dense)");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kHalf, "mfgemm_nn: bf16/fp16 g");
  c10::DeviceGuard dg(g.device());
  const bool out_bf16 = g.scalar_type() == at::kBFloat16;
  Tensor gc = g.contiguous();
  const int64_t M = gc.numel() / n;
  auto shape = gc.sizes().vec();
  shape.back() = k;
  Tensor out = at::empty(shape, gc.options());
  if (M == 0) return out;
  illm::MfgArgs a{};
  Tensor gm, rs;
  bool dense_bf16 = false;
  if (fmt < 0) {
    TORCH_CHECK(w.dim() == 2 && w.size(0) == n && w.size(1) == k && w.is_contiguous(), "mfgemm_nn: dense w [n, k]");
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kHalf, "mfgemm_nn: dense w bf16/fp16");
    TORCH_CHECK(n * k * 2 < (int64_t)INT32_MAX, "mfgemm_nn: dense weight too large for one buffer descriptor");
    dense_bf16 = w.scalar_type() == at::kBFloat16;
    gm = gc.scalar_type() == w.scalar_type() ? gc : gc.to(w.scalar_type());
    a.w_bytes = (uint32_t)(n * k * 2);
    a.ldw = (int)k;
  } else {
    TORCH_CHECK(w.scalar_type() == at::kByte, "mfgemm_nn: low-bit blob must be uint8");
    TORCH_CHECK(w.numel() >= illm::dev_total_bytes((int)fmt, n, k), "mfgemm_nn: weight blob too small");
    if (out_bf16) {
      gm = at::empty({M, n}, gc.options().dtype(at::kHalf));
      rs = at::empty({M}, gc.options().dtype(at::kFloat));
      illm::launch_x_to_f16_rowscale(true, (const uint16_t*)gc.data_ptr(), M, n, (int)n, (uint16_t*)gm.data_ptr(),
                                     rs.data_ptr<float>(), cur_stream());
      a.rs = rs.data_ptr<float>();
    } else {
      gm = gc;
    }
  }
  TORCH_CHECK((M + 256) * n * 2 < (int64_t)UINT32_MAX, "mfgemm_nn: g too large for one buffer descriptor");
  a.x = (const uint16_t*)gm.data_ptr();
  a.M = (int)M;
  a.K = (int)n;
  a.ldx = (int)n;
  a.x_bytes = (uint32_t)(M * n * 2);
  a.w = (const uint8_t*)w.data_ptr();
  a.N = (int)k;
  a.KC = (int)(k / 128);
  a.lut_fmt = (int)fmt;
  a.out_bf16 = out_bf16 ? 1 : 0;
  const MfgPlan p = mfg_plan(M, k, n, tile == illm::MFG_TILE_128x256 ? 0 : tile, ksplit, false);
  const int t = p.tile == illm::MFG_TILE_128x256 ? illm::MFG_TILE_256x256 : p.tile;
  a.sps = p.sps;
  if (p.ksplit > 1) {
    Tensor ws = at::empty({p.ksplit, M, k}, gc.options().dtype(at::kFloat));
    a.out = ws.data_ptr();
    a.out_f32 = 1;
    a.ldo = (int)k;
    a.slab = M * k;
    illm::launch_mfgemm_nn((int)fmt, dense_bf16, t, a, p.ksplit, cur_stream());
    illm::launch_reduce_partials(out_bf16, ws.data_ptr<float>(), p.ksplit, nullptr, (uint16_t*)out.data_ptr(),
                                 (int)M, (int)k, (int)k, cur_stream());
    return out;
  }
  a.out = out.data_ptr();
  a.ldo = (int)k;
  illm::launch_mfgemm_nn((int)fmt, dense_bf16, t, a, 1, cur_stream());
  return out;
}

// ---- QLoRA linear: base GEMM over the low-bit blob with the adapter folded in
Tensor pad_rank(const Tensor& t, int64_t rp) {        // [rows, r] -> bf16 [rows, rp] zero-padded
  Tensor o = at::zeros({t.size(0), rp}, t.options().dtype(at::kBFloat16));
  o.narrow(1, 0, t.size(1)).copy_(t);
  return o;
}

// y = x W^T + s (x A^T) B^T over a low-bit W [n, k] (A [r, k], B [n, r] bf16):
// returns (y, xa) with xa = bf16(s x A^T) zero-padded to a multiple of 32
// columns (kept for the adapter gradients).  One pass over x makes the f16
// copy, its row scales and xa; the rank-r update runs as extra MFMA steps in
// the GEMM epilogue.
std::vector<Tensor> mfgemm_lora(const Tensor& x, const Tensor& w, int64_t fmt, int64_t n, int64_t k,
                                const c10::optional<Tensor>& bias, const Tensor& la, const Tensor& lb, double s) {
  TORCH_CHECK(fmt >= 0 && x.is_cuda() && w.scalar_type() == at::kByte, "mfgemm_lora: low-bit blob on the GPU");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.size(-1) == k && k % 128 == 0 && n % 16 == 0,
              "mfgemm_lora: bf16 x [.., k], k % 128 == 0, n % 16 == 0");
  TORCH_CHECK(la.dim() == 2 && lb.dim() == 2 && la.size(1) == k && lb.size(0) == n && la.size(0) == lb.size(1) &&
              la.size(0) <= 64, "mfgemm_lora: A [r, k], B [n, r], r <= 64");
  TORCH_CHECK(w.numel() >= illm::dev_total_bytes((int)fmt, n, k), "mfgemm_lora: weight blob too small");
  c10::DeviceGuard dg(x.device());
  Tensor xc = x.contiguous();
  const int64_t M = xc.numel() / k, r = la.size(0), rp = (r + 31) / 32 * 32;
  TORCH_CHECK((M + 256) * k * 2 < (int64_t)UINT32_MAX, "mfgemm_lora: activations too large");
  auto shape = xc.sizes().vec();
  shape.back() = n;
  Tensor out = at::empty(shape, xc.options());
  Tensor xa = at::empty({M, rp}, xc.options());
  if (M == 0) return {out, xa};
  Tensor x16 = at::empty({M, k}, xc.options().dtype(at::kHalf));
  Tensor rs = at::empty({M}, xc.options().dtype(at::kFloat));
  Tensor lac = la.to(at::kBFloat16).contiguous();
  illm::launch_x_rowscale_lora(true, (const uint16_t*)xc.data_ptr(), M, k, (int)k, (uint16_t*)x16.data_ptr(),
                               rs.data_ptr<float>(), (const uint16_t*)lac.data_ptr(), (int)r, (float)s,
                               (uint16_t*)xa.data_ptr(), (int)rp, cur_stream());
  Tensor lbp = pad_rank(lb, rp);
  illm::MfgArgs a{};
  a.x = (const uint16_t*)x16.data_ptr();
  a.M = (int)M;
  a.K = (int)k;
  a.ldx = (int)k;
  a.x_bytes = (uint32_t)(M * k * 2);
  a.rs = rs.data_ptr<float>();
  a.w = (const uint8_t*)w.data_ptr();
  a.N = (int)n;
  a.KC = (int)(k / 128);
  a.lut_fmt = (int)fmt;
  a.out_bf16 = 1;
  a.out = out.data_ptr();
  a.ldo = (int)n;
  Tensor bconv;
  if (bias.has_value() && bias->defined()) {
    bconv = bias->to(at::kBFloat16).contiguous();
    a.bias = (const uint16_t*)bconv.data_ptr();
    a.bias_bf16 = 1;
  }
  a.lora_x = (const uint16_t*)xa.data_ptr();
  a.lora_w = (const uint16_t*)lbp.data_ptr();
  a.lora_rp = (int)rp;
  const MfgPlan p = mfg_plan(M, n, k, -1, 1, false);
  a.sps = p.sps;
  illm::launch_mfgemm((int)fmt, false, p.tile, a, 1, cur_stream());
  return {out, xa};
}

// grad_x of the QLoRA linear: gx = g W + (s g B) A; returns (gx, gxa) with
// gxa = bf16(s g B) zero-padded to a multiple of 32 columns
std::vector<Tensor> mfgemm_nn_lora(const Tensor& g, const Tensor& w, int64_t fmt, int64_t n, int64_t k,
                                   const Tensor& la, const Tensor& lb, double s) {
  TORCH_CHECK(fmt >= 0 && g.is_cuda() && w.scalar_type() == at::kByte, "mfgemm_nn_lora: low-bit blob on the GPU");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 && g.size(-1) == n && n % 128 == 0 && k % 256 == 0,
              "mfgemm_nn_lora: bf16 g [.., n], n % 128 == 0, k % 256 == 0");
  TORCH_CHECK(la.dim() == 2 && lb.dim() == 2 && la.size(1) == k && lb.size(0) == n && la.size(0) == lb.size(1) &&
              la.size(0) <= 64, "mfgemm_nn_lora: A [r, k], B [n, r], r <= 64");
  c10::DeviceGuard dg(g.device());
  Tensor gc = g.contiguous();
  const int64_t M = gc.numel() / n, r = la.size(0), rp = (r + 31) / 32 * 32;
  TORCH_CHECK((M + 256) * n * 2 < (int64_t)UINT32_MAX, "mfgemm_nn_lora: g too large");
  auto shape = gc.sizes().vec();
  shape.back() = k;
  Tensor out = at::empty(shape, gc.options());
  Tensor gxa = at::empty({M, rp}, gc.options());
  if (M == 0) return {out, gxa};
  Tensor g16 = at::empty({M, n}, gc.options().dtype(at::kHalf));
  Tensor rs = at::empty({M}, gc.options().dtype(at::kFloat));
  Tensor bt = lb.to(at::kBFloat16).t().contiguous();                 // B^T [r, n]
  illm::launch_x_rowscale_lora(true, (const uint16_t*)gc.data_ptr(), M, n, (int)n, (uint16_t*)g16.data_ptr(),
                               rs.data_ptr<float>(), (const uint16_t*)bt.data_ptr(), (int)r, (float)s,
                               (uint16_t*)gxa.data_ptr(), (int)rp, cur_stream());
  Tensor lat = pad_rank(la.t(), rp);                                  // A^T [k, rp]
  illm::MfgArgs a{};
  a.x = (const uint16_t*)g16.data_ptr();
  a.M = (int)M;
  a.K = (int)n;
  a.ldx = (int)n;
  a.x_bytes = (uint32_t)(M * n * 2);
  a.rs = rs.data_ptr<float>();
  a.w = (const uint8_t*)w.data_ptr();
  a.N = (int)k;
  a.KC = (int)(k / 128);
  a.lut_fmt = (int)fmt;
  a.out_bf16 = 1;
  a.out = out.data_ptr();
  a.ldo = (int)k;
  a.lora_x = (const uint16_t*)gxa.data_ptr();
  a.lora_w = (const uint16_t*)lat.data_ptr();
  a.lora_rp = (int)rp;
  const MfgPlan p = mfg_plan(M, k, n, -1, 1, false);
  a.sps = p.sps;
  illm::launch_mfgemm_nn((int)fmt, false, p.tile == illm::MFG_TILE_128x256 ? 0 : p.tile, a, 1, cur_stream());
  return {out, gxa};
}

// (x16, rs) = per-row power-of-two normalisation of x to f16 (exposed for tests)
std::vector<Tensor> x_to_f16_rowscale(const Tensor& x) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.size(1) % 8 == 0, "x_to_f16_rowscale: 2-D GPU x, K % 8 == 0");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "x_to_f16_rowscale: bf16/fp16");
  c10::DeviceGuard g(x.device());
  Tensor xc = x.contiguous();
  Tensor y = at::empty(xc.sizes(), xc.options().dtype(at::kHalf));
  Tensor rs = at::empty({xc.size(0)}, xc.options().dtype(at::kFloat));
  illm::launch_x_to_f16_rowscale(xc.scalar_type() == at::kBFloat16, (const uint16_t*)xc.data_ptr(), xc.size(0),
                                 xc.size(1), (int)xc.size(1), (uint16_t*)y.data_ptr(), rs.data_ptr<float>(),
                                 cur_stream());
  return {y, rs};
}

}  // namespace

// dense bf16 NT GEMM on the 8-phase 256 x 256 kernel (gemm_8p.hip):
// split-K factor of the dense 8-phase GEMM: a grid of fewer 256 x 256 tiles
// than CUs (M = 1024: qkv / o / down give 64-96 tiles for 256 CUs) splits K
// so the launch fills the chip (gemm8p_auto_split); full grids keep 1
static int g8_auto_split(int64_t M, int64_t N, int64_t K) { return illm::gemm8p_auto_split(M, N, K / 64); }

// y[M, N] = x[M, K] @ w[N, K]^T (+ bias), bf16 or f32 out; K % 64 == 0.
// glu: w rows are 16-row gate/up tile pairs, y [M, N/2] = act(gate) * up.
// ksplit: -1 auto (g8_auto_split), 1 off, else the split-K factor.
// kernel: 0 (the 4-wave 128 x 128-per-wave variant measured 0.70-0.77x
// hipBLASLt in round 4 and was removed in round 5)
Tensor gemm_bf16(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, bool out_f32, int64_t kernel,
                 bool glu, int64_t act, int64_t ksplit, const c10::optional<Tensor>& out_opt, bool accumulate) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
              "gemm_bf16: bf16 GPU tensors");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1, "gemm_bf16: w must be [N, K] with unit inner stride");
  const int64_t K = w.size(1), N = w.size(0);
  TORCH_CHECK(x.size(-1) == K && K % 64 == 0 && K > 0, "gemm_bf16: K must match and be a multiple of 64");
  TORCH_CHECK(!glu || (N % 32 == 0 && !out_f32 && !bias.has_value()),
              "gemm_bf16: GLU needs N % 32 == 0, bf16 out, no bias");
  c10::DeviceGuard g(x.device());
  Tensor x2 = x.reshape({-1, K});
  if (x2.stride(1) != 1 || x2.stride(0) % 8 != 0) x2 = x2.contiguous();
  const int64_t M = x2.size(0);
  const int64_t NO = glu ? N / 2 : N;
  auto shape = x.sizes().vec();
  shape.back() = NO;
  Tensor out;
  int64_t ldo = NO;
  if (out_opt.has_value()) {
    // caller's buffer (a row slice of a larger tensor is fine): [M, NO], unit column stride
    out = *out_opt;
    TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.size(0) == M && out.size(1) == NO && out.stride(1) == 1 &&
                    out.scalar_type() == (out_f32 ? at::kFloat : at::kBFloat16),
                "gemm_bf16: out must be [M, N_out] with unit column stride and the output dtype");
    ldo = out.stride(0);
    // the epilogue writes while other workgroups still read the operands
    auto overlaps = [&](const Tensor& t) {
      const char* o0 = (const char*)out.data_ptr();
      const char* o1 = o0 + ((M - 1) * ldo + NO) * out.element_size();
      const char* t0 = (const char*)t.data_ptr();
      const char* t1 = t0 + t.numel() * t.element_size();
      return o0 < t1 && t0 < o1;
    };
    TORCH_CHECK(!overlaps(x2) && !overlaps(w), "gemm_bf16: out must not overlap x or w");
  } else {
    TORCH_CHECK(!accumulate, "gemm_bf16: accumulate needs out");
    out = at::empty({M, NO}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  }
  TORCH_CHECK(!accumulate || !glu, "gemm_bf16: accumulate: no GLU");
  if (M == 0 || N == 0) return out_opt.has_value() ? out : out.view(shape);
  TORCH_CHECK(w.stride(0) % 8 == 0, "gemm_bf16: w row stride must be a multiple of 8 elements");
  const int64_t xb = (M - 1) * x2.stride(0) * 2 + K * 2, wb = (N - 1) * w.stride(0) * 2 + K * 2;
  TORCH_CHECK(xb < (int64_t)UINT32_MAX && wb < (int64_t)UINT32_MAX, "gemm_bf16: operands over 4 GiB");
  if (bias.has_value())
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N && bias->is_contiguous(),
                "gemm_bf16: bias bf16 [N]");
  illm::G8Args a{};
  a.x = (const uint16_t*)x2.data_ptr();
  a.w = (const uint16_t*)w.data_ptr();
  a.bias = bias.has_value() ? (const uint16_t*)bias->data_ptr() : nullptr;
  a.out = out.data_ptr();
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.ldx = (int)x2.stride(0);
  a.ldw = (int)w.stride(0);
  a.ldo = (int)ldo;
  a.out_f32 = out_f32 ? 1 : 0;
  a.glu = glu ? 1 : 0;
  a.act = (int)act;
  a.accum = accumulate ? 1 : 0;
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)wb;
  a.w_fmt = -1;
  const auto st = at::hip::getCurrentHIPStream().stream();
  TORCH_CHECK(kernel == 0, "gemm_bf16: kernel must be 0");
  const int S = ksplit < 0 ? g8_auto_split(M, N, K) : (int)std::max<int64_t>(1, std::min<int64_t>(ksplit, K / 64));
  Tensor ws;
  if (S > 1) {
    ws = at::empty({(int64_t)S, M, N}, x.options().dtype(at::kFloat));
    a.ksplit = S;
    a.ws = ws.data_ptr<float>();
  }
  illm::launch_gemm8p(a, st);
  if (S > 1) illm::launch_gemm8p_finish(a, st);
  return out_opt.has_value() ? out : out.view(shape);
}

// low-bit weights (tiled device blob, sym_int4 / nf4 / nf3) decoded to bf16
// in LDS inside the same 8-phase GEMM: y = x @ dequant(W)^T (+ bias)
Tensor gemm8p_lowbit(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k,
                     const c10::optional<Tensor>& bias, bool out_f32, bool glu, int64_t act) {
  TORCH_CHECK(x.is_cuda() && blob.is_cuda() && x.scalar_type() == at::kBFloat16, "gemm8p_lowbit: bf16 x on the GPU");
  TORCH_CHECK(illm::gemm8p_supports((int)fmt), "gemm8p_lowbit: unsupported format ", fmt);
  TORCH_CHECK(x.size(-1) == k && k % 128 == 0 && k > 0, "gemm8p_lowbit: in_features must be a multiple of 128");
  TORCH_CHECK(blob.scalar_type() == at::kByte && blob.is_contiguous() &&
              blob.numel() >= illm::dev_total_bytes((int)fmt, n, k), "gemm8p_lowbit: weight blob too small");
  TORCH_CHECK(blob.numel() < (int64_t)UINT32_MAX, "gemm8p_lowbit: blob over 4 GiB");
  TORCH_CHECK(!glu || (n % 32 == 0 && !out_f32 && !bias.has_value()), "gemm8p_lowbit: GLU needs n % 32, bf16 out, no bias");
  c10::DeviceGuard g(x.device());
  Tensor x2 = x.reshape({-1, k});
  if (x2.stride(1) != 1 || x2.stride(0) % 8 != 0) x2 = x2.contiguous();
  const int64_t M = x2.size(0);
  const int64_t nout = glu ? n / 2 : n;
  auto shape = x.sizes().vec();
  shape.back() = nout;
  Tensor out = at::empty({M, nout}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  if (M == 0 || n == 0) return out.view(shape);
  const int64_t xb = (M - 1) * x2.stride(0) * 2 + k * 2;
  TORCH_CHECK(xb < (int64_t)UINT32_MAX, "gemm8p_lowbit: x over 4 GiB");
  if (bias.has_value())
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->numel() == n && bias->is_contiguous(),
                "gemm8p_lowbit: bias bf16 [n]");
  illm::G8Args a{};
  a.x = (const uint16_t*)x2.data_ptr();
  a.w = (const uint16_t*)blob.data_ptr();
  a.bias = bias.has_value() ? (const uint16_t*)bias->data_ptr() : nullptr;
  a.out = out.data_ptr();
  a.M = (int)M;
  a.N = (int)n;
  a.K = (int)k;
  a.ldx = (int)x2.stride(0);
  a.ldw = 0;
  a.ldo = (int)nout;
  a.glu = glu ? 1 : 0;
  a.act = (int)act;
  a.out_f32 = out_f32 ? 1 : 0;
  a.x_bytes = (uint32_t)xb;
  a.w_bytes = (uint32_t)blob.numel();
  a.w_fmt = (int)fmt;
  a.lut_fmt = (int)fmt;
  illm::launch_gemm8p(a, at::hip::getCurrentHIPStream().stream());
  return out.view(shape);
}

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("mfgemm(Tensor x, Tensor w, int fmt, int n, int k, Tensor? bias=None, bool glu=False, int act=0, int tile=-1, int ksplit=0) -> Tensor");
  m.def("x_to_f16_rowscale(Tensor x) -> Tensor[]");
  m.def("gemm_bf16(Tensor x, Tensor w, Tensor? bias=None, bool out_f32=False, int kernel=0, bool glu=False, int act=0, int ksplit=-1, Tensor(a!)? out=None, bool accumulate=False) -> Tensor");
  m.def("gemm8p_lowbit(Tensor x, Tensor blob, int fmt, int n, int k, Tensor? bias=None, bool out_f32=False, bool glu=False, int act=0) -> Tensor");
  m.def("mfgemm_nn(Tensor g, Tensor w, int fmt, int n, int k, int tile=-1, int ksplit=0) -> Tensor");
  m.def("mfgemm_lora(Tensor x, Tensor w, int fmt, int n, int k, Tensor? bias, Tensor la, Tensor lb, float s) -> Tensor[]");
  m.def("mfgemm_nn_lora(Tensor g, Tensor w, int fmt, int n, int k, Tensor la, Tensor lb, float s) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("mfgemm", &mfgemm);
  m.impl("x_to_f16_rowscale", &x_to_f16_rowscale);
  m.impl("gemm_bf16", &gemm_bf16);
  m.impl("gemm8p_lowbit", &gemm8p_lowbit);
  m.impl("mfgemm_nn", &mfgemm_nn);
  m.impl("mfgemm_lora", &mfgemm_lora);
  m.impl("mfgemm_nn_lora", &mfgemm_nn_lora);
}
