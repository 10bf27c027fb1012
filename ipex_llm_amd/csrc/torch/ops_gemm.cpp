// torch.library ops of the dense 8-phase GEMM (csrc/hip/gemm_8p.hip) and its
// in-LDS low-bit variant: prefill / training GEMMs.  (The round-4 MFMA GEMM
// engine, gemm_mfma*.hip, measured 0.63-0.88x dequantize + hipBLASLt and was
// removed in round 6: profiles/mfgemm_engine_sweep_r4.jsonl.)
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
  m.def("x_to_f16_rowscale(Tensor x) -> Tensor[]");
  m.def("gemm_bf16(Tensor x, Tensor w, Tensor? bias=None, bool out_f32=False, int kernel=0, bool glu=False, int act=0, int ksplit=-1, Tensor(a!)? out=None, bool accumulate=False) -> Tensor");
  m.def("gemm8p_lowbit(Tensor x, Tensor blob, int fmt, int n, int k, Tensor? bias=None, bool out_f32=False, bool glu=False, int act=0) -> Tensor");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("x_to_f16_rowscale", &x_to_f16_rowscale);
  m.impl("gemm_bf16", &gemm_bf16);
  m.impl("gemm8p_lowbit", &gemm8p_lowbit);
}
