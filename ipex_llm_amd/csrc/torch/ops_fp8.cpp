// torch.library ops of the torch_fp8 qtypes (reference run_linear_fp8 /
// dynamic_scaled_fp8_quant, SRC/transformers/low_bit_linear.py:168-178, 692-696):
//   fp8_act_quant(x) -> (xq uint8 e4m3 [M, K], sx f32 [M])   per-token scales
//   fp8_linear(x, w uint8 [N, K], w_scale f32 [1]|[N], bias?, e5m2) -> y
// GPU: M <= 16 streams the fp8 weight against bf16/f16 x (GEMV); larger M
// quantizes x per token and runs the block-scaled f8f6f4 MFMA GEMM.
// CPU: the same math in f32 (x quantized per token through e4m3 exactly like
// the GPU prefill path), the numerics reference of the GPU tests.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "../hip/kernels.h"
#include "../hip/kernels_g8.h"

using at::Tensor;

namespace {

void check_w(const Tensor& x, const Tensor& w, const Tensor& ws) {
  TORCH_CHECK(w.dim() == 2 && w.scalar_type() == at::kByte, "fp8_linear: w must be uint8 [N, K] fp8 codes");
  TORCH_CHECK(x.size(-1) == w.size(1), "fp8_linear: x last dim != K");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && (ws.numel() == 1 || ws.numel() == w.size(0)),
              "fp8_linear: w_scale must be f32 [1] or [N]");
}

Tensor decode_w(const Tensor& w, bool e5m2) {
  return w.view(e5m2 ? at::kFloat8_e5m2 : at::kFloat8_e4m3fn).to(at::kFloat);
}

std::tuple<Tensor, Tensor> act_quant_ref(const Tensor& x2) {
  Tensor xf = x2.to(at::kFloat);
  Tensor amax = xf.abs().amax({1}, true);
  Tensor sx = at::where(amax > 0, amax / 448.0, at::ones_like(amax));
  Tensor q = (xf / sx).clamp(-448.0, 448.0).to(at::kFloat8_e4m3fn);
  return {q.view(at::kByte), sx.view({-1})};
}

std::tuple<Tensor, Tensor> fp8_act_quant_cpu(const Tensor& x) {
  Tensor x2 = x.reshape({-1, x.size(-1)});
  return act_quant_ref(x2);
}

std::tuple<Tensor, Tensor> fp8_act_quant_hip(const Tensor& x) {
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "fp8_act_quant: bf16/f16 x");
  Tensor x2 = x.reshape({-1, x.size(-1)}).contiguous();
  const int64_t M = x2.size(0), K = x2.size(1);
  TORCH_CHECK(K % 8 == 0, "fp8_act_quant: K % 8 != 0");
  Tensor xq = at::empty({M, K}, x2.options().dtype(at::kByte));
  Tensor sx = at::empty({M}, x2.options().dtype(at::kFloat));
  if (M > 0)
    illm::launch_fp8_act_quant(x2.scalar_type() == at::kBFloat16, (const uint16_t*)x2.data_ptr(), M, K,
                               xq.data_ptr<uint8_t>(), sx.data_ptr<float>(), at::hip::getCurrentHIPStream().stream());
  return {xq, sx};
}

Tensor fp8_linear_cpu(const Tensor& x, const Tensor& w, const Tensor& w_scale, const c10::optional<Tensor>& bias,
                      bool e5m2) {
  check_w(x, w, w_scale);
  Tensor x2 = x.reshape({-1, x.size(-1)});
  auto [xq, sx] = act_quant_ref(x2);
  Tensor xf = xq.view(at::kFloat8_e4m3fn).to(at::kFloat) * sx.view({-1, 1});
  Tensor y = at::matmul(xf, decode_w(w, e5m2).t()) * w_scale.view({1, -1});
  if (bias.has_value() && bias->defined()) y = y + bias->to(at::kFloat);
  auto shape = x.sizes().vec();
  shape.back() = w.size(0);
  return y.to(x.scalar_type()).view(shape);
}

// the 8-phase 256 x 256 GEMM (gemm_8p.hip) on fp8 operands: 128 k per K-tile,
// v_mfma_scale_f32_16x16x128_f8f6f4, row / column scales in the epilogue
// (ILLM_FP8_8P=0: the older 128 x 128 kernel)
static bool fp8_8p_on() {
  static const bool on = [] {
    const char* e = getenv("ILLM_FP8_8P");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

static void launch_fp8_8p(const Tensor& xq, const Tensor& sx, const Tensor& w, const Tensor& ws, const Tensor& b,
                          bool e5m2, Tensor& y) {
  const int64_t M = xq.size(0), K = xq.size(1), N = w.size(0);
  TORCH_CHECK(M * K < (int64_t)UINT32_MAX && N * K < (int64_t)UINT32_MAX, "fp8 8p: operands over 4 GiB");
  illm::G8Args a{};
  a.x = (const uint16_t*)xq.data_ptr();
  a.w = (const uint16_t*)w.data_ptr();
  a.bias = b.defined() ? (const uint16_t*)b.data_ptr() : nullptr;
  a.out = y.data_ptr();
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.ldx = (int)K;
  a.ldw = (int)K;
  a.ldo = (int)N;
  a.x_bytes = (uint32_t)(M * K);
  a.w_bytes = (uint32_t)(N * K);
  a.w_fmt = illm::G8_FP8;
  a.sx = sx.data_ptr<float>();
  a.sw = ws.data_ptr<float>();
  a.sw_per_channel = ws.numel() == N ? 1 : 0;
  a.w_e5m2 = e5m2 ? 1 : 0;
  a.out_f16 = y.scalar_type() == at::kHalf ? 1 : 0;
  const auto st = at::hip::getCurrentHIPStream().stream();
  // grids smaller than the chip (M = 1024: qkv / o / down) split K into f32
  // slabs reduced (with the scales, bias, rounding) by the finishing launch
  const int S = illm::gemm8p_auto_split(M, N, K / 128);
  Tensor slabs;
  if (S > 1) {
    slabs = at::empty({(int64_t)S, M, N}, y.options().dtype(at::kFloat));
    a.ksplit = S;
    a.ws = slabs.data_ptr<float>();
  }
  illm::launch_gemm8p(a, st);
  if (S > 1) illm::launch_gemm8p_finish(a, st);
}

// kernel-only entry for benchmarks: pre-quantized activations
Tensor fp8_gemm8p(const Tensor& xq, const Tensor& sx, const Tensor& w, const Tensor& ws, bool e5m2) {
  TORCH_CHECK(xq.is_cuda() && xq.dim() == 2 && xq.is_contiguous() && xq.element_size() == 1, "fp8_gemm8p: xq [M, K] bytes");
  TORCH_CHECK(w.is_cuda() && w.dim() == 2 && w.is_contiguous() && w.size(1) == xq.size(1) && xq.size(1) % 128 == 0,
              "fp8_gemm8p: w [N, K] bytes, K % 128 == 0");
  TORCH_CHECK(sx.scalar_type() == at::kFloat && sx.numel() == xq.size(0) && ws.scalar_type() == at::kFloat,
              "fp8_gemm8p: f32 scales");
  c10::DeviceGuard g(xq.device());
  Tensor y = at::empty({xq.size(0), w.size(0)}, xq.options().dtype(at::kBFloat16));
  if (xq.size(0) > 0) launch_fp8_8p(xq, sx.contiguous(), w, ws.contiguous(), Tensor(), e5m2, y);
  return y;
}

Tensor fp8_linear_hip(const Tensor& x, const Tensor& w, const Tensor& w_scale, const c10::optional<Tensor>& bias,
                      bool e5m2) {
  check_w(x, w, w_scale);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "fp8_linear: bf16/f16 x");
  c10::DeviceGuard g(x.device());
  Tensor x2 = x.reshape({-1, x.size(-1)}).contiguous();
  const int64_t M = x2.size(0), K = x2.size(1), N = w.size(0);
  const bool bf16 = x2.scalar_type() == at::kBFloat16;
  auto shape = x.sizes().vec();
  shape.back() = N;
  Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->to(x2.scalar_type()).contiguous();
    TORCH_CHECK(b.numel() == N && b.is_cuda(), "fp8_linear: bias [N] on the device");
  }
  Tensor wc = w.contiguous(), ws = w_scale.contiguous();
  TORCH_CHECK(wc.is_cuda() && ws.is_cuda(), "fp8_linear: weight / scale on the device");
  Tensor y = at::empty({M, N}, x2.options());
  if (M == 0) return y.view(shape);
  illm::Fp8GemmArgs a{};
  a.w = wc.data_ptr<uint8_t>();
  a.sw = ws.data_ptr<float>();
  a.sw_per_channel = ws.numel() == N ? 1 : 0;
  a.bias = b.defined() ? (const uint16_t*)b.data_ptr() : nullptr;
  a.out = (uint16_t*)y.data_ptr();
  a.M = (int)M;
  a.N = (int)N;
  a.K = K;
  auto st = at::hip::getCurrentHIPStream().stream();
  if (M <= 16 && K % 16 == 0) {
    a.x = (const uint16_t*)x2.data_ptr();
    illm::launch_fp8_gemv(bf16, e5m2, a, st);
    return y.view(shape);
  }
  if (K % 128 == 0 && M >= 256 && fp8_8p_on()) {
    auto [xq, sx] = fp8_act_quant_hip(x2);
    launch_fp8_8p(xq, sx, wc, ws, b, e5m2, y);
    return y.view(shape);
  }
  if (N % 128 == 0 && K % 128 == 0) {
    auto [xq, sx] = fp8_act_quant_hip(x2);
    a.xq = xq.data_ptr<uint8_t>();
    a.sx = sx.data_ptr<float>();
    illm::launch_fp8_gemm(bf16, e5m2, a, st);
    return y.view(shape);
  }
  // odd shapes: decode the weight once, library GEMM
  Tensor wd = (decode_w(wc, e5m2) * ws.view({-1, 1})).to(x2.scalar_type());
  Tensor r = at::matmul(x2, wd.t());
  if (b.defined()) r = r + b;
  return r.view(shape);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("fp8_act_quant(Tensor x) -> (Tensor, Tensor)");
  m.def("fp8_linear(Tensor x, Tensor w, Tensor w_scale, Tensor? bias, bool e5m2) -> Tensor");
  m.def("fp8_gemm8p(Tensor xq, Tensor sx, Tensor w, Tensor ws, bool e5m2) -> Tensor");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CPU, m) {
  m.impl("fp8_act_quant", &fp8_act_quant_cpu);
  m.impl("fp8_linear", &fp8_linear_cpu);
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("fp8_act_quant", &fp8_act_quant_hip);
  m.impl("fp8_linear", &fp8_linear_hip);
  m.impl("fp8_gemm8p", &fp8_gemm8p);
}
