// torch.library ops of the k-quant formats (q4_K / q5_K / q6_K / q2_K):
//   kq_quantize(w f32 [n, k] CPU, fmt, imatrix?) -> uint8 GGUF blocks
//   kq_dequantize(blob, fmt, n, k, dtype) -> [n, k]   (CPU: C++, GPU: HIP)
//   kq_linear(x, blob, fmt, n, k) -> x @ W^T          (GPU: HIP GEMV for <= 8
//                                                      rows, else dequant + BLAS;
//                                                      CPU: C++ f32 GEMM)
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "../common/kquant.h"
#include "../cpu/quant_api.h"
#include "../hip/kernels.h"

using at::Tensor;

namespace {

void check_kq(int64_t fmt, int64_t k) {
  TORCH_CHECK(illm::is_kq((int)fmt), "k-quant op: fmt ", fmt, " is not a k-quant format");
  TORCH_CHECK(k % illm::QK_K == 0, "k-quant formats need in_features % 256 == 0, got ", k);
}

Tensor kq_quantize(const Tensor& w, int64_t fmt, const c10::optional<Tensor>& imatrix) {
  TORCH_CHECK(w.dim() == 2, "kq_quantize: [n, k] weight");
  check_kq(fmt, w.size(1));
  Tensor wc = w.to(at::kCPU, at::kFloat).contiguous();
  const int64_t n = wc.size(0), k = wc.size(1);
  Tensor out = at::empty({illm::kq_total_bytes((int)fmt, n, k)}, wc.options().dtype(at::kByte));
  Tensor im;
  if (imatrix.has_value() && imatrix->defined()) {
    im = imatrix->to(at::kCPU, at::kFloat).contiguous();
    TORCH_CHECK(im.numel() == k, "kq_quantize: imatrix must have in_features entries");
  }
  illm_kq_quantize((int)fmt, wc.data_ptr<float>(), n, k, im.defined() ? im.data_ptr<float>() : nullptr,
                   out.data_ptr<uint8_t>());
  return out;
}

Tensor kq_dequantize_cpu(const Tensor& blob, int64_t fmt, int64_t n, int64_t k, at::ScalarType dt) {
  check_kq(fmt, k);
  TORCH_CHECK(blob.numel() == illm::kq_total_bytes((int)fmt, n, k), "kq_dequantize: blob size");
  Tensor b = blob.contiguous();
  Tensor out = at::empty({n, k}, b.options().dtype(at::kFloat));
  illm_kq_dequantize((int)fmt, b.data_ptr<uint8_t>(), n, k, out.data_ptr<float>());
  return out.to(dt);
}

Tensor kq_dequantize_hip(const Tensor& blob, int64_t fmt, int64_t n, int64_t k, at::ScalarType dt) {
  check_kq(fmt, k);
  TORCH_CHECK(blob.numel() == illm::kq_total_bytes((int)fmt, n, k), "kq_dequantize: blob size");
  c10::DeviceGuard g(blob.device());
  const bool bf16 = dt != at::kHalf;
  Tensor out = at::empty({n, k}, blob.options().dtype(bf16 ? at::kBFloat16 : at::kHalf));
  illm::launch_kq_dequant((int)fmt, bf16, blob.data_ptr<uint8_t>(), n, k, (uint16_t*)out.data_ptr(),
                          at::hip::getCurrentHIPStream().stream());
  return dt == at::kFloat ? out.to(at::kFloat) : out;
}

// isa: 0 = auto (integer dots below 512 rows, dequantize + GEMM above -- the
// reference's BIGDL_LLM_LINEAR_THRESHOLD split), 1 = integer AVX2, 2 = integer
// AVX-512 VNNI, 3 = f32 row-dequant reference
Tensor kq_linear_isa(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t isa) {
  check_kq(fmt, k);
  TORCH_CHECK(x.size(-1) == k && blob.numel() == illm::kq_total_bytes((int)fmt, n, k), "kq_linear: shapes");
  Tensor xc = x.to(at::kFloat).contiguous();
  const int64_t m = xc.numel() / k;
  auto shape = x.sizes().vec();
  shape.back() = n;
  Tensor bc = blob.contiguous();
  if (isa == 0 && m >= 512) {
    Tensor w = at::empty({n, k}, xc.options());
    illm_kq_dequantize((int)fmt, bc.data_ptr<uint8_t>(), n, k, w.data_ptr<float>());
    return at::matmul(xc, w.t()).view(shape).to(x.scalar_type());
  }
  Tensor y = at::empty(shape, xc.options());
  if (isa == 3) illm_kq_gemm((int)fmt, xc.data_ptr<float>(), m, bc.data_ptr<uint8_t>(), n, k, y.data_ptr<float>());
  else illm_kq_gemm_int((int)fmt, xc.data_ptr<float>(), m, bc.data_ptr<uint8_t>(), n, k, y.data_ptr<float>(), (int)isa);
  return y.to(x.scalar_type());
}

Tensor kq_linear_cpu(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k) {
  return kq_linear_isa(x, blob, fmt, n, k, 0);
}

Tensor kq_linear_hip(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k) {
  check_kq(fmt, k);
  TORCH_CHECK(x.size(-1) == k && blob.numel() == illm::kq_total_bytes((int)fmt, n, k), "kq_linear: shapes");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "kq_linear: bf16/fp16 activations");
  c10::DeviceGuard g(x.device());
  Tensor xc = x.contiguous();
  const int64_t m = xc.numel() / k;
  const bool bf16 = xc.scalar_type() == at::kBFloat16;
  auto shape = x.sizes().vec();
  shape.back() = n;
  if (m <= 8) {
    Tensor y = at::empty(shape, xc.options());
    if (m > 0)
      illm::launch_kq_gemv((int)fmt, bf16, (const uint16_t*)xc.data_ptr(), (int)m, k, blob.data_ptr<uint8_t>(), n,
                           (uint16_t*)y.data_ptr(), at::hip::getCurrentHIPStream().stream());
    return y;
  }
  // prefill: dequantize once, library GEMM
  Tensor w = kq_dequantize_hip(blob, fmt, n, k, xc.scalar_type());
  return at::matmul(xc, w.t()).view(shape);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("kq_quantize(Tensor w, int fmt, Tensor? imatrix) -> Tensor", &kq_quantize);
  m.def("kq_dequantize(Tensor blob, int fmt, int n, int k, ScalarType dtype) -> Tensor");
  m.def("kq_linear(Tensor x, Tensor blob, int fmt, int n, int k) -> Tensor");
  m.def("kq_linear_isa(Tensor x, Tensor blob, int fmt, int n, int k, int isa) -> Tensor", &kq_linear_isa);
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CPU, m) {
  m.impl("kq_dequantize", &kq_dequantize_cpu);
  m.impl("kq_linear", &kq_linear_cpu);
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("kq_dequantize", &kq_dequantize_hip);
  m.impl("kq_linear", &kq_linear_hip);
}
