// dense_linear(x, w, bias?): decode-size (<= 16 rows) projections over dense
// bf16 / fp16 weights on the streaming skinny-GEMM kernel (dense_gemv.hip);
// larger M and the host go to the library GEMM.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "../hip/kernels.h"

using at::Tensor;

namespace {

Tensor dense_linear_cpu(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias) {
  return at::linear(x, w.to(x.scalar_type()), bias.has_value() && bias->defined()
                                                  ? c10::optional<Tensor>(bias->to(x.scalar_type())) : c10::nullopt);
}

Tensor dense_linear_hip(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias) {
  c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "dense_linear: w must be [N, K]");
  const int64_t M = x.numel() / K;
  const bool ok = (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) &&
                  w.scalar_type() == x.scalar_type() && K % 8 == 0 && M <= 16 && w.is_contiguous();
  if (!ok) return dense_linear_cpu(x, w, bias);        // at::linear on the device (hipBLASLt)
  Tensor xc = x.contiguous();
  Tensor b;
  if (bias.has_value() && bias->defined()) b = bias->to(x.scalar_type()).contiguous();
  auto shape = x.sizes().vec();
  shape.back() = N;
  Tensor y = at::empty(shape, xc.options());
  if (M > 0)
    illm::launch_dense_gemv(x.scalar_type() == at::kBFloat16, (const uint16_t*)xc.data_ptr(), (int)M, K,
                            (const uint16_t*)w.data_ptr(), N, b.defined() ? (const uint16_t*)b.data_ptr() : nullptr,
                            (uint16_t*)y.data_ptr(), at::hip::getCurrentHIPStream().stream());
  return y;
}

// y^T = (x W^T)^T, [N, M]: the skinny GEMM with the roles swapped (training's
// rank-r projections x A^T: "x" = the r factor rows, "w" = the token rows)
// written straight in the caller's [tokens, r] layout; K % 64 == 0, <= 16 rows
Tensor dense_linear_t_hip(const Tensor& x, const Tensor& w) {
  c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), N = w.size(0);
  const int64_t M = x.numel() / K;
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && w.is_contiguous() && x.is_contiguous() && K % 64 == 0 && M <= 16 &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) &&
                  w.scalar_type() == x.scalar_type(),
              "dense_linear_t: one 16-bit dtype, contiguous, K % 64 == 0, <= 16 rows");
  Tensor y = at::empty({N, M}, x.options());
  if (M > 0 && N > 0)
    illm::launch_dense_gemv(x.scalar_type() == at::kBFloat16, (const uint16_t*)x.data_ptr(), (int)M, K,
                            (const uint16_t*)w.data_ptr(), N, nullptr, (uint16_t*)y.data_ptr(),
                            at::hip::getCurrentHIPStream().stream(), true);
  return y;
}

// act(x Wg^T) * (x Wu^T) over a 16-row tile-interleaved gate/up weight [2I, K]
Tensor dense_glu_hip(const Tensor& x, const Tensor& w, int64_t act) {
  c10::DeviceGuard g(x.device());
  const int64_t K = x.size(-1), I = w.size(0) / 2;
  const int64_t M = x.numel() / K;
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && w.size(0) % 32 == 0, "dense_glu: w must be [2I, K], 2I % 32 == 0");
  TORCH_CHECK((x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf) &&
                  w.scalar_type() == x.scalar_type() && K % 8 == 0 && M <= 16 && w.is_contiguous() &&
                  (act == 0 || act == 1),
              "dense_glu: one 16-bit dtype, K % 8 == 0, <= 16 rows, contiguous w, act 0/1");
  Tensor xc = x.contiguous();
  auto shape = x.sizes().vec();
  shape.back() = I;
  Tensor y = at::empty(shape, xc.options());
  if (M > 0)
    illm::launch_dense_glu(x.scalar_type() == at::kBFloat16, (const uint16_t*)xc.data_ptr(), (int)M, K,
                           (const uint16_t*)w.data_ptr(), I, (int)act, (uint16_t*)y.data_ptr(),
                           at::hip::getCurrentHIPStream().stream());
  return y;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("dense_linear(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("dense_glu(Tensor x, Tensor w, int act=0) -> Tensor");
  m.def("dense_linear_t(Tensor x, Tensor w) -> Tensor");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CPU, m) {
  m.impl("dense_linear", &dense_linear_cpu);
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("dense_linear", &dense_linear_hip);
  m.impl("dense_glu", &dense_glu_hip);
  m.impl("dense_linear_t", &dense_linear_t_hip);
}
