// torch.library ops of the training kernels (csrc/hip/train_kernels.hip).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "../hip/kernels.h"
#include "../hip/kernels_train.h"

using at::Tensor;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// fused softmax cross-entropy on a logits chunk [rows, V] (16-bit, rows
// contiguous): returns the per-row loss (f32, 0 for ignored rows) and, when
// grad_scale != 0, overwrites logits with (softmax - onehot) * grad_scale
Tensor ce_fused_(Tensor& logits, const Tensor& labels, int64_t ignore_index, double grad_scale) {
  TORCH_CHECK(logits.is_cuda() && labels.is_cuda(), "ce_fused_: GPU tensors expected");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.size(1) % 8 == 0 && logits.stride(0) % 8 == 0,
              "ce_fused_: logits [rows, V] with unit inner stride, V % 8 == 0");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kHalf, "ce_fused_: bf16/fp16");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0), "ce_fused_: int64 labels [rows]");
  c10::DeviceGuard g(logits.device());
  Tensor lab = labels.contiguous();
  Tensor loss = at::empty({logits.size(0)}, logits.options().dtype(at::kFloat));
  illm::launch_ce_fused(logits.scalar_type() == at::kBFloat16, (uint16_t*)logits.data_ptr(), logits.size(0),
                        logits.stride(0), (int)logits.size(1), lab.data_ptr<int64_t>(), (int)ignore_index,
                        (float)grad_scale, loss.data_ptr<float>(), grad_scale != 0.0, cur_stream());
  return loss;
}

// C[M, N] += alpha * A[M, r] @ B[N, r]^T in place (the LoRA rank-r term)
Tensor lora_update_(Tensor& C, const Tensor& A, const Tensor& B, double alpha) {
  TORCH_CHECK(C.is_cuda() && A.is_cuda() && B.is_cuda(), "lora_update_: GPU tensors expected");
  TORCH_CHECK(C.dim() == 2 && A.dim() == 2 && B.dim() == 2 && A.size(0) == C.size(0) && B.size(0) == C.size(1) &&
              A.size(1) == B.size(1), "lora_update_: C [M, N], A [M, r], B [N, r]");
  const int64_t r = A.size(1);
  TORCH_CHECK(r > 0 && r <= 64 && r % 8 == 0, "lora_update_: r % 8 == 0, r <= 64");
  TORCH_CHECK(C.scalar_type() == A.scalar_type() && C.scalar_type() == B.scalar_type() &&
              (C.scalar_type() == at::kBFloat16 || C.scalar_type() == at::kHalf), "lora_update_: one 16-bit dtype");
  TORCH_CHECK(C.stride(1) == 1 && C.stride(0) % 8 == 0 && C.size(1) % 8 == 0 && ((uintptr_t)C.data_ptr() & 15) == 0,
              "lora_update_: C rows 16-B aligned, N % 8 == 0");
  auto ok16 = [](const Tensor& t) {
    return t.stride(1) == 1 && t.stride(0) % 8 == 0 && ((uintptr_t)t.data_ptr() & 15) == 0;
  };
  TORCH_CHECK(ok16(A) && ok16(B), "lora_update_: A / B rows 16-B aligned with unit inner stride");
  c10::DeviceGuard g(C.device());
  if (C.numel() == 0) return C;
  illm::launch_lora_update(C.scalar_type() == at::kBFloat16, (uint16_t*)C.data_ptr(), C.stride(0),
                           (const uint16_t*)A.data_ptr(), A.stride(0), (const uint16_t*)B.data_ptr(), B.stride(0),
                           (int)C.size(0), (int)C.size(1), (int)r, (float)alpha, cur_stream());
  return C;
}

// out[r, n] = alpha * sum_m a[m, r] * b[m, n] on the MFMA token-axis reduction
// (a [M, r], b [M, N] one 16-bit dtype) -> f32 [r, N]
static void lora_tn_check(const Tensor& a, const Tensor& b) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.dim() == 2 && b.dim() == 2 && a.size(0) == b.size(0),
              "lora_tn: a [M, r], b [M, N] GPU tensors");
  const int64_t r = a.size(1), N = b.size(1);
  TORCH_CHECK(r > 0 && r <= 64 && r % 8 == 0 && N % 8 == 0, "lora_tn: r % 8 == 0, r <= 64, N % 8 == 0");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf),
              "lora_tn: one 16-bit dtype");
  auto ok16 = [](const Tensor& t) {
    return t.stride(1) == 1 && t.stride(0) % 8 == 0 && ((uintptr_t)t.data_ptr() & 15) == 0;
  };
  TORCH_CHECK(ok16(a) && ok16(b), "lora_tn: rows 16-B aligned with unit inner stride");
}

static void lora_tn_launch(const Tensor& a, const Tensor& b, double alpha, Tensor& out, bool trans) {
  if (a.size(0) == 0) return;
  c10::DeviceGuard g(a.device());
  illm::launch_lora_tn(a.scalar_type() == at::kBFloat16, (const uint16_t*)a.data_ptr(), a.stride(0), (int)a.size(1),
                       (const uint16_t*)b.data_ptr(), b.stride(0), (int)a.size(0), (int)b.size(1), (float)alpha,
                       out.data_ptr<float>(), trans, cur_stream());
}

Tensor lora_tn(const Tensor& a, const Tensor& b, double alpha) {
  lora_tn_check(a, b);
  Tensor out = at::zeros({a.size(1), b.size(1)}, a.options().dtype(at::kFloat));
  lora_tn_launch(a, b, alpha, out, false);
  return out;
}

// accumulate alpha a^T b into a caller-zeroed contiguous f32 region: [r, N],
// or [N, r] with trans (several gradients share one zero fill and one cast)
Tensor& lora_tn_acc_(Tensor& out, const Tensor& a, const Tensor& b, double alpha, bool trans) {
  lora_tn_check(a, b);
  const int64_t r = a.size(1), N = b.size(1);
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 2 &&
                  out.size(0) == (trans ? N : r) && out.size(1) == (trans ? r : N),
              "lora_tn_acc_: out must be a contiguous f32 ", trans ? "[N, r]" : "[r, N]", " tensor");
  lora_tn_launch(a, b, alpha, out, trans);
  return out;
}

// out[r, n] = alpha * sum_m a[m, r] * b[m, n]  (a [M, R] f32, R <= 64; b [M, N] 16-bit) -> f32 [R, N]
Tensor skinny_tn(const Tensor& a, const Tensor& b, double alpha) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "skinny_tn: GPU tensors expected");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(0) == b.size(0), "skinny_tn: a [M, R], b [M, N]");
  TORCH_CHECK(a.size(1) <= 64 && b.size(1) % 8 == 0, "skinny_tn: R <= 64, N % 8 == 0");
  TORCH_CHECK(b.scalar_type() == at::kBFloat16 || b.scalar_type() == at::kHalf, "skinny_tn: 16-bit b");
  c10::DeviceGuard g(a.device());
  Tensor af = a.to(at::kFloat).contiguous();
  Tensor bc = b.stride(1) == 1 && b.stride(0) % 8 == 0 ? b : b.contiguous();
  Tensor out = at::zeros({a.size(1), b.size(1)}, a.options().dtype(at::kFloat));
  if (a.size(0) == 0) return out;
  illm::launch_skinny_tn(bc.scalar_type() == at::kBFloat16, af.data_ptr<float>(), (int)a.size(1),
                         (const uint16_t*)bc.data_ptr(), bc.stride(0), (int)a.size(0), (int)b.size(1), (float)alpha,
                         out.data_ptr<float>(), cur_stream());
  return out;
}

void check_bhtd(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.stride(3) == 1, name, ": [B, H, T, D] GPU tensor, unit inner stride");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, name, ": bf16/fp16");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0, name, ": 16-B aligned rows");
}

illm::TrainAttnArgs attn_args(const Tensor& q, const Tensor& k, const Tensor& v, double scale, bool causal,
                              bool ragged_ok = false) {
  check_bhtd(q, "q");
  check_bhtd(k, "k");
  check_bhtd(v, "v");
  const int64_t B = q.size(0), Hq = q.size(1), T = q.size(2), D = q.size(3), Hkv = k.size(1);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && k.size(2) == T && v.size(2) == T && k.size(3) == D &&
              v.size(3) == D && v.size(1) == Hkv && Hq % Hkv == 0, "train attention: shapes");
  TORCH_CHECK((ragged_ok ? T > 0 : T % 64 == 0) && (D == 64 || D == 128),
              "train attention: T % 64 == 0 (backward) / T > 0 (forward), D in {64, 128}");
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type(), "train attention: dtypes");
  illm::TrainAttnArgs a{};
  a.q = (const uint16_t*)q.data_ptr();
  a.qsb = q.stride(0); a.qsh = q.stride(1); a.qst = q.stride(2);
  a.k = (const uint16_t*)k.data_ptr();
  a.ksb = k.stride(0); a.ksh = k.stride(1); a.kst = k.stride(2);
  a.v = (const uint16_t*)v.data_ptr();
  a.vsb = v.stride(0); a.vsh = v.stride(1); a.vst = v.stride(2);
  a.B = (int)B; a.T = (int)T; a.Hq = (int)Hq; a.Hkv = (int)Hkv; a.D = (int)D;
  a.scale = (float)scale;
  a.causal = causal ? 1 : 0;
  return a;
}

// flash attention forward for training: (out [B, T, Hq, D], lse [B, Hq, T] log2 domain)
std::vector<Tensor> train_attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, double scale, bool causal) {
  c10::DeviceGuard g(q.device());
  illm::TrainAttnArgs a = attn_args(q, k, v, scale, causal, true);
  Tensor out = at::empty({q.size(0), q.size(2), q.size(1), q.size(3)}, q.options());
  Tensor lse = at::empty({q.size(0), q.size(1), q.size(2)}, q.options().dtype(at::kFloat));
  a.out = (uint16_t*)out.data_ptr();
  a.lse = lse.data_ptr<float>();
  illm::launch_train_attn_fwd(q.scalar_type() == at::kBFloat16, a, cur_stream());
  return {out, lse};
}

// backward: (dq [B, Hq, T, D], dk, dv [B, Hkv, T, D]); out / dout [B, T, Hq, D]
std::vector<Tensor> train_attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& out,
                                   const Tensor& lse, const Tensor& dout, double scale, bool causal) {
  c10::DeviceGuard g(q.device());
  illm::TrainAttnArgs a = attn_args(q, k, v, scale, causal);
  TORCH_CHECK(out.dim() == 4 && dout.dim() == 4 && out.sizes() == dout.sizes() && out.size(0) == q.size(0) &&
              out.size(1) == q.size(2) && out.size(2) == q.size(1) && out.size(3) == q.size(3),
              "train_attn_bwd: out / dout [B, T, Hq, D]");
  TORCH_CHECK(out.stride(3) == 1 && dout.stride(3) == 1 && out.scalar_type() == q.scalar_type() &&
              dout.scalar_type() == q.scalar_type(), "train_attn_bwd: out / dout layout / dtype");
  TORCH_CHECK(lse.is_contiguous() && lse.scalar_type() == at::kFloat && lse.numel() == q.size(0) * q.size(1) * q.size(2),
              "train_attn_bwd: lse [B, Hq, T] f32");
  Tensor dc = dout.stride(0) % 8 == 0 && dout.stride(1) % 8 == 0 && dout.stride(2) % 8 == 0 ? dout : dout.contiguous();
  a.o = (const uint16_t*)out.data_ptr();
  a.osb = out.stride(0); a.ost = out.stride(1); a.osh = out.stride(2);
  a.dout = (const uint16_t*)dc.data_ptr();
  a.dsb = dc.stride(0); a.dst = dc.stride(1); a.dsh = dc.stride(2);
  a.lse = (float*)lse.data_ptr<float>();
  Tensor delta = at::empty_like(lse);
  a.delta = delta.data_ptr<float>();
  Tensor dq = at::empty({q.size(0), q.size(1), q.size(2), q.size(3)}, q.options());
  Tensor dk = at::empty({k.size(0), k.size(1), k.size(2), k.size(3)}, k.options());
  Tensor dv = at::empty({v.size(0), v.size(1), v.size(2), v.size(3)}, v.options());
  a.dq = (uint16_t*)dq.data_ptr();
  a.dk = (uint16_t*)dk.data_ptr();
  a.dv = (uint16_t*)dv.data_ptr();
  illm::launch_train_attn_bwd(q.scalar_type() == at::kBFloat16, a, cur_stream());
  return {dq, dk, dv};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("train_attn_fwd(Tensor q, Tensor k, Tensor v, float scale, bool causal=True) -> Tensor[]");
  m.def("train_attn_bwd(Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, Tensor dout, float scale, bool causal=True) -> Tensor[]");
  m.def("ce_fused_(Tensor(a!) logits, Tensor labels, int ignore_index=-100, float grad_scale=0.0) -> Tensor");
  m.def("skinny_tn(Tensor a, Tensor b, float alpha=1.0) -> Tensor");
  m.def("lora_update_(Tensor(a!) c, Tensor a, Tensor b, float alpha=1.0) -> Tensor(a!)");
  m.def("lora_tn(Tensor a, Tensor b, float alpha=1.0) -> Tensor");
  m.def("lora_tn_acc_(Tensor(a!) out, Tensor a, Tensor b, float alpha=1.0, bool trans=False) -> Tensor(a!)");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("ce_fused_", &ce_fused_);
  m.impl("skinny_tn", &skinny_tn);
  m.impl("lora_update_", &lora_update_);
  m.impl("lora_tn", &lora_tn);
  m.impl("lora_tn_acc_", &lora_tn_acc_);
  m.impl("train_attn_fwd", &train_attn_fwd);
  m.impl("train_attn_bwd", &train_attn_bwd);
}
