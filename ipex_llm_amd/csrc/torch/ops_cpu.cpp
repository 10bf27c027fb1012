// torch.library registration of the ipex_llm_amd op namespace + CPU impls.
// GPU impls live in ops_hip.cpp; meta ("fake") impls are registered from
// Python (ipex_llm_amd/ops/_meta.py) for torch.compile / graph tracing.
#include <ATen/ATen.h>
#include <torch/library.h>

#include "../common/formats.h"
#include "../cpu/quant_api.h"

using at::Tensor;

namespace {

void check_fmt(int64_t fmt) { TORCH_CHECK(fmt >= 0 && fmt < illm::FMT_COUNT, "bad low-bit fmt ", fmt); }

struct Planes {
  uint8_t* codes;
  uint16_t* scales;
  uint16_t* mins;
};
Planes canon_planes(const Tensor& blob, int64_t fmt, int64_t n, int64_t k) {
  uint8_t* b = blob.data_ptr<uint8_t>();
  Planes p;
  p.codes = b;
  p.scales = (uint16_t*)(b + illm::canon_code_bytes((int)fmt, n, k));
  p.mins = illm::fmt_has_min((int)fmt) ? p.scales + illm::canon_scale_elems(n, k) : nullptr;
  return p;
}

Tensor quantize_cpu(const Tensor& w, int64_t fmt, const c10::optional<Tensor>& imatrix,
                    bool scale_search) {
  check_fmt(fmt);
  TORCH_CHECK(w.dim() == 2, "quantize expects [n, k]");
  const int64_t n = w.size(0), k = w.size(1);
  TORCH_CHECK(k % illm::QBLOCK == 0, "in_features must be a multiple of ", illm::QBLOCK);
  Tensor wf = w.to(at::kFloat).contiguous();
  Tensor blob = at::empty({illm::canon_total_bytes((int)fmt, n, k)}, w.options().dtype(at::kByte));
  Planes p = canon_planes(blob, fmt, n, k);
  Tensor im;
  const float* imp = nullptr;
  if (imatrix.has_value() && imatrix->defined()) {
    im = imatrix->to(at::kFloat).contiguous();
    TORCH_CHECK(im.numel() == k, "imatrix must have in_features elements");
    imp = im.data_ptr<float>();
  }
  illm_quantize((int)fmt, wf.data_ptr<float>(), n, k, imp, scale_search ? 1 : 0, p.codes, p.scales,
                p.mins);
  return blob;
}

Tensor dequantize_cpu(const Tensor& blob, int64_t fmt, int64_t n, int64_t k) {
  check_fmt(fmt);
  Tensor b = blob.contiguous();
  TORCH_CHECK(b.numel() >= illm::canon_total_bytes((int)fmt, n, k), "blob too small");
  Planes p = canon_planes(b, fmt, n, k);
  Tensor out = at::empty({n, k}, b.options().dtype(at::kFloat));
  illm_dequantize((int)fmt, p.codes, p.scales, p.mins, n, k, out.data_ptr<float>());
  return out;
}

Tensor repack_to_device(const Tensor& canon, int64_t fmt, int64_t n, int64_t k) {
  check_fmt(fmt);
  Tensor b = canon.contiguous();
  Planes p = canon_planes(b, fmt, n, k);
  Tensor dev = at::zeros({illm::dev_total_bytes((int)fmt, n, k)}, b.options());
  illm_repack_to_device((int)fmt, p.codes, p.scales, p.mins, n, k, dev.data_ptr<uint8_t>());
  return dev;
}

Tensor repack_from_device(const Tensor& dev, int64_t fmt, int64_t n, int64_t k) {
  check_fmt(fmt);
  Tensor d = dev.contiguous();
  Tensor canon = at::zeros({illm::canon_total_bytes((int)fmt, n, k)}, d.options());
  Planes p = canon_planes(canon, fmt, n, k);
  illm_repack_from_device((int)fmt, d.data_ptr<uint8_t>(), n, k, p.codes, p.scales, p.mins);
  return canon;
}

Tensor linear_cpu_isa(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t isa_req);

Tensor linear_cpu(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k) {
  static const int isa = getenv("ILLM_CPU_ISA") ? atoi(getenv("ILLM_CPU_ISA")) : 0;
  return linear_cpu_isa(x, blob, fmt, n, k, isa);
}

// isa: 0 auto, 1 AVX2, 2 AVX-512 (VNNI for the integer formats), -1 the
// portable per-block dequant-dot loop (tests pin every path)
Tensor linear_cpu_isa(const Tensor& x, const Tensor& blob, int64_t fmt, int64_t n, int64_t k, int64_t isa_req) {
  check_fmt(fmt);
  TORCH_CHECK(x.size(-1) == k, "x last dim must equal in_features");
  Tensor xf = x.reshape({-1, k}).to(at::kFloat).contiguous();
  Tensor b = blob.contiguous();
  Planes p = canon_planes(b, fmt, n, k);
  const int64_t M = xf.size(0);
  // rows above this take dequantize + BLAS (reference: BIGDL_LLM_LINEAR_THRESHOLD,
  // low_bit_linear.py:64); below it the int8-activation integer-dot kernels
  static const int64_t thr = [] {
    const char* e = getenv("IPEX_LLM_LINEAR_THRESHOLD");
    if (!e) e = getenv("BIGDL_LLM_LINEAR_THRESHOLD");
    return e ? (int64_t)atoll(e) : (int64_t)128;
  }();
  const int isa = (int)isa_req;
  if (M > thr) {
    Tensor w = at::empty({n, k}, xf.options());
    illm_dequantize((int)fmt, p.codes, p.scales, p.mins, n, k, w.data_ptr<float>());
    auto shape = x.sizes().vec();
    shape.back() = n;
    return at::mm(xf, w.t()).view(shape);
  }
  Tensor y = at::empty({M, n}, xf.options());
  if (illm_cpu_q4_supported((int)fmt) && isa >= 0 && k % 64 == 0)
    illm_cpu_gemm_q4((int)fmt, xf.data_ptr<float>(), M, p.codes, p.scales, p.mins, n, k, y.data_ptr<float>(), isa);
  else if (illm_cpu_i8_supported((int)fmt) && isa >= 0 && k % 64 == 0)
    illm_cpu_gemm_i8((int)fmt, xf.data_ptr<float>(), M, p.codes, p.scales, p.mins, n, k, y.data_ptr<float>(), isa);
  else if (illm_cpu_lut_supported((int)fmt) && isa >= 0 && k % 64 == 0)
    illm_cpu_gemm_lut((int)fmt, xf.data_ptr<float>(), M, p.codes, p.scales, n, k, y.data_ptr<float>(), isa);
  else
    illm_cpu_gemm((int)fmt, xf.data_ptr<float>(), M, p.codes, p.scales, p.mins, n, k, y.data_ptr<float>());
  auto shape = x.sizes().vec();
  shape.back() = n;
  return y.view(shape);
}

Tensor to_fp8_bytes(const Tensor& x, bool e5m2) {
  Tensor xf = x.to(at::kFloat).contiguous();
  Tensor out = at::empty(xf.sizes(), xf.options().dtype(at::kByte));
  illm_f32_to_fp8(xf.data_ptr<float>(), xf.numel(), e5m2 ? 1 : 0, out.data_ptr<uint8_t>());
  return out;
}

}  // namespace

TORCH_LIBRARY(ipex_llm_amd, m) {
  // host library
  m.def("quantize_cpu(Tensor w, int fmt, Tensor? imatrix, bool scale_search) -> Tensor");
  m.def("dequantize_cpu(Tensor blob, int fmt, int n, int k) -> Tensor");
  m.def("repack_to_device(Tensor canon, int fmt, int n, int k) -> Tensor");
  m.def("repack_from_device(Tensor dev, int fmt, int n, int k) -> Tensor");
  m.def("linear_cpu(Tensor x, Tensor blob, int fmt, int n, int k) -> Tensor");
  m.def("linear_cpu_isa(Tensor x, Tensor blob, int fmt, int n, int k, int isa) -> Tensor");
  m.def("to_fp8_bytes(Tensor x, bool e5m2) -> Tensor");
  // device kernels (ops_hip.cpp)
  m.def("quantize_device(Tensor w, int fmt, bool scale_search) -> Tensor");
  m.def("dequantize_device(Tensor blob, int fmt, int n, int k, ScalarType dtype, bool transpose=False) -> Tensor");
  m.def("gemv(Tensor x, Tensor blob, int fmt, int n, int k, Tensor? bias, int epi, int ksplit, int act) -> Tensor");
  m.def("add_rms_norm(Tensor? x, Tensor(b!)? partials, Tensor(a!)? residual, Tensor w, float eps, bool unit_offset, bool store_residual, bool zero_partials=False) -> Tensor");
  m.def("rms_norm_bwd(Tensor x, Tensor g, Tensor w, float eps, bool unit_offset) -> Tensor");
  m.def("rope_half(Tensor x, Tensor cos, Tensor sin, bool bwd) -> Tensor");
  m.def("act_mul(Tensor g, Tensor u, Tensor? dy, int act) -> Tensor[]");
  m.def("layer_norm(Tensor x, Tensor? w, Tensor? b, float eps) -> Tensor");
  m.def("kernel_errors(Tensor like, bool reset) -> Tensor");
  m.def("rope_kv(Tensor qkv, Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor slots, Tensor pos, Tensor inv_freq, Tensor? q_norm, Tensor? k_norm, float norm_eps, float q_scale, int Hq, int Hkv, int D, int rot_dim, bool interleaved, int kv_fp8, float k_scale, float v_scale) -> ()");
  m.def("attn_decode(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor seq_lens, int nsplit, float scale, float softcap, int window, int kv_fp8, float k_scale, float v_scale, Tensor? alibi) -> Tensor");
  m.def("glu(Tensor gu, int act, int tile=0) -> Tensor");
  m.def("attn_softmax_(Tensor(a!) x) -> ()");
  m.def("reduce_partials(Tensor ws, Tensor? bias, ScalarType dtype) -> Tensor");
  m.def("moe_topk(Tensor logits, int k, bool renorm, int scoring) -> (Tensor, Tensor)");
  m.def("moe_group_topk(Tensor logits, Tensor? bias, int k, int n_group, int topk_group, bool renorm, float scale) -> (Tensor, Tensor)");
  m.def("moe_align(Tensor ids, int e0, int num_local) -> (Tensor, Tensor)");
  m.def("gemv_glu_in(Tensor part, Tensor blob, int fmt, int n, int k, int act, int ksplit, ScalarType dtype, Tensor(a!)? acc=None, Tensor(b!)? zero=None, Tensor? xss=None, int xss_n=0, float xss_eps=0.0) -> Tensor");
  m.def("l3_prefetch(Tensor t, int offset=0, int nbytes=-1, int wgs=1024) -> ()");
  m.def("decode_advance(Tensor? logits, Tensor(a!) ids, Tensor(b!) next_ids, Tensor(c!) pos, Tensor block_tables, int bs, Tensor(d!) slots, Tensor(e!) seq_lens, Tensor? pos_offset=None, Tensor? parts=None) -> ()");
  m.def("gemv_argmax(Tensor x, Tensor blob, int fmt, int n, int k, Tensor? bias=None) -> (Tensor, Tensor)");
  m.def("embed_rms_norm(Tensor ids, Tensor table, Tensor w, float eps, bool unit_offset=False, Tensor(a!)? zero=None) -> (Tensor, Tensor)");
  m.def("rope_kv_fused(Tensor(d!) part, Tensor? bias, Tensor(a!) q_out, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor pos, Tensor block_tables, int tq, Tensor inv_freq, Tensor? q_norm, Tensor? k_norm, float norm_eps, float q_scale, int Hq, int Hkv, int D, int rot_dim, bool interleaved, int kv_fp8, float k_scale, float v_scale, Tensor? pos_offset=None, bool zero_part=False, Tensor? pss=None, int pss_n=0, float pss_eps=0.0) -> ()");
  m.def("attn_prefill(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor seq_lens, int Tq, float scale, float softcap, int window, int kv_fp8, float k_scale, float v_scale) -> Tensor");
  m.def("attn_decode_split(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor seq_lens, int nsplit, float scale, float softcap, int window, int kv_fp8, float k_scale, float v_scale, Tensor? alibi) -> (Tensor, Tensor)");
  m.def("gemv_attn(Tensor po, Tensor pml, Tensor seq_lens, Tensor blob, int fmt, int n, int k, Tensor(a!)? acc, int ksplit, ScalarType dtype, Tensor(b!)? zero=None, int nw=0) -> Tensor");
  m.def("gemm(Tensor x, Tensor blob, int fmt, int n, int k, Tensor? bias) -> Tensor");
  m.def("gemv_accum(Tensor x, Tensor blob, int fmt, int n, int k, Tensor(a!) acc, int ksplit, Tensor(b!)? zero=None, Tensor? rope_cs=None, Tensor? rope_pos=None, int rope_cols=0, int rope_d=0) -> ()");
  m.def("gemv_accum_norm(Tensor x, Tensor blob, int fmt, int n, int k, Tensor(a!) acc, Tensor(b!) ctr, Tensor residual, Tensor(c!) res_out, Tensor norm_w, bool unit_offset, Tensor(d!) xo, Tensor(e!) ss, Tensor(f!)? zero=None) -> ()");
  m.def("gemv_glu_ss(Tensor x, Tensor blob, int fmt, int n, int k, int act, Tensor ss, int ss_n, float eps) -> Tensor");
  m.def("attn_decode_rope(Tensor part, Tensor? bias, Tensor cos_sin, Tensor pos, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor block_tables, Tensor seq_lens, int nsplit, float scale, float softcap, int window, int Hq, int rot_dim, bool interleaved, float q_scale, ScalarType dtype, Tensor? pss=None, int pss_n=0, float pss_eps=0.0, bool prerot=False) -> Tensor");
  m.def("attn_decode_rope_split(Tensor part, Tensor? bias, Tensor cos_sin, Tensor pos, Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor block_tables, Tensor seq_lens, int nsplit, float scale, float softcap, int window, int Hq, int rot_dim, bool interleaved, float q_scale, ScalarType dtype, Tensor? pss=None, int pss_n=0, float pss_eps=0.0, bool prerot=False) -> (Tensor, Tensor)");
  m.def("gemm_glu(Tensor x, Tensor blob, int fmt, int n, int k, int act) -> Tensor");
  m.def("moe_gemm(Tensor x, Tensor blob, int fmt, int n, int k, Tensor off, Tensor rows, int xdiv, bool x_sorted, bool out_sorted, bool glu, int act, bool out_f32) -> Tensor");
  m.def("rwkv_wkv4(Tensor time_decay, Tensor time_first, Tensor k, Tensor v, Tensor(a!) num, Tensor(b!) den, Tensor(c!) mx) -> Tensor");
  m.def("rwkv_wkv5(Tensor w, Tensor u, Tensor r, Tensor k, Tensor v, Tensor(a!) state) -> Tensor");
  m.def("gemv_norm_in(Tensor acc_in, Tensor residual, Tensor(a!) res_out, Tensor norm_w, float eps, bool unit_offset, Tensor blob, int fmt, int n, int k, int epi, int act, Tensor(b!)? acc_out=None, Tensor(c!)? zero=None, Tensor(d!)? ss=None, Tensor? rope_cs=None, Tensor? rope_pos=None, int rope_cols=0, int rope_d=0) -> Tensor");
  m.def("embedding_lowbit(Tensor blob, int fmt, int n, int k, Tensor ids, ScalarType dtype) -> Tensor");
  m.def("moe_gemv(Tensor x, Tensor blob, int fmt, int n, int k, Tensor off, Tensor rows, int xdiv, int npairs, int epi, int ksplit, int act) -> Tensor");
  m.def("moe_combine(Tensor part, Tensor w, Tensor ids, int e0, int num_local, ScalarType dtype) -> Tensor");
  m.def("moe_gemv_accum(Tensor x, Tensor blob, int fmt, int n, int k, Tensor off, Tensor rows, Tensor(a!) acc, Tensor w, int topk, int ksplit) -> ()");
  m.def("moe_route(Tensor x, Tensor router, int k, bool renorm, int scoring, int e0, int num_local, Tensor(a!) counter) -> (Tensor, Tensor, Tensor, Tensor)");
}

at::Tensor kernel_errors_cpu(const at::Tensor& like, bool reset) {
  return at::zeros({4}, like.options().dtype(at::kInt));     // host kernels check shapes up front
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CPU, m) {
  m.impl("kernel_errors", &kernel_errors_cpu);
  m.impl("quantize_cpu", &quantize_cpu);
  m.impl("dequantize_cpu", &dequantize_cpu);
  m.impl("repack_to_device", &repack_to_device);
  m.impl("repack_from_device", &repack_from_device);
  m.impl("linear_cpu", &linear_cpu);
  m.impl("linear_cpu_isa", &linear_cpu_isa);
  m.impl("to_fp8_bytes", &to_fp8_bytes);
}
