// Peer-memory (hipIpc) buffers and the one-shot xGMI all-reduce op.
//   ipc_alloc(nbytes, uncached) -> int  device pointer of a zeroed (uncached) buffer
//   ipc_handle(ptr) -> Tensor       64-byte hipIpcMemHandle (CPU uint8)
//   ipc_open(handle) -> int         peer buffer mapped into this process
//   ipc_close(ptr) / ipc_free(ptr)
//   custom_all_reduce(inp, out, bufs, rank, counter, cap, err, two_shot)  bf16 / fp16 / f32
// The Python side (parallel/comm.py) exchanges handles with
// torch.distributed.all_gather_object once per process group.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include "../hip/kernels.h"
#include "../hip/kernels_dist.h"

using at::Tensor;

int* illm_kernel_err(const c10::Device& dev);   // device kernel error word (ops_hip.cpp)

namespace {

#define HIP_OK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));                \
  } while (0)

// uncached: hipDeviceMallocUncached memory (never held in any L2).  Peer
// buffers are written by OTHER GPUs over xGMI (signal epochs, EP dispatch rows
// and counts) and polled / read by the owner: a coarse-grained hipMalloc line
// the owner's L2 still holds would not see a peer's store (remote writes do not
// invalidate it, and an acquire does not invalidate locally-owned lines), so
// the flags and every peer-written byte live in uncached memory -- the form
// the ROCm custom all-reduces use for their signal buffers.
int64_t ipc_alloc(int64_t nbytes, bool uncached) {
  void* p = nullptr;
  if (uncached) HIP_OK(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocUncached));
  else HIP_OK(hipMalloc(&p, (size_t)nbytes));
  HIP_OK(hipMemset(p, 0, (size_t)nbytes));
  HIP_OK(hipDeviceSynchronize());
  return (int64_t)(uintptr_t)p;
}

Tensor ipc_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, (void*)(uintptr_t)ptr));
  Tensor t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  memcpy(t.data_ptr<uint8_t>(), &h, sizeof(h));
  return t;
}

int64_t ipc_open(const Tensor& handle) {
  TORCH_CHECK(handle.numel() == (int64_t)sizeof(hipIpcMemHandle_t), "bad IPC handle size");
  hipIpcMemHandle_t h;
  Tensor c = handle.to(at::kCPU).contiguous();
  memcpy(&h, c.data_ptr<uint8_t>(), sizeof(h));
  void* p = nullptr;
  HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return (int64_t)(uintptr_t)p;
}

void ipc_close(int64_t ptr) { HIP_OK(hipIpcCloseMemHandle((void*)(uintptr_t)ptr)); }
void ipc_free(int64_t ptr) { HIP_OK(hipFree((void*)(uintptr_t)ptr)); }

void custom_all_reduce(const Tensor& inp, Tensor& out, c10::IntArrayRef bufs, int64_t rank,
                       Tensor& counter, int64_t cap, Tensor& err, int64_t two_shot) {
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.is_contiguous() && out.is_contiguous(),
              "custom_all_reduce: contiguous GPU tensors");
  const auto dt = inp.scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kHalf || dt == at::kFloat, "custom_all_reduce: bf16/fp16/f32 only");
  TORCH_CHECK(out.scalar_type() == dt && out.numel() == inp.numel(), "custom_all_reduce: out must match inp");
  const int64_t bytes = inp.numel() * inp.element_size();
  TORCH_CHECK(bytes % 16 == 0 && bytes <= cap, "custom_all_reduce: message must be 16-B aligned and <= cap");
  TORCH_CHECK((int64_t)bufs.size() >= 1 && (int64_t)bufs.size() <= illm::AR_MAX_RANKS, "1..8 ranks");
  TORCH_CHECK(counter.numel() >= illm::AR_MAX_BLOCKS && counter.scalar_type() == at::kInt, "counter int32[64]");
  c10::DeviceGuard g(inp.device());
  illm::AllReduceArgs a{};
  for (size_t i = 0; i < bufs.size(); i++) a.bufs[i] = (uint8_t*)(uintptr_t)bufs[i];
  a.rank = (int)rank;
  a.world = (int)bufs.size();
  a.in = (const uint4*)inp.data_ptr();
  a.out = (uint4*)out.data_ptr();
  a.nvec = bytes / 16;
  a.cap = cap;
  a.counter = (uint32_t*)counter.data_ptr<int32_t>();
  a.err = err.data_ptr<int32_t>();
  a.kerr = illm_kernel_err(inp.device());
  a.dtype = dt == at::kFloat ? illm::AR_F32 : (dt == at::kBFloat16 ? illm::AR_BF16 : illm::AR_F16);
  // two-shot once every rank reading the whole message from all peers costs
  // more link time than the extra exchange round (> 256 KiB at W > 2)
  a.two_shot = two_shot >= 0 ? (int)two_shot : (a.world > 2 && bytes > (256 << 10) ? 1 : 0);
  if (a.nvec > 0) illm::launch_custom_all_reduce(a, at::hip::getCurrentHIPStream().stream());
}

// out [rows, W * n] (last-dim concat of every rank's inp [rows, n]); n * elsize % 16 == 0
void custom_all_gather(const Tensor& inp, Tensor& out, c10::IntArrayRef bufs, int64_t rank, Tensor& counter,
                       int64_t cap, Tensor& err) {
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.is_contiguous() && out.is_contiguous(),
              "custom_all_gather: contiguous GPU tensors");
  TORCH_CHECK(out.scalar_type() == inp.scalar_type(), "custom_all_gather: out dtype must match");
  const int64_t W = (int64_t)bufs.size();
  TORCH_CHECK(W >= 1 && W <= illm::AR_MAX_RANKS, "1..8 ranks");
  TORCH_CHECK(inp.dim() >= 1 && out.numel() == inp.numel() * W, "custom_all_gather: out must be W x inp");
  const int64_t row_bytes = inp.size(-1) * inp.element_size();
  const int64_t bytes = inp.numel() * inp.element_size();
  TORCH_CHECK(row_bytes % 16 == 0 && bytes <= cap, "custom_all_gather: rows must be 16-B multiples, message <= cap");
  TORCH_CHECK(counter.numel() >= illm::AR_MAX_BLOCKS && counter.scalar_type() == at::kInt, "counter int32[64]");
  c10::DeviceGuard g(inp.device());
  illm::AllReduceArgs a{};
  for (int64_t i = 0; i < W; i++) a.bufs[i] = (uint8_t*)(uintptr_t)bufs[i];
  a.rank = (int)rank;
  a.world = (int)W;
  a.in = (const uint4*)inp.data_ptr();
  a.out = (uint4*)out.data_ptr();
  a.nvec = bytes / 16;
  a.inner = row_bytes / 16;
  a.cap = cap;
  a.counter = (uint32_t*)counter.data_ptr<int32_t>();
  a.err = err.data_ptr<int32_t>();
  a.kerr = illm_kernel_err(inp.device());
  if (a.nvec > 0) illm::launch_custom_all_gather(a, at::hip::getCurrentHIPStream().stream());
}

// ---- expert-parallel peer all-to-all (ep_a2a.hip; Python: parallel/ep.py EPAllToAll)
int64_t ep_buffer_bytes(int64_t world, int64_t cap, int64_t H) { return illm::ep_buffer_bytes((int)world, cap, H); }

// a tensor view of [offset, offset + numel * elsize) of a peer buffer this
// process owns (lifetime: the EPAllToAll that allocated it)
Tensor ep_view(int64_t ptr, int64_t offset, c10::IntArrayRef shape, at::ScalarType dtype, at::Device device) {
  return at::from_blob((void*)((uintptr_t)ptr + offset), shape, at::TensorOptions().dtype(dtype).device(device));
}

// peer wait bound (ILLM_EP_TIMEOUT_S, default 20 s)
static uint64_t ep_timeout_ticks() {
  static const uint64_t t = [] {
    const char* e = getenv("ILLM_EP_TIMEOUT_S");
    const double s = e != nullptr ? atof(e) : 20.0;
    return (uint64_t)((s > 0 ? s : 20.0) * 1e8);
  }();
  return t;
}

static illm::EpA2AArgs ep_args(c10::IntArrayRef bufs, int64_t rank, int64_t cap, int64_t H, const Tensor& epoch) {
  TORCH_CHECK((int64_t)bufs.size() >= 1 && (int64_t)bufs.size() <= illm::EP_MAX_RANKS, "ep: 1..8 ranks");
  TORCH_CHECK(rank >= 0 && rank < (int64_t)bufs.size(), "ep: bad rank");
  TORCH_CHECK(H % 8 == 0 && H > 0, "ep: hidden size must be a multiple of 8");
  TORCH_CHECK(epoch.is_cuda() && epoch.scalar_type() == at::kInt && epoch.numel() == 1, "ep: epoch int32[1] on the GPU");
  illm::EpA2AArgs a{};
  for (size_t i = 0; i < bufs.size(); i++) a.bufs[i] = (uint8_t*)(uintptr_t)bufs[i];
  a.rank = (int)rank;
  a.world = (int)bufs.size();
  a.cap = cap;
  a.H = (int)H;
  a.epoch = (const uint32_t*)epoch.data_ptr<int32_t>();
  a.err = illm_kernel_err(epoch.device());
  a.timeout = ep_timeout_ticks();
  return a;
}

static void ep_check_i32(const Tensor& t, int64_t n, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() >= n, "ep: ", what,
              " must be contiguous int32 with >= ", n, " elements on the GPU");
}

// dispatch: this rank's T tokens x k pairs to the expert owners' recv regions
void ep_dispatch(const Tensor& x, const Tensor& ids, const Tensor& off, const Tensor& rows, Tensor& pos,
                 Tensor& counts, c10::IntArrayRef bufs, int64_t rank, int64_t cap, int64_t el, const Tensor& epoch) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.is_contiguous() &&
              (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf), "ep_dispatch: x [T, H] bf16/fp16");
  c10::DeviceGuard g(x.device());
  illm::EpA2AArgs a = ep_args(bufs, rank, cap, x.size(1), epoch);
  const int64_t T = x.size(0), P = ids.numel();
  TORCH_CHECK(T > 0 && P % T == 0, "ep_dispatch: ids must be [T, k]");
  const int64_t k = P / T;
  TORCH_CHECK(P <= cap, "ep_dispatch: T * k = ", P, " exceeds the region capacity ", cap);
  TORCH_CHECK(el >= 1, "ep_dispatch: experts per rank >= 1");
  ep_check_i32(ids, P, "ids");
  ep_check_i32(off, a.world + 1, "off");
  ep_check_i32(rows, P, "rows");
  ep_check_i32(pos, P, "pos");
  ep_check_i32(counts, a.world + 1, "counts");
  a.x = (const uint16_t*)x.data_ptr();
  a.T = (int)T;
  a.k = (int)k;
  a.el = (int)el;
  a.ids = ids.data_ptr<int32_t>();
  a.off = off.data_ptr<int32_t>();
  a.rows = rows.data_ptr<int32_t>();
  a.pos = pos.data_ptr<int32_t>();
  a.counts = counts.data_ptr<int32_t>();
  a.bf16 = x.scalar_type() == at::kBFloat16;
  illm::launch_ep_dispatch(a, at::hip::getCurrentHIPStream().stream());
}

// return: expert outputs [W * cap, H] (received-slot order) to their sources
void ep_return(const Tensor& out_rows, const Tensor& counts, c10::IntArrayRef bufs, int64_t rank, int64_t cap,
               const Tensor& epoch) {
  TORCH_CHECK(out_rows.is_cuda() && out_rows.dim() == 2 && out_rows.is_contiguous() && out_rows.element_size() == 2,
              "ep_return: out_rows [W * cap, H] 16-bit");
  c10::DeviceGuard g(out_rows.device());
  illm::EpA2AArgs a = ep_args(bufs, rank, cap, out_rows.size(1), epoch);
  TORCH_CHECK(out_rows.size(0) >= a.world * cap, "ep_return: out_rows must hold W * cap rows");
  ep_check_i32(counts, a.world + 1, "counts");
  a.out_rows = (const uint16_t*)out_rows.data_ptr();
  a.counts = counts.data_ptr<int32_t>();
  illm::launch_ep_return(a, at::hip::getCurrentHIPStream().stream());
}

// combine: y [T, H] = sum_j w[t, j] * returned row of pair (t, j)
void ep_combine(Tensor& y, const Tensor& w, const Tensor& ids, const Tensor& off, const Tensor& pos, Tensor& counts,
                c10::IntArrayRef bufs, int64_t rank, int64_t cap, int64_t el, const Tensor& epoch) {
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.is_contiguous() &&
              (y.scalar_type() == at::kBFloat16 || y.scalar_type() == at::kHalf), "ep_combine: y [T, H] bf16/fp16");
  c10::DeviceGuard g(y.device());
  illm::EpA2AArgs a = ep_args(bufs, rank, cap, y.size(1), epoch);
  const int64_t T = y.size(0), P = ids.numel();
  TORCH_CHECK(T > 0 && P % T == 0 && P <= cap, "ep_combine: ids must be [T, k] with T * k <= cap");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == P,
              "ep_combine: w f32 [T, k]");
  ep_check_i32(ids, P, "ids");
  ep_check_i32(off, a.world + 1, "off");
  ep_check_i32(pos, P, "pos");
  ep_check_i32(counts, a.world + 1, "counts");
  a.T = (int)T;
  a.k = (int)(P / T);
  a.el = (int)el;
  a.ids = ids.data_ptr<int32_t>();
  a.off = off.data_ptr<int32_t>();
  a.pos = pos.data_ptr<int32_t>();
  a.counts = counts.data_ptr<int32_t>();
  a.w = w.data_ptr<float>();
  a.y = (uint16_t*)y.data_ptr();
  a.bf16 = y.scalar_type() == at::kBFloat16;
  illm::launch_ep_combine(a, at::hip::getCurrentHIPStream().stream());
}

// table: int64 [5, T] = (param ptr, grad ptr, exp_avg ptr, exp_avg_sq ptr, numel)
void fused_adamw(const Tensor& table, const Tensor& chunk_tensor, const Tensor& chunk_start, int64_t chunk,
                 double lr, double beta1, double beta2, double eps, double weight_decay, double bc1, double bc2,
                 double grad_scale, int64_t param_dtype, int64_t grad_dtype,
                 const c10::optional<Tensor>& step_lr) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kLong && table.dim() == 2 && table.size(0) == 5,
              "fused_adamw: table must be int64 [5, T] on the GPU");
  c10::DeviceGuard g(table.device());
  const int64_t T = table.size(1);
  const int64_t* t = table.data_ptr<int64_t>();
  illm::AdamWArgs a{};
  a.params = t;
  a.grads = t + T;
  a.exp_avg = t + 2 * T;
  a.exp_avg_sq = t + 3 * T;
  a.sizes = t + 4 * T;
  a.chunk_tensor = chunk_tensor.data_ptr<int32_t>();
  a.chunk_start = chunk_start.data_ptr<int64_t>();
  a.chunk = (int)chunk;
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.bias_corr1 = (float)bc1;
  a.bias_corr2 = (float)bc2;
  a.grad_scale = (float)grad_scale;
  a.param_dtype = (int)param_dtype;
  a.grad_dtype = (int)grad_dtype;
  a.step_lr = nullptr;
  if (step_lr.has_value()) {
    TORCH_CHECK(step_lr->is_cuda() && step_lr->scalar_type() == at::kFloat && step_lr->numel() == 2,
                "fused_adamw: step_lr must be f32 [2] (step, lr) on the GPU");
    a.step_lr = step_lr->data_ptr<float>();
  }
  illm::launch_fused_adamw(a, (int)chunk_tensor.numel(), at::hip::getCurrentHIPStream().stream());
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("fused_adamw(Tensor table, Tensor chunk_tensor, Tensor chunk_start, int chunk, float lr, float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2, float grad_scale, int param_dtype, int grad_dtype, Tensor? step_lr=None) -> ()");
  m.def("ipc_alloc(int nbytes, bool uncached=False) -> int", &ipc_alloc);
  m.def("ipc_handle(int ptr) -> Tensor", &ipc_handle);
  m.def("ipc_open(Tensor handle) -> int", &ipc_open);
  m.def("ipc_close(int ptr) -> ()", &ipc_close);
  m.def("ipc_free(int ptr) -> ()", &ipc_free);
  m.def("ep_buffer_bytes(int world, int cap, int H) -> int", &ep_buffer_bytes);
  m.def("ep_view(int ptr, int offset, int[] shape, ScalarType dtype, Device device) -> Tensor", &ep_view);
  m.def("ep_dispatch(Tensor x, Tensor ids, Tensor off, Tensor rows, Tensor(a!) pos, Tensor(b!) counts, int[] bufs, int rank, int cap, int el, Tensor epoch) -> ()");
  m.def("ep_return(Tensor out_rows, Tensor counts, int[] bufs, int rank, int cap, Tensor epoch) -> ()");
  m.def("ep_combine(Tensor(a!) y, Tensor w, Tensor ids, Tensor off, Tensor pos, Tensor(b!) counts, int[] bufs, int rank, int cap, int el, Tensor epoch) -> ()");
  m.def("custom_all_gather(Tensor inp, Tensor(a!) out, int[] bufs, int rank, Tensor(b!) counter, int cap, Tensor(c!) err) -> ()");
  m.def("custom_all_reduce(Tensor inp, Tensor(a!) out, int[] bufs, int rank, Tensor(b!) counter, int cap, Tensor(c!) err, int two_shot=-1) -> ()");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("custom_all_reduce", &custom_all_reduce);
  m.impl("custom_all_gather", &custom_all_gather);
  m.impl("fused_adamw", &fused_adamw);
  m.impl("ep_dispatch", &ep_dispatch);
  m.impl("ep_return", &ep_return);
  m.impl("ep_combine", &ep_combine);
}
