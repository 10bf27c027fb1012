// Peer-memory (hipIpc) buffers and the one-shot xGMI all-reduce op.
//   ipc_alloc(nbytes) -> int        device pointer of a zeroed hipMalloc buffer
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

using at::Tensor;

namespace {

#define HIP_OK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));                \
  } while (0)

int64_t ipc_alloc(int64_t nbytes) {
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, (size_t)nbytes));
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
  a.dtype = dt == at::kFloat ? illm::AR_F32 : (dt == at::kBFloat16 ? illm::AR_BF16 : illm::AR_F16);
  // two-shot once every rank reading the whole message from all peers costs
  // more link time than the extra exchange round (> 256 KiB at W > 2)
  a.two_shot = two_shot >= 0 ? (int)two_shot : (a.world > 2 && bytes > (256 << 10) ? 1 : 0);
  if (a.nvec > 0) illm::launch_custom_all_reduce(a, at::hip::getCurrentHIPStream().stream());
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
  m.def("ipc_alloc(int nbytes) -> int", &ipc_alloc);
  m.def("ipc_handle(int ptr) -> Tensor", &ipc_handle);
  m.def("ipc_open(Tensor handle) -> int", &ipc_open);
  m.def("ipc_close(int ptr) -> ()", &ipc_close);
  m.def("ipc_free(int ptr) -> ()", &ipc_free);
  m.def("custom_all_reduce(Tensor inp, Tensor(a!) out, int[] bufs, int rank, Tensor(b!) counter, int cap, Tensor(c!) err, int two_shot=-1) -> ()");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) {
  m.impl("custom_all_reduce", &custom_all_reduce);
  m.impl("fused_adamw", &fused_adamw);
}
