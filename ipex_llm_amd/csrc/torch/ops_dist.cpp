// Peer-memory (hipIpc) buffers and the one-shot xGMI all-reduce op.
//   ipc_alloc(nbytes) -> int        device pointer of a zeroed hipMalloc buffer
//   ipc_handle(ptr) -> Tensor       64-byte hipIpcMemHandle (CPU uint8)
//   ipc_open(handle) -> int         peer buffer mapped into this process
//   ipc_close(ptr) / ipc_free(ptr)
//   custom_all_reduce(inp, out, bufs, rank, counter, cap, err)
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
                       Tensor& counter, int64_t cap, Tensor& err) {
  TORCH_CHECK(inp.is_cuda() && out.is_cuda() && inp.is_contiguous() && out.is_contiguous(),
              "custom_all_reduce: contiguous GPU tensors");
  TORCH_CHECK(inp.scalar_type() == at::kBFloat16 || inp.scalar_type() == at::kHalf, "bf16/fp16 only");
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
  if (a.nvec > 0)
    illm::launch_custom_all_reduce(inp.scalar_type() == at::kBFloat16, a,
                                   at::hip::getCurrentHIPStream().stream());
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(ipex_llm_amd, m) {
  m.def("ipc_alloc(int nbytes) -> int", &ipc_alloc);
  m.def("ipc_handle(int ptr) -> Tensor", &ipc_handle);
  m.def("ipc_open(Tensor handle) -> int", &ipc_open);
  m.def("ipc_close(int ptr) -> ()", &ipc_close);
  m.def("ipc_free(int ptr) -> ()", &ipc_free);
  m.def("custom_all_reduce(Tensor inp, Tensor(a!) out, int[] bufs, int rank, Tensor(b!) counter, int cap, Tensor(c!) err) -> ()");
}

TORCH_LIBRARY_IMPL(ipex_llm_amd, CUDA, m) { m.impl("custom_all_reduce", &custom_all_reduce); }
