"""LoRA token-axis reductions (dA = gxa^T x, dB^T = xa^T g) at the QLoRA
Llama-3-8B shapes (4096 tokens): the HIP lora_tn kernel vs the library GEMM.
ILLM_LORA_TN_ROWS / ILLM_LORA_TN_WGS select the kernel's row-slice policy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ipex_llm_amd import ops  # noqa: E402

ops.require()

P = torch.ops.ipex_llm_amd
M = 4096
shapes = {"dA_qkv": (24, 4096), "dA_gu": (16, 4096), "dA_o": (8, 4096), "dA_down": (8, 14336),
          "dB_q": (8, 4096), "dB_kv": (8, 1024), "dB_gate": (8, 14336), "dB_down": (8, 4096)}


def t(fn, reps=50):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


res = {"rows": os.environ.get("ILLM_LORA_TN_ROWS", "128"), "wgs": os.environ.get("ILLM_LORA_TN_WGS", "2048")}
tot_k = tot_l = 0.0
for name, (r, N) in shapes.items():
    a = torch.randn(M, r, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    k = t(lambda: P.lora_tn(a, b, 1.0))
    lib = t(lambda: torch.mm(a.t(), b))
    res[name] = [round(k, 1), round(lib, 1)]
    tot_k += k
    tot_l += lib
res["sum_kernel_us"], res["sum_library_us"] = round(tot_k, 1), round(tot_l, 1)
print(json.dumps(res), flush=True)
