#!/bin/bash
# round 6: coalesced transposed dequantization -- tests, per-call bandwidth, QLoRA step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_training.py -k "dequant or lora or qlora or dispatch" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6r_pytest.log 2>&1 || { tail -30 gpurun_out/r6r_pytest.log; exit 2; }
tail -1 gpurun_out/r6r_pytest.log
timeout -k 10 200 python - <<'PY' 2>&1 | tee gpurun_out/dequant_bw_r6.txt
import torch, ipex_llm_amd.ops as ops
from ipex_llm_amd.quantize import get_format
for q in ("nf4", "sym_int4"):
    f = get_format(q).fmt
    for n, k in ((14336, 4096), (4096, 14336), (4096, 4096), (1024, 4096)):
        blob = ops.quantize(torch.randn(n, k, device="cuda") * 0.02, f)
        for tr in (False, True):
            fn = lambda: torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, torch.bfloat16, tr)
            for _ in range(3): fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20): fn()
            e1.record(); e1.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            byt = blob.numel() * blob.element_size() + n * k * 2
            print(f"{q} n={n} k={k} transpose={tr}: {us:.1f} us, {byt / us / 1e6:.2f} TB/s (blob in + bf16 out)")
PY
: > gpurun_out/r6r.jsonl
for i in 1 2; do
  timeout -k 10 500 python tools/bench_qlora.py > gpurun_out/r6r_tmp.log 2>&1 || { tail -5 gpurun_out/r6r_tmp.log; exit 3; }
  tail -1 gpurun_out/r6r_tmp.log | tee -a gpurun_out/r6r.jsonl | cut -c1-200
done
