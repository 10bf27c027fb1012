"""Training flash attention (csrc/hip/train_attn.hip) at the QLoRA shape
(Llama-3-8B, B=8 x T=512, 32 q / 8 kv heads, D=128, causal): per-kernel
timing (events) and a target for rocprofv3 --pmc passes."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main():
    from ipex_llm_amd import ops
    ops.require()
    B, Hq, Hkv, T, D = 8, 32, 8, int(sys.argv[1]) if len(sys.argv) > 1 else 512, 128
    dev = torch.device("cuda")
    q = torch.randn(B, Hq, T, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16)
    A = torch.ops.ipex_llm_amd
    out, lse = A.train_attn_fwd(q, k, v, D ** -0.5, True)
    do = torch.randn_like(out)

    def t(fn, it=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / it * 1e3
    fwd = t(lambda: A.train_attn_fwd(q, k, v, D ** -0.5, True))
    bwd = t(lambda: A.train_attn_bwd(q, k, v, out, lse, do, D ** -0.5, True))
    fl = 4 * B * Hq * T * T / 2 * D
    print(json.dumps({"T": T, "fwd_us": round(fwd, 1), "fwd_TF": round(fl / fwd / 1e6, 1), "bwd_us": round(bwd, 1),
                      "bwd_TF": round(2.5 * fl / bwd / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
