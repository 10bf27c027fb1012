"""Grouped ("FlashMoE") prefill GEMM vs the fp32 reference of the same
low-bit experts: one launch per projection over (token, expert) pairs
sorted by expert (ops.moe_gemm), and the whole NativeMoE prefill block
(route -> align -> gate/up GEMM with GLU epilogue -> down GEMM -> combine)
against its per-expert torch loop.  Reference op: vLLM-XPU fused_moe over
ipex-llm low-bit experts (vllm_for_multi_arc.patch:5933-6116)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("qtype", ["sym_int4", "asym_int4", "sym_int8"])
@pytest.mark.parametrize("T,E,k", [(37, 4, 2), (300, 8, 2), (129, 16, 4), (1700, 4, 2)])
def test_moe_gemm_matches_reference(cuda, qtype, T, E, k):
    from ipex_llm_amd import ops
    from ipex_llm_amd.ops import reference as R
    from ipex_llm_amd.quantize import get_format
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    f = get_format(qtype).fmt
    H, I = 256, 384
    g = torch.Generator(device=cuda).manual_seed(T + E)
    gu = torch.stack([ops.quantize(interleave_glu_rows(torch.randn(I, H, device=cuda, generator=g) * 0.05,
                                                       torch.randn(I, H, device=cuda, generator=g) * 0.05), f)
                      for _ in range(E)])
    dn = torch.stack([ops.quantize(torch.randn(H, I, device=cuda, generator=g) * 0.05, f) for _ in range(E)])
    x = torch.randn(T, H, device=cuda, generator=g).to(torch.bfloat16)
    ids = torch.stack([torch.randperm(E, device=cuda, generator=g)[:k] for _ in range(T)]).to(torch.int32)
    e0, El = (E // 4, E // 2) if E >= 8 else (0, E)       # a slice of local experts (EP-style) on the larger cases
    off, rows = ops.moe_align(ids, e0, El)
    assert int(off[-1]) == int(((ids >= e0) & (ids < e0 + El)).sum())
    gul, dnl = gu[e0:e0 + El].contiguous(), dn[e0:e0 + El].contiguous()
    a = ops.moe_gemm(x, gul, f, 2 * I, H, off, rows, k, False, True, True, 0)
    a_ref = R.moe_gemm(x.float(), gul, f, 2 * I, H, off, rows, k, False, True, True, 0, True)
    n = int(off[-1])
    err = (a[:n].float() - a_ref[:n]).abs().max().item() / (a_ref[:n].abs().max().item() + 1e-6)
    assert err < 2e-2, err
    part = ops.moe_gemm(a, dnl, f, H, I, off, rows, 1, True, False, False, 0, True)
    p_ref = R.moe_gemm(a.float(), dnl, f, H, I, off, rows, 1, True, False, False, 0, True)
    loc = rows[:n].long()
    err = (part[loc] - p_ref[loc]).abs().max().item() / (p_ref[loc].abs().max().item() + 1e-6)
    assert err < 2e-2, err


def test_native_moe_prefill_grouped_vs_loop(cuda):
    from transformers import MixtralConfig
    from ipex_llm_amd.models.builder import random_native_model
    cfg = MixtralConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=1,
                        num_attention_heads=4, num_key_value_heads=2, num_local_experts=8, num_experts_per_tok=2)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=0, std=0.05)
    moe = m.layers[0].mlp
    x = (torch.randn(200, 256, device=cuda) * 0.5).to(torch.bfloat16)
    w, ids = moe.route(x)
    y = moe._experts_gemm(x, w, ids).float()
    ref = moe._experts_loop(x, w, ids).float()
    err = ((y - ref).norm() / ref.norm()).item()
    assert err < 2e-2, err
