"""Prefill / long-query flash-attention HIP kernel (attn_prefill.hip) vs the
fp32 PyTorch reference over the same paged cache."""
import pytest
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _setup(cuda, B, Tq, prefix, Hq, Hkv, D, dtype, bs=64, kv_fp8=0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    L = [prefix + Tq + 7 * b for b in range(B)]      # unequal cached prefixes
    nb = [(x + bs - 1) // bs + 1 for x in L]
    tot = sum(nb)
    kc = torch.randn(tot, Hkv, bs, D, generator=g, device=cuda)
    vc = torch.randn(tot, Hkv, bs, D, generator=g, device=cuda)
    perm = torch.randperm(tot, device=cuda).to(torch.int32)
    bt = torch.zeros(B, max(nb), dtype=torch.int32, device=cuda)
    o = 0
    for b in range(B):
        bt[b, :nb[b]] = perm[o:o + nb[b]]
        o += nb[b]
    if kv_fp8:
        kcache = ops.to_fp8_bytes(kc.cpu(), kv_fp8 == 1).to(cuda)
        vcache = ops.to_fp8_bytes(vc.cpu(), kv_fp8 == 1).to(cuda)
    else:
        kcache, vcache = kc.to(dtype), vc.to(dtype)
        # poison every slot past the sequence ends: the kernel must not read them into P V
        for b in range(B):
            for j in range(L[b], nb[b] * bs):
                blk, off = int(bt[b, j // bs]), j % bs
                kcache[blk, :, off] = float("nan")
                vcache[blk, :, off] = float("nan")
    q = torch.randn(B * Tq, Hq, D, generator=g, device=cuda).to(dtype)
    seq = torch.tensor(L, dtype=torch.int32, device=cuda)
    return q, kcache, vcache, bt, seq, L


def _ref(q, kcache, vcache, bt, L, Tq, scale, softcap, window, kv_fp8, dtype):
    B = bt.shape[0]
    out = []
    for b in range(B):
        kk = ops.api.gather_kv(kcache, bt, b, L[b], kv_fp8, 1.0, torch.float32)
        vv = ops.api.gather_kv(vcache, bt, b, L[b], kv_fp8, 1.0, torch.float32)
        qb = q[b * Tq:(b + 1) * Tq].float()[None]
        out.append(R.attention(qb, kk[None].float(), vv[None].float(), True, scale, softcap, window)[0])
    return torch.cat(out, 0)


@pytest.mark.parametrize("B,Tq,prefix", [(1, 64, 0), (1, 130, 0), (2, 17, 100), (3, 96, 40), (1, 1, 300)])
@pytest.mark.parametrize("Hq,Hkv,D", [(8, 2, 128), (4, 4, 64), (8, 1, 128)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_attn_prefill_matches_reference(cuda, B, Tq, prefix, Hq, Hkv, D, dtype):
    q, kc, vc, bt, seq, L = _setup(cuda, B, Tq, prefix, Hq, Hkv, D, dtype)
    got = ops.attn_prefill(q, kc, vc, bt, seq, Tq, D ** -0.5)
    torch.cuda.synchronize()
    ref = _ref(q, kc, vc, bt, L, Tq, D ** -0.5, 0.0, 0, 0, dtype)
    assert torch.isfinite(got.float()).all()
    assert _rel(got, ref) < 1.5e-2


@pytest.mark.parametrize("softcap,window", [(30.0, 0), (0.0, 48), (50.0, 70)])
def test_attn_prefill_softcap_window(cuda, softcap, window):
    q, kc, vc, bt, seq, L = _setup(cuda, 2, 150, 30, 8, 2, 128, torch.bfloat16, seed=3)
    got = ops.attn_prefill(q, kc, vc, bt, seq, 150, 0.1, softcap, window)
    ref = _ref(q, kc, vc, bt, L, 150, 0.1, softcap, window, 0, torch.bfloat16)
    assert _rel(got, ref) < 1.5e-2


@pytest.mark.parametrize("kv_fp8", [1, 2])
def test_attn_prefill_fp8_cache(cuda, kv_fp8):
    q, kc, vc, bt, seq, L = _setup(cuda, 2, 80, 20, 8, 2, 128, torch.bfloat16, kv_fp8=kv_fp8, seed=5)
    got = ops.attn_prefill(q, kc, vc, bt, seq, 80, 128 ** -0.5, 0.0, 0, kv_fp8, 1.0, 1.0)
    ref = _ref(q, kc, vc, bt, L, 80, 128 ** -0.5, 0.0, 0, kv_fp8, torch.bfloat16)
    assert _rel(got, ref) < 2e-2


def test_native_prefill_uses_kernel_and_matches_sdpa(cuda):
    """engine prefill (HIP flash attention) == the SDPA-over-gathered-keys path"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.decoder import NativeCausalLM
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=11)
    prompts = [list(range(3, 200)), list(range(9, 150))]
    outs = {}
    try:
        for flag in (True, False):
            NativeCausalLM._prefill_attn_native = flag
            outs[flag] = Engine(m).generate(prompts, max_new_tokens=6, use_graph=False)
    finally:
        NativeCausalLM._prefill_attn_native = True
    same = sum(a == b for a, b in zip(sum(outs[True], []), sum(outs[False], [])))
    assert same >= 0.97 * len(sum(outs[True], []))
