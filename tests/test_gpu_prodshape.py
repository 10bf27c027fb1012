"""Production-shape parity: the bench's shapes end to end.

A 2-layer model of Llama-3-8B width (hidden 4096, GQA 32 / 8 heads of 128,
MLP 14336, vocab 128256, rope theta 5e5) at sym_int4 runs the default
production path of bench.py: B = 8 prompts x 1024 tokens through
``Engine.prefill_batch`` with the captured prefill graph (dense 8-phase GEMMs
with split-K slabs and the GLU epilogue over transiently dequantized weights,
paged flash-attention prefill), then 8 captured decode steps at batch 8 (norm-in
GEMVs, o_proj norm-out epilogue, fused-RoPE attention, argmax epilogue).  Every
step's logits are compared with a plain fp32 PyTorch forward of the same
(dequantized) weights over the same tokens, with the comparison smoke() uses.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _cfg():
    from transformers import LlamaConfig
    return LlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=2,
                       num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=2048,
                       rope_theta=500000.0, rms_norm_eps=1e-5)


@torch.no_grad()
def _fp32_forward(model, ids: torch.Tensor) -> torch.Tensor:
    """[B, T] ids -> [B, T, V] fp32 logits: RMSNorm, rotate-half RoPE, causal
    GQA SDPA, SiLU GLU (gate / up rows tile-interleaved in the native layout)"""
    from ipex_llm_amd.models.decoder import deinterleave_glu
    s = model.spec
    dev = ids.device
    W = lambda m: m.dequantize(torch.float32).to(dev)              # noqa: E731

    def rms(x, w):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + s.rms_eps) * w.float()
    B, T = ids.shape
    x = model.embed_tokens.float()[ids]
    inv = model.inv_freq.float().to(dev)
    fr = torch.arange(T, dtype=torch.float32, device=dev)[:, None] * inv[None]
    cos, sin = torch.cat([fr.cos()] * 2, -1), torch.cat([fr.sin()] * 2, -1)

    def rope(t):                                                   # [B, T, H, D]
        a, b = t.chunk(2, -1)
        return t * cos[None, :, None] + torch.cat([-b, a], -1) * sin[None, :, None]
    nh, nkv, hd = s.num_heads, s.num_kv_heads, s.head_dim
    for L in model.layers:
        h = rms(x, L.input_layernorm)
        qkv = h @ W(L.self_attn.qkv_proj).t()
        q, k, v = qkv.split([nh * hd, nkv * hd, nkv * hd], -1)
        q, k, v = rope(q.view(B, T, nh, hd)), rope(k.view(B, T, nkv, hd)), v.view(B, T, nkv, hd)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           is_causal=True, scale=s.scale, enable_gqa=True)
        x = x + o.transpose(1, 2).reshape(B, T, -1) @ W(L.self_attn.o_proj).t()
        h = rms(x, L.post_attention_layernorm)
        g, u = deinterleave_glu(h @ W(L.mlp.gate_up_proj).t())
        x = x + (F.silu(g) * u) @ W(L.mlp.down_proj).t()
    return rms(x, model.norm) @ W(model.lm_head).t()


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_llama3_8b_width_b8x1024_prefill_graph_then_decode(cuda):
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.cache import SequenceState
    torch.manual_seed(0)
    m = random_native_model(_cfg(), "sym_int4", cuda, torch.bfloat16, seed=0)
    e = Engine(m)
    B, n, steps = 8, 1024, 8
    max_len = n + steps + 8
    e._ensure_cache(B, max_len)
    nblk = (max_len + e.block_size - 1) // e.block_size
    seqs = [SequenceState(e.cache.allocator.alloc(nblk)) for _ in range(B)]
    prompts = torch.randint(0, 128256, (B, n), generator=torch.Generator().manual_seed(7))
    logits = [e.prefill_batch(seqs, prompts, use_graph=True).float()]          # captured, then replayed
    assert e._pf_graphs, "prefill graph not captured"
    st = e.decode_step_obj(seqs, max_len, greedy=False, use_graph=True)
    toks = [logits[0].argmax(-1)]
    st.set_state(toks[0], torch.tensor([s.length for s in seqs], device=cuda))
    for i in range(steps):
        st.step()
        logits.append(st.logits.float().clone())
        toks.append(logits[-1].argmax(-1))
        st.ids.copy_(toks[-1])
    # fp32 reference over prompt + the engine's own tokens (teacher forcing)
    full = torch.cat([prompts.to(cuda), torch.stack(toks[:steps], 1)], 1)     # [B, n + steps]
    ref = _fp32_forward(m, full)[:, n - 1:n + steps]                           # positions n-1 .. n+steps-1
    for i, lg in enumerate(logits):
        r = ref[:, i]
        rel = _rel(lg, r)
        assert rel < 3e-2, (i, rel)
        top5 = r.topk(5, -1).indices
        assert (top5 == lg.argmax(-1, keepdim=True)).any(-1).all(), i
