"""Low-bit embedding gather kernel vs the CPU dequantizer."""
import pytest
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.quantize import qtypes as Q

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("qtype", ["sym_int4", "asym_int4", "sym_int8", "nf4", "fp8_e4m3"])
def test_embedding_lowbit_kernel(cuda, qtype):
    fmt = Q.get_format(Q.resolve_qtype(qtype)).fmt
    w = torch.randn(300, 256)
    blob = ops.quantize(w, fmt)
    ref = ops.dequantize(blob, fmt, 300, 256, torch.float32)
    ids = torch.tensor([[0, 5, 299], [17, 17, 42]])
    out = torch.ops.ipex_llm_amd.embedding_lowbit(blob.to(cuda), fmt, 300, 256, ids.to(cuda), torch.bfloat16)
    assert out.shape == (2, 3, 256)
    assert torch.allclose(out.float().cpu(), ref[ids], atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("qtype", ["sym_int4", "asym_int4", "sym_int8"])
def test_gemv_glu_in_matches_glu_then_down(cuda, M, qtype):
    """down GEMV with the activation fused into its input staging == GLU GEMV + down GEMV"""
    fmt = Q.get_format(Q.resolve_qtype(qtype)).fmt
    H, I = 512, 1024
    g = torch.Generator(device="cuda").manual_seed(M)
    gu = ops.quantize(torch.randn(2 * I, H, generator=g, device=cuda) * 0.05, fmt)
    dn = ops.quantize(torch.randn(H, I, generator=g, device=cuda) * 0.05, fmt)
    x = (torch.randn(M, H, generator=g, device=cuda) * 0.5).to(torch.bfloat16)
    a = ops.gemv_glu(x, gu, fmt, 2 * I, H, 0)
    ref = ops.gemv_partials(a, dn, fmt, H, I, 0).sum(0)
    pg = ops.gemv_partials(x, gu, fmt, 2 * I, H, 0)
    out = ops.gemv_glu_in(pg, dn, fmt, H, I, 0, 0, torch.bfloat16).sum(0)
    assert ((out - ref).norm() / ref.norm()).item() < 1e-2
    # atomic form: gate/up accumulated into one slab, down accumulated atomically,
    # and an unrelated consumed buffer zeroed by the launch
    gacc = torch.zeros(M, 2 * I, device=cuda)
    ops.gemv_accum(x, gu, fmt, 2 * I, H, gacc)
    dacc = torch.zeros(M, H, device=cuda)
    junk = torch.ones(8 * 1024 + 4, device=cuda)
    ops.gemv_glu_in(gacc.unsqueeze(0), dn, fmt, H, I, 0, 0, torch.bfloat16, acc=dacc, zero=junk)
    assert ((dacc - ref).norm() / ref.norm()).item() < 1e-2
    assert junk.abs().max().item() == 0.0


def test_decode_mlp_acc_path_matches_glu_path(cuda):
    """batch 3..8 decode: gate/up atomics + down-with-GLU-prologue == GLU GEMV + down"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.decoder import NativeCausalLM
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=4)
    prompts = [list(range(1 + i, 40 + 3 * i)) for i in range(6)]
    outs = {}
    try:
        for flag in (False, True):
            NativeCausalLM._mlp_acc_env = flag
            outs[flag] = Engine(m).generate(prompts, max_new_tokens=10, use_graph=True)
    finally:
        NativeCausalLM._mlp_acc_env = True
    a, b = sum(outs[False], []), sum(outs[True], [])
    assert sum(x == y for x, y in zip(a, b)) >= 0.95 * len(a)


def test_rwkv4_wkv_kernel(cuda):
    """RWKV-4 WKV recurrence kernel vs HF rwkv_linear_attention_cpu (with and without state)"""
    from transformers.models.rwkv.modeling_rwkv import rwkv_linear_attention_cpu
    from ipex_llm_amd.models.rwkv import rwkv_linear_attention_native
    torch.manual_seed(0)
    B, T, C = 2, 37, 192
    w, u = torch.randn(C, device=cuda), torch.randn(C, device=cuda) * 0.5
    k, v = torch.randn(B, T, C, device=cuda), torch.randn(B, T, C, device=cuda)
    ref, rs = rwkv_linear_attention_cpu(w, u, k, v, return_state=True)
    got, gs = rwkv_linear_attention_native(w, u, k, v, return_state=True)
    assert (got - ref).abs().max().item() < 1e-4
    k2, v2 = torch.randn(B, 5, C, device=cuda), torch.randn(B, 5, C, device=cuda)
    r2, _ = rwkv_linear_attention_cpu(w, u, k2, v2, state=[s.clone() for s in rs])
    g2, _ = rwkv_linear_attention_native(w, u, k2, v2, state=gs)
    assert (g2 - r2).abs().max().item() < 1e-4


def test_rwkv_model_on_gpu_matches_cpu(cuda, tmp_path):
    """low-bit RWKV-4 on the GPU (WKV HIP kernel via the patched HF forward) vs the same model on CPU"""
    from transformers import RwkvConfig, RwkvForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    RwkvForCausalLM(RwkvConfig(vocab_size=128, hidden_size=128, num_hidden_layers=2, attention_hidden_size=128,
                               intermediate_size=256, context_length=64, rescale_every=1)).save_pretrained(tmp_path)
    ids = torch.randint(0, 128, (1, 11))
    m = AutoModelForCausalLM.from_pretrained(str(tmp_path), load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    with torch.no_grad():
        want = m(ids).logits
        got = m.to(cuda)(ids.to(cuda)).logits.cpu()
    # the CPU side runs sym_int8 on the int8-activation integer dot (per-64
    # activation quantization, as ggml's q8_0 path): ~1-2 % from the GPU
    assert ((got - want).norm() / want.norm()).item() < 3e-2


def test_hf_eager_family_on_gpu_uses_hip_softmax(cuda, tmp_path):
    """eager-configured HF-forward family (phi) on the GPU: illm_eager runs
    the in-place HIP softmax; logits stay close to the dense fp32 model"""
    from transformers import AutoConfig, AutoModelForCausalLM as HFAuto
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    # (an architecture the native decoder does not run, so the HF eager attention executes)
    cfg = AutoConfig.for_model("opt", hidden_size=128, ffn_dim=256, num_hidden_layers=2, word_embed_proj_dim=128,
                               num_attention_heads=4, vocab_size=256, max_position_embeddings=128)
    torch.manual_seed(0)
    ref = HFAuto.from_config(cfg, attn_implementation="eager").eval()
    p = str(tmp_path / "opt")
    ref.save_pretrained(p)
    ids = torch.randint(3, 256, (2, 16), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = ref(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.bfloat16,
                                             attn_implementation="eager").to(cuda)
    assert m.config._attn_implementation == "illm_eager"
    seen = []
    orig = torch.ops.ipex_llm_amd.attn_softmax_
    import ipex_llm_amd.ops.api as api

    class Spy:
        def __getattr__(self, n):
            return getattr(torch.ops.ipex_llm_amd, n)

        def attn_softmax_(self, x):
            seen.append(tuple(x.shape))
            return orig(x)
    real = api._ops
    api._ops = lambda: Spy()
    try:
        with torch.no_grad():
            got = m(ids.to(cuda)).logits.float().cpu()
    finally:
        api._ops = real
    assert seen and seen[0][-2:] == (16, 16)
    assert ((got - want).norm() / want.norm()).item() < 3e-2


@pytest.mark.parametrize("tile", [0, 16])
def test_glu_kernel_interleaved(cuda, tile):
    """GLU HIP op over halves (tile 0) and the 16-column gate/up interleave of
    the fused gate_up weight (the prefill library-GEMM path) vs the reference"""
    from ipex_llm_amd.models.decoder import deinterleave_glu
    torch.manual_seed(0)
    gu = torch.randn(37, 2 * 512, device=cuda).bfloat16()
    if tile:
        g, u = deinterleave_glu(gu, tile)
    else:
        g, u = gu.chunk(2, -1)
    want = torch.nn.functional.silu(g.float()).bfloat16().float() * u.float()
    got = ops.glu(gu, 0, tile=tile)
    assert torch.ops.ipex_llm_amd.glu is not None
    assert torch.allclose(got.float(), want, atol=1e-2, rtol=1e-2)
