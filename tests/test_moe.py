"""MoE (mixtral / qwen2_moe / qwen3_moe): low-bit expert banks, native MoE
decoder vs the HF forward on the same quantized experts, save/load, and the
routing helpers (reference: qwen3_moe.py:70-142, qwen2_moe.py:380-452)."""
import pytest
import torch

from ipex_llm_amd.ops import reference as R


def _tiny(tmp_path, mt, topk=2):
    from transformers import AutoConfig, AutoModelForCausalLM as HF
    torch.manual_seed(0)
    kw = dict(vocab_size=256, hidden_size=128, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=256)
    if mt == "mixtral":
        kw.update(num_local_experts=4, num_experts_per_tok=topk)
    else:
        kw.update(num_experts=4, num_experts_per_tok=topk, moe_intermediate_size=64, norm_topk_prob=mt == "qwen3_moe")
        if mt == "qwen2_moe":
            kw.update(shared_expert_intermediate_size=128)
        if mt == "qwen3_moe":
            kw.update(head_dim=32)
    cfg = AutoConfig.for_model(mt, **kw)
    hf = HF.from_config(cfg).eval()
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if p.dim() == 3 or "gate" in n:
                p.normal_(0, 0.05)
    p = str(tmp_path / mt)
    hf.save_pretrained(p)
    return hf, p


@pytest.mark.parametrize("mt", ["mixtral", "qwen2_moe", "qwen3_moe"])
def test_native_moe_matches_hf_forward(tmp_path, mt):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.models.moe import HFLowBitExperts
    # every expert active: no routing discontinuity from quantization noise
    hf, p = _tiny(tmp_path, mt, topk=4)
    ids = torch.randint(0, 256, (2, 10))
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    assert isinstance(m.model.layers[0].mlp.experts, HFLowBitExperts)
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        nat = m(ids).logits.float()
        ref = hf(ids).logits.float()
    assert ((nat - ref).norm() / ref.norm()).item() < 3e-2
    g = m.generate(ids, max_new_tokens=4)
    assert g.shape == (2, 14)


def test_moe_save_load_low_bit(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    _, p = _tiny(tmp_path, "qwen2_moe")
    m = AutoModelForCausalLM.from_pretrained(p, load_in_4bit=True, torch_dtype=torch.float32)
    ids = torch.randint(0, 256, (1, 8))
    with torch.no_grad():
        a = m(ids).logits
    m.save_low_bit(str(tmp_path / "q"))
    m2 = AutoModelForCausalLM.load_low_bit(str(tmp_path / "q"))
    with torch.no_grad():
        b = m2(ids).logits
    assert torch.allclose(a, b, atol=1e-5)


def test_moe_align_and_combine_reference():
    ids = torch.tensor([[2, 0], [1, 2], [2, 3]], dtype=torch.int32)
    off, rows = R.moe_align(ids, 0, 4)
    assert off.tolist() == [0, 1, 2, 5, 6]
    assert rows[:6].tolist() == [1, 2, 0, 3, 4, 5]
    # EP: local experts 2..3 only
    off2, rows2 = R.moe_align(ids, 2, 2)
    assert off2.tolist() == [0, 3, 4] and rows2[:4].tolist() == [0, 3, 4, 5]
    part = torch.randn(2, 6, 8)
    w = torch.rand(3, 2)
    y = R.moe_combine(part, w, ids, 2, 2, torch.float32)
    s = part.sum(0)
    exp0 = w[0, 0] * s[0]
    assert torch.allclose(y[0], exp0, atol=1e-6)


def test_hf_lowbit_experts_matches_dequantized_bank():
    from transformers import MixtralConfig
    from transformers.models.mixtral.modeling_mixtral import MixtralExperts
    from ipex_llm_amd.models.moe import HFLowBitExperts
    from ipex_llm_amd.models.decoder import deinterleave_glu
    torch.manual_seed(0)
    cfg = MixtralConfig(hidden_size=128, intermediate_size=64, num_local_experts=4)
    ex = MixtralExperts(cfg)
    with torch.no_grad():
        ex.gate_up_proj.normal_(0, 0.05)
        ex.down_proj.normal_(0, 0.05)
    q = HFLowBitExperts.from_hf(ex, "sym_int8")
    # same forward on the dequantized weights
    for e in range(4):
        gu = q.gate_up.dequantize(e)
        g, u = deinterleave_glu(gu.t().contiguous())
        ex.gate_up_proj.data[e] = torch.cat([g.t(), u.t()], 0)
        ex.down_proj.data[e] = q.down.dequantize(e)
    x = torch.randn(5, 128)
    idx = torch.tensor([[0, 1], [2, 3], [1, 2], [3, 0], [2, 1]])
    w = torch.rand(5, 2)
    with torch.no_grad():
        # the CPU expert GEMMs quantize activations to int8 per 64-block (sym_int8 x q8 dots)
        a, b = q(x, idx, w), ex(x, idx, w)
        assert ((a - b).norm() / b.norm()).item() < 2e-2
