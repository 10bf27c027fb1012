"""vLLM adapter (reference SRC/vllm/xpu/model_convert.py) on duck-typed
vLLM layer classes, and hybrid host/device MoE execution (reference
convert.py:2142-2166, convert_model_hybrid)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F


class ColumnParallelLinear(nn.Module):
    def __init__(self, k, n, bias=True, gather_output=False, skip_bias_add=False):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(n, k) * 0.1)
        self.bias = nn.Parameter(torch.randn(n) * 0.1) if bias else None
        self.gather_output, self.skip_bias_add = gather_output, skip_bias_add

    def forward(self, x):
        if self.skip_bias_add:
            return F.linear(x, self.weight), self.bias
        return F.linear(x, self.weight, self.bias), None


class QKVParallelLinear(ColumnParallelLinear):
    pass


class RowParallelLinear(ColumnParallelLinear):
    reduce_results = True


class ToyVLLMModel(nn.Module):
    def __init__(self):
        super().__init__()
        self.qkv = QKVParallelLinear(128, 384, bias=True)
        self.down = RowParallelLinear(384, 128, bias=True, skip_bias_add=True)
        self.head = nn.Linear(128, 64)

    def forward(self, x):
        h, _ = self.qkv(x)
        y, b = self.down(torch.relu(h))
        return self.head(y + (b if b is not None else 0))


def test_vllm_linears_convert_and_match():
    from ipex_llm_amd.vllm import VLLMLowBitLinear, convert_vllm_linears
    torch.manual_seed(0)
    m = ToyVLLMModel().eval()
    x = torch.randn(5, 128)
    with torch.no_grad():
        want = m(x)
    n = convert_vllm_linears(m, "sym_int8", modules_to_not_convert=["head"])
    assert n == 2 and isinstance(m.qkv, VLLMLowBitLinear) and isinstance(m.down, VLLMLowBitLinear)
    assert isinstance(m.head, nn.Linear)                    # plain nn.Linear is vLLM's business
    y, b = m.down(torch.randn(2, 384))
    assert b is not None and b.shape == (128,)              # skip_bias_add keeps the (out, bias) contract
    with torch.no_grad():
        got = m(x)
    assert ((got - want).norm() / want.norm()).item() < 2e-2
    assert convert_vllm_linears(ToyVLLMModel(), "bf16") == 0


def test_patch_vllm_requires_vllm():
    from ipex_llm_amd.vllm import patch_vllm
    try:
        import vllm  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            patch_vllm("sym_int4")


def _moe(tmp_path):
    from transformers import Qwen2MoeConfig, Qwen2MoeForCausalLM
    torch.manual_seed(0)
    cfg = Qwen2MoeConfig(vocab_size=256, hidden_size=64, intermediate_size=128, moe_intermediate_size=64,
                         shared_expert_intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                         num_key_value_heads=2, num_experts=4, num_experts_per_tok=2, max_position_embeddings=128)
    hf = Qwen2MoeForCausalLM(cfg).eval()
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if n.endswith(".gate.weight"):
                p.normal_(0, 1.0)
    p = str(tmp_path / "moe")
    hf.save_pretrained(p)
    return p


def test_hybrid_islands_cpu(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.hybrid import DeviceIsland, convert_model_hybrid
    p = _moe(tmp_path)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    ids = torch.randint(0, 256, (1, 9), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        want = m(ids).logits.float()
    # islands in float64 on "cpu": exercises the in/out moves + casts and the pinned placement
    convert_model_hybrid(m, device="cpu", dtype=torch.float64)
    layer = m.model.layers[0]
    assert isinstance(layer.self_attn, DeviceIsland) and not isinstance(layer.mlp, DeviceIsland)
    with torch.no_grad():
        got = m(ids).logits.float()
        gen = m.generate(ids, max_new_tokens=3, do_sample=False)
    assert ((got - want).norm() / want.norm()).item() < 2e-2
    assert gen.shape[1] >= 10
    m.to(torch.float32)                                      # islands keep their placement / dtype
    fl = [q for q in layer.self_attn.parameters() if q.is_floating_point()]
    assert fl and all(q.dtype == torch.float64 for q in fl)


@pytest.mark.gpu
def test_hybrid_attention_on_gpu(tmp_path, cuda):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.hybrid import convert_model_hybrid
    p = _moe(tmp_path)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    ids = torch.randint(0, 256, (1, 9), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        want = m(ids).logits.float()
    convert_model_hybrid(m, device=cuda, dtype=torch.bfloat16)
    assert next(m.model.layers[0].self_attn.parameters()).is_cuda
    assert not any(q.is_cuda for n, q in m.named_parameters() if "experts" in n)
    with torch.no_grad():
        got = m(ids).logits.float()
    assert got.device.type == "cpu"
    assert ((got - want).norm() / want.norm()).item() < 6e-2
