"""AutoModel API on CPU: low-bit load, native forward/generate parity with HF,
save_low_bit/load_low_bit round trip (reference test_transformers_api.py)."""
import shutil

import pytest
import torch

ARCHS = [("llama", {}), ("qwen2", {}), ("mistral", {}), ("qwen3", {"head_dim": 32}),
         ("gemma", {"head_dim": 32}), ("gemma2", {"head_dim": 32}), ("phi3", {"pad_token_id": 0})]


def _tiny(tmp_path, mt, extra):
    from transformers import AutoConfig, AutoModelForCausalLM as HF
    torch.manual_seed(0)
    cfg = AutoConfig.for_model(mt, vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                               num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512, **extra)
    hf = HF.from_config(cfg).eval()
    p = str(tmp_path / mt)
    hf.save_pretrained(p)
    return hf, p


@pytest.mark.parametrize("mt,extra", ARCHS)
def test_native_forward_matches_hf(tmp_path, mt, extra):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    hf, p = _tiny(tmp_path, mt, extra)
    ids = torch.randint(0, 320, (2, 12))
    with torch.no_grad():
        ref = hf(ids).logits.float()
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32)
    assert getattr(m, "_illm_native_attached", False)
    with torch.no_grad():
        out = m(ids).logits.float()
    assert ((out - ref).norm() / ref.norm()).item() < 2e-2


def test_low_bit_save_load_generate(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    hf, p = _tiny(tmp_path, "llama", {})
    m = AutoModelForCausalLM.from_pretrained(p, load_in_4bit=True, torch_dtype=torch.float32)
    ids = torch.randint(0, 320, (2, 10))
    with torch.no_grad():
        out = m(ids).logits
        ref = hf(ids).logits
    # int4 vs fp32: logits close on average (reference: <5% mean relative diff)
    assert ((out - ref).abs().mean() / ref.abs().mean()).item() < 0.25
    g = m.generate(ids, max_new_tokens=6)
    assert g.shape == (2, 16) and torch.equal(g[:, :10], ids)
    m.save_low_bit(str(tmp_path / "int4"))
    m2 = AutoModelForCausalLM.load_low_bit(str(tmp_path / "int4"))
    with torch.no_grad():
        out2 = m2(ids).logits
    assert torch.allclose(out, out2, atol=1e-5)
    assert torch.equal(m2.generate(ids, max_new_tokens=6), g)


def test_incremental_forward_with_cache(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    _, p = _tiny(tmp_path, "llama", {})
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32)
    ids = torch.randint(0, 320, (1, 9))
    with torch.no_grad():
        full = m(ids).logits
        o1 = m(ids[:, :6], use_cache=True)
        o2 = m(ids[:, 6:], past_key_values=o1.past_key_values)
    assert torch.allclose(full[:, 6:], o2.logits, atol=1e-4)


def test_optimize_model_generic_module():
    import torch.nn as nn
    from ipex_llm_amd import optimize_model
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    net = nn.Sequential(nn.Linear(128, 256), nn.ReLU(), nn.Linear(256, 64), nn.Linear(64, 30))
    x = torch.randn(3, 128)
    ref = net(x)
    optimize_model(net, low_bit="sym_int8")
    assert isinstance(net[0], LowBitLinear) and isinstance(net[2], LowBitLinear)
    assert not isinstance(net[3], LowBitLinear) or net[3].in_features % 64 == 0
    assert ((net(x) - ref).norm() / ref.norm()).item() < 0.05


def test_remote_code_flash_attn_import_filter(tmp_path):
    """reference patches.py: a remote modelling file importing flash_attn still passes the import check"""
    from ipex_llm_amd.transformers.patches import patch_flash_attn_import, remote_code_patches
    f = tmp_path / "modeling_x.py"
    f.write_text("import torch\nimport flash_attn\nimport einops\n")
    import transformers.dynamic_module_utils as dmu
    assert "flash_attn" in dmu.get_imports(str(f))
    assert "flash_attn" not in patch_flash_attn_import(str(f))
    with remote_code_patches():
        assert "flash_attn" not in dmu.get_imports(str(f)) and "einops" in dmu.get_imports(str(f))


class _CharTok:
    """character-level tokenizer (ids = printable chars + EOS) for the schema tests"""
    chars = [chr(c) for c in range(32, 127)]

    def __init__(self):
        self.eos_token_id = len(self.chars)

    def decode(self, ids, skip_special_tokens=True):
        return "".join(self.chars[i] for i in ids if i < len(self.chars))


def test_json_schema_logits_processor_enforces_schema():
    """schema-constrained decoding (reference xgrammar.create_json_logits_processor
    with a JSON schema): random logits, every finished document is valid"""
    import json
    from ipex_llm_amd.transformers.xgrammar import create_json_logits_processor
    schema = {"type": "object",
              "properties": {"name": {"type": "string", "maxLength": 6}, "age": {"type": "integer"},
                             "kind": {"enum": ["cat", "dog"]},
                             "tags": {"type": "array", "items": {"type": "boolean"}, "maxItems": 2}},
              "required": ["name", "age", "kind"]}
    tok = _CharTok()
    V = tok.eos_token_id + 1
    for seed in range(4):
        g = torch.Generator().manual_seed(seed)
        proc = create_json_logits_processor(tok, V, schema)
        ids = torch.tensor([[0, 1]])                     # "prompt"
        for _ in range(200):
            scores = torch.randn(1, V, generator=g)
            scores[0, tok.eos_token_id] -= 2.0
            nxt = int(torch.argmax(proc(ids, scores)[0]))
            ids = torch.cat([ids, torch.tensor([[nxt]])], 1)
            if nxt == tok.eos_token_id:
                break
        text = tok.decode(ids[0, 2:].tolist())
        assert ids[0, -1].item() == tok.eos_token_id, text
        doc = json.loads(text)
        assert set(doc) >= {"name", "age", "kind"} and doc["kind"] in ("cat", "dog"), doc
        assert isinstance(doc["age"], int) and len(doc["name"]) <= 6
        assert all(isinstance(x, bool) for x in doc.get("tags", []))
