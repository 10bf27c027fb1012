"""Reading reference (``save_low_bit``) checkpoints: ggml CPU-layout blocks
are converted to our canonical planar layout, never reinterpreted.

Layout parity is unpinned: the reference ships no low-bit checkpoint, so the
ggml blobs here are built from the documented block layout
(``vllm_for_multi_arc.patch:4815-4912`` block structs, ``:3944-3975`` nibble
order) and the logits of the loaded model must equal the model they came from.
"""
import json
import os

import pytest
import torch

from ipex_llm_amd.quantize import qtypes as Q
from ipex_llm_amd.transformers import ref_checkpoint as RC


@pytest.mark.parametrize("qt", ["sym_int4", "woq_int4", "asym_int4", "sym_int8", "nf4", "fp4", "fp8_e4m3"])
def test_ggml_canonical_round_trip(qt):
    from ipex_llm_amd import ops
    f = Q.get_format(qt).fmt
    n, k = 24, 192
    w = torch.randn(n, k)
    canon = ops.quantize(w, f)
    g = RC.canonical_to_ggml(canon, qt, n, k)
    back = RC.ggml_to_canonical(g, qt, n, k)
    if qt in ("sym_int8", "fp8_e4m3"):       # f32 scales in ggml: fp16 -> f32 -> fp16 is exact
        assert torch.equal(back, canon)
    else:
        assert torch.equal(back, canon)


def test_q4_0_block_bytes_documented_layout():
    """one 64-element row: [fp16 d][byte j = e[j] | e[j+32] << 4]"""
    from ipex_llm_amd import ops
    w = torch.linspace(-1, 1, 64).reshape(1, 64)
    canon = ops.quantize(w, Q.get_format("sym_int4").fmt)
    g = RC.canonical_to_ggml(canon, "sym_int4", 1, 64)
    assert g.numel() == 34
    d = g[:2].view(torch.float16).float().item()
    qs = g[2:].long()
    codes = torch.cat([qs & 15, qs >> 4])
    deq = (codes.float() - 8) * d
    assert torch.allclose(deq, w.reshape(-1), atol=abs(d) * 1.01)
    # woq: element 2j low, 2j + 1 high
    gw = RC.canonical_to_ggml(canon, "woq_int4", 1, 64)
    qw = gw[2:].long()
    cw = torch.stack([qw & 15, qw >> 4], -1).reshape(-1)
    assert torch.equal(cw, codes)


def test_reference_q4k_layout_round_trip():
    """the reference's 148-byte block_q4_K (fp16 d, fp16 dmin, 8-bit scales
    then mins, GGUF nibble order; VLLM_PATCH:4932-4937) <-> our GGUF 144-byte
    block: exact both ways while the scales fit 6 bits, and its decode formula
    equals our q4_k dequantization"""
    from ipex_llm_amd import ops
    fmt = Q.get_format("q4_k").fmt
    n, k = 6, 512
    w = torch.randn(n, k)
    ours = ops.kq_quantize(w, fmt).reshape(-1).view(torch.uint8)
    ref = RC.canonical_to_ggml(ours, "q4_k", n, k)
    assert ref.numel() == n * (k // 256) * 148
    blk = ref.view(-1, 148)
    assert int(blk[:, 4:20].max()) < 64                     # 6-bit values carried in bytes
    assert torch.equal(RC.ggml_to_canonical(ref, "q4_k", n, k), ours)
    want = ops.kq_dequantize(ours, fmt, n, k).float()
    torch.testing.assert_close(RC.q4k_ref_dequantize(ref, n, k), want, rtol=1e-5, atol=1e-6)
    # an 8-bit scale past 6 bits: decoded and re-quantized (close, not exact)
    big = blk.clone()
    big[:, 4:12] = (big[:, 4:12].to(torch.int32) * 2).clamp(max=255).to(torch.uint8)
    big[:, 0:2] = (big[:, 0:2].contiguous().view(torch.float16) / 2).view(torch.uint8)
    with pytest.warns(UserWarning):
        conv = RC.ggml_to_canonical(big.reshape(-1), "q4_k", n, k)
    dq = ops.kq_dequantize(conv, fmt, n, k).float()
    exact = RC.q4k_ref_dequantize(big.reshape(-1), n, k)
    assert ((dq - exact).norm() / exact.norm()).item() < 0.08


def test_wrong_size_refused():
    with pytest.raises(ValueError):
        RC.ggml_to_canonical(torch.zeros(100, dtype=torch.uint8), "sym_int4", 2, 64)
    with pytest.raises(ValueError):
        RC.ggml_to_canonical(torch.zeros(100, dtype=torch.uint8), "q4_k", 2, 64)


def _split_gate_up(blob, fmt, n2, k):
    from ipex_llm_amd.transformers.low_bit_linear import canon_join, canon_planes
    pl = canon_planes(blob, fmt, n2, k)
    I = n2 // 2

    def de(x):
        if x is None:
            return None, None
        t = x.reshape(I // 16, 2, 16, x.shape[-1])
        return t[:, 0].reshape(I, -1), t[:, 1].reshape(I, -1)
    g = [de(x)[0] for x in pl]
    u = [de(x)[1] for x in pl]
    return canon_join(*g), canon_join(*u)


def _split_rows(blob, fmt, n, k, rows):
    from ipex_llm_amd.transformers.low_bit_linear import canon_join, canon_planes
    pl = canon_planes(blob, fmt, n, k)
    outs, r0 = [], 0
    for r in rows:
        outs.append(canon_join(*[None if x is None else x[r0:r0 + r] for x in pl]))
        r0 += r
    return outs


def _kq_split_rows(blob, n, rows):
    v = blob.view(n, -1)
    outs, r0 = [], 0
    for r in rows:
        outs.append(v[r0:r0 + r].reshape(-1).clone())
        r0 += r
    return outs


def _kq_split_gate_up(blob, n2):
    t = blob.view(n2 // 32, 2, 16, -1)
    return t[:, 0].reshape(-1).clone(), t[:, 1].reshape(-1).clone()


@pytest.mark.parametrize("qt", ["sym_int4", "asym_int4", "q6_k", "q5_k", "q2_k", "q4_k"])
def test_load_reference_checkpoint_logits(tmp_path, qt):
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    kq = qt.endswith("_k")
    h = 256 if kq else 128
    cfg = LlamaConfig(vocab_size=256, hidden_size=h, intermediate_size=2 * h, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    torch.manual_seed(0)
    dense = LlamaForCausalLM(cfg).eval()
    dpath = tmp_path / "dense"
    dense.save_pretrained(dpath)
    ours = AutoModelForCausalLM.from_pretrained(str(dpath), load_in_low_bit=qt, torch_dtype=torch.float32).eval()
    ids = torch.randint(0, 256, (1, 12))
    with torch.no_grad():
        want = ours(ids).logits.float()
    # re-express our weights in the reference layout: separate q/k/v and
    # gate/up projections, ggml blocks, pickled state dict
    fmt = Q.get_format(qt).fmt
    sd = {}
    hd = cfg.hidden_size // cfg.num_attention_heads
    for name, mod in ours.named_modules():
        from ipex_llm_amd.transformers.low_bit_linear import KQuantLinear, LowBitLinear
        if not isinstance(mod, (LowBitLinear, KQuantLinear)):
            continue
        n, k = mod.out_features, mod.in_features
        blob = mod.weight.data.reshape(-1).cpu() if kq else mod.canonical_blob()
        parent = name.rsplit(".", 1)[0]
        if name.endswith("qkv_proj"):
            rows = [cfg.num_attention_heads * hd, cfg.num_key_value_heads * hd, cfg.num_key_value_heads * hd]
            parts = _kq_split_rows(blob, n, rows) if kq else _split_rows(blob, fmt, n, k, rows)
            for p, b, r in zip("qkv", parts, rows):
                sd[f"{parent}.{p}_proj.weight"] = RC.canonical_to_ggml(b, qt, r, k)
        elif name.endswith("gate_up_proj"):
            g, u = _kq_split_gate_up(blob, n) if kq else _split_gate_up(blob, fmt, n, k)
            sd[f"{parent}.gate_proj.weight"] = RC.canonical_to_ggml(g, qt, n // 2, k)
            sd[f"{parent}.up_proj.weight"] = RC.canonical_to_ggml(u, qt, n // 2, k)
        else:
            sd[name + ".weight"] = RC.canonical_to_ggml(blob, qt, n, k)
    for key, v in ours.state_dict().items():
        if "proj" not in key and "lm_head" not in key:
            sd[key] = v.clone()
    rpath = tmp_path / "ref_lowbit"
    os.makedirs(rpath)
    torch.save(sd, rpath / "pytorch_model.bin")
    c = cfg.to_dict()
    c["bigdl_transformers_low_bit"] = qt
    c["torch_dtype"] = "float32"
    with open(rpath / "config.json", "w") as f:
        json.dump(c, f)
    assert RC.is_reference_low_bit_dir(str(rpath))
    loaded = AutoModelForCausalLM.load_low_bit(str(rpath), torch_dtype=torch.float32).eval()
    with torch.no_grad():
        got = loaded(ids).logits.float()
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4)


def test_unknown_layout_refused(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from transformers import LlamaConfig
    cfg = LlamaConfig(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                      num_attention_heads=2, num_key_value_heads=2)
    cfg.save_pretrained(tmp_path)
    with open(tmp_path / "illm_low_bit.json", "w") as f:
        json.dump({"qtype": "sym_int4", "format": "something-else-v9"}, f)
    with pytest.raises(ValueError, match="unknown low-bit layout"):
        AutoModelForCausalLM.load_low_bit(str(tmp_path))
    os.remove(tmp_path / "illm_low_bit.json")
    with pytest.raises(ValueError, match="not a low-bit checkpoint"):
        AutoModelForCausalLM.load_low_bit(str(tmp_path))


def test_own_safetensors_without_marker_refused(tmp_path):
    """one of our save_low_bit directories that lost illm_low_bit.json (but
    kept bigdl_transformers_low_bit in config.json) must not be read as a
    reference (ggml-block) checkpoint: the reference writes .bin only"""
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.ref_checkpoint import load_reference_state_dict
    from transformers import LlamaConfig
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=64, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                      num_attention_heads=2, num_key_value_heads=2)
    from transformers import LlamaForCausalLM
    base = tmp_path / "base"
    LlamaForCausalLM(cfg).save_pretrained(base)
    m = AutoModelForCausalLM.from_pretrained(str(base), load_in_low_bit="sym_int4")
    out = tmp_path / "ours"
    m.save_low_bit(str(out))
    os.remove(out / "illm_low_bit.json")
    with pytest.raises(ValueError, match="not a reference"):
        load_reference_state_dict(str(out))
