"""Native GGUF k-quant formats (q4_k / q5_k / q6_k / q2_k): C++ quantizer +
dequantizer vs the independent numpy GGUF decoder (gguf/reader.py), bits per
weight equal to the reference qtypes, KQuantLinear forward, the converter's
gguf_q4k_s / gguf_q4k_m per-module policy (reference
SRC/transformers/utils.py:337-352) and low-bit checkpoint round trips.
Parity with llama.cpp's quantizer is unpinned (no llama.cpp here): the block
layouts are GGUF's, the search is the published ggml design."""
import numpy as np
import pytest
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.quantize import qtypes as Q

KQ = {"q4_k": (Q.FMT_Q4K, 144, 0.09), "q5_k": (Q.FMT_Q5K, 176, 0.045), "q6_k": (Q.FMT_Q6K, 210, 0.02),
      "q2_k": (Q.FMT_Q2K, 84, 0.45)}
GGUF_T = {"q4_k": 12, "q5_k": 13, "q6_k": 14}


@pytest.mark.parametrize("name", list(KQ))
def test_round_trip_and_bpw(name):
    fmt, bb, tol = KQ[name]
    n, k = 24, 512
    w = torch.randn(n, k) * 0.05
    blob = ops.kq_quantize(w, fmt)
    assert blob.numel() == n * (k // 256) * bb
    assert Q.get_format(name).bits_per_weight == bb * 8 / 256
    deq = ops.kq_dequantize(blob, fmt, n, k)
    rel = ((deq - w).norm() / w.norm()).item()
    assert rel < tol, rel
    if name in GGUF_T:
        from ipex_llm_amd.gguf.reader import dequantize
        ref = dequantize(blob.numpy(), GGUF_T[name], n * k).reshape(n, k)
        np.testing.assert_allclose(deq.numpy(), ref, rtol=1e-6, atol=1e-7)


def test_imatrix_lowers_weighted_error():
    fmt = Q.FMT_Q4K
    torch.manual_seed(1)
    n, k = 32, 256
    w = torch.randn(n, k) * 0.05
    im = torch.rand(k) ** 4 * 10
    e0 = (((ops.kq_dequantize(ops.kq_quantize(w, fmt), fmt, n, k) - w) ** 2) * im).sum()
    e1 = (((ops.kq_dequantize(ops.kq_quantize(w, fmt, im), fmt, n, k) - w) ** 2) * im).sum()
    assert e1 < e0


@pytest.mark.parametrize("name", ["q4_k", "q6_k", "q2_k"])
def test_kquant_linear_cpu(name):
    from ipex_llm_amd.transformers.low_bit_linear import KQuantLinear
    lin = torch.nn.Linear(256, 48, bias=True)
    m = KQuantLinear.from_linear(lin, name)
    x = torch.randn(3, 256)
    want = torch.nn.functional.linear(x, m.dequantize(), lin.bias)
    got = m(x)
    # int8 activations against the super-block codes (csrc/cpu/gemm_kq.cpp,
    # ggml's q8 x k-quant form): equal up to the activation rounding
    assert ((got - want).norm() / want.norm()).item() < 2e-2


def _tiny(path):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=256, hidden_size=256, intermediate_size=512, num_hidden_layers=4,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    m = LlamaForCausalLM(cfg).eval()
    m.save_pretrained(path)
    return m


def test_from_pretrained_kquant_and_mixed_policy(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.low_bit_linear import KQuantLinear
    p = str(tmp_path / "m")
    dense = _tiny(p)
    ids = torch.randint(0, 256, (1, 10))
    with torch.no_grad():
        want = dense(ids).logits
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="q4_k", torch_dtype=torch.float32).eval()
    kq = [mod for mod in m.modules() if isinstance(mod, KQuantLinear)]
    assert kq and all(mod.qtype == Q.Q4_K for mod in kq)
    with torch.no_grad():
        got = m(ids).logits
    rel_kq = ((got - want).norm() / want.norm()).item()
    # a random-init 4-layer model compounds 4-bit error (~0.2 for every 4-bit
    # qtype); q4_k's per-sub-block scale + min must beat per-32 sym_int4
    ms = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int4", torch_dtype=torch.float32).eval()
    with torch.no_grad():
        rel_s4 = ((ms(ids).logits - want).norm() / want.norm()).item()
    assert rel_kq < 0.25 and rel_kq < rel_s4, (rel_kq, rel_s4)
    # gguf_q4k_m: lm_head q6_k; qkv / down of the first half of the layers q6_k
    mm = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="gguf_q4k_m", torch_dtype=torch.float32)
    q = {n: mod.qtype for n, mod in mm.named_modules() if isinstance(mod, KQuantLinear)}
    assert q["lm_head"] == Q.Q6_K
    assert q["model.layers.0.mlp.down_proj"] == Q.Q6_K and q["model.layers.3.mlp.down_proj"] == Q.Q4_K
    assert q["model.layers.1.self_attn.qkv_proj"] == Q.Q6_K and q["model.layers.2.self_attn.o_proj"] == Q.Q4_K
    # save / load round trip keeps the GGUF blocks
    sd = str(tmp_path / "saved")
    m.save_low_bit(sd)
    m2 = AutoModelForCausalLM.load_low_bit(sd, torch_dtype=torch.float32).eval()
    with torch.no_grad():
        assert torch.allclose(m2(ids).logits, got, atol=1e-5)


def test_hidden_not_multiple_of_256_falls_back():
    from ipex_llm_amd.transformers.convert import _convert_one
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    lin = torch.nn.Linear(192, 64)
    m = _convert_one(lin, Q.Q4_K, "cpu")
    assert isinstance(m, LowBitLinear) and m.qtype == Q.ASYM_INT4


def test_iq_qtypes_use_native_2bit_super_blocks():
    """gguf_iq2_xxs / iq2_xs / iq1_s / iq1_m are native IQ lattice
    super-blocks (csrc/common/iquant.h) -- never a 4-bit stand-in"""
    import torch
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.quantize import qtypes as Q
    from ipex_llm_amd.transformers.convert import ggml_convert_low_bit
    for name in ("gguf_iq2_xxs", "gguf_iq2_xs", "gguf_iq1_s", "gguf_iq1_m"):
        f = Q.get_format(name)
        assert f.name == name and f.bits <= 2 and f.kquant
    assert Q.get_format("gguf_iq1_m").bits_per_weight == 1.75
    cfg = LlamaConfig(vocab_size=64, hidden_size=256, intermediate_size=512, num_hidden_layers=1, num_attention_heads=4)
    torch.manual_seed(0)
    m = LlamaForCausalLM(cfg).eval()
    ggml_convert_low_bit(m, "gguf_iq2_xxs", optimize_model=False)
    lins = [x for x in m.model.modules() if type(x).__name__ == "KQuantLinear"]
    assert lins
    for lin in lins:
        bpw = 8 * lin.weight.numel() / (lin.in_features * lin.out_features)
        assert bpw < 3.0, bpw


@pytest.mark.parametrize("qtype", ["q4_k", "q5_k", "q6_k", "q2_k", "gguf_iq2_xxs", "gguf_iq2_xs",
                                   "gguf_iq1_s", "gguf_iq1_m"])
def test_cpu_integer_gemm_from_super_blocks(qtype):
    """csrc/cpu/gemm_kq.cpp: int8 activations x unpacked u8 codes straight from
    the GGUF super-blocks (AVX2 and AVX-512 VNNI) == the f32 GEMM over the
    dequantized weight up to the int8 activation rounding; the auto path
    dequantizes + GEMMs at >= 512 rows (the reference's linear threshold)"""
    import torch
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import get_format
    f = get_format(qtype).fmt
    torch.manual_seed(5)
    n, k = 72, 768
    w = torch.randn(n, k) * 0.02
    blob = ops.kq_quantize(w, f)
    wd = ops.kq_dequantize(blob, f, n, k)
    isas = [1, 2] if "avx512_vnni" in open("/proc/cpuinfo").read() else [1]
    for m in (1, 3, 9):
        x = torch.randn(m, k)
        ref = x @ wd.T
        for isa in isas:
            y = torch.ops.ipex_llm_amd.kq_linear_isa(x, blob, f, n, k, isa)
            assert ((y - ref).norm() / ref.norm()).item() < 2e-2, (qtype, m, isa)
        assert torch.equal(torch.ops.ipex_llm_amd.kq_linear_isa(x, blob, f, n, k, 0),
                           torch.ops.ipex_llm_amd.kq_linear_isa(x, blob, f, n, k, isas[-1]))
    x = torch.randn(512, k)
    y = ops.kq_linear(x, blob, f, n, k)
    assert torch.allclose(y, x @ wd.T, atol=1e-4, rtol=1e-4)
