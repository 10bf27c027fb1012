"""IQ lattice formats (gguf_iq2_xxs / gguf_iq2_xs / gguf_iq1_s): ggml's block
layouts and bits per weight (csrc/common/iquant.h), our own codebooks
(tools/gen_iq_grids.py) and imatrix-weighted quantizers
(csrc/cpu/iquant.cpp).  Reference: SRC/ggml/quantize.py:43-47 (qtype ids),
SRC/transformers/model.py:334-346 (imatrix-driven IQ quantization).  Parity
with ggml's grids is unpinned: the grid tables are not in the reference."""
import pytest
import torch

IQ = {"gguf_iq2_xxs": 2.0625, "gguf_iq2_xs": 2.3125, "gguf_iq1_s": 1.5625}


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("qtype,bpw", list(IQ.items()))
def test_bits_per_weight_and_round_trip(qtype, bpw):
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import get_format
    f = get_format(qtype)
    assert f.kquant and f.bits_per_weight == bpw
    torch.manual_seed(0)
    n, k = 64, 1024
    w = torch.randn(n, k) * 0.02
    blob = ops.kq_quantize(w, f.fmt)
    assert blob.numel() * 8 / (n * k) == bpw
    wd = ops.kq_dequantize(blob, f.fmt, n, k)
    err = _rel(wd, w)
    # Gaussian weights at ~2 / ~1.5 bits: the lattice error budget
    assert err < (0.62 if qtype == "gguf_iq1_s" else 0.42), err
    # the integer-constrained reconstruction beats a crude 1-level sign code
    sign_code = w.sign() * w.abs().mean()
    assert err < _rel(sign_code, w)


def test_imatrix_lowers_weighted_error():
    """importance-weighted search: columns marked important are reconstructed
    better than without the imatrix"""
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import get_format
    f = get_format("gguf_iq2_xxs").fmt
    torch.manual_seed(1)
    n, k = 64, 512
    w = torch.randn(n, k) * 0.02
    im = torch.ones(k)
    im[::2] = 100.0                        # importance varies inside every chunk
    e0 = (ops.kq_dequantize(ops.kq_quantize(w, f), f, n, k) - w)[:, ::2].pow(2).sum()
    e1 = (ops.kq_dequantize(ops.kq_quantize(w, f, im), f, n, k) - w)[:, ::2].pow(2).sum()
    assert e1 < e0, (e1, e0)


@pytest.mark.parametrize("qtype", list(IQ))
def test_cpu_linear_and_model(qtype):
    """the CPU k-quant GEMM decodes IQ blocks; a converted model runs"""
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd import ops, optimize_model
    from ipex_llm_amd.quantize import get_format
    from ipex_llm_amd.transformers.low_bit_linear import KQuantLinear
    f = get_format(qtype).fmt
    torch.manual_seed(2)
    n, k = 48, 512
    w = torch.randn(n, k) * 0.02
    blob = ops.kq_quantize(w, f)
    x = torch.randn(3, k)
    y = ops.kq_linear(x, blob, f, n, k)
    ref = x @ ops.kq_dequantize(blob, f, n, k).T
    assert _rel(y, ref) < 1e-5
    cfg = LlamaConfig(vocab_size=128, hidden_size=256, intermediate_size=512, num_hidden_layers=1,
                      num_attention_heads=4, num_key_value_heads=2)
    m = optimize_model(LlamaForCausalLM(cfg).eval(), low_bit=qtype)
    assert any(isinstance(mod, KQuantLinear) for mod in m.modules())
    with torch.no_grad():
        out = m(torch.randint(0, 128, (1, 5))).logits
    assert torch.isfinite(out).all()
