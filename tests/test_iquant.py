"""IQ lattice formats (gguf_iq2_xxs / gguf_iq2_xs / gguf_iq1_s / gguf_iq1_m): ggml's block
layouts and bits per weight (csrc/common/iquant.h), our own codebooks
(tools/gen_iq_grids.py) and imatrix-weighted quantizers
(csrc/cpu/iquant.cpp).  Reference: SRC/ggml/quantize.py:43-47 (qtype ids),
SRC/transformers/model.py:334-346 (imatrix-driven IQ quantization).  Parity
with ggml's grids is unpinned: the grid tables are not in the reference."""
import pytest
import torch

IQ = {"gguf_iq2_xxs": 2.0625, "gguf_iq2_xs": 2.3125, "gguf_iq1_s": 1.5625, "gguf_iq1_m": 1.75}


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
    assert err < (0.62 if qtype.startswith("gguf_iq1") else 0.42), err
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
    assert _rel(y, ref) < 2e-2                   # int8 activations (csrc/cpu/gemm_kq.cpp)
    cfg = LlamaConfig(vocab_size=128, hidden_size=256, intermediate_size=512, num_hidden_layers=1,
                      num_attention_heads=4, num_key_value_heads=2)
    m = optimize_model(LlamaForCausalLM(cfg).eval(), low_bit=qtype)
    assert any(isinstance(mod, KQuantLinear) for mod in m.modules())
    with torch.no_grad():
        out = m(torch.randint(0, 128, (1, 5))).logits
    assert torch.isfinite(out).all()


def test_iq1_m_finer_scales_beat_iq1_s():
    """iq1_m (3-bit scale per 16 weights, shift sign per 8; ggml's 56-byte block,
    d in the scale words' top nibbles) reconstructs better than iq1_s at 1.75
    vs 1.5625 bpw; the super-block scale round-trips through the nibbles"""
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import get_format
    torch.manual_seed(3)
    w = torch.randn(32, 1024) * 0.02
    errs = {}
    for q in ("gguf_iq1_s", "gguf_iq1_m"):
        f = get_format(q).fmt
        errs[q] = _rel(ops.kq_dequantize(ops.kq_quantize(w, f), f, 32, 1024), w)
    assert errs["gguf_iq1_m"] < errs["gguf_iq1_s"], errs
    f = get_format("gguf_iq1_m").fmt
    blob = ops.kq_quantize(w[:1, :256], f).view(torch.uint8)
    assert blob.numel() == 56
    sc = blob[48:56].to(torch.int32)
    words = sc[0::2] | (sc[1::2] << 8)
    d16 = int(((words[0] >> 12) | ((words[1] >> 8) & 0xF0) | ((words[2] >> 4) & 0xF00) | (words[3] & 0xF000)))
    d = torch.tensor([d16], dtype=torch.int16).view(torch.float16).float().item()
    assert 0 < d < 1
    # every weight is d * odd * (ternary +- 1/8): the block max is within the scale range
    wd = ops.kq_dequantize(blob, f, 1, 256)
    assert wd.abs().max().item() <= d * 15 * 1.125 + 1e-6
