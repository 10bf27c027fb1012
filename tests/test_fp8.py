"""torch_fp8_e4m3 / torch_fp8_e5m2 qtypes (reference run_linear_fp8): the
host op is the f32 emulation of the GPU path (per-token e4m3 activations x
fp8 weight x scales), checked here against an independent torch
formulation; module conversion and low-bit round trip."""
import pytest
import torch

from ipex_llm_amd import ops


def _ref(x, w8, ws, bias, e5m2):
    xf = x.float()
    amax = xf.abs().amax(-1, keepdim=True)
    sx = torch.where(amax > 0, amax / 448, torch.ones_like(amax))
    xq = (xf / sx).clamp(-448, 448).to(torch.float8_e4m3fn).float() * sx
    wd = w8.view(torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn).float() * ws.view(-1, 1)
    y = xq @ wd.t()
    return y + bias.float() if bias is not None else y


@pytest.mark.parametrize("e5m2", [False, True])
@pytest.mark.parametrize("per_channel", [False, True])
def test_fp8_linear_cpu_matches_emulation(e5m2, per_channel):
    torch.manual_seed(0)
    w = torch.randn(96, 256) * 0.05
    x = torch.randn(5, 256)
    b = torch.randn(96)
    w8, ws = ops.fp8_quantize_weight(w, e5m2, per_channel)
    assert w8.dtype == torch.uint8 and ws.numel() == (96 if per_channel else 1)
    y = ops.fp8_linear(x, w8, ws, b, e5m2)
    torch.testing.assert_close(y, _ref(x, w8, ws, b, e5m2), rtol=1e-5, atol=1e-5)
    rel = ((y - (x @ w.t() + b)).norm() / (x @ w.t() + b).norm()).item()
    assert rel < (0.08 if e5m2 else 0.05), rel


def test_fp8_act_quant_cpu():
    x = torch.randn(3, 64) * 4
    q, s = ops.fp8_act_quant(x)
    assert q.dtype == torch.uint8 and s.shape == (3,)
    back = q.view(torch.float8_e4m3fn).float() * s[:, None]
    assert ((back - x).norm() / x.norm()).item() < 0.05
    torch.testing.assert_close(s, x.abs().amax(-1) / 448)


def test_torch_fp8_from_pretrained_round_trip(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.low_bit_linear import TorchFp8Linear
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2)
    ref = LlamaForCausalLM(cfg).eval()
    p = str(tmp_path / "m")
    ref.save_pretrained(p)
    ids = torch.randint(0, 256, (1, 9))
    with torch.no_grad():
        want = ref(ids).logits
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="torch_fp8_e4m3", torch_dtype=torch.float32).eval()
    mods = [x for x in m.modules() if isinstance(x, TorchFp8Linear)]
    assert mods and all(x.weight.dtype == torch.uint8 for x in mods)
    with torch.no_grad():
        got = m(ids).logits
    assert ((got - want).norm() / want.norm()).item() < 0.12   # fp8 weights AND activations
    sd = str(tmp_path / "s")
    m.save_low_bit(sd)
    m2 = AutoModelForCausalLM.load_low_bit(sd, torch_dtype=torch.float32).eval()
    with torch.no_grad():
        assert torch.allclose(m2(ids).logits, got, atol=1e-5)
