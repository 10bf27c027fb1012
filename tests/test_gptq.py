"""GPTQ / AWQ checkpoints load into asym_int4 exactly (reference
convert.py:301-456).  Synthetic packed checkpoints are generated here (no
auto-gptq / autoawq in the image): RTN asymmetric 4-bit, group 128, packed
in the published GPTQ (v1, zero-1) and AWQ (GEMM, interleaved order) layouts."""
import json
import os

import pytest
import torch

ORDER = [0, 2, 4, 6, 1, 3, 5, 7]


def _rtn(w, group):
    N, K = w.shape
    wg = w.view(N, K // group, group)
    lo, hi = wg.min(-1).values, wg.max(-1).values
    s = ((hi - lo) / 15).clamp(min=1e-5)
    z = torch.round(-lo / s).clamp(0, 15)
    q = torch.clamp(torch.round(wg / s[..., None]) + z[..., None], 0, 15).view(N, K).int()
    s16 = s.half()
    return q, z.int(), s16                   # [N,K], [N,G], [N,G]


def _pack_gptq(q, z, s):
    N, K = q.shape
    qw = torch.zeros(K // 8, N, dtype=torch.int32)
    for j in range(8):
        qw |= q.t()[j::8] << (4 * j)
    zz = (z - 1).t().contiguous()            # [G, N], v1 stores zero - 1
    qz = torch.zeros(zz.shape[0], N // 8, dtype=torch.int32)
    for j in range(8):
        qz |= (zz[:, j::8] & 0xF) << (4 * j)
    return qw, qz, s.t().contiguous()


def _pack_awq(q, z, s):
    N, K = q.shape
    qt = q.t().contiguous()                  # [K, N]
    qw = torch.zeros(K, N // 8, dtype=torch.int32)
    zt = z.t().contiguous()
    qz = torch.zeros(zt.shape[0], N // 8, dtype=torch.int32)
    for i, col in enumerate(ORDER):
        qw |= qt[:, col::8] << (4 * i)
        qz |= zt[:, col::8] << (4 * i)
    return qw, qz, s.t().contiguous()


@pytest.mark.parametrize("method", ["gptq", "awq"])
def test_prequantized_checkpoint_loads_exactly(tmp_path, method):
    from safetensors.torch import save_file
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=256, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2)
    ref = LlamaForCausalLM(cfg).eval()
    with torch.no_grad():
        for prm in ref.parameters():
            prm.copy_(prm.half().float())        # the checkpoint stores fp16
    sd = {}
    for name, mod in ref.named_modules():
        if isinstance(mod, torch.nn.Linear) and name != "lm_head":
            q, z, s = _rtn(mod.weight.data.float(), 128)
            g = torch.arange(q.shape[1]) // 128
            mod.weight.data = ((q.float() - z[:, g].float()) * s[:, g].float())   # dequantized reference
            qw, qz, sc = (_pack_gptq if method == "gptq" else _pack_awq)(q, z, s)
            sd[name + ".qweight"], sd[name + ".qzeros"], sd[name + ".scales"] = qw, qz, sc
            if method == "gptq":
                sd[name + ".g_idx"] = g.int()
    for k, v in ref.state_dict().items():
        mod = k.rsplit(".", 1)[0]
        if mod + ".qweight" not in sd:
            sd[k] = v.half()
    p = tmp_path / method
    os.makedirs(p)
    save_file(sd, str(p / "model.safetensors"))
    cfgd = cfg.to_dict()
    cfgd["quantization_config"] = {"quant_method": method, "bits": 4, "group_size": 128, "desc_act": False}
    (p / "config.json").write_text(json.dumps(cfgd))
    m = AutoModelForCausalLM.from_pretrained(str(p), load_in_4bit=True, torch_dtype=torch.float32,
                                             modules_to_not_convert=["lm_head"])
    assert m._illm_prequant == method
    ids = torch.randint(0, 256, (2, 10))
    with torch.no_grad():
        want = ref.float()(ids).logits
        got = m(ids).logits
    # CPU low-bit linears quantize activations to int8 per 64-block (the
    # integer-dot kernels, like ggml's q4 x q8): logits within ~1 %
    assert ((got - want).norm() / want.norm()).item() < 2.5e-2
    # the weights themselves load exactly (scales / zeros as fp16)
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    name = "model.layers.0.self_attn.o_proj"
    lin = dict(m.named_modules())[name]
    if isinstance(lin, LowBitLinear) and lin.g_idx_map is None:
        w_ref = dict(ref.named_modules())[name].weight.data.float()
        assert torch.allclose(lin.dequantize(torch.float32), w_ref, atol=2e-3, rtol=2e-3)
