"""fp8 linear on the MI355X (csrc/hip/fp8_gemm.hip): the f8f6f4 MFMA GEMM
(per-token e4m3 activations) against the host op's f32 emulation of the
same quantized math, and the fp8 GEMV (bf16 activations) against an fp32
PyTorch reference of the decoded weight."""
import pytest
import torch

from ipex_llm_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("e5m2", [False, True])
@pytest.mark.parametrize("M,N,K", [(17, 128, 128), (64, 256, 512), (200, 384, 1024), (1024, 1024, 4096),
                                   (300, 520, 384), (2048, 4096, 2048)])
@pytest.mark.parametrize("per_channel", [False, True])
def test_fp8_gemm_matches_emulation(e5m2, M, N, K, per_channel):
    torch.manual_seed(M + N)
    w = torch.randn(N, K) * 0.05
    x = (torch.randn(M, K) * 2).to(torch.bfloat16)
    b = torch.randn(N).to(torch.bfloat16)
    w8, ws = ops.fp8_quantize_weight(w, e5m2, per_channel)
    want = ops.fp8_linear(x.float(), w8, ws, b.float(), e5m2)          # host: f32 emulation
    xd, wd_, sd, bd = x.cuda(), w8.cuda(), ws.cuda(), b.cuda()
    got = torch.ops.ipex_llm_amd.fp8_linear(xd, wd_, sd, bd, e5m2).float().cpu()     # hand-written MFMA GEMM
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 1e-2, rel
    got2 = ops.fp8_linear(xd, wd_, sd, bd, e5m2).float().cpu()                        # dispatch (library >= 128 rows)
    rel2 = ((got2 - want).norm() / want.norm()).item()
    assert rel2 < 1e-2, rel2


def test_fp8_act_quant_matches_host():
    torch.manual_seed(3)
    x = (torch.randn(37, 1024) * 3).to(torch.bfloat16)
    qh, sh = ops.fp8_act_quant(x.float())
    qd, sd = ops.fp8_act_quant(x.cuda())
    torch.testing.assert_close(sd.cpu(), sh, rtol=1e-6, atol=0)
    # identical codes except where a value sits on a rounding tie
    assert (qd.cpu() != qh).float().mean().item() < 1e-3


@pytest.mark.parametrize("e5m2", [False, True])
@pytest.mark.parametrize("M", [1, 3, 8, 16])
def test_fp8_gemv_matches_fp32(e5m2, M):
    torch.manual_seed(M)
    N, K = 300, 2048
    w = torch.randn(N, K) * 0.05
    x = torch.randn(M, K).to(torch.bfloat16)
    w8, ws = ops.fp8_quantize_weight(w, e5m2)
    wd = w8.view(torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn).float() * ws
    want = x.float() @ wd.t()
    got = ops.fp8_linear(x.cuda(), w8.cuda(), ws.cuda(), None, e5m2).float().cpu()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 1e-2, rel


def test_torch_fp8_model_on_gpu(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2)
    ref = LlamaForCausalLM(cfg).eval()
    p = str(tmp_path / "m")
    ref.save_pretrained(p)
    ids = torch.randint(0, 512, (1, 40))
    with torch.no_grad():
        want = ref(ids).logits
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="torch_fp8_e4m3", torch_dtype=torch.bfloat16)
    m = m.to("cuda").eval()
    with torch.no_grad():
        got = m(ids.cuda()).logits.float().cpu()
        g = m.generate(ids[:, :16].cuda(), max_new_tokens=8, do_sample=False, use_graph=True)
        e = m.generate(ids[:, :16].cuda(), max_new_tokens=8, do_sample=False, use_graph=False)
    assert ((got - want).norm() / want.norm()).item() < 0.12
    assert torch.equal(g.cpu(), e.cpu())
