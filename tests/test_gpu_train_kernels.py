"""Training kernels against fp32 PyTorch references: fused cross-entropy
(loss + in-place logits gradient), the skinny token-axis reduction of the
LoRA gradients, the fused lm_head + CE autograd function, and the HIP flash
attention forward / backward (causal, GQA)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_ce_fused_matches_torch(cuda, dtype):
    torch.manual_seed(0)
    R, V = 37, 4096 + 64
    x = (torch.randn(R, V, device=cuda) * 3).to(dtype)
    lab = torch.randint(0, V, (R,), device=cuda)
    lab[3] = -100
    ref_loss = torch.nn.functional.cross_entropy(x.float(), lab, ignore_index=-100, reduction="none")
    xr = x.float().requires_grad_(True)
    torch.nn.functional.cross_entropy(xr, lab, ignore_index=-100, reduction="sum").backward()
    g = x.clone()
    loss = torch.ops.ipex_llm_amd.ce_fused_(g, lab, -100, 1.0)
    assert torch.allclose(loss, ref_loss, atol=2e-3, rtol=1e-3)
    assert _rel(g, xr.grad) < 1e-2
    assert torch.count_nonzero(g[3]) == 0


@pytest.mark.parametrize("R", [8, 16, 32, 64])
def test_skinny_tn(cuda, R):
    torch.manual_seed(1)
    M, N = 1000, 4096 + 128
    a = torch.randn(M, R, device=cuda)
    b = torch.randn(M, N, device=cuda).bfloat16()
    out = torch.ops.ipex_llm_amd.skinny_tn(a, b, 0.5)
    ref = 0.5 * a.t() @ b.float()
    assert _rel(out, ref) < 1e-5


def test_fused_linear_ce_matches_hf_loss(cuda):
    from ipex_llm_amd.training.fused_ce import fused_linear_cross_entropy
    torch.manual_seed(2)
    B, T, H, V = 2, 300, 256, 2048
    h = (torch.randn(B, T, H, device=cuda) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(V, H, device=cuda) * 0.05).bfloat16()
    lab = torch.randint(0, V, (B, T), device=cuda)
    lab[0, :10] = -100
    loss = fused_linear_cross_entropy(h, w, lab)
    loss.backward()
    hr = h.detach().float().requires_grad_(True)
    logits = hr[:, :-1] @ w.float().t()
    ref = torch.nn.functional.cross_entropy(logits.reshape(-1, V), lab[:, 1:].reshape(-1), ignore_index=-100)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-3 * max(1.0, ref.item())
    assert _rel(h.grad, hr.grad) < 2e-2


def test_fused_ce_patch_honours_num_items_in_batch(cuda):
    """the patched HF forward divides the summed loss by ``num_items_in_batch``
    like the HF loss does (the Trainer passes it under gradient accumulation
    and then does NOT divide by the accumulation steps): two micro-batches with
    the whole batch's item count == one unfused loss over both, gradients too"""
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.training.fused_ce import patch_fused_ce
    torch.manual_seed(4)
    cfg = LlamaConfig(vocab_size=1024, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2)
    ref = LlamaForCausalLM(cfg).to(cuda, torch.bfloat16)
    fused = LlamaForCausalLM(cfg).to(cuda, torch.bfloat16)
    fused.load_state_dict(ref.state_dict())
    for m in (ref, fused):
        m.lm_head.weight.requires_grad_(False)
        m.train()
    patch_fused_ce(fused)
    ids = torch.randint(0, 1024, (4, 64), device=cuda)
    lab = ids.clone()
    lab[0, :20] = -100
    n_items = int((lab[:, 1:] != -100).sum())
    for m in (ref, fused):
        for mb in (slice(0, 2), slice(2, 4)):
            out = m(input_ids=ids[mb], labels=lab[mb], num_items_in_batch=torch.tensor(n_items, device=cuda))
            out.loss.backward()
    assert fused.forward.__name__ == "forward" and getattr(fused, "_illm_fused_ce", False)
    gr = ref.model.layers[0].mlp.down_proj.weight.grad
    gf = fused.model.layers[0].mlp.down_proj.weight.grad
    assert _rel(gf, gr) < 3e-2
    with torch.no_grad():
        lr = ref(input_ids=ids, labels=lab).loss
    lf = fused(input_ids=ids, labels=lab, num_items_in_batch=n_items).loss
    assert abs(lf.item() - lr.item()) < 2e-2 * max(1.0, lr.item())


def _ref_attn(q, k, v, scale, causal):
    G = q.shape[1] // k.shape[1]
    kk = k.float().repeat_interleave(G, 1)
    vv = v.float().repeat_interleave(G, 1)
    s = (q.float() @ kk.transpose(-1, -2)) * scale
    if causal:
        T = q.shape[2]
        s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=q.device), 1), float("-inf"))
    return (torch.softmax(s, -1) @ vv).transpose(1, 2)          # [B, T, H, D]


@pytest.mark.parametrize("B,Hq,Hkv,T,D", [(2, 8, 2, 256, 128), (1, 4, 4, 128, 64), (2, 4, 1, 192, 128)])
@pytest.mark.parametrize("causal", [True, False])
def test_train_flash_attention_fwd_bwd(cuda, B, Hq, Hkv, T, D, causal):
    from ipex_llm_amd.training.flash_attn import flash_attention
    torch.manual_seed(3)
    # HF layout: [B, T, H, D] projections viewed as [B, H, T, D]
    q = torch.randn(B, T, Hq, D, device=cuda).bfloat16().transpose(1, 2).requires_grad_(True)
    k = torch.randn(B, T, Hkv, D, device=cuda).bfloat16().transpose(1, 2).requires_grad_(True)
    v = torch.randn(B, T, Hkv, D, device=cuda).bfloat16().transpose(1, 2).requires_grad_(True)
    scale = 1 / math.sqrt(D)
    out = flash_attention(q, k, v, scale, causal)
    dout = torch.randn_like(out)
    out.backward(dout)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attn(qr, kr, vr, scale, causal)
    ref.backward(dout.float())
    assert _rel(out, ref) < 1e-2
    assert _rel(q.grad, qr.grad) < 2e-2
    assert _rel(k.grad, kr.grad) < 2e-2
    assert _rel(v.grad, vr.grad) < 2e-2


@pytest.mark.parametrize("M,N,r", [(4096, 4096, 8), (300, 1000, 16), (77, 14336, 24), (64, 4104, 64), (1, 8, 8),
                                   (33, 200, 8)])
def test_lora_update_matches_fp32(cuda, M, N, r):
    """C += alpha * A B^T on the rank-update kernel (csrc/hip/lora_update.hip)
    == fp32 torch, incl. a strided column slice as A (the grouped LoRA's xa)"""
    torch.manual_seed(M + r)
    C = torch.randn(M, N, device=cuda).bfloat16()
    wide = torch.randn(M, r + 16, device=cuda).bfloat16()
    A = wide[:, 8:8 + r]                                 # stride r + 16, 16-B aligned start
    B = (torch.randn(N, r, device=cuda) * 0.1).bfloat16()
    ref = C.float() + 0.7 * (A.float() @ B.float().t())
    out = torch.ops.ipex_llm_amd.lora_update_(C.clone(), A, B, 0.7)
    assert ((out.float() - ref).norm() / ref.norm()).item() < 5e-3
    assert (out.float() - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("M,N,r", [(4096, 4096, 24), (300, 1000, 16), (77, 14336, 8), (4100, 4104, 64),
                                   (1, 8, 8), (8192, 1024, 40)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_lora_tn_matches_fp32(cuda, M, N, r, dt):
    """out = alpha a^T b over the token axis on the MFMA reduction
    (csrc/hip/lora_update.hip lora_tn) == fp32 torch, incl. a strided column
    slice as a (the grouped LoRA's xa_all[:, off:off + r])"""
    torch.manual_seed(M + r)
    wide = torch.randn(M, r + 16, device=cuda).to(dt)
    a = wide[:, 8:8 + r]
    b = torch.randn(M, N, device=cuda).to(dt)
    ref = 0.7 * (a.float().t() @ b.float())
    out = torch.ops.ipex_llm_amd.lora_tn(a, b, 0.7)
    assert out.dtype == torch.float32 and out.shape == (r, N)
    assert ((out - ref).norm() / ref.norm()).item() < 1e-4


def test_lora_tn_acc_slab_transposed(cuda):
    """several LoRA gradients accumulated into one zeroed f32 slab, B
    gradients written transposed ([N, r]) by the kernel (training/lora.py _tn_many)"""
    from ipex_llm_amd.training.lora import _tn_many
    torch.manual_seed(5)
    M = 1000
    x = torch.randn(M, 512, device=cuda).bfloat16()
    wide = torch.randn(M, 40, device=cuda).bfloat16()
    xa = wide[:, 8:32]                                   # 24 = q/k/v r=8 slices, strided
    gs = [torch.randn(M, n, device=cuda).bfloat16() for n in (512, 128, 128)]
    gxa = torch.randn(M, 24, device=cuda).bfloat16()
    jobs = [(xa[:, 8 * i:8 * i + 8], g, 0.5, True) for i, g in enumerate(gs)] + [(gxa, x, 1.0, False)]
    outs = _tn_many(jobs, torch.bfloat16)
    for (a, b, al, tr), o in zip(jobs, outs):
        ref = al * (a.float().t() @ b.float())
        ref = ref.t() if tr else ref
        assert o.shape == ref.shape and o.dtype == torch.bfloat16 and o.is_contiguous()
        assert ((o.float() - ref).norm() / ref.norm()).item() < 1e-2
