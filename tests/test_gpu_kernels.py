"""Numerics of the gfx950 HIP kernels against plain-PyTorch fp32 references."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from ipex_llm_amd import ops
from ipex_llm_amd.ops import reference as R
from ipex_llm_amd.quantize import get_format

FMTS = ["sym_int4", "asym_int4", "nf4", "fp4", "nf3", "sym_int8", "fp8_e4m3", "fp8_e5m2",
        "sym_int5", "asym_int5", "fp6"]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("name", FMTS)
def test_quantize_device_matches_host(cuda, name):
    f = get_format(name).fmt
    n, k = 96, 384
    w = torch.randn(n, k) * 0.05
    host = ops.repack_to_device(ops.quantize(w, f), f, n, k)
    dev = torch.ops.ipex_llm_amd.quantize_device(w.to(cuda), f, False).cpu()
    dq_h = R.dequantize_device_blob(host, f, n, k)
    dq_d = R.dequantize_device_blob(dev, f, n, k)
    # identical rounding rules on host and device; allow rare 1-code flips
    assert (dq_h != dq_d).float().mean().item() < 1e-3
    assert _rel(dq_d, w) < (0.25 if name == "nf3" else 0.15)


@pytest.mark.parametrize("name", FMTS)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [1, 5, 16, 17, 40])
@pytest.mark.parametrize("ver", [4, 2, 1])
def test_gemv_formats(cuda, name, dtype, M, ver, monkeypatch):
    if ver == 1:
        monkeypatch.setenv("ILLM_GEMV_V1", "1")
    else:
        monkeypatch.setenv("ILLM_GEMV_VER", str(ver))
    f = get_format(name).fmt
    torch.manual_seed(0)
    for n, k in [(256, 512), (80, 320)]:
        w = torch.randn(n, k, device=cuda) * 0.05
        blob = ops.quantize(w, f)
        x = torch.randn(M, k, device=cuda).to(dtype)
        ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).to(cuda)
        y = torch.ops.ipex_llm_amd.gemv(x, blob, f, n, k, None, 0, 1, 0)
        assert y.shape == (M, n) and y.dtype == dtype
        assert _rel(y, ref) < 1e-2, (name, dtype, M, n, k)
        ws = torch.ops.ipex_llm_amd.gemv(x, blob, f, n, k, None, 1, 2, 0)
        # LUT formats carry bf16/f16-rounded code values into the MFMA
        tol = 5e-3 if name in ("nf4", "nf3") or ver == 4 else 1e-3
        assert _rel(ws.sum(0), ref) < tol
        b = torch.randn(n, device=cuda).to(dtype)
        yb = torch.ops.ipex_llm_amd.gemv(x, blob, f, n, k, b, 0, 0, 0)
        assert _rel(yb, ref + b.float()) < 1e-2


@pytest.mark.parametrize("name", ["sym_int4", "asym_int4", "nf4", "fp8_e4m3", "sym_int8"])
@pytest.mark.parametrize("M", [1, 5, 8, 16])
@pytest.mark.parametrize("n", [512, 528])
def test_gemv_accum_and_zeroing_consumers(cuda, name, M, n):
    """split-K f32-atomic GEMV (v5 EPI_ATOMIC, block-transposed epilogue) vs
    the fp32 reference (n = 528: a partial last tile group); the norm consumer
    must leave the accumulator zeroed."""
    f = get_format(name).fmt
    torch.manual_seed(1)
    k = 1024
    w = torch.randn(n, k, device=cuda) * 0.05
    blob = ops.quantize(w, f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).to(cuda)
    acc = torch.zeros(M, n, device=cuda)
    for ks in (0, 1, 8):
        acc.zero_()
        ops.gemv_accum(x, blob, f, n, k, acc, ks)
        assert _rel(acc, ref) < 5e-3, (name, M, ks)
    res = torch.randn(M, n, device=cuda).bfloat16()
    wn = torch.rand(n, device=cuda).bfloat16() + 0.5
    exp, _ = R.add_rms_norm(acc.bfloat16(), res.clone(), wn, 1e-5)
    out, _ = ops.add_rms_norm(None, res, wn, 1e-5, partials=acc.unsqueeze(0), zero_partials=True)
    assert _rel(out, exp) < 1e-2
    assert acc.abs().max().item() == 0.0


@pytest.mark.parametrize("name", ["sym_int4", "asym_int4", "nf4", "sym_int8"])
@pytest.mark.parametrize("M", [1, 2, 8, 16])
def test_gemv_norm_in(cuda, name, M):
    """residual-add + RMSNorm folded into the GEMV prologue (decode norm-in
    path) vs add_rms_norm followed by the plain GEMV / GLU GEMV; the residual
    is written once to res_out and ``zero`` is cleared."""
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    f = get_format(name).fmt
    torch.manual_seed(2)
    H, n, I = 1024, 768, 256
    acc_in = torch.randn(M, H, device=cuda) * 0.5
    res = torch.randn(M, H, device=cuda).bfloat16()
    wn = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    blob = ops.quantize(torch.randn(n, H, device=cuda) * 0.05, f)
    res_ref = res.clone()
    normed, _ = ops.add_rms_norm(None, res_ref, wn, 1e-5, partials=acc_in.unsqueeze(0))
    acc_out, res_out = torch.zeros(M, n, device=cuda), torch.empty_like(res)
    zero = torch.ones(4 * 33, device=cuda)
    ops.gemv_norm_in(acc_in, res, res_out, wn, 1e-5, False, blob, f, n, H, False, acc_out=acc_out, zero=zero)
    ref = ops.gemv_partials(normed, blob, f, n, H, 1)[0]
    assert _rel(acc_out, ref) < 5e-3, (name, M)
    assert torch.equal(res_out, res_ref)                     # residual + acc, rounded like add_rms_norm
    assert zero.abs().max().item() == 0.0
    gu = ops.quantize(interleave_glu_rows(torch.randn(I, H, device=cuda) * 0.05,
                                          torch.randn(I, H, device=cuda) * 0.05), f)
    res_out2 = torch.empty_like(res)
    y = ops.gemv_norm_in(acc_in, res, res_out2, wn, 1e-5, False, gu, f, 2 * I, H, True, 0)
    assert _rel(y, ops.gemv_glu(normed, gu, f, 2 * I, H, 0)) < 1e-2, (name, M)
    assert torch.equal(res_out2, res_ref)


@pytest.mark.parametrize("name", ["sym_int4", "nf4"])
@pytest.mark.parametrize("M", [1, 4, 8])
def test_gemv_norm_in_deferred(cuda, name, M):
    """deferred RMSNorm: the GEMV stages w * h of its K slice only and reports
    the row sums of squares; the consumer-side row scale (rope_kv_fused pss,
    gemv_glu_in xss) or the GLU epilogue reproduces the normalised path"""
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    f = get_format(name).fmt
    torch.manual_seed(3)
    H, n, I = 1024, 768, 256
    acc_in = torch.randn(M, H, device=cuda) * 0.5
    res = torch.randn(M, H, device=cuda).bfloat16()
    wn = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    blob = ops.quantize(torch.randn(n, H, device=cuda) * 0.05, f)
    res_ref = res.clone()
    normed, _ = ops.add_rms_norm(None, res_ref, wn, 1e-5, partials=acc_in.unsqueeze(0))
    h = (acc_in.bfloat16() + res).float()
    acc_out, res_out = torch.zeros(M, n, device=cuda), torch.empty_like(res)
    ss = torch.zeros(M, device=cuda)
    ops.gemv_norm_in(acc_in, res, res_out, wn, 1e-5, False, blob, f, n, H, False, acc_out=acc_out, ss=ss)
    assert torch.equal(res_out, res_ref)
    assert torch.allclose(ss, h.bfloat16().float().pow(2).sum(-1), rtol=1e-4)
    inv = torch.rsqrt(ss / H + 1e-5)[:, None]
    ref = ops.gemv_partials(normed, blob, f, n, H, 1)[0]
    assert _rel(acc_out * inv, ref) < 1e-2, (name, M)
    # GLU: the epilogue applies the scale itself
    gu = ops.quantize(interleave_glu_rows(torch.randn(I, H, device=cuda) * 0.05,
                                          torch.randn(I, H, device=cuda) * 0.05), f)
    y = ops.gemv_norm_in(acc_in, res, torch.empty_like(res), wn, 1e-5, False, gu, f, 2 * I, H, True, 0,
                         ss=torch.zeros(M, device=cuda))
    assert _rel(y, ops.gemv_glu(normed, gu, f, 2 * I, H, 0)) < 1.5e-2, (name, M)
    # gate/up accumulated unscaled -> down GEMV scales before the activation
    gacc = torch.zeros(M, 2 * I, device=cuda)
    gss = torch.zeros(M, device=cuda)
    ops.gemv_norm_in(acc_in, res, torch.empty_like(res), wn, 1e-5, False, gu, f, 2 * I, H, False, acc_out=gacc,
                     ss=gss)
    dn = ops.quantize(torch.randn(H, I, device=cuda) * 0.05, f)
    d_def = ops.gemv_glu_in(gacc.unsqueeze(0), dn, f, H, I, 0, 0, torch.bfloat16, xss=gss, xss_n=H, xss_eps=1e-5)
    d_ref = ops.gemv_glu_in((gacc * torch.rsqrt(gss / H + 1e-5)[:, None]).unsqueeze(0), dn, f, H, I, 0, 0,
                            torch.bfloat16)
    assert _rel(d_def.sum(0), d_ref.sum(0)) < 1e-3


@pytest.mark.parametrize("name", ["sym_int4", "nf4"])
@pytest.mark.parametrize("M", [1, 5, 8, 16])
@pytest.mark.parametrize("unit", [False, True])
def test_gemv_accum_norm_then_glu_ss(cuda, name, M, unit):
    """o_proj GEMV whose last-arriving split-K workgroups do the residual add
    and the deferred-norm staging (gemv_accum_norm) + the gate/up GEMV that
    applies the row scale (gemv_glu_ss) vs plain fp32 torch: residual, staged
    input, sums of squares, the GLU output; the accumulator is left zeroed and
    the tickets reset (second call on the same buffers agrees)."""
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    f = get_format(name).fmt
    torch.manual_seed(11)
    K, H, I = 1024, 768, 256
    x = torch.randn(M, K, device=cuda).bfloat16()
    wo = torch.randn(H, K, device=cuda) * 0.05
    blob = ops.quantize(wo, f)
    res = torch.randn(M, H, device=cuda).bfloat16()
    wn = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    gu = ops.quantize(interleave_glu_rows(torch.randn(I, H, device=cuda) * 0.05,
                                          torch.randn(I, H, device=cuda) * 0.05), f)
    # fp32 references over the dequantized weights
    wdq = R.dequantize_device_blob(blob.cpu(), f, H, K).to(cuda).float()
    y = x.float() @ wdq.t()
    h_ref = (y.bfloat16().float() + res.float()).bfloat16().float()
    w_eff = wn.float() + 1.0 if unit else wn.float()
    inv = torch.rsqrt(h_ref.pow(2).mean(-1, keepdim=True) + 1e-5)
    xn_ref = h_ref * inv * w_eff
    gdq = R.dequantize_device_blob(gu.cpu(), f, 2 * I, H).to(cuda).float()
    from ipex_llm_amd.models.decoder import deinterleave_glu
    g, u = deinterleave_glu(xn_ref @ gdq.t())
    act_ref = torch.nn.functional.silu(g) * u
    acc = torch.zeros(M, H, device=cuda)
    ctr = torch.zeros(64, dtype=torch.int32, device=cuda)
    for it in range(2):
        res_out, xo = torch.empty_like(res), torch.empty_like(res)
        ss = torch.zeros(M, device=cuda)
        zero = torch.ones(64, device=cuda)
        ops.gemv_accum_norm(x, blob, f, H, K, acc, ctr, res, res_out, wn, unit, xo, ss, zero=zero)
        torch.cuda.synchronize()
        assert acc.abs().max().item() == 0.0 and int(ctr.abs().max()) == 0 and zero.abs().max().item() == 0.0
        assert _rel(res_out, h_ref) < 1e-2, (name, M, it)
        assert _rel(xo, (w_eff * res_out.float()).bfloat16()) < 1e-2
        assert torch.allclose(ss, res_out.float().pow(2).sum(-1), rtol=1e-4)
        out = ops.gemv_glu_ss(xo, gu, f, 2 * I, H, 0, ss, H, 1e-5)
        assert out.shape == (M, I)
        assert _rel(out, act_ref) < 2e-2, (name, M, it)


def test_decode_onorm_matches_standalone_norm(cuda, monkeypatch):
    """batch-8 decode with the o_proj norm-out epilogue vs the standalone
    residual-add + RMSNorm launch: greedy tokens agree (rare last-bit ties)"""
    from transformers import LlamaConfig
    import ipex_llm_amd.models.decoder as D
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=5)
    prompts = [list(range(1 + i, 40 + 3 * i)) for i in range(8)]
    outs = {}
    for flag in (False, True):
        monkeypatch.setattr(D, "ONORM", flag)
        outs[flag] = Engine(m).generate(prompts, max_new_tokens=8, use_graph=True)
    a, b = sum(outs[False], []), sum(outs[True], [])
    assert sum(x == y for x, y in zip(a, b)) >= 0.95 * len(a)


def test_rope_kv_fused_deferred_scale(cuda):
    """rope_kv_fused with pss == rope_kv_fused over the pre-scaled accumulator"""
    torch.manual_seed(5)
    T, Hq, Hkv, D, bs = 4, 8, 2, 128, 16
    N = (Hq + 2 * Hkv) * D
    part = torch.randn(T, N, device=cuda) * 3
    ss = torch.rand(T, device=cuda) * 4096 + 100
    bias = (torch.randn(N, device=cuda) * 0.1).bfloat16()
    inv = torch.rsqrt(ss / 1024 + 1e-5)[:, None]
    pos = torch.tensor([3, 9, 17, 30], device=cuda)
    bt = torch.arange(8, device=cuda, dtype=torch.int32).view(4, 2)
    table = torch.randn(64, D // 2, 2, device=cuda)
    outs = []
    for scaled in (False, True):
        kc = torch.zeros(8, Hkv, bs, D, device=cuda, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
        p = (part * inv if scaled else part.clone()).unsqueeze(0).contiguous()
        ops.rope_kv_fused(p, bias, q, kc, vc, pos, bt, 1, table, Hq, Hkv, D,
                          pss=None if scaled else ss, pss_n=1024, pss_eps=1e-5)
        outs.append((q, kc, vc))
    for a, b in zip(*outs):
        assert _rel(a.float(), b.float()) < 5e-3


@pytest.mark.parametrize("B,interleaved,Hq,Hkv", [(1, False, 8, 2), (2, False, 8, 2), (2, True, 8, 2),
                                                   (2, False, 8, 8), (1, False, 4, 4), (2, False, 4, 2)])
def test_attn_decode_rope_matches_rope_kv(cuda, B, interleaved, Hq, Hkv):
    """decode attention with RoPE + KV append fused in vs rope_kv_fused +
    attn_decode: identical cache contents, same attention output, and the
    qkv accumulator left all zero for the next layer (MHA included)"""
    from ipex_llm_amd.engine.runner import nsplit_for
    torch.manual_seed(3)
    D, bs = 128, 64
    L = [70, 131][:B]
    kc = torch.randn(4 * B, Hkv, bs, D, device=cuda).bfloat16()
    vc = torch.randn(4 * B, Hkv, bs, D, device=cuda).bfloat16()
    bt = torch.arange(4 * B, dtype=torch.int32, device=cuda).flip(0).view(B, 4).contiguous()
    seq_lens = torch.tensor(L, dtype=torch.int32, device=cuda)
    pos = (seq_lens - 1).long()
    W = (Hq + 2 * Hkv) * D
    part = torch.randn(B, W, device=cuda)
    bias = (torch.randn(W, device=cuda) * 0.1).bfloat16()
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    fr = torch.arange(512, device=cuda).float()[:, None] * inv[None]
    cs = torch.stack([fr.cos(), fr.sin()], -1).contiguous()
    ns = nsplit_for(max(L))
    kc1, vc1 = kc.clone(), vc.clone()
    q = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.rope_kv_fused(part.clone().unsqueeze(0), bias, q, kc1, vc1, pos, bt, 1, cs, Hq, Hkv, D, D, interleaved)
    ref = ops.attn_decode(q.view(B, 1, Hq, D), kc1, vc1, bt, seq_lens, ns, D ** -0.5)
    kc2, vc2 = kc.clone(), vc.clone()
    part2 = part.clone()
    got = ops.attn_decode_rope(part2, bias, cs, pos, kc2, vc2, bt, seq_lens, ns, D ** -0.5, 0.0, 0, Hq, D,
                               interleaved, 1.0, torch.bfloat16)
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    assert _rel(got, ref) < 1e-3
    torch.cuda.synchronize()
    assert int((part2 != 0).sum()) == 0, "qkv accumulator not re-zeroed"


@pytest.mark.parametrize("B,Hq,Hkv,D", [(1, 8, 2, 128), (4, 8, 2, 128), (8, 8, 2, 128), (2, 8, 4, 64)])
def test_gemv_rope_epilogue_and_prerot_attention(cuda, B, Hq, Hkv, D):
    """RoPE applied to each split-K partial in the qkv GEMV epilogue (rotation is
    linear) == rotating the finished accumulator; the attention over the
    pre-rotated accumulator (prerot) == the attention that rotates itself;
    the norm-in variant (deferred scale) rotates too"""
    from ipex_llm_amd.engine.runner import nsplit_for
    from ipex_llm_amd.ops.api import _rope_cols
    torch.manual_seed(11)
    f = get_format("sym_int4").fmt
    H, bs = 1024, 64
    N = (Hq + 2 * Hkv) * D
    blob = ops.quantize(torch.randn(N, H, device=cuda) * 0.05, f)
    x = torch.randn(B, H, device=cuda).bfloat16()
    L = [40 + 37 * i for i in range(B)]
    seq_lens = torch.tensor(L, dtype=torch.int32, device=cuda)
    pos = (seq_lens - 1).long()
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    fr = torch.arange(512, device=cuda).float()[:, None] * inv[None]
    cs = torch.stack([fr.cos(), fr.sin()], -1).contiguous()
    rope = (cs, pos, (Hq + Hkv) * D, D)
    a_rot = torch.zeros(B, N, device=cuda)
    a_raw = torch.zeros(B, N, device=cuda)
    ops.gemv_accum(x, blob, f, N, H, a_rot, rope=rope)
    ops.gemv_accum(x, blob, f, N, H, a_raw)
    assert _rel(a_rot, _rope_cols(a_raw, rope, torch.bfloat16)) < 1e-5
    # norm-in (deferred) variant
    acc_in = torch.randn(B, H, device=cuda) * 0.5
    res = torch.randn(B, H, device=cuda).bfloat16()
    wn = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    n_rot, n_raw = torch.zeros(B, N, device=cuda), torch.zeros(B, N, device=cuda)
    ss1, ss2 = torch.zeros(B, device=cuda), torch.zeros(B, device=cuda)
    ops.gemv_norm_in(acc_in, res, torch.empty_like(res), wn, 1e-5, False, blob, f, N, H, False, acc_out=n_rot,
                     ss=ss1, rope=rope)
    ops.gemv_norm_in(acc_in, res, torch.empty_like(res), wn, 1e-5, False, blob, f, N, H, False, acc_out=n_raw,
                     ss=ss2)
    assert _rel(n_rot, _rope_cols(n_raw, rope, torch.bfloat16)) < 1e-5
    if D != 128:
        return                                   # fused-RoPE decode attention: head_dim 128 / 256
    # attention: pre-rotated accumulator vs rotation inside the attention
    nb = (max(L) + bs - 1) // bs                # block-table row covering the longest sequence
    kc = torch.randn(nb * B, Hkv, bs, D, device=cuda).bfloat16()
    vc = torch.randn(nb * B, Hkv, bs, D, device=cuda).bfloat16()
    bt = torch.arange(nb * B, dtype=torch.int32, device=cuda).view(B, nb).contiguous()
    ns = nsplit_for(max(L))
    kc1, vc1, kc2, vc2 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    p1, p2 = a_rot * 8, a_raw * 8
    got = ops.attn_decode_rope(p1, None, cs, pos, kc1, vc1, bt, seq_lens, ns, D ** -0.5, 0.0, 0, Hq, D, False, 1.0,
                               torch.bfloat16, prerot=True)
    ref = ops.attn_decode_rope(p2, None, cs, pos, kc2, vc2, bt, seq_lens, ns, D ** -0.5, 0.0, 0, Hq, D, False, 1.0,
                               torch.bfloat16)
    assert _rel(got, ref) < 2e-2
    assert _rel(kc1.float(), kc2.float()) < 1e-2 and _rel(vc1.float(), vc2.float()) < 1e-2
    torch.cuda.synchronize()
    assert int((p1 != 0).sum()) == 0, "qkv accumulator not re-zeroed"


def test_decode_gemv_rope_matches_attention_rope(cuda):
    """whole-model decode (graph): RoPE in the qkv GEMV epilogue vs in the
    attention / rope kernels -- greedy tokens agree up to rare last-bit ties"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models import decoder as dec
    from ipex_llm_amd.models.builder import random_native_model
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=6)
    prompts = [list(range(1, 50)), list(range(7, 70)), list(range(3, 40)), [5] * 30, list(range(9, 29)),
               list(range(2, 60, 2))]
    outs = {}
    try:
        for flag in (False, True):
            dec.GEMV_ROPE = flag
            outs[flag] = Engine(m).generate(prompts, max_new_tokens=10, use_graph=True)
        eager = Engine(m).generate(prompts, max_new_tokens=10, use_graph=False)
    finally:
        dec.GEMV_ROPE = True
    assert eager == outs[True]
    a, b = sum(outs[False], []), sum(outs[True], [])
    assert sum(x == y for x, y in zip(a, b)) >= 0.95 * len(a)


def test_attn_decode_long_context_combine(cuda):
    """> 1024 splits (> 64 Ki keys): the combine takes its no-LDS path"""
    torch.manual_seed(5)
    Hq, Hkv, D, bs = 2, 1, 64, 256
    L = 70000
    nblk = (L + bs - 1) // bs
    kc = torch.randn(nblk, Hkv, bs, D, device=cuda).bfloat16()
    vc = torch.randn(nblk, Hkv, bs, D, device=cuda).bfloat16()
    bt = torch.randperm(nblk, device=cuda).to(torch.int32).view(1, nblk)
    seq_lens = torch.tensor([L], dtype=torch.int32, device=cuda)
    q = torch.randn(1, 1, Hq, D, device=cuda).bfloat16()
    ns = (L + 63) // 64
    assert ns > 1024
    got = ops.attn_decode(q, kc, vc, bt, seq_lens, ns, D ** -0.5)
    kk = ops.api.gather_kv(kc, bt, 0, L).float()          # [L, Hkv, D]
    vv = ops.api.gather_kv(vc, bt, 0, L).float()
    s = torch.einsum("hd,ld->hl", q[0, 0].float(), kk[:, 0]) * D ** -0.5
    ref = torch.softmax(s, -1) @ vv[:, 0]
    assert _rel(got[0, 0].float(), ref) < 1e-2


@pytest.mark.parametrize("D", [64, 80, 128, 256])
def test_attn_decode_wide_combine(cuda, D):
    """25..4096 splits: the 8-wave combine (split weights in LDS, partial quads
    streamed by (wave, phase)) vs an fp32 reference, uneven batch lengths"""
    torch.manual_seed(6)
    Hq, Hkv, bs = 4, 2, 64
    L = [3000, 1700]
    nblk = sum((x + bs - 1) // bs for x in L)
    kc = torch.randn(nblk, Hkv, bs, D, device=cuda).bfloat16()
    vc = torch.randn(nblk, Hkv, bs, D, device=cuda).bfloat16()
    mb = max((x + bs - 1) // bs for x in L)
    perm = torch.randperm(nblk, device=cuda).to(torch.int32)
    bt = torch.zeros(2, mb, dtype=torch.int32, device=cuda)
    o = 0
    for b, x in enumerate(L):
        n = (x + bs - 1) // bs
        bt[b, :n] = perm[o:o + n]
        o += n
    seq_lens = torch.tensor(L, dtype=torch.int32, device=cuda)
    q = torch.randn(2, 1, Hq, D, device=cuda).bfloat16()
    ns = (max(L) + 63) // 64
    assert 24 < ns <= 4096
    got = ops.attn_decode(q, kc, vc, bt, seq_lens, ns, D ** -0.5)
    for b, x in enumerate(L):
        kk = ops.api.gather_kv(kc, bt, b, x).float()
        vv = ops.api.gather_kv(vc, bt, b, x).float()
        for h in range(Hq):
            s = (kk[:, h // 2] @ q[b, 0, h].float()) * D ** -0.5
            ref = torch.softmax(s, -1) @ vv[:, h // 2]
            assert _rel(got[b, 0, h].float(), ref) < 1e-2, (b, h)


def test_decode_rope_in_mha_multilayer(cuda):
    """multi-layer MHA (Hq == Hkv) decode: fused-RoPE attention path gives the
    same tokens as the rope_kv launch path (the slab re-zeroing covers every
    k/v head)"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.decoder import NativeCausalLM
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                      num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=9)
    prompts = [list(range(1, 50))]
    outs = {}
    try:
        for flag in (False, True):
            NativeCausalLM._rope_in_env = flag
            outs[flag] = Engine(m).generate(prompts, max_new_tokens=12, use_graph=True)
    finally:
        NativeCausalLM._rope_in_env = True
    assert outs[True] == outs[False]


def test_decode_norm_in_matches_standalone_norms(cuda):
    """whole-model decode step: norm-in GEMV prologues vs standalone norms"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.decoder import NativeCausalLM
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=4)
    prompts = [list(range(1, 50)), list(range(7, 70)), list(range(3, 40)), [5] * 30]
    outs = {}
    try:
        for flag in (False, True, "rope"):
            NativeCausalLM._norm_in_env = bool(flag)
            NativeCausalLM._rope_in_env = flag == "rope"
            e = Engine(m)
            t = e.generate(prompts, max_new_tokens=8, use_graph=True)
            outs[flag] = (t, e)
    finally:
        NativeCausalLM._norm_in_env = True
        NativeCausalLM._rope_in_env = True
    assert outs[True][0] == outs["rope"][0]                   # fused RoPE: bit-identical decode
    assert m._norm_in_ok(torch.empty(1, 512, device=cuda, dtype=torch.bfloat16), 2)
    same = sum(a == b for a, b in zip(sum(outs[False][0], []), sum(outs[True][0], [])))
    assert same >= 0.95 * len(sum(outs[True][0], []))       # greedy tokens: rare last-bit ties only


@pytest.mark.parametrize("M", [1, 3, 33])
def test_gemv_glu(cuda, M):
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    I, k = 128, 256
    g = torch.randn(I, k, device=cuda) * 0.05
    u = torch.randn(I, k, device=cuda) * 0.05
    f = get_format("sym_int4").fmt
    blob = ops.quantize(interleave_glu_rows(g, u), f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    full = R.lowbit_linear_ref(x, blob.cpu(), f, 2 * I, k).to(cuda)
    gg, uu = full.view(M, I // 16, 2, 16)[:, :, 0].reshape(M, I), full.view(M, I // 16, 2, 16)[:, :, 1].reshape(M, I)
    ref = torch.nn.functional.silu(gg) * uu
    y = ops.gemv_glu(x, blob, f, 2 * I, k, 0)
    assert _rel(y, ref) < 2e-2


@pytest.mark.parametrize("name", ["sym_int4", "nf4", "fp8_e4m3"])
@pytest.mark.parametrize("M", [100, 700, 900])          # 128 n x 64 m blocks up to 768 rows, 128 x 128 above
def test_lowbit_gemm_glu_epilogue(cuda, name, M):
    """prefill GEMM with act(gate) * up in the epilogue vs GEMM + torch GLU"""
    from ipex_llm_amd.models.decoder import deinterleave_glu, interleave_glu_rows
    from ipex_llm_amd.ops.gemm import lowbit_gemm, lowbit_gemm_glu
    f = get_format(name).fmt
    torch.manual_seed(4)
    I, k = 320, 512
    blob = ops.quantize(interleave_glu_rows(torch.randn(I, k, device=cuda) * 0.05,
                                            torch.randn(I, k, device=cuda) * 0.05), f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    g, u = deinterleave_glu(lowbit_gemm(x, blob, f, 2 * I, k).float())
    for act in (0, 1):
        ref = (torch.nn.functional.silu(g) if act == 0 else torch.nn.functional.gelu(g, approximate="tanh")) * u
        y = lowbit_gemm_glu(x, blob, f, 2 * I, k, act)
        assert y.shape == (M, I) and _rel(y, ref) < 1e-2, (name, M, act)


@pytest.mark.parametrize("M", [200, 1500])             # both block shapes of the auto tile choice
def test_lowbit_gemm_prefill(cuda, M):
    f = get_format("sym_int4").fmt
    n, k = 384, 512
    w = torch.randn(n, k, device=cuda) * 0.05
    blob = ops.quantize(w, f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).to(cuda)
    y = ops.lowbit_matmul(x, blob, f, n, k)
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_add_rms_norm(cuda, dtype):
    M, H = 7, 4096
    x = torch.randn(M, H, device=cuda).to(dtype)
    res = torch.randn(M, H, device=cuda).to(dtype)
    w = (1 + 0.1 * torch.randn(H, device=cuda)).to(dtype)
    ref_n, ref_r = R.add_rms_norm(x, res, w, 1e-5)
    r2 = res.clone()
    out, _ = ops.add_rms_norm(x, r2, w, 1e-5)
    assert torch.equal(r2, ref_r)
    assert _rel(out, ref_n) < 5e-3
    # partial-slab path
    parts = torch.randn(4, M, H, device=cuda) * 0.3
    r3 = res.clone()
    out2, _ = ops.add_rms_norm(None, r3, w, 1e-5, partials=parts)
    ref2, rr2 = R.add_rms_norm(parts.sum(0).to(dtype), res, w, 1e-5)
    assert _rel(r3, rr2) < 5e-3 and _rel(out2, ref2) < 5e-3
    assert _rel(ops.rms_norm(x, w, 1e-5), R.rms_norm(x, w, 1e-5)) < 5e-3


@pytest.mark.parametrize("interleaved", [False, True])
@pytest.mark.parametrize("kv_fp8", [0, 1])
def test_rope_kv(cuda, interleaved, kv_fp8):
    T, Hq, Hkv, D, bs = 5, 8, 2, 128, 64
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=cuda).bfloat16()
    pos = torch.tensor([0, 3, 17, 100, 1000], device=cuda)
    slots = torch.tensor([0, 70, 5, 130, 200], device=cuda)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    store = torch.uint8 if kv_fp8 else torch.bfloat16
    kc = torch.zeros(4, Hkv, bs, D, device=cuda, dtype=store)
    vc = torch.zeros_like(kc)
    q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.rope_kv(qkv, q, kc, vc, slots, pos, inv, Hq, Hkv, D, interleaved=interleaved, kv_fp8=kv_fp8)
    kc2, vc2 = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    ops.rope_kv(qkv.cpu(), q2, kc2, vc2, slots.cpu(), pos.cpu(), inv.cpu(), Hq, Hkv, D, interleaved=interleaved,
                kv_fp8=kv_fp8)
    assert _rel(q.cpu(), q2) < 1e-2
    if kv_fp8:
        tab = R.code_table(6)
        assert _rel(tab[kc.cpu().long()], tab[kc2.long()]) < 5e-2
    else:
        assert _rel(kc.cpu(), kc2) < 1e-2 and torch.equal(vc.cpu(), vc2)


@pytest.mark.parametrize("D", [64, 128])
def test_rope_kv_table_fast_path(cuda, D):
    """prefill RoPE + KV append from the cos/sin table (the vectorized
    16-B-per-lane kernel) vs the CPU path; a padding slot (-1) writes nothing"""
    T, Hq, Hkv, bs = 37, 8, 2, 64
    torch.manual_seed(1)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=cuda).bfloat16()
    pos = torch.arange(T, device=cuda) * 3 + 5
    slots = torch.randperm(4 * bs, device=cuda)[:T]
    slots[7] = -1
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    fr = torch.arange(512, device=cuda).float()[:, None] * inv[None]
    tab = torch.stack([fr.cos(), fr.sin()], -1).contiguous()
    kc = torch.zeros(4, Hkv, bs, D, device=cuda, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.rope_kv(qkv, q, kc, vc, slots, pos, tab, Hq, Hkv, D)
    kc2, vc2 = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    ops.rope_kv(qkv.cpu(), q2, kc2, vc2, slots.cpu(), pos.cpu(), tab.cpu(), Hq, Hkv, D)
    assert _rel(q.cpu(), q2) < 1e-2
    assert _rel(kc.cpu(), kc2) < 1e-2 and torch.equal(vc.cpu(), vc2)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("Tq", [1, 3])
@pytest.mark.parametrize("kv_fp8", [0, 1])
def test_attn_decode(cuda, D, Tq, kv_fp8):
    torch.manual_seed(1)
    B, Hq, Hkv, bs = 3, 8, 2, 64
    lens = [5, 130, 700]
    nblk_per = 12
    perm = torch.randperm(B * nblk_per)
    bt = perm.view(B, nblk_per).int().to(cuda)
    store = torch.uint8 if kv_fp8 else torch.bfloat16
    if kv_fp8:
        kc = torch.randint(0, 120, (B * nblk_per, Hkv, bs, D), device=cuda, dtype=torch.uint8)
        vc = torch.randint(0, 120, (B * nblk_per, Hkv, bs, D), device=cuda, dtype=torch.uint8)
        kc = kc | (torch.randint(0, 2, kc.shape, device=cuda, dtype=torch.uint8) << 7)
    else:
        kc = torch.randn(B * nblk_per, Hkv, bs, D, device=cuda).bfloat16()
        vc = torch.randn(B * nblk_per, Hkv, bs, D, device=cuda).bfloat16()
    q = torch.randn(B, Tq, Hq, D, device=cuda).bfloat16()
    seq = torch.tensor(lens, device=cuda, dtype=torch.int32)
    nsplit = math.ceil(max(lens) / 64) + 2
    out = ops.attn_decode(q, kc, vc, bt, seq, nsplit, D ** -0.5, kv_fp8=kv_fp8)
    for b, L in enumerate(lens):
        kk = ops.api.gather_kv(kc, bt, b, L, kv_fp8, 1.0, torch.float32)
        vv = ops.api.gather_kv(vc, bt, b, L, kv_fp8, 1.0, torch.float32)
        ref = R.attention(q[b:b + 1].float(), kk[None], vv[None], True, D ** -0.5)
        assert _rel(out[b:b + 1], ref) < 1e-2, (b, L)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("Tq", [1, 2])
@pytest.mark.parametrize("atomic", [False, True])
def test_attn_split_then_gemv_attn(cuda, D, Tq, atomic):
    """o_proj over flash-decoding partials merged in the GEMV prologue ==
    o_proj(attn_decode(...)) (combine kernel + plain GEMV)."""
    torch.manual_seed(2)
    B, Hq, Hkv, bs = 3, 8, 2, 64
    lens = [5, 130, 700]
    nblk_per = 12
    bt = torch.randperm(B * nblk_per).view(B, nblk_per).int().to(cuda)
    kc = torch.randn(B * nblk_per, Hkv, bs, D, device=cuda).bfloat16()
    vc = torch.randn(B * nblk_per, Hkv, bs, D, device=cuda).bfloat16()
    q = torch.randn(B, Tq, Hq, D, device=cuda).bfloat16()
    seq = torch.tensor(lens, device=cuda, dtype=torch.int32)
    nsplit = math.ceil(max(lens) / 64) + 2
    f = get_format("sym_int4").fmt
    n, k = 384, Hq * D
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    o = ops.attn_decode(q, kc, vc, bt, seq, nsplit, D ** -0.5).reshape(B * Tq, k)
    ref = R.lowbit_linear_ref(o, blob.cpu(), f, n, k).to(cuda)
    po, pml = ops.attn_decode_split(q, kc, vc, bt, seq, nsplit, D ** -0.5)
    if atomic:
        acc = torch.zeros(B * Tq, n, device=cuda)
        y = ops.gemv_attn(po, pml, seq, blob, f, n, k, acc)
    else:
        y = ops.gemv_attn(po, pml, seq, blob, f, n, k).sum(0)
    assert _rel(y, ref) < 2e-3


def test_moe_topk(cuda):
    logits = torch.randn(9, 64, device=cuda)
    w, ids = ops.moe_topk(logits, 4, True, 0)
    rw, rids = R.moe_topk(logits, 4, True, 0)
    assert torch.equal(ids.cpu(), rids.cpu())
    assert torch.allclose(w, rw, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 8, 1, 1), (1, 4, 7, 300), (3, 2, 5, 4097)])
def test_attn_softmax_inplace(cuda, dtype, shape):
    """In-place row softmax kernel vs the fp32 torch softmax (masked entries included)."""
    torch.manual_seed(0)
    x = (torch.randn(*shape, device=cuda) * 4).to(dtype)
    if shape[-1] > 2:
        x[..., ::3] = float("-inf")
    ref = torch.softmax(x.float(), -1)
    y = ops.attn_softmax_(x)
    assert y.data_ptr() == x.data_ptr()
    torch.testing.assert_close(x.float(), ref, atol=4e-3, rtol=1e-2)
    z = torch.full((2, 33), float("-inf"), device=cuda, dtype=dtype)
    ops.attn_softmax_(z)
    assert (z == 0).all()


def test_attn_decode_fused_combine_repeated_uneven(cuda):
    """the last-arriving split merges the partials handed over by the other
    waves of the launch (write-through stores + atomic counter): many launches
    with uneven lengths / split counts, every output checked, the counters
    must come back to zero (graph replays reuse them)"""
    torch.manual_seed(11)
    B, Hq, Hkv, D, bs = 8, 32, 8, 128, 64
    nblk = B * 40
    kc = torch.randn(nblk, Hkv, bs, D, device=cuda).bfloat16()
    vc = torch.randn(nblk, Hkv, bs, D, device=cuda).bfloat16()
    bt = torch.randperm(nblk, device=cuda).to(torch.int32).view(B, 40)
    worst = 0.0
    for it in range(40):
        lens = torch.randint(1, 40 * bs, (B,), generator=torch.Generator().manual_seed(it))
        seq = lens.to(torch.int32).to(cuda)
        q = torch.randn(B, 1, Hq, D, device=cuda).bfloat16()
        ns = (int(lens.max()) + 63) // 64
        got = ops.attn_decode(q, kc, vc, bt, seq, ns, D ** -0.5)
        ref = ops.api.attn_decode.__wrapped__(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), seq.cpu(), ns, D ** -0.5) \
            if hasattr(ops.api.attn_decode, "__wrapped__") else None
        if ref is None:
            outs = []
            for b in range(B):
                L = int(lens[b])
                kk = ops.api.gather_kv(kc, bt, b, L).float()
                vv = ops.api.gather_kv(vc, bt, b, L).float()
                outs.append(R.attention(q[b:b + 1].float(), kk[None], vv[None], True, D ** -0.5))
            ref = torch.cat(outs, 0)
        worst = max(worst, _rel(got.float(), ref.float()))
    assert worst < 1e-2, worst


def test_attn_decode_fused_combine_opt_in_subprocess(cuda):
    """the opt-in fused combine (ILLM_ATTN_FUSED_COMBINE=1, read once per
    process) passes the repeated uneven-length check and the MHA rope-in
    slab-zeroing checks in a child process"""
    import os
    import subprocess
    import sys
    if os.environ.get("ILLM_ATTN_FUSED_COMBINE") == "1":
        pytest.skip("already the child process")
    env = dict(os.environ, ILLM_ATTN_FUSED_COMBINE="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", __file__, "-k",
                        "fused_combine_repeated or attn_decode_rope_matches or rope_in_mha"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("name", FMTS)
@pytest.mark.parametrize("n,k", [(100, 384), (48, 640), (32, 1024)])
def test_dequantize_device_kernel(cuda, name, n, k):
    """tiled blob -> dense weight on the GPU (library-GEMM prefill path; LDS
    row staging over 4 chunks) vs the host dequantizer of the same blob,
    including partial tiles and chunk groups"""
    f = get_format(name).fmt
    torch.manual_seed(2)
    w = torch.randn(n, k) * 0.05
    blob = ops.repack_to_device(ops.quantize(w, f), f, n, k)
    ref = R.dequantize_device_blob(blob, f, n, k)
    for dt in (torch.bfloat16, torch.float16):
        got = torch.ops.ipex_llm_amd.dequantize_device(blob.to(cuda), f, n, k, dt)
        assert got.shape == (n, k)
        assert torch.allclose(got.float().cpu(), ref.to(dt).float(), atol=1e-3, rtol=1e-2), (name, dt)


@pytest.mark.parametrize("name", ["sym_int4", "nf4", "sym_int8", "fp8_e4m3"])
@pytest.mark.parametrize("n,k", [(64, 384), (48, 640), (4096, 1024)])
def test_dequantize_device_transposed(cuda, name, n, k):
    """W^T [k, n] straight from the blob (the grad_x GEMM operand) == the
    row-major dequant transposed, bit for bit"""
    f = get_format(name).fmt
    torch.manual_seed(3)
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    for dt in (torch.bfloat16, torch.float16):
        w = torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, dt)
        wt = torch.ops.ipex_llm_amd.dequantize_device(blob, f, n, k, dt, True)
        assert wt.shape == (k, n) and torch.equal(wt, w.t())


def test_decode_oproj_combine_with_deferred_norm(cuda):
    """attention partials merged in the o_proj GEMV prologue (opt-in) on top of
    the deferred norm and the GEMV-epilogue RoPE: same greedy tokens as the
    combine launch up to rare last-bit ties, graph == eager"""
    from transformers import LlamaConfig
    from ipex_llm_amd.engine.runner import Engine
    from ipex_llm_amd.models.builder import random_native_model
    from ipex_llm_amd.models.decoder import NativeCausalLM
    cfg = LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=1024, num_hidden_layers=3,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
    m = random_native_model(cfg, "sym_int4", cuda, torch.bfloat16, seed=8)
    prompts = [list(range(1, 50)), list(range(7, 70))]
    outs = {}
    try:
        for flag in (False, True):
            NativeCausalLM._oproj_combine = flag
            outs[flag] = Engine(m).generate(prompts, max_new_tokens=10, use_graph=True)
        eager = Engine(m).generate(prompts, max_new_tokens=10, use_graph=False)
    finally:
        NativeCausalLM._oproj_combine = False
    assert eager == outs[True]
    a, b = sum(outs[False], []), sum(outs[True], [])
    assert sum(x == y for x, y in zip(a, b)) >= 0.95 * len(a)


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_dense_glu_matches_unfused(cuda, M, act, dt):
    """dense_glu (csrc/hip/dense_gemv.hip): act(x Wg^T) * (x Wu^T) over the
    16-row tile-interleaved gate/up weight == the unfused dense path
    (projection, de-interleave, activation, product) and an fp32 reference"""
    import torch.nn.functional as F
    from ipex_llm_amd.models.decoder import deinterleave_glu
    torch.manual_seed(M + 10 * act)
    K, I = 512, 384
    w = (torch.randn(2 * I, K, device=cuda) * 0.05).to(dt)
    x = torch.randn(M, K, device=cuda).to(dt)
    got = torch.ops.ipex_llm_amd.dense_glu(x, w, act)
    y = torch.ops.ipex_llm_amd.dense_linear(x, w, None)
    g, u = deinterleave_glu(y)
    a = F.silu(g) if act == 0 else F.gelu(g, approximate="tanh")
    want = (a * u).float()
    assert got.shape == (M, I) and got.dtype == dt
    assert ((got.float() - want).norm() / want.norm()).item() < 1e-2
    gf, uf = deinterleave_glu(x.float() @ w.float().t())
    ref = (F.silu(gf) if act == 0 else F.gelu(gf, approximate="tanh")) * uf
    assert ((got.float() - ref).norm() / ref.norm()).item() < 2e-2


@pytest.mark.parametrize("env", [{"ILLM_ATTN_V3_NW": "2"}, {"ILLM_ATTN_V3_NW": "8"},
                                 {"ILLM_ATTN_V3_NW": "4", "ILLM_ATTN_V3_FUSE": "1"},
                                 {"ILLM_ATTN_V3_FUSE": "0"}, {"ILLM_ATTN_V3": "0"}])
def test_attn_decode_v3_variants_subprocess(cuda, env):
    """v3 decode attention (attn_dec_v3.cuh) at forced split widths (2 / 4 / 8
    waves of 32 keys), with the in-kernel last-arriver merge, and v2
    (ILLM_ATTN_V3=0): the fp32-reference attention checks, the fused-RoPE
    checks (cache contents, accumulator re-zeroed) and the repeated uneven-length
    launches (counters back to zero) in a child process per setting (the
    settings are read once per process)"""
    import os
    import subprocess
    import sys
    if os.environ.get("ILLM_V3_CHILD") == "1":
        pytest.skip("already the child process")
    e = dict(os.environ, ILLM_V3_CHILD="1", **env)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "gpu", __file__, "-k",
                        "(test_attn_decode or attn_decode_rope_matches or fused_combine_repeated or rope_in_mha "
                        "or gemv_rope_epilogue) and not subprocess"],
                       env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("name", ["sym_int4", "asym_int4", "nf4", "fp8_e4m3"])
def test_gemv_argmax_epilogue(cuda, M, name):
    """lm_head GEMV with the argmax epilogue: the stored logits equal the plain
    GEMV's, and decode_advance over the per-wave partials picks exactly
    torch.argmax of those stored logits (first index on ties: forced ties too)"""
    f = get_format(name).fmt
    torch.manual_seed(7)
    n, k = 1000 + 8, 512                  # a partial last tile
    w = torch.randn(n, k, device=cuda) * 0.05
    w[5] = w[700]                           # duplicate rows -> tied logits
    blob = ops.quantize(w, f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    logits, parts = torch.ops.ipex_llm_amd.gemv_argmax(x, blob, f, n, k, None)
    ref = ops.lowbit_matmul(x, blob, f, n, k)      # (its own split-K order at M > 1)
    assert _rel(logits.float(), ref.float()) < 1e-2
    ids = torch.zeros(M, dtype=torch.long, device=cuda)
    nxt = torch.zeros_like(ids)
    pos = torch.zeros_like(ids)
    bt = torch.zeros(M, 4, dtype=torch.int32, device=cuda)
    slots = torch.zeros_like(ids)
    sl = torch.zeros(M, dtype=torch.int32, device=cuda)
    torch.ops.ipex_llm_amd.decode_advance(None, ids, nxt, pos, bt, 64, slots, sl, None, parts)
    assert torch.equal(nxt, torch.argmax(logits.float(), -1))
    # a row whose max sits in the duplicated pair: first index wins
    x2 = w[700:701].bfloat16().repeat(M, 1) * 4
    logits2, parts2 = torch.ops.ipex_llm_amd.gemv_argmax(x2, blob, f, n, k, None)
    torch.ops.ipex_llm_amd.decode_advance(None, ids, nxt, pos, bt, 64, slots, sl, None, parts2)
    assert torch.equal(nxt, torch.argmax(logits2.float(), -1))


def test_decode_argmax_epilogue_matches_logits_argmax_subprocess(cuda):
    """whole-model greedy decode (graph) with the lm_head argmax epilogue ==
    the logits-scanning decode_advance (ILLM_ARGMAX_EPI=0) token for token"""
    import os
    import subprocess
    import sys
    code = r"""
import torch
from transformers import LlamaConfig
from ipex_llm_amd.engine.runner import Engine
from ipex_llm_amd.models.builder import random_native_model
cfg = LlamaConfig(vocab_size=1000, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                  num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=1024)
m = random_native_model(cfg, "sym_int4", "cuda", torch.bfloat16, seed=3)
prompts = [list(range(1, 40)), list(range(5, 30)), [7] * 20]
print(Engine(m).generate(prompts, max_new_tokens=12, use_graph=True))
"""
    outs = []
    for flag in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, ILLM_ARGMAX_EPI=flag),
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(r.stdout.strip().splitlines()[-1])
    assert outs[0] == outs[1]


def test_embed_rms_norm_matches_gather_then_norm(cuda):
    """decode-step entry kernel: embedding gather + RMSNorm (+ zeroing the
    step's sums-of-squares buffer) == F.embedding then rms_norm, bit for bit;
    an out-of-vocabulary id is reported through the kernel error word"""
    torch.manual_seed(9)
    V, H = 1000, 4096
    table = torch.randn(V, H, device=cuda).bfloat16()
    w = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    ids = torch.tensor([3, 999, 0, 3, 512], device=cuda)
    z = torch.ones(64, device=cuda)
    res, x = torch.ops.ipex_llm_amd.embed_rms_norm(ids, table, w, 1e-5, False, z)
    ref_res = torch.nn.functional.embedding(ids, table)
    assert torch.equal(res, ref_res)
    assert torch.equal(x, ops.rms_norm(ref_res, w, 1e-5))
    assert int(z.count_nonzero()) == 0
    ops.check_kernel_errors(cuda)
    torch.ops.ipex_llm_amd.embed_rms_norm(torch.tensor([V + 5], device=cuda), table, w, 1e-5, False, None)
    with pytest.raises(RuntimeError):
        ops.check_kernel_errors(cuda)


@pytest.mark.parametrize("M", [1, 2, 5, 8])
def test_decode_gemv_forms_at_llama3_8b_shapes(cuda, M):
    """the decode GEMV instantiations (generic / XM 1 plain x / XM 2 deferred
    norm, chosen by shape) at the real Llama-3-8B projection shapes, where
    the weight ring is refilled (K >= 2048): gate/up GLU, down (K = 14336),
    qkv norm-in deferred, lm_head-style store -- vs fp32 torch"""
    from ipex_llm_amd.models.decoder import interleave_glu_rows, deinterleave_glu
    f = get_format("sym_int4").fmt
    torch.manual_seed(12)
    H, I = 4096, 14336
    deq = lambda b, n, k: R.dequantize_device_blob(b.cpu(), f, n, k).to(cuda).float()   # noqa: E731
    x = torch.randn(M, H, device=cuda).bfloat16()
    gu = ops.quantize(interleave_glu_rows(torch.randn(I, H, device=cuda) * 0.02,
                                          torch.randn(I, H, device=cuda) * 0.02), f)
    g, u = deinterleave_glu(x.float() @ deq(gu, 2 * I, H).t())
    y = ops.gemv_glu(x, gu, f, 2 * I, H, 0)
    assert _rel(y, torch.nn.functional.silu(g) * u) < 1e-2
    ssx = torch.rand(M, device=cuda) * H + 1.0                 # gemv_glu_ss: the o_proj norm-out consumer
    inv = torch.rsqrt(ssx / H + 1e-5)[:, None]
    ys = ops.gemv_glu_ss(x, gu, f, 2 * I, H, 0, ssx, H, 1e-5)
    assert _rel(ys, torch.nn.functional.silu(g * inv) * (u * inv)) < 1e-2
    a = torch.randn(M, I, device=cuda).bfloat16()
    dn = ops.quantize(torch.randn(H, I, device=cuda) * 0.02, f)
    acc = torch.zeros(M, H, device=cuda)
    ops.gemv_accum(a, dn, f, H, I, acc)
    assert _rel(acc, a.float() @ deq(dn, H, I).t()) < 5e-3
    lm = ops.quantize(torch.randn(8192, H, device=cuda) * 0.02, f)
    assert _rel(ops.lowbit_matmul(x, lm, f, 8192, H), x.float() @ deq(lm, 8192, H).t()) < 1e-2
    # qkv over the deferred norm of (residual + accumulator)
    qkv = ops.quantize(torch.randn(6144, H, device=cuda) * 0.02, f)
    acc_in = torch.randn(M, H, device=cuda)
    res = torch.randn(M, H, device=cuda).bfloat16()
    wn = (torch.rand(H, device=cuda) + 0.5).bfloat16()
    out, res_out, ss = torch.zeros(M, 6144, device=cuda), torch.empty_like(res), torch.zeros(M, device=cuda)
    ops.gemv_norm_in(acc_in, res, res_out, wn, 1e-5, False, qkv, f, 6144, H, False, acc_out=out, ss=ss)
    h = (acc_in.bfloat16().float() + res.float()).bfloat16().float()
    assert torch.equal(res_out.float(), h)
    xn = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-5) * wn.float()
    assert _rel(out * torch.rsqrt(ss / H + 1e-5)[:, None], xn @ deq(qkv, 6144, H).t()) < 1e-2
    if M <= 2:   # the batch-1 / -2 gate/up over the deferred norm (norm-in GLU)
        y2 = ops.gemv_norm_in(acc_in, res, torch.empty_like(res), wn, 1e-5, False, gu, f, 2 * I, H, True, 0,
                              ss=torch.zeros(M, device=cuda))
        g2, u2 = deinterleave_glu(xn @ deq(gu, 2 * I, H).t())
        assert _rel(y2, torch.nn.functional.silu(g2) * u2) < 1.5e-2


@pytest.mark.parametrize("glu", [False, True])
def test_prefill_gemm_measured_dispatch(cuda, glu):
    """ops/gemm.py _pick: the 8-phase kernel and the library GEMM over the same
    transient weight agree with fp32 torch whichever one a shape picks, and the
    first eager call records a choice"""
    from ipex_llm_amd.models.decoder import deinterleave_glu, interleave_glu_rows
    from ipex_llm_amd.ops import gemm as G
    f = get_format("sym_int4").fmt
    torch.manual_seed(13)
    M, n, k = 1024, 1024, 2048
    wf = (interleave_glu_rows(torch.randn(n // 2, k, device=cuda) * 0.02, torch.randn(n // 2, k, device=cuda) * 0.02)
          if glu else torch.randn(n, k, device=cuda) * 0.02)
    blob = ops.quantize(wf, f)
    W = R.dequantize_device_blob(blob.cpu(), f, n, k).to(cuda).float()
    x = torch.randn(M, k, device=cuda).bfloat16()
    y32 = x.float() @ W.t()
    if glu:
        g, u = deinterleave_glu(y32)
        y32 = torch.nn.functional.silu(g) * u
    run = (lambda: G.lowbit_gemm_glu(x, blob, f, n, k, 0)) if glu else (lambda: G.lowbit_gemm(x, blob, f, n, k))
    saved = dict(G._CHOICE)
    try:
        G._CHOICE.clear()
        y = run()
        assert (G._mbucket(M), n, k, glu, 0) in G.gemm_choices()
        assert _rel(y, y32) < 1e-2
        for c in ("g8d", "lib"):
            G._CHOICE[(G._mbucket(M), n, k, glu, 0)] = c
            assert _rel(run(), y32) < 1e-2, c
    finally:
        G._CHOICE.clear()
        G._CHOICE.update(saved)


def test_x_to_f16_rowscale_exact(cuda):
    """per-row power-of-two f16 normalisation of the fused prefill GEMM input
    (csrc/hip/gemm.hip): exact round trip, row max in [2^14, 2^15)"""
    x = (torch.randn(8, 256, device=cuda) * torch.tensor([1e-6, 1e-2, 1, 30, 1e3, 6e4, 2e5, 1e30],
                                                          device=cuda)[:, None]).bfloat16()
    y, rs = torch.ops.ipex_llm_amd.x_to_f16_rowscale(x)
    assert torch.equal(y.float() * rs[:, None], x.float())
    assert (y.float().abs().amax(1) < 32768).all() and (y.float().abs().amax(1) >= 16384).all()
