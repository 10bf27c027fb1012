"""Low-bit formats: C++ host quantizers vs the torch references, layout
round trips and error bounds (CPU)."""
import pytest
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.ops import reference as R
from ipex_llm_amd.quantize import get_format, resolve_qtype, qtypes as Q

FMTS = ["sym_int4", "woq_int4", "asym_int4", "nf4", "fp4", "nf3", "sym_int8", "fp8_e4m3", "fp8_e5m2",
        "sym_int5", "asym_int5", "fp6"]
ERR = {"nf3": 0.25, "sym_int8": 0.01, "fp8_e4m3": 0.04, "fp8_e5m2": 0.07, "sym_int5": 0.07, "asym_int5": 0.07,
       "fp6": 0.07}


@pytest.mark.parametrize("name", FMTS)
def test_roundtrip_and_layouts(name):
    torch.manual_seed(0)
    f = get_format(name).fmt
    n, k = 40, 320          # exercises row (16) and K (128) padding of the tiled layout
    w = torch.randn(n, k)
    blob = ops.quantize(w, f)
    dq = ops.dequantize(blob, f, n, k)
    assert torch.equal(dq, R.dequantize_canonical(blob, f, n, k))
    dev = ops.repack_to_device(blob, f, n, k)
    assert torch.equal(dq, R.dequantize_device_blob(dev, f, n, k))
    assert torch.equal(ops.repack_from_device(dev, f, n, k), blob)
    err = ((dq - w).norm() / w.norm()).item()
    assert err < ERR.get(name, 0.16), err


def test_qtype_registry_matches_reference_ids():
    assert resolve_qtype("sym_int4") == 2 and resolve_qtype("asym_int4") == 3
    assert resolve_qtype("nf4") == 10 and resolve_qtype("fp8") == 19 and resolve_qtype("woq_int4") == 34
    assert resolve_qtype("gguf_q4k_m") == 102
    # k-quants are native GGUF super-block formats now (test_kquant.py)
    assert get_format("q4_k").name == "q4_k" and get_format("q4_k").kquant
    assert get_format("gguf_q4k_m").name == "q4_k"


def test_sym_int4_q4_0_convention():
    # the max-|x| element of a block maps to code 0 (= -8 d), ggml q4_0 style
    w = torch.zeros(1, 64)
    w[0, 5] = -3.0
    w[0, 7] = 1.0
    f = get_format("sym_int4").fmt
    dq = ops.dequantize(ops.quantize(w, f), f, 1, 64)
    assert abs(dq[0, 5].item() + 3.0) < 1e-3


def test_fp8_matches_torch_rne():
    x = torch.randn(4096) * 10
    for e5m2, dt in ((False, torch.float8_e4m3fn), (True, torch.float8_e5m2)):
        ours = ops.to_fp8_bytes(x, e5m2)
        ref = x.to(dt).view(torch.uint8)
        assert torch.equal(ours, ref)


def test_imatrix_and_scale_search_reduce_error():
    torch.manual_seed(1)
    w = torch.randn(64, 256)
    f = get_format("sym_int4").fmt
    base = (ops.dequantize(ops.quantize(w, f), f, 64, 256) - w).pow(2).mean()
    srch = (ops.dequantize(ops.quantize(w, f, scale_search=True), f, 64, 256) - w).pow(2).mean()
    assert srch <= base
    imat = torch.rand(256) + 0.1
    q = ops.quantize(w, f, imatrix=imat)
    assert q.numel() == ops.quantize(w, f).numel()


def test_cpu_lowbit_gemm_matches_reference():
    torch.manual_seed(2)
    for name in ("sym_int4", "asym_int4", "nf4", "sym_int8", "fp8_e4m3"):
        f = get_format(name).fmt
        w = torch.randn(96, 256) * 0.05
        blob = ops.quantize(w, f)
        x = torch.randn(5, 256)
        ref = x @ R.dequantize_canonical(blob, f, 96, 256).t()
        y = ops.lowbit_matmul(x, blob, f, 96, 256)
        if name in ("sym_int4", "asym_int4", "sym_int8"):
            # int8-activation integer-dot path (per-64-block activation scales;
            # ggml's q4_0 / q8_0 x q8_0 dots do the same)
            assert ((y - ref).norm() / ref.norm()).item() < 1.5e-2
        else:
            assert torch.allclose(y, ref, rtol=1e-4, atol=1e-4)


def test_imatrix_file_roundtrip_and_weighted_quantization(tmp_path):
    import torch
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import qtypes as Q
    from ipex_llm_amd.quantize.imatrix import load_imatrix, read_imatrix, write_imatrix
    torch.manual_seed(0)
    K = 256
    imp = torch.rand(K) ** 4 * 100 + 1e-3
    p = str(tmp_path / "imatrix.dat")
    write_imatrix(p, {"blk.0.attn_q.weight": imp, "blk.0.ffn_down.weight": imp}, ncall=10)
    raw = read_imatrix(p)
    assert torch.allclose(raw["blk.0.attn_q.weight"], imp, rtol=1e-5)
    hf = load_imatrix(p)
    assert "model.layers.0.self_attn.q_proj" in hf and "model.layers.0.self_attn.qkv_proj" in hf
    # importance-weighted quantization lowers the weighted error
    fmt = Q.get_format("sym_int4").fmt
    w = torch.randn(64, K)
    err = lambda blob: (((ops.dequantize(blob, fmt, 64, K) - w) ** 2) * imp).sum().item()  # noqa: E731
    assert err(ops.quantize(w, fmt, imp, True)) < err(ops.quantize(w, fmt, None, False))


def test_attn_softmax_cpu_fallback():
    """CPU path of ops.attn_softmax_ is the in-place fp32 softmax."""
    import torch
    from ipex_llm_amd import ops
    x = torch.randn(2, 3, 17).to(torch.bfloat16)
    ref = torch.softmax(x.float(), -1).to(torch.bfloat16)
    y = ops.attn_softmax_(x)
    assert y is x and torch.equal(x, ref)


def test_attn_softmax_fully_masked_row_is_zero():
    """a fully masked row is zeros on the fallback, as on the HIP kernel"""
    import torch
    from ipex_llm_amd import ops
    x = torch.randn(3, 9).to(torch.bfloat16)
    x[1] = float("-inf")
    ops.attn_softmax_(x)
    assert torch.equal(x[1], torch.zeros(9, dtype=torch.bfloat16))
    assert torch.isfinite(x.float()).all()


@pytest.mark.parametrize("mt", ["granite", "olmo"])   # (families still on the HF forward)
def test_hf_eager_attention_uses_illm_softmax(mt, tmp_path, monkeypatch):
    """an eager-configured HF-forward family is routed through illm_eager
    (ops.attn_softmax_) and keeps the dense model's logits"""
    import torch
    from transformers import AutoConfig, AutoModelForCausalLM as HFAuto
    from ipex_llm_amd import ops
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    cfg = AutoConfig.for_model(mt, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                               num_attention_heads=4, vocab_size=256, max_position_embeddings=128)
    cfg._attn_implementation = "eager"
    torch.manual_seed(0)
    ref = HFAuto.from_config(cfg, attn_implementation="eager").eval()
    p = str(tmp_path / mt)
    ref.save_pretrained(p)
    ids = torch.randint(3, 256, (2, 12), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = ref(ids).logits.float()
    calls = []
    orig = ops.attn_softmax_

    def spy(x):
        calls.append(x.shape)
        return orig(x)
    import ipex_llm_amd.transformers.attention as A
    monkeypatch.setattr(A.ops, "attn_softmax_", spy)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="bf16", torch_dtype=torch.float32,
                                             attn_implementation="eager")
    assert m.config._attn_implementation == "illm_eager"
    with torch.no_grad():
        got = m(ids).logits.float()
    assert calls, "illm_eager attention not used"
    assert ((got - want).norm() / want.norm()).item() < 2e-2


def test_attn_prefill_cpu_fallback_matches_reference():
    """ops.attn_prefill on CPU tensors = per-sequence fp32 reference over the paged cache"""
    import torch
    from ipex_llm_amd import ops
    from ipex_llm_amd.ops import reference as R
    torch.manual_seed(0)
    B, Tq, Hq, Hkv, D, bs = 2, 5, 4, 2, 64, 64
    kc = torch.randn(4, Hkv, bs, D)
    vc = torch.randn(4, Hkv, bs, D)
    bt = torch.tensor([[2, 0], [1, 3]], dtype=torch.int32)
    L = [70, 9]
    seq = torch.tensor(L, dtype=torch.int32)
    q = torch.randn(B * Tq, Hq, D)
    got = ops.attn_prefill(q, kc, vc, bt, seq, Tq, 0.125)
    for b in range(B):
        kk = ops.api.gather_kv(kc, bt, b, L[b], 0, 1.0, torch.float32)
        vv = ops.api.gather_kv(vc, bt, b, L[b], 0, 1.0, torch.float32)
        ref = R.attention(q[b * Tq:(b + 1) * Tq][None], kk[None], vv[None], True, 0.125)[0]
        assert torch.allclose(got[b * Tq:(b + 1) * Tq], ref, atol=1e-5)


@pytest.mark.parametrize("qtype", ["sym_int4", "asym_int4"])
@pytest.mark.parametrize("M", [1, 3, 9, 200])
@pytest.mark.parametrize("isa", ["0", "1"])
def test_cpu_int4_dot_gemm_matches_dequant(qtype, M, isa, monkeypatch):
    """CPU int8-activation integer-dot kernels (AVX-512 VNNI / AVX2) and the
    dequant + BLAS path for M above the threshold vs x @ dequant(W)^T"""
    import subprocess
    import sys
    code = f"""
import torch
from ipex_llm_amd import ops
from ipex_llm_amd.quantize import get_format
f = get_format({qtype!r}).fmt
torch.manual_seed(0)
n, k = 96, 320
w = torch.randn(n, k) * 0.05
blob = ops.quantize(w, f)
x = torch.randn({M}, k)
y = ops.lowbit_matmul(x, blob, f, n, k)
ref = x @ ops.dequantize(blob, f, n, k).T
rel = ((y - ref).norm() / ref.norm()).item()
assert rel < 1.5e-2, rel
print("ok", rel)
"""
    env = dict(__import__("os").environ, ILLM_CPU_ISA=isa)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_mixed_fp4_picks_per_tensor_and_round_trips(tmp_path):
    """mixed_fp4: lower-MSE of sym_int4 / fp4 chosen per tensor (reference
    FP4Params.quantize), and the per-module plan survives save/load"""
    from transformers import LlamaConfig, LlamaForCausalLM
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.transformers.low_bit_linear import LowBitLinear
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2)
    ref = LlamaForCausalLM(cfg).eval()
    with torch.no_grad():       # heavy-tailed weights in layer 1 (fp4's log grid wins there)
        for n, p_ in ref.named_parameters():
            if "layers.1." in n and p_.dim() == 2:
                p_.copy_(torch.distributions.StudentT(1.5).sample(p_.shape).clamp(-50, 50) * 0.01)
    p = str(tmp_path / "m")
    ref.save_pretrained(p)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="mixed_fp4", torch_dtype=torch.float32).eval()
    kinds = {mod.qtype for mod in m.modules() if isinstance(mod, LowBitLinear)}
    assert kinds == {Q.SYM_INT4, Q.FP4}, kinds
    ids = torch.randint(0, 256, (1, 8))
    with torch.no_grad():
        a = m(ids).logits
    sd = str(tmp_path / "s")
    m.save_low_bit(sd)
    m2 = AutoModelForCausalLM.load_low_bit(sd, torch_dtype=torch.float32).eval()
    k2 = {n: mod.qtype for n, mod in m2.named_modules() if isinstance(mod, LowBitLinear)}
    k1 = {n: mod.qtype for n, mod in m.named_modules() if isinstance(mod, LowBitLinear)}
    assert k1 == k2
    with torch.no_grad():
        assert torch.allclose(m2(ids).logits, a, atol=1e-5)


_ISAS = [1, 2, -1]


@pytest.mark.parametrize("qtype", ["sym_int8", "sym_int5", "asym_int5", "nf4", "fp4", "nf3", "fp8_e4m3",
                                   "fp8_e5m2", "fp6"])
@pytest.mark.parametrize("M", [1, 5, 17])
@pytest.mark.parametrize("isa", _ISAS)
def test_cpu_lowbit_gemm_paths_match_dequant(qtype, M, isa):
    """every CPU GEMM path (AVX-512 / VNNI, AVX2, portable) of the 8-bit
    integer formats (int8-activation integer dot) and the LUT / minifloat
    formats (in-register code expansion, exact f32 activations) == x @
    dequant(W)^T; the minifloat decode is checked on every byte value"""
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import get_format
    if isa == 2 and torch.backends.cpu.get_cpu_capability() != "AVX512":
        pytest.skip("no AVX-512 on this host")
    f = get_format(qtype).fmt
    torch.manual_seed(M)
    n, k = 40, 384
    w = torch.randn(n, k) * 0.05
    w[0, :64] = torch.linspace(-0.4, 0.4, 64)             # wide block: exercises large codes
    blob = ops.quantize(w, f)
    x = torch.randn(M, k)
    y = torch.ops.ipex_llm_amd.linear_cpu_isa(x, blob, f, n, k, isa)
    ref = x @ ops.dequantize(blob, f, n, k).T
    rel = ((y - ref).norm() / ref.norm()).item()
    integer = qtype in ("sym_int8", "sym_int5", "asym_int5") and isa >= 0
    assert rel < (1e-2 if integer else 1e-5), (qtype, isa, rel)


@pytest.mark.parametrize("qtype", ["fp8_e4m3", "fp8_e5m2"])
@pytest.mark.parametrize("isa", _ISAS)
def test_cpu_minifloat_decode_every_code(qtype, isa):
    """a weight row holding all 256 codes (scale 1) dotted with one-hot rows
    recovers each code's value exactly (normals, subnormals, signs)"""
    from ipex_llm_amd import ops
    from ipex_llm_amd.quantize import get_format
    if isa == 2 and torch.backends.cpu.get_cpu_capability() != "AVX512":
        pytest.skip("no AVX-512 on this host")
    f = get_format(qtype).fmt
    codes = torch.arange(256, dtype=torch.uint8)
    vals = torch.tensor([float(v) for v in codes.view(torch.float8_e4m3fn if qtype == "fp8_e4m3"
                                                     else torch.float8_e5m2).float()])
    codes[~torch.isfinite(vals)] = 0                      # NaN / inf codes never hold weights
    vals[~torch.isfinite(vals)] = 0.0
    scales = torch.ones(256 // 64, dtype=torch.float16)    # canonical blob: codes | f16 block scales
    blob = torch.cat([codes, scales.view(torch.uint8)])
    assert torch.equal(ops.dequantize(blob, f, 1, 256)[0], vals)
    y = torch.ops.ipex_llm_amd.linear_cpu_isa(torch.eye(256), blob, f, 1, 256, isa)[:, 0]
    assert torch.equal(y, vals)
