"""Randomised-shape fuzz tests driven by hypothesis: format
round trips on the host, and the decode GEMV / atomic GEMV / prefill GEMM and
attention kernels on the GPU against fp32 references, over shapes the
hand-written kernels must handle (ragged tiles, split counts, batch rows)."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from ipex_llm_amd import ops
from ipex_llm_amd.ops import reference as R
from ipex_llm_amd.quantize import get_format

FORMATS = ["sym_int4", "asym_int4", "nf4", "fp4", "sym_int8", "fp8_e4m3", "fp8_e5m2", "sym_int5", "asym_int5",
           "nf3", "fp6"]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@settings(max_examples=40, deadline=None)
@given(fmt=st.sampled_from(FORMATS), n=st.integers(1, 9).map(lambda v: 16 * v), kb=st.integers(1, 6),
       seed=st.integers(0, 2 ** 16))
def test_fuzz_repack_roundtrip_and_dequant(fmt, n, kb, seed):
    f = get_format(fmt).fmt
    k = 64 * kb
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(n, k, generator=g) * 0.05
    blob = ops.quantize(w, f)
    dev = ops.repack_to_device(blob, f, n, k)
    assert torch.equal(ops.repack_from_device(dev, f, n, k), blob)
    dq = ops.dequantize(blob, f, n, k)
    assert _rel(dq, w) < 0.35


@pytest.mark.gpu
@settings(max_examples=25, deadline=None, suppress_health_check=list(HealthCheck))
@given(fmt=st.sampled_from(["sym_int4", "asym_int4", "nf4", "sym_int8", "fp8_e4m3"]), m=st.integers(1, 16),
       nt=st.integers(1, 40), kc=st.integers(1, 12), seed=st.integers(0, 2 ** 16))
def test_fuzz_gpu_gemv_and_accum(fmt, m, nt, kc, seed):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.require()
    f = get_format(fmt).fmt
    n, k = 16 * nt, 128 * kc
    g = torch.Generator(device="cuda").manual_seed(seed)
    w = torch.randn(n, k, generator=g, device="cuda") * 0.05
    blob = ops.quantize(w, f)
    x = torch.randn(m, k, generator=g, device="cuda").bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).cuda()
    y = ops.lowbit_matmul(x, blob, f, n, k)
    assert _rel(y, ref) < 1e-2
    acc = torch.zeros(m, n, device="cuda")
    ops.gemv_accum(x, blob, f, n, k, acc)
    assert _rel(acc, ref) < 5e-3


@pytest.mark.gpu
@settings(max_examples=15, deadline=None, suppress_health_check=list(HealthCheck))
@given(m=st.integers(65, 700), nt=st.integers(1, 24), kc=st.integers(1, 8), seed=st.integers(0, 2 ** 16))
def test_fuzz_gpu_prefill_gemm(m, nt, kc, seed):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.require()
    f = get_format("sym_int4").fmt
    n, k = 16 * nt, 128 * kc
    g = torch.Generator(device="cuda").manual_seed(seed)
    blob = ops.quantize(torch.randn(n, k, generator=g, device="cuda") * 0.05, f)
    x = torch.randn(m, k, generator=g, device="cuda").bfloat16()
    ref = x.float() @ ops.dequantize(blob, f, n, k, torch.float32).t()
    assert _rel(ops.lowbit_matmul(x, blob, f, n, k), ref) < 1e-2


@pytest.mark.gpu
@settings(max_examples=15, deadline=None, suppress_health_check=list(HealthCheck))
@given(B=st.integers(1, 4), Tq=st.integers(1, 150), prefix=st.integers(0, 300), hkv=st.sampled_from([1, 2, 4]),
       group=st.sampled_from([1, 2, 4]), seed=st.integers(0, 2 ** 16))
def test_fuzz_gpu_prefill_attention(B, Tq, prefix, hkv, group, seed):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ops.require()
    D, bs = 128, 64
    Hq = hkv * group
    g = torch.Generator(device="cuda").manual_seed(seed)
    L = [prefix + Tq + 3 * b for b in range(B)]
    nb = [(x + bs - 1) // bs for x in L]
    kc = torch.randn(sum(nb), hkv, bs, D, generator=g, device="cuda").bfloat16()
    vc = torch.randn(sum(nb), hkv, bs, D, generator=g, device="cuda").bfloat16()
    bt = torch.zeros(B, max(nb), dtype=torch.int32, device="cuda")
    o = 0
    for b in range(B):
        bt[b, :nb[b]] = torch.arange(o, o + nb[b], dtype=torch.int32, device="cuda").flip(0)
        o += nb[b]
    seq = torch.tensor(L, dtype=torch.int32, device="cuda")
    q = torch.randn(B * Tq, Hq, D, generator=g, device="cuda").bfloat16()
    got = ops.attn_prefill(q, kc, vc, bt, seq, Tq, D ** -0.5)
    for b in range(B):
        kk = ops.api.gather_kv(kc, bt, b, L[b]).float()
        vv = ops.api.gather_kv(vc, bt, b, L[b]).float()
        ref = R.attention(q[b * Tq:(b + 1) * Tq].float()[None], kk[None], vv[None], True, D ** -0.5)[0]
        assert _rel(got[b * Tq:(b + 1) * Tq], ref) < 2e-2
