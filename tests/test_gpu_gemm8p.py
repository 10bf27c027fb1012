"""8-phase 256x256 dense bf16 GEMM (csrc/hip/gemm_8p.hip) vs an fp32 torch
reference: ragged M / N, K multiples of 64, strided x, bias, f32 output."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1, 8, 64), (300, 520, 192), (1024, 4096, 4096),
                                   (4096, 1000, 1024), (2048, 6144, 4096)])
def test_gemm_bf16_matches_fp32(cuda, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    ref = x.float() @ w.float().t()
    y = torch.ops.ipex_llm_amd.gemm_bf16(x, w)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    assert _rel(y, ref) < 8e-3, (M, N, K)


def test_gemm_bf16_bias_f32_out_strided(cuda):
    torch.manual_seed(5)
    M, N, K = 640, 768, 512
    xb = torch.randn(M, K + 64, device=cuda).bfloat16()
    x = xb[:, 32:32 + K]                               # row stride K + 64
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    ref = x.float() @ w.float().t() + b.float()
    y = torch.ops.ipex_llm_amd.gemm_bf16(x, w, b, True)
    assert y.dtype == torch.float32
    assert _rel(y, ref) < 2e-3
    # repeated calls are deterministic (no race in the LDS-DMA pipeline)
    y2 = torch.ops.ipex_llm_amd.gemm_bf16(x, w, b, True)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("qtype", ["sym_int4", "nf4"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (100, 520, 384), (1024, 4096, 4096), (3000, 1040, 1024)])
def test_gemm8p_lowbit_matches_dequant_fp32(cuda, qtype, M, N, K):
    """weights decoded to bf16 inside the GEMM == dequantize + fp32 matmul"""
    from ipex_llm_amd import ops
    from ipex_llm_amd.ops import reference as R
    from ipex_llm_amd.quantize import get_format
    f = get_format(qtype).fmt
    torch.manual_seed(M + K)
    blob = ops.quantize(torch.randn(N, K, device=cuda) * 0.05, f)
    x = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, N, K, bias=b).to(cuda)
    y = torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, N, K, b)
    assert y.shape == (M, N) and torch.isfinite(y.float()).all()
    assert _rel(y, ref) < 6e-3, (qtype, M, N, K)
    # bit-identical to dequantize-to-bf16 + the dense kernel (same bf16 weights, same order)
    wd = torch.ops.ipex_llm_amd.dequantize_device(blob, f, N, K, torch.bfloat16)
    assert torch.equal(y, torch.ops.ipex_llm_amd.gemm_bf16(x, wd, b, False, 0, False, 0, 1))   # (no split-K)


@pytest.mark.parametrize("qtype", ["sym_int4", "nf4"])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm8p_lowbit_glu_epilogue(cuda, qtype, act):
    """gate/up tile-interleaved weight: act(gate) * up in the epilogue"""
    import torch.nn.functional as F
    from ipex_llm_amd import ops
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    from ipex_llm_amd.quantize import get_format
    f = get_format(qtype).fmt
    torch.manual_seed(act)
    M, I, K = 700, 768, 1024
    wg, wu = torch.randn(I, K, device=cuda) * 0.05, torch.randn(I, K, device=cuda) * 0.05
    blob = ops.quantize(interleave_glu_rows(wg, wu), f)
    x = torch.randn(M, K, device=cuda).bfloat16()
    h = torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, 2 * I, K, None, True).float()   # f32, interleaved
    hg = h.view(M, I // 16, 2, 16)
    g_, u_ = hg[:, :, 0].reshape(M, I), hg[:, :, 1].reshape(M, I)
    ref = (F.silu(g_) if act == 0 else F.gelu(g_, approximate="tanh")) * u_
    y = torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, 2 * I, K, None, False, True, act)
    assert y.shape == (M, I)
    assert _rel(y, ref) < 8e-3


_SCHED_CHILD = r"""
import torch
from ipex_llm_amd import ops
from ipex_llm_amd.quantize import get_format
dev = torch.device("cuda")
for qt in ("sym_int4", "nf4"):
    f = get_format(qt).fmt
    for (M, N, K) in ((256, 256, 128), (300, 520, 384), (1024, 4096, 4096), (3000, 1040, 1024)):
        torch.manual_seed(M + K)
        blob = ops.quantize(torch.randn(N, K, device=dev) * 0.05, f)
        x = torch.randn(M, K, device=dev).bfloat16()
        wd = torch.ops.ipex_llm_amd.dequantize_device(blob, f, N, K, torch.bfloat16)
        y = torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, N, K, None)
        assert torch.equal(y, torch.ops.ipex_llm_amd.gemm_bf16(x, wd, None, False, 0, False, 0, 1)), (qt, M, N, K)
        assert torch.equal(y, torch.ops.ipex_llm_amd.gemm8p_lowbit(x, blob, f, N, K, None))
print("OK")
"""


@pytest.mark.parametrize("var,val", [("ILLM_G8_SCHED", "0"), ("ILLM_G8_SCHED", "1")])
def test_gemm8p_lowbit_decode_schedules_bit_identical(cuda, var, val):
    """both decode schedules of the low-bit kernel (ILLM_G8_SCHED: decode after
    / interleaved into the MFMA clusters, read once per process) == dequantize
    + the dense kernel, bit for bit"""
    import os
    import subprocess
    import sys
    env = dict(os.environ, **{var: val})
    r = subprocess.run([sys.executable, "-c", _SCHED_CHILD], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("M,N,K,S", [(1024, 4096, 4096, -1), (1024, 6144, 4096, 2), (300, 520, 1024, 3),
                                     (700, 4096, 14336, 4), (64, 256, 512, 8)])
def test_gemm_bf16_split_k_matches_fp32(cuda, M, N, K, S):
    """split-K (f32 partials into a zeroed workspace + the finishing launch):
    auto and forced factors, ragged shapes, bias"""
    torch.manual_seed(M + S)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    ref = x.float() @ w.float().t() + b.float()
    y = torch.ops.ipex_llm_amd.gemm_bf16(x, w, b, False, 0, False, 0, S)
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 8e-3, (M, N, K, S)
    y1 = torch.ops.ipex_llm_amd.gemm_bf16(x, w, b, False, 0, False, 0, 1)
    assert _rel(y, y1) < 8e-3


@pytest.mark.parametrize("S", [1, 4])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_bf16_glu_epilogue(cuda, S, act):
    """dense 8-phase GLU: 16-row gate/up tile pairs, act(gate) * up in the
    epilogue (S = 1) or in the split-K finishing launch (S = 4)"""
    import torch.nn.functional as F
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    torch.manual_seed(3 + act)
    M, I, K = 1024, 1024, 2048
    wg, wu = torch.randn(I, K, device=cuda) * 0.05, torch.randn(I, K, device=cuda) * 0.05
    w = interleave_glu_rows(wg, wu).bfloat16()
    x = torch.randn(M, K, device=cuda).bfloat16()
    hg = (x.float() @ w.float().t()).view(M, I // 16, 2, 16)
    g_, u_ = hg[:, :, 0].reshape(M, I), hg[:, :, 1].reshape(M, I)
    ref = (F.silu(g_) if act == 0 else F.gelu(g_, approximate="tanh")) * u_
    y = torch.ops.ipex_llm_amd.gemm_bf16(x, w, None, False, 0, True, act, S)
    assert y.shape == (M, I)
    assert _rel(y, ref) < 8e-3


@pytest.mark.parametrize("S", [1, 3])
def test_gemm_bf16_out_slice_and_accumulate(cuda, S):
    """out= a row slice of a larger buffer (strided rows), accumulate=True:
    out += x w^T with one rounding, plain and split-K"""
    torch.manual_seed(9 + S)
    M, N, K = 700, 1024, 2048
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    big = torch.randn(M + 50, N + 64, device=cuda).bfloat16()
    view = big[10:10 + M, 32:32 + N]
    big0 = big.clone()
    old = view.float().clone()
    y = torch.ops.ipex_llm_amd.gemm_bf16(x, w, None, False, 0, False, 0, S, view, True)
    assert y.data_ptr() == view.data_ptr()
    ref = old + x.float() @ w.float().t()
    assert _rel(view, ref) < 8e-3
    assert torch.equal(big[:10], big0[:10]) and torch.equal(big[10 + M:], big0[10 + M:])
    assert torch.equal(big[:, :32], big0[:, :32]) and torch.equal(big[:, 32 + N:], big0[:, 32 + N:])
    z = torch.empty(M, N, device=cuda).bfloat16()
    torch.ops.ipex_llm_amd.gemm_bf16(x, w, None, False, 0, False, 0, S, z)
    assert _rel(z, x.float() @ w.float().t()) < 8e-3
