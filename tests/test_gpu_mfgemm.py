"""MFMA GEMM engine (csrc/hip/gemm_mfma.hip) against plain-PyTorch fp32
references: every low-bit decode kind, dense bf16/fp16 weights, all block
shapes, split-K, bias, the GLU epilogue, and activations far outside the
f16 range (the per-row power-of-two normalisation)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from ipex_llm_amd import ops
from ipex_llm_amd.ops import reference as R
from ipex_llm_amd.quantize import get_format

LOWBIT = ["sym_int4", "asym_int4", "nf4", "fp4", "sym_int8", "fp8_e4m3", "fp8_e5m2", "asym_int5"]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("name", LOWBIT)
@pytest.mark.parametrize("tile", [0, 1, 2])
def test_mfgemm_lowbit_formats(cuda, name, tile):
    f = get_format(name).fmt
    torch.manual_seed(0)
    M, n, k = 300, 512, 768
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).to(cuda)
    y = torch.ops.ipex_llm_amd.mfgemm(x, blob, f, n, k, None, False, 0, tile, 1)
    assert y.dtype == torch.bfloat16 and y.shape == (M, n)
    assert _rel(y, ref) < 5e-3, (name, tile)


@pytest.mark.parametrize("M", [1, 17, 256, 777, 2048])
@pytest.mark.parametrize("ksplit", [1, 3])
def test_mfgemm_shapes_and_split_k(cuda, M, ksplit):
    f = get_format("sym_int4").fmt
    torch.manual_seed(1)
    n, k = 1040, 1536
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    bias = torch.randn(n, device=cuda).bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k, bias=bias).to(cuda)
    y = torch.ops.ipex_llm_amd.mfgemm(x, blob, f, n, k, bias, False, 0, -1, ksplit)
    assert _rel(y, ref) < 5e-3, (M, ksplit)


def test_mfgemm_large_activations_no_saturation(cuda):
    """bf16 activations beyond the f16 range (|x| up to 3e5) and tiny rows
    (1e-7): the row normalisation keeps both exact, no saturation at 65504"""
    f = get_format("sym_int4").fmt
    torch.manual_seed(2)
    M, n, k = 64, 256, 512
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    x = torch.randn(M, k, device=cuda)
    x[:16] *= 3e5
    x[16:32] *= 1e-7
    x = x.bfloat16()
    assert x.float().abs().max() > 65504
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).to(cuda)
    y = torch.ops.ipex_llm_amd.mfgemm(x, blob, f, n, k)
    assert torch.isfinite(y.float()).all()
    for lo, hi in ((0, 16), (16, 32), (32, 64)):
        assert _rel(y[lo:hi], ref[lo:hi]) < 5e-3, (lo, hi)


def test_x_to_f16_rowscale_exact(cuda):
    x = (torch.randn(8, 256, device=cuda) * torch.tensor([1e-6, 1e-2, 1, 30, 1e3, 6e4, 2e5, 1e30],
                                                          device=cuda)[:, None]).bfloat16()
    y, rs = torch.ops.ipex_llm_amd.x_to_f16_rowscale(x)
    back = y.float() * rs[:, None]
    assert torch.equal(back, x.float())
    assert (y.float().abs().amax(1) < 32768).all() and (y.float().abs().amax(1) >= 16384).all()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tile", [0, 1, 2])
def test_mfgemm_dense(cuda, dtype, tile):
    torch.manual_seed(3)
    M, n, k = 530, 768, 1024
    w = (torch.randn(n, k, device=cuda) * 0.05).to(dtype)
    x = torch.randn(M, k, device=cuda).to(dtype)
    ref = x.float() @ w.float().t()
    y = torch.ops.ipex_llm_amd.mfgemm(x, w, -1, n, k, None, False, 0, tile, 0)
    assert y.dtype == dtype and _rel(y, ref) < 5e-3


@pytest.mark.parametrize("name", ["sym_int4", "nf4"])
def test_mfgemm_glu_epilogue(cuda, name):
    from ipex_llm_amd.models.decoder import interleave_glu_rows
    f = get_format(name).fmt
    torch.manual_seed(4)
    I, k, M = 384, 512, 600
    wg, wu = torch.randn(I, k, device=cuda) * 0.05, torch.randn(I, k, device=cuda) * 0.05
    blob = ops.quantize(interleave_glu_rows(wg, wu), f)
    x = torch.randn(M, k, device=cuda).bfloat16()
    dense = R.dequantize_device_blob(blob.cpu(), f, 2 * I, k).to(cuda)
    gu = x.float() @ dense.t()
    g = gu.view(M, -1, 2, 16)[:, :, 0].reshape(M, I)
    u = gu.view(M, -1, 2, 16)[:, :, 1].reshape(M, I)
    for act in (0, 1):
        ref = (torch.nn.functional.silu(g) if act == 0 else torch.nn.functional.gelu(g, approximate="tanh")) * u
        y = torch.ops.ipex_llm_amd.mfgemm(x, blob, f, 2 * I, k, None, True, act)
        assert y.shape == (M, I) and _rel(y, ref) < 5e-3, (name, act)


@pytest.mark.parametrize("name", ["sym_int4", "nf4", "asym_int4", "sym_int8", "fp8_e4m3"])
@pytest.mark.parametrize("tile", [0, 1])
def test_mfgemm_nn_lowbit(cuda, name, tile):
    """grad_x = g . W over the tiled blob (transposed LDS reads) vs fp32 torch"""
    f = get_format(name).fmt
    torch.manual_seed(5)
    M, n, k = 300, 640, 768
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    g = torch.randn(M, n, device=cuda).bfloat16()
    dense = R.dequantize_device_blob(blob.cpu(), f, n, k).to(cuda)
    ref = g.float() @ dense
    y = torch.ops.ipex_llm_amd.mfgemm_nn(g, blob, f, n, k, tile, 1)
    assert y.shape == (M, k) and _rel(y, ref) < 5e-3, (name, tile)


@pytest.mark.parametrize("M,ksplit", [(64, 1), (1024, 1), (700, 3)])
def test_mfgemm_nn_shapes_tiny_gradients(cuda, M, ksplit):
    """gradients of 1e-6 (f16 would flush) and split-K"""
    f = get_format("nf4").fmt
    torch.manual_seed(6)
    n, k = 1024, 1280
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    g = (torch.randn(M, n, device=cuda) * 1e-6).bfloat16()
    dense = R.dequantize_device_blob(blob.cpu(), f, n, k).to(cuda)
    ref = g.float() @ dense
    y = torch.ops.ipex_llm_amd.mfgemm_nn(g, blob, f, n, k, -1, ksplit)
    assert _rel(y, ref) < 5e-3


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_mfgemm_nn_dense(cuda, dtype):
    torch.manual_seed(7)
    M, n, k = 520, 1152, 640
    w = (torch.randn(n, k, device=cuda) * 0.05).to(dtype)
    g = torch.randn(M, n, device=cuda).to(dtype)
    ref = g.float() @ w.float()
    y = torch.ops.ipex_llm_amd.mfgemm_nn(g, w, -1, n, k)
    assert y.dtype == dtype and _rel(y, ref) < 5e-3


def test_small_m_gemm_and_moe_gemm_large_activations(cuda):
    """the M < ENGINE_MIN_M prefill GEMM, its GLU form and the grouped MoE
    GEMM take the same row-normalised f16 activations: |x| > 65504 and tiny
    rows stay exact instead of saturating"""
    f = get_format("sym_int4").fmt
    torch.manual_seed(3)
    M, n, k = 96, 256, 512
    blob = ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)
    x = torch.randn(M, k, device=cuda)
    x[:16] *= 3e5
    x[16:32] *= 1e-7
    x = x.bfloat16()
    ref = R.lowbit_linear_ref(x, blob.cpu(), f, n, k).to(cuda)
    y = torch.ops.ipex_llm_amd.gemm(x, blob, f, n, k, None)
    assert torch.isfinite(y.float()).all()
    for lo, hi in ((0, 16), (16, 32), (32, M)):
        assert _rel(y[lo:hi], ref[lo:hi]) < 5e-3, (lo, hi)
    # grouped: 2 experts, every token routed to expert (t % 2)
    blob2 = torch.stack([blob, ops.quantize(torch.randn(n, k, device=cuda) * 0.05, f)])
    ids = (torch.arange(M, device=cuda) % 2).view(M, 1).to(torch.int32)
    off, rows = ops.moe_align(ids, 0, 2)
    out = ops.moe_gemm(x, blob2, f, n, k, off, rows, 1, False, False, False, 0, True)
    ref2 = torch.stack([R.lowbit_linear_ref(x[t:t + 1], blob2[t % 2].cpu(), f, n, k)[0] for t in range(M)]).to(cuda)
    assert torch.isfinite(out).all()
    for lo, hi in ((0, 16), (16, 32), (32, M)):
        assert _rel(out[lo:hi], ref2[lo:hi]) < 5e-3, (lo, hi)
