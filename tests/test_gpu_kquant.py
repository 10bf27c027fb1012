"""GPU k-quant kernels (csrc/hip/kquant.hip): the device dequantizer must be
bit-equal (after bf16 rounding) to the C++ host decoder, and the decode GEMV
read straight from the GGUF blocks must match an fp32 PyTorch GEMM over the
dequantized weight for M = 1 / 4 / 8 (and the dequant + GEMM prefill path)."""
import pytest
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.quantize import qtypes as Q

pytestmark = pytest.mark.gpu

FMTS = {"q4_k": Q.FMT_Q4K, "q5_k": Q.FMT_Q5K, "q6_k": Q.FMT_Q6K, "q2_k": Q.FMT_Q2K,
        # IQ lattice formats (csrc/common/iquant.h, codebooks in constant memory)
        "gguf_iq2_xxs": Q.FMT_IQ2XXS, "gguf_iq2_xs": Q.FMT_IQ2XS, "gguf_iq1_s": Q.FMT_IQ1S,
        "gguf_iq1_m": Q.FMT_IQ1M}


@pytest.mark.parametrize("name", list(FMTS))
def test_dequant_matches_host(name):
    fmt = FMTS[name]
    torch.manual_seed(0)
    n, k = 40, 768          # 3 blocks per row: q6_K rows start at odd-block alignment
    w = torch.randn(n, k) * 0.05
    blob = ops.kq_quantize(w, fmt)
    host = ops.kq_dequantize(blob, fmt, n, k)
    dev = ops.kq_dequantize(blob.cuda(), fmt, n, k, torch.bfloat16)
    assert dev.dtype == torch.bfloat16 and dev.device.type == "cuda"
    torch.testing.assert_close(dev.float().cpu(), host.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.parametrize("name", list(FMTS))
@pytest.mark.parametrize("m", [1, 4, 8, 33])
def test_kq_linear_matches_fp32(name, m):
    fmt = FMTS[name]
    torch.manual_seed(1)
    n, k = 136, 1280        # 5 blocks per row, N not a multiple of 4 rows per block
    w = torch.randn(n, k) * 0.05
    blob = ops.kq_quantize(w, fmt)
    wd = ops.kq_dequantize(blob, fmt, n, k)
    x = torch.randn(m, k).to(torch.bfloat16)
    want = x.float() @ wd.t()
    got = ops.kq_linear(x.cuda(), blob.cuda(), fmt, n, k)
    assert got.shape == (m, n) and got.dtype == torch.bfloat16
    rel = ((got.float().cpu() - want).norm() / want.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("qt", ["q4_k", "gguf_iq2_xxs"])
def test_kquant_linear_module_on_gpu(qt):
    from ipex_llm_amd.transformers.low_bit_linear import KQuantLinear
    torch.manual_seed(2)
    lin = torch.nn.Linear(512, 96, bias=True)
    m = KQuantLinear.from_linear(lin, qt).cuda().to(torch.bfloat16)
    x = torch.randn(2, 3, 512)
    want = torch.nn.functional.linear(x, m.dequantize().float().cpu(), lin.bias.detach())
    got = m(x.cuda().to(torch.bfloat16)).float().cpu()
    assert ((got - want).norm() / want.norm()).item() < 1e-2
