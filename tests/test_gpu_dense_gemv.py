"""Dense bf16 / fp16 skinny GEMM (csrc/hip/dense_gemv.hip) vs an fp32
PyTorch reference, and DenseLinear routing decode rows through it."""
import pytest
import torch

from ipex_llm_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M", [1, 2, 3, 5, 8, 13, 16])
@pytest.mark.parametrize("N,K", [(300, 1024), (4096, 4104), (64, 520), (1000, 4096), (200, 14336)])
def test_dense_gemv_matches_fp32(dt, M, N, K):
    ops.require()
    torch.manual_seed(M * 7 + N)
    w = (torch.randn(N, K) * 0.05).to(dt)
    x = torch.randn(M, K).to(dt)
    b = torch.randn(N).to(dt)
    want = x.float() @ w.float().t() + b.float()
    got = torch.ops.ipex_llm_amd.dense_linear(x.cuda(), w.cuda(), b.cuda()).float().cpu()
    rel = ((got - want).norm() / want.norm()).item()
    assert rel < 1e-2, rel


def test_dense_linear_module_uses_kernel():
    from ipex_llm_amd.transformers.low_bit_linear import DenseLinear
    lin = torch.nn.Linear(512, 384)
    m = DenseLinear.from_linear(lin, torch.bfloat16, torch.device("cuda"))
    x = torch.randn(3, 512, device="cuda", dtype=torch.bfloat16)
    with torch.no_grad():
        got = m(x).float()
    want = torch.nn.functional.linear(x.float(), m.weight.float(), m.bias.float())
    assert ((got - want).norm() / want.norm()).item() < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_dense_mfma_rows_independent_of_batch(dt):
    """the MFMA skinny GEMM (K % 64 == 0): each output column is its own MFMA
    column, so row m of a 16-row launch equals the 1-row launch bit for bit
    (the speculative verify's exactness), plain and GLU"""
    ops.require()
    torch.manual_seed(5)
    K, N, I = 4096, 1040, 512
    w = (torch.randn(N, K, device="cuda") * 0.05).to(dt)
    wgu = (torch.randn(2 * I, K, device="cuda") * 0.05).to(dt)
    x = torch.randn(16, K, device="cuda").to(dt)
    full = torch.ops.ipex_llm_amd.dense_linear(x, w, None)
    gfull = torch.ops.ipex_llm_amd.dense_glu(x, wgu, 0)
    for M in (1, 3, 7):
        assert torch.equal(torch.ops.ipex_llm_amd.dense_linear(x[:M].contiguous(), w, None), full[:M])
        assert torch.equal(torch.ops.ipex_llm_amd.dense_glu(x[:M].contiguous(), wgu, 0), gfull[:M])


@pytest.mark.parametrize("r", [8, 16])
def test_dense_linear_t_matches(r):
    """the transposed-output skinny GEMM (training's x A^T in [tokens, r])"""
    ops.require()
    torch.manual_seed(r)
    x2 = torch.randn(1536, 4096, device="cuda").bfloat16()
    A = (torch.randn(r, 4096, device="cuda") * 0.05).bfloat16()
    y = torch.ops.ipex_llm_amd.dense_linear_t(A, x2)
    assert y.shape == (1536, r) and y.is_contiguous()
    assert torch.equal(y, torch.ops.ipex_llm_amd.dense_linear(A, x2, None).t().contiguous())
    ref = x2.float() @ A.float().t()
    assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2
