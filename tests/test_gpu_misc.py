"""Low-bit embedding gather kernel vs the CPU dequantizer."""
import pytest
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.quantize import qtypes as Q

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("qtype", ["sym_int4", "asym_int4", "sym_int8", "nf4", "fp8_e4m3"])
def test_embedding_lowbit_kernel(cuda, qtype):
    fmt = Q.get_format(Q.resolve_qtype(qtype)).fmt
    w = torch.randn(300, 256)
    blob = ops.quantize(w, fmt)
    ref = ops.dequantize(blob, fmt, 300, 256, torch.float32)
    ids = torch.tensor([[0, 5, 299], [17, 17, 42]])
    out = torch.ops.ipex_llm_amd.embedding_lowbit(blob.to(cuda), fmt, 300, 256, ids.to(cuda), torch.bfloat16)
    assert out.shape == (2, 3, 256)
    assert torch.allclose(out.float().cpu(), ref[ids], atol=2e-2, rtol=1e-2)
