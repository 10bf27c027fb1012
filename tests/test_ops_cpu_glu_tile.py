"""GLU over the tile-interleaved gate/up layout on the CPU path (reference)."""
import torch

from ipex_llm_amd import ops
from ipex_llm_amd.models.decoder import deinterleave_glu


def test_glu_tile_reference_cpu():
    torch.manual_seed(0)
    gu = torch.randn(5, 2 * 64)
    g, u = deinterleave_glu(gu, 16)
    want = torch.nn.functional.silu(g) * u
    assert torch.allclose(ops.glu(gu, 0, tile=16), want, atol=1e-6)
