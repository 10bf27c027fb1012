"""Grouped MoE decode kernels (moe_align / grouped GLU GEMV / grouped
partial GEMV / moe_combine) vs an fp32 PyTorch reference on the
dequantized expert weights."""
import pytest
import torch
import torch.nn.functional as F

from ipex_llm_amd import ops
from ipex_llm_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _bank(E, I, H, qtype, dev):
    from ipex_llm_amd.models.moe import LowBitExperts, interleave_expert_glu
    g = torch.Generator(device=dev).manual_seed(0)
    gu = torch.randn(E, 2 * I, H, generator=g, device=dev) * 0.05
    dn = torch.randn(E, H, I, generator=g, device=dev) * 0.05
    return (LowBitExperts.from_dense(interleave_expert_glu(gu), qtype, dev),
            LowBitExperts.from_dense(dn, qtype, dev))


def _ref(x, gub, dnb, w, ids, e0, El):
    from ipex_llm_amd.models.decoder import deinterleave_glu
    T = x.shape[0]
    y = torch.zeros(T, dnb.out_features, device=x.device)
    for t in range(T):
        for j in range(ids.shape[1]):
            e = int(ids[t, j]) - e0
            if not (0 <= e < El):
                continue
            h = x[t].float() @ gub.dequantize(e).t()
            g, u = deinterleave_glu(h[None])
            a = F.silu(g) * u
            y[t] += w[t, j] * (a @ dnb.dequantize(e).t())[0]
    return y


@pytest.mark.parametrize("T", [1, 3, 16])
@pytest.mark.parametrize("qtype", ["sym_int4", "sym_int8", "asym_int4"])
def test_grouped_moe_decode(cuda, T, qtype):
    from ipex_llm_amd.models.moe import NativeMoE
    E, I, H, k = 8, 256, 512, 2
    gub, dnb = _bank(E, I, H, qtype, cuda)
    router = torch.randn(E, H, device=cuda, dtype=torch.bfloat16)
    moe = NativeMoE(router, gub, dnb, k, True, 0)
    x = (torch.randn(T, H, device=cuda) * 0.5).to(torch.bfloat16)
    w, ids = moe.route(x)
    ref = _ref(x, gub, dnb, w, ids, 0, E)
    y = moe._experts_grouped(x, w, ids).float()
    assert ((y - ref).norm() / ref.norm()).item() < 2e-2
    loop = moe._experts_loop(x, w, ids).float()
    assert ((loop - ref).norm() / ref.norm()).item() < 2e-2


def test_moe_align_matches_reference(cuda):
    ids = torch.randint(0, 16, (12, 4), device=cuda, dtype=torch.int32)
    for e0, El in ((0, 16), (4, 8)):
        off, rows = ops.moe_align(ids, e0, El)
        roff, rrows = R.moe_align(ids.cpu(), e0, El)
        assert off.cpu().tolist() == roff.tolist()
        n = int(roff[-1])
        assert rows[:n].cpu().tolist() == rrows[:n].tolist()


def test_expert_parallel_slices_sum_to_full(cuda):
    """two EP 'ranks' (experts 0-3 and 4-7) computed separately sum to the full block"""
    from ipex_llm_amd.models.moe import LowBitExperts, NativeMoE
    E, I, H, k = 8, 128, 256, 2
    gub, dnb = _bank(E, I, H, "sym_int4", cuda)
    router = torch.randn(E, H, device=cuda, dtype=torch.bfloat16)
    x = torch.randn(4, H, device=cuda).to(torch.bfloat16)
    full = NativeMoE(router, gub, dnb, k, True, 0)
    w, ids = full.route(x)
    y = full._experts_grouped(x, w, ids).float()
    parts = []
    for r in range(2):
        sl = slice(4 * r, 4 * r + 4)
        g2 = LowBitExperts(4, gub.out_features, gub.in_features, "sym_int4", "meta")
        g2.weight = torch.nn.Parameter(gub.weight[sl].contiguous(), requires_grad=False)
        d2 = LowBitExperts(4, dnb.out_features, dnb.in_features, "sym_int4", "meta")
        d2.weight = torch.nn.Parameter(dnb.weight[sl].contiguous(), requires_grad=False)
        m = NativeMoE(router, g2, d2, k, True, 0, expert_offset=4 * r, num_experts=E)
        parts.append(m._experts_grouped(x, w, ids).float())
    assert torch.allclose(parts[0] + parts[1], y, atol=2e-2, rtol=2e-2)
