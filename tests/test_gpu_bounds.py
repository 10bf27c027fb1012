"""Device-side bounds checks: a block table pointing outside
the KV cache makes the attention / rope_kv kernels skip the access and set
the kernel error word instead of faulting; ops.check_kernel_errors raises."""
import pytest
import torch

from ipex_llm_amd import ops

pytestmark = pytest.mark.gpu


def test_bad_block_table_is_reported_not_faulted():
    ops.require()
    dev = torch.device("cuda")
    ops.check_kernel_errors(dev)                       # clean slate
    B, Hq, Hkv, D, bs, nblk = 1, 8, 2, 128, 64, 4
    kc = torch.randn(nblk, Hkv, bs, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(nblk, Hkv, bs, D, device=dev).to(torch.bfloat16)
    q = torch.randn(B, 1, Hq, D, device=dev).to(torch.bfloat16)
    good = torch.tensor([[0, 1]], dtype=torch.int32, device=dev)
    lens = torch.tensor([100], dtype=torch.int32, device=dev)
    ops.attn_decode(q, kc, vc, good, lens, 2, D ** -0.5)
    assert ops.check_kernel_errors(dev) == 0
    bad = torch.tensor([[0, 1000]], dtype=torch.int32, device=dev)   # block 1000 of a 4-block cache
    ops.attn_decode(q, kc, vc, bad, lens, 2, D ** -0.5)
    with pytest.raises(ops.KernelError, match="block-table"):
        ops.check_kernel_errors(dev)
    assert ops.check_kernel_errors(dev) == 0           # reset by the read
    # rope_kv with a slot past the cache end: skipped + reported
    qkv = torch.randn(1, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    qo = torch.empty(1, Hq, D, device=dev, dtype=torch.bfloat16)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=dev, dtype=torch.float32) / D))
    ops.rope_kv(qkv, qo, kc, vc, torch.tensor([nblk * bs + 5], device=dev), torch.tensor([3], device=dev), inv,
                Hq, Hkv, D)
    with pytest.raises(ops.KernelError, match="slot"):
        ops.check_kernel_errors(dev)
