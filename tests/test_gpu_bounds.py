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


def test_seq_len_past_block_table_or_split_grid_is_reported():
    """more keys than the block-table row holds, or than the split grid covers:
    the sequence's splits leave and the error word says so"""
    ops.require()
    dev = torch.device("cuda")
    ops.check_kernel_errors(dev)
    B, Hq, Hkv, D, bs, nblk = 1, 8, 2, 128, 64, 4
    kc = torch.randn(nblk, Hkv, bs, D, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    q = torch.randn(B, 1, Hq, D, device=dev).to(torch.bfloat16)
    bt = torch.tensor([[0, 1]], dtype=torch.int32, device=dev)            # 128 keys of room
    ops.attn_decode(q, kc, vc, bt, torch.tensor([128], dtype=torch.int32, device=dev), 2, D ** -0.5)
    assert ops.check_kernel_errors(dev) == 0
    ops.attn_decode(q, kc, vc, bt, torch.tensor([200], dtype=torch.int32, device=dev), 4, D ** -0.5)
    with pytest.raises(ops.KernelError, match="sequence length"):
        ops.check_kernel_errors(dev)
    ops.attn_decode(q, kc, vc, bt, torch.tensor([100], dtype=torch.int32, device=dev), 1, D ** -0.5)  # 64-key grid
    with pytest.raises(ops.KernelError, match="sequence length"):
        ops.check_kernel_errors(dev)


def test_bad_token_id_in_lowbit_embedding_is_reported():
    from ipex_llm_amd.quantize import qtypes as Q
    ops.require()
    dev = torch.device("cuda")
    ops.check_kernel_errors(dev)
    fmt = Q.get_format(Q.resolve_qtype("sym_int4")).fmt
    blob = ops.quantize(torch.randn(300, 256), fmt).to(dev)
    torch.ops.ipex_llm_amd.embedding_lowbit(blob, fmt, 300, 256, torch.tensor([[0, 299]], device=dev), torch.bfloat16)
    assert ops.check_kernel_errors(dev) == 0
    out = torch.ops.ipex_llm_amd.embedding_lowbit(blob, fmt, 300, 256, torch.tensor([[5, 300]], device=dev),
                                                  torch.bfloat16)
    assert torch.isfinite(out.float()).all()                              # clamped row, no fault
    with pytest.raises(ops.KernelError, match="vocabulary"):
        ops.check_kernel_errors(dev)


def test_decode_advance_past_block_table_gives_no_slot():
    ops.require()
    dev = torch.device("cuda")
    ops.check_kernel_errors(dev)
    bs = 16
    ids = torch.zeros(2, dtype=torch.long, device=dev)
    nxt = torch.zeros_like(ids)
    pos = torch.tensor([14, 30], dtype=torch.long, device=dev)             # row 1 steps onto position 31 of 32
    bt = torch.tensor([[3, 4], [5, 6]], dtype=torch.int32, device=dev)
    slots = torch.zeros(2, dtype=torch.long, device=dev)
    lens = torch.zeros(2, dtype=torch.int32, device=dev)
    torch.ops.ipex_llm_amd.decode_advance(None, ids, nxt, pos, bt, bs, slots, lens, None)
    assert ops.check_kernel_errors(dev) == 0
    assert slots.tolist() == [3 * bs + 15, 6 * bs + 15] and lens.tolist() == [16, 32]
    torch.ops.ipex_llm_amd.decode_advance(None, ids, nxt, pos, bt, bs, slots, lens, None)   # position 32: no room
    assert slots.tolist()[1] == -1 and slots.tolist()[0] == 4 * bs + 0
    with pytest.raises(ops.KernelError, match="sequence length"):
        ops.check_kernel_errors(dev)


_DEBUG_LIB = __import__("os").path.join(__import__("os").path.dirname(ops.__file__), "..", "_C_debug.so")


def _debug_lib_current():
    """the debug build exists and is newer than every native source"""
    import glob
    import os
    if not os.path.exists(_DEBUG_LIB):
        return False
    csrc = os.path.join(os.path.dirname(_DEBUG_LIB), "csrc")
    srcs = [f for ext in ("hip", "cpp", "h", "cuh") for f in glob.glob(os.path.join(csrc, "**", "*." + ext),
                                                                          recursive=True)]
    return os.path.getmtime(_DEBUG_LIB) >= max(os.path.getmtime(f) for f in srcs)


@pytest.mark.skipif(not _debug_lib_current(), reason="debug build absent or older than _C.so "
                    "(python -m ipex_llm_amd._build --debug)")
def test_device_debug_build_runs_model_clean():
    """the ILLM_DEVICE_DEBUG build (launch-geometry checks in the hot
    kernels) runs a native decode in a child process without a failed check,
    with the same tokens as the release build"""
    import os
    import subprocess
    import sys
    code = r'''
import torch, sys
from transformers import LlamaConfig
from ipex_llm_amd import ops
ops.require()
from ipex_llm_amd.engine.runner import Engine
from ipex_llm_amd.models.builder import random_native_model
cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                  num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
m = random_native_model(cfg, "sym_int4", torch.device("cuda"), torch.bfloat16, seed=0)
out = Engine(m).generate([list(range(1, 40)), list(range(3, 20))], max_new_tokens=6, use_graph=False)
ops.check_kernel_errors()
print("TOKENS", out)
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for lib in ("_C.so", "_C_debug.so"):
        env = dict(os.environ, IPEX_LLM_AMD_LIB=lib, PYTHONPATH=root)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "[illm device check]" not in r.stdout + r.stderr
        res[lib] = [ln for ln in r.stdout.splitlines() if ln.startswith("TOKENS")]
    assert res["_C.so"] == res["_C_debug.so"]
