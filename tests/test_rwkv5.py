"""RWKV-5 (remote-code ``model_type == "rwkv5"``): WKV-5 recurrence and the
patched time-mix forward (reference ``SRC/transformers/models/rwkv5.py``).

The remote modeling file is not available offline, so the block below is a
stand-in with the same attributes and the reference CPU path's math
(``rwkv5.py:122-163``: per-head outer-product state, GroupNorm, gate); parity
with the hub code itself is unpinned.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from ipex_llm_amd.models.rwkv import patch_rwkv5, rwkv5_wkv, rwkv5_wkv_reference


def _naive_wkv5(w, u, r, k, v, state):
    """element-wise formula: out[j] = sum_i r[i] (u[i] k[i] v[j] + s[i][j]); s = k v^T + w s"""
    B, T, H, S = k.shape
    st = state.clone().double()
    out = torch.zeros(B, T, H, S, dtype=torch.float64)
    for b in range(B):
        for h in range(H):
            s = st[b, h]
            for t in range(T):
                kk, vv, rr = k[b, t, h].double(), v[b, t, h].double(), r[b, t, h].double()
                a = torch.outer(kk, vv)
                out[b, t, h] = rr @ (u[h].double()[:, None] * a + s)
                s = a + w[h].double()[:, None] * s
            st[b, h] = s
    return out, st


def _inputs(B, T, H, S, device="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    w = torch.exp(-torch.exp(torch.randn(H, S, generator=g) * 0.5 - 1.0))
    u = torch.randn(H, S, generator=g) * 0.3
    r, k, v = (torch.randn(B, T, H, S, generator=g) * 0.5 for _ in range(3))
    st = torch.randn(B, H, S, S, generator=g) * 0.1
    return [x.to(device) for x in (w, u, r, k, v, st)]


def test_wkv5_reference_matches_formula():
    w, u, r, k, v, st = _inputs(2, 5, 2, 8)
    want, wst = _naive_wkv5(w, u, r, k, v, st)
    s2 = st.clone()
    got = rwkv5_wkv_reference(w, u, r, k, v, s2)
    assert torch.allclose(got.double(), want, atol=1e-5)
    assert torch.allclose(s2.double(), wst, atol=1e-5)


class _Rwkv5TimeMix(nn.Module):
    """attribute-compatible stand-in for the remote-code RWKV-5 time-mix block"""

    def __init__(self, C, H, layer_id):
        super().__init__()
        self.layer_id = layer_id
        S = C // H
        self.time_decay = nn.Parameter(torch.randn(H, S) * 0.5 - 1.0)
        self.time_faaaa = nn.Parameter(torch.randn(H, S) * 0.3)
        for n in ("key", "value", "receptance", "gate"):
            setattr(self, f"time_mix_{n}", nn.Parameter(torch.rand(1, 1, C)))
        self.key, self.value, self.receptance, self.gate, self.output = (nn.Linear(C, C, bias=False)
                                                                        for _ in range(5))
        self.ln_x = nn.GroupNorm(H, C)
        with torch.no_grad():
            self.ln_x.weight.uniform_(0.5, 1.5)
            self.ln_x.bias.uniform_(-0.1, 0.1)

    def ref_forward(self, hidden, state):
        """reference semantics, one token at a time (rwkv5.py CPU path)"""
        B, T, C = hidden.shape
        H = self.time_decay.shape[0]
        S = C // H
        li = self.layer_id
        outs = []
        for t in range(T):
            x = hidden[:, t:t + 1]
            sh = state[0][:, :, li].unsqueeze(1)
            mix = {n: x * getattr(self, f"time_mix_{n}") + sh * (1 - getattr(self, f"time_mix_{n}"))
                   for n in ("key", "value", "receptance", "gate")}
            kk = self.key(mix["key"]).view(B, H, S, 1)
            vv = self.value(mix["value"]).view(B, H, 1, S)
            rr = self.receptance(mix["receptance"]).view(B, H, 1, S)
            gg = F.silu(self.gate(mix["gate"]))
            w = torch.exp(-torch.exp(self.time_decay.float())).view(H, S, 1)
            u = self.time_faaaa.float().view(H, S, 1)
            a = kk @ vv
            s = state[1][..., li]
            o = (rr @ (u * a + s)).view(B, C)
            state[1][..., li] = a + w * s
            state[0][:, :, li] = x[:, 0]
            o = F.group_norm(o, H, self.ln_x.weight, self.ln_x.bias, self.ln_x.eps).view(B, 1, C) * gg
            outs.append(self.output(o))
        return torch.cat(outs, 1), state


def _state(B, C, H, L, device="cpu"):
    S = C // H
    return [torch.zeros(B, C, L, device=device), torch.zeros(B, H, S, S, L, device=device)]


@torch.no_grad()
def test_rwkv5_patched_forward_matches_reference_cpu():
    torch.manual_seed(0)
    B, C, H, T = 2, 64, 4, 9
    blocks = nn.ModuleList([_Rwkv5TimeMix(C, H, i) for i in range(2)])
    x = torch.randn(B, T, C)
    ref_state = _state(B, C, H, 2)
    want = x
    for blk in blocks:
        want, ref_state = blk.ref_forward(want, ref_state)
    assert patch_rwkv5(blocks) == 2
    st = _state(B, C, H, 2)
    # prompt chunk, then one-token steps: same as the token-by-token reference
    got = x[:, :6]
    for blk in blocks:
        got, st = blk(got, st)
    steps = [got]
    for t in range(6, T):
        y = x[:, t:t + 1]
        for blk in blocks:
            y, st = blk(y, st)
        steps.append(y)
    got = torch.cat(steps, 1)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4)
    assert torch.allclose(st[1], ref_state[1], atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("S", [32, 64, 128])
def test_wkv5_kernel(cuda, S):
    """HIP WKV-5 vs the fp32 reference, carrying the state across two calls
    (chunk boundary of the kernel's 32-step staging crossed)"""
    B, T, H = 2, 45, 3
    w, u, r, k, v, st = _inputs(B, T, H, S, seed=S)
    s_ref = st.clone()
    want = rwkv5_wkv_reference(w, u, r, k, v, s_ref)
    s_gpu = st.to(cuda)
    got = rwkv5_wkv(w.to(cuda), u.to(cuda), r.to(cuda), k.to(cuda), v.to(cuda), s_gpu)
    assert torch.ops.ipex_llm_amd.rwkv_wkv5 is not None
    assert (got.cpu() - want).abs().max().item() < 1e-4 * max(1.0, want.abs().max().item())
    assert (s_gpu.cpu() - s_ref).abs().max().item() < 1e-4 * max(1.0, s_ref.abs().max().item())
    _, _, r2, k2, v2, _ = _inputs(B, 1, H, S, seed=S + 1)
    want2 = rwkv5_wkv_reference(w, u, r2, k2, v2, s_ref)
    got2 = rwkv5_wkv(w.to(cuda), u.to(cuda), r2.to(cuda), k2.to(cuda), v2.to(cuda), s_gpu)
    assert (got2.cpu() - want2).abs().max().item() < 1e-4 * max(1.0, want2.abs().max().item())


@pytest.mark.gpu
@torch.no_grad()
def test_rwkv5_patched_forward_gpu_matches_cpu(cuda):
    """patched time-mix block on the GPU (WKV-5 HIP kernel) vs the CPU reference"""
    torch.manual_seed(1)
    B, C, H, T = 2, 128, 2, 20
    blk = _Rwkv5TimeMix(C, H, 0)
    x = torch.randn(B, T, C)
    want, ws = blk.ref_forward(x, _state(B, C, H, 1))
    patch_rwkv5(blk)
    blk = blk.to(cuda)
    got, gs = blk(x.to(cuda), _state(B, C, H, 1, cuda))
    assert torch.allclose(got.cpu(), want, atol=1e-3, rtol=1e-3)
    assert torch.allclose(gs[1].cpu(), ws[1], atol=1e-4)
