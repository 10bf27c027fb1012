"""Mixture-of-Experts: low-bit expert banks, grouped-GEMV decode, EP.

Reference: the fused MoE decode paths of ``SRC/transformers/models/
qwen3_moe.py:70-142`` / ``qwen2_moe.py:380-452`` / ``deepseek.py:274-343``
(``xe_linear.moe_forward_vec`` over per-expert weight pointer tables, top-k
via ``moe_softmax_topk``), and the generic low-bit-linear path the reference
uses for Mixtral.  Expert parallelism is not in the reference
library (vLLM's expert_map only).

MI355X design:
  * one projection of all E experts is ONE uint8 parameter [E, bytes]
    (:class:`LowBitExperts`), tiled for the MFMA GEMV on the GPU and in the
    portable canonical layout on the host / in checkpoints;
  * decode (<= 16 tokens): ``moe_route`` (router GEMV, top-k and the
    device-side per-expert pair lists in ONE launch) -> grouped GLU GEMV over
    experts (blockIdx.z = expert, all tokens routed to an expert share one
    weight stream) -> grouped down GEMV whose epilogue applies the routing
    weight and adds into the token's f32 row by atomics, read (and
    re-zeroed) by the next residual-add + RMSNorm (:meth:`NativeMoE.forward_acc`,
    three launches per block).  Standalone forwards end with ``moe_combine``
    over split-K slabs instead.  No host sync, hipGraph-capturable;
  * prefill / CPU: tokens grouped per expert and run as low-bit GEMMs;
  * expert parallel: rank r owns experts [e0, e0 + El); routing is computed
    everywhere, every rank runs its local experts over all tokens and the
    partial outputs are summed with one all-reduce over the EP group (the
    all-to-all token dispatch variant for large prefill batches is in
    ``parallel/ep.py``).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..quantize import qtypes as Q


def _dev_total(fmt, n, k):
    from ..ops.reference import dev_total
    return dev_total(fmt, n, k)


def _canon_total(fmt, n, k):
    from ..transformers.low_bit_linear import _canon_total as ct
    return ct(fmt, n, k)


class LowBitExperts(nn.Module):
    """E low-bit [n, k] weights (one projection of every expert)."""

    def __init__(self, num_experts: int, n: int, k: int, qtype="sym_int4", device=None):
        super().__init__()
        self.num_experts, self.out_features, self.in_features = num_experts, n, k
        self.qtype = Q.resolve_qtype(qtype)
        f = Q.get_format(self.qtype)
        if f is None:
            raise ValueError("LowBitExperts needs a low-bit qtype")
        self.fmt = f.fmt
        device = torch.device(device) if device is not None else torch.device("cpu")
        nb = _dev_total(self.fmt, n, k) if device.type == "cuda" else _canon_total(self.fmt, n, k)
        self.weight = nn.Parameter(torch.zeros(num_experts, nb, dtype=torch.uint8, device=device),
                                   requires_grad=False)

    @classmethod
    @torch.no_grad()
    def from_dense(cls, w: torch.Tensor, qtype="sym_int4", device=None):
        """w: [E, n, k] dense."""
        E, n, k = w.shape
        dev = torch.device(device) if device is not None else w.device
        m = cls(E, n, k, qtype, device="meta")
        blobs = []
        for e in range(E):
            we = w[e].to(dev) if dev.type == "cuda" else w[e].float().cpu()
            if dev.type == "cuda" and we.dtype not in (torch.bfloat16, torch.float16, torch.float32):
                we = we.float()
            blobs.append(ops.quantize(we, m.fmt))
        m.weight = nn.Parameter(torch.stack(blobs), requires_grad=False)
        return m

    def matmul(self, x: torch.Tensor, e: int) -> torch.Tensor:
        return ops.lowbit_matmul(x, self.weight[e], self.fmt, self.out_features, self.in_features)

    def dequantize(self, e: int, dtype=torch.float32):
        return ops.dequantize(self.weight[e], self.fmt, self.out_features, self.in_features, dtype)

    def _apply(self, fn, recurse=True):
        w = self.weight
        if w is not None and w.device.type != "meta":
            tgt = fn(torch.empty(0, dtype=torch.uint8, device=w.device)).device
            if tgt.type != w.device.type:
                n, k = self.out_features, self.in_features
                if tgt.type == "cuda":
                    new = torch.stack([ops.repack_to_device(w[e].cpu(), self.fmt, n, k) for e in range(w.shape[0])]).to(tgt)
                else:
                    new = torch.stack([ops.repack_from_device(w[e], self.fmt, n, k) for e in range(w.shape[0])])
                self.weight = nn.Parameter(new, requires_grad=False)
                return self
        return super()._apply(fn, recurse)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        w = self.weight
        if w.is_cuda and not keep_vars:
            n, k = self.out_features, self.in_features
            w = torch.stack([ops.repack_from_device(w[e], self.fmt, n, k) for e in range(w.shape[0])])
        destination[prefix + "weight"] = w if keep_vars else w.detach().cpu()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        key = prefix + "weight"
        if key not in state_dict:
            if strict:
                missing_keys.append(key)
            return
        blob = state_dict[key]
        n, k = self.out_features, self.in_features
        if blob.dtype != torch.uint8:
            new = LowBitExperts.from_dense(blob, self.qtype, "cpu").weight
        else:
            new = blob.reshape(self.num_experts, -1)
        if self.weight.is_cuda:
            new = torch.stack([ops.repack_to_device(new[e], self.fmt, n, k) for e in range(new.shape[0])]).to(self.weight.device)
        self.weight = nn.Parameter(new.clone(), requires_grad=False)

    def extra_repr(self):
        return (f"experts={self.num_experts}, in_features={self.in_features}, out_features={self.out_features}, "
                f"qtype={Q.qtype_name(self.qtype)}")


def interleave_expert_glu(gate_up: torch.Tensor, tile: int = 16) -> torch.Tensor:
    """[E, 2I, H] (gate rows then up rows) -> 16-row tiles alternating gate/up,
    the layout of the GLU-epilogue GEMV (see decoder.interleave_glu_rows)."""
    E, I2, H = gate_up.shape
    I = I2 // 2
    g, u = gate_up[:, :I], gate_up[:, I:]
    return torch.stack([g.reshape(E, I // tile, tile, H), u.reshape(E, I // tile, tile, H)], 2).reshape(E, I2, H)


class NativeMoE(nn.Module):
    """Sparse MoE block (mixtral / qwen2_moe / qwen3_moe semantics)."""

    def __init__(self, router: torch.Tensor, gate_up: LowBitExperts, down: LowBitExperts, top_k: int,
                 renorm: bool, act: int = 0, shared_mlp: Optional[nn.Module] = None,
                 shared_gate: Optional[torch.Tensor] = None, expert_offset: int = 0, num_experts: Optional[int] = None,
                 ep_group=None):
        super().__init__()
        self.router = nn.Parameter(router, requires_grad=False)          # [E_total, H]
        self.gate_up, self.down = gate_up, down                          # local experts
        self.top_k, self.renorm, self.act = top_k, renorm, act
        self.shared_mlp = shared_mlp
        self.shared_gate = nn.Parameter(shared_gate, requires_grad=False) if shared_gate is not None else None
        self.e0 = expert_offset
        self.num_experts = num_experts or router.shape[0]
        self.ep_group = ep_group
        # token-sharded expert parallel (parallel.ep.enable_token_sharded_ep):
        # an exchange object; None = replicated tokens + one EP all-reduce
        self.ep_a2a = None

    @property
    def local_experts(self) -> int:
        return self.gate_up.num_experts

    def route(self, x: torch.Tensor):
        logits = F.linear(x, self.router.to(x.dtype))
        return ops.moe_topk(logits.float(), self.top_k, self.renorm, 0)

    def _router_w(self, dtype):
        # keyed on the parameter's storage and version counter: load_state_dict /
        # in-place updates invalidate the cast copy the fused route reads
        src = self.router
        key = (src.data_ptr(), src._version, dtype, src.device)
        c = self.__dict__.get("_router_cast")
        if c is None or c[0] != key:
            c = (key, src.detach().to(dtype).contiguous())
            self.__dict__["_router_cast"] = c
        return c[1]

    def _route_counter(self, device):
        c = self.__dict__.get("_route_ctr")
        if c is None or c.device != device:
            c = torch.zeros(1, dtype=torch.int32, device=device)
            self.__dict__["_route_ctr"] = c
        return c

    def graph_max_tokens(self) -> int:
        """tokens per forward that stay on device-only launches (capturable):
        the grouped GEMV up to 16 tokens, the grouped GEMM above"""
        a2a = getattr(self, "ep_a2a", None)
        if a2a is not None:       # the peer exchange is capturable, the exact-split one is not
            return a2a.max_tokens if a2a.capturable else 0
        dev = self.gate_up.weight.device
        if dev.type == "cuda" and ops.native_gpu(self.gate_up.weight) and self.gate_up.out_features % 32 == 0:
            return 1 << 30
        return 16

    def fused_route_ok(self, x2: torch.Tensor) -> bool:
        return (x2.is_cuda and x2.shape[0] <= 16 and ops.native_gpu(x2) and self.num_experts <= 512
                and self.top_k <= 16 and self.local_experts <= 512 and x2.shape[-1] % 8 == 0
                and self.gate_up.in_features * 2 * min(16, x2.shape[0]) <= 150 * 1024)

    def _route_fused(self, x2):
        return ops.moe_route(x2, self._router_w(x2.dtype), self.top_k, self.renorm, 0, self.e0,
                             self.local_experts, self._route_counter(x2.device))

    def acc_ok(self, x2: torch.Tensor) -> bool:
        """decode block can accumulate into a residual-norm f32 slab"""
        sm = self.shared_mlp
        return (getattr(self, "ep_a2a", None) is None and self.fused_route_ok(x2)
                and (sm is None or (isinstance(sm, SharedExpertMLP) and hasattr(sm.gate_up_proj, "fmt")
                                    and hasattr(sm.down_proj, "fmt") and getattr(sm.down_proj, "bias", None) is None)))

    @torch.no_grad()
    def forward_acc(self, x2: torch.Tensor, acc: torch.Tensor) -> torch.Tensor:
        """decode: acc [T, H] f32 (zero on entry) += MoE(x2), three launches
        for the routed experts (+ the shared expert's two GEMVs)."""
        w, ids, off, rows = self._route_fused(x2)
        gu, dn = self.gate_up, self.down
        a = ops.moe_gemv_glu(x2, gu.weight, gu.fmt, gu.out_features, gu.in_features, off, rows, self.top_k, self.act)
        ops.moe_gemv_accum(a, dn.weight, dn.fmt, dn.out_features, dn.in_features, off, rows, acc, w, self.top_k)
        sm = self.shared_mlp
        if sm is not None and self.ep_group is not None:
            import torch.distributed as dist
            if dist.get_rank(self.ep_group) != 0:     # the EP all-reduce sums it in once
                sm = None
        if sm is not None:
            sg, sd = sm.gate_up_proj, sm.down_proj
            sa = ops.gemv_glu(x2, sg.weight, sg.fmt, sg.out_features, sg.in_features, sm.act)
            if self.shared_gate is None:
                ops.gemv_accum(sa, sd.weight, sd.fmt, sd.out_features, sd.in_features, acc)
            else:
                s = sd(sa).float()
                acc.add_(torch.sigmoid(F.linear(x2, self.shared_gate.to(x2.dtype)).float()) * s)
        return acc

    def _experts_grouped(self, x, w, ids, off=None, rows=None):
        """decode: device-side launches only, no host sync"""
        El = self.local_experts
        if off is None:
            off, rows = ops.moe_align(ids, self.e0, El)
        gu, dn = self.gate_up, self.down
        a = ops.moe_gemv_glu(x, gu.weight, gu.fmt, gu.out_features, gu.in_features, off, rows, self.top_k, self.act)
        part = ops.moe_gemv_partials(a, dn.weight, dn.fmt, dn.out_features, dn.in_features, off, rows)
        return ops.moe_combine(part, w, ids, self.e0, El, x.dtype)

    def _experts_gemm(self, x, w, ids):
        """prefill ("FlashMoE"): pairs sorted by expert on the device, ONE
        grouped MFMA GEMM per projection over every local expert (GLU in the
        gate/up epilogue, f32 per-pair rows from the down GEMM), one combine
        launch applying the routing weights.  No host sync: capturable."""
        El = self.local_experts
        off, rows = ops.moe_align(ids, self.e0, El)
        gu, dn = self.gate_up, self.down
        a = ops.moe_gemm(x, gu.weight, gu.fmt, gu.out_features, gu.in_features, off, rows, self.top_k,
                         False, True, True, self.act)
        part = ops.moe_gemm(a, dn.weight, dn.fmt, dn.out_features, dn.in_features, off, rows, 1,
                            True, False, False, 0, True)
        return ops.moe_combine(part.unsqueeze(0), w, ids, self.e0, El, x.dtype)

    def grouped_gemm_ok(self, x2: torch.Tensor) -> bool:
        return (x2.is_cuda and ops.native_gpu(x2) and x2.dtype in (torch.bfloat16, torch.float16)
                and self.gate_up.in_features % 8 == 0 and self.down.in_features % 8 == 0
                and self.local_experts <= 4096 and self.gate_up.out_features % 32 == 0)

    def _experts_loop(self, x, w, ids):
        """CPU / fallback: per-expert token groups through low-bit GEMMs"""
        from .decoder import deinterleave_glu
        T, H = x.shape
        y = torch.zeros(T, H, dtype=torch.float32, device=x.device)
        flat = ids.reshape(-1).long()
        local = flat - self.e0
        for e in torch.unique(local[(local >= 0) & (local < self.local_experts)]).tolist():
            sel = (local == e).nonzero(as_tuple=True)[0]
            tok = sel // self.top_k
            h = self.gate_up.matmul(x[tok], e)
            g, u = deinterleave_glu(h)
            a = (F.silu(g.float()) if self.act == 0 else F.gelu(g.float(), approximate="tanh")) * u.float()
            o = self.down.matmul(a.to(x.dtype), e).float()
            y.index_add_(0, tok, o * w.reshape(-1)[sel].float()[:, None])
        return y.to(x.dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        a2a = getattr(self, "ep_a2a", None)
        if a2a is not None:
            # token-sharded EP: this rank's tokens go to their experts' owners
            # and come back weighted (exact T*k rows each way)
            from ..parallel.ep import _local_expert_fn
            w, ids = self.route(x2)
            fn = self.__dict__.get("_ep_fn") or self.__dict__.setdefault("_ep_fn", _local_expert_fn(self))
            y = a2a(x2, w, ids, fn)
        elif self.fused_route_ok(x2):
            w, ids, off, rows = self._route_fused(x2)
            y = self._experts_grouped(x2, w, ids, off, rows)
        else:
            w, ids = self.route(x2)
            if x2.is_cuda and x2.shape[0] <= 16 and ops.native_gpu(x2) and \
                    self.gate_up.in_features * 2 * min(16, x2.shape[0]) <= 150 * 1024:
                y = self._experts_grouped(x2, w, ids)
            elif self.grouped_gemm_ok(x2):
                y = self._experts_gemm(x2, w, ids)
            else:
                y = self._experts_loop(x2, w, ids)
        if self.ep_group is not None and a2a is None:
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, self.ep_group)
        if self.shared_mlp is not None:
            s = self.shared_mlp(x2)
            if self.shared_gate is not None:
                s = torch.sigmoid(F.linear(x2, self.shared_gate.to(x2.dtype))) * s
            y = y + s
        return y.reshape(shp)


class SharedExpertMLP(nn.Module):
    """Dense-shaped GLU MLP (shared expert) on low-bit linears."""

    def __init__(self, gate_up: nn.Module, down: nn.Module, act: int = 0):
        super().__init__()
        self.gate_up_proj, self.down_proj, self.act = gate_up, down, act

    def forward(self, x):
        from .decoder import deinterleave_glu
        gu = self.gate_up_proj
        if x.is_cuda and hasattr(gu, "fmt") and x.shape[0] <= ops.GEMV_MAX_M and ops.native_gpu(x):
            a = ops.gemv_glu(x, gu.weight, gu.fmt, gu.out_features, gu.in_features, self.act)
        else:
            g, u = deinterleave_glu(gu(x))
            a = (F.silu(g) if self.act == 0 else F.gelu(g, approximate="tanh")) * u
        return self.down_proj(a.contiguous())


class HFLowBitExperts(nn.Module):
    """Drop-in for HF ``*Experts`` modules (3-D gate_up_proj/down_proj
    params; forward(hidden, top_k_index, top_k_weights)) on low-bit banks,
    so the HF forward path also runs quantized experts."""

    def __init__(self, gate_up: LowBitExperts, down: LowBitExperts, act: int = 0):
        super().__init__()
        self.gate_up, self.down, self.act = gate_up, down, act
        self.num_experts = gate_up.num_experts

    @classmethod
    def from_hf(cls, experts: nn.Module, qtype, device=None):
        act_fn = getattr(experts, "act_fn", None)
        act = 1 if act_fn is not None and "gelu" in type(act_fn).__name__.lower() else 0
        gu = interleave_expert_glu(experts.gate_up_proj.data)
        dev = device or experts.gate_up_proj.device
        return cls(LowBitExperts.from_dense(gu, qtype, dev), LowBitExperts.from_dense(experts.down_proj.data, qtype, dev),
                   act)

    def forward(self, hidden_states, top_k_index, top_k_weights):
        moe = NativeMoE.__new__(NativeMoE)
        nn.Module.__init__(moe)
        moe.gate_up, moe.down, moe.act = self.gate_up, self.down, self.act
        ep = getattr(self, "_ep", None)
        moe.top_k, moe.e0 = top_k_index.shape[-1], ep["e0"] if ep else 0
        x = hidden_states.reshape(-1, hidden_states.shape[-1]).contiguous()
        ids = top_k_index.to(torch.int32)
        w = top_k_weights.float()
        if x.is_cuda and x.shape[0] <= 16 and ops.native_gpu(x):
            y = NativeMoE._experts_grouped(moe, x, w, ids)
        elif NativeMoE.grouped_gemm_ok(moe, x):
            y = NativeMoE._experts_gemm(moe, x, w, ids)
        else:
            y = NativeMoE._experts_loop(moe, x, w, ids)
        if ep is not None:
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, ep["group"])
        return y.to(hidden_states.dtype)
