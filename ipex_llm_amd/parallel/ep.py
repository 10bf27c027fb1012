"""Expert parallelism for MoE models (Mixtral / Qwen2-MoE / Qwen3-MoE).

The reference library has no EP (only vLLM's ``expert_map``
in the patched fused-MoE, ``VLLM_PATCH:11514-11516``; DeepSeek decode
requires ``ep_size == 1``, ``models/deepseek.py:335``).  BASELINE config 3
(Mixtral 8x7B on 8x MI355X) needs it, so it is native here:

* :func:`shard_experts` -- rank r keeps experts [r*E/W, (r+1)*E/W) of every
  MoE block (before or after quantization).  Attention / dense layers stay
  replicated (or tensor-parallel via ``parallel.tp``).
* decode ("replicated tokens") mode, used by :class:`models.moe.NativeMoE`:
  every rank routes all tokens, runs its local experts through the grouped
  GEMV, and ONE all-reduce over the EP group sums the partial outputs.  For
  decode batches this is a single small message per MoE layer, which the
  one-shot xGMI all-reduce handles in one launch.
* token-sharded mode (``ep_mode="a2a"``, BASELINE config 3): each rank owns
  different tokens (its own sequences: attention is data-parallel, never
  replicated); every MoE block sends each (token, expert) pair to the owner
  of its expert, the owner runs its local experts on what it received and
  sends the rows back; the source applies the routing weights.  Two
  transports, both sending EXACTLY T*k rows of H per rank per direction:
    - :class:`EPAllToAll` (GPU, one node): the HIP peer kernels of
      ``csrc/hip/ep_a2a.hip`` write straight into the destination's
      IPC-mapped receive region over xGMI (each GPU reaches its 7 peers on 7
      links at once), device-side counts/offsets and epoch flags -- no host
      sync, hipGraph-capturable;
    - :class:`ExactSplitAllToAll` (gloo / multi-node / CPU): counts are
      exchanged first, then ``all_to_all_single`` with exact split sizes
      (host sync; not capturable).
  Every rank must run the same number of MoE calls (lockstep forwards).
"""
from __future__ import annotations

import socket
from typing import Callable, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .comm import PEER_UNCACHED, barrier, get_rank, get_world_size


def expert_range(num_experts: int, rank: int, world: int):
    if num_experts % world:
        raise ValueError(f"expert parallel: {num_experts} experts not divisible by {world} ranks")
    per = num_experts // world
    return rank * per, per


@torch.no_grad()
def shard_experts(model: nn.Module, group=None) -> nn.Module:
    """Keep only this rank's experts in every MoE block (HF module tree,
    dense 3-D expert params or converted :class:`HFLowBitExperts`)."""
    from ..models.moe import HFLowBitExperts
    rank, world = get_rank(group), get_world_size(group)
    if world == 1:
        return model
    if group is None:
        group = dist.group.WORLD
    for mod in model.modules():
        ex = getattr(mod, "experts", None)
        if ex is None or not hasattr(mod, "gate"):
            continue
        if isinstance(ex, HFLowBitExperts):
            E = ex.gate_up.num_experts
            e0, per = expert_range(E, rank, world)
            for bank in (ex.gate_up, ex.down):
                bank.weight = nn.Parameter(bank.weight[e0:e0 + per].contiguous(), requires_grad=False)
                bank.num_experts = per
            ex.num_experts = per
        elif isinstance(getattr(ex, "gate_up_proj", None), nn.Parameter):
            E = ex.gate_up_proj.shape[0]
            e0, per = expert_range(E, rank, world)
            ex.gate_up_proj = nn.Parameter(ex.gate_up_proj.data[e0:e0 + per].contiguous(), requires_grad=False)
            ex.down_proj = nn.Parameter(ex.down_proj.data[e0:e0 + per].contiguous(), requires_grad=False)
            ex.num_experts = per
        else:
            continue
        mod._ep = {"e0": e0, "local": per, "group": group, "num_experts": E}
        ex._ep = mod._ep
    model._ep = {"group": group, "rank": rank, "world": world}
    return model



ExpertFn = Callable[[torch.Tensor, torch.Tensor], torch.Tensor]


def _local_expert_fn(moe) -> ExpertFn:
    """(recv_x [R, H], recv_e [R] global expert ids, -1 = empty slot) ->
    expert outputs [R, H] (rows of empty slots are unspecified): ONE grouped
    MFMA GEMM per projection over this rank's experts on the GPU (FlashMoE
    path, pairs sorted by expert on the device), the per-expert loop
    elsewhere."""
    from .. import ops

    def fn(recv_x: torch.Tensor, recv_e: torch.Tensor) -> torch.Tensor:
        El = moe.local_experts
        if recv_x.is_cuda and ops.native_gpu(recv_x) and moe.grouped_gemm_ok(recv_x):
            off2, rows2 = ops.moe_align(recv_e.view(-1, 1), moe.e0, El)
            gu, dn = moe.gate_up, moe.down
            a = ops.moe_gemm(recv_x, gu.weight, gu.fmt, gu.out_features, gu.in_features, off2, rows2, 1,
                             False, True, True, moe.act)
            return ops.moe_gemm(a, dn.weight, dn.fmt, dn.out_features, dn.in_features, off2, rows2, 1,
                                True, False, False, 0, False)
        import torch.nn.functional as F
        from ..models.decoder import deinterleave_glu
        out = torch.zeros_like(recv_x)
        local = recv_e.long() - moe.e0
        for e in torch.unique(local[(local >= 0) & (local < El)]).tolist():
            sel = (local == e).nonzero(as_tuple=True)[0]
            g, u = deinterleave_glu(moe.gate_up.matmul(recv_x[sel], e))
            a = (F.silu(g.float()) if moe.act == 0 else F.gelu(g.float(), approximate="tanh")) * u.float()
            out[sel] = moe.down.matmul(a.to(recv_x.dtype), e).to(out.dtype)
        return out
    return fn


class ExactSplitAllToAll:
    """Exact-count token exchange over any process group (gloo on CPU, RCCL
    across nodes): pair counts per destination are exchanged first, then one
    ``all_to_all_single`` with exact split sizes moves the T*k token rows
    (and their expert ids) and a second one brings the results back.  Needs
    the counts on the host, so it is not capturable."""

    capturable = False

    def __init__(self, group=None, experts_per_rank: int = 1):
        self.group = group
        self.world = get_world_size(group)
        self.el = experts_per_rank
        self.last_sent_rows = 0              # rows this rank sent in the last call (bytes = rows * H * elsize)

    def __call__(self, x: torch.Tensor, w: torch.Tensor, ids: torch.Tensor, expert_fn: ExpertFn) -> torch.Tensor:
        T, H = x.shape
        k = ids.shape[1]
        ids32 = ids.reshape(-1).to(torch.int32)
        dest = torch.div(ids32, self.el, rounding_mode="floor").long()
        order = torch.argsort(dest, stable=True)                     # pairs grouped by destination
        send_counts = torch.bincount(dest, minlength=self.world)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        send_x = x[order // k].contiguous()
        recv_x = x.new_empty(sum(rc), H)
        dist.all_to_all_single(recv_x, send_x, rc, sc, group=self.group)
        recv_e = ids32.new_empty(sum(rc))
        dist.all_to_all_single(recv_e, ids32[order].contiguous(), rc, sc, group=self.group)
        self.last_sent_rows = int(sum(sc))
        out = expert_fn(recv_x, recv_e).to(x.dtype).contiguous()
        back = x.new_empty(sum(sc), H)
        dist.all_to_all_single(back, out, sc, rc, group=self.group)
        y = torch.zeros(T, H, dtype=torch.float32, device=x.device)
        y.index_add_(0, order // k, back.float() * w.reshape(-1).float()[order][:, None])
        return y.to(x.dtype)


class EPAllToAll:
    """Capturable peer all-to-all for one intra-node EP group (HIP kernels of
    ``csrc/hip/ep_a2a.hip``).

    Collective constructor: every rank allocates one IPC buffer
    ``[signals | counts | meta [W][cap] | recv [W][cap][H] | ret [W][cap][H]]``
    (``cap = max_tokens * top_k``: dropless even if every pair of a source
    goes to one rank) and maps every peer's.  ``__call__`` runs
      dispatch  (pairs sorted by destination on the device, written into the
                 owners' recv regions; exactly T*k rows leave the rank),
      experts   (``expert_fn`` over the receive buffer; slots without a pair
                 carry expert -1 and are skipped by the grouped GEMM),
      return    (result rows back into the sources' ret regions),
      combine   (routing-weighted sum per token, fixed order),
    with the call epoch advanced on the device: no host sync anywhere.  A
    peer that stays silent (EP_TIMEOUT_S) sets ERR_PEER in the kernel error
    word (ops.check_kernel_errors raises) and the output becomes NaN."""

    SIG_BYTES = 2 * 64 * 8 * 4
    CNT_BYTES = 256
    capturable = True

    def __init__(self, group=None, hidden: int = 0, max_tokens: int = 8192, top_k: int = 2,
                 experts_per_rank: int = 1, dtype=torch.bfloat16, device=None):
        from .. import ops
        ops.require()
        self.group = group
        self.world, self.rank = get_world_size(group), get_rank(group)
        if self.world > 8:
            raise ValueError("EPAllToAll supports up to 8 ranks (one xGMI node)")
        if dtype not in (torch.bfloat16, torch.float16) or hidden % 8:
            raise ValueError("EPAllToAll: bf16/fp16 activations with hidden % 8 == 0")
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise RuntimeError("EPAllToAll needs all ranks on one node")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.H, self.k, self.el, self.dtype = hidden, top_k, experts_per_rank, dtype
        self.max_tokens = max_tokens
        self.cap = max_tokens * top_k
        A = torch.ops.ipex_llm_amd
        W, cap, H = self.world, self.cap, hidden
        self.nbytes = A.ep_buffer_bytes(W, cap, H)
        with torch.cuda.device(self.device):
            self._own = A.ipc_alloc(self.nbytes, PEER_UNCACHED)
            handle = A.ipc_handle(self._own)
        handles = [None] * W
        dist.all_gather_object(handles, handle.tolist(), group=group)
        self._opened, ptrs = [], []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    ptrs.append(self._own)
                else:
                    p = A.ipc_open(torch.tensor(h, dtype=torch.uint8))
                    self._opened.append(p)
                    ptrs.append(p)
        self.ptrs = ptrs
        base = self.SIG_BYTES + self.CNT_BYTES
        self.meta = A.ep_view(self._own, base, [W * cap], torch.int32, self.device)
        self.recv = A.ep_view(self._own, base + W * cap * 4, [W * cap, H], dtype, self.device)
        self.epoch = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.counts = torch.zeros(W + 1, dtype=torch.int32, device=self.device)
        self._off = None
        barrier(group)

    def eligible(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.device == self.device and x.dtype == self.dtype and x.dim() == 2
                and x.shape[1] == self.H and 0 < x.shape[0] <= self.max_tokens)

    def __call__(self, x: torch.Tensor, w: torch.Tensor, ids: torch.Tensor, expert_fn: ExpertFn) -> torch.Tensor:
        from .. import ops
        T = x.shape[0]
        if not self.eligible(x) or ids.shape[1] != self.k:
            raise ValueError(f"EPAllToAll: x must be [1..{self.max_tokens}, {self.H}] {self.dtype} on "
                             f"{self.device} with top-{self.k} ids (got {tuple(x.shape)} {x.dtype})")
        A = torch.ops.ipex_llm_amd
        x = x.contiguous()
        ids32 = ids.to(torch.int32).contiguous()
        self.epoch.add_(1)
        dest = torch.div(ids32, self.el, rounding_mode="floor")
        off, rows = ops.moe_align(dest, 0, self.world)               # pairs sorted by destination rank
        pos = torch.empty(T * self.k, dtype=torch.int32, device=x.device)
        A.ep_dispatch(x, ids32, off, rows, pos, self.counts, self.ptrs, self.rank, self.cap, self.el, self.epoch)
        out = expert_fn(self.recv, self.meta).contiguous()
        if out.dtype != self.dtype:
            out = out.to(self.dtype)
        A.ep_return(out, self.counts, self.ptrs, self.rank, self.cap, self.epoch)
        y = torch.empty_like(x)
        A.ep_combine(y, w.float().contiguous(), ids32, off, pos, self.counts, self.ptrs, self.rank, self.cap,
                     self.el, self.epoch)
        self._off = off
        return y

    @property
    def last_sent_rows(self) -> int:
        """rows this rank dispatched in the last call (host sync; tests)"""
        return 0 if self._off is None else int(self._off[self.world].item())

    def received_counts(self):
        """pairs received from every source in the last call (host sync)"""
        return self.counts[:self.world].tolist()

    def close(self):
        A = torch.ops.ipex_llm_amd
        torch.cuda.synchronize(self.device)
        barrier(self.group)
        for p in self._opened:
            A.ipc_close(p)
        A.ipc_free(self._own)
        self._opened = []


class TieredAllToAll:
    """Two peer exchanges: a small-capacity one for decode-sized calls (the
    receiver's grouped GEMM runs over W * cap_small rows) and a large one for
    prefill chunks.  The tier is picked by T, so every rank of one forward
    must be on the same side of ``small.max_tokens`` (lockstep phases; a
    mismatch times out as ERR_PEER, never silently)."""

    capturable = True

    def __init__(self, small: "EPAllToAll", big: "EPAllToAll"):
        self.small, self.big = small, big
        self.max_tokens = big.max_tokens
        self._last = small

    def __call__(self, x, w, ids, expert_fn):
        self._last = self.small if x.shape[0] <= self.small.max_tokens else self.big
        return self._last(x, w, ids, expert_fn)

    @property
    def last_sent_rows(self) -> int:
        return self._last.last_sent_rows

    def received_counts(self):
        return self._last.received_counts()

    def close(self):
        self.small.close()
        self.big.close()


def make_ep_all_to_all(group, hidden: int, top_k: int, experts_per_rank: int, dtype, device,
                       max_tokens: Optional[int] = None, decode_tokens: int = 64):
    """Collective: the best exchange for ``group`` -- the peer kernels for an
    intra-node RCCL group on the GPU (ILLM_EP_P2P=0 disables, =force also
    takes it over a gloo group of GPU processes; a decode tier of
    ``decode_tokens`` plus a prefill tier of ``max_tokens``), exact-split
    ``all_to_all_single`` otherwise."""
    import os
    from .. import ops
    dev = torch.device(device)
    mode = os.environ.get("ILLM_EP_P2P", "1")      # 0: never, force: also over a gloo group (tests)
    p2p = (dev.type == "cuda" and mode != "0" and (mode == "force" or dist.get_backend(group) == "nccl")
           and dtype in (torch.bfloat16, torch.float16) and hidden % 8 == 0 and get_world_size(group) <= 8
           and ops.available())
    if p2p:
        mt = max_tokens or int(os.environ.get("ILLM_EP_MAX_TOKENS", "8192"))
        small = EPAllToAll(group, hidden, min(decode_tokens, mt), top_k, experts_per_rank, dtype, dev)
        if mt <= decode_tokens:
            return small
        return TieredAllToAll(small, EPAllToAll(group, hidden, mt, top_k, experts_per_rank, dtype, dev))
    return ExactSplitAllToAll(group, experts_per_rank)


def enable_token_sharded_ep(model, max_tokens: Optional[int] = None):
    """Switch every EP-sharded NativeMoE block of ``model`` to token-sharded
    all-to-all mode (collective: call on every rank).  One exchange object is
    shared by all blocks of the model (their calls are serialized)."""
    from ..models.moe import NativeMoE
    blocks = [m for m in model.modules() if isinstance(m, NativeMoE) and m.ep_group is not None]
    if not blocks:
        return model
    b0 = blocks[0]
    dev = b0.gate_up.weight.device
    dtype = getattr(model, "dtype", None) or torch.bfloat16
    a2a = make_ep_all_to_all(b0.ep_group, b0.gate_up.in_features, b0.top_k, b0.local_experts, dtype, dev,
                             max_tokens)
    for b in blocks:
        b.ep_a2a = a2a
    model._ep_a2a = a2a
    return model


def ep_moe_all_to_all(x: torch.Tensor, moe, group=None) -> torch.Tensor:
    """Token-sharded MoE: x [T_local, H] are THIS rank's tokens; ``moe`` is
    the rank's :class:`NativeMoE` (local experts [e0, e0+El)).  Returns the
    routed-experts output for the local tokens (shared expert not included).
    Uses the block's exchange (``enable_token_sharded_ep``) or an exact-split
    one."""
    a2a = getattr(moe, "ep_a2a", None) or ExactSplitAllToAll(group, moe.local_experts)
    w, ids = moe.route(x)
    return a2a(x.contiguous(), w, ids, _local_expert_fn(moe))
