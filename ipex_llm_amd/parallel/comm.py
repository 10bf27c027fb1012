"""Process groups and collectives: RCCL over xGMI + a one-shot peer all-reduce.

Reference: oneCCL through ``torch.distributed('ccl')``
(``SRC/transformers/pipeline_parallel.py:108-112``), the row-parallel
all-reduce inside ``LowBitLinear.forward`` (``low_bit_linear.py:715-722``)
and the patched DG2 LL256 all-reduce.

MI355X design: one process per GPU, ``torch.distributed`` with the ``nccl``
backend (= RCCL on ROCm) for everything, plus :class:`CustomAllReduce` for
the small, latency-bound tensor-parallel messages of decode (8 x 4096 bf16 =
64 KiB per o_proj/down_proj).  On a fully connected 8-GPU xGMI node a ring
all-reduce of such a message is latency bound and uses one link at a time;
the one-shot kernel (``csrc/hip/allreduce.hip``) reads all 7 peers over 7
links in a single launch and is hipGraph-capturable.  On CPU (tests) the
backend is ``gloo`` and everything goes through ``dist.all_reduce``.
"""
from __future__ import annotations

import os
import socket
from datetime import timedelta
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

# peer (hipIpc) buffers of the custom all-reduce / EP all-to-all are allocated
# uncached (ops_dist.cpp ipc_alloc): other GPUs write flags and data into them
# over xGMI.  ILLM_PEER_CACHED=1 restores plain hipMalloc (A/B only).
PEER_UNCACHED = os.environ.get("ILLM_PEER_CACHED", "0") != "1"

_CUSTOM: Dict[int, "CustomAllReduce"] = {}


def env_rank_world() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", 0))))


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> Tuple[int, int, int]:
    """Initialise the default process group from torchrun-style env vars.
    Returns (rank, world_size, local_rank).  backend defaults to ``nccl``
    (RCCL) when a GPU is visible, else ``gloo``."""
    rank, world, local = env_rank_world()
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size(), local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1 or backend == "gloo":
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend, rank=rank, world_size=world, timeout=timedelta(seconds=timeout_s), **kw)
    return rank, world, local


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank(group=None) -> int:
    return dist.get_rank(group) if is_dist() else 0


def get_world_size(group=None) -> int:
    return dist.get_world_size(group) if is_dist() else 1


def barrier(group=None):
    if is_dist():
        dist.barrier(group=group)


def _custom_enabled() -> bool:
    return os.environ.get("IPEX_LLM_AMD_CUSTOM_AR", "1") not in ("0", "false", "False")


def all_reduce_inplace(t: torch.Tensor, group=None) -> torch.Tensor:
    """Sum ``t`` over ``group``.  Small GPU messages take the one-shot xGMI
    kernel when a :class:`CustomAllReduce` was set up for the group; the
    rest go to RCCL (or gloo on CPU).  Returns the reduced tensor (may be a
    new tensor for the custom path)."""
    if not is_dist() or get_world_size(group) == 1:
        return t
    car = _CUSTOM.get(id(group)) if t.is_cuda else None
    if car is not None and car.eligible(t):
        return car(t, out=t)
    dist.all_reduce(t, group=group)
    return t


def all_gather_last_dim(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate every rank's ``t`` along the last dim (vocab-parallel
    logits).  GPU messages that fit take the capturable peer all-gather of
    the group's :class:`CustomAllReduce` (written straight into the
    concatenated layout); the rest go to RCCL / gloo."""
    w = get_world_size(group)
    if w == 1:
        return t
    car = _CUSTOM.get(id(group)) if t.is_cuda else None
    if car is not None and car.gather_eligible(t):
        return car.all_gather_last_dim(t)
    parts = [torch.empty_like(t) for _ in range(w)]
    dist.all_gather(parts, t.contiguous(), group=group)
    return torch.cat(parts, dim=-1)


def broadcast_tensor(t: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if is_dist() and get_world_size(group) > 1:
        dist.broadcast(t, src=src, group=group)
    return t


class CustomAllReduce:
    """One-shot peer all-reduce for one intra-node process group.

    Collective constructor: every rank allocates a peer buffer
    ([signal | 2 x data | 2 x result], ``cap`` bytes each), the hipIpc
    handles are all-gathered and opened.  Messages up to 256 KiB take the
    one-shot form, larger ones (up to ``cap``) the two-shot form
    (reduce-scatter + all-gather through the result halves).
    ``__call__`` is capturable in a hipGraph (device-side epochs)."""

    SIGNAL = 8192

    def __init__(self, group=None, device=None, max_bytes: int = 8 << 20):
        from .. import ops
        ops.require()
        self.group = group
        self.world = get_world_size(group)
        self.rank = get_rank(group)
        if self.world > 8:
            raise ValueError("CustomAllReduce supports up to 8 ranks (one xGMI node)")
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise RuntimeError("CustomAllReduce needs all ranks on one node")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.cap = int(max_bytes)
        A = torch.ops.ipex_llm_amd
        with torch.cuda.device(self.device):
            self._own = A.ipc_alloc(self.SIGNAL + 4 * self.cap, PEER_UNCACHED)   # signals | data x2 | result x2
            handle = A.ipc_handle(self._own)
        handles = [None] * self.world
        dist.all_gather_object(handles, handle.tolist(), group=group)
        self._opened = []
        ptrs = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    ptrs.append(self._own)
                else:
                    p = A.ipc_open(torch.tensor(h, dtype=torch.uint8))
                    self._opened.append(p)
                    ptrs.append(p)
        self.ptrs = ptrs
        self.counter = torch.zeros(64, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        barrier(group)

    def eligible(self, t: torch.Tensor) -> bool:
        nb = t.numel() * t.element_size()
        return (t.dtype in (torch.bfloat16, torch.float16, torch.float32) and t.is_contiguous() and nb % 16 == 0
                and 0 < nb <= self.cap and t.device == self.device)

    def gather_eligible(self, t: torch.Tensor) -> bool:
        return (t.dtype in (torch.bfloat16, torch.float16, torch.float32) and t.dim() >= 1
                and (t.shape[-1] * t.element_size()) % 16 == 0 and 0 < t.numel() * t.element_size() <= self.cap
                and t.device == self.device)

    def all_gather_last_dim(self, t: torch.Tensor) -> torch.Tensor:
        """[..., n] on every rank -> [..., W * n] (rank r's block at columns
        r*n..), one launch, capturable"""
        t = t.contiguous()
        out = t.new_empty(*t.shape[:-1], self.world * t.shape[-1])
        torch.ops.ipex_llm_amd.custom_all_gather(t, out, self.ptrs, self.rank, self.counter, self.cap, self.err)
        return out

    def __call__(self, t: torch.Tensor, out: Optional[torch.Tensor] = None, two_shot: int = -1) -> torch.Tensor:
        """sum over the group; ``out`` may alias ``t`` (each block reads its
        slice before it writes it)"""
        out = torch.empty_like(t) if out is None else out
        torch.ops.ipex_llm_amd.custom_all_reduce(t, out, self.ptrs, self.rank, self.counter, self.cap, self.err,
                                                 two_shot)
        return out

    def check(self):
        """raise if a call timed out waiting for a peer (the kernels also set
        ERR_PEER in the device error word: ops.check_kernel_errors raises)"""
        if int(self.err.item()) != 0:
            raise RuntimeError("custom all-reduce timed out waiting for a peer")

    def close(self):
        A = torch.ops.ipex_llm_amd
        torch.cuda.synchronize(self.device)
        barrier(self.group)
        for p in self._opened:
            A.ipc_close(p)
        A.ipc_free(self._own)
        self._opened = []


def setup_custom_all_reduce(group=None, max_bytes: int = 8 << 20) -> Optional[CustomAllReduce]:
    """Collective: create (once) the custom all-reduce for ``group`` if the
    group is intra-node, on GPU and the feature is enabled."""
    if not is_dist() or get_world_size(group) == 1 or not torch.cuda.is_available() or not _custom_enabled():
        return None
    if dist.get_backend(group) != "nccl" and os.environ.get("ILLM_AR_P2P") != "force":
        return None                 # force: also over a gloo group (ranks sharing one GPU: smoke tests)
    key = id(group)
    if key not in _CUSTOM:
        try:
            _CUSTOM[key] = CustomAllReduce(group, max_bytes=max_bytes)
        except RuntimeError:
            return None
    return _CUSTOM[key]
