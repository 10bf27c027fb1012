"""Data-parallel fine-tuning over RCCL (one process per GPU).

Reference: HF Trainer DDP with ``ddp_backend="ccl"``
(``alpaca_qlora_finetuning.py:156-160, 263-269``): torch DDP over oneCCL.

Two ways in here:

* :func:`wrap_ddp` -- torch ``DistributedDataParallel`` with a bucket size
  chosen for xGMI rings (see below).
* :class:`GradBucketSync` -- a gradient synchroniser written for the QLoRA
  case, where only the adapters train: every trainable gradient lives in ONE
  flat buffer per dtype (``p.grad`` are views into it, so no copy in or out),
  the buffer is cut into buckets in reverse registration order (the order
  backward produces them), and a bucket's all-reduce is issued the moment its
  last gradient has been accumulated (``register_post_accumulate_grad_hook``),
  asynchronously, so the collectives overlap the rest of backward.  The 1/world
  average is folded in before the reduce (one in-place scale per bucket, no
  extra pass after it).  ``finish()`` waits on the outstanding work before the
  optimizer step.

Bucket size on MI355X: ring all-reduce over point-to-point xGMI is link-bound
(7 links x ~153 GB/s per GPU); a bucket must be large enough that the ring's
2(W-1) latency-bound steps are amortised (tens of MB), and LoRA gradients are
small (Llama-3-8B r=8 on 7 projections: 21M params, 42 MB in bf16), so the
default 32 MB gives two buckets: the first overlaps backward, the second the
tail.  Works with any torch.distributed backend (nccl = RCCL on ROCm; gloo on
CPU for tests).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def wrap_ddp(model: nn.Module, device_ids=None, bucket_cap_mb: float = 32.0, **kwargs) -> nn.Module:
    """torch DDP with an xGMI-sized bucket and gradients as bucket views."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    if device_ids is None and torch.cuda.is_available() and next(model.parameters()).is_cuda:
        device_ids = [torch.cuda.current_device()]
    return DDP(model, device_ids=device_ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
               find_unused_parameters=kwargs.pop("find_unused_parameters", False), **kwargs)


class _Bucket:
    __slots__ = ("flat", "params", "pending", "work")

    def __init__(self, flat: torch.Tensor, params: List[nn.Parameter]):
        self.flat = flat
        self.params = params
        self.pending = len(params)
        self.work = None


class GradBucketSync:
    """Bucketed, backward-overlapped gradient all-reduce for the trainable
    parameters of ``model`` (see the module docstring).

    Usage::

        sync = GradBucketSync(model)          # after get_peft_model, before the optimizer
        sync.broadcast_parameters()           # identical adapters on every rank
        for batch in data:
            loss = model(**batch).loss
            loss.backward()                   # buckets reduce as their grads complete
            sync.finish()                     # wait for the last buckets
            opt.step(); sync.zero_grad()

    Gradient accumulation (the reference recipe's
    ``gradient_accumulation_steps``): run every micro-batch but the last
    under ``with sync.no_sync():`` -- its gradients accumulate locally in the
    flat buffer and no collective is issued; the last backward reduces the
    accumulated sum.  A second backward outside ``no_sync`` before
    ``finish()`` would add into buffers whose all-reduce is in flight, so it
    raises instead.
    """

    def __init__(self, model: nn.Module, group=None, bucket_cap_mb: float = 32.0, average: bool = True):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.average = average
        self.params = [p for p in model.parameters() if p.requires_grad]
        # backward produces gradients roughly in reverse registration order
        order = list(reversed(self.params))
        cap = int(bucket_cap_mb * 2 ** 20)
        self.buckets: List[_Bucket] = []
        self._of: Dict[int, _Bucket] = {}
        by_key: Dict[tuple, List[nn.Parameter]] = {}
        for p in order:
            by_key.setdefault((p.device, p.dtype), []).append(p)
        self._flats = []
        for (dev, dt), ps in by_key.items():
            flat = torch.zeros(sum(p.numel() for p in ps), dtype=dt, device=dev)
            self._flats.append(flat)
            off, start, cur, cur_bytes = 0, 0, [], 0
            for p in ps:
                n = p.numel()
                p.grad = flat[off:off + n].view_as(p)            # gradient lives in the flat buffer
                cur.append(p)
                off += n
                cur_bytes += n * flat.element_size()
                if cur_bytes >= cap:
                    self._add_bucket(flat[start:off], cur)
                    start, cur, cur_bytes = off, [], 0
            if cur:
                self._add_bucket(flat[start:off], cur)
        self._hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]
        self._sync = True

    class _NoSync:
        def __init__(self, owner):
            self.owner = owner

        def __enter__(self):
            self.owner._check_idle("no_sync()")
            self.owner._sync = False
            return self.owner

        def __exit__(self, *exc):
            self.owner._sync = True
            return False

    def no_sync(self):
        """Context for accumulation micro-batches: gradients accumulate in the
        flat buffer, no bucket is reduced (the next synced backward reduces
        the sum)."""
        return GradBucketSync._NoSync(self)

    def _check_idle(self, what):
        if any(b.work is not None or b.pending != len(b.params) for b in self.buckets):
            raise RuntimeError(f"GradBucketSync: {what} while a synced backward is in flight; call finish() first")

    def _add_bucket(self, flat, params):
        b = _Bucket(flat, params)
        self.buckets.append(b)
        for p in params:
            self._of[id(p)] = b

    def _ready(self, p: nn.Parameter):
        b = self._of.get(id(p))
        if b is None or not self._sync:
            return
        if b.pending <= 0 or b.work is not None:
            raise RuntimeError("GradBucketSync: a second backward reached a bucket whose all-reduce is already "
                               "issued; wrap accumulation micro-batches in no_sync() and call finish() per step")
        if p.grad is not None and p.grad.data_ptr() != b.flat.data_ptr() and not self._is_view(p, b):
            # autograd replaced the gradient tensor (e.g. set_to_none zero_grad): copy it back in
            self._rebind(p, b)
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    @staticmethod
    def _is_view(p, b):
        g = p.grad
        base = b.flat.data_ptr()
        end = base + b.flat.numel() * b.flat.element_size()
        return g is not None and base <= g.data_ptr() < end

    def _rebind(self, p, b):
        off = 0
        for q in b.params:
            n = q.numel()
            if q is p:
                view = b.flat[off:off + n].view_as(p)
                view.copy_(p.grad)
                p.grad = view
                return
            off += n

    def _launch(self, b: _Bucket):
        if self.world == 1:
            return
        if self.average:
            b.flat.div_(self.world)
        b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket's all-reduce (buckets whose gradients never
        arrived this step, e.g. frozen-by-LISA layers, are reduced now so all
        ranks issue the same collectives)."""
        for b in self.buckets:
            if b.pending > 0:
                b.pending = 0
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
            b.pending = len(b.params)

    def zero_grad(self):
        for f in self._flats:
            f.zero_()

    @torch.no_grad()
    def broadcast_parameters(self, src: int = 0):
        if self.world == 1:
            return
        for p in self.params:
            dist.broadcast(p.data, src=src, group=self.group)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
