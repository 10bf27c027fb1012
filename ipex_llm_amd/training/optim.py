"""AdamW with a single fused multi-tensor HIP launch per parameter group.

The reference's trainers use torch AdamW (``qlora.py`` ``TrainingArguments``
whitelists ``adamw_torch``/``adamw_hf``...).  LoRA fine-tuning has many
tiny adapter tensors, so :class:`FusedAdamW` updates all of a group's
params/moments in ONE kernel (``csrc/hip/optim.hip``: chunk table ->
workgroups, f32 moments, bf16 or f32 params).  On CPU it runs the same
math with torch ``_foreach`` ops.  Semantics = ``torch.optim.AdamW``
(decoupled weight decay, bias correction).

``capturable=True`` keeps the step count and learning rate of each group in a
device tensor and the pointer/chunk tables cached, so ``step()`` issues no
host-to-device copy and can be captured in a hipGraph together with the
forward and backward (tools/bench_qlora.py --graph).  After changing
``group["lr"]`` call :meth:`sync_lr` (outside capture).  The device step is
mirrored into ``state[p]["step"]`` by :meth:`state_dict` and re-seeded from
it after :meth:`load_state_dict` (checkpoint / resume keeps the bias
correction), and switching between capturable and eager steps carries it.
"""
from __future__ import annotations

import math
from typing import Iterable

import torch

from .. import ops

CHUNK = 16384


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, capturable: bool = False):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.capturable = capturable
        self._tables = {}          # (device, dtype, ptrs) -> (table, chunk_tensor, chunk_start)
        self._step_lr = {}         # group index -> f32 [2] (step, lr) on the device

    def sync_lr(self):
        """copy each group's current ``lr`` into its device (step, lr) pair"""
        for gi, group in enumerate(self.param_groups):
            sl = self._step_lr.get(gi)
            if sl is not None:
                sl[1].fill_(float(group["lr"]))

    def _dev_step_lr(self, gi, group, dev, host_step: int = 0):
        sl = self._step_lr.get(gi)
        if sl is None or sl.device != dev:
            sl = torch.tensor([float(host_step), float(group["lr"])], dtype=torch.float32, device=dev)
            self._step_lr[gi] = sl
        return sl

    def _sync_host_steps(self):
        """copy every device step count into the per-parameter state (one
        host read per group; outside capture)"""
        for gi, sl in self._step_lr.items():
            step = int(round(float(sl[0].item())))
            for p in self.param_groups[gi]["params"]:
                st = self.state.get(p)
                if st:
                    st["step"] = step

    def state_dict(self):
        self._sync_host_steps()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._step_lr.clear()                  # re-seeded from state["step"] by the next capturable step
        self._tables.clear()

    def _state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = 0
            st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
            st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self._step_lr and not self.capturable:
            self._sync_host_steps()            # switched from capturable steps: continue the count
            self._step_lr.clear()
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            b1, b2 = group["betas"]
            sts = [self._state(p) for p in ps]
            if self.capturable and all(p.is_cuda for p in ps) and ops.native_gpu(ps[0]):
                sl = self._dev_step_lr(gi, group, ps[0].device, host_step=int(sts[0]["step"]))
                sl[0:1].add_(1.0)               # device-side step count (captured with the update)
                self._fused(group, ps, sts, 0.0, 0.0, step_lr=sl)
                continue
            for s in sts:
                s["step"] += 1
            step = sts[0]["step"]
            bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
            gpu = [i for i, p in enumerate(ps) if p.is_cuda and p.is_contiguous() and p.grad.is_contiguous()
                   and p.dtype in (torch.float32, torch.bfloat16) and p.grad.dtype == p.dtype]
            if gpu and ops.native_gpu(ps[gpu[0]]):
                self._fused(group, [ps[i] for i in gpu], [sts[i] for i in gpu], bc1, bc2)
                rest = [i for i in range(len(ps)) if i not in set(gpu)]
            else:
                rest = list(range(len(ps)))
            for i in rest:
                self._ref(group, ps[i], sts[i], bc1, bc2)
        return loss

    def _fused(self, group, ps, sts, bc1, bc2, step_lr=None):
        b1, b2 = group["betas"]
        by_dtype = {}
        for p, s in zip(ps, sts):
            by_dtype.setdefault((p.device, p.dtype), []).append((p, s))
        for (dev, dt), items in by_dtype.items():
            rows = [[p.data_ptr() for p, _ in items], [p.grad.data_ptr() for p, _ in items],
                    [s["exp_avg"].data_ptr() for _, s in items], [s["exp_avg_sq"].data_ptr() for _, s in items],
                    [p.numel() for p, _ in items]]
            key = (dev, dt, tuple(tuple(r) for r in rows))
            cached = self._tables.get(key) if step_lr is not None else None
            if cached is None:
                table = torch.tensor(rows, dtype=torch.int64).to(dev, non_blocking=True)
                ct, cs = [], []
                for ti, (p, _) in enumerate(items):
                    for st in range(0, p.numel(), CHUNK):
                        ct.append(ti)
                        cs.append(st)
                chunk_tensor = torch.tensor(ct, dtype=torch.int32).to(dev, non_blocking=True)
                chunk_start = torch.tensor(cs, dtype=torch.int64).to(dev, non_blocking=True)
                cached = (table, chunk_tensor, chunk_start)
                if step_lr is not None:
                    self._tables[key] = cached
            table, chunk_tensor, chunk_start = cached
            pd = 0 if dt == torch.float32 else 1
            torch.ops.ipex_llm_amd.fused_adamw(table, chunk_tensor, chunk_start, CHUNK, group["lr"], b1, b2,
                                               group["eps"], group["weight_decay"], bc1, bc2, 1.0, pd, pd, step_lr)

    @staticmethod
    def _ref(group, p, s, bc1, bc2):
        b1, b2 = group["betas"]
        g = p.grad.float()
        pf = p.float()
        pf.mul_(1 - group["lr"] * group["weight_decay"])
        s["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
        s["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (s["exp_avg_sq"] / bc2).sqrt_().add_(group["eps"])
        pf.addcdiv_(s["exp_avg"], denom, value=-group["lr"] / bc1)
        p.copy_(pf)
