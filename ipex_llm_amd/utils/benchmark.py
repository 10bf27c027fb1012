"""BenchmarkWrapper: first-token / next-token latency of ``generate``.

Reference: ``SRC/utils/benchmark_util_4_47.py`` (a full copy of HF
``generate`` per transformers version, timing each step with
``xpu.synchronize``: ``first_cost``, ``rest_cost_mean``, ``encoder_time``,
``peak_memory``) and the all-in-one CSV columns (``run.py:596-600``).

The native engine already records per-step times (HIP-synchronised) for
every ``generate`` call, so the wrapper only forwards and collects them --
no copied generate loop.  For models without the native path it times
``generate`` with a streamer hook.
"""
from __future__ import annotations

import csv
import os
import time
from typing import Dict, List, Optional

import torch


class _StepTimer:
    """streamer that timestamps every emitted step"""

    def __init__(self, sync):
        self.sync, self.t = sync, []

    def put(self, value):
        self.sync()
        self.t.append(time.perf_counter())

    def end(self):
        pass


class BenchmarkWrapper:
    def __init__(self, model, do_print: bool = False, verbose: bool = False):
        self.model, self.do_print, self.verbose = model, do_print, verbose
        self.first_cost = 0.0
        self.rest_cost_mean = 0.0
        self.encoder_time = 0.0
        self.peak_memory = 0.0

    def __getattr__(self, name):
        return getattr(self.model, name)

    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def _sync(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def generate(self, *args, **kwargs):
        if torch.cuda.is_available():
            torch.cuda.reset_peak_memory_stats()
        native = getattr(self.model, "_illm_native_attached", False)
        if native and "streamer" not in kwargs:
            out = self.model.generate(*args, **kwargs)
            self.first_cost = float(getattr(self.model, "first_cost", 0.0))
            self.rest_cost_mean = float(getattr(self.model, "rest_cost_mean", 0.0))
        else:
            st = _StepTimer(self._sync)
            self._sync()
            t0 = time.perf_counter()
            st.t.append(t0)
            out = self.model.generate(*args, streamer=st, **kwargs)
            ts = st.t
            # first put() is the prompt for HF streamers, then one per step
            steps = [b - a for a, b in zip(ts[:-1], ts[1:])]
            if len(steps) >= 2 and steps[0] < 1e-3:
                steps = [steps[0] + steps[1]] + steps[2:]
            self.first_cost = steps[0] if steps else 0.0
            rest = steps[1:]
            self.rest_cost_mean = sum(rest) / len(rest) if rest else 0.0
        if torch.cuda.is_available():
            self.peak_memory = torch.cuda.max_memory_reserved() / 2 ** 30
        if self.do_print:
            print(f"=========First token cost {self.first_cost:.4f} s=========")
            print(f"=========Rest tokens cost average {self.rest_cost_mean:.4f} s "
                  f"({max(0, (out.shape[1] if hasattr(out, 'shape') else 0))} tokens out)=========")
            if self.verbose:
                print(f"=========Peak memory {self.peak_memory:.2f} GB=========")
        return out


CSV_COLUMNS = ["model", "1st token avg latency (ms)", "2+ avg latency (ms/token)", "encoder time (ms)",
               "input/output tokens", "batch_size", "actual input/output tokens", "num_beams", "low_bit",
               "cpu_embedding", "model loading time (s)", "peak mem (GB)", "streaming", "use_fp16_torch_dtype"]


def append_csv(path: str, rows: List[Dict]):
    """all-in-one-compatible CSV sink (reference run.py:596-600 columns)"""
    new = not os.path.exists(path)
    with open(path, "a", newline="") as f:
        w = csv.DictWriter(f, fieldnames=CSV_COLUMNS, extrasaction="ignore")
        if new:
            w.writeheader()
        for r in rows:
            w.writerow(r)
