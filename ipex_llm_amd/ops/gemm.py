"""Prefill-size (M > 64) low-bit GEMM dispatch.

Two paths: the MFMA kernel with in-register dequant (``csrc/hip/gemm.hip``:
f16 MFMA, weights decoded straight from the tiled blob, never
materialised), and dequantize to a transient dense weight + library GEMM
(hipBLASLt).  Measured on MI355X at Llama-3-8B shapes (sym_int4, the fused
kernel with its round-3 128 n x 64 m blocks below M = 1024,
profiles/prefill_gemm_r3_small_tile6.jsonl): the fused kernel wins for the
wide projections (M = 256: qkv 40 vs 53 us, gate_up 93 vs 129; M = 384:
gate_up 130 vs 134) and for every shape at M <= 128 except the long-K down
projection (M = 128: 113 vs 84 us -- its 4096-wide output gives few blocks
for 14336-deep K); the library path wins above (M = 1024: qkv 64.7 vs 82,
o 50 vs 62, gate_up 239 vs 318, down 138 vs 184).
``ILLM_GEMM_LIB=1`` / ``ILLM_GEMM_FUSED=1`` force either path (A/B runs).
"""
from __future__ import annotations

import contextlib
import os
import weakref
from typing import Dict

import torch
import torch.nn.functional as F

_USE_LIB = os.environ.get("ILLM_GEMM_LIB", "0") == "1"
_USE_FUSED = os.environ.get("ILLM_GEMM_FUSED", "0") == "1"
FUSED_MAX_M = 128          # fused kernel for every shape up to here (K <= FUSED_LONG_K)
FUSED_LONG_K = 8192        # deeper K (down projections): library path from M > 64
FUSED_QKV_MAX_M = 256      # N >= 6144 (fused qkv) up to here
FUSED_WIDE_MAX_M = 384     # N >= FUSED_WIDE_N (gate/up pairs) up to here
FUSED_WIDE_N = 12288


def use_fused(M: int, n: int, k: int = 0) -> bool:
    if _USE_LIB:
        return False
    if _USE_FUSED:
        return True
    if k > FUSED_LONG_K:
        return M <= 64
    if n >= FUSED_WIDE_N:
        return M <= FUSED_WIDE_MAX_M
    if n >= 6144:
        return M <= FUSED_QKV_MAX_M
    return M <= FUSED_MAX_M


# ---- dense-weight prefetch for the library path ---------------------------
# The library path's dequantize is memory-bound and the GEMM it feeds is
# compute-bound: the decoder asks for the NEXT layer's dense weights while
# the current layer computes, and they are written on a side HIP stream, so
# the dequant traffic overlaps the MFMA work instead of sitting between the
# GEMMs.  At most one layer's weights are held ahead (consumed entries are
# dropped).  Opt-in (ILLM_GEMM_PREFETCH=1): measured on MI355X (Llama-3-8B,
# 1024-token prompts) the overlapped dequant contends with the GEMMs for HBM
# and CUs -- first token B=1 21.1 -> 22.0 ms, B=8 104.3 -> 103.3 ms.
_PREFETCH = os.environ.get("ILLM_GEMM_PREFETCH", "0") == "1"
_ready = {}                 # (blob ptr, n, k, dtype) -> (dense weight, event)
_side = {}                  # device index -> side stream


def _key(blob, n, k, dtype):
    return (blob.data_ptr(), n, k, dtype)


def prefetch_dense(items, M: int, dtype) -> None:
    """Dequantize ``items`` = [(blob, fmt, n, k)] on a side stream for an
    upcoming library-path GEMM with M rows (no-op for fused-path shapes,
    during graph capture, or when disabled)."""
    if not _PREFETCH or not items or torch.cuda.is_current_stream_capturing():
        return
    ops = torch.ops.ipex_llm_amd
    for blob, fmt, n, k in items:
        if not blob.is_cuda or use_fused(M, n, k):
            continue
        key = _key(blob, n, k, dtype)
        if key in _ready:
            continue
        dev = blob.device.index
        st = _side.get(dev)
        if st is None:
            st = _side[dev] = torch.cuda.Stream(device=blob.device)
        with torch.cuda.stream(st):
            w = ops.dequantize_device(blob, fmt, n, k, dtype)
            ev = torch.cuda.Event()
            ev.record(st)
        _ready[key] = (w, ev)


# ---- resident dense shadow of the low-bit weights for prefill -------------
# Decode streams the low-bit blob (bandwidth-bound); prefill at M >= 512 is
# compute-bound and runs the library GEMM on a dequantized copy that the path
# above re-creates on every call (2 B/weight written and re-read: ~20 % of a
# 1024-token prefill GEMM).  With 288 GB of HBM3E per MI355X the dequantized
# copy can simply stay resident: ILLM_PREFILL_DENSE_GB=<budget> keeps up to
# that many GB of bf16/f16 shadows (first use dequantizes, later prefills
# reuse it; numerics identical to the dequantize-per-call path).  Default 0:
# nothing kept (the low-bit footprint only).
_DENSE_BUDGET = float(os.environ.get("ILLM_PREFILL_DENSE_GB", "0")) * 2 ** 30
_dense_bytes = [0]           # bytes charged to the budget by every resident shadow (incl. training/lora.py's)


class ChargedCache(dict):
    """key -> (weakref to blob, shadow, charged bytes): removing an entry (pop,
    del, clear, the blob's weakref callback) refunds its bytes to the budget"""

    def pop(self, key, *default):
        ent = super().pop(key, None)
        if ent is None:
            return default[0] if default else None
        _dense_bytes[0] -= ent[2]
        # entries of other caches that view this entry's storage (charged 0) go too:
        # a surviving view would keep the bytes alive after their refund
        for c, k in self.__dict__.get("_links", {}).pop(key, ()):
            c.pop(k)
        return ent

    def link(self, key, other: "ChargedCache", okey):
        """drop ``other[okey]`` (a view of this entry's shadow) with ``self[key]``"""
        self.__dict__.setdefault("_links", {}).setdefault(key, []).append((other, okey))

    def __delitem__(self, key):
        self.pop(key)

    def clear(self):
        for k in list(self.keys()):
            self.pop(k)

    def _pop_if(self, key, ref):
        ent = self.get(key)
        if ent is not None and ent[0] is ref:      # a newer entry under a reused address stays
            self.pop(key)

    def put(self, key, blob, w, charged: int):
        self.pop(key)
        super().__setitem__(key, (weakref.ref(blob, lambda r, key=key, c=self: c._pop_if(key, r)), w, charged))
        _dense_bytes[0] += charged


_dense_cache = ChargedCache()  # (blob ptr, version, n, k, dtype) -> (weakref to blob, dense weight, bytes)


def dense_fits(nbytes: int) -> bool:
    """another ``nbytes`` of resident shadow stays within the budget"""
    return _DENSE_BUDGET > 0 and _dense_bytes[0] + nbytes <= _DENSE_BUDGET


# a prefill graph being captured records the addresses of the shadows it reads:
# they are pinned in the graph's own entry (Engine._pf_graphs), so dropping a
# cache entry (budget change, dense_cache_clear) can never free memory a
# captured graph still reads
_capture_pins = None


@contextlib.contextmanager
def pin_dense_shadows():
    global _capture_pins
    prev, _capture_pins = _capture_pins, []
    try:
        yield _capture_pins
    finally:
        _capture_pins = prev


def set_dense_budget(gb: float) -> None:
    """budget (GiB) of dequantized weights kept resident by ``_dense_weight``
    (frozen low-bit weights: the cache never goes stale); 0 disables"""
    global _DENSE_BUDGET
    _DENSE_BUDGET = float(gb) * 2 ** 30
    if _DENSE_BUDGET <= 0:
        dense_cache_clear()


def dense_cache_clear() -> None:
    _dense_cache.clear()


def auto_dense_budget(device, cap_gb: float = float("inf")) -> float:
    """Inference default for the prefill shadow (engine construction): an
    explicit ILLM_PREFILL_DENSE_GB wins; otherwise 0 -- the model keeps its
    low-bit footprint only and prefill dequantizes each weight once per GEMM
    into a transient buffer for the dense 8-phase kernel (``use_g8d``).  A
    resident shadow (ILLM_PREFILL_DENSE_GB=48 on MI355X: a Llama-3-8B INT4
    model adds 15 GB next to its 4.5 GB) saves that ~3-4 % dequant pass;
    ``cap_gb`` bounds an explicit request.  Returns the budget in GiB."""
    env = os.environ.get("ILLM_PREFILL_DENSE_GB")
    gb = min(float(env), cap_gb) if env is not None else 0.0
    if gb * 2 ** 30 > _DENSE_BUDGET:
        set_dense_budget(gb)
    return gb


def _dense_drop(key):
    _dense_cache.pop(key, None)


def _dense_weight(blob, fmt, n, k, dtype):
    if _DENSE_BUDGET > 0:
        # keyed by address, validated by identity: an entry lives exactly as
        # long as its blob (weakref callback), so a later model whose blob
        # reuses the address never sees another model's weights
        key = (blob.data_ptr(), blob._version, n, k, dtype)
        ent = _dense_cache.get(key)
        if ent is not None:
            if ent[0]() is blob:
                if _capture_pins is not None and torch.cuda.is_current_stream_capturing():
                    _capture_pins.append(ent[1])
                return ent[1]
            _dense_drop(key)
        w = torch.ops.ipex_llm_amd.dequantize_device(blob, fmt, n, k, dtype)
        if torch.cuda.is_current_stream_capturing():
            return w                # captured: a transient of the graph's pool, never cached
        nb = w.numel() * w.element_size()
        if dense_fits(nb):
            _dense_cache.put(key, blob, w, nb)
        return w
    hit = _ready.pop(_key(blob, n, k, dtype), None) if _ready else None
    if hit is None:
        return torch.ops.ipex_llm_amd.dequantize_device(blob, fmt, n, k, dtype)
    w, ev = hit
    cur = torch.cuda.current_stream(blob.device)
    cur.wait_event(ev)
    w.record_stream(cur)           # allocated on the side stream, used (and freed) here
    return w


def drop_prefetched() -> None:
    """Release prefetched weights nobody consumed (e.g. an aborted forward)."""
    _ready.clear()


# ---- the 8-phase 256 x 256 GEMM (csrc/hip/gemm_8p.hip): bf16 MFMA, weights
# decoded to bf16 in LDS just in time (bit-identical to dequantize-to-bf16 +
# GEMM), LDS-DMA activations, counted-vmcnt pipeline, staggered wave-rows.
# sym_int4 and the nf4 / nf3 LUT formats; bf16 activations; from G8_MIN_M rows
# (ILLM_GEMM_8P=0 disables it).
_G8 = os.environ.get("ILLM_GEMM_8P", "0") == "1"     # opt-in: 0.6-0.7x dequant + hipBLASLt so far (profiles/gemm8p_sweep_r4.jsonl)
G8_MIN_M = int(os.environ.get("ILLM_GEMM_8P_MIN_M", "1024"))
_G8_FMTS = None


def _g8_fmts():
    global _G8_FMTS
    if _G8_FMTS is None:
        from ..quantize import get_format
        _G8_FMTS = {get_format(q).fmt for q in ("sym_int4", "nf4", "nf3")}
    return _G8_FMTS


def use_g8(x, M: int, n: int, k: int, fmt: int, glu: bool = False) -> bool:
    return (_G8 and not _USE_LIB and not _USE_FUSED and x.is_cuda and x.dtype == torch.bfloat16 and M >= G8_MIN_M
            and k % 128 == 0 and (not glu or n % 32 == 0) and fmt in _g8_fmts() and _DENSE_BUDGET <= 0
            and hasattr(torch.ops.ipex_llm_amd, "gemm8p_lowbit"))


# ---- default prefill path: stream-dequantize + the dense 8-phase GEMM -------
# The in-LDS-dequant kernel above decodes every weight tile once per 256-row
# M block (32 times at M = 8192); on gfx950 that decode (~3.5 VALU per weight)
# competes with the MFMAs for the SIMD's vector issue (an MFMA holds it 8 of
# its 16 cycles) and the kernel runs at ~0.67x of a dense GEMM
# (profiles/g8_sched_sweep_r5.jsonl).  Decoding each weight ONCE into a
# transient bf16 copy (dequantize_device, HBM-bound: ~3-4 % of the GEMM) and
# running the dense 8-phase kernel (gemm_8p.hip: LDS-DMA, counted vmcnt,
# split-K for grids smaller than the chip, GLU in the epilogue) keeps the
# low-bit footprint -- no resident shadow -- and no library GEMM.
# ILLM_GEMM_G8D=0 falls back to dequantize + hipBLASLt (A/B).
_G8D = os.environ.get("ILLM_GEMM_G8D", "1") == "1"
G8D_MIN_M = int(os.environ.get("ILLM_GEMM_G8D_MIN_M", "512"))


def use_g8d(x, M: int, n: int, k: int, glu: bool = False) -> bool:
    return (_G8D and not _USE_LIB and not _USE_FUSED and x.is_cuda and x.dtype == torch.bfloat16
            and M >= G8D_MIN_M and k % 64 == 0 and (not glu or n % 32 == 0)
            and hasattr(torch.ops.ipex_llm_amd, "gemm_bf16"))


# ---- measured dispatch: dense 8-phase kernel vs the library GEMM -----------
# Over the same transient bf16 weight, the 8-phase kernel reaches 0.8-0.9x
# hipBLASLt at M = 8192 and 0.5-0.8x at M = 1024 (profiles/g8d_slab_splitk_sweep_r5.jsonl);
# end to end the library path took the Llama-3-8B first token from 98.9 to 90.3 ms
# at B = 8 x 1024 and 19.8 to 18.5 ms at B = 1 (profiles/prefill_lib_ab_r6.jsonl).
# Each (M, N, K, GLU) shape times both once, outside graph capture (the engine's
# eager warm-up precedes every prefill capture), and keeps the faster; a shape first
# seen under capture takes the 8-phase kernel.  ILLM_GEMM_AUTOTUNE=0: always 8-phase.
_AUTOTUNE = os.environ.get("ILLM_GEMM_AUTOTUNE", "1") == "1"
_CHOICE: Dict[tuple, str] = {}


def _time_ms(fn, reps: int = 3) -> float:
    fn()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    t1.synchronize()
    return t0.elapsed_time(t1) / reps


def _mbucket(M: int) -> int:
    """rows rounded up to a power of two: serving sees every prompt length, and one
    timing per bucket keeps the table (and the warm-up cost) bounded"""
    return 1 << max(0, int(M) - 1).bit_length()


def _pick(key: tuple, g8d_fn, lib_fn, *more) -> str:
    """'g8d' | 'lib' | 'lib1' ... (the extra candidates ``more``, in order);
    key = (M, N, K, kind, act), M bucketed"""
    key = (_mbucket(key[0]),) + tuple(key[1:])
    c = _CHOICE.get(key)
    if c is None:
        if not _AUTOTUNE or torch.cuda.is_current_stream_capturing():
            return "g8d"
        names = ["g8d", "lib"] + [f"lib{i + 1}" for i in range(len(more))]
        times = [_time_ms(f) for f in (g8d_fn, lib_fn) + more]
        c = _CHOICE[key] = names[min(range(len(times)), key=times.__getitem__)]
        if os.environ.get("ILLM_GEMM_AUTOTUNE_LOG"):
            print(f"[gemm] M={key[0]} N={key[1]} K={key[2]} glu={key[3]}: "
                  + ", ".join(f"{n} {t * 1e3:.1f} us" for n, t in zip(names, times)) + f" -> {c}", flush=True)
    return c


def gemm_choices() -> Dict[tuple, str]:
    """the measured per-shape choices so far: (M, N, K, glu, act) -> 'g8d' | 'lib'"""
    return dict(_CHOICE)


def lowbit_gemm(x, blob, fmt, n, k, bias=None):
    ops = torch.ops.ipex_llm_amd
    M = x.numel() // k
    bf16_bias = bias is None or bias.dtype == torch.bfloat16
    if use_g8(x, M, n, k, fmt) and bf16_bias:
        return ops.gemm8p_lowbit(x, blob, fmt, n, k, bias)
    if use_g8d(x, M, n, k) and bf16_bias:
        # candidates timed with their weight preparation: the 8-phase kernel and
        # the library over the transient bf16 weight.  (The in-LDS low-bit
        # 8-phase kernel, no transient weight, lost every Llama-3-8B prefill shape
        # as a third candidate: 0.55-0.85x, profiles/prefill_choices_b{1,8}_r6.txt.)
        def dw():
            return _dense_weight(blob, fmt, n, k, x.dtype)
        c = _pick((M, n, k, False, 0), lambda: ops.gemm_bf16(x, dw(), bias), lambda: F.linear(x, dw(), bias))
        return F.linear(x, dw(), bias) if c == "lib" else ops.gemm_bf16(x, dw(), bias)
    if use_fused(M, n, k) and hasattr(ops, "gemm"):
        return ops.gemm(x, blob, fmt, n, k, bias)
    w = _dense_weight(blob, fmt, n, k, x.dtype)
    return F.linear(x, w, bias)


def lowbit_gemm_glu(x, blob, fmt, n, k, act: int = 0):
    """act(x @ Wg^T) * (x @ Wu^T) for a tile-interleaved gate/up weight at
    prefill M: the fused kernel applies the activation in its epilogue (no
    [M, 2I] round trip, no elementwise launches)."""
    ops = torch.ops.ipex_llm_amd
    M = x.numel() // k
    if use_g8(x, M, n, k, fmt, glu=True):
        return ops.gemm8p_lowbit(x, blob, fmt, n, k, None, False, True, act)
    if use_g8d(x, M, n, k, glu=True) and act in (0, 1):
        from .api import glu

        def dw():
            return _dense_weight(blob, fmt, n, k, x.dtype)

        def lib():
            return glu(F.linear(x, dw()), act, tile=16)
        c = _pick((M, n, k, True, act), lambda: ops.gemm_bf16(x, dw(), None, False, 0, True, act), lib)
        return lib() if c == "lib" else ops.gemm_bf16(x, dw(), None, False, 0, True, act)
    if use_fused(M, n, k) and hasattr(ops, "gemm_glu"):
        return ops.gemm_glu(x, blob, fmt, n, k, act)
    from .api import glu
    return glu(lowbit_gemm(x, blob, fmt, n, k), act, tile=16)
