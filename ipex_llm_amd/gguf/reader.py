"""Pure-Python GGUF (v2/v3) reader and writer with vectorized dequantizers.

Reference: ``SRC/transformers/gguf/gguf.py:31-424`` (header, key/values,
tensor infos, dequantization of f32/f16/q4_0/q4_1/q5_0/q5_1/q8_0/q6_k).
Here the tensor data is memory-mapped (a 70B GGUF is never read whole) and
every block format is dequantized with numpy array ops, including the
k-quants q4_k / q5_k / q6_k used by the common Q4_K_M / Q5_K_M files.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Any, Dict, List, Tuple

import numpy as np

GGUF_MAGIC = b"GGUF"

# ggml tensor types
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 0, 1, 2, 3, 6, 7, 8, 9
Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 10, 11, 12, 13, 14, 15
BF16 = 30
# (elements per block, bytes per block)
BLOCK = {F32: (1, 4), F16: (1, 2), BF16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q5_0: (32, 22), Q5_1: (32, 24),
         Q8_0: (32, 34), Q2_K: (256, 84), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210)}
TYPE_NAMES = {F32: "F32", F16: "F16", BF16: "BF16", Q4_0: "Q4_0", Q4_1: "Q4_1", Q5_0: "Q5_0", Q5_1: "Q5_1",
              Q8_0: "Q8_0", Q2_K: "Q2_K", Q4_K: "Q4_K", Q5_K: "Q5_K", Q6_K: "Q6_K"}

# key/value types
(T_U8, T_I8, T_U16, T_I16, T_U32, T_I32, T_F32, T_BOOL, T_STR, T_ARR, T_U64, T_I64, T_F64) = range(13)
_SCALAR = {T_U8: "<B", T_I8: "<b", T_U16: "<H", T_I16: "<h", T_U32: "<I", T_I32: "<i", T_F32: "<f",
           T_BOOL: "<?", T_U64: "<Q", T_I64: "<q", T_F64: "<d"}


@dataclass
class TensorInfo:
    name: str
    shape: Tuple[int, ...]        # GGUF order: ne[0] (fastest) first
    ggml_type: int
    offset: int

    @property
    def numel(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n

    @property
    def nbytes(self) -> int:
        be, bb = BLOCK[self.ggml_type]
        return self.numel // be * bb


class GGUFReader:
    def __init__(self, path: str):
        self.path = path
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        self.pos = 0
        if bytes(self.mm[:4]) != GGUF_MAGIC:
            raise ValueError(f"{path}: not a GGUF file")
        self.pos = 4
        self.version = self._u32()
        if self.version not in (2, 3):
            raise ValueError(f"GGUF version {self.version} not supported")
        n_tensors, n_kv = self._u64(), self._u64()
        self.kv: Dict[str, Any] = {}
        for _ in range(n_kv):
            k = self._str()
            self.kv[k] = self._value(self._u32())
        self.tensors: Dict[str, TensorInfo] = {}
        for _ in range(n_tensors):
            name = self._str()
            nd = self._u32()
            shape = tuple(self._u64() for _ in range(nd))
            t = self._u32()
            off = self._u64()
            self.tensors[name] = TensorInfo(name, shape, t, off)
        align = int(self.kv.get("general.alignment", 32))
        self.data_start = (self.pos + align - 1) // align * align

    # ---- primitive readers
    def _take(self, n):
        b = self.mm[self.pos:self.pos + n]
        self.pos += n
        return bytes(b)

    def _u32(self):
        return struct.unpack("<I", self._take(4))[0]

    def _u64(self):
        return struct.unpack("<Q", self._take(8))[0]

    def _str(self):
        return self._take(self._u64()).decode("utf-8", errors="replace")

    def _value(self, t):
        if t in _SCALAR:
            fmt = _SCALAR[t]
            return struct.unpack(fmt, self._take(struct.calcsize(fmt)))[0]
        if t == T_STR:
            return self._str()
        if t == T_ARR:
            it, n = self._u32(), self._u64()
            if it in _SCALAR and it != T_BOOL:
                dt = np.dtype(_SCALAR[it])
                arr = np.frombuffer(self._take(n * dt.itemsize), dtype=dt)
                return arr.tolist()
            return [self._value(it) for _ in range(n)]
        raise ValueError(f"unknown GGUF value type {t}")

    # ---- tensors
    def raw(self, name: str) -> np.ndarray:
        ti = self.tensors[name]
        s = self.data_start + ti.offset
        return self.mm[s:s + ti.nbytes]

    def tensor(self, name: str) -> np.ndarray:
        """dequantized float32 array in torch order (shape reversed: [..., ne1, ne0])"""
        ti = self.tensors[name]
        flat = dequantize(self.raw(name), ti.ggml_type, ti.numel)
        return flat.reshape(tuple(reversed(ti.shape)))

    @property
    def architecture(self) -> str:
        return self.kv.get("general.architecture", "llama")


# ------------------------------------------------------------------ dequant
def _f16(b: np.ndarray) -> np.ndarray:
    return b.copy().view(np.float16).astype(np.float32)


def dequantize(raw: np.ndarray, t: int, n: int) -> np.ndarray:
    if t == F32:
        return raw.view(np.float32)[:n].astype(np.float32)
    if t == F16:
        return raw.view(np.float16)[:n].astype(np.float32)
    if t == BF16:
        return (raw.view(np.uint16)[:n].astype(np.uint32) << 16).view(np.float32)
    be, bb = BLOCK[t]
    blk = raw[: n // be * bb].reshape(-1, bb)
    if t == Q4_0:
        d = _f16(blk[:, 0:2])
        qs = blk[:, 2:18]
        q = np.concatenate([qs & 0xF, qs >> 4], 1).astype(np.float32) - 8
        return (q * d).reshape(-1)
    if t == Q4_1:
        d, m = _f16(blk[:, 0:2]), _f16(blk[:, 2:4])
        qs = blk[:, 4:20]
        q = np.concatenate([qs & 0xF, qs >> 4], 1).astype(np.float32)
        return (q * d + m).reshape(-1)
    if t in (Q5_0, Q5_1):
        o = 2 if t == Q5_0 else 4
        d = _f16(blk[:, 0:2])
        m = _f16(blk[:, 2:4]) if t == Q5_1 else 0.0
        qh = blk[:, o:o + 4].copy().view(np.uint32)                      # [nb, 1]
        qs = blk[:, o + 4:o + 20]
        j = np.arange(16, dtype=np.uint32)
        hi0 = ((qh >> j) & 1).astype(np.uint8) << 4
        hi1 = ((qh >> (j + 16)) & 1).astype(np.uint8) << 4
        q = np.concatenate([(qs & 0xF) | hi0, (qs >> 4) | hi1], 1).astype(np.float32)
        if t == Q5_0:
            q -= 16
        return (q * d + m).reshape(-1)
    if t == Q8_0:
        d = _f16(blk[:, 0:2])
        q = blk[:, 2:34].copy().view(np.int8).astype(np.float32)
        return (q * d).reshape(-1)
    if t in (Q4_K, Q5_K):
        d, dmin = _f16(blk[:, 0:2]), _f16(blk[:, 2:4])
        sc, mn = _k_scales(blk[:, 4:16])                                   # [nb, 8] each
        if t == Q4_K:
            qs = blk[:, 16:144].reshape(-1, 4, 32)                         # 4 x 32 bytes -> 8 sub-blocks of 32
            q = np.stack([qs & 0xF, qs >> 4], 2).reshape(-1, 8, 32).astype(np.float32)
        else:
            qh = blk[:, 16:48]                                             # [nb, 32]
            qs = blk[:, 48:176].reshape(-1, 4, 32)
            lo = np.stack([qs & 0xF, qs >> 4], 2).reshape(-1, 8, 32)
            bits = ((qh[:, None, :] >> np.arange(8, dtype=np.uint8)[None, :, None]) & 1) << 4   # [nb, 8, 32]
            q = (lo | bits).astype(np.float32)
        x = d[:, :, None] * sc[:, :, None] * q - dmin[:, :, None] * mn[:, :, None]
        return x.reshape(-1)
    if t == Q6_K:
        ql = blk[:, 0:128]
        qh = blk[:, 128:192]
        sc = blk[:, 192:208].copy().view(np.int8).astype(np.float32)      # [nb, 16]
        d = _f16(blk[:, 208:210])
        out = np.empty((blk.shape[0], 256), dtype=np.float32)
        for half in range(2):
            l = ql[:, 64 * half:64 * half + 64]
            h = qh[:, 32 * half:32 * half + 32]
            q1 = ((l[:, 0:32] & 0xF) | (((h >> 0) & 3) << 4)).astype(np.int32) - 32
            q2 = ((l[:, 32:64] & 0xF) | (((h >> 2) & 3) << 4)).astype(np.int32) - 32
            q3 = ((l[:, 0:32] >> 4) | (((h >> 4) & 3) << 4)).astype(np.int32) - 32
            q4 = ((l[:, 32:64] >> 4) | (((h >> 6) & 3) << 4)).astype(np.int32) - 32
            s = sc[:, 8 * half:8 * half + 8]
            base = 128 * half
            idx = np.arange(32)
            for qi, q in enumerate((q1, q2, q3, q4)):
                isc = s[:, 2 * qi + idx // 16]                             # scale per 16 elements
                out[:, base + 32 * qi:base + 32 * qi + 32] = d * isc * q
        return out.reshape(-1)
    if t == Q2_K:                       # C++ decoder (csrc/cpu/kquant.cpp), same block layout
        import torch
        from .. import ops
        from ..quantize import qtypes as Qt
        nb = blk.shape[0]
        return ops.kq_dequantize(torch.from_numpy(np.ascontiguousarray(blk).reshape(-1)), Qt.FMT_Q2K, nb,
                                 256).numpy().reshape(-1)
    raise NotImplementedError(f"GGUF tensor type {TYPE_NAMES.get(t, t)} is not supported")


# GGUF k-quant type -> our native qtype name (blocks used as-is, quantize/qtypes.py)
KQUANT_QTYPE = {Q2_K: "q2_k", Q4_K: "q4_k", Q5_K: "q5_k", Q6_K: "q6_k"}


def _k_scales(s: np.ndarray):
    """12 packed bytes -> 8 six-bit scales and 8 six-bit mins (q4_K / q5_K)"""
    s = s.astype(np.uint8)
    sc = np.empty((s.shape[0], 8), dtype=np.float32)
    mn = np.empty((s.shape[0], 8), dtype=np.float32)
    for j in range(8):
        if j < 4:
            sc[:, j] = s[:, j] & 63
            mn[:, j] = s[:, j + 4] & 63
        else:
            sc[:, j] = (s[:, j + 4] & 0xF) | ((s[:, j - 4] >> 6) << 4)
            mn[:, j] = (s[:, j + 4] >> 4) | ((s[:, j] >> 6) << 4)
    return sc, mn


# ------------------------------------------------------------------ writer
def quantize_q8_0(x: np.ndarray) -> bytes:
    b = x.reshape(-1, 32).astype(np.float32)
    amax = np.abs(b).max(1, keepdims=True)
    d = amax / 127.0
    q = np.where(d > 0, np.round(b / np.where(d > 0, d, 1)), 0).astype(np.int8)
    out = np.empty((b.shape[0], 34), dtype=np.uint8)
    out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q.view(np.uint8)
    return out.tobytes()


def quantize_q4_0(x: np.ndarray) -> bytes:
    b = x.reshape(-1, 32).astype(np.float32)
    idx = np.abs(b).argmax(1)
    vmax = b[np.arange(b.shape[0]), idx][:, None]
    d = vmax / -8.0
    inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0)
    q = np.clip(np.floor(b * inv + 8.5), 0, 15).astype(np.uint8)
    out = np.empty((b.shape[0], 18), dtype=np.uint8)
    out[:, 0:2] = d.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q[:, :16] | (q[:, 16:] << 4)
    return out.tobytes()


class GGUFWriter:
    """Minimal GGUF v3 writer (metadata + F32/F16/Q8_0/Q4_0 and the
    Q2_K/Q4_K/Q5_K/Q6_K k-quant tensors, the latter by the C++ quantizer)."""

    def __init__(self, path: str, arch: str = "llama"):
        self.path, self.kv, self.tensors = path, {"general.architecture": (T_STR, arch)}, []

    def add(self, key: str, value, vtype: int = None):
        if vtype is None:
            vtype = T_STR if isinstance(value, str) else T_BOOL if isinstance(value, bool) else \
                T_U32 if isinstance(value, int) else T_F32 if isinstance(value, float) else T_ARR
        self.kv[key] = (vtype, value)

    def add_tensor(self, name: str, arr: np.ndarray, ggml_type: int = F32):
        arr = np.ascontiguousarray(arr, dtype=np.float32)
        if ggml_type == F32:
            data = arr.tobytes()
        elif ggml_type == F16:
            data = arr.astype(np.float16).tobytes()
        elif ggml_type == Q8_0:
            data = quantize_q8_0(arr)
        elif ggml_type == Q4_0:
            data = quantize_q4_0(arr)
        elif ggml_type in KQUANT_QTYPE:
            import torch
            from .. import ops
            from ..quantize import qtypes as Qt
            fmt = Qt.get_format(KQUANT_QTYPE[ggml_type]).fmt
            data = ops.kq_quantize(torch.from_numpy(arr.reshape(-1, arr.shape[-1])), fmt).numpy().tobytes()
        else:
            raise NotImplementedError(TYPE_NAMES.get(ggml_type, ggml_type))
        self.tensors.append((name, tuple(reversed(arr.shape)), ggml_type, data))

    @staticmethod
    def _s(s: str) -> bytes:
        b = s.encode()
        return struct.pack("<Q", len(b)) + b

    def _val(self, t, v) -> bytes:
        if t == T_STR:
            return self._s(v)
        if t == T_ARR:
            items = list(v)
            if items and isinstance(items[0], str):
                return struct.pack("<IQ", T_STR, len(items)) + b"".join(self._s(x) for x in items)
            if items and isinstance(items[0], float):
                return struct.pack("<IQ", T_F32, len(items)) + np.asarray(items, np.float32).tobytes()
            return struct.pack("<IQ", T_I32, len(items)) + np.asarray(items, np.int32).tobytes()
        return struct.pack(_SCALAR[t], v)

    def write(self):
        align = 32
        head = GGUF_MAGIC + struct.pack("<IQQ", 3, len(self.tensors), len(self.kv))
        for k, (t, v) in self.kv.items():
            head += self._s(k) + struct.pack("<I", t) + self._val(t, v)
        off = 0
        infos = b""
        offsets = []
        for name, shape, t, data in self.tensors:
            offsets.append(off)
            infos += self._s(name) + struct.pack("<I", len(shape)) + b"".join(struct.pack("<Q", d) for d in shape)
            infos += struct.pack("<IQ", t, off)
            off += (len(data) + align - 1) // align * align
        with open(self.path, "wb") as f:
            f.write(head + infos)
            pad = (-f.tell()) % align
            f.write(b"\0" * pad)
            for (name, shape, t, data), o in zip(self.tensors, offsets):
                f.write(data)
                f.write(b"\0" * ((-len(data)) % align))
