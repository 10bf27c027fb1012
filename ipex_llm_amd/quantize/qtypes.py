"""Low-bit qtype registry.

Numeric ids are kept identical to the reference registry
(`python/llm/src/ipex_llm/ggml/quantize.py:28-64`) so that checkpoints written
by the reference (`config.json: bigdl_transformers_low_bit=<name>`) resolve to
the same format here.  What each id *means on the device* is ours: every format
is described by a :class:`QFormat` record that drives the C++ quantizers
(``csrc/cpu/quant.cpp``), the MI355X tile repacker and the HIP GEMV/GEMM
decoders (``csrc/hip/lowbit_gemv.hip``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

# --- ids (reference parity) -------------------------------------------------
SYM_INT4 = 2
ASYM_INT4 = 3
SYM_INT5 = 6
ASYM_INT5 = 7
SYM_INT8 = 8
NF4 = 10
NF3 = 11
FP16 = 12
FP8E4 = 15
FP4 = 16
MOFQ4 = 17
MOFQ8 = 18
FP8E5 = 19
BF16 = 20
IQ2_XXS = 21
IQ2_XS = 22
Q2_K = 23
IQ1_S = 24
IQ1_M = 25
Q6_K = 26
Q4_K = 27
Q5_K = 28
FP6 = 29
FP6_K = 30
SYM_INT4_RTN = 31
SYM_INT8_RTN = 32
ASYM_INT4_RTN = 33
WOQ_INT4 = 34
TORCH_FP8E5 = 35
TORCH_FP8E4 = 36
GGUF_Q4K_S = 101
GGUF_Q4K_M = 102

ggml_tensor_qtype: Dict[str, int] = {
    "sym_int4": SYM_INT4, "asym_int4": ASYM_INT4, "sym_int5": SYM_INT5,
    "asym_int5": ASYM_INT5, "sym_int8": SYM_INT8, "nf4": NF4, "nf3": NF3,
    "fp16": FP16, "fp8_e4m3": FP8E4, "fp4": FP4, "mixed_fp4": MOFQ4,
    "mixed_fp8": MOFQ8, "fp8_e5m2": FP8E5, "fp8": FP8E5, "bf16": BF16,
    "gguf_iq2_xxs": IQ2_XXS, "gguf_iq2_xs": IQ2_XS, "q2_k": Q2_K,
    "gguf_iq1_s": IQ1_S, "gguf_iq1_m": IQ1_M, "q6_k": Q6_K, "q4_k": Q4_K,
    "q5_k": Q5_K, "fp6": FP6, "fp6_k": FP6_K, "sym_int4_rtn": SYM_INT4_RTN,
    "sym_int8_rtn": SYM_INT8_RTN, "asym_int4_rtn": ASYM_INT4_RTN,
    "woq_int4": WOQ_INT4, "torch_fp8_e5m2": TORCH_FP8E5, "torch_fp8": TORCH_FP8E5,
    "torch_fp8_e4m3": TORCH_FP8E4,
}
gguf_mixed_qtype: Dict[str, int] = {"gguf_q4k_s": GGUF_Q4K_S, "gguf_q4k_m": GGUF_Q4K_M}

# C++ format codes (must match csrc/common/formats.h :: enum Fmt).
# Storage containers: 4-bit codes (int or 16-entry LUT) or 8-bit codes
# (int8/uint8 or OCP fp8).  5-bit and 6-bit grids are quantized on their own
# grid and stored in the 8-bit container (fp6 = e3m2 grid, exactly
# representable in e4m3), 3-bit nf3 in the 4-bit LUT container.
FMT_SYM_INT4, FMT_ASYM_INT4, FMT_NF4, FMT_FP4, FMT_SYM_INT8, FMT_FP8E4, FMT_FP8E5, \
    FMT_SYM_INT5, FMT_ASYM_INT5, FMT_NF3, FMT_FP6 = range(11)
# GGUF k-quant super-block formats (csrc/common/kquant.h): the block bytes
# are the storage on host and device (GGUF tensors load as-is)
FMT_Q4K, FMT_Q5K, FMT_Q6K, FMT_Q2K = 11, 12, 13, 14
# IQ lattice super-blocks (csrc/common/iquant.h): ggml's layouts and bits
# per weight, our own codebooks
FMT_IQ2XXS, FMT_IQ2XS, FMT_IQ1S, FMT_IQ1M = 15, 16, 17, 18
KQ_BLOCK_BYTES = {FMT_Q4K: 144, FMT_Q5K: 176, FMT_Q6K: 210, FMT_Q2K: 84,
                  FMT_IQ2XXS: 66, FMT_IQ2XS: 74, FMT_IQ1S: 50, FMT_IQ1M: 56}

NF4_TABLE = [
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
    -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
    0.07958029955625534, 0.16093020141124725, 0.24611230194568634,
    0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
    0.7229568362236023, 1.0,
]
# NF3: 8-level normal-float grid (symmetric-ish, includes 0), absmax scaled.
NF3_TABLE = [-1.0, -0.5350227355957031, -0.2469314038753510, 0.0,
             0.1833375245332718, 0.3819939494132996, 0.6229856610298157, 1.0]
# FP4 = OCP e2m1 magnitudes (sign in bit 3)
FP4_TABLE = [0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0,
             -0.0, -0.5, -1.0, -1.5, -2.0, -3.0, -4.0, -6.0]


@dataclass(frozen=True)
class QFormat:
    """Static description of one weight format."""
    name: str
    qtype: int
    fmt: int                 # C++ enum
    bits: int                # bits per code in the packed code plane
    block: int               # elements per scale block along K
    has_min: bool = False    # second per-block fp16 plane (asym formats)
    gpu: bool = True         # has a tiled MI355X layout + HIP decoder
    k_align: int = 64        # K must be a multiple of this
    kquant: bool = False     # GGUF k-quant super-blocks (KQuantLinear, not the tiled layout)

    @property
    def bits_per_weight(self) -> float:
        if self.kquant:
            return KQ_BLOCK_BYTES[self.fmt] * 8 / 256
        return self.bits + 16 / self.block * (2 if self.has_min else 1)



_FORMATS: Dict[int, QFormat] = {
    SYM_INT4: QFormat("sym_int4", SYM_INT4, FMT_SYM_INT4, 4, 64),
    WOQ_INT4: QFormat("woq_int4", WOQ_INT4, FMT_SYM_INT4, 4, 64),
    ASYM_INT4: QFormat("asym_int4", ASYM_INT4, FMT_ASYM_INT4, 4, 64, has_min=True),
    NF4: QFormat("nf4", NF4, FMT_NF4, 4, 64),
    FP4: QFormat("fp4", FP4, FMT_FP4, 4, 64),
    NF3: QFormat("nf3", NF3, FMT_NF3, 4, 64),
    SYM_INT8: QFormat("sym_int8", SYM_INT8, FMT_SYM_INT8, 8, 64),
    FP8E4: QFormat("fp8_e4m3", FP8E4, FMT_FP8E4, 8, 64),
    FP8E5: QFormat("fp8_e5m2", FP8E5, FMT_FP8E5, 8, 64),
    SYM_INT5: QFormat("sym_int5", SYM_INT5, FMT_SYM_INT5, 8, 64),
    ASYM_INT5: QFormat("asym_int5", ASYM_INT5, FMT_ASYM_INT5, 8, 64, has_min=True),
    FP6: QFormat("fp6", FP6, FMT_FP6, 8, 64),
    Q4_K: QFormat("q4_k", Q4_K, FMT_Q4K, 4, 256, has_min=True, k_align=256, kquant=True),
    Q5_K: QFormat("q5_k", Q5_K, FMT_Q5K, 5, 256, has_min=True, k_align=256, kquant=True),
    Q6_K: QFormat("q6_k", Q6_K, FMT_Q6K, 6, 256, k_align=256, kquant=True),
    Q2_K: QFormat("q2_k", Q2_K, FMT_Q2K, 2, 256, has_min=True, k_align=256, kquant=True),
    IQ2_XXS: QFormat("gguf_iq2_xxs", IQ2_XXS, FMT_IQ2XXS, 2, 256, k_align=256, kquant=True),
    IQ2_XS: QFormat("gguf_iq2_xs", IQ2_XS, FMT_IQ2XS, 2, 256, k_align=256, kquant=True),
    IQ1_S: QFormat("gguf_iq1_s", IQ1_S, FMT_IQ1S, 1, 256, k_align=256, kquant=True),
    IQ1_M: QFormat("gguf_iq1_m", IQ1_M, FMT_IQ1M, 1, 256, k_align=256, kquant=True),
}
# qtypes stored in a format of equal or higher precision.  gguf_iq2_xxs /
# gguf_iq2_xs / gguf_iq1_s / gguf_iq1_m are native IQ lattice formats with
# ggml's block layouts and bits per weight (2.0625 / 2.3125 / 1.5625 / 1.75) but
# OUR codebooks (ggml's grid tables are not in the reference repository;
# csrc/common/iquant.h): IQ-coded GGUF tensors are therefore not loadable.
_ALIAS = {
    FP6_K: FP6,
    SYM_INT4_RTN: SYM_INT4, ASYM_INT4_RTN: ASYM_INT4, SYM_INT8_RTN: SYM_INT8,
    # gguf mixed policies resolve per module (mixed_kquant_qtype); q4_k otherwise
    GGUF_Q4K_S: Q4_K, GGUF_Q4K_M: Q4_K,
}
# in_features % 256 != 0: the reference's fallback formats
# (SRC/transformers/utils.py:380-401, check_hidden_size)
KQ_FALLBACK = {Q4_K: ASYM_INT4, Q5_K: ASYM_INT5, Q6_K: SYM_INT8, Q2_K: ASYM_INT4,
               IQ2_XXS: ASYM_INT4, IQ2_XS: ASYM_INT4, IQ1_S: ASYM_INT4, IQ1_M: ASYM_INT4}


def is_kquant(qtype) -> bool:
    f = get_format(qtype)
    return f is not None and f.kquant


def mixed_kquant_qtype(qtype, module_name: str, num_layers: Optional[int]) -> int:
    """Per-module qtype of the gguf_q4k_s / gguf_q4k_m policies (reference
    SRC/transformers/utils.py:337-352): lm_head q6_k; v / down of the first
    half (q4k_m: q6_k) or first eighth (q4k_s: q5_k) of the layers.  q/k/v
    are one merged qkv_proj here, so the v rule applies to qkv_proj."""
    qtype = resolve_qtype(qtype)
    if qtype not in (GGUF_Q4K_S, GGUF_Q4K_M):
        return qtype
    if module_name.endswith("lm_head"):
        return Q6_K
    import re
    m = re.search(r"layers\.(\d+)\.", module_name)
    leaf = module_name.rsplit(".", 1)[-1]
    hot = leaf in ("v_proj", "qkv_proj", "down_proj", "w2")
    if m is None or not hot or not num_layers:
        return Q4_K
    layer = int(m.group(1))
    if qtype == GGUF_Q4K_M:
        return Q6_K if layer < num_layers // 2 else Q4_K
    return Q5_K if layer < num_layers // 8 else Q4_K


def resolve_qtype(q) -> int:
    """Accept a name (``"sym_int4"``), an id, or a BitsAndBytes-style alias."""
    if isinstance(q, int):
        return q
    if q is None:
        return SYM_INT4
    name = str(q).lower()
    alias = {"int4": "sym_int4", "4bit": "sym_int4", "int8": "sym_int8",
             "8bit": "sym_int8", "bnb_nf4": "nf4", "fp8_e4m3fn": "fp8_e4m3"}
    name = alias.get(name, name)
    if name in ggml_tensor_qtype:
        return ggml_tensor_qtype[name]
    if name in gguf_mixed_qtype:
        return gguf_mixed_qtype[name]
    raise ValueError(f"unknown low-bit qtype {q!r}; known: {sorted(ggml_tensor_qtype)}")


def qtype_name(qtype: int) -> str:
    for k, v in ggml_tensor_qtype.items():
        if v == qtype:
            return k
    for k, v in gguf_mixed_qtype.items():
        if v == qtype:
            return k
    return str(qtype)


def get_format(qtype) -> Optional[QFormat]:
    """Storage format for a qtype, or None for dense (fp16/bf16/torch_fp8)."""
    qtype = resolve_qtype(qtype)
    if qtype in (FP16, BF16, TORCH_FP8E4, TORCH_FP8E5):
        return None
    if qtype in (MOFQ4, MOFQ8):
        # mixed formats resolve per tensor at quantization time
        return None
    if qtype in _FORMATS:
        return _FORMATS[qtype]
    if qtype in _ALIAS:
        return _FORMATS[_ALIAS[qtype]]
    raise ValueError(f"qtype {qtype_name(qtype)} has no storage format")


def is_dense(qtype) -> bool:
    return resolve_qtype(qtype) in (FP16, BF16)


def get_block_size(qtype) -> int:
    f = get_format(qtype)
    return f.block if f is not None else 1


def storage_bytes(qtype, n: int, k: int) -> int:
    """Bytes of the canonical planar blob for an [n, k] weight."""
    f = get_format(qtype)
    if f.kquant:
        return n * (k // 256) * KQ_BLOCK_BYTES[f.fmt]
    codes = n * k * f.bits // 8
    scales = n * (k // f.block) * 2
    mins = scales if f.has_min else 0
    return codes + scales + mins
