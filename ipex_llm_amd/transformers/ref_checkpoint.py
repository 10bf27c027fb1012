"""Read low-bit checkpoints written by the reference's ``save_low_bit``.

Reference: ``SRC/transformers/model.py:59-103`` (``save_low_bit`` moves the
model to the CPU and calls ``save_pretrained(safe_serialization=False)``, so
``pytorch_model.bin`` holds every ``FP4Params`` blob in the ggml CPU layout)
and ``model.py:532-788`` (``load_low_bit``).  The CPU layout is an array of
interleaved blocks of 64 elements (``VLLM_PATCH:4815-4912``, ``csrc/xpu/
common.h``):

==============  =========================================  =======
qtype           block                                      bytes
==============  =========================================  =======
sym_int4 q4_0   fp16 d, 32 B nibbles                       34
nf4 / fp4       same as q4_0, codes index the LUT           34
woq_int4        fp16 d, 32 B nibbles (even/odd interleave)  34
asym_int4 q4_1  fp16 d, fp16 m, 32 B nibbles               36
sym_int8 q8_0   f32 d, 64 int8                              68
fp8 e4m3/e5m2   f32 d, 64 codes                             68
q5_k / q6_k /   ggml k-quant super-blocks of 256 (standard  176 /
q2_k            block_q5_K / q6_K / q2_K), kept as is       210 / 84
==============  =========================================  =======

The k-quant rows are the reference's ``block_q5_K`` / ``block_q6_K`` /
``block_q2_K`` (``VLLM_PATCH:4928-4966``): the GGUF layouts our k-quant
kernels read, so they pass through unchanged (merged projections are
assembled by whole rows).  Its ``block_q4_K`` (148 bytes, ``VLLM_PATCH:4932-4937``)
is NOT the GGUF one: fp16 d, fp16 dmin, then 16 bytes of 8-bit scales and mins
instead of 12 packed 6-bit ones, then the 128 bytes of nibbles.  It is
repacked into the GGUF block (144 bytes) our q4_k kernels read: bytes 0-7 are
taken as the eight sub-block scales and 8-15 as the eight mins, the nibbles in
GGUF order (the reference defines no dequantizer for this struct, so the
order inside the 16 bytes is an assumption -- parity unpinned).  When every
scale / min is < 64 -- what ggml's 6-bit q4_K quantizer produces -- the repack
is exact; otherwise the block is decoded and re-quantized (lossy, warned).
``q5_0`` / ``q5_1`` (sym_int5 / asym_int5), ``fp6`` and ``fp6_k`` have no
element order in the reference sources: those checkpoints are refused.

Nibble order inside a q4_0 block (``load_qblocks``, ``VLLM_PATCH:3944-3975``):
byte j holds element j (low nibble) and element j + 32 (high nibble);
woq_int4 puts element 2j in the low and 2j + 1 in the high nibble of byte j.

Our checkpoints are ``ipex_llm_amd/canonical-planar-v1`` (codes of a row,
then all fp16 scales, then mins; ``csrc/common/formats.h``).  A q4_0 blob has
exactly the byte count of our sym_int4 blob, so loading one as the other
would pass every size check and decode garbage: the layout is therefore
recognised from the directory (reference: ``bigdl_transformers_low_bit`` in
``config.json`` and no ``illm_low_bit.json``), every blob is converted
block by block, and an unknown qtype or layout is refused.

Loading is weights-only: ``torch.load(weights_only=True)`` with a local stub
allow-listed for the reference's ``FP4Params`` parameter class, so nothing
from the file is executed.  Layout parity is unpinned: the reference ships no
low-bit checkpoint fixture, so tests build blobs from the documented layout.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch

from ..quantize import qtypes as Q

OUR_FORMAT = "ipex_llm_amd/canonical-planar-v1"

# qtype -> (block bytes, scale kind, has min, nibble order)
_GGML = {
    Q.SYM_INT4: (34, "f16", False, "q4_0"),
    Q.NF4: (34, "f16", False, "q4_0"),
    Q.FP4: (34, "f16", False, "q4_0"),
    Q.WOQ_INT4: (34, "f16", False, "woq"),
    Q.ASYM_INT4: (36, "f16", True, "q4_0"),
    Q.SYM_INT8: (68, "f32", False, "byte"),
    Q.FP8E4: (68, "f32", False, "byte"),
    Q.FP8E5: (68, "f32", False, "byte"),
}


# k-quants whose reference block is the GGUF one (kept as is)
_KQ_PASS = (Q.Q5_K, Q.Q6_K, Q.Q2_K)


def supported_qtypes():
    return [Q.qtype_name(q) for q in list(_GGML) + list(_KQ_PASS) + [Q.Q4_K]]


def _q4k_ref_to_gguf(raw: torch.Tensor, n: int, k: int) -> torch.Tensor:
    """reference 148-byte block_q4_K rows -> GGUF 144-byte blocks (see module doc)"""
    nb = n * (k // 256)
    blk = raw.view(nb, 148)
    hdr, sc8, qs = blk[:, :4], blk[:, 4:20], blk[:, 20:]
    sc, mn = sc8[:, :8].to(torch.int32), sc8[:, 8:].to(torch.int32)
    if int(sc.max()) >= 64 or int(mn.max()) >= 64:
        import warnings
        warnings.warn("reference q4_K block with 8-bit scales >= 64: decoded and re-quantized (lossy)")
        from .. import ops
        w = q4k_ref_dequantize(raw, n, k)
        return ops.kq_quantize(w, Q.get_format(Q.Q4_K).fmt, None).reshape(-1).view(torch.uint8)
    q = torch.zeros(nb, 12, dtype=torch.int32)
    q[:, 0:4] = sc[:, 0:4] | ((sc[:, 4:8] >> 4) << 6)
    q[:, 4:8] = mn[:, 0:4] | ((mn[:, 4:8] >> 4) << 6)
    q[:, 8:12] = (sc[:, 4:8] & 15) | ((mn[:, 4:8] & 15) << 4)
    return torch.cat([hdr, q.to(torch.uint8), qs], 1).reshape(-1).contiguous()


def _q4k_gguf_to_ref(raw: torch.Tensor, n: int, k: int) -> torch.Tensor:
    """inverse of :func:`_q4k_ref_to_gguf` (export / tests)"""
    nb = n * (k // 256)
    blk = raw.view(nb, 144)
    hdr, q, qs = blk[:, :4], blk[:, 4:16].to(torch.int32), blk[:, 16:]
    sc = torch.zeros(nb, 8, dtype=torch.int32)
    mn = torch.zeros(nb, 8, dtype=torch.int32)
    sc[:, :4], mn[:, :4] = q[:, 0:4] & 63, q[:, 4:8] & 63
    sc[:, 4:] = (q[:, 8:12] & 15) | ((q[:, 0:4] >> 6) << 4)
    mn[:, 4:] = (q[:, 8:12] >> 4) | ((q[:, 4:8] >> 6) << 4)
    return torch.cat([hdr, sc.to(torch.uint8), mn.to(torch.uint8), qs], 1).reshape(-1).contiguous()


def q4k_ref_dequantize(raw: torch.Tensor, n: int, k: int) -> torch.Tensor:
    """fp32 [n, k] from reference 148-byte q4_K blocks: w = d sc q - dmin mn
    per 32-element sub-block (GGUF nibble order: byte 32 c + l holds elements
    64 c + l (low) and 64 c + 32 + l (high))"""
    nb = n * (k // 256)
    blk = raw.reshape(-1).view(torch.uint8).view(nb, 148)
    d = blk[:, 0:2].contiguous().view(torch.float16).float()          # [nb, 1]
    dm = blk[:, 2:4].contiguous().view(torch.float16).float()
    sc, mn = blk[:, 4:12].float(), blk[:, 12:20].float()
    qs = blk[:, 20:].view(nb, 4, 32)
    e = torch.stack([qs & 15, qs >> 4], 2).reshape(nb, 8, 32).float()   # [nb, sub-block, 32]
    w = d[:, :, None] * sc[:, :, None] * e - dm[:, :, None] * mn[:, :, None]
    return w.reshape(n, k)


def is_reference_low_bit_dir(path: str) -> bool:
    """config.json names a reference low-bit qtype and none of our metadata is present"""
    cfg = os.path.join(str(path), "config.json")
    if not os.path.isfile(cfg) or os.path.exists(os.path.join(str(path), "illm_low_bit.json")):
        return False
    try:
        with open(cfg) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return False
    return bool(d.get("bigdl_transformers_low_bit"))


def ggml_to_canonical(blob: torch.Tensor, qtype, n: int, k: int) -> torch.Tensor:
    """reference ggml-CPU-layout blob of W[n, k] -> our canonical planar blob"""
    qt = Q.resolve_qtype(qtype)
    if qt == Q.Q4_K:
        raw = blob.reshape(-1).contiguous().view(torch.uint8)
        if k % 256 or raw.numel() != n * (k // 256) * 148:
            raise ValueError(f"reference q4_K blob has {raw.numel()} bytes, expected {n * (k // 256) * 148} "
                             f"([{n}, {k}], 148-byte blocks)")
        return _q4k_ref_to_gguf(raw, n, k)
    if qt in _KQ_PASS:
        from .. import ops
        raw = blob.reshape(-1).contiguous().view(torch.uint8)
        want = torch.ops.ipex_llm_amd.kq_total_bytes(Q.get_format(qt).fmt, n, k) if hasattr(
            torch.ops.ipex_llm_amd, "kq_total_bytes") else None
        if k % 256:
            raise ValueError(f"reference low-bit checkpoint: k-quant in_features {k} is not a multiple of 256")
        bb = {Q.Q5_K: 176, Q.Q6_K: 210, Q.Q2_K: 84}[qt]
        if raw.numel() != n * (k // 256) * bb or (want is not None and raw.numel() != want):
            raise ValueError(f"reference low-bit blob has {raw.numel()} bytes, expected {n * (k // 256) * bb} "
                             f"({Q.qtype_name(qt)} [{n}, {k}], {bb}-byte super-blocks)")
        del ops
        return raw.clone()
    if qt not in _GGML:
        raise ValueError(f"reference low-bit checkpoint: qtype {Q.qtype_name(qt)} is not supported "
                         f"(supported: {', '.join(supported_qtypes())})")
    bb, sk, has_min, order = _GGML[qt]
    if k % 64:
        raise ValueError(f"reference low-bit checkpoint: in_features {k} is not a multiple of 64")
    nb = n * (k // 64)
    raw = blob.reshape(-1).contiguous().view(torch.uint8)
    if raw.numel() != nb * bb:
        raise ValueError(f"reference low-bit blob has {raw.numel()} bytes, expected {nb * bb} "
                         f"({Q.qtype_name(qt)} [{n}, {k}], {bb}-byte blocks)")
    blk = raw.view(nb, bb)
    hdr = 4 if sk == "f32" else (4 if has_min else 2)
    if sk == "f32":
        d = blk[:, :4].contiguous().view(torch.float32).reshape(nb).to(torch.float16)
    else:
        d = blk[:, :2].contiguous().view(torch.float16).reshape(nb)
    m = blk[:, 2:4].contiguous().view(torch.float16).reshape(nb) if has_min else None
    qs = blk[:, hdr:]
    if order == "woq":
        # byte j = (e[2j] | e[2j+1] << 4)  ->  byte j = (e[j] | e[j+32] << 4)
        lo, hi = qs & 15, qs >> 4
        e = torch.stack([lo, hi], -1).reshape(nb, 64)
        qs = e[:, :32] | (e[:, 32:] << 4)
    parts = [qs.reshape(-1), d.contiguous().view(torch.uint8).reshape(-1)]
    if m is not None:
        parts.append(m.contiguous().view(torch.uint8).reshape(-1))
    return torch.cat(parts)


def canonical_to_ggml(blob: torch.Tensor, qtype, n: int, k: int) -> torch.Tensor:
    """inverse of :func:`ggml_to_canonical` (tests / export to the reference layout)"""
    qt = Q.resolve_qtype(qtype)
    if qt == Q.Q4_K:
        return _q4k_gguf_to_ref(blob.reshape(-1).view(torch.uint8), n, k)
    if qt in _KQ_PASS:
        return blob.reshape(-1).view(torch.uint8).clone()
    bb, sk, has_min, order = _GGML[qt]
    nb = n * (k // 64)
    cb = nb * (32 if bb in (34, 36) else 64)
    raw = blob.reshape(-1).view(torch.uint8)
    qs = raw[:cb].view(nb, -1)
    d = raw[cb:cb + 2 * nb].view(torch.float16)
    if order == "woq":
        lo, hi = qs & 15, qs >> 4
        e = torch.cat([lo, hi], -1)
        qs = e[:, 0::2] | (e[:, 1::2] << 4)
    hdr = [d.float().contiguous().view(torch.uint8).view(nb, 4)] if sk == "f32" else [d.contiguous().view(torch.uint8).view(nb, 2)]
    if has_min:
        m = raw[cb + 2 * nb:cb + 4 * nb].view(torch.float16)
        hdr.append(m.contiguous().view(torch.uint8).view(nb, 2))
    return torch.cat(hdr + [qs], 1).reshape(-1)


def _fp4params_stub():
    """local stand-in for ``ipex_llm.transformers.low_bit_linear.FP4Params``
    (allow-listed for the weights-only unpickler; never imports the reference)"""
    cls = type("FP4Params", (torch.nn.Parameter,), {})
    cls.__module__ = "ipex_llm.transformers.low_bit_linear"
    return cls


def load_reference_state_dict(path: str) -> Dict[str, torch.Tensor]:
    # the reference's save_low_bit always writes pytorch_model*.bin
    # (safe_serialization=False, SRC/transformers/model.py:59-103); a
    # safetensors-only directory carrying bigdl_transformers_low_bit is one of
    # OUR checkpoints that lost illm_low_bit.json (canonical planar blobs with
    # sym_int4 sizes identical to ggml blocks): refuse it instead of
    # converting planar bytes as ggml blocks
    files = sorted(glob.glob(os.path.join(path, "pytorch_model*.bin")))
    if not files:
        if glob.glob(os.path.join(path, "*.safetensors")):
            raise ValueError(f"{path}: safetensors shards without illm_low_bit.json -- not a reference "
                             "save_low_bit checkpoint (those are pytorch_model*.bin); restore illm_low_bit.json "
                             "or re-save with save_low_bit")
        raise FileNotFoundError(f"no pytorch_model*.bin under {path}")
    stub = _fp4params_stub()
    out = {}
    for f in files:
        if f.endswith(".index.json"):
            continue
        with torch.serialization.safe_globals([stub]):
            sd = torch.load(f, map_location="cpu", weights_only=True)
        for key, v in sd.items():
            out[key] = v.data if isinstance(v, torch.nn.Parameter) else v
    return out


def convert_reference_state_dict(ref_sd: Dict[str, torch.Tensor], model: torch.nn.Module, qtype) -> Dict[str, torch.Tensor]:
    """Map the reference keys/blobs onto ``model`` (built by our converter on
    meta, shapes only): low-bit blobs -> canonical planar, merged projections
    assembled (q/k/v -> qkv_proj, gate/up -> 16-row tile-interleaved
    gate_up_proj) without re-quantizing."""
    from .low_bit_linear import KQuantLinear, LowBitLinear, canon_join, canon_planes
    from ..models.decoder import interleave_glu_rows
    out: Dict[str, torch.Tensor] = {}
    used = set()

    def canon(key, n, k):
        used.add(key)
        t = ref_sd[key]
        if t.dtype == torch.uint8 or t.dtype == torch.bfloat16 and Q.resolve_qtype(qtype) == Q.NF4:
            return ggml_to_canonical(t, qtype, n, k)
        raise ValueError(f"{key}: expected a low-bit uint8 blob, got {t.dtype}")

    kq = Q.resolve_qtype(qtype) in _KQ_PASS + (Q.Q4_K,)
    for name, mod in model.named_modules():
        if not isinstance(mod, (LowBitLinear, KQuantLinear)):
            continue
        n, k, fmt = mod.out_features, mod.in_features, getattr(mod, "fmt", None)
        wk = name + ".weight"
        if wk in ref_sd:
            out[wk] = canon(wk, n, k)
        elif kq:
            # super-block rows are self-contained: merge / interleave whole rows
            parent = name.rsplit(".", 1)[0]
            leaf = name.rsplit(".", 1)[-1]
            if leaf == "qkv_proj" and all(f"{parent}.{p}_proj.weight" in ref_sd for p in "qkv"):
                per = [ref_sd[f"{parent}.{p}_proj.weight"].numel() for p in "qkv"]
                rows = [n * p // sum(per) for p in per]
                out[wk] = torch.cat([canon(f"{parent}.{p}_proj.weight", r, k) for p, r in zip("qkv", rows)])
            elif leaf == "gate_up_proj" and f"{parent}.gate_proj.weight" in ref_sd:
                half = n // 2
                g = canon(f"{parent}.gate_proj.weight", half, k).view(half, -1)
                u = canon(f"{parent}.up_proj.weight", half, k).view(half, -1)
                out[wk] = interleave_glu_rows(g, u).reshape(-1)
            else:
                raise KeyError(f"reference checkpoint has no weight for {name}")
        else:
            parent = name.rsplit(".", 1)[0]
            leaf = name.rsplit(".", 1)[-1]
            if leaf == "qkv_proj" and all(f"{parent}.{p}_proj.weight" in ref_sd for p in "qkv"):
                # q rows, then k, then v: sizes from the bias-free blob lengths
                per = [ref_sd[f"{parent}.{p}_proj.weight"].numel() for p in "qkv"]
                tot = sum(per)
                rows = [n * p // tot for p in per]
                planes = [canon_planes(canon(f"{parent}.{p}_proj.weight", r, k), fmt, r, k)
                          for p, r in zip("qkv", rows)]
                cat = [None if planes[0][i] is None else torch.cat([pl[i] for pl in planes], 0) for i in range(3)]
                out[wk] = canon_join(*cat)
            elif leaf == "gate_up_proj" and f"{parent}.gate_proj.weight" in ref_sd:
                half = n // 2
                g = canon_planes(canon(f"{parent}.gate_proj.weight", half, k), fmt, half, k)
                u = canon_planes(canon(f"{parent}.up_proj.weight", half, k), fmt, half, k)
                out[wk] = canon_join(*[None if g[i] is None else interleave_glu_rows(g[i], u[i]) for i in range(3)])
            else:
                raise KeyError(f"reference checkpoint has no weight for {name}")
        for bname in ("bias",):
            bk = f"{name}.{bname}"
            if mod.bias is not None:
                parent = name.rsplit(".", 1)[0]
                if bk in ref_sd:
                    out[bk] = ref_sd[bk]
                    used.add(bk)
                elif name.endswith("qkv_proj") and f"{parent}.q_proj.bias" in ref_sd:
                    out[bk] = torch.cat([ref_sd[f"{parent}.{p}_proj.bias"] for p in "qkv"])
                    used.update(f"{parent}.{p}_proj.bias" for p in "qkv")
    for key, v in ref_sd.items():
        if key not in used and key not in out:
            out[key] = v
    return out
