"""Native decoder-only LM executed on the ipex_llm_amd kernels.

One arch-spec-driven implementation covers the llama family the reference
optimizes with per-model forwards (``SRC/transformers/models/llama.py``,
``mistral``, ``qwen2.py``, ``qwen3.py``, ``gemma.py``, ``gemma2.py``,
``phi3.py``, ``yuan``/``internlm2``-style fused projections, ``mixtral`` /
``qwen2_moe`` / ``qwen3_moe.py`` MoE blocks ...).  Differences between those
models are data (``DecoderSpec``), not code.

Per layer and decode step the GPU work is:
  rms_norm(+residual)          add_rms_norm kernel (fused with the previous
                               projection's split-K partial reduction)
  qkv projection               low-bit skinny GEMM (MFMA)
  RoPE + KV append             rope_kv kernel (paged cache, device positions)
  attention                    flash-decoding kernel over the paged cache
  o projection                 low-bit skinny GEMM -> f32 split-K partials
  gate/up + SiLU*up            low-bit skinny GEMM with the GLU epilogue
  down projection              low-bit skinny GEMM -> partials -> next norm
so the whole step is ~9 launches per layer, no host synchronisation, and is
captured once per (batch, max_len bucket) as a hipGraph (engine/graph.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..ops import reference as R
from ..transformers.low_bit_linear import LowBitLinear, DenseLinear


@dataclass
class DecoderSpec:
    model_type: str
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int
    rms_eps: float = 1e-6
    rot_dim: Optional[int] = None
    rope_interleaved: bool = False
    max_position: int = 8192
    qkv_bias: bool = False
    o_bias: bool = False
    mlp_bias: bool = False
    qk_norm: bool = False
    act: int = 0                      # 0 silu, 1 gelu(tanh)
    tie_embeddings: bool = False
    embed_scale: float = 1.0
    norm_unit_offset: bool = False
    sliding_window: int = 0
    sliding_window_layers: Optional[List[bool]] = None
    attn_softcap: float = 0.0
    final_softcap: float = 0.0
    sandwich_norm: bool = False
    query_scale: Optional[float] = None
    rope_attention_scaling: float = 1.0
    # block layout knobs of the non-llama families (models/generic.py)
    norm_type: str = "rms"            # "rms" | "layer"
    pos_type: str = "rope"            # "rope" | "alibi" | "learned"
    parallel_residual: str = "none"   # "none" | "shared" (one norm) | "two" (two norms)
    glu: bool = True
    act_fn: str = "silu"
    # MoE
    num_experts: int = 0
    top_k: int = 0
    moe_intermediate: int = 0
    norm_topk: bool = True
    shared_expert_intermediate: int = 0
    moe_layer_mask: Optional[List[bool]] = None

    @property
    def scale(self) -> float:
        return self.query_scale if self.query_scale is not None else 1.0 / math.sqrt(self.head_dim)

    def is_moe_layer(self, i: int) -> bool:
        if self.num_experts <= 0:
            return False
        return True if self.moe_layer_mask is None else self.moe_layer_mask[i]


def compute_inv_freq(hf_config, head_dim: int, rot_dim: int):
    """inv_freq (+ attention scaling) via the HF rope registry when present."""
    try:
        from transformers.modeling_rope_utils import ROPE_INIT_FUNCTIONS
        params = getattr(hf_config, "rope_parameters", None) or getattr(hf_config, "rope_scaling", None) or {}
        rtype = params.get("rope_type", params.get("type", "default")) if isinstance(params, dict) else "default"
        if rtype != "default" and rtype in ROPE_INIT_FUNCTIONS:
            inv, scale = ROPE_INIT_FUNCTIONS[rtype](hf_config, "cpu")
            return inv.float(), float(scale)
        theta = params.get("rope_theta", None) if isinstance(params, dict) else None
    except Exception:  # pragma: no cover - transformers layout differences
        theta = None
    theta = theta or getattr(hf_config, "rope_theta", 10000.0)
    inv = 1.0 / (theta ** (torch.arange(0, rot_dim, 2, dtype=torch.float32) / rot_dim))
    return inv, 1.0


@dataclass
class AttnMeta:
    """Per-step attention metadata; all tensors are device tensors."""
    B: int
    Tq: int
    block_tables: torch.Tensor      # int32 [B, max_blocks]
    seq_lens: torch.Tensor          # int32 [B] (keys incl. the new tokens)
    nsplit: int
    seq_lens_host: Optional[List[int]] = None
    pos_offset: Optional[torch.Tensor] = None   # [B] cache index = pos - offset (compressed KV)


def interleave_glu_rows(gate: torch.Tensor, up: torch.Tensor, tile: int = 16) -> torch.Tensor:
    """[I, K] gate + [I, K] up -> [2I, K] with 16-row tiles alternating
    (gate tile p, up tile p, ...): the layout the GLU-epilogue GEMV expects."""
    I, K = gate.shape
    assert I % tile == 0, "intermediate size must be a multiple of 16"
    return torch.stack([gate.view(I // tile, tile, K), up.view(I // tile, tile, K)], 1).reshape(2 * I, K)


# decode-size GLU over dense (bf16 / fp16) gate/up weights in one streaming
# launch (csrc/hip/dense_gemv.hip dense_glu); ILLM_DENSE_GLU=0 for A/B
_DENSE_GLU = __import__("os").environ.get("ILLM_DENSE_GLU", "1") != "0"
# rows up to which it runs -- every decode / verify size: a row's result must
# not depend on how many rows share the launch, or the k + 1-row speculative
# verify stops reproducing one-token greedy decoding (capping it at 2 rows
# dropped the generated-token agreement to 0.016, profiles/spec_glu2_r4.jsonl).
# MI355X, Llama-3-8B bf16 (profiles/spec_glu16_r4.jsonl, spec_noglu_r4.jsonl):
# one-token decode 3.790 -> 3.522 ms/token; speculative k = 2 3.444 ms/token
# the kernel serves at most 16 rows (TORCH_CHECK in dense_glu_hip): larger
# settings are clamped so bigger batches take the unfused path
DENSE_GLU_MAX_M = min(int(__import__("os").environ.get("ILLM_DENSE_GLU_MAX_M", "16")), 16)


def deinterleave_glu(gu: torch.Tensor, tile: int = 16):
    shp = gu.shape[:-1]
    I = gu.shape[-1] // 2
    x = gu.reshape(-1, I // tile, 2, tile)
    return x[:, :, 0].reshape(*shp, I), x[:, :, 1].reshape(*shp, I)


def _ksplit(n: int, k: int) -> int:
    nt, kc = (n + 15) // 16, (k + 127) // 128
    ks = 1
    while nt * ks < 768 and kc >= 4 * 2 * (ks * 2):
        ks *= 2
    return ks


# rows handled by the atomic split-K GEMV (ops.gemv_accum): its consumers
# read ONE f32 slab instead of ks.  With the block-transposed atomic epilogue
# (one row segment per wave instruction) the atomic GEMV costs about what the
# slab-store one does up to 8 rows (MI355X, Llama-3-8B decode: batch 4
# 2.191 -> 2.128 ms/step, batch 8 2.392 -> 2.382)
ACC_MAX_M = int(__import__("os").environ.get("ILLM_ACC_MAX_M", "8"))
# residual-add + RMSNorm folded into the consuming GEMV's prologue: every
# workgroup re-derives the full-row norm, fine for 1-2 rows, far too much
# redundant slab traffic at 4-8 (batch 8: 2.38 -> 3.08 ms/step)
NORM_IN_MAX_M = int(__import__("os").environ.get("ILLM_NORM_IN_MAX_M", "2"))
# deferred RMSNorm (lowbit_gemv5.cuh ndefer): the consuming GEMV stages
# w * (residual + acc) for its own K slice only and the 1/rms row scale is
# applied by the qkv consumer (RoPE / fused-RoPE attention) or in the gate/up
# GLU epilogue -- no full-row pass per workgroup, so the norm-in path extends
# to larger decode batches (ILLM_DEFER_NORM=0 restores the full-row prologue)
DEFER_NORM = __import__("os").environ.get("ILLM_DEFER_NORM", "1") != "0"
DEFER_MAX_M = int(__import__("os").environ.get("ILLM_DEFER_MAX_M", "8"))
# ... and up to this batch for the gate/up GLU launch too (every GLU workgroup
# stages the full K of acc + residual: at batch 8 that replicated row read
# costs more than the standalone norm launch, MI355X probe
# profiles/gemv5_defer_r3.jsonl: GLU 24.7 us deferred vs 19.7 us on a normed x)
DEFER_GLU_MAX_M = int(__import__("os").environ.get("ILLM_DEFER_GLU_MAX_M", "4"))
# above it: gate/up as a split-K atomic GEMV staging only its own K slice
# (deferred norm), act(g / rms) * (u / rms) applied by the down GEMV while it
# stages its input -- no norm launch, no full-row read per workgroup
# Opt-in (ILLM_DEFER_MLP_ACC=1): measured slower on MI355X at batch 8 than the
# standalone norm + GLU GEMV it replaces (2.49 vs 2.38 ms/step, same box,
# profiles/bench_b8_r3_mlpacc*.json): the down GEMV's input staging from the
# [8, 28672] f32 gate/up slab costs more than the norm launch
DEFER_MLP_ACC = __import__("os").environ.get("ILLM_DEFER_MLP_ACC", "0") == "1"
# decode batches from this size on (up to DEFER_MAX_M) let the o_proj GEMV's
# last-arriving split-K workgroups do the residual add and stage the deferred
# gate/up input (ops.gemv_accum_norm -> ops.gemv_glu_ss): no standalone
# add_rms_norm launch between attention and MLP (ILLM_ONORM=0 restores it)
ONORM = __import__("os").environ.get("ILLM_ONORM", "1") != "0"
ONORM_MIN_M = int(__import__("os").environ.get("ILLM_ONORM_MIN_M", "5"))
# decode batches up to this size take the fused-RoPE attention (qkv accumulated
# atomically into one slab read by the attention, re-zeroed by its combine).
# Measured on MI355X (Llama-3-8B, L=1024): batch 1 1.960 -> 1.910 ms/token,
# batch 4 2.128 -> 2.109 ms/step; at batch 8 every split wave re-rotating q
# costs more than the rope launch it saves (2.382 -> 2.527)
ROPE_IN_MAX_M = int(__import__("os").environ.get("ILLM_ROPE_IN_MAX_M", "4"))
# ... unless the qkv GEMV rotates q / k itself: RoPE is linear, so each
# split-K workgroup rotates its partial before the atomic add (epilogue in
# lowbit_gemv5.cuh) and the attention reads rotated q / k -- no per-split
# re-rotation, no rope launch, at every decode batch up to ACC_MAX_M
# (ILLM_GEMV_ROPE=0 keeps the rotation in the attention / rope kernels)
GEMV_ROPE = __import__("os").environ.get("ILLM_GEMV_ROPE", "1") != "0"


class NativeAttention(nn.Module):
    def __init__(self, spec: DecoderSpec, qkv_proj: nn.Module, o_proj: nn.Module,
                 q_norm: Optional[torch.Tensor] = None, k_norm: Optional[torch.Tensor] = None,
                 sliding_window: int = 0):
        super().__init__()
        self.spec = spec
        self.qkv_proj, self.o_proj = qkv_proj, o_proj
        self.q_norm = nn.Parameter(q_norm, requires_grad=False) if q_norm is not None else None
        self.k_norm = nn.Parameter(k_norm, requires_grad=False) if k_norm is not None else None
        self.sliding_window = sliding_window
        self.lf = None                      # Yuan 2.0 localized filtering (models/yuan.py YuanLF)


class NativeMLP(nn.Module):
    """gate_up_proj holds the tile-interleaved [gate; up] rows."""

    def __init__(self, spec: DecoderSpec, gate_up_proj: nn.Module, down_proj: nn.Module):
        super().__init__()
        self.spec = spec
        self.gate_up_proj, self.down_proj = gate_up_proj, down_proj


class NativeLayer(nn.Module):
    def __init__(self, spec, attn, mlp, ln1, ln2, pre_ff=None, post_ff=None):
        super().__init__()
        self.self_attn, self.mlp = attn, mlp
        self.input_layernorm = nn.Parameter(ln1, requires_grad=False)
        self.post_attention_layernorm = nn.Parameter(ln2, requires_grad=False)
        self.pre_feedforward_layernorm = nn.Parameter(pre_ff, requires_grad=False) if pre_ff is not None else None
        self.post_feedforward_layernorm = nn.Parameter(post_ff, requires_grad=False) if post_ff is not None else None


def linear(x: torch.Tensor, mod: nn.Module) -> torch.Tensor:
    return mod(x)


class NativeCausalLM(nn.Module):
    def __init__(self, spec: DecoderSpec, embed: torch.Tensor, layers: List[NativeLayer], norm: torch.Tensor,
                 lm_head: nn.Module, inv_freq: torch.Tensor, dtype=torch.bfloat16):
        super().__init__()
        self.spec = spec
        self.dtype = dtype
        if isinstance(embed, nn.Module):     # CPU / disk / low-bit embedding module
            self.embed_module = embed
            self.embed_tokens = None
        else:
            self.embed_module = None
            self.embed_tokens = nn.Parameter(embed, requires_grad=False)
        self.layers = nn.ModuleList(layers)
        self.norm = nn.Parameter(norm, requires_grad=False)
        self.lm_head = lm_head
        self.register_buffer("inv_freq", inv_freq.float(), persistent=False)
        self.rope_cache: Optional[torch.Tensor] = None
        self.tp_group = None
        self.alibi = None                   # [Hq] f32 ALiBi slopes (generic families)
        # pipeline-parallel stage flags (parallel/pipeline.py): a stage owns a
        # contiguous layer range; only the first embeds, only the last has
        # the final norm + lm_head
        self.first_stage = True
        self.last_stage = True
        self.layer_offset = 0
        self._acc_bufs = {}

    def ensure_rope_cache(self, max_pos: int):
        """f32 [max_pos, rot/2, 2] cos/sin table (HF fp32 formula, incl. the
        rope attention scaling) so the RoPE kernel does a lookup, not sincos."""
        if self.rope_cache is not None and self.rope_cache.shape[0] >= max_pos and \
                self.rope_cache.device == self.inv_freq.device:
            return self.rope_cache
        n = max(max_pos, 256)
        pos = torch.arange(n, device=self.inv_freq.device, dtype=torch.float32)
        freqs = pos[:, None] * self.inv_freq[None, :]
        sc = self.spec.rope_attention_scaling
        self.rope_cache = torch.stack([freqs.cos() * sc, freqs.sin() * sc], -1).contiguous()
        return self.rope_cache

    @property
    def device(self):
        return self.layers[0].input_layernorm.device

    def graph_max_batch(self) -> int:
        """Largest one-token-per-sequence decode batch whose ``forward_tokens``
        is hipGraph-capture safe (no host sync, no data-dependent routing
        baked in at capture).  0: never capture."""
        s = self.spec
        group = s.num_heads // s.num_kv_heads
        if group > 16 or s.head_dim not in (64, 80, 96, 128, 256):
            return 0                      # SDPA fallback reads seq_lens on the host
        lim = 1 << 30
        for L in self.layers:
            mlp = L.mlp
            if type(mlp).__name__ == "NativeMoE":
                lim = min(lim, mlp.graph_max_tokens())
            elif not isinstance(mlp, NativeMLP) and not hasattr(mlp, "graph_max_tokens"):
                lim = min(lim, 16)
        return lim

    # ------------------------------------------------------------------ cache
    def make_cache(self, max_tokens: int, batch: int = 1, block_size: int = 64, kv_fp8: int = 0,
                   num_blocks: Optional[int] = None):
        from .cache import PagedKVCache
        s = self.spec
        nblk = num_blocks or batch * ((max_tokens + block_size - 1) // block_size)
        self.ensure_rope_cache(max_tokens + 1)
        cache = PagedKVCache(len(self.layers), nblk, s.num_kv_heads, s.head_dim, block_size, self.dtype,
                             self.device, kv_fp8)
        if any(L.self_attn.lf is not None for L in self.layers):
            # Yuan LFA: h and conv1 output of every position, slot-addressed,
            # plus one zero row standing for position -1
            H = s.hidden_size
            cache.lf = [torch.zeros(nblk * block_size + 1, H + H // 2, dtype=self.dtype, device=self.device)
                        for _ in self.layers]
        return cache

    # ------------------------------------------------------------------ pieces
    def _attention(self, li: int, attn: NativeAttention, q: torch.Tensor, meta: AttnMeta, cache) -> torch.Tensor:
        s = self.spec
        T = q.shape[0]
        group = s.num_heads // s.num_kv_heads
        softcap = s.attn_softcap
        window = attn.sliding_window
        kc, vc = cache.k[li], cache.v[li]
        if meta.Tq * group <= 16 and (s.head_dim in (64, 80, 96, 128, 256) or not q.is_cuda):
            o = ops.attn_decode(q.view(meta.B, meta.Tq, s.num_heads, s.head_dim), kc, vc, meta.block_tables,
                                meta.seq_lens, meta.nsplit, s.scale, softcap, window, cache.kv_fp8,
                                cache.k_scale, cache.v_scale, self.alibi, meta.seq_lens_host)
            return o.view(T, s.num_heads * s.head_dim)
        if group <= 16 and meta.Tq <= 16 and (s.head_dim in (64, 80, 96, 128, 256) or not q.is_cuda):
            # short query chunks (speculative verify of k + 1 tokens, tiny
            # prefills): the decode kernel over <= 16 // group tokens at a
            # time, the later tokens' keys cut off by a shorter length, so
            # every query row is reduced exactly as in one-token decoding
            # (greedy speculative output == plain greedy output)
            c = 16 // group
            qv = q.view(meta.B, meta.Tq, s.num_heads, s.head_dim)
            outs = []
            for t0 in range(0, meta.Tq, c):
                n = min(c, meta.Tq - t0)
                cut = meta.Tq - t0 - n
                lens = meta.seq_lens - cut if cut else meta.seq_lens
                lens_h = None if meta.seq_lens_host is None else [int(v) - cut for v in meta.seq_lens_host]
                outs.append(ops.attn_decode(qv[:, t0:t0 + n].contiguous(), kc, vc, meta.block_tables, lens,
                                            meta.nsplit, s.scale, softcap, window, cache.kv_fp8, cache.k_scale,
                                            cache.v_scale, self.alibi, lens_h))
            return torch.cat(outs, 1).view(T, s.num_heads * s.head_dim)
        if q.is_cuda and self.alibi is None and s.head_dim in (64, 128) and cache.bs % 64 == 0 and self._prefill_attn_native \
                and ops.native_gpu(q):
            # prefill / long query chunk: flash-attention HIP kernel over the paged cache
            o = ops.attn_prefill(q.view(T, s.num_heads, s.head_dim), kc, vc, meta.block_tables, meta.seq_lens,
                                 meta.Tq, s.scale, softcap, window, cache.kv_fp8, cache.k_scale, cache.v_scale)
            return o.view(T, s.num_heads * s.head_dim)
        # other head dims: gather the sequence's keys and use SDPA
        lens = meta.seq_lens_host if meta.seq_lens_host is not None else meta.seq_lens.tolist()
        qv = q.view(meta.B, meta.Tq, s.num_heads, s.head_dim)
        outs = []
        for b in range(meta.B):
            L = int(lens[b])
            kk = ops.api.gather_kv(kc, meta.block_tables, b, L, cache.kv_fp8, cache.k_scale, q.dtype)
            vv = ops.api.gather_kv(vc, meta.block_tables, b, L, cache.kv_fp8, cache.v_scale, q.dtype)
            if softcap or not q.is_cuda or self.alibi is not None:
                outs.append(R.attention(qv[b:b + 1], kk[None], vv[None], True, s.scale, softcap, window, None,
                                        self.alibi))
                continue
            qq = qv[b].transpose(0, 1)[None]                 # [1, Hq, Tq, D]
            k4 = kk.transpose(0, 1)[None]
            v4 = vv.transpose(0, 1)[None]
            Tq = qq.shape[2]
            if Tq == L and not window:
                o = F.scaled_dot_product_attention(qq, k4, v4, is_causal=True, scale=s.scale, enable_gqa=True)
            else:
                qpos = (L - Tq) + torch.arange(Tq, device=q.device)
                kpos = torch.arange(L, device=q.device)
                mask = kpos[None, :] <= qpos[:, None]
                if window:
                    mask &= kpos[None, :] > (qpos[:, None] - window)
                o = F.scaled_dot_product_attention(qq, k4, v4, attn_mask=mask, scale=s.scale, enable_gqa=True)
            outs.append(o[0].transpose(0, 1)[None])
        o = outs[0] if len(outs) == 1 else torch.cat(outs, 0)      # (a 1-element cat is a slow strided copy)
        return o.reshape(T, s.num_heads * s.head_dim)

    def _tp_ok(self, mod) -> bool:
        """row-parallel layer of this model's TP group (or not row-parallel)"""
        g = getattr(mod, "mp_group", None)
        return g is None or g is self.tp_group

    @staticmethod
    def _reduce(acc: torch.Tensor, mod) -> torch.Tensor:
        """sum a row-parallel layer's f32 split-K accumulator over its TP group
        in place (custom xGMI all-reduce / RCCL): the fused norm consumers then
        read the full output exactly as on one GPU"""
        g = getattr(mod, "mp_group", None)
        if g is None:
            return acc
        from ..parallel.comm import all_reduce_inplace
        out = all_reduce_inplace(acc, g)
        if out is not acc:
            acc.copy_(out)
        return acc

    def _acc(self, n: int, t: int, device, tag: str = "", dtype=torch.float32) -> torch.Tensor:
        """Zeroed f32 [t, n] accumulator for the split-K atomic GEMV
        (ops.gemv_accum); its consumer re-zeroes it after reading (or a later
        launch does, ``tag``-separated buffers of the norm-in path), so one
        buffer per shape serves every layer and every hipGraph replay."""
        key = (n, t, tag, dtype)
        buf = self._acc_bufs.get(key)
        if buf is None or buf.device != device:
            buf = torch.zeros(t, n, dtype=dtype, device=device)
            self._acc_bufs[key] = buf
        return buf

    def _ctr(self, device, n: int = 4096) -> torch.Tensor:
        """int32 tickets of the last-arriver GEMV epilogues (ops.gemv_accum_norm):
        zero once, every launch's last arriver resets its own"""
        buf = self._acc_bufs.get(("ctr", device))
        if buf is None or buf.numel() < n:
            buf = torch.zeros(n, dtype=torch.int32, device=device)
            self._acc_bufs[("ctr", device)] = buf
        return buf

    # decode (norm-in + fused-RoPE path): attention partials merged in the o_proj
    # GEMV prologue instead of a combine launch (ILLM_OPROJ_COMBINE=1), with
    # ILLM_OPROJ_KS K slices (32 = one head per workgroup) of ILLM_OPROJ_NW waves
    _oproj_combine = __import__("os").environ.get("ILLM_OPROJ_COMBINE", "0") == "1"
    _oproj_ks = int(__import__("os").environ.get("ILLM_OPROJ_KS", "32"))
    _oproj_nw = int(__import__("os").environ.get("ILLM_OPROJ_NW", "8"))

    # ILLM_PREFILL_ATTN=sdpa: torch SDPA over gathered keys instead of the HIP kernel (A/B)
    _prefill_attn_native = __import__("os").environ.get("ILLM_PREFILL_ATTN", "hip") != "sdpa"

    # opt-in: measured on MI355X (Llama-3-8B, L=1024) the prologue merge is
    # replicated by every o_proj N-tile group (64x re-reads of the partials:
    # 128 MB of L2 traffic at batch 8), costing more than the combine launch
    # it saves (batch 1: 2.07 vs 2.06 ms/token, batch 8: 3.04 vs 2.83)
    _attn_fuse = __import__("os").environ.get("ILLM_ATTN_OPROJ_FUSE", "0") == "1"

    def _attn_oproj_fuse_ok(self, attn, q, meta) -> bool:
        """decode attention whose split partials are merged inside the o_proj
        GEMV prologue (no combine launch): native GPU, <= 16 rows, plain
        low-bit o_proj, no sandwich norm / TP, bounded split count."""
        s, o = self.spec, attn.o_proj
        group = s.num_heads // s.num_kv_heads
        return (self._attn_fuse and q.is_cuda and not s.sandwich_norm and self.tp_group is None
                and q.shape[0] <= 16 and meta.Tq * group <= 16 and meta.nsplit <= 128
                and s.head_dim in (64, 80, 96, 128, 256) and s.head_dim % 8 == 0
                and isinstance(o, LowBitLinear) and o.bias is None and o.mp_group is None
                and ops.native_gpu(q))

    def _attn_oproj_norm(self, li, attn, q, meta, cache, residual, norm_w):
        s, o = self.spec, attn.o_proj
        T = q.shape[0]
        po, pml = ops.attn_decode_split(q.view(meta.B, meta.Tq, s.num_heads, s.head_dim), cache.k[li], cache.v[li],
                                        meta.block_tables, meta.seq_lens, meta.nsplit, s.scale, s.attn_softcap,
                                        attn.sliding_window, cache.kv_fp8, cache.k_scale, cache.v_scale, None)
        if T <= ACC_MAX_M:
            acc = self._acc(o.out_features, T, q.device)
            ops.gemv_attn(po, pml, meta.seq_lens, o.weight, o.fmt, o.out_features, o.in_features, acc, 0, q.dtype)
            out, _ = ops.add_rms_norm(None, residual, norm_w, s.rms_eps, partials=acc.unsqueeze(0),
                                      unit_offset=s.norm_unit_offset, zero_partials=True)
        else:
            part = ops.gemv_attn(po, pml, meta.seq_lens, o.weight, o.fmt, o.out_features, o.in_features, None, 0,
                                 q.dtype)
            out, _ = ops.add_rms_norm(None, residual, norm_w, s.rms_eps, partials=part,
                                      unit_offset=s.norm_unit_offset)
        return out

    def _proj_residual_norm(self, x, proj, residual, norm_w, post_norm_w=None):
        """residual += proj(x); return rms_norm(residual) * norm_w."""
        s = self.spec
        fused = (x.is_cuda and isinstance(proj, LowBitLinear) and proj.bias is None and self._tp_ok(proj)
                 and post_norm_w is None and x.shape[0] <= ops.GEMV_MAX_M)
        if fused and x.shape[0] <= ACC_MAX_M and ops.native_gpu(x):
            # split-K f32 atomics into one zeroed slab (summed over the TP group
            # for a row-parallel layer); the norm reads + re-zeroes it
            acc = self._acc(proj.out_features, x.shape[0], x.device)
            ops.gemv_accum(x, proj.weight, proj.fmt, proj.out_features, proj.in_features, acc)
            self._reduce(acc, proj)
            out, _ = ops.add_rms_norm(None, residual, norm_w, s.rms_eps, partials=acc.unsqueeze(0),
                                      unit_offset=s.norm_unit_offset, zero_partials=True)
            return out
        if fused:
            part = ops.gemv_partials(x, proj.weight, proj.fmt, proj.out_features, proj.in_features, 0)
            if proj.mp_group is not None:
                part = self._reduce(part.sum(0, keepdim=True), proj)
            out, _ = ops.add_rms_norm(None, residual, norm_w, s.rms_eps, partials=part,
                                      unit_offset=s.norm_unit_offset)
            return out
        y = proj(x)
        if self.tp_group is not None and not getattr(proj, "mp_group", None):
            from ..parallel.comm import all_reduce_inplace
            y = all_reduce_inplace(y, self.tp_group)
        if post_norm_w is not None:
            y = ops.rms_norm(y, post_norm_w, s.rms_eps, s.norm_unit_offset)
        out, _ = ops.add_rms_norm(y.contiguous(), residual, norm_w, s.rms_eps, unit_offset=s.norm_unit_offset)
        return out

    # decode (T <= ACC_MAX_M) with the residual add + RMSNorm folded into the
    # prologue of the GEMV that consumes them (qkv, gate/up): two norm
    # launches per layer fewer.  ILLM_NORM_IN=0 restores the standalone norms.
    _norm_in_env = __import__("os").environ.get("ILLM_NORM_IN", "1") != "0"

    _embed_norm_env = __import__("os").environ.get("ILLM_EMBED_NORM", "1") != "0"

    def _embed_norm_ok(self, ids: torch.Tensor) -> bool:
        e = self.embed_tokens
        return (self._embed_norm_env and self.embed_module is None and self.spec.embed_scale == 1.0
                and isinstance(e, torch.Tensor) and e.is_cuda and ids.is_cuda and e.dim() == 2
                and e.dtype == self.dtype and e.dtype in (torch.bfloat16, torch.float16) and e.is_contiguous()
                and self.layers[0].input_layernorm.dtype == e.dtype and self.spec.hidden_size % 8 == 0
                and ops.native_gpu(ids))

    def _defer_ok(self, ref: torch.Tensor, T: int) -> bool:
        return DEFER_NORM and T <= min(ACC_MAX_M, DEFER_MAX_M)

    def _norm_in_ok(self, ref: torch.Tensor, T: int) -> bool:
        lim = max(NORM_IN_MAX_M, DEFER_MAX_M if self._defer_ok(ref, T) else 0)
        if not (self._norm_in_env and T <= min(ACC_MAX_M, lim) and ref.is_cuda
                and not self.spec.sandwich_norm and not self._attn_fuse and not self._glu_in_enabled
                and self.spec.hidden_size % 8 == 0 and ops.native_gpu(ref)):
            return False
        ok = self.__dict__.get("_norm_in_layers")
        if ok is None:
            def lowbit(m, bias_ok=False):
                return isinstance(m, LowBitLinear) and self._tp_ok(m) and (bias_ok or m.bias is None)
            ok = all(isinstance(L.mlp, NativeMLP) and lowbit(L.mlp.gate_up_proj) and lowbit(L.mlp.down_proj)
                     and lowbit(L.self_attn.o_proj) and lowbit(L.self_attn.qkv_proj, True)
                     and L.self_attn.qkv_proj.mp_group is None and L.mlp.gate_up_proj.mp_group is None
                     and (L.self_attn.qkv_proj.bias is None or L.self_attn.qkv_proj.bias.dtype == ref.dtype)
                     and L.post_feedforward_layernorm is None for L in self.layers)
            self.__dict__["_norm_in_layers"] = ok
        return ok

    # decode (one new token per sequence) attention that applies RoPE to q/k
    # from the qkv accumulator and appends the new key/value itself: one
    # launch per layer fewer.  ILLM_ROPE_IN=0 restores the rope_kv launch.
    _rope_in_env = __import__("os").environ.get("ILLM_ROPE_IN", "1") != "0"

    def _rope_in_ok(self, meta: "AttnMeta", cache) -> bool:
        s = self.spec
        group = s.num_heads // s.num_kv_heads
        # (compressed KV: seq_lens are cache lengths, the rotary position comes from pos)
        return (self._rope_in_env and meta.Tq == 1 and cache.kv_fp8 == 0
                and self._capture_q is None and self.rope_cache is not None
                and ((s.head_dim == 128 and group <= 16) or (s.head_dim == 256 and group <= 8))
                and all(L.self_attn.q_norm is None and L.self_attn.k_norm is None for L in self.layers))

    def _qkv_bias_free(self) -> bool:
        ok = self.__dict__.get("_qkv_nobias")
        if ok is None:
            ok = all(getattr(L.self_attn.qkv_proj, "bias", None) is None for L in self.layers)
            self.__dict__["_qkv_nobias"] = ok
        return ok

    def _qkv_native(self, ref: torch.Tensor) -> bool:
        """every layer's qkv projection runs the native atomic GEMV"""
        ok = self.__dict__.get("_qkv_native_ok")
        if ok is None:
            ok = all(isinstance(L.self_attn.qkv_proj, LowBitLinear) and L.self_attn.qkv_proj.mp_group is None
                     and (L.self_attn.qkv_proj.bias is None or L.self_attn.qkv_proj.bias.dtype == ref.dtype)
                     for L in self.layers)
            self.__dict__["_qkv_native_ok"] = ok
        return ok and ref.is_cuda and ops.native_gpu(ref)

    def _fused_mlp_ok(self, x, layer, need_env: bool = True) -> bool:
        mlp = layer.mlp
        if not (x.is_cuda and isinstance(mlp, NativeMLP) and x.shape[0] <= 16):
            return False
        gu, dn = mlp.gate_up_proj, mlp.down_proj
        return (isinstance(gu, LowBitLinear) and isinstance(dn, LowBitLinear) and gu.bias is None and dn.bias is None
                and gu.mp_group is None and self._tp_ok(dn) and layer.post_feedforward_layernorm is None
                and dn.in_features % 16 == 0 and (self._glu_in_enabled or not need_env) and ops.native_gpu(x))

    def _mlp_acc_ok(self, x, layer) -> bool:
        """decode MLP as gate/up atomic GEMV -> down GEMV taking act(gate) * up
        from that accumulator in its input staging (atomic out): the GLU
        epilogue's unsplittable launch and the [T, I] round trip go away"""
        return (self._mlp_acc_env and x.shape[0] <= ACC_MAX_M and self._fused_mlp_ok(x, layer, need_env=False))

    _mlp_acc_env = __import__("os").environ.get("ILLM_MLP_ACC", "0") == "1"

    # measured neutral at B=1 and ~1% slower at B=8 on MI355X (the down GEMV's
    # slab-reading prologue costs what the split gate/up GEMV saves): opt-in
    _capture_q = None
    _capture_w = 32
    _glu_in_enabled = __import__("os").environ.get("ILLM_FUSED_GLU_IN", "0") == "1"

    def _mlp(self, x, mlp: nn.Module):
        s = self.spec
        if not isinstance(mlp, NativeMLP):
            return mlp(x)                                   # MoE / custom block returns down-proj input
        gu = mlp.gate_up_proj
        if x.is_cuda and isinstance(gu, LowBitLinear) and gu.bias is None and x.shape[0] <= ops.GEMV_MAX_M \
                and ops.native_gpu(x):
            return ops.gemv_glu(x, gu.weight, gu.fmt, gu.out_features, gu.in_features, s.act)
        if x.is_cuda and isinstance(gu, LowBitLinear) and gu.bias is None and gu.g_idx_map is None \
                and gu.mp_group is None and x.dtype in (torch.bfloat16, torch.float16) and ops.native_gpu(x):
            # prefill: the activation runs in the GEMM epilogue (no [T, 2I] round trip)
            from ..ops.gemm import lowbit_gemm_glu
            return lowbit_gemm_glu(x.contiguous(), gu.weight, gu.fmt, gu.out_features, gu.in_features, s.act)
        if _DENSE_GLU and x.is_cuda and isinstance(gu, DenseLinear) and gu.bias is None and gu.mp_group is None \
                and x.shape[0] <= DENSE_GLU_MAX_M and s.act in (0, 1) and x.dtype == gu.weight.dtype \
                and ops.native_gpu(x) \
                and gu.out_features % 32 == 0 and gu.in_features % 8 == 0:
            # decode / verify rows on dense weights: one streaming launch, GLU in its epilogue
            return torch.ops.ipex_llm_amd.dense_glu(x, gu.weight, s.act)
        y = gu(x)
        g, u = deinterleave_glu(y)
        a = F.silu(g) if s.act == 0 else F.gelu(g, approximate="tanh")
        return (a * u).contiguous()

    def _prefetch_layer(self, li: int, T: int, dtype, prefetch_dense):
        L = self.layers[li]
        mods = [getattr(L.self_attn, "qkv_proj", None), getattr(L.self_attn, "o_proj", None)]
        if isinstance(L.mlp, NativeMLP):
            mods += [L.mlp.gate_up_proj, L.mlp.down_proj]
        items = [(m.weight, m.fmt, m.out_features, m.in_features) for m in mods
                 if isinstance(m, LowBitLinear) and m.mp_group is None and m.g_idx_map is None
                 and m.compute_dtype in (None, dtype)]
        prefetch_dense(items, T, dtype)

    # ------------------------------------------------------------------ forward
    def forward_tokens(self, ids: torch.Tensor, pos: torch.Tensor, slots: torch.Tensor, meta: AttnMeta,
                       cache, logits_idx: Optional[torch.Tensor] = None, return_hidden: bool = False,
                       hidden_in: Optional[torch.Tensor] = None):
        """ids/pos/slots: [T] (T = B * Tq, sequence-major).  Returns logits
        [len(logits_idx) or T, vocab] in f32.  Pipeline stages: ``hidden_in``
        is the previous stage's residual stream [T, H]; a non-last stage
        returns its residual stream instead of logits."""
        s = self.spec
        T = ids.shape[0]
        ss_zeroed = None
        if hidden_in is None and self._embed_norm_ok(ids):
            # one launch: embedding gather (the residual stream), the first
            # layer's RMSNorm and the zeroing of the step's deferred-norm sums
            defer0 = self._norm_in_ok(self.embed_tokens, T) and self._defer_ok(self.embed_tokens, T)
            ss_zeroed = self._acc(T, 2 * len(self.layers), ids.device, "SS") if defer0 else None
            residual, x = torch.ops.ipex_llm_amd.embed_rms_norm(ids.contiguous(), self.embed_tokens,
                                                               self.layers[0].input_layernorm, s.rms_eps,
                                                               s.norm_unit_offset, ss_zeroed)
        else:
            if hidden_in is not None:
                residual = hidden_in.to(self.dtype).contiguous().clone()
            else:
                h = self.embed_module(ids).to(self.dtype) if self.embed_module is not None else \
                    F.embedding(ids, self.embed_tokens)
                if s.embed_scale != 1.0:
                    h = h * torch.tensor(s.embed_scale, dtype=h.dtype, device=h.device)
                residual = h.contiguous()
            x = ops.rms_norm(residual, self.layers[0].input_layernorm, s.rms_eps, s.norm_unit_offset)
        rope = self.rope_cache if self.rope_cache is not None else self.inv_freq
        # norm-in decode: the down projection's atomic accumulator stays pending
        # and the next layer's qkv GEMV adds + normalises it in its prologue;
        # the residual ping-pongs between two buffers (written by one workgroup)
        norm_in = self._norm_in_ok(residual, T)
        pend = None                     # accumulator awaiting residual-add + norm
        consumed = None                 # accumulator read by the last launch: zeroed by the next GEMV
        res_pp = (residual, torch.empty_like(residual)) if norm_in else None
        # deferred norm: per-(layer, norm) row sums of squares, zeroed once per step
        defer = norm_in and self._defer_ok(residual, T)
        ss_all = None
        if defer:
            ss_all = self._acc(T, 2 * len(self.layers), x.device, "SS")
            if ss_zeroed is not ss_all:
                ss_all.zero_()
        ss_q = None                     # sums of squares of the current layer's qkv input (deferred)
        zero_gu = None                  # consumed gate/up accumulator (batch > DEFER_GLU_MAX_M), zeroed next
        # fused-RoPE decode attention (batch <= ROPE_IN_MAX_M, one token each): the qkv
        # GEMV accumulates into one atomic slab that the attention reads and the
        # combine launch re-zeroes
        rope_ok = self._rope_in_ok(meta, cache) and self._qkv_native(residual)
        prerot = (GEMV_ROPE and rope_ok and T <= ACC_MAX_M and s.rot_dim == s.head_dim and not s.rope_interleaved
                  and s.head_dim in (64, 128) and self._qkv_bias_free())
        rope_in = rope_ok and (T <= ROPE_IN_MAX_M or prerot)
        qrope = (self.rope_cache, pos, (s.num_heads + s.num_kv_heads) * s.head_dim, s.head_dim) if prerot else None
        nxt_res = lambda r: res_pp[1] if r is res_pp[0] else res_pp[0]
        zero_next = None                # consumed atomic slab the next accumulating GEMV zeroes
        from ..utils import trace as _trace
        # prefill on the library GEMM path: dense weights of layer li + 1 are
        # dequantized on a side stream while layer li computes
        pf = T > ops.GEMV_MAX_M and x.is_cuda and ops.native_gpu(x) and not torch.cuda.is_current_stream_capturing()
        if pf:
            from ..ops.gemm import drop_prefetched, prefetch_dense
            drop_prefetched()          # entries of an earlier (aborted) forward are keyed by possibly reused pointers
            self._prefetch_layer(0, T, x.dtype, prefetch_dense)
        for li, layer in enumerate(self.layers):
            if pf and li + 1 < len(self.layers):
                self._prefetch_layer(li + 1, T, x.dtype, prefetch_dense)
            if _trace.ENABLED:
                # per-layer roctx marker (host-side: eager forwards / prefill)
                with _trace.trace_range(f"layer{li + self.layer_offset}"):
                    pass
            attn = layer.self_attn
            qp = attn.qkv_proj
            ss_q = None
            q = torch.empty(T, s.num_heads, s.head_dim, dtype=x.dtype, device=x.device)
            if x.is_cuda and isinstance(qp, LowBitLinear) and qp.mp_group is None and T <= ops.GEMV_MAX_M \
                    and (qp.bias is None or qp.bias.dtype == x.dtype) and ops.native_gpu(x):
                # split-K GEMV reduced (+bias) inside the RoPE/KV kernel, slots from the block table:
                # T <= 16 accumulates with atomics into one zeroed slab (re-zeroed by the kernel)
                if T <= ACC_MAX_M or rope_in:
                    part = self._acc(qp.out_features, T, x.device)
                    ss_q = None
                    if pend is not None:
                        r2 = nxt_res(residual)
                        ss_q = ss_all[2 * li] if defer else None
                        ops.gemv_norm_in(pend, residual, r2, layer.input_layernorm, s.rms_eps, s.norm_unit_offset,
                                         qp.weight, qp.fmt, qp.out_features, qp.in_features, False, acc_out=part,
                                         ss=ss_q, rope=qrope, zero=zero_gu)
                        zero_gu = None
                        residual, consumed, pend = r2, pend, None
                    else:
                        ops.gemv_accum(x, qp.weight, qp.fmt, qp.out_features, qp.in_features, part,
                                       zero=zero_next, rope=qrope)
                        zero_next = None
                    qkv_acc = part
                    part = part.unsqueeze(0)
                else:
                    part = ops.gemv_partials(x, qp.weight, qp.fmt, qp.out_features, qp.in_features, 0)
                if not rope_in:
                    ops.rope_kv_fused(part, qp.bias, q, cache.k[li], cache.v[li], pos, meta.block_tables, meta.Tq,
                                      rope, s.num_heads, s.num_kv_heads, s.head_dim, s.rot_dim, s.rope_interleaved,
                                      attn.q_norm, attn.k_norm, s.rms_eps, 1.0, cache.kv_fp8, cache.k_scale,
                                      cache.v_scale, meta.pos_offset, zero_part=T <= ACC_MAX_M,
                                      pss=ss_q, pss_n=s.hidden_size, pss_eps=s.rms_eps)
                elif not (norm_in and self._oproj_combine and attn.o_proj.bias is None):
                    a_rope = ops.attn_decode_rope(qkv_acc, qp.bias, self.rope_cache, pos, cache.k[li], cache.v[li],
                                                  meta.block_tables, meta.seq_lens, meta.nsplit, s.scale,
                                                  s.attn_softcap, attn.sliding_window, s.num_heads, s.rot_dim,
                                                  s.rope_interleaved, 1.0, x.dtype, pss=ss_q,
                                                  pss_n=s.hidden_size, pss_eps=s.rms_eps,
                                                  prerot=prerot).view(T, -1)
            else:
                qkv = attn.lf.qkv(x, cache.lf[li], slots, pos, meta, cache.bs) if attn.lf is not None else qp(x)
                ops.rope_kv(qkv, q, cache.k[li], cache.v[li], slots, pos, rope, s.num_heads,
                            s.num_kv_heads, s.head_dim, s.rot_dim, s.rope_interleaved, attn.q_norm, attn.k_norm,
                            s.rms_eps, 1.0, cache.kv_fp8, cache.k_scale, cache.v_scale)
            if self._capture_q is not None:            # SnapKV observation window
                self._capture_q[li] = q[-self._capture_w:].clone()
            if norm_in:
                # o_proj -> atomic slab P (zeroing the slab the qkv prologue consumed);
                # the gate/up GEMV adds P to the residual and normalises in its prologue;
                # down -> atomic slab D (zeroing P), pending for the next layer's qkv
                o, mlp = attn.o_proj, layer.mlp
                H = o.out_features
                accP, accD = self._acc(H, T, x.device, "P"), self._acc(H, T, x.device, "D")
                zero_qkv = None
                onorm = (ONORM and defer and ONORM_MIN_M <= T and not (T > DEFER_GLU_MAX_M and DEFER_MLP_ACC)
                         and o.mp_group is None and o.bias is None and H % 4 == 0
                         and not (rope_in and self._oproj_combine and o.bias is None))
                if rope_in and self._oproj_combine and o.bias is None:
                    # split attention without its combine launch: the o_proj GEMV
                    # merges each head's partials while staging its K slice (head-
                    # aligned slices: one head per workgroup), the qkv slab is
                    # zeroed by the gate/up launch below
                    po, pml = ops.attn_decode_rope_split(qkv_acc, qp.bias, self.rope_cache, pos, cache.k[li],
                                                         cache.v[li], meta.block_tables, meta.seq_lens, meta.nsplit,
                                                         s.scale, s.attn_softcap, attn.sliding_window, s.num_heads,
                                                         s.rot_dim, s.rope_interleaved, 1.0, x.dtype, pss=ss_q,
                                                         pss_n=s.hidden_size, pss_eps=s.rms_eps, prerot=prerot)
                    ops.gemv_attn(po, pml, meta.seq_lens, o.weight, o.fmt, H, o.in_features, accP,
                                  self._oproj_ks, x.dtype, zero=consumed, nw=self._oproj_nw)
                    zero_qkv = qkv_acc
                else:
                    a = a_rope if rope_in else self._attention(li, attn, q, meta, cache)
                    if onorm:
                        # o_proj + residual add + deferred-norm staging of the gate/up input
                        r2 = nxt_res(residual)
                        xo = self._acc(H, T, x.device, "XO", self.dtype)
                        ops.gemv_accum_norm(a, o.weight, o.fmt, H, o.in_features, accP, self._ctr(x.device),
                                            residual, r2, layer.post_attention_layernorm, s.norm_unit_offset, xo,
                                            ss_all[2 * li + 1], zero=consumed)
                        residual = r2
                    else:
                        ops.gemv_accum(a, o.weight, o.fmt, H, o.in_features, accP, 0, zero=consumed)
                self._reduce(accP, o)
                gu, dn = mlp.gate_up_proj, mlp.down_proj
                if onorm:
                    act = ops.gemv_glu_ss(xo, gu.weight, gu.fmt, gu.out_features, gu.in_features, s.act,
                                          ss_all[2 * li + 1], s.hidden_size, s.rms_eps)
                    ops.gemv_accum(act, dn.weight, dn.fmt, dn.out_features, dn.in_features, accD, 0, zero=zero_qkv)
                elif defer and T > DEFER_GLU_MAX_M and DEFER_MLP_ACC:
                    r2 = nxt_res(residual)
                    gacc = self._acc(gu.out_features, T, x.device, "GU")
                    ss2 = ss_all[2 * li + 1]
                    ops.gemv_norm_in(accP, residual, r2, layer.post_attention_layernorm, s.rms_eps,
                                     s.norm_unit_offset, gu.weight, gu.fmt, gu.out_features, gu.in_features, False,
                                     acc_out=gacc, zero=zero_qkv, ss=ss2)
                    residual = r2
                    ops.gemv_glu_in(gacc.unsqueeze(0), dn.weight, dn.fmt, dn.out_features, dn.in_features, s.act, 0,
                                    x.dtype, acc=accD, zero=accP, xss=ss2, xss_n=s.hidden_size, xss_eps=s.rms_eps)
                    zero_gu = gacc              # zeroed by the next layer's qkv launch (its readers are done)
                elif defer and T > DEFER_GLU_MAX_M:
                    # standalone residual-add + norm (re-zeroes P), plain GLU GEMV
                    xn, _ = ops.add_rms_norm(None, residual, layer.post_attention_layernorm, s.rms_eps,
                                             partials=accP.unsqueeze(0), unit_offset=s.norm_unit_offset,
                                             zero_partials=True)
                    act = ops.gemv_glu(xn, gu.weight, gu.fmt, gu.out_features, gu.in_features, s.act)
                    ops.gemv_accum(act, dn.weight, dn.fmt, dn.out_features, dn.in_features, accD, 0, zero=zero_qkv)
                else:
                    r2 = nxt_res(residual)
                    act = ops.gemv_norm_in(accP, residual, r2, layer.post_attention_layernorm, s.rms_eps,
                                           s.norm_unit_offset, gu.weight, gu.fmt, gu.out_features, gu.in_features,
                                           True, s.act, zero=zero_qkv, ss=ss_all[2 * li + 1] if defer else None)
                    residual = r2
                    ops.gemv_accum(act, dn.weight, dn.fmt, dn.out_features, dn.in_features, accD, 0, zero=accP)
                self._reduce(accD, dn)
                consumed = None
                if li + 1 < len(self.layers):
                    pend = accD
                else:   # last layer: the final (or stage-boundary) norm reads and re-zeroes D
                    nxt = self.norm if self.last_stage else layer.input_layernorm
                    x, _ = ops.add_rms_norm(None, residual, nxt, s.rms_eps, partials=accD.unsqueeze(0),
                                            unit_offset=s.norm_unit_offset, zero_partials=True)
                continue
            if not rope_in and self._attn_oproj_fuse_ok(attn, q, meta):
                x = self._attn_oproj_norm(li, attn, q, meta, cache, residual, layer.post_attention_layernorm)
            elif s.sandwich_norm:
                a = a_rope if rope_in else self._attention(li, attn, q, meta, cache)
                x = self._proj_residual_norm(a, attn.o_proj, residual, layer.pre_feedforward_layernorm,
                                             post_norm_w=layer.post_attention_layernorm)
            else:
                a = a_rope if rope_in else self._attention(li, attn, q, meta, cache)
                x = self._proj_residual_norm(a, attn.o_proj, residual, layer.post_attention_layernorm)
            if li + 1 < len(self.layers):
                nxt = self.layers[li + 1].input_layernorm
            else:   # stage boundary: the next norm lives on the next stage
                nxt = self.norm if self.last_stage else layer.input_layernorm
            if self._mlp_acc_ok(x, layer):
                # gate/up atomics into one f32 slab -> down GEMV applies act(g)*u while
                # staging its input, atomics into the norm's slab; the gate/up slab is
                # zeroed by the next layer's qkv GEMV (all its readers are done by then)
                gu, dn = layer.mlp.gate_up_proj, layer.mlp.down_proj
                gacc = self._acc(gu.out_features, x.shape[0], x.device, "GU")
                if zero_next is gacc:          # no accumulating launch in between took the zeroing
                    gacc.zero_()
                    zero_next = None
                ops.gemv_accum(x, gu.weight, gu.fmt, gu.out_features, gu.in_features, gacc, 0, zero=zero_next)
                dacc = self._acc(dn.out_features, x.shape[0], x.device)
                ops.gemv_glu_in(gacc.unsqueeze(0), dn.weight, dn.fmt, dn.out_features, dn.in_features, s.act, 0,
                                x.dtype, acc=dacc)
                self._reduce(dacc, dn)
                x, _ = ops.add_rms_norm(None, residual, nxt, s.rms_eps, partials=dacc.unsqueeze(0),
                                        unit_offset=s.norm_unit_offset, zero_partials=True)
                zero_next = gacc
                continue
            if self._fused_mlp_ok(x, layer):
                # gate/up split-K slabs -> down GEMV applies act(g)*u while staging its input
                gu, dn = layer.mlp.gate_up_proj, layer.mlp.down_proj
                pg = ops.gemv_partials(x, gu.weight, gu.fmt, gu.out_features, gu.in_features, 0)
                pd = ops.gemv_glu_in(pg, dn.weight, dn.fmt, dn.out_features, dn.in_features, s.act, 0, x.dtype)
                if dn.mp_group is not None:
                    pd = self._reduce(pd.sum(0, keepdim=True), dn)
                x, _ = ops.add_rms_norm(None, residual, nxt, s.rms_eps, partials=pd, unit_offset=s.norm_unit_offset)
                continue
            mlp = layer.mlp
            if type(mlp).__name__ == "NativeMoE" and layer.post_feedforward_layernorm is None \
                    and self.tp_group is None and x.shape[0] <= 16 and mlp.acc_ok(x):
                # MoE decode: routed experts (and a shared expert) add into the
                # norm's f32 slab; no combine launch, no [T, H] bf16 round trip.
                # Expert parallel: each rank adds its local experts' share, the
                # slab is summed over the EP group (one all-reduce per block)
                acc = self._acc(s.hidden_size, x.shape[0], x.device)
                mlp.forward_acc(x, acc)
                if mlp.ep_group is not None:
                    from ..parallel.comm import all_reduce_inplace
                    r = all_reduce_inplace(acc, mlp.ep_group)
                    if r is not acc:
                        acc.copy_(r)
                x, _ = ops.add_rms_norm(None, residual, nxt, s.rms_eps, partials=acc.unsqueeze(0),
                                        unit_offset=s.norm_unit_offset, zero_partials=True)
                continue
            act = self._mlp(x, layer.mlp)
            if isinstance(layer.mlp, NativeMLP):
                x = self._proj_residual_norm(act, layer.mlp.down_proj, residual, nxt,
                                             post_norm_w=layer.post_feedforward_layernorm)
            else:
                y = act
                if layer.post_feedforward_layernorm is not None:
                    y = ops.rms_norm(y, layer.post_feedforward_layernorm, s.rms_eps, s.norm_unit_offset)
                x, _ = ops.add_rms_norm(y.contiguous(), residual, nxt, s.rms_eps, unit_offset=s.norm_unit_offset)
        if zero_next is not None:
            zero_next.zero_()
        if zero_gu is not None:
            zero_gu.zero_()
        if not self.last_stage:
            return residual
        if return_hidden:
            return x
        if logits_idx is not None:
            x = x.index_select(0, logits_idx)
        logits = self.lm_head(x.contiguous())
        if s.final_softcap:
            logits = torch.tanh(logits.float() / s.final_softcap) * s.final_softcap
        return logits.float()
