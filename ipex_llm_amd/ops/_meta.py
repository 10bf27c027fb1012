"""Fake (meta) implementations of the native ops, so torch.compile / export
and meta-device shape propagation can trace through them."""
from __future__ import annotations

import torch
from torch.library import register_fake

from .reference import dev_total as _dev_total


@register_fake("ipex_llm_amd::quantize_device")
def _(w, fmt, scale_search):
    return w.new_empty((_dev_total(fmt, w.shape[0], w.shape[1]),), dtype=torch.uint8)


@register_fake("ipex_llm_amd::dequantize_device")
def _(blob, fmt, n, k, dtype, transpose=False):
    return blob.new_empty((k, n) if transpose else (n, k), dtype=dtype)


@register_fake("ipex_llm_amd::gemv")
def _(x, blob, fmt, n, k, bias, epi, ksplit, act):
    M = x.numel() // k
    if epi == 1:
        return x.new_empty((max(ksplit, 1), M, n), dtype=torch.float32)
    shape = list(x.shape)
    shape[-1] = n // 2 if epi == 2 else n
    return x.new_empty(shape)


@register_fake("ipex_llm_amd::add_rms_norm")
def _(x, partials, residual, w, eps, unit_offset, store_residual, zero_partials=False):
    if x is not None:
        return torch.empty_like(x)
    if residual is not None:
        return torch.empty_like(residual)
    return w.new_empty((partials.shape[1], w.shape[0]))


@register_fake("ipex_llm_amd::rms_norm_bwd")
def _(x, g, w, eps, unit_offset):
    return torch.empty_like(x)


@register_fake("ipex_llm_amd::rope_half")
def _(x, cos, sin, bwd):
    return x.new_empty(x.shape)


@register_fake("ipex_llm_amd::act_mul")
def _(g, u, dy, act):
    if dy is None:
        return [torch.empty_like(g)]
    return [torch.empty_like(g), torch.empty_like(u)]


@register_fake("ipex_llm_amd::layer_norm")
def _(x, w, b, eps):
    return torch.empty_like(x)


@register_fake("ipex_llm_amd::rope_kv")
def _(qkv, q_out, k_cache, v_cache, slots, pos, inv_freq, q_norm, k_norm, norm_eps, q_scale, Hq, Hkv,
      D, rot_dim, interleaved, kv_fp8, k_scale, v_scale):
    return None


@register_fake("ipex_llm_amd::attn_decode")
def _(q, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap, window, kv_fp8, k_scale,
      v_scale, alibi):
    return torch.empty_like(q)


@register_fake("ipex_llm_amd::attn_softmax_")
def _(x):
    return None


@register_fake("ipex_llm_amd::glu")
def _(gu, act, tile=0):
    shape = list(gu.shape)
    shape[-1] //= 2
    return gu.new_empty(shape)


@register_fake("ipex_llm_amd::reduce_partials")
def _(ws, bias, dtype):
    return ws.new_empty(ws.shape[1:], dtype=dtype)


@register_fake("ipex_llm_amd::moe_topk")
def _(logits, k, renorm, scoring):
    T = logits.numel() // logits.shape[-1]
    return logits.new_empty((T, k), dtype=torch.float32), logits.new_empty((T, k), dtype=torch.int32)


@register_fake("ipex_llm_amd::moe_group_topk")
def _(logits, bias, k, n_group, topk_group, renorm, scale):
    T = logits.numel() // logits.shape[-1]
    return (logits.new_empty((T, k), dtype=torch.float32), logits.new_empty((T, k), dtype=torch.int32))


@register_fake("ipex_llm_amd::moe_align")
def _(ids, e0, num_local):
    return ids.new_empty((num_local + 1,), dtype=torch.int32), ids.new_empty((max(ids.numel(), 1),), dtype=torch.int32)


@register_fake("ipex_llm_amd::moe_gemv")
def _(x, blob, fmt, n, k, off, rows, xdiv, npairs, epi, ksplit, act):
    if epi == 2:
        return x.new_empty((npairs, n // 2))
    return x.new_empty((max(ksplit, 1), npairs, n), dtype=torch.float32)


@register_fake("ipex_llm_amd::moe_combine")
def _(part, w, ids, e0, num_local, dtype):
    return part.new_empty((w.numel() // w.shape[-1], part.shape[-1]), dtype=dtype)


@register_fake("ipex_llm_amd::moe_gemv_accum")
def _(x, blob, fmt, n, k, off, rows, acc, w, topk, ksplit):
    return None


@register_fake("ipex_llm_amd::moe_route")
def _(x, router, k, renorm, scoring, e0, num_local, counter):
    T = x.shape[0]
    return (x.new_empty((T, k), dtype=torch.float32), x.new_empty((T, k), dtype=torch.int32),
            x.new_empty((num_local + 1,), dtype=torch.int32), x.new_empty((T * k,), dtype=torch.int32))


@register_fake("ipex_llm_amd::rope_kv_fused")
def _(part, bias, q_out, k_cache, v_cache, pos, block_tables, tq, inv_freq, q_norm, k_norm, norm_eps, q_scale, Hq,
      Hkv, D, rot_dim, interleaved, kv_fp8, k_scale, v_scale, pos_offset=None, zero_part=False, pss=None, pss_n=0,
      pss_eps=0.0):
    return None


@register_fake("ipex_llm_amd::gemv_accum")
def _(x, blob, fmt, n, k, acc, ksplit, zero=None, rope_cs=None, rope_pos=None, rope_cols=0, rope_d=0):
    return None


@register_fake("ipex_llm_amd::gemv_accum_norm")
def _(x, blob, fmt, n, k, acc, ctr, residual, res_out, norm_w, unit_offset, xo, ss, zero=None):
    return None


@register_fake("ipex_llm_amd::gemv_glu_ss")
def _(x, blob, fmt, n, k, act, ss, ss_n, eps):
    return x.new_empty((x.numel() // k, n // 2))


@register_fake("ipex_llm_amd::gemv_norm_in")
def _(acc_in, residual, res_out, norm_w, eps, unit_offset, blob, fmt, n, k, epi, act, acc_out=None, zero=None,
      ss=None, rope_cs=None, rope_pos=None, rope_cols=0, rope_d=0):
    if epi == 2:
        return residual.new_empty((residual.numel() // k, n // 2))
    return torch.empty_like(acc_out)


@register_fake("ipex_llm_amd::gemv_glu_in")
def _(part, blob, fmt, n, k, act, ksplit, dtype, acc=None, zero=None, xss=None, xss_n=0, xss_eps=0.0):
    if acc is not None:
        return acc
    return part.new_empty((max(ksplit, 1), part.shape[1], n), dtype=torch.float32)


@register_fake("ipex_llm_amd::attn_prefill")
def _(q, k_cache, v_cache, block_tables, seq_lens, Tq, scale, softcap, window, kv_fp8, k_scale, v_scale):
    return torch.empty_like(q)


@register_fake("ipex_llm_amd::attn_decode_split")
def _(q, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap, window, kv_fp8, k_scale, v_scale, alibi):
    B, Tq, Hq, D = q.shape
    return (q.new_empty((B, Hq, Tq, nsplit, D), dtype=torch.float32),
            q.new_empty((B, Hq, Tq, nsplit, 2), dtype=torch.float32))


@register_fake("ipex_llm_amd::gemv_attn")
def _(po, pml, seq_lens, blob, fmt, n, k, acc, ksplit, dtype, zero=None, nw=0):
    M = po.shape[0] * po.shape[2]
    if acc is not None:
        return torch.empty_like(acc)
    return po.new_empty((max(ksplit, 1), M, n), dtype=torch.float32)


@register_fake("ipex_llm_amd::gemm")
def _(x, blob, fmt, n, k, bias):
    shape = list(x.shape)
    shape[-1] = n
    return x.new_empty(shape)


@register_fake("ipex_llm_amd::attn_decode_rope")
def _(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap, window, Hq,
      rot_dim, interleaved, q_scale, dtype, pss=None, pss_n=0, pss_eps=0.0, prerot=False):
    return part.new_empty((part.shape[0], 1, Hq, k_cache.shape[3]), dtype=dtype)


@register_fake("ipex_llm_amd::attn_decode_rope_split")
def _(part, bias, cos_sin, pos, k_cache, v_cache, block_tables, seq_lens, nsplit, scale, softcap, window, Hq,
      rot_dim, interleaved, q_scale, dtype, pss=None, pss_n=0, pss_eps=0.0, prerot=False):
    B, D = part.shape[0], k_cache.shape[3]
    return (part.new_empty((B, Hq, 1, nsplit, D)), part.new_empty((B, Hq, 1, nsplit, 2)))


@register_fake("ipex_llm_amd::gemm_glu")
def _(x, blob, fmt, n, k, act):
    shape = list(x.shape)
    shape[-1] = n // 2
    return x.new_empty(shape)


@register_fake("ipex_llm_amd::moe_gemm")
def _(x, blob, fmt, n, k, off, rows, xdiv, x_sorted, out_sorted, glu, act, out_f32):
    return x.new_empty((rows.shape[0], n // 2 if glu else n), dtype=torch.float32 if out_f32 else x.dtype)


@register_fake("ipex_llm_amd::rwkv_wkv4")
def _(time_decay, time_first, k, v, num, den, mx):
    return torch.empty_like(k)


@register_fake("ipex_llm_amd::rwkv_wkv5")
def _(w, u, r, k, v, state):
    return torch.empty_like(k, dtype=torch.float32)


@register_fake("ipex_llm_amd::fp8_act_quant")
def _(x):
    x2 = x.reshape(-1, x.shape[-1])
    return x2.new_empty(x2.shape, dtype=torch.uint8), x2.new_empty(x2.shape[0], dtype=torch.float32)


@register_fake("ipex_llm_amd::fp8_linear")
def _(x, w, w_scale, bias, e5m2):
    return x.new_empty(*x.shape[:-1], w.shape[0])


@register_fake("ipex_llm_amd::dense_linear")
def _(x, w, bias):
    return x.new_empty(*x.shape[:-1], w.shape[0])


@register_fake("ipex_llm_amd::kernel_errors")
def _(like, reset):
    return like.new_empty(4, dtype=torch.int32)


@register_fake("ipex_llm_amd::x_to_f16_rowscale")
def _(x):
    return [x.new_empty(x.shape, dtype=torch.float16), x.new_empty((x.shape[0],), dtype=torch.float32)]


@register_fake("ipex_llm_amd::ce_fused_")
def _(logits, labels, ignore_index=-100, grad_scale=0.0):
    return logits.new_empty((logits.shape[0],), dtype=torch.float32)


@register_fake("ipex_llm_amd::skinny_tn")
def _(a, b, alpha=1.0):
    return a.new_empty((a.shape[1], b.shape[1]), dtype=torch.float32)


@register_fake("ipex_llm_amd::lora_tn")
def _(a, b, alpha=1.0):
    return a.new_empty((a.shape[1], b.shape[1]), dtype=torch.float32)


@register_fake("ipex_llm_amd::dense_glu")
def _(x, w, act=0):
    return x.new_empty((*x.shape[:-1], w.shape[0] // 2))


@register_fake("ipex_llm_amd::lora_tn_acc_")
def _(out, a, b, alpha=1.0, trans=False):
    return out


@register_fake("ipex_llm_amd::lora_update_")
def _(c, a, b, alpha=1.0):
    return c


@register_fake("ipex_llm_amd::train_attn_fwd")
def _(q, k, v, scale, causal=True):
    B, H, T, D = q.shape
    return [q.new_empty((B, T, H, D)), q.new_empty((B, H, T), dtype=torch.float32)]


@register_fake("ipex_llm_amd::train_attn_bwd")
def _(q, k, v, out, lse, dout, scale, causal=True):
    return [torch.empty_like(q, memory_format=torch.contiguous_format),
            torch.empty_like(k, memory_format=torch.contiguous_format),
            torch.empty_like(v, memory_format=torch.contiguous_format)]


@register_fake("ipex_llm_amd::gemm_bf16")
def _(x, w, bias=None, out_f32=False, kernel=0, glu=False, act=0, ksplit=-1, out=None, accumulate=False):
    if out is not None:
        return out
    shape = list(x.shape)
    shape[-1] = w.shape[0] // 2 if glu else w.shape[0]
    return x.new_empty(shape, dtype=torch.float32 if out_f32 else x.dtype)


@register_fake("ipex_llm_amd::gemm8p_lowbit")
def _(x, blob, fmt, n, k, bias=None, out_f32=False, glu=False, act=0):
    shape = list(x.shape)
    shape[-1] = n // 2 if glu else n
    return x.new_empty(shape, dtype=torch.float32 if out_f32 else x.dtype)


@register_fake("ipex_llm_amd::fp8_gemm8p")
def _(xq, sx, w, ws, e5m2):
    return xq.new_empty((xq.shape[0], w.shape[0]), dtype=torch.bfloat16)


@register_fake("ipex_llm_amd::gemv_argmax")
def _gemv_argmax(x, blob, fmt, n, k, bias=None):
    M = x.numel() // k
    return x.new_empty(*x.shape[:-1], n), x.new_empty(((n + 15) // 16, M, 2), dtype=torch.float32)


@register_fake("ipex_llm_amd::dense_linear_t")
def _(x, w):
    return x.new_empty((w.shape[0], x.numel() // x.shape[-1]))
