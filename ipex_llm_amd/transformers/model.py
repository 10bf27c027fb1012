"""HF-compatible AutoModel API with low-bit loading.

Reference: ``SRC/transformers/model.py`` -- ``_BaseAutoModelClass``
(``from_pretrained`` 106-388, ``from_gguf`` 391-408, ``load_convert``
411-528, ``load_low_bit`` 532-788), ``save_low_bit`` (59-103) and the
AutoModel* subclasses (791-833).

Usage (one import change from HF)::

    from ipex_llm_amd.transformers import AutoModelForCausalLM
    model = AutoModelForCausalLM.from_pretrained(path, load_in_4bit=True).to("cuda")
    model.save_low_bit("llama-int4")
    model = AutoModelForCausalLM.load_low_bit("llama-int4").to("cuda")

The low-bit checkpoint keeps the portable canonical (GGML-style planar)
layout (``model.safetensors``), ``config.json`` carries
``bigdl_transformers_low_bit`` (reference key) and ``illm_low_bit.json`` the
conversion flags needed to rebuild the module tree before loading.
"""
from __future__ import annotations

import copy
import json
import logging
import os
import types
from typing import Optional

import torch
import torch.nn as nn

from ..quantize import qtypes as Q
from .convert import ggml_convert_low_bit
from ..models.yuan import register as _register_yuan

_register_yuan()                     # model_type "yuan" (Yuan 2.0 LFA) known to the Auto* classes

logger = logging.getLogger("ipex_llm_amd")
LOW_BIT_META = "illm_low_bit.json"


def _resolve_qtype_from_kwargs(kwargs):
    load_in_4bit = kwargs.pop("load_in_4bit", False)
    load_in_8bit = kwargs.pop("load_in_8bit", False)
    load_in_low_bit = kwargs.pop("load_in_low_bit", None)
    qc = kwargs.pop("quantization_config", None)
    q = None
    if qc is not None:
        d = qc if isinstance(qc, dict) else (qc.to_dict() if hasattr(qc, "to_dict") else vars(qc))
        method = str(d.get("quant_method", "")).lower()
        if method in ("gptq", "awq"):
            q = "asym_int4"
            kwargs["_illm_prequant"] = (method, d)
        elif d.get("load_in_4bit") or d.get("bnb_4bit_quant_type"):
            q = "nf4" if d.get("bnb_4bit_quant_type", "nf4") == "nf4" else "sym_int4"
        elif d.get("load_in_8bit"):
            q = "sym_int8"
    if load_in_low_bit is not None:
        q = load_in_low_bit
    elif load_in_4bit and q is None:
        q = "sym_int4"
    elif load_in_8bit and q is None:
        q = "sym_int8"
    return q


def _checkpoint_quant_config(path):
    cfg_file = os.path.join(path, "config.json") if os.path.isdir(str(path)) else None
    if cfg_file is None or not os.path.exists(cfg_file):
        return None
    try:
        with open(cfg_file) as f:
            qc = json.load(f).get("quantization_config")
    except (OSError, ValueError):
        return None
    return qc if isinstance(qc, dict) else None


def load_in_pre_quant(path) -> bool:
    qc = _checkpoint_quant_config(path)
    return qc is not None and str(qc.get("quant_method", "")).lower() in ("gptq", "awq")


def save_low_bit(self, save_dir: str, *args, **kwargs):
    """Write config + portable low-bit weights (reference model.py:59-103)."""
    os.makedirs(save_dir, exist_ok=True)
    from safetensors.torch import save_file
    sd = {}
    for k, v in self.state_dict().items():
        sd[k] = v.detach().cpu().contiguous()
    # de-duplicate shared storage (tied weights) for safetensors
    seen = {}
    for k in list(sd):
        key = (sd[k].data_ptr(), sd[k].numel(), sd[k].dtype)
        if key in seen and sd[k].numel() > 0:
            sd[k] = sd[k].clone()
        seen[key] = k
    tp = getattr(self, "_tp", None)
    if tp is not None and tp["world"] > 1:
        # per-rank shard (reference: DeepSpeed AutoTP saves per rank); config + meta from rank 0
        save_file(sd, os.path.join(save_dir, f"model-tp{tp['rank']:02d}-of-{tp['world']:02d}.safetensors"),
                  metadata={"format": "pt"})
        if tp["rank"] != 0:
            import torch.distributed as dist
            dist.barrier(group=tp["group"])
            return
    else:
        save_file(sd, os.path.join(save_dir, "model.safetensors"), metadata={"format": "pt"})
    cfg = getattr(self, "config", None)
    if cfg is not None:
        cfg.bigdl_transformers_low_bit = Q.qtype_name(getattr(self, "_illm_qtype", Q.SYM_INT4))
        cfg.save_pretrained(save_dir)
    meta = {"qtype": Q.qtype_name(getattr(self, "_illm_qtype", Q.SYM_INT4)),
            "optimize_model": bool(getattr(self, "_illm_pre", False)),
            "modules_to_not_convert": getattr(self, "_illm_skip", []),
            "mixed_precision": bool(getattr(self, "_illm_mixed", False)),
            "format": "ipex_llm_amd/canonical-planar-v1"}
    if tp is not None and tp["world"] > 1:
        meta["tensor_parallel"] = int(tp["world"])
    if getattr(self, "_illm_qtype", None) in (Q.MOFQ4, Q.MOFQ8):
        # mixed_fp4 / mixed_fp8 pick a format per tensor: record the plan
        from .low_bit_linear import LowBitLinear
        meta["module_qtypes"] = {n: Q.qtype_name(m.qtype) for n, m in self.named_modules()
                                 if isinstance(m, LowBitLinear)}
    with open(os.path.join(save_dir, LOW_BIT_META), "w") as f:
        json.dump(meta, f, indent=2)
    gc = getattr(self, "generation_config", None)
    if gc is not None:
        try:
            gc.save_pretrained(save_dir)
        except Exception:  # pragma: no cover
            pass
    if tp is not None and tp["world"] > 1:
        import torch.distributed as dist
        dist.barrier(group=tp["group"])


def _attach(model, qtype, flags):
    model.save_low_bit = types.MethodType(save_low_bit, model)
    model._illm_qtype = Q.resolve_qtype(qtype)
    model._illm_skip = list(flags.get("modules_to_not_convert") or [])
    model._illm_mixed = bool(flags.get("mixed_precision", False))
    return model


def _reinit_meta_buffers(model: nn.Module, config):
    """Non-persistent buffers (rotary inv_freq) stay on meta after an
    empty-weights build: re-create those modules on the host."""
    for name, mod in list(model.named_modules()):
        metas = [b for b in mod.buffers(recurse=False) if b.device.type == "meta"]
        if not metas:
            continue
        try:
            new = mod.__class__(config=config)
        except Exception:
            try:
                new = mod.__class__(config)
            except Exception:
                continue
        parent = model.get_submodule(name.rsplit(".", 1)[0]) if "." in name else model
        setattr(parent, name.rsplit(".", 1)[-1], new)


def _remote_family(path, kwargs) -> bool:
    """chatglm / qwen v1 checkpoint loaded through the native mapping (the
    default; ILLM_REMOTE_CODE=1 runs the checkpoint's own remote code instead)"""
    if os.environ.get("ILLM_REMOTE_CODE", "0") == "1":
        return False
    from .remote_families import family_of
    return family_of(path) is not None


class _BaseAutoModelClass:
    HF_Model = None

    @classmethod
    def from_pretrained(cls, *args, **kwargs):
        path = kwargs.pop("pretrained_model_name_or_path", None) if not args else args[0]
        args = args[1:] if args else ()
        qtype = _resolve_qtype_from_kwargs(kwargs)
        optimize_model = kwargs.pop("optimize_model", True)
        modules_to_not_convert = kwargs.pop("modules_to_not_convert", None)
        speculative = kwargs.pop("speculative", False)
        pp_stages = kwargs.pop("pipeline_parallel_stages", 1)
        imatrix = kwargs.pop("imatrix", None)
        embedding_qtype = kwargs.pop("embedding_qtype", None)
        mixed_precision = kwargs.pop("mixed_precision", False)
        cpu_embedding = kwargs.pop("cpu_embedding", False)
        disk_embedding = kwargs.pop("disk_embedding", False)
        kv_fp8 = kwargs.pop("kv_cache_fp8", None)
        tensor_parallel = kwargs.pop("tensor_parallel", False)
        expert_parallel = kwargs.pop("expert_parallel", False)
        tp_group = kwargs.pop("tp_group", None)
        kwargs.pop("model_hub", None)
        prequant = kwargs.pop("_illm_prequant", None)
        if prequant is None and path is not None and (qtype is not None or load_in_pre_quant(path)):
            qc = _checkpoint_quant_config(path)
            if qc is not None and str(qc.get("quant_method", "")).lower() in ("gptq", "awq"):
                # GPTQ / AWQ checkpoints always load as asym_int4 (reference model.py)
                prequant = (str(qc["quant_method"]).lower(), qc)
                qtype = "asym_int4"
        torch_dtype = kwargs.pop("torch_dtype", kwargs.pop("dtype", "auto"))
        if qtype is None:
            return cls.HF_Model.from_pretrained(path, *args, torch_dtype=torch_dtype, **kwargs)
        kwargs.setdefault("low_cpu_mem_usage", True)
        if prequant is not None:
            from ..gptq import load_gptq_model
            model = load_gptq_model(cls.HF_Model, path, prequant, torch_dtype=torch_dtype, **kwargs)
        elif _remote_family(path, kwargs):
            # chatglm / qwen v1: the checkpoint re-expressed as the in-library
            # Glm / Qwen2 model (remote_families.py), then the normal path
            from .remote_families import load_remote_family
            model = load_remote_family(path, torch_dtype)
        else:
            from .patches import remote_code_patches
            with remote_code_patches():        # remote code importing flash_attn stays loadable
                model = cls.HF_Model.from_pretrained(path, *args, torch_dtype=torch_dtype, **kwargs)
        model = model.to("cpu")
        if tensor_parallel or tp_group is not None:
            # AutoTP on the dense weights; each rank quantizes only its shard
            from ..parallel.tp import auto_tp
            auto_tp(model, tp_group)
            # decode-sized row-parallel messages take the xGMI peer all-reduce
            # (RCCL stays the fallback for large / ineligible messages)
            tp = getattr(model, "_tp", None)
            if tp is not None:
                from ..parallel.comm import setup_custom_all_reduce
                setup_custom_all_reduce(tp["group"])
        if expert_parallel:
            # each rank keeps (and quantizes) only its experts
            from ..parallel.ep import shard_experts
            shard_experts(model, None if expert_parallel is True else expert_parallel)
        imatrix_data = None
        if imatrix is not None:
            from ..quantize.imatrix import load_imatrix
            imatrix_data = load_imatrix(imatrix, model)
        ggml_convert_low_bit(model, qtype, optimize_model, None, modules_to_not_convert,
                             imatrix_data=imatrix_data, embedding_qtype=embedding_qtype,
                             mixed_precision=mixed_precision, cpu_embedding=cpu_embedding,
                             disk_embedding=disk_embedding)
        _attach(model, qtype, {"modules_to_not_convert": modules_to_not_convert,
                               "mixed_precision": mixed_precision})
        if kv_fp8 or os.environ.get("IPEX_LLM_QUANTIZE_KV_CACHE", "0") == "1":
            model._illm_kv_fp8 = True
        if speculative:
            from ..generation.speculative import enable_self_speculative
            enable_self_speculative(model, path, torch_dtype=torch_dtype, **kwargs)
        if pp_stages > 1:
            from ..parallel.pipeline import pipeline_parallel
            model = pipeline_parallel(model, pp_stages)
        return model

    @classmethod
    def from_gguf(cls, fpath: str, optimize_model: bool = True, cpu_embedding: bool = False,
                  low_bit: str = "sym_int4", keep_kquant: bool = True, torch_dtype=torch.float16):
        """Load a GGUF file (reference model.py:391-408 / gguf/api.py).
        ``keep_kquant``: Q2_K/Q4_K/Q5_K/Q6_K projections keep their GGUF
        blocks (native k-quant kernels); other tensors go to ``low_bit``."""
        from ..gguf.api import load_gguf_model
        model, tokenizer = load_gguf_model(fpath, dtype=torch_dtype, keep_kquant=keep_kquant)
        ggml_convert_low_bit(model, low_bit, optimize_model, cpu_embedding=cpu_embedding)
        _attach(model, low_bit, {})
        return model, tokenizer

    @classmethod
    def load_convert(cls, q_k, optimize_model, *args, **kwargs):
        kwargs["load_in_low_bit"] = q_k
        kwargs["optimize_model"] = optimize_model
        return cls.from_pretrained(*args, **kwargs)

    @classmethod
    def load_low_bit(cls, pretrained_model_name_or_path, *model_args, **kwargs):
        """Rebuild the module tree on meta, convert shapes only, stream the
        saved blobs in (reference model.py:532-788)."""
        from accelerate import init_empty_weights
        from safetensors.torch import load_file
        from transformers import AutoConfig
        path = pretrained_model_name_or_path
        trust = kwargs.pop("trust_remote_code", False)
        torch_dtype = kwargs.pop("torch_dtype", kwargs.pop("dtype", None))
        kwargs.pop("optimize_model", None)
        from .patches import remote_code_patches
        with remote_code_patches():
            config = AutoConfig.from_pretrained(path, trust_remote_code=trust)
        meta_path = os.path.join(path, LOW_BIT_META)
        flags = json.load(open(meta_path)) if os.path.exists(meta_path) else {}
        from .ref_checkpoint import OUR_FORMAT, is_reference_low_bit_dir
        ref_layout = is_reference_low_bit_dir(path)
        if flags and flags.get("format", OUR_FORMAT) != OUR_FORMAT:
            raise ValueError(f"load_low_bit: unknown low-bit layout {flags.get('format')!r} in {meta_path}")
        if not flags and not ref_layout:
            raise ValueError(f"load_low_bit: {path} is not a low-bit checkpoint (no {LOW_BIT_META} and no "
                             "bigdl_transformers_low_bit in config.json)")
        qtype = flags.get("qtype") or getattr(config, "bigdl_transformers_low_bit", "sym_int4")
        dt = torch_dtype if isinstance(torch_dtype, torch.dtype) else \
            getattr(config, "torch_dtype", None) or torch.float16
        if isinstance(dt, str):
            dt = getattr(torch, dt)
        with init_empty_weights():
            model = cls.HF_Model.from_config(config, torch_dtype=dt, trust_remote_code=trust)
        tp_world = int(flags.get("tensor_parallel", 1) or 1)
        tp_group = kwargs.pop("tp_group", None)
        want_tp = kwargs.pop("tensor_parallel", False) or tp_group is not None
        if tp_world > 1:
            # per-rank TP checkpoint: shard the empty module tree exactly like
            # from_pretrained(tensor_parallel=True) did, then load this rank's file
            from ..parallel.comm import get_rank, get_world_size
            from ..parallel.tp import auto_tp
            if get_world_size(tp_group) != tp_world:
                raise ValueError(f"load_low_bit: checkpoint was saved with tensor_parallel={tp_world}, "
                                 f"running with {get_world_size(tp_group)} ranks")
            auto_tp(model, tp_group)
        elif want_tp:
            raise ValueError("load_low_bit: tensor_parallel needs a checkpoint saved under tensor parallelism")
        from . import convert as _cv
        _cv._MIXED_PLAN[0] = flags.get("module_qtypes")
        try:
            ggml_convert_low_bit(model, qtype, flags.get("optimize_model", True), None,
                                 flags.get("modules_to_not_convert"), convert_shape_only=True,
                                 mixed_precision=flags.get("mixed_precision", False))
        finally:
            _cv._MIXED_PLAN[0] = None
        wfile = os.path.join(path, "model.safetensors")
        if tp_world > 1:
            wfile = os.path.join(path, f"model-tp{get_rank(tp_group):02d}-of-{tp_world:02d}.safetensors")
        if ref_layout:
            # reference save_low_bit: ggml CPU-layout blocks, converted (never reinterpreted)
            from .ref_checkpoint import convert_reference_state_dict, load_reference_state_dict
            sd = convert_reference_state_dict(load_reference_state_dict(path), model, qtype)
        elif os.path.exists(wfile):
            sd = load_file(wfile)
        else:
            sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
        missing, unexpected = model.load_state_dict(sd, strict=False, assign=True)
        out_emb = model.get_output_embeddings() if hasattr(model, "get_output_embeddings") else None
        head_saved = out_emb is not None and getattr(out_emb, "weight", None) is not None and \
            out_emb.weight.device.type != "meta" and not out_emb.weight.is_floating_point()
        # (a tied head quantized on its own -- low-bit blob in the checkpoint -- stays untied)
        if getattr(config, "tie_word_embeddings", False) and hasattr(model, "tie_weights") and not head_saved:
            try:
                model.tie_weights()
            except Exception:  # pragma: no cover
                pass
        _reinit_meta_buffers(model, config)
        still_meta = [n for n, p in model.named_parameters() if p.device.type == "meta"]
        if still_meta:
            raise RuntimeError(f"load_low_bit: parameters left uninitialised: {still_meta[:5]}")
        _attach(model, qtype, flags)
        if tp_world > 1 and getattr(model, "_tp", None) is not None:
            from ..parallel.comm import setup_custom_all_reduce
            setup_custom_all_reduce(model._tp["group"])
        from .convert import _optimize_post
        if flags.get("optimize_model", True):
            _optimize_post(model)
        try:
            from transformers import GenerationConfig
            model.generation_config = GenerationConfig.from_pretrained(path)
        except Exception:
            pass
        return model.eval()


def _hf(name):
    import transformers
    return getattr(transformers, name)


class _Lazy(type):
    def __getattribute__(cls, item):
        if item == "HF_Model":
            return _hf(type.__getattribute__(cls, "_hf_name"))
        return type.__getattribute__(cls, item)


class AutoModelForCausalLM(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForCausalLM"


class AutoModel(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModel"


class AutoModelForSpeechSeq2Seq(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForSpeechSeq2Seq"


class AutoModelForSeq2SeqLM(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForSeq2SeqLM"


class AutoModelForSequenceClassification(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForSequenceClassification"


class AutoModelForMaskedLM(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForMaskedLM"


class AutoModelForQuestionAnswering(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForQuestionAnswering"


class AutoModelForNextSentencePrediction(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForNextSentencePrediction"


class AutoModelForMultipleChoice(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForMultipleChoice"


class AutoModelForTokenClassification(_BaseAutoModelClass, metaclass=_Lazy):
    _hf_name = "AutoModelForTokenClassification"


class AutoModelForImageTextToText(_BaseAutoModelClass, metaclass=_Lazy):
    """vision-language models (qwen2_vl, mllama, llava, ... ; reference
    transformers/model.py Qwen2VL class and the vision examples)"""
    _hf_name = "AutoModelForImageTextToText"


# reference name of the same family
AutoModelForVision2Seq = AutoModelForImageTextToText
