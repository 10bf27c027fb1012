"""``llm_patch``: one-line switch of transformers (and peft, when present)
to the MI355X low-bit implementations.

Reference: ``SRC/llm_patching.py:29-85`` (patches ``transformers.AutoModel*``,
``TrainingArguments`` and ``peft.get_peft_model``/``LoraConfig``/
``prepare_model_for_kbit_training``; ``llm_unpatch`` restores them).
"""
from __future__ import annotations

import importlib

_saved = {}
patched = None


def _set(mod, name, value):
    _saved.setdefault((mod.__name__, name), getattr(mod, name, None))
    setattr(mod, name, value)


def llm_patch(train: bool = False):
    global patched
    import transformers
    from . import transformers as ours
    for cls in ("AutoModelForCausalLM", "AutoModel", "AutoModelForSeq2SeqLM", "AutoModelForSpeechSeq2Seq",
                "AutoModelForSequenceClassification", "AutoModelForMaskedLM", "AutoModelForQuestionAnswering",
                "AutoModelForTokenClassification", "AutoModelForMultipleChoice"):
        if hasattr(ours, cls):
            _set(transformers, cls, getattr(ours, cls))
    if train:
        from .training import args as targs, lora
        _set(transformers, "TrainingArguments", targs.TrainingArguments)
        try:
            peft = importlib.import_module("peft")
            for name in ("get_peft_model", "LoraConfig", "prepare_model_for_kbit_training", "PeftModel"):
                _set(peft, name, getattr(lora, name))
        except ImportError:
            pass
    patched = "Train" if train else "Inference"
    return patched


def llm_unpatch():
    global patched
    for (modname, name), value in list(_saved.items()):
        mod = importlib.import_module(modname)
        if value is None:
            if hasattr(mod, name):
                delattr(mod, name)
        else:
            setattr(mod, name, value)
    _saved.clear()
    patched = None
