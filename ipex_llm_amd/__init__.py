"""ipex_llm_amd -- an MI355X-native (CDNA4 / gfx950) low-bit LLM library with
the capabilities of IPEX-LLM: HF-compatible AutoModel API, GGML-style low-bit
checkpoints, hand-written HIP kernels (MFMA low-bit GEMV/GEMM, fused norms,
RoPE+KV, paged flash-decoding), hipGraph decode, RCCL tensor / pipeline /
expert parallelism and QLoRA finetuning.

Reference package: ``python/llm/src/ipex_llm/__init__.py`` (exports
``optimize_model`` and ``llm_convert``).
"""
__version__ = "0.1.0"


def optimize_model(*args, **kwargs):
    from .optimize import optimize_model as _om
    return _om(*args, **kwargs)


def llm_convert(*args, **kwargs):
    from .convert_model import llm_convert as _lc
    return _lc(*args, **kwargs)
