"""vLLM's OpenAI-server command line (reference
``SRC/vllm/xpu/entrypoints/openai/cli_args.py``): the flags a reference
deployment passes, with ``--load-in-low-bit``.  Flags that configure vLLM
internals with no counterpart here (swap space, tokenizer pools, LoRA
adapter modules, tool parsers...) are accepted and ignored so existing
launch scripts keep working; ``unsupported()`` names the ones that were set."""
from __future__ import annotations

import argparse

# accepted for compatibility, no effect (value-taking flags)
_IGNORED_VALUE = ["--swap-space", "--tokenizer-mode", "--served-model-name-alias", "--chat-template",
                  "--response-role", "--lora-modules", "--prompt-adapters", "--tool-call-parser",
                  "--max-seq-len-to-capture", "--distributed-executor-backend", "--kv-cache-dtype",
                  "--pipeline-parallel-size", "--quantization", "--revision", "--download-dir",
                  "--allowed-origins", "--allowed-methods", "--allowed-headers", "--uvicorn-log-level",
                  "--max-num-batched-tokens"]
_IGNORED_FLAG = ["--disable-log-requests", "--disable-log-stats", "--allow-credentials", "--enable-auto-tool-choice",
                 "--disable-custom-all-reduce", "--enable-chunked-prefill", "--disable-frontend-multiprocessing"]


def make_arg_parser(parser: argparse.ArgumentParser = None) -> argparse.ArgumentParser:
    p = parser or argparse.ArgumentParser(description="ipex_llm_amd OpenAI-compatible server (vLLM command line)")
    p.add_argument("--model", required=True, help="HF checkpoint directory or hub id")
    p.add_argument("--tokenizer", default=None)
    p.add_argument("--served-model-name", default=None)
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--api-key", default=None, help="required bearer token (Authorization header)")
    p.add_argument("--load-in-low-bit", default="sym_int4", help="ipex-llm low-bit format of the linears")
    p.add_argument("--dtype", default="auto", choices=["auto", "bfloat16", "float16", "half"])
    p.add_argument("--max-model-len", type=int, default=4096)
    p.add_argument("--max-num-seqs", type=int, default=64)
    p.add_argument("--block-size", type=int, default=64)
    p.add_argument("--gpu-memory-utilization", type=float, default=0.9)
    p.add_argument("--tensor-parallel-size", "-tp", type=int, default=1)
    p.add_argument("--enforce-eager", action="store_true")
    p.add_argument("--enable-prefix-caching", action=argparse.BooleanOptionalAction, default=True)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--trust-remote-code", action="store_true")
    p.add_argument("--device", default=None)
    for f in _IGNORED_VALUE:
        p.add_argument(f, default=None, help=argparse.SUPPRESS)
    for f in _IGNORED_FLAG:
        p.add_argument(f, action="store_true", help=argparse.SUPPRESS)
    return p


def unsupported(args) -> list:
    """the compatibility-only flags that were set (logged by the server)"""
    out = []
    for f in _IGNORED_VALUE:
        if getattr(args, f[2:].replace("-", "_"), None) is not None:
            out.append(f)
    for f in _IGNORED_FLAG:
        if getattr(args, f[2:].replace("-", "_"), False):
            out.append(f)
    return out
