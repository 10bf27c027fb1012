"""Command line: chat / generate / serve / convert / env-check / bench.

Reference: ``SRC/cli/llm-cli`` and ``llm-chat`` (dispatch to the native
``main-<family>`` llama.cpp binaries), ``scripts/ipex-llm-init`` (env setup)
and ``env-check.sh``.  Here every command runs in-process on the native
engine:  ``python -m ipex_llm_amd.cli <command> ...``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _load(args):
    import torch
    from ..transformers import AutoModelForCausalLM
    if getattr(args, "load_low_bit", False):
        model = AutoModelForCausalLM.load_low_bit(args.model)
    elif args.model.endswith(".gguf"):
        model, tok = AutoModelForCausalLM.from_gguf(args.model, low_bit=args.low_bit)
        return model.to(args.device), tok
    else:
        model = AutoModelForCausalLM.from_pretrained(args.model, load_in_low_bit=args.low_bit,
                                                     torch_dtype=torch.bfloat16 if args.device != "cpu" else torch.float32)
    from transformers import AutoTokenizer
    tok = AutoTokenizer.from_pretrained(args.model)
    return model.to(args.device), tok


def cmd_generate(args):
    model, tok = _load(args)
    ids = tok(args.prompt, return_tensors="pt").input_ids.to(args.device)
    t0 = time.perf_counter()
    out = model.generate(ids, max_new_tokens=args.n_predict, do_sample=args.temperature > 0,
                         temperature=max(args.temperature, 1e-5))
    dt = time.perf_counter() - t0
    print(tok.decode(out[0][ids.shape[1]:], skip_special_tokens=True))
    print(f"\n[{out.shape[1] - ids.shape[1]} tokens, {dt:.2f} s, first {getattr(model, 'first_cost', 0) * 1e3:.1f} ms, "
          f"next {getattr(model, 'rest_cost_mean', 0) * 1e3:.2f} ms/token]", file=sys.stderr)


def cmd_chat(args):
    model, tok = _load(args)
    history = []
    print("chat (empty line or 'exit' quits)")
    for line in sys.stdin:
        line = line.strip()
        if not line or line == "exit":
            break
        history.append({"role": "user", "content": line})
        if getattr(tok, "chat_template", None):
            ids = tok.apply_chat_template(history, add_generation_prompt=True, return_tensors="pt")
        else:
            ids = tok("".join(f"{m['role']}: {m['content']}\n" for m in history) + "assistant:",
                      return_tensors="pt").input_ids
        ids = ids.to(args.device)
        out = model.generate(ids, max_new_tokens=args.n_predict)
        reply = tok.decode(out[0][ids.shape[1]:], skip_special_tokens=True)
        history.append({"role": "assistant", "content": reply})
        print(reply, flush=True)


def cmd_env_check(args):
    import platform
    info = {"python": platform.python_version(), "machine": platform.machine()}
    try:
        import torch
        info["torch"] = torch.__version__
        info["hip"] = getattr(torch.version, "hip", None)
        info["gpu_visible"] = torch.cuda.is_available()
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(0)
            info["gpu"] = {"name": p.name, "arch": getattr(p, "gcnArchName", ""), "mem_gb": round(p.total_memory / 2 ** 30, 1),
                           "count": torch.cuda.device_count()}
    except Exception as e:  # pragma: no cover
        info["torch_error"] = str(e)
    from .. import ops
    info["native_extension"] = ops.load(build_if_missing=False)
    from ..utils.device import check_avx2, check_avx512
    info["cpu"] = {"avx2": check_avx2(), "avx512": check_avx512(), "cores": os.cpu_count()}
    print(json.dumps(info, indent=2))
    return info


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ipex_llm_amd", description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)

    def model_args(p):
        p.add_argument("-m", "--model", required=True)
        p.add_argument("--low-bit", default="sym_int4")
        p.add_argument("--load-low-bit", action="store_true")
        p.add_argument("--device", default="cuda")
        p.add_argument("-n", "--n-predict", type=int, default=128)
        p.add_argument("-t", "--temperature", type=float, default=0.0)

    g = sub.add_parser("generate", help="one completion (llm-cli)")
    model_args(g)
    g.add_argument("-p", "--prompt", required=True)
    c = sub.add_parser("chat", help="interactive chat (llm-chat)")
    model_args(c)
    s = sub.add_parser("serve", help="OpenAI-compatible HTTP server")
    s.add_argument("rest", nargs=argparse.REMAINDER)
    cv = sub.add_parser("convert", help="HF -> low-bit directory or GGUF (llm-convert)")
    cv.add_argument("rest", nargs=argparse.REMAINDER)
    sub.add_parser("env-check", help="print the software / GPU environment")
    b = sub.add_parser("bench", help="decode benchmark (bench.py)")
    b.add_argument("rest", nargs=argparse.REMAINDER)
    ai = sub.add_parser("bench-all", help="all-in-one benchmark: YAML config -> CSV (dev/benchmark/all-in-one)")
    ai.add_argument("--config", default=None)
    ai.add_argument("--out", default="all_in_one.csv")
    ai.add_argument("--baseline", default=None, help="regression check against this CSV")
    ai.add_argument("--threshold", type=float, default=5.0)
    pp = sub.add_parser("ppl", help="strided perplexity of a text file (dev/benchmark/perplexity)")
    pp.add_argument("--model_path", required=True)
    pp.add_argument("--data_path", required=True)
    pp.add_argument("--precision", default="sym_int4")
    pp.add_argument("--chunk_size", type=int, default=512)
    pp.add_argument("--stride", type=int, default=0)
    pp.add_argument("--max_tokens", type=int, default=None)
    pp.add_argument("--device", default="cuda")
    a = ap.parse_args(argv)
    if a.cmd == "bench-all":
        from ..utils import all_in_one as A
        cfg = A.load_config(a.config)
        A.run(cfg, a.out)
        missing = A.check_results(a.out, cfg)
        out = {"csv": a.out, "missing": missing}
        if a.baseline:
            out["regressions"] = A.compare(a.baseline, a.out, a.threshold)
        print(json.dumps(out, indent=2))
        return 1 if missing or out.get("regressions") else 0
    if a.cmd == "ppl":
        import torch
        from transformers import AutoTokenizer
        from ..transformers import AutoModelForCausalLM
        from ..utils.perplexity import strided_perplexity, text_ids
        tok = AutoTokenizer.from_pretrained(a.model_path)
        model = AutoModelForCausalLM.from_pretrained(a.model_path, load_in_low_bit=a.precision,
                                                     torch_dtype=torch.float16 if a.device != "cpu" else torch.float32)
        model = model.to(a.device).eval()
        r = strided_perplexity(model, text_ids(tok, a.data_path, a.max_tokens), a.chunk_size, a.stride or None)
        print(json.dumps({"model": a.model_path, "precision": a.precision, **r}))
        return r
    if a.cmd == "generate":
        return cmd_generate(a)
    if a.cmd == "chat":
        return cmd_chat(a)
    if a.cmd == "serve":
        from ..serving.api_server import main as serve
        return serve(a.rest)
    if a.cmd == "convert":
        from ..convert_model import main as conv
        return conv(a.rest)
    if a.cmd == "env-check":
        return cmd_env_check(a)
    if a.cmd == "bench":
        import runpy
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        sys.argv = ["bench.py"] + a.rest
        runpy.run_path(os.path.join(root, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
