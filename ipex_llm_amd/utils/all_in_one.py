"""All-in-one benchmark harness (YAML config -> CSV), with the regression
check against a baseline CSV.

Reference: ``python/llm/dev/benchmark/all-in-one/run.py`` + ``config.yaml``
(models x in-out pairs x batch sizes x ``test_api``; first-token and
next-token latency, peak memory, model loading time into one CSV per run,
columns ``run.py:596-600``), ``test/benchmark/check_results.py:24-65``
(completeness) and the 5 % regression threshold of
``csv_to_html.py -t 5.0`` in the reference's CI.

Here the timed generate is this library's (native engine where the family
has one: HIP-synchronised first / next token costs recorded by the engine;
otherwise the HF generate timed through a streamer, utils/benchmark.py).
No network: ``repo_id`` entries are local checkpoint directories (joined to
``local_model_hub``) or ``random:<arch>`` -- random-init weights of a named
architecture (``llama2-7b``, ``llama3-8b``, ``tiny-llama``) generated in
place, with synthetic prompt ids (the reference's own ``DUMMY_IDS`` mode).

    python -m ipex_llm_amd.cli bench-all --config config.yaml --out results.csv
"""
from __future__ import annotations

import csv
import os
import time
from typing import Dict, Iterable, List, Optional

import torch

from .benchmark import CSV_COLUMNS, BenchmarkWrapper, append_csv

DEFAULT_CONFIG = {
    "repo_id": ["random:tiny-llama"],
    "local_model_hub": "",
    "warm_up": 1,
    "num_trials": 3,
    "num_beams": 1,
    "low_bit": "sym_int4",
    "batch_size": 1,
    "in_out_pairs": ["32-32", "1024-128"],
    "test_api": ["transformer_int4_fp16_gpu"],
    "cpu_embedding": False,
    "streaming": False,
    "use_fp16_torch_dtype": True,
}

# test_api -> (device, torch dtype of the non-linear layers, loader)
APIS = {
    "transformer_int4_gpu": ("cuda", torch.float32, "auto"),
    "transformer_int4_fp16_gpu": ("cuda", torch.float16, "auto"),
    "transformer_int4_bf16_gpu": ("cuda", torch.bfloat16, "auto"),
    "optimize_model_gpu": ("cuda", torch.float16, "optimize"),
    "speculative_gpu": ("cuda", torch.bfloat16, "speculative"),
    "transformer_int4": ("cpu", torch.float32, "auto"),
    "optimize_model": ("cpu", torch.float32, "optimize"),
    "speculative_cpu": ("cpu", torch.bfloat16, "speculative"),
}

RANDOM_ARCHS = {
    "tiny-llama": dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=4096),
    "llama2-7b": dict(vocab_size=32000, hidden_size=4096, intermediate_size=11008, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=32, max_position_embeddings=4096),
    "llama3-8b": dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192,
                      rope_theta=500000.0),
}


def load_config(path: Optional[str] = None) -> Dict:
    cfg = dict(DEFAULT_CONFIG)
    if path:
        import yaml
        with open(path) as f:
            cfg.update(yaml.safe_load(f) or {})
    for k in ("repo_id", "in_out_pairs", "test_api"):
        if isinstance(cfg[k], str):
            cfg[k] = [cfg[k]]
    bs = cfg["batch_size"]
    cfg["batch_size"] = bs if isinstance(bs, list) else [bs]
    return cfg


def _model_path(repo: str, hub: str) -> str:
    if repo.startswith("random:"):
        return repo
    if hub and not os.path.isabs(repo):
        cand = os.path.join(hub, repo.split("/")[-1])
        if os.path.isdir(cand):
            return cand
        cand = os.path.join(hub, repo)
        if os.path.isdir(cand):
            return cand
    return repo


def load_model(repo: str, api: str, low_bit: str, hub: str = "", cpu_embedding: bool = False):
    """-> (model, vocab_size, load seconds)"""
    from ..transformers import AutoModelForCausalLM
    dev, dtype, how = APIS[api]
    if dev == "cuda" and not torch.cuda.is_available():
        raise RuntimeError(f"{api} needs a GPU")
    path = _model_path(repo, hub)
    t0 = time.perf_counter()
    if path.startswith("random:"):
        import tempfile
        from transformers import LlamaConfig, LlamaForCausalLM
        arch = path.split(":", 1)[1]
        if arch not in RANDOM_ARCHS:
            raise KeyError(f"unknown random architecture {arch!r} ({sorted(RANDOM_ARCHS)})")
        torch.manual_seed(0)
        with tempfile.TemporaryDirectory() as tmp:
            LlamaForCausalLM(LlamaConfig(**RANDOM_ARCHS[arch])).save_pretrained(tmp)
            model = _load(AutoModelForCausalLM, tmp, how, low_bit, dtype, cpu_embedding)
    else:
        model = _load(AutoModelForCausalLM, path, how, low_bit, dtype, cpu_embedding)
    model = model.to(dev).eval()
    if dev == "cuda":
        torch.cuda.synchronize()
    return model, model.config.vocab_size, time.perf_counter() - t0


def _load(auto, path, how, low_bit, dtype, cpu_embedding):
    kw = dict(torch_dtype=dtype, cpu_embedding=cpu_embedding)
    if how == "optimize":
        from transformers import AutoModelForCausalLM as HF
        from ..optimize import optimize_model
        return optimize_model(HF.from_pretrained(path, torch_dtype=dtype), low_bit=low_bit)
    if how == "speculative":
        return auto.from_pretrained(path, load_in_low_bit=low_bit, speculative=True, **kw)
    return auto.from_pretrained(path, load_in_low_bit=low_bit, **kw)


def run_one(model, vocab: int, in_len: int, out_len: int, batch: int, num_beams: int = 1, warm_up: int = 1,
            num_trials: int = 3) -> Dict:
    """first-token latency (ms), next-token latency (ms/token), actual token
    counts and peak memory over ``num_trials`` timed generate calls"""
    bm = BenchmarkWrapper(model)
    g = torch.Generator().manual_seed(in_len * 31 + batch)
    ids = torch.randint(3, vocab, (batch, in_len), generator=g)
    dev = next(model.parameters()).device
    ids = ids.to(dev)
    firsts, rests, out = [], [], None
    for t in range(warm_up + num_trials):
        out = bm.generate(ids, max_new_tokens=out_len, min_new_tokens=out_len, num_beams=num_beams,
                          do_sample=False)
        if t >= warm_up:
            firsts.append(bm.first_cost)
            rests.append(bm.rest_cost_mean)
    n_out = (out.shape[1] - in_len) if hasattr(out, "shape") else out_len
    return {"1st token avg latency (ms)": round(1e3 * sum(firsts) / len(firsts), 2),
            "2+ avg latency (ms/token)": round(1e3 * sum(rests) / len(rests), 2),
            "encoder time (ms)": 0.0,
            "input/output tokens": f"{in_len}-{out_len}",
            "actual input/output tokens": f"{in_len}-{n_out}",
            "batch_size": batch, "num_beams": num_beams,
            "peak mem (GB)": round(bm.peak_memory, 2)}


def run(cfg: Dict, out_csv: str, apis: Optional[Iterable[str]] = None, log=print) -> List[Dict]:
    rows = []
    for api in (apis or cfg["test_api"]):
        if api not in APIS:
            log(f"[all-in-one] test_api {api!r} not supported here, skipped")
            continue
        for repo in cfg["repo_id"]:
            try:
                model, vocab, load_s = load_model(repo, api, cfg["low_bit"], cfg.get("local_model_hub", ""),
                                                  cfg.get("cpu_embedding", False))
            except Exception as e:                      # keep going: the CSV records what ran
                log(f"[all-in-one] {repo} / {api}: load failed: {e}")
                continue
            for pair in cfg["in_out_pairs"]:
                i, o = (int(v) for v in str(pair).split("-"))
                for bs in cfg["batch_size"]:
                    r = run_one(model, vocab, i, o, bs, cfg.get("num_beams", 1), cfg.get("warm_up", 1),
                                cfg.get("num_trials", 3))
                    r.update({"model": repo, "low_bit": cfg["low_bit"], "cpu_embedding": cfg.get("cpu_embedding"),
                              "model loading time (s)": round(load_s, 2), "streaming": cfg.get("streaming"),
                              "use_fp16_torch_dtype": cfg.get("use_fp16_torch_dtype"), "test_api": api})
                    append_csv(out_csv, [r])
                    rows.append(r)
                    log(f"[all-in-one] {repo} {api} {pair} bs={bs}: first {r['1st token avg latency (ms)']} ms, "
                        f"next {r['2+ avg latency (ms/token)']} ms/token")
            del model
            if torch.cuda.is_available():
                torch.cuda.empty_cache()
    return rows


def read_csv(path: str) -> List[Dict]:
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def check_results(path: str, cfg: Dict) -> List[str]:
    """completeness (reference check_results.py): every model x in-out pair x
    batch of the config has a row; returns the missing combinations"""
    have = {(r["model"], r["input/output tokens"], str(r["batch_size"])) for r in read_csv(path)}
    return [f"{m} {p} bs={b}" for m in cfg["repo_id"] for p in cfg["in_out_pairs"] for b in cfg["batch_size"]
            if (m, str(p), str(b)) not in have]


def compare(baseline: str, current: str, threshold: float = 5.0) -> List[Dict]:
    """rows whose first- or next-token latency regressed by more than
    ``threshold`` percent against the baseline CSV (reference CI: -t 5.0)"""
    key = lambda r: (r["model"], r["input/output tokens"], str(r["batch_size"]), r.get("low_bit", ""))  # noqa: E731
    base = {key(r): r for r in read_csv(baseline)}
    bad = []
    for r in read_csv(current):
        b = base.get(key(r))
        if b is None:
            continue
        for col in ("1st token avg latency (ms)", "2+ avg latency (ms/token)"):
            old, new = float(b[col]), float(r[col])
            if old > 0 and (new - old) / old * 100 > threshold:
                bad.append({"row": key(r), "metric": col, "baseline": old, "current": new,
                            "change_pct": round((new - old) / old * 100, 2)})
    return bad


__all__ = ["CSV_COLUMNS", "DEFAULT_CONFIG", "APIS", "load_config", "load_model", "run_one", "run", "check_results",
           "compare", "read_csv"]
