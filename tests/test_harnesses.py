"""Benchmark / accuracy harnesses (reference dev/benchmark): the all-in-one
YAML -> CSV runner with its completeness and 5 % regression checks, and the
strided perplexity recipe (run_wikitext.py).  Tiny random models, CPU."""
import csv
import math

import pytest
import torch


def test_all_in_one_yaml_to_csv_and_checks(tmp_path):
    from ipex_llm_amd.utils import all_in_one as A
    cfg_path = tmp_path / "config.yaml"
    cfg_path.write_text("repo_id:\n  - 'random:tiny-llama'\nwarm_up: 1\nnum_trials: 2\nlow_bit: 'sym_int4'\n"
                        "batch_size: 1\nin_out_pairs:\n  - '16-4'\n  - '40-6'\ntest_api:\n  - 'transformer_int4'\n"
                        "  - 'transformer_int4_gpu'\n")
    cfg = A.load_config(str(cfg_path))
    assert cfg["batch_size"] == [1] and cfg["in_out_pairs"] == ["16-4", "40-6"]
    out = str(tmp_path / "r.csv")
    logs = []
    rows = A.run(cfg, out, log=logs.append)
    assert len(rows) == 2                         # the GPU api is skipped (logged) on a CPU box
    with open(out) as f:
        got = list(csv.DictReader(f))
    assert list(got[0].keys()) == A.CSV_COLUMNS
    assert {r["input/output tokens"] for r in got} == {"16-4", "40-6"}
    assert all(r["actual input/output tokens"] == r["input/output tokens"] for r in got)
    assert all(float(r["1st token avg latency (ms)"]) > 0 and float(r["2+ avg latency (ms/token)"]) > 0 for r in got)
    assert A.check_results(out, cfg) == []
    cfg2 = dict(cfg, in_out_pairs=["16-4", "40-6", "64-8"])
    assert A.check_results(out, cfg2) == ["random:tiny-llama 64-8 bs=1"]
    # regression check: +10 % first-token latency over the baseline is flagged at 5 %, not at 20 %
    slow = str(tmp_path / "slow.csv")
    with open(slow, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=A.CSV_COLUMNS)
        w.writeheader()
        for r in got:
            r = dict(r)
            r["1st token avg latency (ms)"] = str(float(r["1st token avg latency (ms)"]) * 1.10)
            w.writerow(r)
    bad = A.compare(out, slow, 5.0)
    assert len(bad) == 2 and all(b["metric"] == "1st token avg latency (ms)" for b in bad)
    assert A.compare(out, slow, 20.0) == []


def _tiny(tmp_path):
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=128, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512)
    m = LlamaForCausalLM(cfg).eval()
    p = str(tmp_path / "m")
    m.save_pretrained(p)
    return m, p


def test_strided_perplexity_matches_direct_nll(tmp_path):
    from ipex_llm_amd.utils.perplexity import strided_perplexity
    ref, _ = _tiny(tmp_path)
    ids = torch.randint(0, 128, (1, 96), generator=torch.Generator().manual_seed(3))
    # one window == the plain next-token NLL of the whole sequence
    r = strided_perplexity(ref, ids, max_length=96)
    with torch.no_grad():
        lg = ref(ids).logits[0, :-1].float()
    nll = torch.nn.functional.cross_entropy(lg, ids[0, 1:]).item()
    assert r["tokens"] == 95 and r["windows"] == 1
    assert abs(r["nll"] - nll) < 1e-5 and abs(r["ppl"] - math.exp(nll)) < 1e-3
    # disjoint windows: a window's first token has no context (HF recipe): 3 x 31;
    # overlapping windows score every token but the first exactly once
    d = strided_perplexity(ref, ids, max_length=32)
    assert d["windows"] == 3 and d["tokens"] == 93
    o = strided_perplexity(ref, ids, max_length=48, stride=16)
    assert o["tokens"] == 95


def test_lowbit_perplexity_close_to_dense(tmp_path):
    from ipex_llm_amd.transformers import AutoModelForCausalLM
    from ipex_llm_amd.utils.perplexity import strided_perplexity
    ref, p = _tiny(tmp_path)
    ids = torch.randint(0, 128, (1, 128), generator=torch.Generator().manual_seed(4))
    dense = strided_perplexity(ref, ids, max_length=64)
    m = AutoModelForCausalLM.from_pretrained(p, load_in_low_bit="sym_int8", torch_dtype=torch.float32).eval()
    q = strided_perplexity(m, ids, max_length=64)
    assert abs(q["ppl"] - dense["ppl"]) / dense["ppl"] < 0.02


@pytest.mark.gpu
def test_all_in_one_gpu_api(tmp_path):
    """transformer_int4_fp16_gpu on a random tiny llama: the native engine's
    HIP-synchronised first / next token costs land in the CSV"""
    from ipex_llm_amd.utils import all_in_one as A
    cfg = A.load_config(None)
    cfg.update(repo_id=["random:tiny-llama"], in_out_pairs=["64-8"], test_api=["transformer_int4_fp16_gpu"],
               num_trials=2, batch_size=[1, 2])
    out = str(tmp_path / "g.csv")
    rows = A.run(cfg, out)
    assert len(rows) == 2 and A.check_results(out, cfg) == []
    assert all(r["1st token avg latency (ms)"] > 0 and r["2+ avg latency (ms/token)"] > 0 for r in rows)
    assert all(r["peak mem (GB)"] > 0 for r in rows)
