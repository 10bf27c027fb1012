"""bench.py's multi-rank modes as a code-path smoke on the one-GPU test box:
2 ranks launched by torch.distributed.run share cuda:0 (gloo rendezvous, the
peer all-reduce / all-to-all forced over it: BENCH_SHARED_GPU=1), a reduced
model (2 layers, short prompts).  Checks the one JSON line of rank 0:
  * default data-parallel mode + its tensor-parallel side run (``tp_side``),
  * ``--tp`` (AutoTP, strong scaling),
  * ``--ep`` (token-sharded expert parallel, Mixtral architecture).
The 8-GPU numbers come from the driver's scaling run; this only proves the
paths the driver will take run end to end through the captured decode graph."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra):
    env = dict(os.environ, BENCH_SHARED_GPU="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--layers", "2", "--batch", "2",
           "--prompt-len", "64", *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_dp_with_tp_side():
    out = _run([])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["scaling"] == "weak"
    assert out["value"] > 0 and out["config"]["global_batch"] == 4
    tp = out["tp_side"]
    assert tp["parallelism"] == "tp2" and tp["scaling"] == "strong" and tp["value"] > 0
    assert tp["global_batch"] == 2


def _run_single():
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--layers", "2",
           "--batch", "2", "--prompt-len", "64"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


def test_bench_tp():
    """--tp over 2 ranks: the sharded model's next tokens equal the world-1
    run's (same weight seed and prompts; bench.py keeps both identical)"""
    out = _run(["--tp", "--no-tp-side"])
    assert out["config"]["parallelism"] == "tp2" and out["scaling"] == "strong" and out["value"] > 0
    assert "tp_side" not in out
    one = _run_single()
    assert one["n_gpus"] == 1 and one["config"]["parallelism"] == "dp1"
    assert out["sample_next_ids"] == one["sample_next_ids"], (out["sample_next_ids"], one["sample_next_ids"])


def test_bench_ep_mixtral():
    out = _run(["--ep", "--model", "mixtral-8x7b"])
    assert out["config"]["parallelism"] == "ep2" and out["config"]["model"] == "Mixtral-8x7B"
    assert out["value"] > 0 and "tp_side" not in out
