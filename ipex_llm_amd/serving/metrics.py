"""Prometheus metrics of the serving engine.

Reference: the vLLM server's ``mount_metrics`` / ``PROMETHEUS_MULTIPROC_DIR``
(``SRC/vllm/xpu/entrypoints/openai/api_server.py:99, 210-215, 338-372``) and
the benchmark CSV columns (first-token / next-token latency).  SURVEY §5.5:
TTFT, TPOT, queue length and KV utilisation.

Each engine owns its own ``CollectorRegistry`` (several engines in one
process, e.g. tests, do not collide); ``/metrics`` on the API server renders
it in the Prometheus text format.
"""
from __future__ import annotations

from typing import Optional

try:
    from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
    from prometheus_client import CONTENT_TYPE_LATEST
    _OK = True
except Exception:  # pragma: no cover - prometheus_client is optional
    _OK = False
    CONTENT_TYPE_LATEST = "text/plain; version=0.0.4; charset=utf-8"

_LAT_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.02, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0)


class EngineMetrics:
    """Counters / histograms / gauges updated by ``LLMEngine``."""

    def __init__(self, model_name: str = "ipex-llm-amd"):
        self.enabled = _OK
        if not _OK:
            return
        self.registry = CollectorRegistry()
        lab = ["model"]
        self.model = model_name
        r = self.registry
        self.requests = Counter("ipex_llm_requests", "requests received", lab, registry=r)
        self.finished = Counter("ipex_llm_requests_finished", "requests finished by reason", lab + ["reason"],
                                registry=r)
        self.prompt_tokens = Counter("ipex_llm_prompt_tokens", "prefilled prompt tokens", lab, registry=r)
        self.prefix_hits = Counter("ipex_llm_prefix_cache_hit_tokens", "prompt tokens served from cached KV blocks",
                                   lab, registry=r)
        self.gen_tokens = Counter("ipex_llm_generation_tokens", "generated tokens", lab, registry=r)
        self.preemptions = Counter("ipex_llm_preemptions", "sequences preempted (recompute)", lab, registry=r)
        self.ttft = Histogram("ipex_llm_time_to_first_token_seconds", "time to first token", lab,
                              buckets=_LAT_BUCKETS, registry=r)
        self.tpot = Histogram("ipex_llm_time_per_output_token_seconds", "mean inter-token latency per request",
                              lab, buckets=_LAT_BUCKETS, registry=r)
        self.e2e = Histogram("ipex_llm_e2e_request_latency_seconds", "request latency", lab,
                             buckets=_LAT_BUCKETS, registry=r)
        self.step = Histogram("ipex_llm_engine_step_seconds", "one scheduler step (prefill + decode)", lab,
                              buckets=_LAT_BUCKETS, registry=r)
        self.running = Gauge("ipex_llm_num_requests_running", "sequences in the running batch", lab, registry=r)
        self.waiting = Gauge("ipex_llm_num_requests_waiting", "queued requests", lab, registry=r)
        self.kv_usage = Gauge("ipex_llm_kv_cache_usage_ratio", "fraction of KV blocks in use", lab, registry=r)

    # ------------------------------------------------------------ hooks
    def on_request(self, n_prompt: int):
        if self.enabled:
            self.requests.labels(self.model).inc()

    def on_prefill(self, n_tokens: int):
        if self.enabled:
            self.prompt_tokens.labels(self.model).inc(n_tokens)

    def on_prefix_hit(self, n_tokens: int):
        if self.enabled and n_tokens:
            self.prefix_hits.labels(self.model).inc(n_tokens)

    def on_tokens(self, n: int):
        if self.enabled and n:
            self.gen_tokens.labels(self.model).inc(n)

    def on_first_token(self, seconds: float):
        if self.enabled:
            self.ttft.labels(self.model).observe(seconds)

    def on_finish(self, reason: str, e2e_s: float, n_generated: int, first_token_s: Optional[float]):
        if not self.enabled:
            return
        self.finished.labels(self.model, reason.split(":")[0]).inc()
        self.e2e.labels(self.model).observe(e2e_s)
        if first_token_s is not None and n_generated > 1:
            self.tpot.labels(self.model).observe((e2e_s - first_token_s) / (n_generated - 1))

    def on_step(self, seconds: float, running: int, waiting: int, kv_used: float, preempted: int):
        if not self.enabled:
            return
        self.step.labels(self.model).observe(seconds)
        self.running.labels(self.model).set(running)
        self.waiting.labels(self.model).set(waiting)
        self.kv_usage.labels(self.model).set(kv_used)
        if preempted:
            self.preemptions.labels(self.model).inc(preempted)

    def render(self) -> bytes:
        if not self.enabled:
            return b"# prometheus_client not installed\n"
        return generate_latest(self.registry)
