"""Prometheus metrics (`core/services/metrics.go`: histogram `api_call{method,path}`), plus the
serving metrics the reference lacks: TTFT, inter-token latency, token counters, per-model
engine gauges (batch size, KV blocks, prefix-cache hit ratio, HBM in use)."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

CONTENT_TYPE = "text/plain; version=0.0.4; charset=utf-8"


class Metrics:
    def __init__(self):
        self.registry = CollectorRegistry()
        r = self.registry
        self.api_call = Histogram("api_call", "api calls", ["method", "path"], registry=r)
        self.ttft = Histogram("localai_ttft_seconds", "time to first token", ["model"], registry=r,
                              buckets=(0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1, 2, 5, 10, 30))
        self.itl = Histogram("localai_inter_token_latency_seconds", "mean inter-token latency per request",
                             ["model"], registry=r,
                             buckets=(0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1))
        self.out_tokens = Counter("localai_output_tokens_total", "generated tokens", ["model"], registry=r)
        self.prompt_tokens = Counter("localai_prompt_tokens_total", "prompt tokens", ["model"], registry=r)
        self.requests = Counter("localai_requests_total", "inference requests", ["model", "endpoint"], registry=r)
        self.running = Gauge("localai_engine_running_sequences", "sequences being decoded", ["model"], registry=r)
        self.waiting = Gauge("localai_engine_waiting_sequences", "queued sequences", ["model"], registry=r)
        self.kv_free = Gauge("localai_engine_kv_blocks_free", "free KV pages", ["model"], registry=r)
        self.prefix_hit = Gauge("localai_engine_prefix_cache_hit_ratio", "prefix cache hit ratio", ["model"],
                                registry=r)
        self.hbm_used = Gauge("localai_gpu_hbm_used_bytes", "HBM in use", ["device"], registry=r)

    def observe_engines(self, manager):
        for lm in manager.list_loaded():
            sv = getattr(lm, "servicer", None)
            eng = getattr(sv, "engine", None) if sv is not None else None
            if eng is None:
                continue
            s = eng.sched
            self.running.labels(lm.id).set(s.num_running)
            self.waiting.labels(lm.id).set(s.num_waiting)
            bm = s.blocks()
            self.kv_free.labels(lm.id).set(bm.num_free)
            q = bm.query_tokens
            self.prefix_hit.labels(lm.id).set((bm.hit_tokens / q) if q else 0.0)
            try:
                import torch
                if eng.device.type == "cuda":
                    free, tot = torch.cuda.mem_get_info(eng.device)
                    self.hbm_used.labels(str(eng.device)).set(tot - free)
            except Exception:
                pass

    def render(self) -> bytes:
        return generate_latest(self.registry)
