"""Streaming chat-completions load generator, run as separate client processes so the
measuring client never shares a GIL with the server under test.

    python -m localai_amd.utils.loadgen        (reads one JSON job per stdin line)

job  = {"url", "model", "contents": [...], "max_tokens": n | [n per content], "extra": {...}}
reply= {"ttft": [s...], "tokens": n, "per": [n per content], "events": e, "errors": k}   (one JSON line per job)

`tokens` is the server's final usage.completion_tokens; `events` is counted on the wire: the SSE
events that carried non-empty generated text (the server emits one per token, skipping tokens
whose text is empty, e.g. half of a UTF-8 sequence), so the caller can check the reported count
against what was actually streamed.
"""
from __future__ import annotations

import asyncio
import json
import os
import subprocess
import sys
import time
from typing import List, Tuple


async def _wave(job) -> dict:
    import aiohttp
    conn = aiohttp.TCPConnector(limit=0)
    timeout = aiohttp.ClientTimeout(total=3600)
    errors = 0
    async with aiohttp.ClientSession(connector=conn, timeout=timeout) as sess:
        mt = job["max_tokens"]

        async def one(i, c):
            nonlocal errors
            body = {"model": job["model"], "stream": True, "max_tokens": mt[i] if isinstance(mt, list) else mt,
                    "messages": [{"role": "user", "content": c}], **job.get("extra", {})}
            t0 = time.perf_counter()
            ttft = None
            ntok = 0
            nev = 0
            try:
                async with sess.post(job["url"], json=body) as resp:
                    resp.raise_for_status()
                    async for raw in resp.content:
                        if not raw.startswith(b"data:"):
                            continue
                        data = raw[5:].strip()
                        if data == b"[DONE]":
                            break
                        if b'"content":""' not in data and (b'"content":"' in data or b'"text":"' in data):
                            nev += 1
                            if ttft is None:
                                ttft = time.perf_counter() - t0
                        u = data.rfind(b'"completion_tokens":')
                        if u >= 0:
                            e = u + 20
                            while data[e:e + 1].isdigit():
                                e += 1
                            ntok = int(data[u + 20:e])
            except Exception:
                errors += 1
            return (ttft if ttft is not None else time.perf_counter() - t0), ntok, nev
        res = await asyncio.gather(*[one(i, c) for i, c in enumerate(job["contents"])])
    return {"ttft": [r[0] for r in res], "tokens": sum(r[1] for r in res), "per": [r[1] for r in res],
            "events": sum(r[2] for r in res), "errors": errors}


def _main():
    for line in sys.stdin:
        line = line.strip()
        if not line:
            continue
        job = json.loads(line)
        if job.get("quit"):
            break
        out = asyncio.run(_wave(job))
        sys.stdout.write(json.dumps(out) + "\n")
        sys.stdout.flush()


class LoadGen:
    """Pool of client processes; a wave's requests are split round-robin across them."""

    def __init__(self, n_procs: int = 2):
        env = dict(os.environ)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        env["CUDA_VISIBLE_DEVICES"] = ""  # clients never touch the GPU
        env["HIP_VISIBLE_DEVICES"] = ""
        self.procs = [subprocess.Popen([sys.executable, "-m", "localai_amd.utils.loadgen"], stdin=subprocess.PIPE,
                                       stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
                      for _ in range(max(1, n_procs))]

    def wave(self, url: str, model: str, contents: List[str], max_tokens, extra=None) -> Tuple[list, int]:
        """One concurrent wave; max_tokens: one budget for all, or a list (one per content).
        Per-request completion counts (in content order) are left in self.last_per."""
        n = len(self.procs)
        parts = [contents[i::n] for i in range(n)]
        mts = [max_tokens[i::n] if isinstance(max_tokens, list) else max_tokens for i in range(n)]
        for p, part, mt in zip(self.procs, parts, mts):
            p.stdin.write(json.dumps({"url": url, "model": model, "contents": part, "max_tokens": mt,
                                      "extra": extra or {}}) + "\n")
            p.stdin.flush()
        ttft, tokens, events, errors = [], 0, 0, 0
        per = [0] * len(contents)
        for k, (p, part) in enumerate(zip(self.procs, parts)):
            r = json.loads(p.stdout.readline())
            ttft += r["ttft"]
            tokens += r["tokens"]
            events += r["events"]
            errors += r["errors"]
            for j, v in enumerate(r.get("per", [])):
                per[k + j * n] = v
        if errors:
            raise RuntimeError(f"{errors} streaming requests failed")
        self.last_events = events
        self.last_per = per
        return ttft, tokens

    def close(self):
        for p in self.procs:
            try:
                p.stdin.write(json.dumps({"quit": True}) + "\n")
                p.stdin.flush()
                p.wait(10)
            except Exception:
                p.kill()


if __name__ == "__main__":
    _main()
