"""Streaming chat-completions load generator, run as separate client processes so the
measuring client never shares a GIL with the server under test.

    python -m localai_amd.utils.loadgen        (reads one JSON job per stdin line)

job  = {"url", "model", "contents": [...], "max_tokens": n | [n per content], "extra": {...}}
       (+ "offsets": [s per content] for open-loop arrivals)
reply= {"ttft": [s...], "tokens": n, "per": [n per content], "events": e, "merged": m, "bad": b,
        "lat": [s...], "gaps_ms": [...], "errors": k}   (one JSON line per job)

`tokens` is the server's final usage.completion_tokens.  The rest is counted on the wire: `events`
are the SSE events that carried generated text.  Every chunk carries the running usage (as the
reference's chat.go:41-53 does), so a token whose own text was empty (half of a UTF-8 sequence,
held back) shows up as a jump of 2+ in the next event's count (`merged`), a token whose text went
out in two events as an event that does not advance the count (`split`), and tokens after the
last text event (an incomplete UTF-8 sequence at the very end) as `tail`:
events - split + merged + tail == tokens for every well-formed stream.  `bad` counts streams whose
running count went backwards or ended above the final usage; `gaps_ms` are the per-token
inter-token latencies.
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
    offsets = job.get("offsets")
    gaps_ms: List[float] = []
    async with aiohttp.ClientSession(connector=conn, timeout=timeout) as sess:
        mt = job["max_tokens"]
        t_job = time.perf_counter()

        async def one(i, c):
            nonlocal errors
            if offsets:   # open-loop arrivals: this request is sent at its offset from the job start
                await asyncio.sleep(max(0.0, t_job + offsets[i] - time.perf_counter()))
            body = {"model": job["model"], "stream": True, "max_tokens": mt[i] if isinstance(mt, list) else mt,
                    "messages": [{"role": "user", "content": c}], **job.get("extra", {})}
            t0 = time.perf_counter()
            ttft = None
            ntok = 0     # the final usage.completion_tokens
            nev = 0      # events that carried generated text
            prev = 0     # running completion_tokens of the last text event (every chunk carries usage)
            merged = 0   # tokens that arrived inside a later event (their own text was empty)
            split = 0    # events that did not advance the count (a token's text sent in two parts)
            mono = True
            t_last = None
            try:
                async with sess.post(job["url"], json=body) as resp:
                    resp.raise_for_status()
                    async for raw in resp.content:
                        if not raw.startswith(b"data:"):
                            continue
                        data = raw[5:].strip()
                        if data == b"[DONE]":
                            break
                        u = data.rfind(b'"completion_tokens":')
                        cnt = None
                        if u >= 0:
                            e = u + 20
                            while data[e:e + 1].isdigit():
                                e += 1
                            cnt = int(data[u + 20:e])
                            ntok = cnt
                        if b'"content":""' not in data and (b'"content":"' in data or b'"text":"' in data):
                            now = time.perf_counter()
                            nev += 1
                            if ttft is None:
                                ttft = now - t0
                            if cnt is not None:
                                if cnt < prev:
                                    mono = False
                                elif cnt == prev:
                                    split += 1
                                else:
                                    if t_last is not None:
                                        gaps_ms.append((now - t_last) * 1e3 / (cnt - prev))
                                    merged += cnt - prev - 1
                                    prev = cnt
                            t_last = now
            except Exception:
                errors += 1
            ok = mono and ntok >= prev
            # tokens after the last text event (an incomplete UTF-8 sequence at the very end has no text)
            tail = max(0, ntok - prev)
            return ((ttft if ttft is not None else time.perf_counter() - t0), ntok, nev, merged, ok,
                    (t_last - t0) if t_last is not None else 0.0, split, tail)
        res = await asyncio.gather(*[one(i, c) for i, c in enumerate(job["contents"])])
    return {"ttft": [r[0] for r in res], "tokens": sum(r[1] for r in res), "per": [r[1] for r in res],
            "events": sum(r[2] for r in res), "merged": sum(r[3] for r in res),
            "split": sum(r[6] for r in res), "tail": sum(r[7] for r in res),
            "bad": sum(0 if r[4] else 1 for r in res), "lat": [r[5] for r in res],
            "gaps_ms": gaps_ms, "errors": errors}


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

    def wave(self, url: str, model: str, contents: List[str], max_tokens, extra=None,
             offsets: List[float] = None) -> Tuple[list, int]:
        """One concurrent wave; max_tokens: one budget for all, or a list (one per content);
        offsets: open-loop arrival time of each request (seconds from the wave start).
        Per-request completion counts (in content order) are left in self.last_per, the wire
        accounting (events, merged tokens, malformed streams, per-token gaps, latencies) in
        self.last_wire."""
        n = len(self.procs)
        parts = [contents[i::n] for i in range(n)]
        mts = [max_tokens[i::n] if isinstance(max_tokens, list) else max_tokens for i in range(n)]
        offs = [offsets[i::n] if offsets else None for i in range(n)]
        for p, part, mt, off in zip(self.procs, parts, mts, offs):
            job = {"url": url, "model": model, "contents": part, "max_tokens": mt, "extra": extra or {}}
            if off:
                job["offsets"] = off
            p.stdin.write(json.dumps(job) + "\n")
            p.stdin.flush()
        ttft, tokens, events, errors, merged, bad, split, tail = [], 0, 0, 0, 0, 0, 0, 0
        per = [0] * len(contents)
        lat = [0.0] * len(contents)
        tt = [0.0] * len(contents)
        gaps: List[float] = []
        for k, (p, part) in enumerate(zip(self.procs, parts)):
            r = json.loads(p.stdout.readline())
            ttft += r["ttft"]
            tokens += r["tokens"]
            events += r["events"]
            errors += r["errors"]
            merged += r.get("merged", 0)
            bad += r.get("bad", 0)
            split += r.get("split", 0)
            tail += r.get("tail", 0)
            gaps += r.get("gaps_ms", [])
            for j, v in enumerate(r.get("per", [])):
                per[k + j * n] = v
            for j, v in enumerate(r.get("lat", [])):
                lat[k + j * n] = v
            for j, v in enumerate(r["ttft"]):
                tt[k + j * n] = v
        if errors:
            raise RuntimeError(f"{errors} streaming requests failed")
        self.last_events = events
        self.last_per = per
        self.last_wire = {"events": events, "merged": merged, "split": split, "tail": tail, "bad": bad,
                          "gaps_ms": gaps, "lat": lat, "ttft": tt}
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
