"""Summarise an engine trace (LOCALAI_AMD_TRACE): per-step durations and the host gaps between
consecutive engine steps (emit / schedule / upload time the GPU is idle)."""
import json
import sys

ev = json.load(open(sys.argv[1]))["traceEvents"]
steps = sorted((e for e in ev if e.get("ph") == "X" and e["name"] in ("prefill", "decode")), key=lambda e: e["ts"])
for kind in ("prefill", "decode"):
    ds = [e["dur"] for e in steps if e["name"] == kind]
    if ds:
        print(f"{kind}: {len(ds)} steps, total {sum(ds) / 1e3:.1f} ms, mean {sum(ds) / len(ds) / 1e3:.2f} ms")
gaps = [b["ts"] - (a["ts"] + a["dur"]) for a, b in zip(steps, steps[1:])]
gaps = [g for g in gaps if g < 50e3]  # ignore idle between waves
if gaps:
    gaps.sort()
    print(f"host gaps: {len(gaps)}, total {sum(gaps) / 1e3:.1f} ms, median {gaps[len(gaps) // 2]:.0f} us, "
          f"p90 {gaps[int(len(gaps) * .9)]:.0f} us")
dec = [e for e in steps if e["name"] == "decode"]
if dec:
    k = [e["args"].get("device_steps", 1) for e in dec]
    b = [e["args"].get("batch", 0) for e in dec]
    print(f"decode round trips: mean device steps {sum(k) / len(k):.2f}, mean batch {sum(b) / len(b):.1f}")
    per = sum(e["dur"] for e in dec) / max(1, sum(k))
    print(f"decode: {per / 1e3:.2f} ms per device step (host-timed, incl. sync + emit)")
