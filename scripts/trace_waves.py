"""Wave-level timeline of an engine trace (LOCALAI_AMD_TRACE) from a bench run: for every burst of
request arrivals, when arrivals start / end, when the first prefill step starts, when prefill ends,
first tokens (p50), the decode span, and the idle time before the next wave."""
import json
import sys

ev = json.load(open(sys.argv[1]))["traceEvents"]
arr = sorted(e["ts"] for e in ev if e.get("name") == "arrival")
ft = sorted(e["ts"] for e in ev if e.get("name") == "first_token")
steps = sorted((e for e in ev if e.get("ph") == "X" and e["name"] in ("prefill", "decode")), key=lambda e: e["ts"])
# waves: arrival bursts separated by > 100 ms
waves, cur = [], [arr[0]]
for t in arr[1:]:
    if t - cur[-1] > 100e3:
        waves.append(cur)
        cur = []
    cur.append(t)
waves.append(cur)
for i, w in enumerate(waves):
    a0, a1 = w[0], w[-1]
    nxt = waves[i + 1][0] if i + 1 < len(waves) else float("inf")
    st = [s for s in steps if a0 <= s["ts"] < nxt]
    pf = [s for s in st if s["name"] == "prefill"]
    dc = [s for s in st if s["name"] == "decode"]
    f = [t for t in ft if a0 <= t < nxt]
    end = max(s["ts"] + s["dur"] for s in st) if st else a1
    ms = lambda x: (x - a0) / 1e3  # noqa: E731
    print(f"wave {i}: {len(w)} arrivals over {ms(a1):.1f} ms; first prefill at {ms(pf[0]['ts']) if pf else -1:.1f}, "
          f"{len(pf)} prefill steps until {ms(pf[-1]['ts'] + pf[-1]['dur']) if pf else -1:.1f} ms "
          f"(busy {sum(s['dur'] for s in pf) / 1e3:.1f}); first tokens p50 {ms(sorted(f)[len(f) // 2]) if f else -1:.1f} "
          f"ms; {len(dc)} decode runs until {ms(end):.1f} ms; next wave after {(nxt - end) / 1e3 if nxt < 1e30 else 0:.1f} ms idle")
