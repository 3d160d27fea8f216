"""Per-run host/device split of the decode phase in an engine trace (LOCALAI_AMD_TRACE): for the
last wave, every decode run's wall time (replay + sync + emit), its device steps, and the gap
to the next run (scheduling + input upload), so the exposed host time per step can be read off."""
import json
import sys

ev = json.load(open(sys.argv[1]))["traceEvents"]
steps = sorted((e for e in ev if e.get("ph") == "X" and e["name"] in ("prefill", "decode")), key=lambda e: e["ts"])
last_pf = max(i for i, s in enumerate(steps) if s["name"] == "prefill")
runs = [s for s in steps[last_pf + 1:] if s["name"] == "decode"]
tot_dur = tot_gap = 0.0
nsteps = 0
for a, b in zip(runs, runs[1:] + [None]):
    k = a.get("args", {}).get("device_steps", 1)
    gap = (b["ts"] - a["ts"] - a["dur"]) if b else 0.0
    tot_dur += a["dur"]
    tot_gap += gap
    nsteps += k
    print(f"run K={k:2d} batch={a.get('args', {}).get('batch')}: {a['dur'] / 1e3:7.2f} ms ({a['dur'] / 1e3 / k:5.2f}/step), gap {gap / 1e3:5.2f} ms")
print(f"{len(runs)} runs, {nsteps} steps: run wall {tot_dur / 1e3:.1f} ms, gaps {tot_gap / 1e3:.1f} ms, "
      f"{(tot_dur + tot_gap) / 1e3 / max(nsteps, 1):.2f} ms/step")
