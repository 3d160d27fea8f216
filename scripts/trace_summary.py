"""Summarise an engine trace (LOCALAI_AMD_TRACE=...json, utils/trace.py): per-phase totals,
decode-step size histogram, host gaps between GPU phases, request arrival spread.

    python scripts/trace_summary.py gpurun_out/trace_http.json [--from-s 0]
"""
import argparse
import collections
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-s", type=float, default=0.0, help="skip events before this many seconds")
    a = ap.parse_args()
    doc = json.load(open(a.trace))
    evs = doc["traceEvents"] if isinstance(doc, dict) else doc
    t_min = min(e["ts"] for e in evs if "ts" in e)
    evs = [e for e in evs if "ts" in e and (e["ts"] - t_min) / 1e6 >= a.from_s]
    phases = sorted((e for e in evs if e.get("ph") == "X" and e.get("name") in ("prefill", "decode")),
                    key=lambda e: e["ts"])
    tot = collections.Counter()
    n = collections.Counter()
    ks = collections.Counter()
    for e in phases:
        tot[e["name"]] += e["dur"]
        n[e["name"]] += 1
        if e["name"] == "decode":
            ks[(e["args"].get("device_steps"), min(256, e["args"].get("batch", 0)) // 32 * 32)] += 1
    gaps = [b["ts"] - (a_["ts"] + a_["dur"]) for a_, b in zip(phases, phases[1:])]
    span = (phases[-1]["ts"] + phases[-1]["dur"] - phases[0]["ts"]) if phases else 0
    print(f"span {span / 1e3:.1f} ms: prefill {tot['prefill'] / 1e3:.1f} ms in {n['prefill']} calls, "
          f"decode {tot['decode'] / 1e3:.1f} ms in {n['decode']} calls, host gaps {sum(gaps) / 1e3:.1f} ms "
          f"(max {max(gaps) / 1e3 if gaps else 0:.2f} ms)")
    print("decode calls by (device steps K, batch bucket):")
    for (k, b), c in sorted(ks.items()):
        print(f"  K={k} batch>={b}: {c}")
    arr = sorted(e["ts"] for e in evs if e.get("name") == "arrival")
    if arr:
        print(f"arrivals: {len(arr)} over {(arr[-1] - arr[0]) / 1e3:.1f} ms")
    pre = [e for e in phases if e["name"] == "prefill"]
    if pre:
        print("prefill calls (ms, seqs, tokens):", [(round(e["dur"] / 1e3, 1), e["args"].get("seqs"),
                                                      e["args"].get("tokens")) for e in pre[:24]])


if __name__ == "__main__":
    main()
