"""Summarise a rocprofv3 --kernel-trace --stats run into a markdown table.

    python scripts/prof_summary.py <prof_dir> <title> [--decode-steps N] > profiles/<name>.md
"""
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)  # drop argument list
    n = n.replace("void ", "")
    n = re.sub(r"at::native::", "", n)
    if len(n) > 90:
        n = n[:87] + "..."
    return n


def main():
    d, title = sys.argv[1], sys.argv[2]
    steps = None
    if "--decode-steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--decode-steps") + 1])
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = list(csv.DictReader(open(stats[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    if trace:
        tr = list(csv.DictReader(open(trace[0])))
        t0 = min(int(r["Start_Timestamp"]) for r in tr)
        t1 = max(int(r["End_Timestamp"]) for r in tr)
        print(f"- kernels: {len(tr)} dispatches, busy {tot / 1e6:.1f} ms over a {(t1 - t0) / 1e6:.1f} ms window "
              f"({100 * tot / max(1, t1 - t0):.0f}% GPU-busy)")
    if steps:
        print(f"- per decode step: {tot / 1e3 / steps:.1f} us of kernel time ({steps} steps)")
    print("\n| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for r in rows[:25]:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")
    if trace and "--steady" in sys.argv:
        steady(tr, int(sys.argv[sys.argv.index("--steady") + 1]))


def steady(tr, n_layers):
    """Decode-only steady state: every dispatch after the last prefill-attention kernel, per
    decode step (= attn_decode dispatches / n_layers)."""
    pre = [int(r["End_Timestamp"]) for r in tr if "attn_prefill" in r["Kernel_Name"]]
    t_cut = max(pre) if pre else 0
    sel = [r for r in tr if int(r["Start_Timestamp"]) > t_cut]
    if not sel:
        return
    steps = sum(1 for r in sel if "attn_decode" in r["Kernel_Name"]) / n_layers
    agg = {}
    for r in sel:
        k = short(r["Kernel_Name"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c, t = agg.get(k, (0, 0))
        agg[k] = (c + 1, t + d)
    busy = sum(t for _, t in agg.values())
    span = max(int(r["End_Timestamp"]) for r in sel) - min(int(r["Start_Timestamp"]) for r in sel)
    print(f"\n## Decode steady state (after the last prefill kernel)\n")
    print(f"- {steps:.0f} decode steps, {busy / 1e3 / max(steps, 1):.1f} us kernel time per step, "
          f"{span / 1e3 / max(steps, 1):.1f} us wall per step ({100 * busy / max(span, 1):.0f}% GPU-busy)")
    print("\n| kernel | calls/step | us/step | avg us | % |\n|---|---:|---:|---:|---:|")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"| `{k}` | {c / max(steps, 1):.1f} | {t / 1e3 / max(steps, 1):.1f} | {t / c / 1e3:.1f} | "
              f"{100 * t / busy:.1f} |")


if __name__ == "__main__":
    main()


def by_grid(tr, n_layers, top=16):
    """Steady-state decode time per (kernel, grid size): separates the shapes one kernel serves
    (e.g. the GEMV's qkv / o / gate_up / down launches)."""
    pre = [int(r["End_Timestamp"]) for r in tr if "attn_prefill" in r["Kernel_Name"]]
    t_cut = max(pre) if pre else 0
    sel = [r for r in tr if int(r["Start_Timestamp"]) > t_cut]
    steps = sum(1 for r in sel if "attn_decode" in r["Kernel_Name"]) / n_layers
    gcol = next((c for c in ("Grid_Size", "Grid_Size_X", "grid_size") if c in sel[0]), None)
    agg = {}
    for r in sel:
        k = (short(r["Kernel_Name"]), r.get(gcol, "?") if gcol else "?")
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c, t = agg.get(k, (0, 0))
        agg[k] = (c + 1, t + d)
    print("\n## Steady state by (kernel, grid)\n\n| kernel | grid | calls/step | avg us | us/step |\n|---|---:|---:|---:|---:|")
    for (k, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"| `{k}` | {g} | {c / max(steps, 1):.1f} | {t / c / 1e3:.1f} | {t / 1e3 / max(steps, 1):.1f} |")


if __name__ == "__main__" and "--by-grid" in sys.argv:
    d = sys.argv[1]
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    by_grid(list(csv.DictReader(open(trace[0]))), int(sys.argv[sys.argv.index("--by-grid") + 1]))
