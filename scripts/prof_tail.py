"""Per-kernel totals of the dispatches in the LAST `ms` milliseconds of a rocprofv3 kernel trace
(e.g. the final prefill-dominated wave of a bench run).

    python scripts/prof_tail.py <prof_dir> <ms> [title]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    d, ms = sys.argv[1], float(sys.argv[2])
    title = sys.argv[3] if len(sys.argv) > 3 else "tail window"
    tr = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
    t1 = max(int(r["End_Timestamp"]) for r in tr)
    lo = t1 - ms * 1e6
    win = [r for r in tr if int(r["Start_Timestamp"]) >= lo]
    agg = defaultdict(lambda: [0, 0.0])
    for r in win:
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    t0 = min(int(r["Start_Timestamp"]) for r in win)
    print(f"# {title}\n\n- last {ms:.0f} ms of the trace: {len(win)} dispatches, {busy / 1e3:.1f} ms busy over "
          f"{(t1 - t0) / 1e6:.1f} ms\n")
    print("| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"| `{k}` | {n} | {us / 1e3:.2f} | {us / n:.1f} | {100 * us / busy:.1f} |")


if __name__ == "__main__":
    main()
