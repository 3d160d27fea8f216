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


if __name__ == "__main__":
    main()
