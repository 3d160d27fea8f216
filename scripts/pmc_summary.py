"""Average rocprofv3 counter values per kernel over the counter CSVs of a run directory:
python scripts/pmc_summary.py gpurun_out/pmc3 > table.md"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "counters*.csv"))):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
            name = row.get("Counter_Name") or row.get("Counter-Name")
            val = row.get("Counter_Value") or row.get("Counter-Value")
            if not name or val is None:
                continue
            short = k.split("(")[0][:70]
            g = row.get("Grid_Size") or row.get("Grid-Size")
            if g:
                short += f" [grid {g}]"
            acc[short][name].append(float(val))
names = sorted({n for v in acc.values() for n in v})
print("| kernel | " + " | ".join(names) + " |")
print("|---|" + "---:|" * len(names))
for k, v in acc.items():
    if not any(t in k for t in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("qgemm", "attn"))):
        continue
    cells = []
    for n in names:
        xs = v.get(n)
        cells.append(f"{sum(xs) / len(xs):.4g}" if xs else "")
    print(f"| `{k}` | " + " | ".join(cells) + " |")
