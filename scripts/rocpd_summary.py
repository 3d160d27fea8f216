"""Per-kernel tables from a rocprofv3 database (rocpd sqlite, the default output of
`rocprofv3 --kernel-trace --stats -d DIR -o NAME -- ...`).

  python scripts/rocpd_summary.py DB [--top 25]
  python scripts/rocpd_summary.py DB --marker moe_router --marker-grid 65536 --per-step 32

With --marker: the steady-state window is the longest run of consecutive dispatches of the
marker kernel (name substring) launched with grid_x == marker-grid (e.g. the fused MoE router at
T tokens: grid_x = 256 * T); every kernel between the first and the last marker of that run is
averaged per step (marker count / per-step markers), so the table is one decode step."""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name)
    n = n.replace("void ", "")
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--marker", default="")
    ap.add_argument("--marker-grid", type=int, default=0)
    ap.add_argument("--per-step", type=int, default=1)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    if a.marker:
        idx = [i for i, r in enumerate(rows) if a.marker in r[0] and (not a.marker_grid or r[3] == a.marker_grid)]
        # longest run of markers with no other-grid marker in between
        other = {i for i, r in enumerate(rows) if a.marker in r[0]} - set(idx)
        best, cur = [], []
        for i in idx:
            if cur and any(cur[-1] < o < i for o in other):
                cur = []
            cur.append(i)
            if len(cur) > len(best):
                best = list(cur)
        if len(best) < 2 * a.per_step:
            raise SystemExit("no steady window found")
        nsteps = (len(best) - 1) // a.per_step
        lo = best[0]
        hi = best[nsteps * a.per_step]  # window = whole steps, marker to marker
        win = rows[lo:hi]
        t_wall = (rows[hi][1] - rows[lo][1]) / 1e3
        print(f"steady window: {nsteps} steps, {len(win)} dispatches, wall {t_wall / nsteps:.1f} us/step")
    else:
        win, nsteps = rows, 1
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e, _ in win:
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"kernel time {tot / nsteps:.1f} us per step" if a.marker else f"kernel time {tot:.1f} us")
    print("| kernel | calls/step | us/step | us/call | % |")
    print("|---|---:|---:|---:|---:|")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{k}` | {n / nsteps:.1f} | {t / nsteps:.1f} | {t / n:.1f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main()
