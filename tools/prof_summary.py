"""Summarise a rocprofv3 --kernel-trace run (rocpd .db or csv kernel_trace) per kernel name:
calls, total us, average us, share.  Optionally restrict to the dispatches of the last
--last-steps training steps (grouping by --per-step dispatches is not attempted: pass a
grid filter instead).

usage: python tools/prof_summary.py <run_results.db | run_kernel_trace.csv> [--top N] [--csv out.csv]
"""
import argparse
import collections
import csv
import re
import sqlite3


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", name).replace("void ", "").strip()[:140]


def load(path):
    rows = []
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for name, dur, gx, gy, gz, wx in db.execute(
                "select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels"):
            rows.append((name, float(dur), (gx, gy, gz, wx)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"]),
                             (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z"),
                              r.get("Workgroup_Size_X"))))
    return rows


def summarize(rows, by_grid=False):
    acc = collections.OrderedDict()
    for name, dur, grid in rows:
        key = (short(name), grid) if by_grid else short(name)
        c = acc.setdefault(key, [0, 0.0])
        c[0] += 1
        c[1] += dur
    tot = sum(v[1] for v in acc.values())
    out = sorted(((k, n, t) for k, (n, t) in acc.items()), key=lambda x: -x[2])
    return out, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    out, tot = summarize(load(a.path), a.by_grid)
    print(f"{'calls':>7} {'total_us':>11} {'avg_us':>9} {'share':>6}  kernel")
    for k, n, t in out[:a.top]:
        print(f"{n:7d} {t / 1e3:11.1f} {t / n / 1e3:9.2f} {100 * t / tot:5.1f}%  {k}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "grid", "calls", "total_us", "avg_us", "share"])
            for k, n, t in out:
                name, grid = (k if a.by_grid else (k, ""))
                w.writerow([name, grid, n, round(t / 1e3, 2), round(t / n / 1e3, 3), round(t / tot, 5)])


if __name__ == "__main__":
    main()
