"""Cross-check bench.py's roofline / GEMM census timings against the rocprofv3 kernel trace of the
same command: bench times each GEMM op of the step with 3 warm-up + 30 back-to-back launches (HIP
events, time_gemm); in the trace these are bursts of identical (GEMM [+ split-K reduce]) dispatches.
For every burst this prints the per-launch kernel time (GEMM + reduce durations from the trace) and
the per-launch wall time (burst span / launches) -- the latter is what HIP events measure.

usage: python tools/roofline_check.py <run_kernel_trace.csv> [config c2|c4]
"""
import csv
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def main():
    path = sys.argv[1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    names = [n for _, _, n in rows]
    i, bursts = 0, []
    while i < len(rows):
        found = False
        for period in (1, 2):
            j = i
            while j + period < len(rows) and names[j + period] == names[j] and \
                    ("gemm" in names[j] or "splitk" in names[j]):
                j += 1
            n = (j + period - i) // period
            if n >= 30 and "gemm" in names[i]:
                seg = rows[i:i + n * period]
                busy = sum(e - s for s, e, _ in seg) / n / 1e3
                wall = (seg[-1][1] - seg[0][0]) / n / 1e3
                bursts.append((" + ".join(short(x) for x in names[i:i + period])[:90], period, n, busy, wall))
                i += n * period
                found = True
                break
        if not found:
            i += 1
    labels = []
    try:
        from bench import census_shapes
        from replicatinggpt_amd.config import PRESETS
        cfg = PRESETS[sys.argv[2] if len(sys.argv) > 2 else "c2"]
        labels = [s[0] for s in census_shapes(cfg, cfg.batch_size, cfg.block_size)]
    except Exception:   # labels are a convenience; the bursts stand on their own
        pass
    print(f"{'op':12s} {'kernels/launch':>14s} {'launches':>8s} {'kernel us':>10s} {'wall us':>8s}  kernels")
    for k, (name, period, n, busy, wall) in enumerate(bursts):
        lab = labels[k] if k < len(labels) and len(bursts) == len(labels) else f"burst{k}"
        print(f"{lab:12s} {period:14d} {n:8d} {busy:10.2f} {wall:8.2f}  {name}")


if __name__ == "__main__":
    main()
