"""Timeline statistics of a rocprofv3 kernel trace (csv) over a window of training steps:
per queue busy time, the union of all kernels' busy time (GPU not idle), and the idle gaps.
usage: python tools/trace_timeline.py <run_kernel_trace.csv> [marker-kernel-substring] [steps] [skip] [gaps]
The window is the last `steps` occurrences of the marker kernel (default k_embed_fwd: one per step)
before the last `skip` ones (bench.py's in-step probe adds 8 steps after the timed region)."""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_embed_fwd"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
                     re.sub(r"\(.*$", "", name).replace("void ", "").replace("cg::", "")[:48]))
    rows.sort()
    marks = [s for s, e, q, n in rows if marker in n]
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    if skip:
        marks = marks[:-skip]
    if len(marks) < steps + 1:
        print("not enough steps"); return
    t0, t1 = marks[-steps - 1], marks[-1]
    win = [(max(s, t0), min(e, t1), q, n) for s, e, q, n in rows if e > t0 and s < t1]
    wall = t1 - t0
    print(f"window: {steps} steps, {wall / 1e3 / steps:.1f} us/step")
    per_q = {}
    for s, e, q, n in win:
        per_q[q] = per_q.get(q, 0) + (e - s)
    for q, t in sorted(per_q.items()):
        print(f"  queue {q}: busy {t / 1e3 / steps:8.1f} us/step ({t / wall:.0%}) [sum of kernel times]")
    # union of busy intervals
    busy, cur_s, cur_e, last = 0, None, None, None
    gaps = []
    for s, e, q, n in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, cur_e, last, (q, n)))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        if e >= (cur_e or 0):
            last = (q, n)
    busy += cur_e - cur_s
    print(f"  any kernel running: {busy / 1e3 / steps:.1f} us/step ({busy / wall:.0%}); idle "
          f"{(wall - busy) / 1e3 / steps:.1f} us/step in {len(gaps) / steps:.0f} gaps/step")
    gaps.sort(reverse=True)
    for g, at, prev, nxt in gaps[:int(sys.argv[5]) if len(sys.argv) > 5 else 12]:
        print(f"    gap {g / 1e3:6.1f} us: after q{prev[0]} {prev[1]:48s} -> q{nxt[0]} {nxt[1]}")


if __name__ == "__main__":
    main()
