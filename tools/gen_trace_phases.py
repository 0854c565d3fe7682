"""Per-phase kernel breakdown of a generate() kernel trace (rocprofv3 --kernel-trace csv of
tools/f32_fwd_ab.py gen, which runs generate twice): the LAST generate, split at its first window
(k_ffn_f32) launch into phase 1 (per-token decode against the K/V caches) and phase 2 (window steps).
usage: python tools/gen_trace_phases.py <kernel_trace.csv> [top]"""
import collections
import csv
import sys


def main(path, top=14):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    # generate boundaries: gaps > 20 ms between kernels
    cuts = [0] + [i for i in range(1, len(rows)) if st[i] - en[i - 1] > 20e6] + [len(rows)]
    segs = [(cuts[i], cuts[i + 1]) for i in range(len(cuts) - 1)]
    a, b = [s for s in segs if s[1] - s[0] > 1000][-1]   # the last generate (> 1000 launches)
    g = rows[a:b]
    first_win = next((i for i, r in enumerate(g) if "k_ffn_f32" in r["Kernel_Name"]), len(g))
    for name, rs in (("phase 1 (decode)", g[:first_win]), ("phase 2 (window)", g[first_win:])):
        if not rs:
            continue
        span = (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e6
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e6
        print(f"== {name}: {len(rs)} kernels, span {span:.1f} ms, kernel-busy {busy:.1f} ms")
        agg = collections.defaultdict(lambda: [0, 0])
        for r in rs:
            k = agg[r["Kernel_Name"][:96]]
            k[0] += 1
            k[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
            print(f"  {t / 1e6:7.2f} ms {n:6d} x {t / n / 1e3:7.2f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:3]))
