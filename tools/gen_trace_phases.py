"""Per-phase kernel breakdown of a generate() kernel trace (rocprofv3 --kernel-trace csv of
tools/f32_fwd_ab.py gen, which runs generate twice): the LAST generate, split at its first window
window launch (k_decode_window) into phase 1 (per-token steps against the K/V caches) and phase 2.
usage: python tools/gen_trace_phases.py <kernel_trace.csv> [top]"""
import collections
import csv
import sys


def main(path, top=14):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    emb = [i for i, r in enumerate(rows) if "k_decode_embed" in r["Kernel_Name"]]
    # the last generate: its 256 phase-1 steps each start with k_decode_embed (phase 2: k_decode_window)
    p1 = emb[-256] if len(emb) >= 256 else (emb[0] if emb else 0)
    win = [i for i, r in enumerate(rows) if "k_decode_window" in r["Kernel_Name"] and i > p1]
    p2 = win[0] if win else len(rows)
    cnt = [i for i, r in enumerate(rows) if "k_counter_add" in r["Kernel_Name"]]
    end = cnt[-1] + 1 if cnt else len(rows)
    g1, g2 = rows[p1:p2], rows[p2:end]
    for name, rs in (("phase 1 (per-token steps)", g1), ("phase 2 (window steps)", g2)):
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
