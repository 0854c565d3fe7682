"""Per-kernel table from tools/pmc_step.sh passes: duration-weighted view of MFMA busy, VALU,
wait fractions, LDS conflicts and HBM bytes (FETCH_SIZE x2 per MI355X_MICROARCH.md §HBM).
usage: python tools/pmc_table.py <dir>"""
import collections
import csv
import glob
import re
import sys


def kname(n):
    n = n.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n).replace("void ", "").replace("cg::", "").strip()[:44]


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for path in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                acc[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for path in sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    m = lambda k, c: (sum(acc[k][c]) / len(acc[k][c])) if acc[k].get(c) else float("nan")
    print(f"{'kernel':44s} {'n':>4s} {'mfma%':>6s} {'valu%':>6s} {'wait%':>6s} {'winst%':>6s} {'act%':>6s} "
          f"{'ldsconf':>8s} {'MB_rd':>7s} {'MB_wr':>7s} {'L2hit':>6s} {'waves':>7s}")
    rows = []
    for k in acc:
        wc = m(k, "SQ_WAVE_CYCLES")
        gui = m(k, "GRBM_GUI_ACTIVE") / 8  # per XCD cycles
        simd_cycles = gui * 1024 / 1  # 1024 SIMDs... per-XCD cycles x (128 SIMDs x 8 XCDs)
        mf = m(k, "SQ_VALU_MFMA_BUSY_CYCLES") / simd_cycles * 100
        valu = m(k, "SQ_ACTIVE_INST_VALU") * 4 / simd_cycles * 100
        hit, miss = m(k, "TCC_HIT_sum"), m(k, "TCC_MISS_sum")
        rows.append((m(k, "SQ_VALU_MFMA_BUSY_CYCLES"), k, len(acc[k].get("SQ_WAVES", [])), mf, valu,
                     m(k, "SQ_WAIT_ANY") / wc * 100, m(k, "SQ_WAIT_INST_ANY") / wc * 100,
                     m(k, "SQ_ACTIVE_INST_ANY") / wc * 100, m(k, "SQ_LDS_BANK_CONFLICT"),
                     2 * m(k, "FETCH_SIZE") / 1024, m(k, "WRITE_SIZE") / 1024, hit / (hit + miss + 1e-9) * 100,
                     m(k, "SQ_WAVES")))
    for _, k, n, mf, va, w, wi, a, lc, fr, wr, h, wv in sorted(rows, key=lambda r: -r[0]):
        print(f"{k:44s} {n:4d} {mf:6.1f} {va:6.1f} {w:6.1f} {wi:6.1f} {a:6.1f} {lc:8.0f} {fr:7.1f} {wr:7.1f} {h:6.1f} {wv:7.0f}")


if __name__ == "__main__":
    main()
