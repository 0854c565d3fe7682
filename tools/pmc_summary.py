"""Per-kernel averages of every counter in the rocprofv3 --pmc csv passes under a directory.
usage: python tools/pmc_summary.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import re
import sys


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = re.sub(r"\(.*$", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
                if filt not in k:
                    continue
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k[:100])
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
