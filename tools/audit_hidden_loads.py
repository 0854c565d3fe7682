"""Audit of hidden register loads (common.h gload16/gload4: inline-asm global loads hipcc does not
count): in every kernel of a hipcc -S file, no instruction may read or write a hidden load's
destination registers between the load and the next `s_waitcnt vmcnt` (cdna_hip_programming.md 5.7
item 1).  Linear scan per kernel; prints offending lines.
usage: python tools/audit_hidden_loads.py <file.s> [kernel-substring]"""
import re
import sys


def regs(tok):
    out = set()
    for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|v(\d+)", tok):
        out |= set(range(int(a), int(b) + 1)) if a else {int(c)}
    return out


def main():
    s = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    bad = 0
    for n in re.findall(r"^(_Z\S+):", s, re.M):
        if filt not in n:
            continue
        a = s.index(n + ":")
        body = s[a:s.index(".Lfunc_end", a)].split("\n")
        pending = {}   # register -> line of its hidden load
        in_asm = False
        for i, l in enumerate(body):
            t = l.strip()
            if t.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if t.startswith(";;#ASMEND"):
                in_asm = False
                continue
            if not t or t.startswith((";", ".")):
                continue
            if "s_waitcnt" in t and "vmcnt" in t:
                pending.clear()
                continue
            m = re.match(r"global_load_dword(x4)?\s+(v\[\d+:\d+\]|v\d+),", t)
            if in_asm and m and "lds" not in t:
                for r in regs(m.group(2)):
                    pending[r] = i
                continue
            hit = regs(t) & set(pending)
            if hit:
                bad += 1
                print(f"{n[:60]} line {i}: {t[:80]}  (touches v{sorted(hit)[0]} loaded at line {pending[min(hit)]})")
    print("hidden-load audit:", "CLEAN" if not bad else f"{bad} violations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
