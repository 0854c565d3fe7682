"""Instruction trace of one kernel's loop(s) in a hipcc -S file: every s_waitcnt / barrier / branch /
spill with running counts of MFMA, VALU, DS and VMEM instructions since the trace start.
usage: python tools/isa_trace.py <file.s> <kernel-substring> [loop-depth=2] [max-lines]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    n = [x for x in re.findall(r"^(_Z\S+):", s, re.M) if sys.argv[2] in x][0]
    depth = sys.argv[3] if len(sys.argv) > 3 else "2"
    lim = int(sys.argv[4]) if len(sys.argv) > 4 else 400
    a = s.index(n + ":")
    body = s[a:s.index(".Lfunc_end", a)].split("\n")
    st = [i for i, l in enumerate(body) if "Loop Header" in l and f"Depth={depth}" in l][0]
    cnt = dict(mfma=0, valu=0, ds=0, vmem=0)
    out = 0
    for i in range(st, len(body)):
        t = body[i].strip()
        if not t or t.startswith((";", ".")):
            if re.match(r"^\.LBB", body[i]) and i > st and "Loop" not in body[i]:
                print(i, body[i][:60])
            continue
        op = t.split()[0]
        if op.startswith("v_mfma"):
            cnt["mfma"] += 1
        elif op.startswith("v_"):
            cnt["valu"] += 1
        elif op.startswith("ds_"):
            cnt["ds"] += 1
        elif op.startswith(("global_", "buffer_", "scratch_")):
            cnt["vmem"] += 1
        if op in ("s_waitcnt", "s_barrier") or op.startswith(("s_cbranch", "scratch_", "s_branch")):
            print(i, t[:50], cnt)
            out += 1
            if out > lim:
                break


if __name__ == "__main__":
    main()
