"""Per-loop instruction counts of the kernels in a hipcc --save-temps .s file (static counts of each
innermost loop body: VALU excluding MFMA, MFMA, v_mov, LDS, VMEM).
usage: python tools/isa_loops.py <file.s> [kernel-substring]"""
import collections
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for n in re.findall(r"^(_Z\S+):", s, re.M):
        if filt not in n:
            continue
        a = s.index(n + ":")
        b = s.index(".Lfunc_end", a)
        lines = s[a:b].split("\n")
        heads = [i for i, l in enumerate(lines) if re.match(r"^\.LBB\S+:", l) and
                 ("Loop Header" in l or (i + 1 < len(lines) and "Loop Header" in lines[i + 1]))]
        out = []
        for h in heads:
            lab = lines[h].split(":")[0]
            ends = [i for i, l in enumerate(lines) if "branch" in l and l.strip().endswith(lab)]
            if not ends:
                continue
            body = [l.split()[0] for l in lines[h + 1:ends[-1] + 1]
                    if l.strip() and not l.strip().startswith((";", "."))]
            c = collections.Counter(body)
            valu = sum(x for k, x in c.items() if k.startswith("v_") and "mfma" not in k)
            mfma = sum(x for k, x in c.items() if "mfma" in k)
            lds = sum(x for k, x in c.items() if k.startswith("ds_"))
            vmem = sum(x for k, x in c.items() if k.startswith(("global_", "buffer_")))
            depth = re.search(r"Header: Depth=(\d)", lines[h] + lines[h + 1])
            out.append(f"L{h}(d{depth.group(1) if depth else '?'}): valu {valu} mfma {mfma} mov {c['v_mov_b32_e32']} "
                       f"lds {lds} vmem {vmem}")
        print(n[:90], "|", "; ".join(out))


if __name__ == "__main__":
    main()
