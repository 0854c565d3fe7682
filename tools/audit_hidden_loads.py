"""Audit of hidden register loads (common.h gload16/gload4/gload4s: inline-asm global loads hipcc does
not count): in every kernel of a hipcc -S file, no instruction may read or write a hidden load's
destination registers before an `s_waitcnt vmcnt(N)` has retired that load (cdna_hip_programming.md
5.7 item 1).  vmcnt retires in issue order, so a wait with N > 0 retires the load only when at least N
vector-memory instructions were issued after it.

Dataflow over each kernel's control-flow graph (basic blocks split at labels and branches; a
conditional branch has its target and the fall-through as successors), to a fixed point: the state
is, per register, the fewest VMEM instructions issued since its hidden load.  A register is pending
where it is pending on EVERY path that reaches the point (states merge by intersection): the
union ("on some path") flags ~200 instructions in attention_d64.hip, all on paths the kernels cannot
take -- `ring_wait(pf)`'s two waits (`vmcnt(4)` when the next tile's DMAs were issued, `vmcnt(0)`
when not) compile to two conditional branches on the same `pf`, and the path that skips both does
not exist.  The hazard the round-5 residual-prefetch trial hit -- hipcc copying a hidden load's
destination register between the load and its wait -- lies on every path from the load
and is flagged either way; tests/test_hidden_load_audit.py runs the audit on the product sources and
checks it flags that pattern (straight line and round a loop back-edge).
usage: python tools/audit_hidden_loads.py <file.s> [kernel-substring]"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
HIDDEN = re.compile(r"global_load_dword(x2|x3|x4)?\s+(v\[\d+:\d+\]|v\d+),")
BRANCH = re.compile(r"^s_(c?branch\S*|cbranch\S*)\s+(\.L\w+)")
WAIT = re.compile(r"vmcnt\((\d+)\)")
CAP = 64


def regs(tok):
    out = set()
    for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|(?<![\w])v(\d+)", tok):
        out |= set(range(int(a), int(b) + 1)) if a else {int(c)}
    return out


def _blocks(body):
    """[(label or None, [(line, text, in_asm)], successor labels, falls through)]"""
    blocks, cur, in_asm = [], None, False

    def new(label):
        b = {"label": label, "ins": [], "succ": [], "fall": True}
        blocks.append(b)
        return b
    cur = new(None)
    for i, l in enumerate(body):
        t = l.strip()
        lm = re.match(r"^(\.L\w+):", t)
        if lm:
            cur = new(lm.group(1))
            continue
        if t.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if t.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not t or t.startswith((";", ".")):
            continue
        cur["ins"].append((i, t, in_asm))
        b = BRANCH.match(t)
        if b:
            cur["succ"].append(b.group(2))
            cur["fall"] = not t.startswith("s_branch ")
            cur = new(None)
        elif t.startswith("s_endpgm"):
            cur["fall"] = False
            cur = new(None)
    return blocks


def _transfer(block, state, report):
    st = dict(state)
    for line, t, in_asm in block["ins"]:
        if t.startswith("s_waitcnt"):
            w = WAIT.search(t)
            if w:
                n = int(w.group(1))
                st = {r: c for r, c in st.items() if c < n}
            continue
        m = HIDDEN.match(t)
        if in_asm and m and " lds" not in t:
            st = {r: min(c + 1, CAP) for r, c in st.items()}
            for r in regs(m.group(2)):
                st[r] = 0
            continue
        if st and report is not None:
            hit = regs(t) & set(st)
            if hit:
                report(line, t, min(hit))
        if VMEM.match(t):
            st = {r: min(c + 1, CAP) for r, c in st.items()}
    return st


def _merge(a, b):
    """pending on every path: intersection, the fewest VMEM instructions since the load"""
    return {r: min(c, b[r]) for r, c in a.items() if r in b}


def audit(text, filt=""):
    """list of (kernel, line, instruction, register) violations"""
    out = []
    for n in re.findall(r"^(_Z\S+):", text, re.M):
        if filt not in n:
            continue
        a = text.index(n + ":")
        body = text[a:text.index(".Lfunc_end", a)].split("\n")
        blocks = _blocks(body)
        index = {b["label"]: k for k, b in enumerate(blocks) if b["label"]}
        succ = []
        for k, b in enumerate(blocks):
            s = [index[x] for x in b["succ"] if x in index]
            if b["fall"] and k + 1 < len(blocks):
                s.append(k + 1)
            succ.append(s)
        entry = [None] * len(blocks)
        entry[0] = {}
        work = [0]
        while work:
            k = work.pop()
            o = _transfer(blocks[k], entry[k], None)
            for s in succ[k]:
                m = o if entry[s] is None else _merge(entry[s], o)
                if entry[s] is None or m != entry[s]:
                    entry[s] = m
                    work.append(s)
        seen = set()
        for k, b in enumerate(blocks):
            if entry[k] is not None:
                def report(line, t, r, n=n):
                    if (line, r) not in seen:
                        seen.add((line, r))
                        out.append((n, line, t, r))
                _transfer(b, entry[k], report)
    return out


def main():
    s = open(sys.argv[1]).read()
    bad = audit(s, sys.argv[2] if len(sys.argv) > 2 else "")
    for n, line, t, r in bad:
        print(f"{n[:60]} line {line}: {t[:80]}  (touches pending v{r})")
    print("hidden-load audit:", "CLEAN" if not bad else f"{len(bad)} violations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
