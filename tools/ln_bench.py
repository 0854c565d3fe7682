"""Times the LayerNorm backward at the C2 / C4 shapes as the model calls it (bf16 dy, fp32 residual
gradient, bf16 consumer copy with dropout, consumer column sums): the whole call, the row kernel
alone and the partials reduce alone, over rows-per-block values (cg_set_tuning ln_rpb).  GPU only.
usage: python tools/ln_bench.py [rpb,rpb,...] [waves,waves,...]   (waves: cg_set_tuning ln_waves, 0 = automatic)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import ops  # noqa: E402
from tools.attn_bench import _time  # noqa: E402


def run(M, C, p):
    dev = torch.device("cuda")
    x = torch.randn(M, C, device=dev)
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dres = torch.randn(M, C, device=dev)
    w, b = torch.randn(C, device=dev), torch.randn(C, device=dev)
    mean, rstd = x.mean(1), 1 / x.std(1)
    dx = torch.empty_like(x)
    lp = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    dw, db, cs = torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty(C, device=dev)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(ops.layernorm_bwd_workspace(M, C) // 4 + 1, device=dev)
    full = _time(lambda: ops.layernorm_bwd(dy, x, w, mean, rstd, dres, dx, lp, dw, db, False, ws, cs, False, p, 1,
                                           call, 3))
    rows = _time(lambda: ops.layernorm_bwd_rows(dy, x, w, mean, rstd, dres, dx, lp, ws, True, p, 1, call, 3))
    red = _time(lambda: ops.layernorm_bwd_reduce(ws, M, C, True, dw, db, cs, False, False))
    byts = M * C * (4 + 2 + 4 + 4 + 2)
    return full, rows, red, byts


if __name__ == "__main__":
    lib = L.load()
    L.check(lib.cg_set_tuning(b"ln_pf", int(os.environ.get("LN_PF", "0"))), "tuning")   # next-row prefetch A/B
    L.check(lib.cg_set_tuning(b"ln_nt", int(os.environ.get("LN_NT", "-1"))), "tuning")   # non-temporal streams A/B
    rpbs = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0]
    waves = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
    for M, C in ((16384, 384), (65536, 768)):
        for p in (0.0, 0.2):
            for wv in waves:
                for rpb in rpbs:
                    L.check(lib.cg_set_tuning(b"ln_waves", wv), "tuning")
                    L.check(lib.cg_set_tuning(b"ln_rpb", rpb), "tuning")
                    full, rows, red, byts = run(M, C, p)
                    print(f"M={M} C={C} p={p} waves={wv} rpb={rpb}: full {full:7.1f} us  rows {rows:7.1f} us "
                          f"({byts / rows / 1e3:6.0f} GB/s)  reduce {red:6.1f} us", flush=True)
    L.check(lib.cg_set_tuning(b"ln_rpb", 0), "tuning")
    L.check(lib.cg_set_tuning(b"ln_waves", 0), "tuning")
