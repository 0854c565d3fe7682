"""Address audit of the persistent bf16 GEMM (the illegal-address faults of round 3's
register-staged-ring and L2-prefetch trials).  Runs the diagnostic build (`make bounds`,
CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_bounds.so: gemm_pk.hip CG_PK_BOUNDS) over every shape and
split the round-3 scans ran (tools/gemm_scan2.py: C2 and C4 forward / dgrad products, weight
gradients at splits 4, 7, 8, 13, 14, 16, 32), capped grids, uneven splits and the census shapes with
their fused epilogues, and prints the in-kernel violation counts: LDS-DMA source chunks outside their
operand (A, B; the past-the-end reloads included), items outside the output / slab range, and the
address stream of the removed L2-prefetch trial (db80795) re-derived without being issued, PF = 1..3.
First a positive control (windows shortened by 1 KB) shows the counters do count.  GPU only."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import PRESETS  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import ops  # noqa: E402

NAMES = ["A dma", "B dma", "item/slab", "pf1", "pf2", "pf3"]


def counts(lib):
    buf = (ctypes.c_ulonglong * 8)()
    L.check(lib.cg_debug_pk_bounds(buf), "bounds")
    return list(buf)[:6]


def gemm(M, N, K, at, bt, split, dev):
    A = torch.randn((K, M) if at else (M, K), device=dev).to(torch.bfloat16)
    B = torch.randn((K, N) if bt else (N, K), device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.float32 if split > 1 or at else torch.bfloat16, device=dev)
    ws = torch.empty(max(1, ops.gemm_workspace(M, N, split) // 4), dtype=torch.float32, device=dev)
    ops.gemm(A, B, out, True, bool(at), bool(bt), M, N, K, A.shape[1], B.shape[1], N, 0, None, None, 0, None, 0,
             0.0, 0, None, 0, 0.0, split, ws if split > 1 else None)


def main():
    lib = L.load()
    if not hasattr(lib, "cg_debug_pk_bounds"):
        raise SystemExit("not the bounds build: CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_bounds.so")
    dev = torch.device("cuda")
    # positive control
    L.check(lib.cg_debug_pk_bounds_reset(), "reset")
    L.check(lib.cg_set_tuning(b"pk_flags", 128), "tuning")
    gemm(16384, 384, 384, 0, 0, 1, dev)
    torch.cuda.synchronize()
    L.check(lib.cg_set_tuning(b"pk_flags", 0), "tuning")
    ctl = counts(lib)
    print(f"positive control (windows 1 KB short, C2 proj fwd): {dict(zip(NAMES, ctl))}", flush=True)
    assert ctl[0] > 0 and ctl[1] > 0, "the bounds counters did not count"
    cases = []
    for cfg, d, M in (("c2", 384, 16384), ("c4", 768, 65536)):
        F4 = 4 * d
        for name, m, n, k, at, bt in (("qkv_fwd", M, 3 * d, d, 0, 0), ("proj_fwd", M, d, d, 0, 0),
                                      ("ffn1_fwd", M, F4, d, 0, 0), ("ffn2_fwd", M, d, F4, 0, 0),
                                      ("proj_dgrad", M, d, d, 0, 1), ("qkv_dgrad", M, d, 3 * d, 0, 1),
                                      ("ffn2_dgrad", M, F4, d, 0, 1), ("ffn1_dgrad", M, d, F4, 0, 1)):
            cases.append((cfg, name, m, n, k, at, bt, 1, 0))
        for name, m, n in (("proj_wgrad", d, d), ("qkv_wgrad", 3 * d, d), ("ffn2_wgrad", d, F4),
                           ("ffn1_wgrad", F4, d)):
            for split in (4, 7, 8, 13, 14, 16, 32):
                cases.append((cfg, name, m, n, M, 1, 1, split, 0))
    for grid in (37, 77):   # capped grids: several items per block, items of several splits per block
        cases.append(("cap", "qkv_wgrad", 1152, 384, 16384, 1, 1, 14, grid))
        cases.append(("cap", "ffn1_fwd", 16384, 1536, 384, 0, 0, 1, grid))
    total = [0] * 6
    for cfg, name, m, n, k, at, bt, split, grid in cases:
        L.check(lib.cg_debug_pk_bounds_reset(), "reset")
        L.check(lib.cg_set_tuning(b"gemm_max_grid", grid), "tuning")
        gemm(m, n, k, at, bt, split, dev)
        torch.cuda.synchronize()
        c = counts(lib)
        total = [a + b for a, b in zip(total, c)]
        if any(c):
            print(f"VIOLATION {cfg} {name} M={m} N={n} K={k} split={split} grid={grid}: {dict(zip(NAMES, c))}",
                  flush=True)
    L.check(lib.cg_set_tuning(b"gemm_max_grid", 0), "tuning")
    # the training census with the step's fused epilogues (C2)
    L.check(lib.cg_debug_pk_bounds_reset(), "reset")
    cfg = PRESETS["c2"]
    for name, m, n, k, at, bt, kind, _ in bench.census_shapes(cfg, cfg.batch_size, cfg.block_size):
        run, _ = bench.census_op(name, m, n, k, at, bt, kind, dev)
        run()
    torch.cuda.synchronize()
    c = counts(lib)
    total = [a + b for a, b in zip(total, c)]
    print(f"{len(cases)} scan cases + the C2 census (fused epilogues): violations {dict(zip(NAMES, total))}",
          flush=True)


if __name__ == "__main__":
    main()
