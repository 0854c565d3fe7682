"""Where does the persistent fp32 GEMM (k_gemm_f32p, generate()'s window products) spend its time?
Loads the what-if build (make -C replicatinggpt_amd/csrc whatif; gemm.hip CG_F32P_WHATIF) and times the
four C5 window shapes with pk_flags 0 (all), 16 (no in-loop loads), 32 (no MFMAs), 64 (no epilogue
stores), 256 (fragment reads only in a tile's first K-step), 512 (LDS store + barrier only
there) and combinations.  Wrong results (timing only).  GPU only.
usage: python tools/f32p_whatif.py [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CHARPT_LIB", os.path.join(ROOT, "replicatinggpt_amd", "libcharpt_hip_whatif.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from f32_fwd_ab import SHAPES, graph_us, launch_fn  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402

MODES = [("all", 0), ("noload", 16), ("noMFMA", 32), ("nostore", 64), ("noload+nostore", 80),
         ("noMFMA+nostore", 96), ("skeleton", 112), ("noread", 256), ("nosync", 512), ("noread+nosync", 768),
         ("noread+nosync+noload+nostore", 848)]


def main(rounds):
    lib = L.load()
    dev = torch.device("cuda")
    t = {(n, f): [] for n, *_ in SHAPES for _, f in MODES}
    for _ in range(rounds):
        for name, M, N, K, kind in SHAPES:
            run = launch_fn(M, N, K, kind, dev)
            for _, f in MODES:
                L.check(lib.cg_set_tuning(b"pk_flags", f))
                t[(name, f)].append(graph_us(run))
            del run
            torch.cuda.empty_cache()
    L.check(lib.cg_set_tuning(b"pk_flags", 0))
    for name, M, N, K, kind in SHAPES:
        row = "  ".join(f"{m} {statistics.median(t[(name, f)]):6.1f}" for m, f in MODES)
        print(f"{name:5s} M={M} N={N} K={K} epi {kind} | {row}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
