"""Where the persistent 128x128 GEMM's time goes, by subtraction: loads the what-if build
(make -C replicatinggpt_amd/csrc whatif; gemm_pk.hip CG_PK_WHATIF) and times each C2 shape with the
in-loop LDS-DMAs, the MFMAs and/or the item epilogues skipped (pk_flags bits 4 / 5 / 6 -- wrong
results, timing only; WHATIF_MODES=stores: bit 3, only each block's last item stores).  GPU only.  usage: python tools/gemm_whatif.py [c2|c4]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CHARPT_LIB"] = os.path.join(ROOT, "replicatinggpt_amd", "libcharpt_hip_whatif.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gemm_scan import gemm_fn, graph_time  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402

MODES = [("all", 0), ("no DMA", 16), ("no MFMA", 32), ("no epilogue", 64), ("no DMA+epi", 80),
         ("no MFMA+epi", 96), ("no DMA+MFMA", 48), ("none (loop skeleton)", 112)]
if os.environ.get("WHATIF_MODES") == "stores":   # the item-end stores: all / the block's last item only / none
    MODES = [("all", 0), ("last item only", 8), ("no epilogue", 64)]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    lib = L.load()
    d, M = (384, 16384) if cfg == "c2" else (768, 65536)
    shapes = [("qkv_fwd", M, 3 * d, d, 0, 0, 1), ("ffn1_fwd", M, 4 * d, d, 0, 0, 1), ("ffn2_fwd", M, d, 4 * d, 0, 0, 1),
              ("ffn2_dgrad", M, 4 * d, d, 0, 1, 1), ("ffn2_wgrad", d, 4 * d, M, 1, 1, 14 if cfg == "c2" else 7)]
    L.check(lib.cg_set_tuning(b"gemm_variant", 9))
    print(f"{'shape':12s} " + " ".join(f"{n:>14s}" for n, _ in MODES))
    for name, m, n, k, at, bt, split in shapes:
        ts = []
        for _, fl in MODES:
            L.check(lib.cg_set_tuning(b"pk_flags", fl))
            ts.append(1e3 * graph_time(gemm_fn(m, n, k, at, bt, split)))   # ms -> us
        print(f"{name:12s} " + " ".join(f"{t:12.1f}us" for t in ts), flush=True)
    L.check(lib.cg_set_tuning(b"pk_flags", 0))
    L.check(lib.cg_set_tuning(b"gemm_variant", 0))


if __name__ == "__main__":
    main()
