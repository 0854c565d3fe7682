"""Why does k_gemm_pk<128x128> fill LDS at ~11.6 B/clk/CU on the C2 products and ~23 on the C4 weight
gradients?    Loads the what-if build (make -C replicatinggpt_amd/csrc whatif;
gemm_pk.hip CG_PK_WHATIF) and times M = 16384, N = 1536 with

  * K in {384, 1536, 6144}            -- per-item K depth (6 / 24 / 96 K-steps per item)
  * NN (K-contiguous A and B, 128-B row segments per K-tile) vs TT (the wgrad layout: 256-B row
    segments of 64 K rows)
  * grid = every resident slot (512) vs 256 blocks (one per CU)
  * pk_flags 0 (all), 32 (no MFMA), 96 (no MFMA, no epilogue), 112 (no DMA, MFMA, epilogue)

and reports per launch: us, LDS-DMA fill bytes per us per CU (and per clock at 2.1 GHz), and the
per-K-step time of the busiest slot.  Wrong results (timing only).  GPU only.
usage: python tools/gemm_fill_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CHARPT_LIB", os.path.join(ROOT, "replicatinggpt_amd", "libcharpt_hip_whatif.so"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from gemm_scan import gemm_fn, graph_time  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402

CLK = 2.1e3   # MHz assumed for B/clk (the stamps saw 2.17-2.28 GHz under these loads)
CUS = 256


def main():
    lib = L.load()
    L.check(lib.cg_set_tuning(b"gemm_variant", 9))
    modes = [("all", 0), ("noMFMA", 32), ("noMFMA+epi", 96), ("skeleton", 112)]
    M, N = int(os.environ.get("DIAG_M", 16384)), int(os.environ.get("DIAG_N", 1536))
    ks = [int(k) for k in os.environ.get("DIAG_K", "384,1536,6144").split(",")]
    grids = [int(g) for g in os.environ.get("DIAG_GRID", "0,256").split(",")]
    print(f"M={M} N={N}; fill = items*(128+128)*K*2 B; per-CU rate over {CUS} CUs; B/clk at {CLK:.0f} MHz")
    for k in ks:
        for lay, at, bt in (("NN", 0, 0), ("TT", 1, 1)):
            for grid in grids:
                L.check(lib.cg_set_tuning(b"gemm_max_grid", grid))
                items = (M // 128) * (N // 128)
                slots = grid if grid else 512
                ksteps_busiest = -(-items // slots) * (k // 64)
                fill = items * 256 * k * 2
                line = f"K={k:5d} {lay} grid={slots:3d} kst/slot={ksteps_busiest:4d} |"
                for name, fl in modes:
                    L.check(lib.cg_set_tuning(b"pk_flags", fl))
                    t = graph_time(gemm_fn(M, N, k, at, bt, 1)) * 1e-3   # s
                    gbs_cu = fill / t / CUS / 1e9
                    cyc = t * CLK * 1e6 / ksteps_busiest
                    line += f" {name} {t*1e6:6.1f}us {gbs_cu:5.1f}GB/s/CU={gbs_cu*1e3/CLK:4.1f}B/clk {cyc:5.0f}cyc/kst |"
                print(line, flush=True)
    L.check(lib.cg_set_tuning(b"pk_flags", 0))
    L.check(lib.cg_set_tuning(b"gemm_max_grid", 0))
    L.check(lib.cg_set_tuning(b"gemm_variant", 0))


if __name__ == "__main__":
    main()
