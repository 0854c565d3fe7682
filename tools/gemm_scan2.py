"""GEMM variant / split-K scan over the training census of one config (bench.gemm_census shapes):
forward and dgrad products x variants, weight-gradient products x variants x split-K.  Each cell
is a hipGraph of 20 back-to-back launches (split-K includes its reduce kernel), best of 5.  GPU
only.

usage: python tools/gemm_scan2.py [c2|c4] [fwd variants] [wgrad variants] [wgrad splits]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_scan import gemm_fn, graph_time  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402


def valid(v, M, N):
    """Variants whose tile does not divide the problem fall back silently; skip them."""
    if v in (11, 21, 25):
        return M % 256 == 0 and N % 128 == 0
    if v == 22:
        return M % 128 == 0 and N % 256 == 0
    if v == 24:
        return M % 256 == 0 and N % 256 == 0
    return M % 128 == 0 and N % 128 == 0


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    fv = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "9,10,12,21,22,23").split(",")]
    wv = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "9,10,12,21,22,23").split(",")]
    splits = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "1,2,4,8,16,32").split(",")]
    d, M = (384, 16384) if cfg == "c2" else (768, 65536)
    F4 = 4 * d
    lib = L.load()
    fwd = [("qkv_fwd", M, 3 * d, d, 0, 0), ("proj_fwd", M, d, d, 0, 0), ("ffn1_fwd", M, F4, d, 0, 0),
           ("ffn2_fwd", M, d, F4, 0, 0), ("proj_dgrad", M, d, d, 0, 1), ("qkv_dgrad", M, d, 3 * d, 0, 1),
           ("ffn2_dgrad", M, F4, d, 0, 1), ("ffn1_dgrad", M, d, F4, 0, 1)]
    best = {}
    for name, m, n, k, at, bt in fwd:
        line = f"{cfg} {name:11s} M={m:6d} N={n:5d} K={k:5d} |"
        for v in fv:
            if not valid(v, m, n):
                continue
            L.check(lib.cg_set_tuning(b"gemm_variant", v))
            t = graph_time(gemm_fn(m, n, k, at, bt))
            line += f" v{v} {t * 1e3:6.1f}us"
            if t < best.get(name, (1e9,))[0]:
                best[name] = (t, v, 1)
        print(line, flush=True)
    wg = [("proj_wgrad", d, d, M), ("qkv_wgrad", 3 * d, d, M), ("ffn2_wgrad", d, F4, M), ("ffn1_wgrad", F4, d, M)]
    for name, m, n, k in wg:
        for split in splits:
            if k // 64 < split or (split - 1) * (-(-(k // 64) // split)) >= k // 64:
                continue
            line = f"{cfg} {name:11s} M={m:6d} N={n:5d} K={k:6d} split {split:2d} |"
            for v in wv:
                if not valid(v, m, n):
                    continue
                L.check(lib.cg_set_tuning(b"gemm_variant", v))
                t = graph_time(gemm_fn(m, n, k, 1, 1, split))
                line += f" v{v} {t * 1e3:6.1f}us"
                if t < best.get(name, (1e9,))[0]:
                    best[name] = (t, v, split)
            print(line, flush=True)
    L.check(lib.cg_set_tuning(b"gemm_variant", 0))
    for name, (t, v, split) in best.items():
        print(f"BEST {cfg} {name:11s} v{v} split {split:2d} {t * 1e3:6.1f}us", flush=True)


if __name__ == "__main__":
    main()
