"""The 256x256 persistent GEMM on its two schedules (cg_set_tuning "gemm_variant": 24 = one barrier
per K-tile, 26 = the staggered 8-phase schedule), plus the automatic choice, same process: every
census op of the config (bench.census_op: the step's fused epilogue) whose shape the 256x256 tile
divides -- outputs compared bit for bit between the variants, then the per-launch time of each (HIP
events over a hipGraph replay of 30 launches, bench.time_gemm), rounds interleaved.
usage: [AB_VARIANTS=0,24,26] python tools/gemm_sch_ab.py [c4|c2] [rounds]  (26: the A/B library, CHARPT_LIB)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import PRESETS, _lib as L  # noqa: E402

VARIANTS = tuple(int(v) for v in os.environ.get("AB_VARIANTS", "0,24,26").split(","))


def set_v(v):
    L.check(L.load().cg_set_tuning(b"gemm_variant", v), "gemm_variant")


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = PRESETS[cfg_name]
    dev = torch.device("cuda")
    shapes = [s for s in bench.census_shapes(cfg, cfg.batch_size, cfg.block_size)
              if not s[4] and s[1] % 256 == 0 and s[2] % 256 == 0]
    for name, M, N, K, at, bt, kind, cnt in shapes:
        outs = []
        for v in VARIANTS:
            set_v(v)
            torch.manual_seed(5)
            st = {}
            run, _ = bench.census_op(name, M, N, K, at, bt, kind, dev, capture=st)
            run()
            torch.cuda.synchronize()
            outs.append({k: t.clone() for k, t in st.items() if k in ("out", "bits", "part", "delta")})
            del st, run
            torch.cuda.empty_cache()
        same = [all(torch.equal(outs[0][k], o[k]) for k in outs[0]) for o in outs[1:]]
        print(f"{name:11s} M={M} N={N} K={K} {kind:17s} bitwise vs auto: "
              + " ".join(f"v{v} {'equal' if s else 'DIFFERENT'}" for v, s in zip(VARIANTS[1:], same)), flush=True)
        del outs
    times = {(s[0], v): [] for s in shapes for v in VARIANTS}
    for r in range(rounds):
        for name, M, N, K, at, bt, kind, cnt in shapes:
            for v in VARIANTS:
                set_v(v)
                times[(name, v)].append(bench.time_gemm(name, M, N, K, at, bt, kind, dev))
                torch.cuda.empty_cache()
        print(f"round {r} done", flush=True)
    fam = {v: 0.0 for v in VARIANTS}
    for name, M, N, K, at, bt, kind, cnt in shapes:
        t = {v: statistics.median(times[(name, v)]) * 1e3 for v in VARIANTS}
        for v in VARIANTS:
            fam[v] += t[v] * cnt
        tf = {v: 2.0 * M * N * K / (t[v] * 1e-6) / 1e12 for v in VARIANTS}
        print(f"{name:11s} {kind:17s} " + "  ".join(f"v{v} {t[v]:7.1f} us ({tf[v]:5.0f} TF)" for v in VARIANTS)
              + (f"  26/24 {(t[26] / t[24] - 1) * 100:+.1f} %" if 26 in t else ""), flush=True)
    print("family per step: " + "  ".join(f"v{v} {fam[v]:.1f} us" for v in VARIANTS)
          + (f"  (26 vs 24: {(fam[26] / fam[24] - 1) * 100:+.1f} %)" if 26 in fam else ""))
    set_v(0)


if __name__ == "__main__":
    main()
