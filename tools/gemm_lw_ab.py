"""Loader-wave persistent GEMM (cg_set_tuning "gemm_lw") against the default one, same process:
every C2 / C4 census op (bench.census_op: the step's fused epilogue) -- outputs compared bit for bit
between the two variants, then the per-launch time of each (HIP events over a hipGraph replay of 30
launches, bench.time_gemm), rounds interleaved.  usage: python tools/gemm_lw_ab.py [c2|c4] [rounds]

Historical: the "gemm_lw" knob and its kernel variant were removed after this A/B (round 5,
profiles/r5_gemm_loader_wave_ab.txt: +23 % on the C2 family); cg_set_tuning now rejects the key,
so the script only runs against a tree that still carries the variant."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import PRESETS, _lib as L  # noqa: E402


def set_lw(v):
    L.check(L.load().cg_set_tuning(b"gemm_lw", v), "gemm_lw")


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = PRESETS[cfg_name]
    dev = torch.device("cuda")
    shapes = bench.census_shapes(cfg, cfg.batch_size, cfg.block_size)
    # bitwise check: same seeded operands through both variants
    for name, M, N, K, at, bt, kind, cnt in shapes:
        outs = []
        for lw in (0, 1):
            set_lw(lw)
            torch.manual_seed(5)
            st = {}
            run, _ = bench.census_op(name, M, N, K, at, bt, kind, dev, capture=st)
            run()
            torch.cuda.synchronize()
            outs.append({k: v.clone() for k, v in st.items() if k in ("out", "bits", "part", "delta")})
        same = all(torch.equal(outs[0][k], outs[1][k]) for k in outs[0])
        print(f"{name:11s} bitwise {'equal' if same else 'DIFFERENT'}", flush=True)
    times = {(s[0], lw): [] for s in shapes for lw in (0, 1)}
    for r in range(rounds):
        for name, M, N, K, at, bt, kind, cnt in shapes:
            for lw in (0, 1):
                set_lw(lw)
                times[(name, lw)].append(bench.time_gemm(name, M, N, K, at, bt, kind, dev))
                torch.cuda.empty_cache()
    fam = {0: 0.0, 1: 0.0}
    for name, M, N, K, at, bt, kind, cnt in shapes:
        t0, t1 = statistics.median(times[(name, 0)]) * 1e3, statistics.median(times[(name, 1)]) * 1e3
        fam[0] += t0 * cnt
        fam[1] += t1 * cnt
        print(f"{name:11s} {kind:17s} lw0 {t0:6.2f} us  lw1 {t1:6.2f} us  ({(t1 / t0 - 1) * 100:+.1f} %)", flush=True)
    print(f"family per step: lw0 {fam[0]:.1f} us  lw1 {fam[1]:.1f} us ({(fam[1] / fam[0] - 1) * 100:+.1f} %)")
    set_lw(0)


if __name__ == "__main__":
    main()
