"""One cg_set_tuning knob at two values over census GEMMs, same process: outputs compared bit for
bit (bench.census_op with the step's fused epilogue), then the per-launch time of each (HIP events
over a hipGraph replay of 30 launches, bench.time_gemm), rounds interleaved.
usage: python tools/gemm_knob_ab.py <c2|c4> <knob> <value_a> <value_b> [rounds] [name,name,...]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import PRESETS, _lib as L  # noqa: E402


def main():
    cfg_name, knob, va, vb = sys.argv[1], sys.argv[2].encode(), int(sys.argv[3]), int(sys.argv[4])
    rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    names = sys.argv[6].split(",") if len(sys.argv) > 6 else None
    cfg = PRESETS[cfg_name]
    dev = torch.device("cuda")
    lib = L.load()
    shapes = [s for s in bench.census_shapes(cfg, cfg.batch_size, cfg.block_size) if names is None or s[0] in names]
    for name, M, N, K, at, bt, kind, cnt in shapes:
        outs = []
        for v in (va, vb):
            L.check(lib.cg_set_tuning(knob, v), "knob")
            torch.manual_seed(5)
            st = {}
            run, _ = bench.census_op(name, M, N, K, at, bt, kind, dev, capture=st)
            run()
            torch.cuda.synchronize()
            outs.append({k: t.clone() for k, t in st.items() if k in ("out", "bits", "part", "delta")})
        same = all(torch.equal(outs[0][k], outs[1][k]) for k in outs[0])
        print(f"{name:11s} M={M} N={N} K={K} {kind:17s} bitwise {'equal' if same else 'DIFFERENT'}", flush=True)
    times = {(s[0], v): [] for s in shapes for v in (va, vb)}
    for r in range(rounds):
        for name, M, N, K, at, bt, kind, cnt in shapes:
            for v in (va, vb):
                L.check(lib.cg_set_tuning(knob, v), "knob")
                times[(name, v)].append(bench.time_gemm(name, M, N, K, at, bt, kind, dev))
                torch.cuda.empty_cache()
    L.check(lib.cg_set_tuning(knob, 0), "knob")
    fam = {va: 0.0, vb: 0.0}
    for name, M, N, K, at, bt, kind, cnt in shapes:
        t = {v: statistics.median(times[(name, v)]) * 1e3 for v in (va, vb)}
        for v in (va, vb):
            fam[v] += t[v] * cnt
        print(f"{name:11s} {kind:17s} {knob.decode()}={va}: {t[va]:7.2f} us  {knob.decode()}={vb}: {t[vb]:7.2f} us "
              f"({(t[vb] / t[va] - 1) * 100:+.1f} %)", flush=True)
    print(f"per step: {fam[va]:.1f} us vs {fam[vb]:.1f} us ({(fam[vb] / fam[va] - 1) * 100:+.1f} %)")


if __name__ == "__main__":
    main()
