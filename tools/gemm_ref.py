"""Calibration only (not part of the product path): times torch.matmul (hipBLASLt) on the same
GEMM shapes/layouts as bench.gemm_census, next to the charpt kernel, to see the headroom a
library kernel shows on MI355X for these (small-K / small-N) shapes.  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import PRESETS  # noqa: E402
import bench  # noqa: E402


def time_torch(M, N, K, at, bt, dev, reps=30):
    A = torch.randn((K, M) if at else (M, K), device=dev).to(torch.bfloat16)
    B = torch.randn((K, N) if bt else (N, K), device=dev).to(torch.bfloat16)
    a = A.t() if at else A
    b = B if bt else B.t()
    for _ in range(3):
        torch.matmul(a, b)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        torch.matmul(a, b)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    cfg = PRESETS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    B = cfg.batch_size if len(sys.argv) <= 2 else int(sys.argv[2])
    dev = torch.device("cuda")
    cen = bench.gemm_census(cfg, B, cfg.block_size, dev)
    tot_c = tot_t = 0.0
    for c in cen:
        shp = dict(M=c["M"], N=c["N"], K=c["K"])
        at = c["name"].endswith("wgrad")
        bt = c["name"].endswith("wgrad") or c["name"].endswith("dgrad")
        tt = time_torch(c["M"], c["N"], c["K"], at, bt, dev)
        tot_c += c["ms"] * c["launches"]
        tot_t += tt * c["launches"]
        print(f"{c['name']:12s} {shp}  charpt {c['ms']*1e3:7.1f} us {c['flops']/c['ms']/1e9:6.0f} TF   "
              f"torch {tt*1e3:7.1f} us {c['flops']/tt/1e9:6.0f} TF", flush=True)
    print(f"step total: charpt {tot_c:.3f} ms  torch {tot_t:.3f} ms")


if __name__ == "__main__":
    main()
