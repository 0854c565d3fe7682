"""The bench's GEMM census (bench.gemm_census: every GEMM of the C2 / C4 step with the step's fused
epilogue, HIP events over a hipGraph replay of 30 launches) printed per op -- for A/B runs of two
library builds (CHARPT_LIB=...).  usage: python tools/census.py [c2|c4] [tag] [cold]
(cold: every launch's operands cycled past the Infinity Cache, bench.census_op)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import PRESETS  # noqa: E402


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(os.environ.get("CHARPT_LIB", "product"))
    cfg = PRESETS[cfg_name]
    cold = len(sys.argv) > 3 and sys.argv[3] == "cold"
    cen = bench.gemm_census(cfg, cfg.batch_size, cfg.block_size, torch.device("cuda"), cold=cold)
    fam = bench.gemm_family(cen)
    line = " ".join(f"{c['name']}={c['ms'] * 1e3:.1f}" for c in cen)
    print(f"{tag:28s} {cfg_name} family {fam['ms_per_step']:.4f} ms/step ({fam['frac']:.4f}) | {line}", flush=True)


if __name__ == "__main__":
    main()
