"""Per-launch time of census GEMM ops with whichever library CHARPT_LIB names (bench.time_gemm: HIP
events over a hipGraph replay of 30 launches, median of rounds).  Run once with the product library
and once with the what-if build (Makefile p8whatif: k_gemm_p8's bf16 epilogue without its stores) to
price the item epilogue's stores.
usage: [CHARPT_LIB=...] python tools/p8_whatif.py <c2|c4> [rounds] [name,name,...]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import PRESETS, _lib as L  # noqa: E402


def main():
    cfg = PRESETS[sys.argv[1]]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    names = sys.argv[3].split(",") if len(sys.argv) > 3 else None
    dev = torch.device("cuda")
    L.load()
    shapes = [s for s in bench.census_shapes(cfg, cfg.batch_size, cfg.block_size) if names is None or s[0] in names]
    times = {s[0]: [] for s in shapes}
    for _ in range(rounds):
        for name, M, N, K, at, bt, kind, cnt in shapes:
            times[name].append(bench.time_gemm(name, M, N, K, at, bt, kind, dev))
            torch.cuda.empty_cache()
    print(f"library {os.path.basename(L.LIB_PATH)}")
    for name, M, N, K, at, bt, kind, cnt in shapes:
        print(f"{name:11s} M={M} N={N} K={K} {kind:17s} {statistics.median(times[name]) * 1e3:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
