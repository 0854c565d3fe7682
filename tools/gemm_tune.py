"""Times every charpt bf16 GEMM shape of a training step under each kernel variant
(cg_set_tuning("gemm_variant", v)) and prints a table + JSON.  GPU only."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L, PRESETS  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--variants", default="1,2,3,4")
    ap.add_argument("--batch", type=int, default=None)
    a = ap.parse_args()
    cfg = PRESETS[a.config]
    B = a.batch or cfg.batch_size
    dev = torch.device("cuda")
    lib = L.load()
    res = {}
    for v in [int(x) for x in a.variants.split(",")]:
        L.check(lib.cg_set_tuning(b"gemm_variant", v))
        cen = bench.gemm_census(cfg, B, cfg.block_size, dev)
        res[v] = {c["name"]: c["ms"] for c in cen}
        tot = sum(c["ms"] * c["launches"] for c in cen)
        print(f"variant {v}: step GEMM total {tot:.3f} ms")
        for c in cen:
            print(f"   {c['name']:12s} M={c['M']:6d} N={c['N']:5d} K={c['K']:6d} {c['ms']*1e3:8.1f} us "
                  f"{c['flops']/c['ms']/1e9:7.1f} TF")
    best = {n: min(res, key=lambda v: res[v][n]) for n in res[next(iter(res))]}
    print("best:", json.dumps(best))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
