"""Split-K scan of the weight-gradient GEMMs with bf16 slabs (cg_epilogue_t.flags CG_GEMM_SLAB_BF16, the training
step's form): GEMM + standalone slab reduce per call, hipGraph of 20 calls (bench._time_ms), against
the split functional._wgrad_split picks.  GPU only.
usage: python tools/wgrad_split_scan.py [c2|c4] [splits]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from replicatinggpt_amd import _lib as L, ops  # noqa: E402
from replicatinggpt_amd import functional as Fn  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    splits = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "8,12,14,16,18,24,28,32,40,48,56,64").split(",")]
    d, M = (384, 16384) if cfg == "c2" else (768, 65536)
    lib = L.load()
    for name, m, n in (("proj_wgrad", d, d), ("qkv_wgrad", 3 * d, d), ("ffn2_wgrad", d, 4 * d),
                       ("ffn1_wgrad", 4 * d, d)):
        A = (torch.randn(M, m, device="cuda") * 0.5).to(torch.bfloat16)
        B = (torch.randn(M, n, device="cuda") * 0.5).to(torch.bfloat16)
        out = torch.empty(m, n, device="cuda")
        pick = Fn._wgrad_split(m, n, M, True)
        line = f"{cfg} {name:10s} M={m:5d} N={n:5d} K={M} (picked {pick:2d}) |"
        nkt = M // 64
        for sp in sorted(set(splits + [pick])):
            per = -(-nkt // sp)
            if (sp - 1) * per >= nkt:
                continue
            ws = torch.empty(ops.gemm_workspace(m, n, sp) // 4, dtype=torch.float32, device="cuda")

            def run(sp=sp, ws=ws):
                ops.gemm(A, B, out, True, True, True, m, n, M, m, n, n, 0, None, None, 0, None, 0, 0.0, 0, None, 0,
                         0.0, sp, ws, L.GEMM_SLAB_BF16)
            t = bench._time_ms(run) * 1e3
            line += f" s{sp} {t:5.1f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
