"""The C2 residual GEMMs with the next LayerNorm: cg_gemm_resid_layernorm (one launch) against
cg_gemm (bias [+ dropout] + residual) + cg_layernorm_fwd, per call (bench._time_ms: hipGraph of 20
calls, HIP events), rounds interleaved.  usage: python tools/gemm_ln_bench.py [rounds]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _time_ms  # noqa: E402
from replicatinggpt_amd import ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda")
    M, N = 16384, 384
    for name, K, p in (("proj_fwd + ln2", 384, 0.0), ("ffn2_fwd + ln1", 1536, 0.2)):
        a = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        bias, lw, lb = (torch.randn(N, device=dev) for _ in range(3))
        resid = torch.randn(M, N, device=dev)
        x = torch.empty(M, N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
        call = torch.zeros(1, dtype=torch.int64, device=dev)

        def fused():
            ops.gemm_resid_layernorm(a, w, x, M, N, K, K, K, N, bias, resid, N, p, 1, call, 3, lw, lb, y, mean, rstd,
                                     1e-5)

        def gemm_only():
            ops.gemm(a, w, x, True, False, False, M, N, K, K, K, N, 4 if p > 0 else 3, bias, resid, N, None, 0, p, 1,
                     call, 3, 0.0, 1, None)

        def two():
            gemm_only()
            ops.layernorm_fwd(x, lw, lb, y, mean, rstd, 1e-5)
        t = {"fused": [], "gemm+ln": [], "gemm": []}
        for r in range(rounds):
            t["fused"].append(_time_ms(fused) * 1e3)
            t["gemm+ln"].append(_time_ms(two) * 1e3)
            t["gemm"].append(_time_ms(gemm_only) * 1e3)
        print(f"{name} (M {M} N {N} K {K} p {p}): " + "  ".join(f"{k} {statistics.median(v):6.2f} us" for k, v in t.items()),
              flush=True)


if __name__ == "__main__":
    main()
