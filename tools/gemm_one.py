"""Runs one charpt bf16 GEMM shape/variant REPS times (for rocprofv3 PMC passes).  GPU only.
usage: python tools/gemm_one.py M N K at bt variant [reps] [split]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import ops  # noqa: E402


def main():
    M, N, K, at, bt, v = (int(x) for x in sys.argv[1:7])
    reps = int(sys.argv[7]) if len(sys.argv) > 7 else 20
    split = int(sys.argv[8]) if len(sys.argv) > 8 else 1
    lib = L.load()
    L.check(lib.cg_set_tuning(b"gemm_variant", v))
    A = torch.randn((K, M) if at else (M, K), device="cuda").to(torch.bfloat16)
    B = torch.randn((K, N) if bt else (N, K), device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.float32 if split > 1 else torch.bfloat16, device="cuda")
    ws = torch.empty(max(1, ops.gemm_workspace(M, N, split) // 4), dtype=torch.float32, device="cuda")
    for _ in range(reps):
        ops.gemm(A, B, out, True, bool(at), bool(bt), M, N, K, A.shape[1], B.shape[1], N, 0, None, None, 0, None, 0,
                 0.0, 0, None, 0, 0.0, split, ws if split > 1 else None)
    torch.cuda.synchronize()
    print("done", M, N, K, at, bt, v)


if __name__ == "__main__":
    main()
