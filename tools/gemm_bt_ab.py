"""A/B of the N = 384 dgrad GEMMs with a transposed-B operand (the weight as stored, b_trans = 1:
the training path) against a pre-transposed weight copy (b_trans = 0, the forward's operand
layout), plain bf16 stores, hot operands, HIP events over REPS launches.  GPU only.
usage: python tools/gemm_bt_ab.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import ops  # noqa: E402


def time_one(A, B, out, M, N, K, bt, reps):
    def run():
        ops.gemm(A, B, out, True, False, bool(bt), M, N, K, A.shape[1], B.shape[1], N, 0, None, None, 0, None, 0,
                 0.0, 0, None, 0, 0.0, 1, None)
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    M, N = 16384, 384
    for K in (384, 1152, 1536):
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        W = (torch.randn(K, N, device="cuda") * K ** -0.5).to(torch.bfloat16)   # weight [out = K, in = N]
        Wt = W.t().contiguous()                                                 # [in, out]
        o1 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        o0 = torch.empty_like(o1)
        t1 = time_one(A, W, o1, M, N, K, 1, reps)
        t0 = time_one(A, Wt, o0, M, N, K, 0, reps)
        same = torch.equal(o0.view(torch.int16), o1.view(torch.int16))
        print(f"M={M} N={N} K={K}: b_trans=1 {t1:7.2f} us   b_trans=0 (pre-transposed) {t0:7.2f} us   "
              f"bitwise equal {same}", flush=True)


if __name__ == "__main__":
    main()
