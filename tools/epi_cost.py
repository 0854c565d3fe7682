"""Cost of the fused GEMM epilogues on the C2 FFN shapes: the same product timed with the plain
store and with the epilogue the training step uses (hipGraph of 20 launches, best of 5).  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_scan import graph_time  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import ops  # noqa: E402


def case(M, N, K, bt, epi, out_dtype, p=0.0):
    dev = "cuda"
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = (torch.randn(K, N, device=dev) if bt else torch.randn(N, K, device=dev)).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=out_dtype, device=dev)
    bias = torch.randn(N, device=dev)
    resid = torch.randn(M, N, device=dev)
    aux = torch.randn(M, N, device=dev).to(torch.bfloat16)
    call = torch.tensor([3], dtype=torch.int64, device=dev)

    def run():
        ops.gemm(A, B, out, True, False, bool(bt), M, N, K, K, B.shape[1], N, epi,
                 bias if epi in (1, 2, 3, 4) else None, resid if epi in (3, 4) else None, N,
                 aux if epi == 5 else None, N, p, 1234, call if p > 0 else None, 1, 0.0, 1, None)
    return graph_time(run) * 1e3


def main():
    M, d = 16384, 384
    F4 = 4 * d
    rows = [("ffn1_fwd store bf16", M, F4, d, 0, L.EPI_STORE, torch.bfloat16, 0.0),
            ("ffn1_fwd bias_relu bf16", M, F4, d, 0, L.EPI_BIAS_RELU, torch.bfloat16, 0.0),
            ("ffn2_fwd store f32", M, d, F4, 0, L.EPI_STORE, torch.float32, 0.0),
            ("ffn2_fwd bias_resid f32", M, d, F4, 0, L.EPI_BIAS_RESID, torch.float32, 0.0),
            ("ffn2_fwd bias_drop_resid f32 p=0.2", M, d, F4, 0, L.EPI_BIAS_DROP_RESID, torch.float32, 0.2),
            ("ffn2_dgrad store bf16", M, F4, d, 1, L.EPI_STORE, torch.bfloat16, 0.0),
            ("ffn2_dgrad relu_bwd bf16", M, F4, d, 1, L.EPI_RELU_BWD, torch.bfloat16, 0.0),
            ("proj_fwd bias_resid f32", M, d, d, 0, L.EPI_BIAS_RESID, torch.float32, 0.0),
            ("qkv_fwd store bf16", M, 3 * d, d, 0, L.EPI_STORE, torch.bfloat16, 0.0)]
    flags = [int(a) for a in sys.argv[1:]] or [0]
    lib = L.load()
    print(f"{'pk_flags':38s} " + " ".join(f"{f:9d}" for f in flags), flush=True)
    for name, m, n, k, bt, epi, dt, p in rows:
        ts = []
        for f in flags:
            L.check(lib.cg_set_tuning(b"pk_flags", f))
            ts.append(case(m, n, k, bt, epi, dt, p))
        L.check(lib.cg_set_tuning(b"pk_flags", 0))
        print(f"{name:38s} " + " ".join(f"{t:6.1f} us" for t in ts), flush=True)


if __name__ == "__main__":
    main()
