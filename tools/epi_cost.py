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


def case_fused(M, N, K, kind):
    """The two fused forms the training step launches: bias+ReLU with keep bits (W1 forward) and
    ReLU-backward from keep bits with the b1 column partials (W2 dgrad)."""
    dev = "cuda"
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    bits = torch.randint(-2**31, 2**31 - 1, (M, N // 32), dtype=torch.int32, device=dev)
    if kind == "bits":
        B = torch.randn(N, K, device=dev).to(torch.bfloat16)
        bias = torch.randn(N, device=dev)
        run = lambda: ops.gemm_bias_relu_bits(A, B, out, M, N, K, K, K, N, bias, bits, N // 32)
    else:
        B = torch.randn(K, N, device=dev).to(torch.bfloat16)
        part = torch.empty(M // 64, N, device=dev)
        run = lambda: ops.gemm_relu_bwd_colpart(A, B, out, M, N, K, K, N, N, bits, N // 32, part)
    return graph_time(run) * 1e3


def main():
    M, d = 16384, 384
    F4 = 4 * d
    rows = [("ffn1_fwd store bf16", M, F4, d, 0, L.EPI_STORE, torch.bfloat16, 0.0),
            ("ffn1_fwd bias_relu bf16", M, F4, d, 0, L.EPI_BIAS_RELU, torch.bfloat16, 0.0),
            ("ffn2_fwd store bf16", M, d, F4, 0, L.EPI_STORE, torch.bfloat16, 0.0),
            ("ffn2_fwd store f32", M, d, F4, 0, L.EPI_STORE, torch.float32, 0.0),
            ("ffn2_fwd bias_resid f32", M, d, F4, 0, L.EPI_BIAS_RESID, torch.float32, 0.0),
            ("ffn2_fwd bias_drop_resid f32 p=0.2", M, d, F4, 0, L.EPI_BIAS_DROP_RESID, torch.float32, 0.2),
            ("ffn2_dgrad store bf16", M, F4, d, 1, L.EPI_STORE, torch.bfloat16, 0.0),
            ("ffn2_dgrad relu_bwd bf16", M, F4, d, 1, L.EPI_RELU_BWD, torch.bfloat16, 0.0),
            ("proj_fwd store bf16", M, d, d, 0, L.EPI_STORE, torch.bfloat16, 0.0),
            ("proj_fwd store f32", M, d, d, 0, L.EPI_STORE, torch.float32, 0.0),
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
    for name, kind, n, k in (("ffn1_fwd bias_relu+bits bf16", "bits", F4, d),
                             ("ffn2_dgrad relu_bwd bits+colpart bf16", "colpart", F4, d)):
        print(f"{name:38s} " + " ".join(f"{case_fused(M, n, k, kind):6.1f} us" for _ in flags), flush=True)


if __name__ == "__main__":
    main()
