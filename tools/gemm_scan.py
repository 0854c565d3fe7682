"""GEMM timing scan: each shape/variant replayed from a hipGraph of 20 back-to-back launches
(no host launch overhead), plus an HBM copy of the same bytes as a floor.  GPU only.

usage: python tools/gemm_scan.py [variants=1,2,3,4]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import ops  # noqa: E402

REPS = 20


def graph_time(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / REPS)
    return best


def gemm_fn(M, N, K, at, bt, split=1):
    dev = "cuda"
    A = torch.randn((K, M) if at else (M, K), device=dev).to(torch.bfloat16)
    B = torch.randn((K, N) if bt else (N, K), device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.float32 if split > 1 else torch.bfloat16, device=dev)
    ws = torch.empty(max(1, ops.gemm_workspace(M, N, split) // 4), dtype=torch.float32, device=dev)

    def run():
        ops.gemm(A, B, out, True, bool(at), bool(bt), M, N, K, A.shape[1], B.shape[1], N, 0, None, None, 0, None, 0,
                 0.0, 0, None, 0, 0.0, split, ws if split > 1 else None)
    return run


def main():
    lib = L.load()
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3,4").split(",")]
    if os.environ.get("SCAN") == "k":
        shapes = [(16384, 384, k, 0, 0) for k in (64, 128, 256, 384, 768, 1536, 3072)] + \
                 [(m, 384, 384, 0, 0) for m in (2048, 4096, 8192, 32768)]
    else:
        shapes = None
    shapes = shapes or [(16384, 384, 384, 0, 0), (65536, 384, 384, 0, 0), (16384, 1536, 384, 0, 0), (16384, 384, 1536, 0, 0),
              (16384, 1152, 384, 0, 0), (16384, 384, 1536, 0, 1), (16384, 1536, 384, 0, 1), (384, 1536, 16384, 1, 1), (4096, 4096, 4096, 0, 1)]
    if os.environ.get("SCAN") == "w":
        for M, N, K in [(384, 1536, 16384), (1536, 384, 16384), (1152, 384, 16384), (384, 384, 16384)]:
            for split in (4, 8, 16, 32):
                line = f"wgrad TT M={M:5d} N={N:5d} K={K:6d} split {split:2d} |"
                for v in variants:
                    L.check(lib.cg_set_tuning(b"gemm_variant", v))
                    t = graph_time(gemm_fn(M, N, K, 1, 1, split))
                    line += f" v{v} {t*1e3:6.1f}us {2*M*N*K/t/1e9:5.0f}TF"
                print(line, flush=True)
        L.check(lib.cg_set_tuning(b"gemm_variant", 0))
        return
    for M, N, K, at, bt in shapes:
        byts = 2 * (M * K + N * K + M * N)
        x = torch.empty(byts // 4, dtype=torch.float32, device="cuda")
        y = torch.empty_like(x)
        tc = graph_time(lambda: y.copy_(x))
        line = f"M={M:6d} N={N:5d} K={K:5d} {'T' if at else 'N'}{'T' if bt else 'N'} bytes {byts/1e6:6.1f}MB " \
               f"copy {tc*1e3:6.1f}us |"
        for v in variants:
            L.check(lib.cg_set_tuning(b"gemm_variant", v))
            t = graph_time(gemm_fn(M, N, K, at, bt))
            line += f" v{v} {t*1e3:6.1f}us {2*M*N*K/t/1e9:5.0f}TF"
        print(line, flush=True)
    L.check(lib.cg_set_tuning(b"gemm_variant", 0))


if __name__ == "__main__":
    main()
