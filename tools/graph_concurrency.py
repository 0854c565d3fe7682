"""Does a hipGraph replay run kernels captured on two forked streams concurrently on MI355X?
Times (a) two independent workloads serialized on one stream, (b) forked onto two streams,
eager and graph-replayed.  GPU only; calibration for engine.py's side-stream overlap."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L, ops  # noqa: E402


def main():
    L.load()
    dev = "cuda"
    M, N, K = 16384, 1536, 384
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = torch.randn(N, K, device=dev).to(torch.bfloat16)
    C1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    C2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(32 << 20, device=dev)
    y = torch.empty_like(x)

    def g1(out):
        ops.gemm(A, B, out, True, False, False, M, N, K, K, K, N, 0, None, None, 0, None, 0, 0.0, 0, None, 0, 0.0, 1,
                 None)

    side = torch.cuda.Stream()

    def serial():
        for _ in range(4):
            g1(C1)
            g1(C2)

    def forked():
        cur = torch.cuda.current_stream()
        for _ in range(4):
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                g1(C2)
            g1(C1)
            cur.wait_stream(side)

    def timeit(fn, graph):
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                fn()
            run = gr.replay
        else:
            run = fn
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best * 1e3 / 8

    for v in (9, 23):
        L.check(L.load().cg_set_tuning(b"gemm_variant", v))
        for mg in (0, 256):
            L.check(L.load().cg_set_tuning(b"gemm_max_grid", mg))
            print(f"variant {v} max_grid {mg}: per-GEMM us  serial eager {timeit(serial, False):6.1f}  "
                  f"forked eager {timeit(forked, False):6.1f}  serial graph {timeit(serial, True):6.1f}  "
                  f"forked graph {timeit(forked, True):6.1f}", flush=True)
    L.check(L.load().cg_set_tuning(b"gemm_variant", 0))
    L.check(L.load().cg_set_tuning(b"gemm_max_grid", 0))


if __name__ == "__main__":
    main()
