"""Calibration (GPU, 1 process): do external events recorded inside a hipGraph order host-issued
work on another stream correctly (the DP engine queues RCCL all-reduces behind per-bucket events
recorded inside the captured backward)?  Each replay: a chain of GEMMs, then counter += 1 (side
stream branch), external event, more GEMMs.  After each replay the host makes stream X wait on the
event and copies the counter: every copy must equal the replay index (no stale reads), and the
copy should complete before the graph ends (overlap)."""
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
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)

    def gemm():
        ops.gemm(A, B, C, True, False, False, M, N, K, K, K, N, 0, None, None, 0, None, 0, 0.0, 0, None, 0, 0.0, 1,
                 None)

    side = torch.cuda.Stream()
    ev = torch.cuda.Event(external=True)
    cap = torch.cuda.Stream()

    def body():
        cur = torch.cuda.current_stream()
        for _ in range(20):
            gemm()
        ops.counter_add(ctr, 1)
        side.wait_stream(cur)
        ev.record(side)
        cur.wait_stream(side)
        for _ in range(40):
            gemm()

    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        body()
    torch.cuda.current_stream().wait_stream(cap)
    torch.cuda.synchronize()
    ctr.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    ctr.zero_()
    X = torch.cuda.Stream()
    outs = torch.zeros(50, dtype=torch.int64, device=dev)
    e_end = [torch.cuda.Event(enable_timing=True) for _ in range(50)]
    e_x = [torch.cuda.Event(enable_timing=True) for _ in range(50)]
    e_start = [torch.cuda.Event(enable_timing=True) for _ in range(50)]
    for i in range(50):
        e_start[i].record()
        g.replay()
        e_end[i].record()
        X.wait_event(ev)
        with torch.cuda.stream(X):
            outs[i:i + 1].copy_(ctr)
            e_x[i].record(X)
        torch.cuda.current_stream().wait_stream(X)
    torch.cuda.synchronize()
    got = outs.cpu().tolist()
    stale = sum(1 for i, v in enumerate(got) if v != i + 1)
    t_x = [e_start[i].elapsed_time(e_x[i]) for i in range(50)]
    t_end = [e_start[i].elapsed_time(e_end[i]) for i in range(50)]
    print(f"stale reads: {stale}/50  (values {got[:8]}...)")
    print(f"median: side-copy done at {sorted(t_x)[25]:.3f} ms, graph done at {sorted(t_end)[25]:.3f} ms "
          f"-> {'OVERLAPPED' if sorted(t_x)[25] < sorted(t_end)[25] else 'serialized'}")


if __name__ == "__main__":
    main()
