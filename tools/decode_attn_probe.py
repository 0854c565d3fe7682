"""Probe: what the phase-1 decode attention (cg_decode_attn, C5: B = 256, H = 6, D = 21, [B, H, 256, D]
cache) waits on.  Per-launch time from a hipGraph of 20 launches (HIP events) at several key counts, batch
sizes and cache row strides, beside a plain copy of the same K / V bytes.
usage: python tools/decode_attn_probe.py [ab]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import ops  # noqa: E402


def graph_us(run, reps=20):
    run()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            run()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


def case(B, H, D, n, sj, T=256):
    dev = torch.device("cuda")
    kc = torch.randn(B, H, T, sj, device=dev)
    vc = torch.randn(B, H, T, sj, device=dev)
    q = torch.randn(B, 3 * H * D, device=dev)
    o = torch.empty(B, H * D, device=dev)
    sb, sh = H * T * sj, T * sj

    def run():
        ops.decode_attn(q, 3 * H * D, kc, 0, vc, 0, sb, sh, sj, B, H, D, None, n, D ** -0.5, o)
    t = graph_us(run)
    mb = 2 * B * H * n * D * 4 / 1e6
    ks, vs = kc[:, :, :n], vc[:, :, :n]
    dst = torch.empty_like(ks)

    def copy():
        dst.copy_(ks)
        dst.copy_(vs)
    tc = graph_us(copy)
    print(f"B={B:4d} H={H} D={D} n={n:3d} row stride {sj:3d}: {t:7.2f} us  ({mb:6.1f} MB of K/V rows, "
          f"{mb / t:5.2f} TB/s); copy of those rows {tc:7.2f} us", flush=True)


def window(B, H, D, T):
    """phase 2's call: the last query against a window's qkv rows (row stride 3 C)"""
    C = H * D
    qkv = torch.randn(B, T, 3 * C, device="cuda")
    q = torch.randn(B, 3 * C, device="cuda")
    o = torch.empty(B, C, device="cuda")

    def run():
        ops.decode_attn(q, 3 * C, qkv, C, qkv, 2 * C, T * 3 * C, D, 3 * C, B, H, D, None, T, D ** -0.5, o)
    t = graph_us(run)
    print(f"B={B:4d} H={H} D={D} n={T:3d} window qkv rows: {t:7.2f} us", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ab":   # lane-per-key (0) vs coalesced-chunk (1) kernel
        from replicatinggpt_amd import _lib as L
        for v in (0, 1, 0, 1):
            L.check(L.load().cg_set_tuning(b"decode_attn_rows", v))
            print(f"decode_attn_rows {v}", flush=True)
            for n in (1, 64, 128, 256):
                case(256, 6, 21, n, 21)
            window(256, 6, 21, 256)
        sys.exit(0)
    for n in (64, 128, 256):
        case(256, 6, 21, n, 21)
    for B in (32, 64, 128):
        case(B, 6, 21, 256, 21)
    case(256, 6, 21, 256, 24)
    case(256, 6, 21, 256, 32)
