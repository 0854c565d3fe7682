"""Times the charpt attention kernels at the C2 / C4 training shapes: the keep-bit kernel alone,
the forward on premade keep bits, the forward with its keep bits (what bench.py's kernel_census
counts) and the backward (dQ + dK/dV).  Each figure = HIP events around one hipGraph replay of
`reps` back-to-back calls.  GPU only.  ATTN_CFG = c2 | c4 | all; ATTN_P = one dropout p."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import functional as Fn, ops  # noqa: E402


def _time(fn, reps=20):
    for _ in range(3):
        fn()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3   # us


def bench(B, T, H, D, p):
    dev = torch.device("cuda")
    d = H * D
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    o = torch.empty(B * T, d, dtype=torch.bfloat16, device=dev)
    do = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = (H * D) ** -0.5
    st = {}
    mask = torch.empty(ops.attn_mask_bytes(B, H, T) // 8, dtype=torch.int64, device=dev)
    lse = torch.empty((B, H, T), dtype=torch.float32, device=dev)
    t_mask = _time(lambda: ops.attn_dropmask(B, H, T, p, 1, call, 0, mask)) if p > 0 else 0.0

    def fwd_pre():
        ops.attn_fwd(qkv, B, T, H, D, 0, d, 2 * d, qkv.stride(0), o, d, lse, scale, p, 1, call, 0,
                     mask if p > 0 else None, p > 0)
    t_fpre = _time(fwd_pre)

    def fwd():
        st["lse"], st["mask"] = Fn.attention_fwd(qkv, B, T, H, D, o, scale, p, 1, call, 0)
    t_f = _time(fwd)
    t_b = _time(lambda: Fn.attention_bwd(qkv, B, T, H, D, o, do, st["lse"], scale, p, 1, call, 0, st["mask"]))
    fl = 4.0 * B * H * (T * (T + 1) / 2) * D   # causal algorithmic flops (QK^T + PV), bench.py kernel_census
    print(f"  B={B} T={T} H={H} D={D} p={p}: mask {t_mask:7.1f} us | fwd(premasked) {t_fpre:7.1f} us "
          f"({fl / t_fpre / 1e6:6.1f} TF) | fwd {t_f:7.1f} us ({fl / t_f / 1e6:6.1f} TF = {fl / t_f / 1e6 / 2500:.3f}) | "
          f"bwd {t_b:7.1f} us ({2 * fl / t_b / 1e6:6.1f} TF = {2 * fl / t_b / 1e6 / 2500:.3f})", flush=True)


if __name__ == "__main__":
    L.load()
    cfg = os.environ.get("ATTN_CFG", "all")
    ps = (0.2,) if cfg != "all" else (0.0, 0.2)
    if "ATTN_P" in os.environ:
        ps = (float(os.environ["ATTN_P"]),)
    for p in ps:
        if cfg in ("c2", "all"):
            bench(64, 256, 6, 64, p)
        if cfg in ("c4", "all"):
            bench(64, 1024, 12, 64, p)
