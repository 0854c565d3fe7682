"""Times the charpt attention kernels (fwd, bwd) at the C2 / C4 training shapes for every
per-wave width variant (cg_set_tuning "attn_variant"). GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import functional as Fn  # noqa: E402


def bench(B, T, H, D, p, reps=20):
    dev = torch.device("cuda")
    d = H * D
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    o = torch.empty(B * T, d, dtype=torch.bfloat16, device=dev)
    do = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = (H * D) ** -0.5
    for _ in range(3):
        lse, mask = Fn.attention_fwd(qkv, B, T, H, D, o, scale, p, 1, call, 0)
        Fn.attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, 1, call, 0, mask)
    s, m, e = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    s.record()
    for _ in range(reps):
        lse, mask = Fn.attention_fwd(qkv, B, T, H, D, o, scale, p, 1, call, 0)
    m.record()
    for _ in range(reps):
        Fn.attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, 1, call, 0, mask)
    e.record()
    e.synchronize()
    tf, tb = s.elapsed_time(m) / reps, m.elapsed_time(e) / reps
    fl = 4.0 * B * H * T * T / 2 * D  # causal fwd flops (QK^T + PV)
    print(f"  B={B} T={T} H={H} D={D} p={p}: fwd {tf*1e3:7.1f} us ({fl/tf/1e9:6.1f} TF)  "
          f"bwd {tb*1e3:7.1f} us ({2.5*fl/tb/1e9:6.1f} TF at 2.5x fwd flops)", flush=True)


if __name__ == "__main__":
    lib = L.load()
    variants = [int(a) for a in sys.argv[1:]] or [0, 1, 2, 3]
    for var in variants:
        L.check(lib.cg_set_tuning(b"attn_variant", var))
        print(f"attn_variant {var}", flush=True)
        cfg = os.environ.get("ATTN_CFG", "all")  # c2 | c4 | all (PMC runs: one shape per run)
        ps = (0.2,) if cfg != "all" else (0.0, 0.2)
        for p in ps:
            if cfg in ("c2", "all"):
                bench(64, 256, 6, 64, p)
            if cfg in ("c4", "all"):
                bench(64, 1024, 12, 64, p)
