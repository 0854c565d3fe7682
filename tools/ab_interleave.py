"""Same-process interleaved A/B of cg_set_tuning variants: each round times every variant once
(HIP events around a hipGraph replay of 20 back-to-back calls), rounds repeated, median and min per
variant reported -- box-to-box and run-to-run drift (±4 % at C4) cancels out of the comparison.
usage: python tools/ab_interleave.py attn_fwd|attn_bwd|adamw <knob> <v,v,...> [rounds] [cfg c2|c4]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import functional as Fn, ops  # noqa: E402
from tools.attn_bench import _time  # noqa: E402

SHAPES = {"c2": (64, 256, 6, 64), "c4": (64, 1024, 12, 64)}


def attn_work(kind, cfg, p=0.2):
    B, T, H, D = SHAPES[cfg]
    dev = torch.device("cuda")
    C = H * D
    qkv = (torch.randn(B * T, 3 * C, device=dev) * 0.5).to(torch.bfloat16)
    o = torch.empty(B * T, C, dtype=torch.bfloat16, device=dev)
    do = torch.randn(B * T, C, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    mask = torch.empty(ops.attn_mask_bytes(B, H, T) // 8, dtype=torch.int64, device=dev)
    lse = torch.empty((B, H, T), dtype=torch.float32, device=dev)
    ops.attn_dropmask(B, H, T, p, 1, call, 0, mask)
    scale = C ** -0.5
    fwd = lambda: ops.attn_fwd(qkv, B, T, H, D, 0, C, 2 * C, qkv.stride(0), o, C, lse, scale, p, 1, call, 0, mask, True)
    fwd()
    if kind == "attn_fwd":
        return fwd
    return lambda: Fn.attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, 1, call, 0, mask)


def adamw_work(cfg):
    n = 10788992 if cfg == "c2" else 85997568
    dev = torch.device("cuda")
    p, g, m, v = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
    v.abs_()
    p16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    step = torch.ones(1, dtype=torch.int64, device=dev)
    return lambda: ops.adamw(p, g, m, v, p16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)


def main():
    kind, knob, vals = sys.argv[1], sys.argv[2].encode(), [int(x) for x in sys.argv[3].split(",")]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 7
    cfg = sys.argv[5] if len(sys.argv) > 5 else "c4"
    lib = L.load()
    fn = adamw_work(cfg) if kind == "adamw" else attn_work(kind, cfg)
    res = {v: [] for v in vals}
    try:
        for _ in range(rounds):
            for v in vals:
                L.check(lib.cg_set_tuning(knob, v))
                res[v].append(_time(fn))
    finally:
        L.check(lib.cg_set_tuning(knob, 0))
    for v in vals:
        print(f"{kind} {cfg} {knob.decode()}={v}: median {statistics.median(res[v]):8.1f} us  min {min(res[v]):8.1f} us  "
              f"[{' '.join(f'{x:.1f}' for x in res[v])}]", flush=True)


if __name__ == "__main__":
    main()
