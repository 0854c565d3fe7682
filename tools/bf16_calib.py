"""bf16 gradient calibration: how far torch's OWN bf16 path (torch.autocast over
the oracle's functional forward, GPT1.py:176-194) lands from the fp32 oracle on the C2 step, per
parameter -- the yardstick charpt's bf16 gradients are held to.  Also emulates single rounding
points on the fp32 oracle (CALIB_ROUND=<point>) to find which one a per-parameter error comes from.

usage: python tools/bf16_calib.py [cpu|cuda] [batch]     (test infrastructure: reads oracle/)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gpt1_oracle as O  # noqa: E402


SEED = 0x1337   # GPTConfig.dropout_seed


def normrel(a, b):
    a, b = a.double().flatten().cpu(), b.double().flatten().cpu()
    return float((a - b).norm() / b.norm())


def grads(P, idx, tgt, ocfg, dev, autocast):
    Pd = {k: v.to(dev) for k, v in P.items()}
    ctx = torch.autocast(device_type=dev, dtype=torch.bfloat16) if autocast else torch.autocast(dev, enabled=False)
    with ctx:
        _, loss, g = O.loss_and_grads(Pd, idx.to(dev), tgt.to(dev), ocfg, train=True, seed=SEED, call=0)
    return float(loss), {k: v.float().cpu() for k, v in g.items()}


def main():
    dev = sys.argv[1] if len(sys.argv) > 1 else "cpu"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    ocfg = O.OracleConfig(block_size=256, n_embd=384, n_head=6, n_layers=6, dropout=0.2)
    g = torch.Generator().manual_seed(17)
    idx = torch.randint(0, 65, (B, 256), generator=g)
    tgt = torch.randint(0, 65, (B, 256), generator=g)
    torch.manual_seed(1337)
    P = O.init_params(ocfg)
    t0 = time.time()
    l32, g32 = grads(P, idx, tgt, ocfg, dev, False)
    t1 = time.time()
    l16, g16 = grads(P, idx, tgt, ocfg, dev, True)
    t2 = time.time()
    print(f"B={B} dev={dev}: loss fp32 {l32:.6f} ({t1 - t0:.1f} s) autocast-bf16 {l16:.6f} ({t2 - t1:.1f} s)")
    rows = sorted(((normrel(g16[k], g32[k]), k) for k in g32), reverse=True)
    for r, k in rows[:16]:
        print(f"  {k:40s} normrel {r:.4f}")
    rs = sorted(r for r, _ in rows)
    print(f"  median {rs[len(rs) // 2]:.4f}  max {rs[-1]:.4f}")


if __name__ == "__main__":
    main()
