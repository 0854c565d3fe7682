"""Merged resident attention backward (k_attn_bwd_d64r, C2 shape) with its workgroups in the
longest-first per-XCD order (cg_set_tuning "attn_bwd_lpt" 1: every dK/dV workgroup of an XCD's
(b, h) range before its dQ workgroups) against the interleaved order (0), same process: gradients
compared bit for bit, then the backward time (tools/attn_bench._time: HIP events around a hipGraph
replay of 20 calls), rounds interleaved.  usage: python tools/attn_lpt_ab.py [rounds] [p]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import functional as Fn  # noqa: E402
from tools.attn_bench import _time  # noqa: E402


def set_lpt(v):
    L.check(L.load().cg_set_tuning(b"attn_bwd_lpt", v), "attn_bwd_lpt")


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
    B, T, H, D = 64, 256, 6, 64
    dev = torch.device("cuda")
    d = H * D
    torch.manual_seed(3)
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    o = torch.empty(B * T, d, dtype=torch.bfloat16, device=dev)
    do = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = d ** -0.5
    lse, mask = Fn.attention_fwd(qkv, B, T, H, D, o, scale, p, 1, call, 0)
    grads = []
    for v in (0, 1):
        set_lpt(v)
        g = Fn.attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, 1, call, 0, mask)
        torch.cuda.synchronize()
        grads.append(g.clone() if torch.is_tensor(g) else [t.clone() for t in g])
    same = torch.equal(grads[0], grads[1]) if torch.is_tensor(grads[0]) else all(
        torch.equal(a, b) for a, b in zip(grads[0], grads[1]))
    print(f"C2 attention backward p={p}: gradients bitwise {'equal' if same else 'DIFFERENT'} across orders", flush=True)
    t = {0: [], 1: []}
    for r in range(rounds):
        for v in (0, 1):
            set_lpt(v)
            t[v].append(_time(lambda: Fn.attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, 1, call, 0, mask)))
    set_lpt(1)
    m0, m1 = statistics.median(t[0]), statistics.median(t[1])
    print(f"bwd interleaved (0): median {m0:.2f} us  {[round(x, 2) for x in t[0]]}")
    print(f"bwd dK/dV first (1): median {m1:.2f} us  {[round(x, 2) for x in t[1]]}  ({(m1 / m0 - 1) * 100:+.1f} %)")


if __name__ == "__main__":
    main()
