"""Which elements a GEMM-hosted deferred AdamW job (cg_adamw_defer taken by a part-filling
persistent GEMM's free blocks) gets wrong against cg_adamw -- for A/B builds through CHARPT_LIB.
GPU only.  usage: python tools/early_probe2.py [batch,batch,...]  (the A/B build's cg_set_tuning
"adam_batch": 1 = product loop, 4 = four disjoint chunks in flight per thread, 5 = four chunks in flight
with batches stepping by nthr -- overlapping, round 4's candidate bug)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L, ops  # noqa: E402


def main():
    for batch in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1").split(",")]:
        L.check(L.load().cg_set_tuning(b"adam_batch", batch))
        for rep in range(3):
            probe(batch, rep)


def probe(batch, rep):
    torch.manual_seed(0)
    dev = "cuda"
    n = 1 << 20
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev) * 0.1
    m = torch.randn(n, device=dev) * 0.01
    v = torch.rand(n, device=dev) * 0.01
    pb = torch.zeros(n, dtype=torch.bfloat16, device=dev)
    step = torch.tensor([3], dtype=torch.int64, device=dev)
    args = (1e-3, 0.9, 0.999, 1e-8, 0.01)
    ref = [t.clone() for t in (p, m, v, pb)]
    ops.adamw(ref[0], g, ref[1], ref[2], ref[3], *args, step)
    P, M_, V_, PB = p.clone(), m.clone(), v.clone(), pb.clone()
    a, b = 4096, 300000
    ops.adamw_defer(P[a:a + b], g[a:a + b], M_[a:a + b], V_[a:a + b], PB[a:a + b], *args, step)
    x = torch.randn(16384, 384, device=dev).to(torch.bfloat16)
    w = torch.randn(384, 384, device=dev).to(torch.bfloat16)
    y = torch.empty(16384, 384, dtype=torch.bfloat16, device=dev)
    ops.gemm(x, w, y, True, False, False, 16384, 384, 384, 384, 384, 384, 0, None, None, 0, None, 0, 0.0, 0, None, 0,
             0.0, 1, None)
    L.check(L.load().cg_flush_deferred(L.ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    bad = (P != ref[0])[a:a + b].view(-1, 4).any(1).nonzero().view(-1)
    same = (P == p)[a:a + b].view(-1, 4).all(1).nonzero().view(-1)
    nthr = 128 * 256
    print("lib", os.path.basename(L.LIB_PATH), "adam_batch", batch, "rep", rep, "wrong chunks", bad.numel(), "of", b // 4, "never updated", same.numel(),
          "first wrong", bad[:6].tolist(), "mod nthr", (bad[:6] % nthr).tolist(), "div nthr", (bad[:6] // nthr).tolist(),
          flush=True)


if __name__ == "__main__":
    main()
