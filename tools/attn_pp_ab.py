"""C4 attention forward: the 8-wave ping-pong kernel (k_attn_fwd_pp; A/B build, cg_set_tuning
"attn_variant" 4, T % 256 == 0, 512 <= T <= 1024) against the shipped 4-wave ring kernel (0), same process:
O and the log-sum-exp compared bit for bit on the same premade keep bits, then the forward time
(tools/attn_bench._time: HIP events around a hipGraph replay of 20 calls), rounds interleaved.
usage: CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_ab.so python tools/attn_pp_ab.py [rounds] [T]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L, ops  # noqa: E402
from tools.attn_bench import _time  # noqa: E402


def set_v(v):
    L.check(L.load().cg_set_tuning(b"attn_variant", v), "attn_variant")


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    B, H, D = 64, 12, 64
    dev = torch.device("cuda")
    d = H * D
    scale = d ** -0.5
    fl = 4.0 * B * H * (T * (T + 1) / 2) * D
    torch.manual_seed(1)
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    for p in (0.0, 0.2):
        mask = torch.empty(ops.attn_mask_bytes(B, H, T) // 8, dtype=torch.int64, device=dev)
        if p > 0:
            ops.attn_dropmask(B, H, T, p, 1, call, 0, mask)
        outs = {}
        for v in (0, 4):
            set_v(v)
            o = torch.full((B * T, d), float("nan"), dtype=torch.bfloat16, device=dev)
            lse = torch.full((B, H, T), float("nan"), dtype=torch.float32, device=dev)

            def fwd():
                ops.attn_fwd(qkv, B, T, H, D, 0, d, 2 * d, qkv.stride(0), o, d, lse, scale, p, 1, call, 0,
                             mask if p > 0 else None, p > 0)
            fwd()
            torch.cuda.synchronize()
            outs[v] = (o.clone(), lse.clone(), fwd)
        same_o = torch.equal(outs[4][0], outs[0][0])
        same_l = torch.equal(outs[4][1], outs[0][1])
        nan = bool(torch.isnan(outs[4][0].float()).any() or torch.isnan(outs[4][1]).any())
        print(f"T={T} p={p}: O bitwise {'equal' if same_o else 'DIFFERENT'}, lse bitwise "
              f"{'equal' if same_l else 'DIFFERENT'}, nan {nan}", flush=True)
        if not (same_o and same_l):
            diff = (outs[4][0].float() - outs[0][0].float()).abs()
            print(f"  max |dO| {diff.max().item():.3e} at {int(diff.argmax())}; rows differing "
                  f"{int((diff.view(B * T, d) > 0).any(1).sum())}", flush=True)
        t = {0: [], 4: []}
        for r in range(rounds):
            for v in (0, 4):
                set_v(v)
                t[v].append(_time(outs[v][2]))
        set_v(0)
        m0, m4 = statistics.median(t[0]), statistics.median(t[4])
        print(f"  ring (0):      median {m0:7.1f} us ({fl / m0 / 1e6:6.1f} TF = {fl / m0 / 1e6 / 2500:.3f})")
        print(f"  ping-pong (4): median {m4:7.1f} us ({fl / m4 / 1e6:6.1f} TF = {fl / m4 / 1e6 / 2500:.3f})  "
              f"({(m4 / m0 - 1) * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
