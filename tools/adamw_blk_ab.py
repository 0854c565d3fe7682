"""C4 AdamW (86 M params, 30 B/param = 2.58 GB) against the HBM streaming ceiling
the same box shows.  Interleaved rounds (same process) of the grid-stride modes (adamw_mode 1 plain,
2 NT x2 = the C4 default, 3 plain x2) and the block-contiguous modes (6 NT x2, 7 plain x2, 8 NT x4,
9 plain x1; adamw_blocks = 4/8/16 per CU), each 20 launches replayed from a hipGraph on the step's
long-lived buffers (bench._time_ms, warm 20), every mode bitwise against mode 1; and a float4 copy of
the same 2.58 GB (read 16 B + write 14 B per param, as AdamW) for the box's ceiling.
The block-contiguous modes were measured slower (profiles/r6_adamw_ceiling_c4.txt) and removed from the
library; this script needs the commit that had them (git log -S k_adamw_blk).
usage: python tools/adamw_blk_ab.py [c4|c2]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import _time_ms  # noqa: E402
from replicatinggpt_amd import _lib, ops  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    n = 85997568 if cfg == "c4" else 10788992
    dev = torch.device("cuda:0")
    lib = _lib.load()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    gen = torch.Generator(device=dev).manual_seed(0)
    base = [torch.randn(n, device=dev, generator=gen) * 0.01 for _ in range(4)]
    base[3].abs_()
    p, g, m, v = (t.clone() for t in base)
    p16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    step = torch.full((1,), 3, dtype=torch.int64, device=dev)
    variants = [(1, 0), (2, 0), (3, 0), (6, 4 * cus), (6, 8 * cus), (6, 16 * cus), (7, 4 * cus), (7, 8 * cus),
                (8, 4 * cus), (9, 8 * cus)]
    ref = None
    for mode, nb in variants:   # bitwise: one update from the same state
        _lib.check(lib.cg_set_tuning(b"adamw_mode", mode))
        _lib.check(lib.cg_set_tuning(b"adamw_blocks", nb))
        q = [t.clone() for t in base]
        q16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
        ops.adamw(q[0], q[1], q[2], q[3], q16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
        torch.cuda.synchronize()
        out = (q[0], q[2], q[3], q16)
        if ref is None:
            ref = out
        eq = all(torch.equal(a, b) for a, b in zip(out, ref))
        print(f"mode {mode} blocks {nb}: bitwise vs mode 1 {'equal' if eq else 'DIFFERENT'}", flush=True)
        del q, q16
    src = torch.empty(n * 16 // 4, dtype=torch.float32, device=dev)
    dst = torch.empty(n * 14 // 4, dtype=torch.float32, device=dev)
    res = {}
    for r in range(3):
        for mode, nb in variants:
            _lib.check(lib.cg_set_tuning(b"adamw_mode", mode))
            _lib.check(lib.cg_set_tuning(b"adamw_blocks", nb))
            t = _time_ms(lambda: ops.adamw(p, g, m, v, p16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step), warm=20)
            res.setdefault((mode, nb), []).append(t)
        t = _time_ms(lambda: dst.copy_(src[:dst.numel()]), warm=5)
        res.setdefault(("copy 14/16", 0), []).append(t)
    _lib.check(lib.cg_set_tuning(b"adamw_mode", 0))
    _lib.check(lib.cg_set_tuning(b"adamw_blocks", 0))
    for k, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        byts = 30 * n if k[0] != "copy 14/16" else 28 * n
        print(f"{str(k[0]):>10s} blocks {k[1]:5d}: {t * 1e3:8.1f} us  {byts / (t * 1e-3) / 1e9:7.1f} GB/s  "
              f"(runs {', '.join(f'{x * 1e3:.1f}' for x in ts)})", flush=True)


if __name__ == "__main__":
    main()
