"""AdamW kernel variants (cg_set_tuning adamw_mode 0..3) at the C2 and C4 parameter counts: HBM
GB/s for the 30 B/param pass (20 launches replayed from a hipGraph, as bench.py's census) and a
bitwise check of every variant against mode 0.  usage: python tools/adamw_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib, ops  # noqa: E402
from bench import _time_ms  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lib = _lib.load()
    for name, n in (("c2", 10788992), ("c4", 85997568)):
        gen = torch.Generator(device=dev).manual_seed(0)
        base = [torch.randn(n, device=dev, generator=gen) * 0.01 for _ in range(4)]
        base[3].abs_()
        step = torch.full((1,), 3, dtype=torch.int64, device=dev)
        ref = None
        for mode in ((0, 2, 3, 4, 5, 0, 2, 3, 4, 5) if name == "c4" else (0, 1, 3, 5, 0, 1, 3, 5)):
            _lib.check(lib.cg_set_tuning(b"adamw_mode", mode), "tuning")
            p, g, m, v = (t.clone() for t in base)
            p16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
            ops.adamw(p, g, m, v, p16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
            out = (p.clone(), m.clone(), v.clone(), p16.clone())
            if ref is None:
                ref = out
            same = all(torch.equal(a, b) for a, b in zip(out, ref))
            t = _time_ms(lambda: ops.adamw(p, g, m, v, p16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step))
            print(f"{name} n={n} mode {mode}: {t * 1e3:8.1f} us  {30 * n / t / 1e6:7.1f} GB/s  "
                  f"({30 * n / t / 1e6 / 8000:.3f} of 8 TB/s)  bitwise={same}", flush=True)
        del base, p, g, m, v, p16, ref, out
        torch.cuda.empty_cache()
    _lib.check(lib.cg_set_tuning(b"adamw_mode", 0), "tuning")


if __name__ == "__main__":
    main()
