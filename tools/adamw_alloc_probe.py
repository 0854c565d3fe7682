"""C4 AdamW census conditions: the same 30 B/param launch timed (bench._time_ms, warm 20) on buffers
allocated as bench.kernel_census does, three times in a row, then on a second allocation after the
first is freed, and with each mode -- to see whether the census figure depends on the allocation.
usage: python tools/adamw_alloc_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib, ops  # noqa: E402
from bench import _time_ms  # noqa: E402


def run(tag, n, dev, modes=(0,)):
    lib = _lib.load()
    pp, g, m, v = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
    v.abs_()
    p16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    step_t = torch.ones(1, dtype=torch.int64, device=dev)
    for mode in modes:
        _lib.check(lib.cg_set_tuning(b"adamw_mode", mode), "tuning")
        for rep in range(3):
            t = _time_ms(lambda: ops.adamw(pp, g, m, v, p16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step_t), warm=20)
            print(f"{tag} mode {mode} rep {rep}: {t * 1e3:7.1f} us  {30 * n / t / 1e6 / 8000:.3f} of 8 TB/s", flush=True)
    _lib.check(lib.cg_set_tuning(b"adamw_mode", 0), "tuning")


def main():
    dev = torch.device("cuda")
    n = 85914752
    junk = torch.empty(3 << 28, dtype=torch.uint8, device=dev)   # 768 MB of other allocations first, as in bench
    junk.fill_(1)
    run("first alloc", n, dev, modes=(0, 2, 4, 5))
    del junk
    torch.cuda.empty_cache()
    run("second alloc", n, dev, modes=(0, 4))


if __name__ == "__main__":
    main()
