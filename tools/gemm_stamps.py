"""Where the persistent 128x128 GEMM's K-steps spend their cycles: loads the stamp-instrumented
diagnostic library (make -C replicatinggpt_amd/csrc stamps; gemm_pk.hip CG_PK_STAMPS) and prints,
per shape, the per-wave s_memtime cycles of each K-step's head wait (vmcnt + barrier) and of its
fragment reads + MFMA/DMA issue, the epilogue cycles per item and the clock the waves ran at --
every op of the training census with the step's fused epilogue (bench.census_op).
GPU only.  usage: python tools/gemm_stamps.py [c2|c4]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["CHARPT_LIB"] = os.path.join(ROOT, "replicatinggpt_amd", "libcharpt_hip_stamps.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import bench  # noqa: E402
from replicatinggpt_amd import PRESETS  # noqa: E402
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import functional as Fn  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    lib = L.load()
    lib.cg_debug_pk_stamps.argtypes = [ctypes.c_void_p]
    c = PRESETS[cfg]
    L.check(lib.cg_set_tuning(b"gemm_variant", 9))
    buf = (ctypes.c_ulonglong * 8)()
    for name, m, n, k, at, bt, kind, _ in bench.census_shapes(c, c.batch_size, c.block_size):
        split = Fn._wgrad_split(m, n, k, True) if kind == "wgrad" else 1
        fn, _ = bench.census_op(name, m, n, k, at, bt, kind, torch.device("cuda"))
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        lib.cg_debug_pk_stamps_reset()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        lib.cg_debug_pk_stamps(ctypes.addressof(buf))
        sw, sm, se, steps, wall, real, waves = list(buf)[:7]
        waves = max(waves, 1)
        items = m // 128 * (n // 128) * split
        clk = wall / max(real, 1) * 100.0   # MHz
        print(f"{cfg} {name:11s} {kind:16s} M={m:6d} N={n:5d} K={k:6d} split {split:2d}: {a.elapsed_time(b) * 1e3:7.1f} us | "
              f"per wave {wall / waves:8.0f} cyc @ {clk:5.0f} MHz, {steps / waves:5.1f} K-steps: "
              f"head wait {sw / steps:6.0f} cyc/step, reads+MFMA {sm / steps:6.0f} cyc/step, "
              f"epilogue {se / max(1, items * 4):6.0f} cyc/item-wave, other {(wall - sw - sm - se) / waves:7.0f} cyc/wave",
              flush=True)
    L.check(lib.cg_set_tuning(b"gemm_variant", 0))


if __name__ == "__main__":
    main()
