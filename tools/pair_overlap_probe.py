"""How much would one launch per backward (dgrad, wgrad) pair buy?  Both products of a Linear's
backward read the same dY and are independent (GPT1.py:111-112,136,143,145 backward).  Times, per
C2 pair: the dgrad alone, the wgrad alone (each 20 back-to-back launches from a hipGraph, census
epilogues), their sequential sum, and the two issued eagerly on two streams at once (20 pairs, the
hardware runs them concurrently on two queues) -- an upper bound on what co-scheduling the pair
in one launch could save.  GPU only.  usage: python tools/pair_overlap_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    from replicatinggpt_amd import PRESETS
    cfg = PRESETS["c2"]
    shapes = {s[0]: s for s in bench.census_shapes(cfg, cfg.batch_size, cfg.block_size)}
    pairs = [("proj_dgrad", "proj_wgrad"), ("qkv_dgrad", "qkv_wgrad"), ("ffn2_dgrad", "ffn2_wgrad"),
             ("ffn1_dgrad", "ffn1_wgrad")]
    reps = 20
    for a, b in pairs:
        ta = bench.time_gemm(*shapes[a][:7], dev)
        tb = bench.time_gemm(*shapes[b][:7], dev)
        ra, _ = bench.census_op(*shapes[a][:7], dev)
        rb, _ = bench.census_op(*shapes[b][:7], dev)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(3):
            ra(); rb()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s1.wait_stream(torch.cuda.current_stream())
            s2.wait_stream(torch.cuda.current_stream())
            for _ in range(reps):
                with torch.cuda.stream(s1):
                    ra()
                with torch.cuda.stream(s2):
                    rb()
            torch.cuda.current_stream().wait_stream(s1)
            torch.cuda.current_stream().wait_stream(s2)
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
        print(f"{a:11s} {ta * 1e3:6.1f} us  {b:11s} {tb * 1e3:6.1f} us  sequential {(ta + tb) * 1e3:6.1f} us  "
              f"two streams {best * 1e3:6.1f} us  ({best / (ta + tb):.2f}x)", flush=True)


if __name__ == "__main__":
    main()
