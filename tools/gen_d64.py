"""generate() at head size 64 (the keys-on-lanes decode attention holds 4 x 64 floats per
lane at D = 64 -- k_decode_attn<64> allocates 256 VGPRs, one wave per SIMD): the C2-shape model
(6L/6H/384d, block 256, random init, fp32 and bf16) decoding 64 sequences x 400 new tokens (256
K/V-cached steps, then the sliding window), greedy, after a capture / warm-up call; the decode
attention kernel's share from a rocprofv3 kernel trace of this command.  GPU only."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from replicatinggpt_amd import BigramLanguageModel, PRESETS
    for dt in ("fp32", "bf16"):
        torch.manual_seed(1337)
        m = BigramLanguageModel(PRESETS["c2"].with_(dtype=dt, dropout=0.0)).to("cuda").eval()
        idx = torch.zeros((64, 1), dtype=torch.long, device="cuda")
        with torch.no_grad():
            m.generate(idx, 400, greedy=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = m.generate(idx, 400, greedy=True)
            torch.cuda.synchronize()
        dt_s = time.perf_counter() - t0
        print(f"C2-shape {dt} generate 64x400 (D = 64): {dt_s * 1e3:.1f} ms = {64 * 400 / dt_s:.0f} tok/s, "
              f"checksum {int(out.sum())}", flush=True)


if __name__ == "__main__":
    main()
