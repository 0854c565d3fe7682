"""One C5 generate() (256 sequences x 500 new tokens, greedy, fp32, reference-trained C1 weights) after a
capture/warm-up call -- the command under rocprofv3 --kernel-trace for the decode kernel census.
GPU only."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from safetensors.torch import load_file
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    sd = load_file(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                                "model_c1_trained.safetensors"))
    m = BigramLanguageModel(GPTConfig(dtype="fp32"))
    m.load_state_dict(sd, strict=False)
    m = m.to("cuda").eval()
    idx = torch.zeros((256, 1), dtype=torch.long, device="cuda")
    with torch.no_grad():
        m.generate(idx, 500, greedy=True, generator=torch.Generator().manual_seed(1337))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = m.generate(idx, 500, greedy=True, generator=torch.Generator().manual_seed(1337))
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"generate 256x500: {dt * 1e3:.1f} ms = {256 * 500 / dt:.0f} tok/s, checksum {int(out.sum())}", flush=True)


if __name__ == "__main__":
    main()
