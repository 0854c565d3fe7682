"""Probe (GPU): time the as-is generate() path at C5 (256 sequences) for a few steps at short and
full-window lengths, and one fp32 forward at [256, 256] in the C1 shape."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from safetensors.torch import load_file
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    sd = load_file(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "model_c1_trained.safetensors"))
    m = BigramLanguageModel(GPTConfig(dtype="fp32"))
    m.load_state_dict(sd, strict=False)
    m = m.to("cuda").eval()
    for L in (1, 64, 256):
        idx = torch.randint(0, 65, (256, L), device="cuda")
        with torch.no_grad():
            for _ in range(2):
                m(idx)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                m(idx)
            torch.cuda.synchronize()
        print(f"fp32 forward [256,{L}]: {(time.perf_counter()-t0)/5*1e3:.2f} ms", flush=True)
    m16 = BigramLanguageModel(GPTConfig(dtype="bf16"))
    m16.load_state_dict(sd, strict=False)
    m16 = m16.to("cuda").eval()
    idx = torch.randint(0, 65, (256, 256), device="cuda")
    with torch.no_grad():
        for _ in range(2):
            m16(idx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            m16(idx)
        torch.cuda.synchronize()
    print(f"bf16 forward [256,256]: {(time.perf_counter()-t0)/5*1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
