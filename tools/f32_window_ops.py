"""The C5 window's fp32 launches one at a time (for counter passes): the fused FFN with ln2
(k_ffn_f32), ln1 + QKV and the projection + residual (the row linears, default 16-row form), and the
resident causal attention (k_attn_fwd_f32res), each replayed 20 times in a hipGraph, at generate()'s
window shape (256 sequences x T = 256, C = 126, H = 504, 6 heads of 21).  GPU only.
usage: python tools/f32_window_ops.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import ops  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from f32_fwd_ab import graph_us  # noqa: E402


def main():
    M, C, H = 65536, 126, 504
    dev = torch.device("cuda")
    torch.manual_seed(3)
    x = torch.randn(M, C, device=dev)
    lw, lb = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    w1, b1 = torch.randn(H, C, device=dev) / C ** 0.5, torch.randn(H, device=dev)
    w2, b2 = torch.randn(C, H, device=dev) / H ** 0.5, torch.randn(C, device=dev)
    wq = torch.randn(3 * C, C, device=dev) / C ** 0.5
    wp, bp = torch.randn(C, C, device=dev) / C ** 0.5, torch.randn(C, device=dev)
    out = torch.empty(M, C, device=dev)
    qkv = torch.empty(M, 3 * C, device=dev)
    from replicatinggpt_amd import functional as Fn
    Bq, T, NH, D = 256, 256, 6, 21
    att = torch.empty(M, C, device=dev)
    runs = {
        "ffn_ln": lambda: ops.ffn_fwd_f32(x, lw, lb, 1e-5, w1, b1, w2, b2, x, out),
        "ln_qkv": lambda: ops.linear_rows_f32(x, lw, lb, 1e-5, wq, None, None, qkv),
        "proj_resid": lambda: ops.linear_rows_f32(x, None, None, 0.0, wp, bp, x, out),
        "attn_res": lambda: Fn.attention_fwd(qkv, Bq, T, NH, D, att, D ** -0.5, 0.0, 0, None, 0),
    }
    for name, run in runs.items():
        print(f"{name:10s} {graph_us(run):8.1f} us", flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
