"""Per-workgroup timeline of the resident C2 attention kernels (diagnostic build, `make attnstamps`,
CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_attnstamps.so): for the forward (k_attn_fwd_d64r) and the
merged backward (k_attn_bwd_d64r: even workgroups dQ, odd dK/dV), each workgroup's start, the end of
its prologue (every operand load issued and the first tiles landed: the kernel's first wait) and its
end, from s_memrealtime (100 MHz), plus the CU it ran on (HW_ID, XCC_ID).  Prints per kind: the
prologue and compute durations, how many workgroups started only after another one ended (the
second round of a grid larger than the resident slots), and the kernel span.  GPU only.

usage: CHARPT_LIB=replicatinggpt_amd/libcharpt_hip_attnstamps.so python tools/attn_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L  # noqa: E402
from replicatinggpt_amd import functional as Fn, ops  # noqa: E402


def stamps(lib, n):
    buf = (ctypes.c_ulonglong * (4 * n))()
    if lib.cg_debug_attn_stamps(buf, n) != 0:
        raise SystemExit("cg_debug_attn_stamps failed (not the attnstamps build?)")
    return np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)


def report(name, st):
    t0 = st[:, 0].min()
    start, mid, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, (st[:, 2] - t0) / 100.0   # us
    kind = (st[:, 3] >> 48) & 0xff
    xcc = (st[:, 3] >> 40) & 0xff
    hw = st[:, 3] & 0xffffffff
    cu = (xcc << 16) | ((hw >> 8) & 0xff)   # XCC + HW_ID's CU [11:8], SH [12], SE [15:13] fields
    first_end = end.min()
    print(f"== {name}: {len(st)} workgroups on {len(np.unique(cu))} CUs, span {end.max():.2f} us "
          f"(first end {first_end:.2f} us)")
    for k in sorted(set(kind.tolist())):
        m = kind == k
        late = start[m] > first_end
        lab = {0: "dQ", 1: "dK/dV", 2: "fwd"}.get(int(k), str(k))
        pro, comp, tot = mid[m] - start[m], end[m] - mid[m], end[m] - start[m]
        print(f"  {lab:6s} n={m.sum():4d}  prologue {np.median(pro):6.2f} us (p90 {np.percentile(pro, 90):6.2f})  "
              f"compute {np.median(comp):6.2f} us (p90 {np.percentile(comp, 90):6.2f})  "
              f"total {np.median(tot):6.2f}  second-round starts {late.sum():4d}  "
              f"start p50/max {np.median(start[m]):6.2f}/{start[m].max():6.2f}  end p50/max "
              f"{np.median(end[m]):6.2f}/{end[m].max():6.2f}")
    per_cu = np.bincount(np.unique(cu, return_inverse=True)[1])
    print(f"  workgroups per CU: {np.bincount(per_cu).tolist()} (index = count)")


def main():
    lib = L.load()
    B, T, H, D, p = 64, 256, 6, 64, 0.2
    dev = torch.device("cuda")
    d = H * D
    torch.manual_seed(0)
    qkv = torch.randn(B * T, 3 * d, device=dev).to(torch.bfloat16)
    o = torch.empty(B * T, d, dtype=torch.bfloat16, device=dev)
    do = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = d ** -0.5
    for rep in range(3):   # warm; the last repetition is reported
        lse, mask = Fn.attention_fwd(qkv, B, T, H, D, o, scale, p, 1, call, 0)
        torch.cuda.synchronize()
        sf = stamps(lib, B * H)
        Fn.attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, 1, call, 0, mask)
        torch.cuda.synchronize()
        sb = stamps(lib, 2 * B * H)
    report("k_attn_fwd_d64r (C2)", sf)
    report("k_attn_bwd_d64r (C2)", sb)


if __name__ == "__main__":
    main()
