import os, sys, torch
sys.path.insert(0, os.getcwd())
from replicatinggpt_amd import _lib as L, ops
from tools.attn_bench import _time
dev = torch.device("cuda"); L.load()
M, C, p = 65536, 768, 0.2
call = torch.zeros(1, dtype=torch.int64, device=dev)
x = torch.randn(M, C, device=dev)
w = torch.randn(C, device=dev)
dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
dres, dx = torch.randn(M, C, device=dev), torch.empty(M, C, device=dev)
lp = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
dw, db, cs = (torch.empty(C, device=dev) for _ in range(3))
ws = torch.empty(ops.layernorm_bwd_workspace(M, C) // 4 + 1, device=dev)
for name, mean, rstd in (("empty", torch.empty(M, device=dev), torch.empty(M, device=dev)),
                         ("real", x.mean(1), 1 / x.std(1)),
                         ("nan", torch.full((M,), float("nan"), device=dev), torch.full((M,), float("nan"), device=dev)),
                         ("denorm", torch.zeros(M, device=dev), torch.full((M,), 1e-39, device=dev))):
    t = _time(lambda: ops.layernorm_bwd(dy, x, w, mean, rstd, dres, dx, lp, dw, db, False, ws, cs, False, p, 1, call, 3))
    print(name, f"{t:.1f} us", flush=True)
