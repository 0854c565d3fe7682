import torch, sys
sys.path.insert(0, '/root/repo')
from replicatinggpt_amd import ops, _lib as L
torch.manual_seed(0)
dev = 'cuda'
n = 1 << 20
p = torch.randn(n, device=dev); g = torch.randn(n, device=dev) * 0.1
m = torch.randn(n, device=dev) * 0.01; v = torch.rand(n, device=dev) * 0.01
pb = torch.zeros(n, dtype=torch.bfloat16, device=dev)
step = torch.tensor([3], dtype=torch.int64, device=dev)
args = (1e-3, 0.9, 0.999, 1e-8, 0.01)
ref = [t.clone() for t in (p, m, v, pb)]
ops.adamw(ref[0], g, ref[1], ref[2], ref[3], *args, step)
# (b) deferred region + flush + segments
for mode in ('flush', 'gemm'):
    P, M_, V_, PB = p.clone(), m.clone(), v.clone(), pb.clone()
    a, b = 4096, 300000
    ops.adamw_defer(P[a:a + b], g[a:a + b], M_[a:a + b], V_[a:a + b], PB[a:a + b], *args, step)
    if mode == 'gemm':   # a part-filling persistent GEMM takes the job on its free blocks
        x = torch.randn(16384, 384, device=dev).to(torch.bfloat16)
        w = torch.randn(384, 384, device=dev).to(torch.bfloat16)
        y = torch.empty(16384, 384, dtype=torch.bfloat16, device=dev)
        y2 = torch.empty_like(y)
        ops.gemm(x, w, y, True, False, False, 16384, 384, 384, 384, 384, 384, 0, None, None, 0, None, 0, 0.0, 0, None, 0, 0.0, 1, None)
    L.check(L.load().cg_flush_deferred(L.ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    ops.adamw_segments(P, g, M_, V_, PB, [0, a, a + b, n - a - b], *args, step)
    torch.cuda.synchronize()
    print(mode, all(torch.equal(x, y) for x, y in zip((P, M_, V_, PB.view(torch.int16)), (ref[0], ref[1], ref[2], ref[3].view(torch.int16)))))
    if mode == 'gemm':
        ops.gemm(x, w, y2, True, False, False, 16384, 384, 384, 384, 384, 384, 0, None, None, 0, None, 0, 0.0, 0, None, 0, 0.0, 1, None)
        torch.cuda.synchronize()
        print('gemm output same with side adam', torch.equal(y.view(torch.int16), y2.view(torch.int16)))
