"""The torch.library seam: every charpt:: op has a fake (meta) implementation, and the
functional ops -- charpt::layer_norm, charpt::linear, charpt::causal_attention (nn.LayerNorm,
nn.Linear and the all-heads Head.forward of GPT1.py:100-136) -- carry register_autograd formulas
whose backward is itself one custom op.  torch.library.opcheck runs each through schema, FakeTensor,
autograd-registration and AOT-dispatch (static and dynamic shapes) checks on the MI355X, and the
values are checked against fp64 torch."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def relerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _ops():
    from replicatinggpt_amd import ops
    return ops


def test_every_op_has_a_fake():
    from torch._library.custom_ops import CustomOpDef
    O = _ops()
    defs = [v for v in vars(O).values() if isinstance(v, CustomOpDef)]
    assert len(defs) >= 30
    for d in defs:
        assert d._abstract_fn is not None, d._name


def test_opcheck_out_style_ops():
    """Mutating (out-style) kernels: schema (declared mutations), fake and AOT-dispatch checks."""
    O = _ops()
    x = torch.randn(64, 384, device=DEV)
    w, b = torch.randn(384, device=DEV), torch.randn(384, device=DEV)
    y = torch.empty(64, 384, dtype=torch.bfloat16, device=DEV)
    mean, rstd = torch.empty(64, device=DEV), torch.empty(64, device=DEV)
    torch.library.opcheck(O.layernorm_fwd, (x, w, b, y, mean, rstd, 1e-5))
    A = torch.randn(128, 256, device=DEV).to(torch.bfloat16)
    Bm = torch.randn(128, 256, device=DEV).to(torch.bfloat16)
    out = torch.empty(128, 128, device=DEV)
    torch.library.opcheck(O.gemm, (A, Bm, out, True, False, False, 128, 128, 256, 256, 256, 128, 0, None, None, 0,
                                   None, 0, 0.0, 0, None, 0, 0.0, 1, None))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("bias", [True, False])
def test_opcheck_linear(dt, bias):
    O = _ops()
    torch.manual_seed(0)
    x = torch.randn(4, 32, 128, device=DEV).to(dt).requires_grad_(True)
    w = (torch.randn(256, 128, device=DEV) * 0.1).to(dt).requires_grad_(True)
    bb = torch.randn(256, device=DEV).requires_grad_(True) if bias else None
    torch.library.opcheck(O.linear, (x, w, bb))
    y = O.linear(x, w, bb)
    ref_x, ref_w = x.detach().double().requires_grad_(True), w.detach().double().requires_grad_(True)
    ref_b = bb.detach().double().requires_grad_(True) if bias else None
    ref = torch.nn.functional.linear(ref_x, ref_w, ref_b)
    g = torch.randn_like(ref)
    y.backward(g.to(y.dtype))
    ref.backward(g.to(y.dtype).double())
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert relerr(y, ref) < tol
    assert relerr(x.grad, ref_x.grad) < tol
    assert relerr(w.grad, ref_w.grad) < tol
    if bias:
        assert relerr(bb.grad, ref_b.grad) < 1e-5


def test_opcheck_layer_norm():
    O = _ops()
    torch.manual_seed(1)
    x = (torch.randn(3, 40, 384, device=DEV) * 2 + 0.5).requires_grad_(True)
    w = (torch.randn(384, device=DEV) * 0.1 + 1).requires_grad_(True)
    b = (torch.randn(384, device=DEV) * 0.1).requires_grad_(True)
    torch.library.opcheck(O.layer_norm, (x, w, b, 1e-5))
    y, _, _ = O.layer_norm(x, w, b, 1e-5)
    xr, wr, br = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    ref = torch.nn.functional.layer_norm(xr, (384,), wr, br, 1e-5)
    g = torch.randn_like(ref)
    y.backward(g.float())
    ref.backward(g)
    assert relerr(y, ref) < 1e-5
    for a, r in ((x, xr), (w, wr), (b, br)):
        assert relerr(a.grad, r.grad) < 1e-5


@pytest.mark.parametrize("dt,T,H,D", [(torch.bfloat16, 128, 2, 64), (torch.float32, 37, 3, 21)])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_opcheck_causal_attention(dt, T, H, D, p):
    from oracle import philox
    import numpy as np
    O = _ops()
    torch.manual_seed(2)
    B, d = 2, H * D
    qkv = (torch.randn(B, T, 3 * d, device=DEV) * 0.7).to(dt).requires_grad_(True)
    call = torch.tensor([7], dtype=torch.int64, device=DEV)
    scale = (3.0 * D) ** -0.5
    args = (qkv, H, D, scale, p, 13, call, 2)
    torch.library.opcheck(O.causal_attention, args)
    o, lse = O.causal_attention(*args)
    q = qkv.detach().double()[..., :d].view(B, T, H, D).requires_grad_(True)
    k = qkv.detach().double()[..., d:2 * d].view(B, T, H, D).requires_grad_(True)
    v = qkv.detach().double()[..., 2 * d:].view(B, T, H, D).requires_grad_(True)
    s = torch.einsum("bthd,bshd->bhts", q, k) * scale
    s = s.masked_fill(~torch.tril(torch.ones(T, T, dtype=torch.bool, device=DEV)), float("-inf"))
    P = torch.softmax(s, -1)
    if p > 0:
        keep = philox.keep_mask(13, (7 << 8) | 2, np.arange(B * H * T * T, dtype=np.uint64), p)
        P = P * torch.from_numpy(keep.reshape(B, H, T, T)).to(DEV).double() * float(np.float32(1 / (1 - p)))
    ref = torch.einsum("bhts,bshd->bthd", P, v).reshape(B, T, d)
    g = torch.randn_like(ref)
    o.backward(g.to(o.dtype))
    ref.backward(g.to(o.dtype).double())
    tol, gtol = (1e-5, 1e-5) if dt == torch.float32 else (2e-2, 2e-2)
    assert relerr(o, ref) < tol
    want = torch.cat([t.grad.reshape(B, T, d) for t in (q, k, v)], -1)
    assert relerr(qkv.grad, want) < gtol


def test_linear_backward_inside_defer_matches_eager():
    """inside functional.DEFER the split-K reduce of a weight gradient may stay
    pending past linear_wgrad only when its output is a flat gradient slot.  charpt::linear's
    backward writes a temporary it reads right away (to_act / autograd), so its reduce must be
    complete when linear_wgrad returns: the same bits with DEFER on and off, at a shape whose
    weight gradient takes split-K (K = 4096 tokens), followed by another GEMM that would pick up a
    still-pending reduce in its tail."""
    from replicatinggpt_amd import functional as Fn
    O = _ops()
    torch.manual_seed(3)
    x = torch.randn(4096, 256, device=DEV).to(torch.bfloat16)
    w = (torch.randn(384, 256, device=DEV) * 0.1).to(torch.bfloat16)
    dy = torch.randn(4096, 384, device=DEV).to(torch.bfloat16)
    assert Fn._wgrad_split(384, 256, 4096, True) > 1
    ref = O.linear_backward(dy, x, w, True)
    torch.cuda.synchronize()
    with Fn.DEFER:
        got = O.linear_backward(dy, x, w, True)
        dw_now = got[1].clone()       # read before DEFER closes
        O.linear_backward(dy, x, w, False)   # a later persistent GEMM on the same stream
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    assert torch.equal(dw_now, ref[1])


def test_wgrad_into_temporary_inside_defer_is_complete():
    """linear_wgrad into a non-slot fp32 target inside DEFER (the HeadLossFn non-slot fallback's
    form): the output is complete on return, bitwise the eager result."""
    from replicatinggpt_amd import functional as Fn
    torch.manual_seed(4)
    dy = torch.randn(8192, 128, device=DEV).to(torch.bfloat16)
    a = torch.randn(8192, 384, device=DEV).to(torch.bfloat16)
    ref = torch.empty(128, 384, device=DEV)
    Fn.linear_wgrad(dy, a, ref, 0.0)
    tmp = torch.full((128, 384), float("nan"), device=DEV)
    with Fn.DEFER:
        Fn.linear_wgrad(dy, a, tmp, 0.0)
        snap = tmp.clone()
    torch.cuda.synchronize()
    assert torch.equal(snap, ref)


def _deferred_workload(seed):
    """One stream's share of a training backward's deferred work (include/charpt.h "deferred work"):
    a split-K weight gradient with bf16 slabs and a deferred reduce, a queued column-sum reduce, an
    AdamW update of that gradient queued for a GEMM's free blocks, a part-filling persistent GEMM
    (out[16384, 384] = a b^T: 384 128x128 items on 512 slots, like the N = 384 dgrads) that takes the
    pending jobs, and the stream's flush.  Operand extents: a [16384, 1152], b [384, 1152] (NT)."""
    from replicatinggpt_amd import _lib as L
    g = torch.Generator(device=DEV).manual_seed(seed)
    M, N, K = 384, 1536, 16384
    t = {"dy": torch.randn(K, M, device=DEV, generator=g).to(torch.bfloat16),
         "x": torch.randn(K, N, device=DEV, generator=g).to(torch.bfloat16),
         "part": torch.randn(256, 1152, device=DEV, generator=g),
         "a": torch.randn(16384, 1152, device=DEV, generator=g).to(torch.bfloat16),
         "b": torch.randn(384, 1152, device=DEV, generator=g).to(torch.bfloat16),
         "p": torch.randn(M * N, device=DEV, generator=g) * 0.02}
    t["ws"] = torch.empty(_ops().gemm_workspace(M, N, 14) // 4, device=DEV)
    t["gw"] = torch.empty(M, N, device=DEV)
    t["gb"] = torch.zeros(1152, device=DEV)
    t["m"], t["v"] = torch.zeros_like(t["p"]), torch.zeros_like(t["p"])
    t["pb"] = torch.empty(M * N, dtype=torch.bfloat16, device=DEV)
    t["out"] = torch.empty(16384, 384, dtype=torch.bfloat16, device=DEV)
    t["step"] = torch.ones(1, dtype=torch.int64, device=DEV)
    flags = L.GEMM_SLAB_BF16 | L.GEMM_DEFER_REDUCE
    return t, flags


def _run_deferred(t, flags, sync=None):
    import ctypes
    from replicatinggpt_amd import _lib as L
    O = _ops()
    step = sync or (lambda: None)
    M, N, K = 384, 1536, 16384
    step()
    O.gemm(t["dy"], t["x"], t["gw"], True, True, True, M, N, K, M, N, N, 0, None, None, 0, None, 0, 0.0, 0, None, 0,
           0.0, 14, t["ws"], flags)
    step()
    O.reduce_rows(t["part"], 256, 1152, t["gb"], False, True)
    step()
    O.adamw_defer(t["p"], t["gw"].view(-1), t["m"], t["v"], t["pb"], 1e-3, 0.9, 0.999, 1e-8, 0.01, t["step"])
    step()
    O.gemm(t["a"], t["b"], t["out"], True, False, False, 16384, 384, 1152, 1152, 1152, 384, 0, None, None, 0, None,
           0, 0.0, 0, None, 0, 0.0, 1, None)
    step()
    L.check(L.load().cg_flush_deferred(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))


def test_deferred_work_two_threads_two_streams_match_single_thread():
    """deferral is per call and its queues per stream, so two host threads, each
    driving its own stream with deferred split-K reduces, queued column sums and deferred AdamW
    jobs -- their library calls interleaved step by step through a barrier -- produce exactly the
    bits of the same two workloads run one after the other on one thread."""
    import threading
    ref = []
    for seed in (11, 12):
        t, flags = _deferred_workload(seed)
        _run_deferred(t, flags)
        torch.cuda.synchronize()
        ref.append({k: v.clone() for k, v in t.items()})
    work = [_deferred_workload(seed) for seed in (11, 12)]
    streams = [torch.cuda.Stream() for _ in work]
    torch.cuda.synchronize()
    bar = threading.Barrier(2)
    errs = []

    def body(i):
        try:
            torch.cuda.set_device(0)
            with torch.cuda.stream(streams[i]):
                _run_deferred(*work[i], sync=lambda: bar.wait(timeout=60))
        except BaseException as e:   # noqa: BLE001 -- reported below
            errs.append(e)
            bar.abort()

    th = [threading.Thread(target=body, args=(i,)) for i in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    torch.cuda.synchronize()
    assert not errs, errs
    for (t, _), r in zip(work, ref):
        for k in ("gw", "gb", "p", "m", "v", "pb", "out"):
            assert torch.equal(t[k], r[k]), k


def test_discard_deferred_reports_taken_adam_jobs():
    """cg_discard_deferred drops a stream's queue without launching it and reports how many
    deferred AdamW jobs launches had already taken (a failed backward: 0 = no parameter touched)."""
    import ctypes
    from replicatinggpt_amd import _lib as L
    O = _ops()
    t, flags = _deferred_workload(5)
    t["gw"].fill_(0.125)
    p0 = t["p"].clone()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = ctypes.c_int(-1)
    O.adamw_defer(t["p"], t["gw"].view(-1), t["m"], t["v"], t["pb"], 1e-3, 0.9, 0.999, 1e-8, 0.01, t["step"])
    L.check(L.load().cg_discard_deferred(st, ctypes.byref(n)))
    L.check(L.load().cg_flush_deferred(st))
    torch.cuda.synchronize()
    assert n.value == 0 and torch.equal(t["p"], p0)
    O.adamw_defer(t["p"], t["gw"].view(-1), t["m"], t["v"], t["pb"], 1e-3, 0.9, 0.999, 1e-8, 0.01, t["step"])
    O.gemm(t["a"], t["b"], t["out"], True, False, False, 16384, 384, 1152, 1152, 1152, 384, 0, None, None, 0, None,
           0, 0.0, 0, None, 0, 0.0, 1, None)   # 384 items on 512 slots: its free blocks take the job
    L.check(L.load().cg_discard_deferred(st, ctypes.byref(n)))
    torch.cuda.synchronize()
    assert n.value == 1 and not torch.equal(t["p"], p0)
