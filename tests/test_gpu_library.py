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
