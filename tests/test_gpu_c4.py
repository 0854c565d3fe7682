"""C4-shape parity on the MI355X (BASELINE configs[3]: 12L / 12H / 768d, block 1024).

The reference's attention width is set by block_size (GPT1.py:13,106,114-116); at T = 1024 the
bf16 MFMA kernels run 16 query blocks per (b, h) through the XCD-remapped grid, the keep-bit buffer
is ~50 MB per layer at B = 64, and cg_gemm dispatches the forward / dgrad products to the 8-wave
256x256 kernel and the weight gradients to the 128x128 kernel with split-K.  Each is checked here
at the C4 geometry against an fp64 reference (attention: with the oracle's Philox keep mask), and a
2-layer C4-width model against the CPU oracle (fp32) and against itself in bf16.
Tolerances: the north_star's -- fp32 1e-5 relative, bf16 2e-2 (conftest.bf16_close: per element, by
max and by norm)."""
import numpy as np
import pytest

import torch

from conftest import bf16_close

from oracle import gpt1_oracle as O
from oracle import philox

pytestmark = pytest.mark.gpu
DEV = "cuda"
T4, H4, D4, C4 = 1024, 12, 64, 768


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def relerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _attn_ref(q, k, v, scale, p, seed, stream):
    """q, k, v [B, T, H, D] float64 (CPU): masked softmax attention with the oracle keep mask."""
    B, T, H, D = q.shape
    s = torch.einsum("bthd,bshd->bhts", q, k) * scale
    s = s.masked_fill(~torch.tril(torch.ones(T, T, dtype=torch.bool)), float("-inf"))
    P = torch.softmax(s, dim=-1)
    if p > 0:
        idx = np.arange(B * H * T * T, dtype=np.uint64).reshape(B, H, T, T)
        keep = torch.from_numpy(philox.keep_mask(seed, stream, idx, p))
        P = P * keep.double() * float(np.float32(1 / (1 - p)))
    return torch.einsum("bhts,bshd->bthd", P, v)


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_c4_attention_fwd_bwd_vs_fp64(p):
    """bf16 attention_fwd / attention_bwd at T=1024, H=12, D=64 (the C4 head geometry), B=1,
    scale n_embd^-0.5, against fp64 with the identical Philox keep mask."""
    from replicatinggpt_amd import functional as Fn
    torch.manual_seed(41)
    B, d = 1, H4 * D4
    qkv = (torch.randn(B * T4, 3 * d) * 0.8).to(torch.bfloat16)
    q = qkv[:, :d].double().view(B, T4, H4, D4).requires_grad_(True)
    k = qkv[:, d:2 * d].double().view(B, T4, H4, D4).requires_grad_(True)
    v = qkv[:, 2 * d:].double().view(B, T4, H4, D4).requires_grad_(True)
    scale = C4 ** -0.5
    call = torch.tensor([3], dtype=torch.int64, device=DEV)
    site = 4
    ref = _attn_ref(q, k, v, scale, p, 77, (3 << 8) | site)
    dout = torch.randn(B, T4, H4, D4).to(torch.bfloat16)
    ref.backward(dout.double())
    qd = qkv.to(DEV)
    o = torch.empty(B * T4, d, dtype=torch.bfloat16, device=DEV)
    lse, mask = Fn.attention_fwd(qd, B, T4, H4, D4, o, scale, p, 77, call, site)
    assert (mask is not None) == (p > 0)
    dqkv = Fn.attention_bwd(qd, B, T4, H4, D4, o, dout.reshape(B * T4, d).to(DEV), lse, scale, p, 77, call, site,
                            mask)
    torch.cuda.synchronize()
    assert relerr(o, ref.reshape(B * T4, d)) < 2e-2
    for i, t in enumerate((q, k, v)):
        ok, st = bf16_close(dqkv[:, i * d:(i + 1) * d], t.grad.reshape(B * T4, d))
        assert ok, ("qkv"[i], st)
    ok, st = bf16_close(o, ref.reshape(B * T4, d))
    assert ok, ("o", st)
    # logsumexp (fp32, per (b, h, t)) of the unmasked-row softmax
    s = torch.einsum("bthd,bshd->bhts", q.detach(), k.detach()) * scale
    s = s.masked_fill(~torch.tril(torch.ones(T4, T4, dtype=torch.bool)), float("-inf"))
    # the bf16 kernels' row sums run on the matrix core over the bf16-rounded weights O is built from
    # (each within 2^-8 relative), so |lse - ref| <= ln(1 + 2^-8) < 2^-8 per row
    assert float((lse.double().cpu() - torch.logsumexp(s, -1).double().cpu()).abs().max()) < 2.0 ** -8


def _decode_keep_bits(mask, BH, T):
    """Keep-bit buffer of the MFMA kernels (attention_common.h) -> two bool arrays [BH, T, T]
    (FWD and BWD tiles decoded), blocks outside the stored tiles False."""
    NB, NP = T // 32, T // 64
    ntile = NB + (NB - 1) ** 2 // 4
    words = mask.cpu().numpy().view(np.uint32).reshape(2, BH, ntile, 64)
    lanes = np.arange(64)
    r = np.arange(16)
    accrow = (r[:, None] & 3) + 8 * (r[:, None] >> 2) + 4 * (lanes[None, :] >> 5)     # [16, 64]
    col = np.broadcast_to(lanes[None, :] & 31, (16, 64))
    out = np.zeros((2, BH, T, T), dtype=bool)

    def bits(w, s, fwd):   # [BH, 64] words -> [BH, 16, 64]: FWD bit 8 s + (r >> 1) + 16 (r & 1), BWD 16 s + r
        sh = ((8 * s + (r >> 1) + 16 * (r & 1)) if fwd else (16 * s + r)).astype(np.uint32)
        return ((w[:, None, :] >> sh[None, :, None]) & np.uint32(1)).astype(bool)

    for qb in range(NB):
        for kt in range(qb // 2 + 1):
            t = qb + (qb - 1) ** 2 // 4 + kt if qb else kt
            for s in range(2):
                out[0][:, 32 * qb + col, 64 * kt + 32 * s + accrow] = bits(words[0, :, t], s, True)
    for kb in range(NB):
        for qt in range(kb // 2, NP):
            t = kb * NP - ((kb - 1) ** 2 // 4 if kb else 0) + qt - kb // 2
            for s in range(2):
                out[1][:, 64 * qt + 32 * s + accrow, 32 * kb + col] = bits(words[1, :, t], s, False)
    return out


@pytest.mark.parametrize("p", [0.2, 0.6])
def test_c4_dropmask_bits_match_oracle(p):
    """cg_attn_dropmask at T=1024 (272 FWD and 272 BWD 64-row tiles per (b, h)): every keep bit of the
    MFMA kernels' layouts equals the oracle's keep(((b H + h) T + q) T + key).  p = 0.6 takes the
    kernel's other decision form (threshold above 2^15: saturating subtract)."""
    from replicatinggpt_amd import ops
    B, H, T, seed, site = 1, 2, T4, 0x5EED, 6
    call = torch.tensor([11], dtype=torch.int64, device=DEV)
    n = ops.attn_mask_bytes(B, H, T) // 8
    mask = torch.zeros(n, dtype=torch.int64, device=DEV)
    ops.attn_dropmask(B, H, T, p, seed, call, site, mask)
    torch.cuda.synchronize()
    got = _decode_keep_bits(mask, B * H, T)
    keep = philox.keep_mask(seed, (11 << 8) | site, np.arange(B * H * T * T, dtype=np.uint64), p).reshape(B * H, T, T)
    # every element of the blocks on or below the diagonal (diagonal blocks whole: the kernels apply
    # the causal mask themselves), nothing above
    tri = np.kron(np.tril(np.ones((T // 32, T // 32), dtype=bool)), np.ones((32, 32), dtype=bool))
    assert np.array_equal(got[0], keep & tri)
    assert np.array_equal(got[1], keep & tri)
    # the measured keep rate of the 16-bit decision (p = 0.2 -> 13107 / 65536 dropped)
    assert abs(float(keep.mean()) - (1 - round(p * 65536) / 65536)) < 2e-3


def _c4_gemm_cases():
    from bench import census_shapes
    from replicatinggpt_amd import PRESETS
    return census_shapes(PRESETS["c4"], 64, T4)


@pytest.mark.parametrize("case", range(12))
def test_c4_gemm_dispatch_vs_fp64(case):
    """Every bf16 GEMM shape of one C4 training step (M = B T = 65536 tokens) through the model's own
    dispatch -- functional.linear_fwd / linear_dgrad (the 8-wave 256x256 kernel at >= 2 tiles per
    CU) and linear_wgrad (128x128 persistent kernel, deterministic split-K 16 / 4 / 8) -- against an
    fp64 product of the same bf16 operands (fp32 accumulation: 1e-5 relative for fp32 outputs)."""
    from replicatinggpt_amd import functional as Fn
    name, M, N, K, at, bt, kind, _ = _c4_gemm_cases()[case]
    torch.manual_seed(100 + case)
    if kind == "wgrad":
        # out[N_, K_] = dy[M_, N_]^T x[M_, K_]: census (M, N, K) = (N_, K_, tokens)
        dy = (torch.randn(K, M, device=DEV) * 0.5).to(torch.bfloat16)
        x = (torch.randn(K, N, device=DEV) * 0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device=DEV)
        Fn.linear_wgrad(dy, x, out, 0.0)
        ref = dy.double().t() @ x.double()
        split = Fn._wgrad_split(M, N, K, True)
        assert split > 1
        assert relerr(out, ref) < 1e-5, (name, split)
        return
    A = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16) if not bt else \
        (torch.randn(K, N, device=DEV) * 0.05).to(torch.bfloat16)
    ref = A.double() @ (W.double().t() if not bt else W.double())
    out = torch.empty(M, N, device=DEV)
    if not bt:
        Fn.linear_fwd(A, W, out)
    else:
        Fn.linear_dgrad(A, W, out)
    assert relerr(out, ref) < 1e-5, name
    if name == "ffn1_fwd":   # the model's bias + ReLU epilogue, bf16 out
        bias = torch.randn(N, device=DEV)
        h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        Fn.linear_fwd(A, W, h, "bias_relu", bias=bias)
        assert relerr(h, torch.relu(ref + bias.double())) < 8e-3
    if name == "ffn2_fwd":   # bias + Philox dropout + residual (fp32 out) against the oracle mask
        bias, resid = torch.randn(N, device=DEV), torch.randn(M, N, device=DEV)
        call = torch.tensor([2], dtype=torch.int64, device=DEV)
        o = torch.empty(M, N, device=DEV)
        Fn.linear_fwd(A, W, o, "bias_drop_resid", bias=bias, resid=resid, dropout_p=0.2, seed=9, rng_call=call,
                      site=3)
        for r0 in (0, M // 2 + 64, M - 1024):   # 1024-row bands (the oracle mask over all 50 M elements is slow)
            rows = slice(r0, r0 + 1024)
            idx = np.arange(r0 * N, (r0 + 1024) * N, dtype=np.uint64)
            keep = torch.from_numpy(philox.keep_mask(9, (2 << 8) | 3, idx, 0.2).reshape(1024, N)).double()
            want = resid[rows].double().cpu() + keep * (ref[rows].cpu() + bias.double().cpu()) * 1.25
            assert relerr(o[rows], want) < 1e-5, r0
    if name == "ffn2_dgrad":  # ReLU-backward epilogue against the ReLU output
        h = torch.relu(torch.randn(M, N, device=DEV)).to(torch.bfloat16)
        g = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        Fn.linear_dgrad(A, W, g, "relu_bwd", aux=h)
        assert relerr(g, ref * (h.double() > 0)) < 8e-3


def _model(dtype, layers=2):
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    cfg = GPTConfig(block_size=T4, n_embd=C4, n_head=H4, n_layers=layers, dropout=0.0, dtype=dtype)
    torch.manual_seed(1337)
    return BigramLanguageModel(cfg).to(DEV), cfg


def test_c4_width_model_fp32_matches_oracle():
    """2-layer model at the C4 width and context (d=768, H=12, hs=64, T=1024), fp32 HIP path: loss
    and every parameter gradient against the CPU oracle from the same seeded init."""
    m, cfg = _model("fp32")
    ocfg = O.OracleConfig(block_size=T4, n_embd=C4, n_head=H4, n_layers=2, dropout=0.0)
    torch.manual_seed(1337)
    P = O.init_params(ocfg)
    g = torch.Generator().manual_seed(8)
    idx = torch.randint(0, 65, (1, T4), generator=g)
    tgt = torch.randint(0, 65, (1, T4), generator=g)
    _, loss = m(idx.to(DEV), tgt.to(DEV))
    loss.backward()
    _, rl, rg = O.loss_and_grads(P, idx, tgt, ocfg)
    assert abs(float(loss) - float(rl)) < 1e-5 * max(1.0, float(rl))
    for name, prm in m.named_parameters():
        assert relerr(prm.grad, rg[name]) < 1e-4, name


def test_c4_width_model_bf16_close_to_fp32():
    """The same model on the bf16 path (the C4 bench path: 256x256 GEMMs, MFMA attention at T=1024)
    against the fp32 path: loss within 1 %, gradients within 5 % by norm (bf16 rounding flips a few
    ReLU / mask-adjacent terms, so per-element agreement is not the bar)."""
    m32, _ = _model("fp32")
    m16, _ = _model("bf16")
    g = torch.Generator().manual_seed(9)
    idx = torch.randint(0, 65, (2, T4), generator=g).to(DEV)
    tgt = torch.randint(0, 65, (2, T4), generator=g).to(DEV)
    _, l32 = m32(idx, tgt)
    l32.backward()
    _, l16 = m16(idx, tgt)
    l16.backward()
    assert abs(float(l16) - float(l32)) < 1e-2 * float(l32)
    g32 = dict(m32.named_parameters())
    for n, p in m16.named_parameters():
        a, b = p.grad.double(), g32[n].grad.double()
        assert float((a - b).norm() / b.norm()) < 5e-2, n
        assert float(torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0)) > 0.998, n
