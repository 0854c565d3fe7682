"""torch.library custom ops over the charpt C ABI (include/charpt.h).

Each op is a thin, out-style wrapper: the caller (replicatinggpt_amd.functional) allocates every
output/workspace through PyTorch's caching allocator, and the op launches the HIP kernel on the
current stream (so whole training steps are capturable into a hipGraph).  Ops are registered for
the "cuda" (= HIP on ROCm) device only: calling them on CPU tensors raises -- the product has no
CPU fallback.
"""
from typing import List, Optional

import torch
from torch import Tensor

from . import _lib as L

_NS = "charpt"


def _s(t):
    return L.stream_ptr(t.device)


def _op(name, mutates):
    return torch.library.custom_op(f"{_NS}::{name}", mutates_args=mutates, device_types="cuda")


# ---------------------------------------------------------------------------------------
@_op("rng_snapshot", ("counter", "snap"))
def rng_snapshot(counter: Tensor, snap: Tensor) -> None:
    L.check(L.load().cg_rng_snapshot(L.ptr(counter), L.ptr(snap), _s(counter)), "rng_snapshot")


@_op("counter_add", ("counter",))
def counter_add(counter: Tensor, delta: int) -> None:
    L.check(L.load().cg_counter_add(L.ptr(counter), delta, _s(counter)), "counter_add")


@_op("dropout_mask", ("out",))
def dropout_mask(out: Tensor, p: float, seed: int, rng_call: Optional[Tensor], site: int) -> None:
    L.check(L.load().cg_dropout_mask(L.ptr(out), out.numel(), p, seed, L.ptr(rng_call), site, _s(out)), "dropout_mask")


@_op("dropout_apply", ("out",))
def dropout_apply(x: Tensor, out: Tensor, p: float, seed: int, rng_call: Optional[Tensor], site: int) -> None:
    C = x.shape[-1]
    rows = x.numel() // C
    L.check(L.load().cg_dropout_apply(L.ptr(x), rows, C, C, L.ptr(out), L.dtype_code(out.dtype), p, seed,
                                      L.ptr(rng_call), site, _s(x)), "dropout_apply")


@_op("sum_scaled", ("out", "ws"))
def sum_scaled(x: Tensor, scale: float, out: Tensor, ws: Tensor) -> None:
    L.check(L.load().cg_sum_f32(L.ptr(x), x.numel(), scale, L.ptr(out), L.ptr(ws), _s(x)), "sum_f32")


@_op("cast_bf16", ("out",))
def cast_bf16(x: Tensor, out: Tensor) -> None:
    L.check(L.load().cg_cast_f32_bf16(L.ptr(x), L.ptr(out), x.numel(), _s(x)), "cast_f32_bf16")


@_op("gather_batch", ("x", "y"))
def gather_batch(data: Tensor, ix: Tensor, x: Tensor, y: Tensor) -> None:
    B, T = x.shape
    L.check(L.load().cg_gather_batch(L.ptr(data), int(data.dtype == torch.uint8), L.ptr(ix), L.ptr(x), L.ptr(y), B,
                                     T, _s(x)), "gather_batch")


# ---------------------------------------------------------------------------------------
@_op("embed_fwd", ("x",))
def embed_fwd(idx: Tensor, wte: Tensor, wpe: Tensor, x: Tensor) -> None:
    B, T = idx.shape
    V, C = wte.shape
    L.check(L.load().cg_embed_fwd(L.ptr(idx), L.ptr(wte), L.ptr(wpe), L.ptr(x), B, T, C, V, _s(x)), "embed_fwd")


@_op("embed_bwd", ("dwte", "dwpe", "ws"))
def embed_bwd(idx: Tensor, dx: Tensor, dwte: Optional[Tensor], dwpe: Optional[Tensor], accumulate: bool,
              ws: Tensor) -> None:
    B, T = idx.shape
    C = dx.shape[-1]
    V = dwte.shape[0] if dwte is not None else 1
    L.check(L.load().cg_embed_bwd(L.ptr(idx), L.ptr(dx), L.ptr(dwte), L.ptr(dwpe), B, T, C, V, int(accumulate),
                                  L.ptr(ws), _s(dx)), "embed_bwd")


def embed_bwd_workspace(B, T, C, V):
    return L.load().cg_embed_bwd_workspace(B, T, C, V)


# ---------------------------------------------------------------------------------------
@_op("layernorm_fwd", ("y", "mean", "rstd"))
def layernorm_fwd(x: Tensor, w: Tensor, b: Tensor, y: Tensor, mean: Tensor, rstd: Tensor, eps: float) -> None:
    C = x.shape[-1]
    rows = x.numel() // C
    L.check(L.load().cg_layernorm_fwd(L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(y), L.dtype_code(y.dtype), L.ptr(mean),
                                      L.ptr(rstd), rows, C, eps, _s(x)), "layernorm_fwd")


@_op("layernorm_fwd_attn_dropmask", ("y", "mean", "rstd", "mask"))
def layernorm_fwd_attn_dropmask(x: Tensor, w: Tensor, b: Tensor, y: Tensor, mean: Tensor, rstd: Tensor, eps: float,
                                B: int, H: int, T: int, dropout_p: float, seed: int, rng_call: Optional[Tensor],
                                site: int, mask: Tensor) -> None:
    """layernorm_fwd and attn_dropmask (the keep bits of the attention the LayerNorm feeds) in one
    launch; same results as the two ops."""
    C = x.shape[-1]
    rows = x.numel() // C
    L.check(L.load().cg_layernorm_fwd_attn_dropmask(L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(y), L.dtype_code(y.dtype),
                                                    L.ptr(mean), L.ptr(rstd), rows, C, eps, B, H, T, dropout_p, seed,
                                                    L.ptr(rng_call), site, L.ptr(mask), _s(x)),
            "layernorm_fwd_attn_dropmask")


@_op("layernorm_bwd", ("dx", "dx_lp", "dw", "db", "ws", "lp_colsum"))
def layernorm_bwd(dy: Tensor, x: Tensor, w: Tensor, mean: Tensor, rstd: Tensor, dres: Optional[Tensor], dx: Tensor,
                  dx_lp: Optional[Tensor], dw: Optional[Tensor], db: Optional[Tensor], accumulate: bool,
                  ws: Tensor, lp_colsum: Optional[Tensor], colsum_accumulate: bool, lp_p: float, lp_seed: int,
                  lp_rng_call: Optional[Tensor], lp_site: int) -> None:
    # (no defaults: torch.library drops trailing default-valued arguments from the boxed call, which
    #  would hide a mutated argument from its version-counter bookkeeping)
    C = x.shape[-1]
    rows = x.numel() // C
    L.check(L.load().cg_layernorm_bwd_ex(L.ptr(dy), L.dtype_code(dy.dtype), L.ptr(x), L.ptr(w), L.ptr(mean),
                                         L.ptr(rstd), L.ptr(dres), L.ptr(dx), L.ptr(dx_lp), lp_p, lp_seed,
                                         L.ptr(lp_rng_call), lp_site, L.ptr(dw), L.ptr(db), L.ptr(lp_colsum),
                                         int(accumulate), int(colsum_accumulate), L.ptr(ws), rows, C, _s(x)),
            "layernorm_bwd")


@_op("layernorm_bwd_rows", ("dx", "dx_lp", "ws"))
def layernorm_bwd_rows(dy: Tensor, x: Tensor, w: Tensor, mean: Tensor, rstd: Tensor, dres: Optional[Tensor],
                       dx: Tensor, dx_lp: Optional[Tensor], ws: Tensor, lp_colsum: bool, lp_p: float, lp_seed: int,
                       lp_rng_call: Optional[Tensor], lp_site: int) -> None:
    """layernorm_bwd without its column-sum reduce: the partials stay in ``ws`` for
    layernorm_bwd_reduce (launched on any stream ordered after this one)."""
    C = x.shape[-1]
    rows = x.numel() // C
    L.check(L.load().cg_layernorm_bwd_rows(L.ptr(dy), L.dtype_code(dy.dtype), L.ptr(x), L.ptr(w), L.ptr(mean),
                                           L.ptr(rstd), L.ptr(dres), L.ptr(dx), L.ptr(dx_lp), lp_p, lp_seed,
                                           L.ptr(lp_rng_call), lp_site, int(lp_colsum), L.ptr(ws), rows, C, _s(x)),
            "layernorm_bwd_rows")


@_op("layernorm_bwd_reduce", ("dw", "db", "lp_colsum"))
def layernorm_bwd_reduce(ws: Tensor, rows: int, C: int, colsum_partials: bool, dw: Optional[Tensor],
                         db: Optional[Tensor], lp_colsum: Optional[Tensor], accumulate: bool,
                         colsum_accumulate: bool, defer: bool = False) -> None:
    """defer: queued on the stream's deferral queue (CG_DEFER) until cg_flush_deferred."""
    L.check(L.load().cg_layernorm_bwd_reduce_ex(L.ptr(ws), rows, C, int(colsum_partials), L.ptr(dw), L.ptr(db),
                                                L.ptr(lp_colsum), int(accumulate), int(colsum_accumulate),
                                                L.DEFER if defer else 0, _s(ws)), "layernorm_bwd_reduce")


def layernorm_bwd_workspace(rows, C):
    return L.load().cg_layernorm_bwd_workspace(rows, C)


# ---------------------------------------------------------------------------------------
def _gemm_extents(a, b, out, a_trans, b_trans, M, N, K, lda, ldb, ldc, what="gemm"):
    """Host check that every element cg_gemm will address lies inside its tensor (the C ABI sees
    only pointers): A(m,k) = A[k lda + m] (a_trans) or A[m lda + k]; B(n,k) likewise; C[m ldc + n]."""
    need_a = (K - 1) * lda + M if a_trans else (M - 1) * lda + K
    need_b = (K - 1) * ldb + N if b_trans else (N - 1) * ldb + K
    need_c = (M - 1) * ldc + N
    for name, t, need in (("A", a, need_a), ("B", b, need_b), ("C", out, need_c)):
        if t is None or t.device.type == "meta":
            continue
        # views (a column block of qkv, ...) address their storage past their own numel
        avail = t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()
        if need > avail:
            raise ValueError(f"charpt {what}: operand {name} needs {need} elements for M={M} N={N} K={K} "
                             f"(trans {int(a_trans)}{int(b_trans)}, ld {lda}/{ldb}/{ldc}), its storage has {avail}")


@_op("gemm", ("out", "ws"))
def gemm(a: Tensor, b: Tensor, out: Tensor, op_bf16: bool, a_trans: bool, b_trans: bool, M: int, N: int, K: int,
         lda: int, ldb: int, ldc: int, epi: int, bias: Optional[Tensor], resid: Optional[Tensor], ld_resid: int,
         aux: Optional[Tensor], ld_aux: int, dropout_p: float, seed: int, rng_call: Optional[Tensor], site: int,
         beta: float, split_k: int, ws: Optional[Tensor], flags: int = 0) -> None:
    """flags: cg_epilogue_t.flags (L.GEMM_SLAB_BF16 | L.GEMM_DEFER_REDUCE) of a split-K weight gradient."""
    _gemm_extents(a, b, out, a_trans, b_trans, M, N, K, lda, ldb, ldc)
    e = L.Epilogue(epi, L.ptr(bias), L.ptr(resid), ld_resid, L.ptr(aux),
                   L.dtype_code(aux.dtype) if aux is not None else 0, ld_aux, dropout_p, seed, L.ptr(rng_call), site,
                   beta, None, flags)
    L.check(L.load().cg_gemm(L.CG_BF16 if op_bf16 else L.CG_F32, int(a_trans), int(b_trans), M, N, K, L.ptr(a), lda,
                             L.ptr(b), ldb, L.ptr(out), L.dtype_code(out.dtype), ldc, e, split_k, L.ptr(ws), _s(out)),
            "gemm")


@_op("gemm_bias_relu_bits", ("out", "bits"))
def gemm_bias_relu_bits(a: Tensor, b: Tensor, out: Tensor, M: int, N: int, K: int, lda: int, ldb: int, ldc: int,
                        bias: Tensor, bits: Tensor, ld_bits: int) -> None:
    """out = bf16 relu(a[M,K] @ b[N,K]^T + bias) and its ReLU keep bits (CG_BITS: int32 words
    [M, ld_bits], bit n % 32 of word n / 32 = out[m, n] != 0) for the ReLU-backward dgrad.  Fails
    (CG_EINVAL) unless cg_gemm_relu_bits_supported."""
    _gemm_extents(a, b, out, False, False, M, N, K, lda, ldb, ldc, "gemm_bias_relu_bits")
    e = L.Epilogue(L.EPI_BIAS_RELU, L.ptr(bias), None, 0, L.ptr(bits), L.CG_BITS, ld_bits, 0.0, 0, None, 0, 0.0)
    L.check(L.load().cg_gemm(L.CG_BF16, 0, 0, M, N, K, L.ptr(a), lda, L.ptr(b), ldb, L.ptr(out),
                             L.dtype_code(out.dtype), ldc, e, 1, None, _s(out)), "gemm_bias_relu_bits")


@_op("gemm_relu_bwd_colpart", ("out", "colpart"))
def gemm_relu_bwd_colpart(a: Tensor, b: Tensor, out: Tensor, M: int, N: int, K: int, lda: int, ldb: int, ldc: int,
                          aux: Tensor, ld_aux: int, colpart: Tensor) -> None:
    """out = relu_bwd(a[M,K] @ b[N,K]^T, aux) in bf16 with the column sums of every 64-row block of
    the output into colpart [M/64, N] (the consumer's bias-gradient partials; cg_reduce_rows folds
    them).  Fails (CG_EINVAL) unless the dispatch takes the 128x128 persistent kernel."""
    _gemm_extents(a, b, out, False, True, M, N, K, lda, ldb, ldc, "gemm_relu_bwd_colpart")
    e = L.Epilogue(L.EPI_RELU_BWD, None, None, 0, L.ptr(aux), L.dtype_code(aux.dtype), ld_aux, 0.0, 0, None, 0, 0.0,
                   L.ptr(colpart))
    L.check(L.load().cg_gemm(L.CG_BF16, 0, 1, M, N, K, L.ptr(a), lda, L.ptr(b), ldb, L.ptr(out),
                             L.dtype_code(out.dtype), ldc, e, 1, None, _s(out)), "gemm_relu_bwd_colpart")


@_op("gemm_store_rowdot", ("out", "delta"))
def gemm_store_rowdot(a: Tensor, b: Tensor, out: Tensor, M: int, N: int, K: int, lda: int, ldb: int, ldc: int,
                      o: Tensor, ld_o: int, T: int, delta: Tensor) -> None:
    """out = bf16(a[M,K] @ b[N,K]^T) (the attention-output gradient dO) and the attention backward's
    delta[b, h, t] = sum_e out[b*T + t, 64h + e] * o[b*T + t, 64h + e] (fp32 [M/T, N/64, T]) from
    the rounded values.  Fails (CG_EINVAL) unless cg_gemm_rowdot_supported."""
    _gemm_extents(a, b, out, False, True, M, N, K, lda, ldb, ldc, "gemm_store_rowdot")
    e = L.Epilogue(L.EPI_STORE_ROWDOT, None, None, T, L.ptr(o), L.dtype_code(o.dtype), ld_o, 0.0, 0, None, 0, 0.0,
                   L.ptr(delta))
    L.check(L.load().cg_gemm(L.CG_BF16, 0, 1, M, N, K, L.ptr(a), lda, L.ptr(b), ldb, L.ptr(out),
                             L.dtype_code(out.dtype), ldc, e, 1, None, _s(out)), "gemm_store_rowdot")


@_op("gemm_resid_layernorm", ("out", "y", "mean", "rstd"))
def gemm_resid_layernorm(a: Tensor, w: Tensor, out: Tensor, M: int, N: int, K: int, lda: int, ldw: int, ldc: int,
                         bias: Tensor, resid: Tensor, ld_resid: int, dropout_p: float, seed: int,
                         rng_call: Optional[Tensor], site: int, ln_w: Tensor, ln_b: Tensor, y: Tensor, mean: Tensor,
                         rstd: Tensor, eps: float) -> None:
    """out = resid + dropout(a[M,K] @ w[N,K]^T + bias) (fp32; dropout_p 0: none) and y = LayerNorm(out;
    ln_w, ln_b) (bf16, row stride N), mean, rstd in one launch -- the bits of gemm(...,
    "bias_[drop_]resid") followed by layernorm_fwd.  Fails (CG_EINVAL) unless
    gemm_resid_layernorm_supported(M, N, K)."""
    _gemm_extents(a, w, out, False, False, M, N, K, lda, ldw, ldc, "gemm_resid_layernorm")
    kind = L.EPI_BIAS_DROP_RESID if dropout_p > 0 else L.EPI_BIAS_RESID
    e = L.Epilogue(kind, L.ptr(bias), L.ptr(resid), ld_resid, None, 0, 0, dropout_p, seed, L.ptr(rng_call), site, 0.0)
    L.check(L.load().cg_gemm_resid_layernorm(M, N, K, L.ptr(a), lda, L.ptr(w), ldw, L.ptr(out), ldc, e, L.ptr(ln_w),
                                             L.ptr(ln_b), L.ptr(y), L.ptr(mean), L.ptr(rstd), eps, _s(out)),
            "gemm_resid_layernorm")


@_op("linear_rows_f32", ("out",))
def linear_rows_f32(a: Tensor, ln_w: Optional[Tensor], ln_b: Optional[Tensor], eps: float, w: Tensor,
                    bias: Optional[Tensor], resid: Optional[Tensor], out: Tensor, relu: bool = False) -> None:
    """out = [resid +] act(a' @ w^T [+ bias]), a' = LayerNorm(a; ln_w, ln_b, eps) (or a when ln_w is None),
    act = relu when relu (bias, no resid), fp32, K <= 128, one launch -- the bits of [layernorm_fwd +]
    gemm(..., "store" / "bias" / "bias_relu" / "bias_resid").  Fails (CG_EINVAL) unless
    linear_rows_f32_supported(M, N, K)."""
    M, K = a.shape
    N = w.shape[0]
    for t, name in ((a, "a"), (w, "w"), (bias, "bias"), (resid, "resid"), (out, "out"), (ln_w, "ln_w"),
                    (ln_b, "ln_b")):
        if t is None:
            continue
        if t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"linear_rows_f32: {name} must be a float32 device tensor")
        if t.dim() == 2 and t.stride(1) != 1:
            raise ValueError(f"linear_rows_f32: {name} must have unit column stride")
    if (ln_w is None) != (ln_b is None) or (ln_w is not None and (ln_w.numel() != K or ln_b.numel() != K)):
        raise ValueError("linear_rows_f32: ln_w and ln_b both [K] or both None")
    if tuple(w.shape) != (N, K) or (bias is not None and bias.numel() != N) or tuple(out.shape) != (M, N) or \
            (resid is not None and tuple(resid.shape) != (M, N)):
        raise ValueError(f"linear_rows_f32: shapes a {tuple(a.shape)} w {tuple(w.shape)} out {tuple(out.shape)}")
    L.check(L.load().cg_linear_rows_f32(M, N, K, L.ptr(a), a.stride(0), L.ptr(ln_w), L.ptr(ln_b), eps, L.ptr(w),
                                        w.stride(0), L.ptr(bias), int(relu), L.ptr(resid),
                                        resid.stride(0) if resid is not None else 0, L.ptr(out), out.stride(0),
                                        _s(out)), "linear_rows_f32")


def linear_rows_f32_supported(M, N, K):
    return bool(L.load().cg_linear_rows_f32_supported(M, N, K))


@_op("ffn_fwd_f32", ("out",))
def ffn_fwd_f32(a: Tensor, ln_w: Optional[Tensor], ln_b: Optional[Tensor], eps: float, w1: Tensor, b1: Tensor,
                w2: Tensor, b2: Tensor, resid: Tensor, out: Tensor) -> None:
    """out = resid + (relu(a' @ w1^T + b1) @ w2^T + b2), a' = LayerNorm(a; ln_w, ln_b, eps) (or a when
    ln_w is None), fp32, one launch (FeedForward + its ln2 in eval) -- the bits of layernorm_fwd, then
    gemm(..., "bias_relu") into an [M, H] buffer, then gemm(..., "bias_resid").  Fails (CG_EINVAL)
    unless ffn_fwd_f32_supported(M, C, H)."""
    M, C = a.shape
    H = w1.shape[0]
    for t, name in ((a, "a"), (w1, "w1"), (b1, "b1"), (w2, "w2"), (b2, "b2"), (resid, "resid"), (out, "out"),
                    (ln_w, "ln_w"), (ln_b, "ln_b")):
        if t is None:
            continue
        if t.dtype != torch.float32 or not t.is_cuda:
            raise ValueError(f"ffn_fwd_f32: {name} must be a float32 device tensor")
        if t.dim() == 2 and t.stride(1) != 1:
            raise ValueError(f"ffn_fwd_f32: {name} must have unit column stride")
    if (ln_w is None) != (ln_b is None) or (ln_w is not None and (ln_w.numel() != C or ln_b.numel() != C)):
        raise ValueError("ffn_fwd_f32: ln_w and ln_b both [C] or both None")
    if tuple(w1.shape) != (H, C) or tuple(w2.shape) != (C, H) or b1.numel() != H or b2.numel() != C or \
            tuple(resid.shape) != (M, C) or tuple(out.shape) != (M, C):
        raise ValueError(f"ffn_fwd_f32: shapes a {tuple(a.shape)} w1 {tuple(w1.shape)} w2 {tuple(w2.shape)} "
                         f"b1 {b1.numel()} b2 {b2.numel()} resid {tuple(resid.shape)} out {tuple(out.shape)}")
    L.check(L.load().cg_ffn_fwd_f32(M, C, H, L.ptr(a), a.stride(0), L.ptr(ln_w), L.ptr(ln_b), eps, L.ptr(w1),
                                    w1.stride(0), L.ptr(b1), L.ptr(w2), w2.stride(0), L.ptr(b2), L.ptr(resid),
                                    resid.stride(0), L.ptr(out), out.stride(0), _s(out)), "ffn_fwd_f32")


def ffn_fwd_f32_supported(M, C, H):
    return bool(L.load().cg_ffn_fwd_f32_supported(M, C, H))


def gemm_resid_layernorm_supported(M, N, K):
    return bool(L.load().cg_gemm_resid_layernorm_supported(M, N, K))


def gemm_rowdot_supported(M, N, K, lda, ldb, ldc):
    return bool(L.load().cg_gemm_rowdot_supported(0, 1, M, N, K, lda, ldb, ldc))


@_op("reduce_rows", ("out",))
def reduce_rows(part: Tensor, rows: int, N: int, out: Tensor, accumulate: bool, defer: bool = False) -> None:
    """defer: queued on the stream's deferral queue (CG_DEFER) until cg_flush_deferred."""
    L.check(L.load().cg_reduce_rows_ex(L.ptr(part), rows, N, L.ptr(out), int(accumulate), L.DEFER if defer else 0,
                                       _s(out)), "reduce_rows")


def gemm_workspace(M, N, split_k):
    return L.load().cg_gemm_workspace(M, N, split_k)


@_op("colsum", ("out", "ws"))
def colsum(x: Tensor, out: Tensor, accumulate: bool, ws: Tensor) -> None:
    N = x.shape[-1]
    rows = x.numel() // N
    L.check(L.load().cg_colsum(L.ptr(x), L.dtype_code(x.dtype), rows, N, N, L.ptr(out), int(accumulate), L.ptr(ws),
                               _s(x)), "colsum")


def colsum_workspace(rows, N):
    return L.load().cg_colsum_workspace(rows, N)


# ---------------------------------------------------------------------------------------
@_op("attn_fwd", ("o", "lse", "mask"))
def attn_fwd(qkv: Tensor, B: int, T: int, H: int, D: int, q_off: int, k_off: int, v_off: int, ld: int, o: Tensor,
             ld_o: int, lse: Tensor, scale: float, dropout_p: float, seed: int, rng_call: Optional[Tensor],
             site: int, mask: Optional[Tensor], mask_ready: bool = False) -> None:
    es = qkv.element_size()
    base = qkv.data_ptr()
    fn = L.load().cg_attn_fwd_premasked if mask_ready else L.load().cg_attn_fwd
    L.check(fn(L.dtype_code(qkv.dtype), B, T, H, D, base + q_off * es, base + k_off * es, base + v_off * es, ld,
               L.ptr(o), ld_o, L.ptr(lse), scale, dropout_p, seed, L.ptr(rng_call), site, L.ptr(mask), _s(qkv)),
            "attn_fwd")


@_op("attn_dropmask", ("mask",))
def attn_dropmask(B: int, H: int, T: int, dropout_p: float, seed: int, rng_call: Optional[Tensor], site: int,
                  mask: Tensor) -> None:
    L.check(L.load().cg_attn_dropmask(B, H, T, dropout_p, seed, L.ptr(rng_call), site, L.ptr(mask), _s(mask)),
            "attn_dropmask")


def attn_mask_bytes(B, H, T):
    return L.load().cg_attn_mask_bytes(B, H, T)


@_op("attn_bwd", ("dqkv", "ws"))
def attn_bwd(qkv: Tensor, B: int, T: int, H: int, D: int, q_off: int, k_off: int, v_off: int, ld: int, o: Tensor,
             ld_o: int, dout: Tensor, ld_do: int, lse: Tensor, dqkv: Tensor, ld_d: int, scale: float,
             dropout_p: float, seed: int, rng_call: Optional[Tensor], site: int, mask: Optional[Tensor],
             ws: Tensor, delta: Optional[Tensor] = None) -> None:
    """delta: rowsum(dO * O) precomputed (gemm_store_rowdot), fp32 [B, H, T]; None: computed here."""
    es = qkv.element_size()
    base, dbase = qkv.data_ptr(), dqkv.data_ptr()
    L.check(L.load().cg_attn_bwd_delta(L.dtype_code(qkv.dtype), B, T, H, D, base + q_off * es, base + k_off * es,
                                       base + v_off * es, ld, L.ptr(o), ld_o, L.ptr(dout), ld_do, L.ptr(lse),
                                       L.ptr(delta), dbase + q_off * es, dbase + k_off * es, dbase + v_off * es, ld_d,
                                       scale, dropout_p, seed, L.ptr(rng_call), site, L.ptr(mask), L.ptr(ws),
                                       _s(qkv)), "attn_bwd")


def attn_bwd_workspace(B, T, H, D):
    return L.load().cg_attn_bwd_workspace(B, T, H, D)


# ---------------------------------------------------------------------------------------
@_op("ce_fwd", ("loss_rows", "lse"))
def ce_fwd(logits: Tensor, targets: Optional[Tensor], loss_rows: Optional[Tensor], lse: Tensor) -> None:
    V = logits.shape[-1]
    rows = logits.numel() // V
    L.check(L.load().cg_ce_fwd(L.ptr(logits), rows, V, V, L.ptr(targets), L.ptr(loss_rows), L.ptr(lse),
                               _s(logits)), "ce_fwd")


@_op("ce_bwd", ("dlogits", "dlogits_lp"))
def ce_bwd(logits: Tensor, targets: Tensor, lse: Tensor, g: Tensor, g_mult: float, dlogits: Optional[Tensor],
           dlogits_lp: Optional[Tensor]) -> None:
    V = logits.shape[-1]
    rows = logits.numel() // V
    L.check(L.load().cg_ce_bwd(L.ptr(logits), rows, V, V, L.ptr(targets), L.ptr(lse), L.ptr(g), g_mult,
                               L.ptr(dlogits), V, L.ptr(dlogits_lp), _s(logits)), "ce_bwd")


def head_workspace(M: int, V: int) -> int:
    return int(L.load().cg_head_workspace(M, V))


@_op("head_fwd", ("logits", "lse", "loss", "ws"))
def head_fwd(a: Tensor, wpad: Tensor, bias: Tensor, targets: Optional[Tensor], logits: Tensor, lse: Tensor,
             loss: Optional[Tensor], ws: Optional[Tensor]) -> None:
    M, C = a.shape
    V = logits.shape[-1]
    L.check(L.load().cg_head_fwd(L.ptr(a), L.ptr(wpad), wpad.shape[0], L.ptr(bias), L.ptr(targets), L.ptr(logits),
                                 L.ptr(lse), L.ptr(loss), L.ptr(ws), M, C, V, _s(a)), "head_fwd")


@_op("head_bwd", ("dl", "db", "ws"))
def head_bwd(logits: Tensor, lse: Tensor, targets: Optional[Tensor], g_loss: Optional[Tensor], g_mult: float,
             g_logits: Optional[Tensor], dl: Tensor, db: Optional[Tensor], db_accumulate: bool, ws: Tensor,
             defer: bool = False) -> None:
    """defer: the db column-sum reduce is queued on the stream's deferral queue (CG_DEFER)."""
    M, V = logits.shape
    L.check(L.load().cg_head_bwd_ex(L.ptr(logits), L.ptr(lse), L.ptr(targets), L.ptr(g_loss), g_mult,
                                    L.ptr(g_logits), L.ptr(dl), dl.stride(0), L.ptr(db), int(db_accumulate), L.ptr(ws),
                                    M, V, L.DEFER if defer else 0, _s(logits)), "head_bwd")


# ---------------------------------------------------------------------------------------
# batched decode (decode.py)
@_op("decode_window", ("out",))
def decode_window(idx: Tensor, len_dev: Tensor, out: Tensor) -> None:
    B, T = out.shape
    L.check(L.load().cg_decode_window(L.ptr(idx), idx.stride(0), B, T, L.ptr(len_dev), L.ptr(out), _s(idx)),
            "decode_window")


@_op("decode_embed", ("x",))
def decode_embed(idx: Tensor, wte: Tensor, wpe: Tensor, len_dev: Tensor, x: Tensor) -> None:
    B, C = x.shape
    L.check(L.load().cg_decode_embed(L.ptr(idx), idx.stride(0), L.ptr(wte), L.ptr(wpe), C, L.ptr(len_dev), L.ptr(x),
                                     B, _s(x)), "decode_embed")


@_op("decode_kv_append", ("kcache", "vcache"))
def decode_kv_append(qkv: Tensor, k_off: int, v_off: int, len_dev: Tensor, kcache: Tensor, vcache: Tensor) -> None:
    B, H, Tmax, D = kcache.shape
    L.check(L.load().cg_decode_kv_append(L.ptr(qkv), qkv.stride(0), k_off, v_off, B, H, D, Tmax, L.ptr(len_dev),
                                         L.ptr(kcache), L.ptr(vcache), _s(qkv)), "decode_kv_append")


@_op("decode_qkv_f32", ("qkv", "kcache", "vcache"))
def decode_qkv_f32(x: Tensor, ln_w: Tensor, ln_b: Tensor, eps: float, w: Tensor, qkv: Tensor, len_dev: Tensor,
                   kcache: Tensor, vcache: Tensor) -> None:
    """qkv = LayerNorm(x) @ w^T and its K / V columns appended to the caches at position len - 1, fp32,
    one launch -- the bits of linear_rows_f32(x, ln_w, ln_b, eps, w, ...) then decode_kv_append."""
    B, C = x.shape
    _, H, Tmax, D = kcache.shape
    for t, name in ((x, "x"), (w, "w"), (qkv, "qkv"), (kcache, "kcache"), (vcache, "vcache")):
        if t.dtype != torch.float32 or not t.is_cuda or t.stride(-1) != 1:
            raise ValueError(f"decode_qkv_f32: {name} must be a float32 device tensor with unit column stride")
    if tuple(w.shape) != (3 * C, C) or tuple(qkv.shape) != (B, 3 * C) or H * D != C or \
            tuple(kcache.shape) != (B, H, Tmax, D) or not kcache.is_contiguous() or \
            tuple(vcache.shape) != tuple(kcache.shape) or not vcache.is_contiguous():
        raise ValueError(f"decode_qkv_f32: shapes x {tuple(x.shape)} w {tuple(w.shape)} kcache {tuple(kcache.shape)}")
    L.check(L.load().cg_decode_qkv_f32(B, C, H, L.ptr(x), x.stride(0), L.ptr(ln_w), L.ptr(ln_b), eps, L.ptr(w),
                                       w.stride(0), L.ptr(qkv), qkv.stride(0), L.ptr(len_dev), Tmax, L.ptr(kcache),
                                       L.ptr(vcache), _s(x)), "decode_qkv_f32")


@_op("decode_attn", ("o",))
def decode_attn(q: Tensor, ldq: int, k: Tensor, k_off: int, v: Tensor, v_off: int, sb: int, sh: int, sj: int, B: int,
                H: int, D: int, len_dev: Optional[Tensor], nkeys: int, scale: float, o: Tensor) -> None:
    es = k.element_size()
    L.check(L.load().cg_decode_attn(L.ptr(q), ldq, k.data_ptr() + k_off * es, v.data_ptr() + v_off * es, sb, sh, sj,
                                    B, H, D, L.ptr(len_dev), nkeys, scale, L.ptr(o), o.stride(0), _s(q)),
            "decode_attn")


@_op("decode_sample", ("idx",))
def decode_sample(logits: Tensor, greedy: bool, seed: Tensor, len_dev: Tensor, idx: Tensor) -> None:
    B, V = logits.shape
    L.check(L.load().cg_decode_sample(L.ptr(logits), logits.stride(0), V, B, int(greedy), L.ptr(seed),
                                      L.ptr(len_dev), L.ptr(idx), idx.stride(0), _s(logits)), "decode_sample")


# ---------------------------------------------------------------------------------------
@_op("adamw", ("p", "m", "v", "p_bf16"))
def adamw(p: Tensor, g: Tensor, m: Tensor, v: Tensor, p_bf16: Optional[Tensor], lr: float, beta1: float, beta2: float,
          eps: float, weight_decay: float, step: Tensor) -> None:
    L.check(L.load().cg_adamw(L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), L.ptr(p_bf16), p.numel(), lr, beta1, beta2, eps,
                              weight_decay, L.ptr(step), _s(p)), "adamw")


@_op("adamw_defer", ("p", "m", "v", "p_bf16"))
def adamw_defer(p: Tensor, g: Tensor, m: Tensor, v: Tensor, p_bf16: Tensor, lr: float, beta1: float, beta2: float,
                eps: float, weight_decay: float, step: Tensor) -> None:
    """adamw over one region, queued: run by the free blocks of the next part-filling persistent GEMM
    launch on this stream, or by cg_flush_deferred (csrc gemm.hip cg_adamw_defer); same bits."""
    L.check(L.load().cg_adamw_defer(L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), L.ptr(p_bf16), p.numel(), lr, beta1,
                                    beta2, eps, weight_decay, L.ptr(step), _s(p)), "adamw_defer")


@_op("adamw_segments", ("p", "m", "v", "p_bf16"))
def adamw_segments(p: Tensor, g: Tensor, m: Tensor, v: Tensor, p_bf16: Optional[Tensor], segs: List[int],
                   lr: float, beta1: float, beta2: float, eps: float, weight_decay: float, step: Tensor) -> None:
    """adamw over [start, start + length) segments of the flat buffers (segs = [s0, n0, s1, n1, ...])."""
    arr = (L.ctypes.c_int64 * len(segs))(*segs)
    L.check(L.load().cg_adamw_segments(L.ptr(p), L.ptr(g), L.ptr(m), L.ptr(v), L.ptr(p_bf16), arr, len(segs) // 2, lr,
                                       beta1, beta2, eps, weight_decay, L.ptr(step), _s(p)), "adamw_segments")


# ---------------------------------------------------------------------------------------
# Fake (meta) implementations of the out-style ops above: each returns None and only writes
# buffers it declares as mutated, so FakeTensor / torch.compile tracing treats it as a no-op on
# shapes.
for _name, _obj in list(globals().items()):
    if isinstance(_obj, torch._library.custom_ops.CustomOpDef):
        _obj.register_fake(lambda *a, **k: None)


# ---------------------------------------------------------------------------------------
# Functional ops with fake + autograd registrations (torch.library.register_fake /
# register_autograd): the traceable seam of the GPT1.py module surface outside the fused model
# path -- nn.LayerNorm (GPT1.py:159-160,173), nn.Linear (:103-105,131,143,145,174) and the causal
# softmax-attention of Head / MultiHeadAttention (:109-123,134-135), all heads at once.  The
# fused training nodes (functional.AttnSublayerFn / FFNSublayerFn / HeadLossFn) stay
# autograd.Functions: they write parameter gradients straight into the model's flat gradient
# buffer, hand bf16 gradient copies between sublayers (GradLink) and fork side-stream work --
# effects a functional custom op cannot express.  Forward and backward are each ONE custom op, so a
# tracer only ever sees their fakes; all host-side kernel selection stays inside the real bodies.
def _flat_rows(x):
    return x.reshape(-1, x.shape[-1])


@torch.library.custom_op(f"{_NS}::layer_norm", mutates_args=(), device_types="cuda")
def layer_norm(x: Tensor, weight: Tensor, bias: Tensor, eps: float) -> tuple[Tensor, Tensor, Tensor]:
    """y = (x - mean) * rstd * weight + bias over the last dim (fp32); also returns mean, rstd."""
    x2 = _flat_rows(x).contiguous()
    rows = x2.shape[0]
    y = torch.empty_like(x2)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    layernorm_fwd(x2, weight, bias, y, mean, rstd, eps)
    return y.view(x.shape), mean, rstd


@layer_norm.register_fake
def _(x, weight, bias, eps):
    rows = x.numel() // x.shape[-1]
    return torch.empty_like(x), x.new_empty(rows), x.new_empty(rows)


@torch.library.custom_op(f"{_NS}::layer_norm_backward", mutates_args=(), device_types="cuda")
def layer_norm_backward(dy: Tensor, x: Tensor, weight: Tensor, mean: Tensor, rstd: Tensor) -> tuple[Tensor, Tensor, Tensor]:
    x2 = _flat_rows(x).contiguous()
    rows, C = x2.shape
    dx = torch.empty_like(x2)
    dw = torch.empty(C, dtype=torch.float32, device=x.device)
    db = torch.empty(C, dtype=torch.float32, device=x.device)
    ws = torch.empty(layernorm_bwd_workspace(rows, C) // 4 + 1, dtype=torch.float32, device=x.device)
    layernorm_bwd(_flat_rows(dy).float().contiguous(), x2, weight, mean, rstd, None, dx, None, dw, db, False, ws, None,
                  False, 0.0, 0, None, 0)
    return dx.view(x.shape), dw, db


@layer_norm_backward.register_fake
def _(dy, x, weight, mean, rstd):
    C = x.shape[-1]
    return torch.empty_like(x), x.new_empty(C), x.new_empty(C)


def _ln_setup(ctx, inputs, output):
    x, weight, _, _ = inputs
    _, mean, rstd = output
    ctx.save_for_backward(x, weight, mean, rstd)


def _ln_backward(ctx, dy, _dmean, _drstd):
    x, weight, mean, rstd = ctx.saved_tensors
    dx, dw, db = layer_norm_backward(dy, x, weight, mean, rstd)
    return dx, dw, db, None


layer_norm.register_autograd(_ln_backward, setup_context=_ln_setup)


@torch.library.custom_op(f"{_NS}::linear", mutates_args=(), device_types="cuda")
def linear(x: Tensor, weight: Tensor, bias: Optional[Tensor]) -> Tensor:
    """y = x weight^T (+ bias): fp32 (exact f32 MFMA) or bf16 (bf16 MFMA, fp32 accumulate) operands,
    bias fp32, output in x's dtype."""
    from . import functional as Fn
    x2 = _flat_rows(x).contiguous()
    out = torch.empty((x2.shape[0], weight.shape[0]), dtype=x.dtype, device=x.device)
    Fn.linear_fwd(x2, weight.contiguous(), out, "bias" if bias is not None else "store", bias=bias)
    return out.view(*x.shape[:-1], weight.shape[0])


@linear.register_fake
def _(x, weight, bias):
    return x.new_empty((*x.shape[:-1], weight.shape[0]))


@torch.library.custom_op(f"{_NS}::linear_backward", mutates_args=(), device_types="cuda")
def linear_backward(dy: Tensor, x: Tensor, weight: Tensor, with_bias: bool) -> tuple[Tensor, Tensor, Tensor]:
    """(dx, dweight, dbias): dy weight, dy^T x (fp32 accumulation, deterministic split-K), colsum(dy);
    dbias is empty when with_bias is False."""
    from . import functional as Fn
    dy2 = _flat_rows(dy).to(x.dtype).contiguous()
    x2 = _flat_rows(x).contiguous()
    w = weight.contiguous()
    dx = torch.empty_like(x2)
    Fn.linear_dgrad(dy2, w, dx)
    dw32 = torch.empty(w.shape, dtype=torch.float32, device=x.device)
    Fn.linear_wgrad(dy2, x2, dw32, 0.0)
    dw = dw32 if w.dtype == torch.float32 else Fn.to_act(dw32, w.dtype)
    db = torch.empty(w.shape[0] if with_bias else 0, dtype=torch.float32, device=x.device)
    if with_bias:
        Fn.colsum_into(dy2, db, 0.0)
    return dx.view(x.shape), dw, db


@linear_backward.register_fake
def _(dy, x, weight, with_bias):
    return torch.empty_like(x), torch.empty_like(weight), x.new_empty(weight.shape[0] if with_bias else 0,
                                                                      dtype=torch.float32)


def _lin_setup(ctx, inputs, output):
    x, weight, bias = inputs
    ctx.save_for_backward(x, weight)
    ctx.with_bias = bias is not None


def _lin_backward(ctx, dy):
    x, weight = ctx.saved_tensors
    dx, dw, db = linear_backward(dy, x, weight, ctx.with_bias)
    return dx, dw, (db if ctx.with_bias else None)


linear.register_autograd(_lin_backward, setup_context=_lin_setup)


@torch.library.custom_op(f"{_NS}::causal_attention", mutates_args=(), device_types="cuda")
def causal_attention(qkv: Tensor, n_head: int, head_size: int, scale: float, dropout_p: float, seed: int,
                     rng_call: Optional[Tensor], site: int) -> tuple[Tensor, Tensor]:
    """All heads of GPT1.py's Head.forward at once: qkv [B, T, 3*H*D] (queries of every head, then
    keys, then values; head-major inside each) -> (out [B, T, H*D] = the torch.cat of GPT1.py:135,
    logsumexp [B, H, T]).  Causal mask, softmax with scale (n_embd^-0.5), Philox dropout on
    the probabilities (dropout stream (rng_call, site), key seed)."""
    from . import functional as Fn
    B, T, _ = qkv.shape
    d = n_head * head_size
    q2 = qkv.reshape(B * T, 3 * d).contiguous()
    o = torch.empty((B * T, d), dtype=qkv.dtype, device=qkv.device)
    lse, _mask = Fn.attention_fwd(q2, B, T, n_head, head_size, o, scale, dropout_p, seed, rng_call, site)
    return o.view(B, T, d), lse


@causal_attention.register_fake
def _(qkv, n_head, head_size, scale, dropout_p, seed, rng_call, site):
    B, T, _ = qkv.shape
    return qkv.new_empty((B, T, n_head * head_size)), qkv.new_empty((B, n_head, T), dtype=torch.float32)


@torch.library.custom_op(f"{_NS}::causal_attention_backward", mutates_args=(), device_types="cuda")
def causal_attention_backward(dout: Tensor, qkv: Tensor, out: Tensor, lse: Tensor, n_head: int, head_size: int,
                              scale: float, dropout_p: float, seed: int, rng_call: Optional[Tensor],
                              site: int) -> Tensor:
    """d qkv of causal_attention (the forward's dropout keep bits are regenerated from the stream)."""
    from . import functional as Fn
    B, T, _ = qkv.shape
    d = n_head * head_size
    q2 = qkv.reshape(B * T, 3 * d).contiguous()
    dq = Fn.attention_bwd(q2, B, T, n_head, head_size, out.reshape(B * T, d).contiguous(),
                          dout.reshape(B * T, d).to(qkv.dtype).contiguous(), lse.contiguous(), scale, dropout_p, seed,
                          rng_call, site, None)
    return dq.view(qkv.shape)


@causal_attention_backward.register_fake
def _(dout, qkv, out, lse, n_head, head_size, scale, dropout_p, seed, rng_call, site):
    return torch.empty_like(qkv)


def _attn_setup(ctx, inputs, output):
    qkv, n_head, head_size, scale, p, seed, rng_call, site = inputs
    o, lse = output
    ctx.save_for_backward(qkv, o, lse, rng_call)
    ctx.args = (n_head, head_size, scale, p, seed, site)


def _attn_backward(ctx, dout, _dlse):
    qkv, o, lse, rng_call = ctx.saved_tensors
    n_head, head_size, scale, p, seed, site = ctx.args
    dq = causal_attention_backward(dout, qkv, o, lse, n_head, head_size, scale, p, seed, rng_call, site)
    return dq, None, None, None, None, None, None, None


causal_attention.register_autograd(_attn_backward, setup_context=_attn_setup)
