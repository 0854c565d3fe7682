"""Autograd functions for the char-GPT hot path, each a fixed sequence of charpt kernels.

The fused training path is two autograd nodes per Block (GPT1.py:162-165):

  AttnSublayer:  x + proj(attn(qkv(ln1(x))))            (GPT1.py:163, 134-136, 109-123)
  FFNSublayer:   x + drop(W2 relu(W1 ln2(x) + b1) + b2)  (GPT1.py:164, 142-147)

plus the embedding (GPT1.py:179-181) and the ln_f + lm_head + cross-entropy tail
(GPT1.py:183-192).  Standalone module calls (Head, MultiHeadAttention, FeedForward, LayerNorm
outside a model) use the elementary functions at the bottom.

Parameter gradients are written by the kernels straight into the model's flat fp32 gradient
buffer ("grad slots"), see ``Region``; the residual-stream gradient is fp32, activations and
GEMM operands are bf16 (or fp32 in exact mode).
"""
import contextlib
import ctypes
import os
import math

import torch

from . import _lib as L
from . import ops

EPI = {"store": L.EPI_STORE, "bias": L.EPI_BIAS, "bias_relu": L.EPI_BIAS_RELU, "bias_resid": L.EPI_BIAS_RESID,
       "bias_drop_resid": L.EPI_BIAS_DROP_RESID, "relu_bwd": L.EPI_RELU_BWD}


class SideStream:
    """An optional second HIP stream for work off the backward's critical path (weight gradients,
    bias column sums, their split-K reductions) and for the forward's dropout keep bits.  The dgrad
    chain keeps the main stream; hipGraph replay keeps the fork/join as graph edges, so the two
    branches can run concurrently.  Tensors read by side work are kept alive until ``join()``,
    which makes the main stream wait for everything forked so far; the model's embedding backward
    (the last autograd node), AdamW.step and TrainStep call it.

    OFF by default: measured on MI355X (profiles/r2_side_stream_ab.txt) the graph spreads the two
    branches over hardware queues and every cross-queue edge costs ~10-20 us of idle GPU, more than
    the overlap buys -- one stream is as fast or up to 1.7 % faster at C2 (GPU 100 % busy, 17 us idle per step) and
    4.3 % faster at C4.  CHARPT_SIDE: "1" all of the above on the side stream, "mask" only the keep
    bits, "0" (default) one stream."""

    def __init__(self):
        mode = os.environ.get("CHARPT_SIDE", "0")
        self.enabled = mode == "1"
        self.premask = mode in ("1", "mask")
        self._streams = {}
        self._keep = []
        self._pending = set()

    def stream(self, device):
        s = self._streams.get(device)
        if s is None:
            s = self._streams[device] = torch.cuda.Stream(device=device)
        return s

    @contextlib.contextmanager
    def run(self, device, *keep):
        if not self.enabled or device.type != "cuda":
            yield
            return
        cur = torch.cuda.current_stream(device)
        s = self.stream(device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            yield
        self._keep.extend(t for t in keep if t is not None)
        self._pending.add(device)

    def join(self, device=None):
        devs = [device] if device is not None else list(self._pending)
        for d in devs:
            if d in self._pending:
                torch.cuda.current_stream(d).wait_stream(self.stream(d))
                self._pending.discard(d)
        if not self._pending:
            self._keep.clear()


SIDE = SideStream()


class DeferredReduces:
    """The training backward's deferred work, asked for call by call (include/charpt.h "deferred
    work"): the weight gradients into flat gradient slots leave their split-K slab reduce pending
    (cg_epilogue_t.flags CG_GEMM_DEFER_REDUCE) for the tail of the next persistent GEMM launch on the
    same stream (csrc/gemm_common.h RedJob: same summation order, same bits), and the LayerNorm /
    bias-gradient column-sum reduces into slots are queued (CG_DEFER) for one multi-job launch.  The
    queues are per stream in the library; this object only records which streams it queued work on
    and keeps the workspaces alive.  Leaving ``with DEFER:`` flushes those streams (before anything
    reads the gradients: the optimizer or the DP all-reduce); leaving it by an exception DISCARDS
    their queues instead (cg_discard_deferred) and records in ``aborted_adam`` how many deferred
    AdamW updates had already been taken by GEMM launches.  CHARPT_DEFER_SPLITK=0 turns it off (A/B)."""

    def __init__(self):
        self.enabled = os.environ.get("CHARPT_DEFER_SPLITK", "1") != "0"
        # the LayerNorm / bias-gradient column-sum reduces likewise: queued and launched as ONE
        # multi-job kernel at the flush -- on one hardware queue each was a ~5 us launch for ~1 us
        # of work (CHARPT_DEFER_PARTIALS=0: one launch each, for A/B)
        self.partials_on = os.environ.get("CHARPT_DEFER_PARTIALS", "1") != "0"
        self.active = False
        self.keep = []
        self.streams = {}        # (device index, cuda_stream handle) -> stream, every stream work was queued on
        self.aborted_adam = 0

    def __enter__(self):
        if self.enabled and torch.cuda.is_available():
            self.active = True
            self.aborted_adam = 0
        return self

    def note_stream(self):
        """The current stream will hold deferred work (flushed / discarded at exit)."""
        st = torch.cuda.current_stream()
        self.streams[(st.device.index, st.cuda_stream)] = st

    @contextlib.contextmanager
    def partials(self, *keep):
        """Yields whether the column-sum reduce calls made inside may be queued (their ``defer``
        argument): their outputs must be flat gradient slots, which nothing reads before DEFER
        closes; ``keep``: their partials, held until the flush."""
        if not (self.active and self.partials_on):
            yield False
            return
        self.note_stream()
        yield True
        self.keep.extend(t for t in keep if t is not None)

    def flush(self):
        """Launch everything pending on the streams this scope queued work on (each on its own stream)."""
        lib = L.load()
        for (dev, h) in list(self.streams):
            with torch.cuda.device(dev):   # (the library keys queues by the stream's own device too)
                L.check(lib.cg_flush_deferred(ctypes.c_void_p(h)), "flush_deferred")

    def discard(self):
        """Drop what is pending (a failed backward); returns the AdamW jobs launches had already taken."""
        lib = L.load()
        taken = 0
        for (dev, h) in list(self.streams):
            n = ctypes.c_int(0)
            with torch.cuda.device(dev):
                L.check(lib.cg_discard_deferred(ctypes.c_void_p(h), ctypes.byref(n)), "discard_deferred")
            taken += n.value
        return taken

    def __exit__(self, exc_type, *exc):
        if self.active:
            try:
                if exc_type is None:
                    self.flush()
                else:
                    self.aborted_adam = self.discard()
                if SIDE.enabled:   # the flush runs on the stream its reduces were enqueued on: join it
                    for d in {dv for dv, _ in self.streams} or {torch.cuda.current_device()}:
                        dev = torch.device("cuda", d)
                        torch.cuda.current_stream(dev).wait_stream(SIDE.stream(dev))
            finally:
                self.active = False
                self.keep.clear()
                self.streams.clear()
        return False


DEFER = DeferredReduces()


class EarlyAdam:
    """The training step's AdamW for the weight matrices, moved into the backward (engine.TrainStep,
    one rank): once a matrix's gradient is final and the backward reads its bf16 shadow no more --
    right after its dgrad, whose launch also finishes its split-K reduce -- its update is queued
    (cg_adamw_defer) for the free blocks of the next part-filling persistent GEMM launch (the N = 384
    dgrads and the projection weight gradient have 128-224 of 512 slots free), so it runs beside
    those GEMMs instead of in the optimizer's launch; optim.AdamW.step then updates only the rest
    (cg_adamw_segments).  Same element arithmetic, so the same bits (tests/test_gpu_train.py).  The
    step count is incremented when the backward starts.  Off with grad accumulation (beta 1), the
    side stream, DP, or CHARPT_EARLY_ADAM=0."""

    def __init__(self):
        self.enabled = os.environ.get("CHARPT_EARLY_ADAM", "1") != "0"
        self.opt = None

    def begin(self, opt):
        self.opt = None
        if not (self.enabled and torch.cuda.is_available() and DEFER.enabled and not SIDE.enabled):
            return False
        if not (hasattr(opt, "early_ok") and opt.early_ok()):
            return False
        opt.early_begin()
        self.opt = opt
        return True

    def region_done(self, region, g, beta):
        """``region``'s gradient ``g`` (written with ``beta``) is final; its shadow is read no more."""
        if self.opt is not None and g is not None and beta == 0.0 and g is region.slot:
            self.opt.early_region(region)

    def end(self):
        self.opt = None


EARLY = EarlyAdam()
# LayerNorm backward column-sum reduce on the side stream (CHARPT_LN_REDUCE_SIDE=0: in line, for A/B runs)
LN_REDUCE_SIDE = os.environ.get("CHARPT_LN_REDUCE_SIDE", "1") != "0"
# FFN b1 gradient fused into the ReLU-backward dgrad epilogue (CHARPT_FUSE_COLPART=0: separate colsum)
FUSE_COLPART = os.environ.get("CHARPT_FUSE_COLPART", "1") != "0"
# ReLU keep bits (1 bit per hidden unit) for the W2 dgrad instead of re-reading the bf16 h: set 0 for A/B
RELU_BITS = os.environ.get("CHARPT_RELU_BITS", "1") != "0"
# Measurement-only what-if switches (results are WRONG with any of them): CHARPT_WHATIF=skip_wgrad,
# skip_attn, skip_lnbwd drop those kernels from the step to see how much of the step time they hold.
WHATIF = set(filter(None, os.environ.get("CHARPT_WHATIF", "").split(",")))


def site_stream(call, site):
    """Dropout stream id (mirrors csrc/common.h dropout_stream and oracle.site_stream)."""
    return (int(call) << 8) | int(site)


# ---------------------------------------------------------------------------------------
# parameters as the kernels see them
# ---------------------------------------------------------------------------------------
class Region:
    """A contiguous fp32 weight region made of one or more nn.Parameters (e.g. all heads'
    query/key/value weights form one [3d, d] QKV region).

    master : fp32 tensor of the whole region (a view of the model's flat buffer when packed,
             else a temporary concatenation)
    slot   : matching view of the flat fp32 gradient buffer (None when not packed)
    shadow : matching view of the flat bf16 shadow (None when not packed)
    parts  : [(param, element_offset)] in region order
    """

    __slots__ = ("master", "slot", "shadow", "parts", "padded")

    def __init__(self, master, parts, slot=None, shadow=None, padded=None):
        self.master, self.parts, self.slot, self.shadow = master, parts, slot, shadow
        # (shadow, slot) views of a row-padded allocation (zero rows past the weight): the LM head's
        # K-padded GEMM operand / gradient destination (FlatStore pad_rows)
        self.padded = padded

    @staticmethod
    def of(*params):
        """Unpacked region built from loose parameters (standalone module use)."""
        parts, off = [], 0
        for p in params:
            parts.append((p, off))
            off += p.numel()
        if len(params) == 1:
            master = params[0].detach()
        else:
            master = torch.cat([p.detach().reshape(-1) for p in params]).view(-1, params[0].shape[-1])
        return Region(master, parts)

    @property
    def params(self):
        return [p for p, _ in self.parts]

    def needs_grad(self):
        return any(p.requires_grad for p, _ in self.parts)

    def operand(self, dtype):
        """The weight as a GEMM operand in ``dtype``."""
        if dtype == torch.float32:
            return self.master
        if self.shadow is not None:
            return self.shadow
        out = torch.empty(self.master.shape, dtype=torch.bfloat16, device=self.master.device)
        ops.cast_bf16(self.master.contiguous(), out)
        return out

    # -- gradient destination ----------------------------------------------------------
    def grad_target(self):
        """Decide where this region's gradient goes; returns (tensor, beta, finish) where
        ``finish()`` returns the per-param values the autograd Function must return."""
        if not self.needs_grad():
            return None, 0.0, lambda: [None] * len(self.parts)
        if self.slot is not None:
            grads = [p.grad for p, _ in self.parts]
            if all(g is None for g in grads):
                def assign():
                    with torch.no_grad():
                        for p, off in self.parts:
                            if p.requires_grad:
                                p.grad = self.slot.view(-1)[off:off + p.numel()].view(p.shape)
                    return [None] * len(self.parts)
                return self.slot, 0.0, assign
            if all(g is not None and g.data_ptr() == self.slot.view(-1)[off:].data_ptr() and g.shape == p.shape
                   for (p, off), g in zip(self.parts, grads)):
                return self.slot, 1.0, lambda: [None] * len(self.parts)
        tmp = torch.empty(self.master.shape, dtype=torch.float32, device=self.master.device)

        def ret():
            return [tmp.view(-1)[off:off + p.numel()].view(p.shape) if p.requires_grad else None
                    for p, off in self.parts]
        return tmp, 0.0, ret


def _flat2(t):
    return t.reshape(-1, t.shape[-1])


def _is_bf16(dt):
    return dt == torch.bfloat16


# ---------------------------------------------------------------------------------------
# GEMM helpers (all three nn.Linear products)
# ---------------------------------------------------------------------------------------
def linear_fwd(x2, w, out, epi="store", bias=None, resid=None, aux=None, dropout_p=0.0, seed=0, rng_call=None,
               site=0):
    """out[M,N] = epi(x2[M,K] @ w[N,K]^T)"""
    M, K = x2.shape
    N = w.shape[0]
    ops.gemm(x2, w, out, _is_bf16(x2.dtype), False, False, M, N, K, K, K, out.stride(0), EPI[epi], bias, resid,
             resid.stride(0) if resid is not None else 0, aux, aux.stride(0) if aux is not None else 0,
             float(dropout_p), int(seed), rng_call, int(site), 0.0, 1, None)
    return out


# CHARPT_GEMM_LN=1: the residual GEMMs with the next LayerNorm in their epilogue (cg_gemm_resid_
# layernorm).  Off by default: bitwise equal, the kernel alone is 3 us faster than GEMM + LayerNorm
# at the C2 projection and 0.6 us at FFN2, but the C2 step measured 2.8446 vs 2.8410 ms with ln2 and
# ln_f fused (and 2.870 vs 2.811 with every ln1 too, which loses the LayerNorm + keep-bit launch):
# profiles/r5_gemm_ln_ab.txt
GEMM_LN = os.environ.get("CHARPT_GEMM_LN", "0") == "1"


def linear_fwd_resid_ln(x2, w, out, bias, resid, next_ln, act, dropout_p=0.0, seed=0, rng_call=None, site=0):
    """out[M,N] = resid + dropout(x2 @ w^T + bias) (fp32) and, when the kernel takes this shape
    (cg_gemm_resid_layernorm: N = 384, bf16), the LayerNorm that reads out next (next_ln = (weight
    Region, bias Region, eps): the same block's ln2 after the projection, the next block's ln1 or ln_f
    after the FFN) in the same launch.  Returns the handoff (key, y, mean, rstd) that pre_ln() gives
    the consumer, or None after the plain GEMM."""
    M, K = x2.shape
    N = w.shape[0]
    if next_ln is None or not GEMM_LN or act != torch.bfloat16 or not ops.gemm_resid_layernorm_supported(M, N, K):
        linear_fwd(x2, w, out, "bias_drop_resid" if dropout_p > 0 else "bias_resid", bias=bias, resid=resid,
                   dropout_p=dropout_p, seed=seed, rng_call=rng_call, site=site)
        return None
    lw, lb, eps = next_ln
    y = torch.empty((M, N), dtype=act, device=x2.device)
    mean = torch.empty(M, dtype=torch.float32, device=x2.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x2.device)
    ops.gemm_resid_layernorm(x2, w, out, M, N, K, x2.stride(0), w.stride(0), out.stride(0), bias, resid,
                             resid.stride(0), float(dropout_p), int(seed), rng_call, int(site), lw.master, lb.master,
                             y, mean, rstd, float(eps))
    return ((lw.master.data_ptr(), lb.master.data_ptr(), act, float(eps)), y, mean, rstd)


def pre_ln(x, ln_w, ln_b, act, eps=1e-5):
    """(y, mean, rstd) of LayerNorm(x; ln_w, ln_b) when the GEMM that wrote x computed them
    (linear_fwd_resid_ln's handoff on the tensor) for exactly this LayerNorm, else None."""
    h = getattr(x, "_charpt_ln", None)
    if h is None or h[0] != (ln_w.master.data_ptr(), ln_b.master.data_ptr(), act, float(eps)):
        return None
    return h[1], h[2], h[3]


def linear_dgrad(dy2, w, out, epi="store", aux=None):
    """out[M,K] = epi(dy2[M,N] @ w[N,K])"""
    M, N = dy2.shape
    K = w.shape[1]
    ops.gemm(dy2, w, out, _is_bf16(dy2.dtype), False, True, M, K, N, N, K, out.stride(0), EPI[epi], None, None, 0,
             aux, aux.stride(0) if aux is not None else 0, 0.0, 0, None, 0, 0.0, 1, None)
    return out


_SLOTS = {}


def _gemm_slots():
    """Resident blocks of the persistent bf16 GEMM (csrc/gemm_pk.hip: 2 per CU)."""
    dev = torch.cuda.current_device() if torch.cuda.is_available() else -1
    if dev not in _SLOTS:
        _SLOTS[dev] = 2 * (torch.cuda.get_device_properties(dev).multi_processor_count if dev >= 0 else 256)
    return _SLOTS[dev]


def _wgrad_split(M, N, K, fast):
    """Split-K factor of a weight-gradient GEMM (K = tokens).  bf16 path: the persistent kernel
    hands each resident block ceil(items / slots) items of ceil(K-tiles / split) reduction depth
    (any split: the last one is shorter), and every split adds an fp32 slab to write and reduce, so
    minimise   ceil(tiles * split / slots) * ceil(K-tiles / split) * (1 + split / 50)
    over splits 1..32 -- e.g. 14 / 16 / 14 / 32 at C2 and 7 / 4 / 7 / 14 at C4 (FFN2, QKV, FFN1, proj),
    within 3 % of the measured best of each (tools/gemm_scan2.py, profiles/r2_gemm_scan_wgrad_splits.txt;
    the power-of-two splits of round 1 were up to 25 % slower)."""
    if fast:
        tiles, slots = -(-M // 128) * -(-N // 128), _gemm_slots()
        nkt = K // 64
        best, best_cost = 1, None
        for split in range(1, 33):
            per = -(-nkt // split)
            if (split - 1) * per >= nkt or per < 4:   # an empty last split / too little depth
                continue
            cost = -(-tiles * split // slots) * per * (1 + split / 50)
            if best_cost is None or cost < best_cost:
                best, best_cost = split, cost
        return best
    tiles = -(-M // 64) * -(-N // 64)
    split = 1
    while tiles * split * 2 <= 1024 and split < 32 and K % (64 * split * 2) == 0 and K // (split * 2) >= 256:
        split *= 2
    return split


# The training path's weight gradients (flat gradient slots) take their split-K partial sums through
# bf16 slabs (per call: cg_epilogue_t.flags CG_GEMM_SLAB_BF16 -- half the slab bytes written and read back; each per-split
# partial rounded once to bf16, the sum over splits in fp32 -- torch's bf16 path rounds the whole
# gradient to bf16).  Temporaries (charpt::linear's backward) keep fp32 slabs.  CHARPT_SLAB_BF16=0: A/B.
SLAB_BF16 = os.environ.get("CHARPT_SLAB_BF16", "1") != "0"


def linear_wgrad(dy2, x2, out, beta, into_slot=False):
    """out[N,K] (+)= dy2[M,N]^T @ x2[M,K]   (fp32, deterministic split-K).

    into_slot: ``out`` is a region's flat gradient slot, which nothing reads before DEFER closes,
    so inside ``with DEFER:`` its split-K reduce may stay pending past this call.  Any other
    output (a temporary, a tensor handed to autograd) gets its pending reduces flushed right after
    the GEMM, so it is complete when this returns.  Slot outputs use bf16 split-K slabs (SLAB_BF16)."""
    if "skip_wgrad" in WHATIF:
        return out
    M, N = dy2.shape
    K = x2.shape[1]
    fast = _is_bf16(dy2.dtype) and N % 128 == 0 and K % 128 == 0 and M % 64 == 0
    split = _wgrad_split(N, K, M, fast)
    ws = None
    defer = DEFER.active and into_slot and split > 1
    if split > 1:
        ws = torch.empty(ops.gemm_workspace(N, K, split) // 4, dtype=torch.float32, device=dy2.device)
        if defer:
            # its reduce may run after this call returns
            DEFER.keep.extend((ws, dy2, x2))
            DEFER.note_stream()
    flags = (L.GEMM_SLAB_BF16 if SLAB_BF16 and into_slot and split > 1 else 0) | (L.GEMM_DEFER_REDUCE if defer else 0)
    ops.gemm(dy2, x2, out, _is_bf16(dy2.dtype), True, True, N, K, M, N, K, out.stride(0), L.EPI_STORE, None,
             None, 0, None, 0, 0.0, 0, None, 0, float(beta), split, ws, flags)
    return out


def _colpart_ok(dy2, w, aux, out_ld):
    """Whether cg_gemm's dispatch can write the ReLU-backward dgrad out[M,F] = relu_bwd(dy2 @ w)
    together with its column partials (the b1 gradient) -- asked from the library itself
    (cg_gemm_colpart_supported: same predicate as the dispatch, current tuning knobs included)."""
    if not (FUSE_COLPART and _is_bf16(dy2.dtype) and _is_bf16(aux.dtype) and dy2.is_cuda):
        return False
    if dy2.stride(1) != 1 or w.stride(1) != 1 or aux.stride(1) != 1 or aux.stride(0) % 8:
        return False
    if any(t.data_ptr() % 16 for t in (dy2, w, aux)):
        return False
    M, K = dy2.shape
    F = w.shape[1]
    return bool(L.load().cg_gemm_colpart_supported(0, 1, M, F, K, dy2.stride(0), w.stride(0), out_ld))


def _relu_bits_ok(a, w1, w2, F):
    """Whether the FeedForward can keep ReLU keep bits instead of reading h back in its W2 dgrad:
    both its W1 forward (writes them) and W2 dgrad (reads them) products must take a persistent
    kernel (cg_gemm_relu_bits_supported, asked from the library itself)."""
    if not (RELU_BITS and _is_bf16(a.dtype) and a.is_cuda and a.stride(1) == 1):
        return False
    M, C = a.shape
    lib = L.load()
    return bool(lib.cg_gemm_relu_bits_supported(0, 0, M, F, C, a.stride(0), w1.stride(0), F) and
                lib.cg_gemm_relu_bits_supported(0, 1, M, F, C, C, w2.stride(0), F))


def colsum_into(x2, out, beta):
    ws = torch.empty(ops.colsum_workspace(x2.shape[0], x2.shape[1]) // 4 + 1, dtype=torch.float32, device=x2.device)
    ops.colsum(x2, out, bool(beta), ws)


def layernorm(x2, w, b, out_dtype, eps=1e-5):
    rows, C = x2.shape
    y = torch.empty((rows, C), dtype=out_dtype, device=x2.device)
    mean = torch.empty(rows, dtype=torch.float32, device=x2.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x2.device)
    ops.layernorm_fwd(x2, w, b, y, mean, rstd, float(eps))
    return y, mean, rstd


# CHARPT_LN_MASK=0: the attention keep bits in their own launch (A/B of layernorm_attn_mask)
LN_MASK = os.environ.get("CHARPT_LN_MASK", "1") != "0"


def layernorm_attn_mask(x2, w, b, out_dtype, B, H, T, p, seed, rng_call, site, eps=1e-5):
    """layernorm() and the dropout keep bits of the attention it feeds (cg_attn_dropmask) in one
    launch: the Philox work runs beside the LayerNorm's memory traffic.  Returns (y, mean, rstd,
    mask); same values as the two launches."""
    rows, C = x2.shape
    dev = x2.device
    y = torch.empty((rows, C), dtype=out_dtype, device=dev)
    mean = torch.empty(rows, dtype=torch.float32, device=dev)
    rstd = torch.empty(rows, dtype=torch.float32, device=dev)
    mask = torch.empty(ops.attn_mask_bytes(B, H, T) // 8, dtype=torch.int64, device=dev)
    ops.layernorm_fwd_attn_dropmask(x2, w, b, y, mean, rstd, float(eps), B, H, T, float(p), int(seed), rng_call,
                                    int(site), mask)
    return y, mean, rstd, mask


class GradLink:
    """What a sublayer's backward wants for its incoming residual-stream gradient (GPT1.py:163-164:
    the gradient of x + f(x) arrives at f as-is): a bf16 copy with the sublayer's output dropout
    applied (FeedForward, GPT1.py:146) or plain (the attention projection), plus that tensor's
    column sums as the sublayer's output-bias gradient.  Created in the sublayer's forward and
    attached to its output tensor; the NEXT sublayer's forward picks it up from its input and its
    LayerNorm backward -- the kernel that produces the gradient -- fills it (cg_layernorm_bwd_ex),
    so the consumer skips its dropout / cast and column-sum passes.  The consumer uses the copy only
    if its gradient is the exact buffer the producer wrote (data_ptr check), else recomputes."""
    __slots__ = ("p", "seed", "rng_call", "site", "bias", "act", "lp", "dx_ptr", "bias_done")

    def __init__(self, p, seed, rng_call, site, bias, act):
        self.p, self.seed, self.rng_call, self.site, self.bias, self.act = p, seed, rng_call, site, bias, act
        self.lp, self.dx_ptr, self.bias_done = None, None, False

    def take(self, d32):
        ok = self.lp is not None and self.dx_ptr == d32.data_ptr()
        lp, done = (self.lp, self.bias_done) if ok else (None, False)
        self.lp, self.dx_ptr, self.bias_done = None, None, False
        return lp, done


def _link_of(x):
    return getattr(x, "_charpt_link", None)


def layernorm_bwd(dy2, x2, w_reg, b_reg, mean, rstd, dres=None, want_lp=False, link=None):
    """dx (fp32) = dres + LN'(dy); LN weight/bias grads into their regions.  ``link``: the
    consumer of dx (GradLink) -- its bf16 (dropout-applied) copy and bias column sums are produced
    in the same kernel."""
    rows, C = x2.shape
    dev = x2.device
    dx = torch.empty((rows, C), dtype=torch.float32, device=dev)
    use_link = link is not None and link.act == torch.bfloat16
    lp = torch.empty((rows, C), dtype=torch.bfloat16, device=dev) if (want_lp or use_link) else None
    gw, bw, fw = w_reg.grad_target()
    gb, bb, fb = b_reg.grad_target()
    gcs, bcs, fcs = None, 0.0, None
    if use_link and link.bias is not None and link.bias.slot is not None:
        gcs, bcs, fcs = link.bias.grad_target()
    ws = torch.empty(ops.layernorm_bwd_workspace(rows, C) // 4 + 1, dtype=torch.float32, device=dev)
    p = float(link.p) if use_link else 0.0
    seed, rng, site = (int(link.seed) if use_link else 0), (link.rng_call if (use_link and p > 0) else None), \
        (int(link.site) if use_link else 0)
    # the column-sum reduce (LN weight/bias grads, the consumer's bias grad) only feeds the optimizer:
    # when every target is a flat gradient slot (read after SIDE.join) it runs on the side stream,
    # off the dgrad chain; otherwise (tensors handed back to autograd) in line
    slots_only = dev.type == "cuda" and (gw is not None or gb is not None or gcs is not None) and \
        (gw is None or gw is w_reg.slot) and (gb is None or gb is b_reg.slot) and \
        (gcs is None or gcs is link.bias.slot)
    side = LN_REDUCE_SIDE and SIDE.enabled and slots_only
    if "skip_lnbwd" in WHATIF:
        pass
    elif side:
        ops.layernorm_bwd_rows(dy2, x2, w_reg.master, mean, rstd, dres, dx, lp, ws, gcs is not None, p, seed, rng,
                               site)
        with SIDE.run(dev, ws):
            ops.layernorm_bwd_reduce(ws, rows, C, gcs is not None, gw, gb, gcs, bool(bw or bb), bool(bcs))
    elif slots_only and DEFER.active and DEFER.partials_on:
        # the reduce joins the backward's one multi-job launch at the DEFER flush
        ops.layernorm_bwd_rows(dy2, x2, w_reg.master, mean, rstd, dres, dx, lp, ws, gcs is not None, p, seed, rng,
                               site)
        with DEFER.partials(ws) as queued:
            ops.layernorm_bwd_reduce(ws, rows, C, gcs is not None, gw, gb, gcs, bool(bw or bb), bool(bcs), queued)
    else:
        ops.layernorm_bwd(dy2, x2, w_reg.master, mean, rstd, dres, dx, lp, gw, gb, bool(bw or bb), ws, gcs, bool(bcs),
                          p, seed, rng, site)
    if use_link:
        link.lp, link.dx_ptr, link.bias_done = lp, dx.data_ptr(), gcs is not None
        if fcs is not None:
            fcs()
    return dx, (lp if want_lp and not use_link else None), fw() + fb()


def attention_fwd(qkv, B, T, H, D, out, scale, p, seed, rng_call, site, premask=None):
    """Returns (lse, mask): mask holds the dropout keep bits of the MFMA path (None when p == 0
    or when the generic kernels, which regenerate Philox in place, are used).  ``premask`` =
    (mask, event): keep bits already generated -- on the side stream (the main stream waits on the
    event instead of generating them) or, event None, earlier on this stream (layernorm_attn_mask)."""
    d = H * D
    lse = torch.empty((B, H, T), dtype=torch.float32, device=qkv.device)
    mask, ready = None, False
    if p > 0 and premask is not None:
        mask, ev = premask
        if ev is not None:
            torch.cuda.current_stream(qkv.device).wait_event(ev)
        ready = True
    elif p > 0 and T % 16 == 0:
        mask = torch.empty(ops.attn_mask_bytes(B, H, T) // 8, dtype=torch.int64, device=qkv.device)
    if "skip_attn" in WHATIF:
        return lse, mask
    ops.attn_fwd(qkv, B, T, H, D, 0, d, 2 * d, qkv.stride(0), out, out.stride(0), lse, float(scale), float(p),
                 int(seed), rng_call, int(site), mask, ready)
    return lse, mask


def premask_ok(act, T, D):
    """The bf16 MFMA attention path (csrc fast_attn_ok) reads precomputed keep bits."""
    return act == torch.bfloat16 and D == 64 and T % 64 == 0


# CHARPT_ROWDOT=0: the attention backward computes delta = rowsum(dO * O) itself (A/B of the proj
# dgrad's CG_EPI_STORE_ROWDOT epilogue)
ROWDOT = os.environ.get("CHARPT_ROWDOT", "1") != "0"


def rowdot_ok(dy2, w, o, T, D):
    """Whether the attention-output gradient dO = dy2 @ w can come out of cg_gemm together with the
    attention backward's delta (CG_EPI_STORE_ROWDOT) -- only where the sequence-resident attention
    backward (T <= 256, head_size 64) reads it; asked from the library (cg_gemm_rowdot_supported)."""
    if not (ROWDOT and D == 64 and T <= 256 and T % 64 == 0 and _is_bf16(dy2.dtype) and _is_bf16(o.dtype)
            and dy2.is_cuda):
        return False
    if dy2.stride(1) != 1 or w.stride(1) != 1 or o.stride(1) != 1 or o.stride(0) % 8:
        return False
    if any(t.data_ptr() % 16 for t in (dy2, w, o)):
        return False
    M, K = dy2.shape
    N = w.shape[1]
    return M % T == 0 and ops.gemm_rowdot_supported(M, N, K, dy2.stride(0), w.stride(0), N)


def attention_bwd(qkv, B, T, H, D, o, do, lse, scale, p, seed, rng_call, site, mask=None, delta=None):
    d = H * D
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(ops.attn_bwd_workspace(B, T, H, D) // 4 + 1, dtype=torch.float32, device=qkv.device)
    if "skip_attn" in WHATIF:
        return dqkv
    ops.attn_bwd(qkv, B, T, H, D, 0, d, 2 * d, qkv.stride(0), o, o.stride(0), do, do.stride(0), lse, dqkv,
                 dqkv.stride(0), float(scale), float(p), int(seed), rng_call, int(site), mask, ws, delta)
    return dqkv


def to_act(x2, dtype):
    """fp32 activation -> GEMM operand dtype (bf16 copy through the cast kernel)."""
    if x2.dtype == dtype:
        return x2
    out = torch.empty(x2.shape, dtype=dtype, device=x2.device)
    ops.cast_bf16(x2.contiguous(), out)
    return out


def _regions_params(regs):
    out = []
    for r in regs:
        out += r.params
    return out


class LayerCtx:
    """Per-call context for a sublayer: geometry, dropout and dtype."""
    __slots__ = ("n_head", "head_size", "scale", "p", "seed", "rng_call", "site", "act", "premask", "next_ln")

    def __init__(self, n_head, head_size, scale, p, seed, rng_call, site, act, premask=None, next_ln=None):
        self.n_head, self.head_size, self.scale, self.p = n_head, head_size, scale, p
        self.seed, self.rng_call, self.site, self.act = seed, rng_call, site, act
        self.premask = premask   # (mask tensor, event) from BigramLanguageModel._launch_premasks
        self.next_ln = next_ln   # (weight Region, bias Region, eps) of the LayerNorm that reads the output


# ---------------------------------------------------------------------------------------
# fused training nodes
# ---------------------------------------------------------------------------------------
class EmbeddingFn(torch.autograd.Function):
    """x = wte[idx] + wpe[arange(T)]  (GPT1.py:179-181)"""

    @staticmethod
    def forward(ctx, idx, wte_reg, wpe_reg, *params):
        B, T = idx.shape
        V, C = wte_reg.master.shape
        x = torch.empty((B, T, C), dtype=torch.float32, device=idx.device)
        ops.embed_fwd(idx, wte_reg.master, wpe_reg.master, x)
        ctx.save_for_backward(idx)
        ctx.regs = (wte_reg, wpe_reg)
        return x

    @staticmethod
    def backward(ctx, dx):
        (idx,) = ctx.saved_tensors
        wte_reg, wpe_reg = ctx.regs
        B, T = idx.shape
        V, C = wte_reg.master.shape
        gt, bt, ft = wte_reg.grad_target()
        gp, bp, fp = wpe_reg.grad_target()
        if gt is not None or gp is not None:
            ws = torch.empty(ops.embed_bwd_workspace(B, T, C, V) // 4 + 1, dtype=torch.float32, device=dx.device)
            if bt != bp and gt is not None and gp is not None:
                ops.embed_bwd(idx, dx.contiguous(), gt, None, bool(bt), ws)
                ops.embed_bwd(idx, dx.contiguous(), None, gp[:T], bool(bp), ws)
            else:
                ops.embed_bwd(idx, dx.contiguous(), gt, gp[:T] if gp is not None else None, bool(bt or bp), ws)
            if gp is not None and not bp and T < gp.shape[0]:
                gp[T:].zero_()  # positions beyond T get no gradient (overwrite mode)
        SIDE.join(dx.device)   # last node of the model backward: every gradient is final after this
        return (None, None, None, *ft(), *fp())


class AttnSublayerFn(torch.autograd.Function):
    """x + proj(MultiHeadAttention(ln1(x)))   (GPT1.py:163, 134-136, 109-123)."""

    @staticmethod
    def forward(ctx, x, lc, ln_w, ln_b, qkv_w, proj_w, proj_b, *params):
        B, T, C = x.shape
        x2 = x.reshape(B * T, C)
        act = lc.act
        pm = lc.premask
        pre = pre_ln(x, ln_w, ln_b, act)
        if pre is not None:   # ln1 came with x from the previous FFN's GEMM (the keep bits: attention_fwd)
            a, mean, rstd = pre
        elif pm is None and lc.p > 0 and LN_MASK and premask_ok(act, T, lc.head_size):
            a, mean, rstd, mask = layernorm_attn_mask(x2, ln_w.master, ln_b.master, act, B, lc.n_head, T, lc.p,
                                                      lc.seed, lc.rng_call, lc.site)
            pm = (mask, None)
        else:
            a, mean, rstd = layernorm(x2, ln_w.master, ln_b.master, act)
        qkv = torch.empty((B * T, 3 * C), dtype=act, device=x.device)
        linear_fwd(a, qkv_w.operand(act), qkv)
        o = torch.empty((B * T, C), dtype=act, device=x.device)
        lse, ctx.mask = attention_fwd(qkv, B, T, lc.n_head, lc.head_size, o, lc.scale, lc.p, lc.seed, lc.rng_call,
                                      lc.site, pm)
        out = torch.empty((B * T, C), dtype=torch.float32, device=x.device)
        ln_next = linear_fwd_resid_ln(o, proj_w.operand(act), out, proj_b.master, x2, lc.next_ln, act)
        ctx.save_for_backward(x2, a, mean, rstd, qkv, o, lse)
        ctx.lc, ctx.regs, ctx.shape = lc, (ln_w, ln_b, qkv_w, proj_w, proj_b), (B, T, C)
        ctx.in_link = _link_of(x)
        ctx.link = GradLink(0.0, 0, None, 0, proj_b, act)
        out_v = out.view(B, T, C)
        out_v._charpt_link = ctx.link
        if ln_next is not None:
            out_v._charpt_ln = ln_next
        return out_v

    @staticmethod
    def backward(ctx, dout):
        x2, a, mean, rstd, qkv, o, lse = ctx.saved_tensors
        lc = ctx.lc
        ln_w, ln_b, qkv_w, proj_w, proj_b = ctx.regs
        B, T, C = ctx.shape
        act = lc.act
        d32 = dout.reshape(B * T, C).contiguous()
        dy, bias_done = ctx.link.take(d32)
        if dy is None:
            dy = to_act(d32, act)
        dev = x2.device
        # proj: dW = dy^T o, db = colsum(dy) (side stream, unless fused upstream), do = dy W
        g_pw, beta_pw, f_pw = proj_w.grad_target()
        g_pb, beta_pb, f_pb = proj_b.grad_target()
        with SIDE.run(dev, dy, o):
            if g_pw is not None:
                linear_wgrad(dy, o, g_pw, beta_pw, g_pw is proj_w.slot)
            if g_pb is not None and not bias_done:
                colsum_into(dy, g_pb, beta_pb)
        do = torch.empty((B * T, C), dtype=act, device=x2.device)
        wp = proj_w.operand(act)
        delta = None
        if rowdot_ok(dy, wp, o, T, lc.head_size):
            # dO and the attention backward's delta = rowsum(dO * O) from one epilogue (the attention
            # kernel then loads neither O nor computes the row dots)
            delta = torch.empty((B, lc.n_head, T), dtype=torch.float32, device=dev)
            ops.gemm_store_rowdot(dy, wp, do, B * T, C, C, dy.stride(0), wp.stride(0), do.stride(0), o, o.stride(0),
                                  T, delta)
        else:
            linear_dgrad(dy, wp, do)
        EARLY.region_done(proj_w, g_pw, beta_pw)   # the projection weight's last read this step
        dqkv = attention_bwd(qkv, B, T, lc.n_head, lc.head_size, o, do, lse, lc.scale, lc.p, lc.seed, lc.rng_call,
                             lc.site, ctx.mask, delta)
        g, beta, f_qkv = qkv_w.grad_target()
        if g is not None:
            with SIDE.run(dev, dqkv, a):
                linear_wgrad(dqkv, a, g, beta, g is qkv_w.slot)
        da = torch.empty((B * T, C), dtype=act, device=x2.device)
        linear_dgrad(dqkv, qkv_w.operand(act), da)
        EARLY.region_done(qkv_w, g, beta)
        dx, _, f_ln = layernorm_bwd(da, x2, ln_w, ln_b, mean, rstd, dres=d32, link=ctx.in_link)
        return (dx.view(B, T, C), None, None, None, None, None, None, *f_ln, *f_qkv(), *f_pw(), *f_pb())


# generate()'s fp32 window blocks run the FeedForward as one fused launch (ops.ffn_fwd_f32: the hidden
# activations never reach HBM); CHARPT_FFN_FUSED=0 keeps the two GEMMs (A/B)
FFN_FUSED = os.environ.get("CHARPT_FFN_FUSED", "1") == "1"
FFN_LN = os.environ.get("CHARPT_FFN_LN", "1") == "1"   # ln2 inside that launch (0: its own launch)


def ffn_sublayer_infer(x, lc, ln_w, ln_b, w1, b1, w2, b2):
    """FFNSublayerFn.forward for fp32 inference without autograd (no dropout, nothing saved):
    x + W2 relu(W1 ln2(x) + b1) + b2 in one launch, ln2 included -- the bits of the LayerNorm + two-GEMM path
    (tests/test_gpu_ops.py::test_ffn_f32_fused_matches_two_gemms).  None where it does not apply
    (bf16, dropout, fewer than 2049 rows -- the small-M GEMMs are faster there -- or a shape the
    kernel does not take)."""
    if not FFN_FUSED or lc.act != torch.float32 or lc.p > 0:
        return None
    B, T, C = x.shape
    M, H = B * T, w1.master.shape[0]
    if M <= 2048 or not ops.ffn_fwd_f32_supported(M, C, H):
        return None
    x2 = x.reshape(M, C)
    out = torch.empty((M, C), dtype=torch.float32, device=x.device)
    pre = pre_ln(x, ln_w, ln_b, lc.act)
    lw, lb = ln_w.master, ln_b.master
    if FFN_LN and pre is None and ((lw.data_ptr() | lb.data_ptr() | x2.data_ptr()) & 7) == 0:
        # ln2 inside the launch: k_ln_fwd's narrow-row body, cg_layernorm_fwd's choice for these pointers
        ops.ffn_fwd_f32(x2, lw, lb, 1e-5, w1.operand(lc.act), b1.master, w2.operand(lc.act), b2.master, x2, out)
    else:
        a = pre[0] if pre is not None else layernorm(x2, lw, lb, lc.act)[0]
        ops.ffn_fwd_f32(a, None, None, 0.0, w1.operand(lc.act), b1.master, w2.operand(lc.act), b2.master, x2, out)
    return out.view(B, T, C)


# generate()'s fp32 window blocks run the attention sublayer's two Linears as row-resident launches
# (ops.linear_rows_f32: ln1 inside the QKV launch, the residual inside the projection's);
# CHARPT_ATTN_ROWS=0 keeps the LayerNorm + GEMM launches (A/B)
ATTN_ROWS = os.environ.get("CHARPT_ATTN_ROWS", "1") == "1"


def attn_sublayer_infer(x, lc, ln_w, ln_b, qkv_w, proj_w, proj_b):
    """AttnSublayerFn.forward for fp32 inference without autograd (no dropout, nothing saved):
    ln1 + the QKV product in one launch, the attention, the projection + residual in one launch --
    the bits of the LayerNorm + GEMM path (tests/test_gpu_model.py::test_fp32_eval_forward_fused_*).
    None where it does not apply (bf16, dropout, fewer than 2049 rows, a shape the kernel does not
    take)."""
    if not ATTN_ROWS or lc.act != torch.float32 or lc.p > 0 or lc.premask is not None:
        return None
    B, T, C = x.shape
    M = B * T
    if M <= 2048 or not ops.linear_rows_f32_supported(M, 3 * C, C) or not ops.linear_rows_f32_supported(M, C, C):
        return None
    act = lc.act
    x2 = x.reshape(M, C)
    lw, lb = ln_w.master, ln_b.master
    qkv = torch.empty((M, 3 * C), dtype=act, device=x.device)
    pre = pre_ln(x, ln_w, ln_b, act)
    if FFN_LN and pre is None and ((lw.data_ptr() | lb.data_ptr() | x2.data_ptr()) & 7) == 0:
        ops.linear_rows_f32(x2, lw, lb, 1e-5, qkv_w.operand(act), None, None, qkv)   # ln1 inside
    else:
        a = pre[0] if pre is not None else layernorm(x2, lw, lb, act)[0]
        ops.linear_rows_f32(a, None, None, 0.0, qkv_w.operand(act), None, None, qkv)
    o = torch.empty((M, C), dtype=act, device=x.device)
    attention_fwd(qkv, B, T, lc.n_head, lc.head_size, o, lc.scale, lc.p, lc.seed, lc.rng_call, lc.site, None)
    out = torch.empty((M, C), dtype=torch.float32, device=x.device)
    ops.linear_rows_f32(o, None, None, 0.0, proj_w.operand(act), proj_b.master, x2, out)
    return out.view(B, T, C)


class FFNSublayerFn(torch.autograd.Function):
    """x + Dropout(W2 relu(W1 ln2(x) + b1) + b2)   (GPT1.py:164, 142-147)."""

    @staticmethod
    def forward(ctx, x, lc, ln_w, ln_b, w1, b1, w2, b2, *params):
        B, T, C = x.shape
        x2 = x.reshape(B * T, C)
        act = lc.act
        pre = pre_ln(x, ln_w, ln_b, act)   # ln2 from the projection GEMM's epilogue
        a, mean, rstd = pre if pre is not None else layernorm(x2, ln_w.master, ln_b.master, act)
        F4 = w1.master.shape[0]
        h = torch.empty((B * T, F4), dtype=act, device=x.device)
        bits = None
        if _relu_bits_ok(a, w1.operand(act), w2.operand(act), F4):
            # the W2 dgrad's ReLU mask as 1 bit per element (h itself stays for the W2 weight gradient)
            bits = torch.empty((B * T, F4 // 32), dtype=torch.int32, device=x.device)
            w1op = w1.operand(act)
            ops.gemm_bias_relu_bits(a, w1op, h, B * T, F4, C, a.stride(0), w1op.stride(0), h.stride(0), b1.master,
                                    bits, bits.stride(0))
        else:
            linear_fwd(a, w1.operand(act), h, "bias_relu", bias=b1.master)
        out = torch.empty((B * T, C), dtype=torch.float32, device=x.device)
        ln_next = linear_fwd_resid_ln(h, w2.operand(act), out, b2.master, x2, lc.next_ln, act, dropout_p=lc.p,
                                      seed=lc.seed, rng_call=lc.rng_call, site=lc.site)
        ctx.save_for_backward(x2, a, mean, rstd, h, bits)
        ctx.lc, ctx.regs, ctx.shape = lc, (ln_w, ln_b, w1, b1, w2, b2), (B, T, C)
        ctx.in_link = _link_of(x)
        ctx.link = GradLink(lc.p, lc.seed, lc.rng_call, lc.site, b2, act)
        out_v = out.view(B, T, C)
        out_v._charpt_link = ctx.link
        if ln_next is not None:
            out_v._charpt_ln = ln_next
        return out_v

    @staticmethod
    def backward(ctx, dout):
        x2, a, mean, rstd, h, bits = ctx.saved_tensors
        lc = ctx.lc
        ln_w, ln_b, w1, b1, w2, b2 = ctx.regs
        B, T, C = ctx.shape
        act = lc.act
        d32 = dout.reshape(B * T, C).contiguous()
        dz2, bias_done = ctx.link.take(d32)
        if dz2 is None:
            dz2 = torch.empty((B * T, C), dtype=act, device=x2.device)
            ops.dropout_apply(d32, dz2, float(lc.p), int(lc.seed), lc.rng_call, int(lc.site))
        dev = x2.device
        g_w2, beta_w2, f_w2 = w2.grad_target()
        g_b2, beta_b2, f_b2 = b2.grad_target()
        with SIDE.run(dev, dz2, h):
            if g_w2 is not None:
                linear_wgrad(dz2, h, g_w2, beta_w2, g_w2 is w2.slot)
            if g_b2 is not None and not bias_done:
                colsum_into(dz2, g_b2, beta_b2)
        dz1 = torch.empty_like(h)
        g_w1, beta_w1, f_w1 = w1.grad_target()
        g_b1, beta_b1, f_b1 = b1.grad_target()
        part = None
        if g_b1 is not None and _colpart_ok(dz2, w2.operand(act), h, dz1.stride(0)):
            # b1's gradient (column sums of dz1) fused into the ReLU-backward dgrad's epilogue as
            # per-64-row partials; only their fold runs on the side stream
            M, F4 = h.shape
            part = torch.empty((M // 64, F4), dtype=torch.float32, device=dev)
            wt = w2.operand(act)
            mk = h if bits is None else bits
            ops.gemm_relu_bwd_colpart(dz2, wt, dz1, M, F4, dz2.shape[1], dz2.stride(0), wt.stride(0), dz1.stride(0),
                                      mk, mk.stride(0), part)
        else:
            linear_dgrad(dz2, w2.operand(act), dz1, "relu_bwd", aux=h if bits is None else bits)
        EARLY.region_done(w2, g_w2, beta_w2)   # W2's gradient is final (its reduce went with this dgrad)
        with SIDE.run(dev, dz1, a, part):
            if g_w1 is not None:
                linear_wgrad(dz1, a, g_w1, beta_w1, g_w1 is w1.slot)
            if g_b1 is not None:
                if part is not None:
                    with DEFER.partials(part) if g_b1 is b1.slot else contextlib.nullcontext(False) as queued:
                        ops.reduce_rows(part, part.shape[0], part.shape[1], g_b1, bool(beta_b1), queued)
                else:
                    colsum_into(dz1, g_b1, beta_b1)
        da = torch.empty((B * T, C), dtype=act, device=x2.device)
        linear_dgrad(dz1, w1.operand(act), da)
        EARLY.region_done(w1, g_w1, beta_w1)
        dx, _, f_ln = layernorm_bwd(da, x2, ln_w, ln_b, mean, rstd, dres=d32, link=ctx.in_link)
        return (dx.view(B, T, C), None, None, None, None, None, None, None, *f_ln, *f_w1(), *f_b1(), *f_w2(),
                *f_b2())


class HeadLossFn(torch.autograd.Function):
    """ln_f -> lm_head -> (optional) mean cross entropy   (GPT1.py:183-192)."""

    @staticmethod
    def forward(ctx, x, targets, act, ln_w, ln_b, lm_w, lm_b, *params):
        B, T, C = x.shape
        M = B * T
        x2 = x.reshape(M, C)
        pre = pre_ln(x, ln_w, ln_b, act)   # ln_f from the last FFN GEMM's epilogue
        a, mean, rstd = pre if pre is not None else layernorm(x2, ln_w.master, ln_b.master, act)
        V = lm_w.master.shape[0]
        ctx.fused = _head_fused_ok(act, lm_w, M, C, V)
        ctx.in_link = _link_of(x)
        if ctx.fused:
            return HeadLossFn._fused_forward(ctx, x, x2, targets, act, a, mean, rstd, (ln_w, ln_b, lm_w, lm_b))
        logits = torch.empty((M, V), dtype=torch.float32, device=x.device)
        linear_fwd(a, lm_w.operand(act), logits, "bias", bias=lm_b.master)
        lse = torch.empty(M, dtype=torch.float32, device=x.device)
        ctx.regs, ctx.shape, ctx.act = (ln_w, ln_b, lm_w, lm_b), (B, T, C), act
        ctx.set_materialize_grads(False)
        if targets is None:
            ctx.save_for_backward(x2, a, mean, rstd, logits, lse)
            ctx.has_targets = False
            return logits.view(B, T, V)
        t1 = targets.reshape(M)
        loss_rows = torch.empty(M, dtype=torch.float32, device=x.device)
        ops.ce_fwd(logits, t1, loss_rows, lse)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        ws = torch.empty(1024, dtype=torch.float32, device=x.device)
        ops.sum_scaled(loss_rows, 1.0 / M, loss, ws)
        ctx.save_for_backward(x2, a, mean, rstd, logits, lse, t1)
        ctx.has_targets = True
        return logits, loss

    @staticmethod
    def backward(ctx, *grads):
        ln_w, ln_b, lm_w, lm_b = ctx.regs
        B, T, C = ctx.shape
        act = ctx.act
        M = B * T
        if ctx.has_targets:
            x2, a, mean, rstd, logits, lse, t1 = ctx.saved_tensors
            g_logits, g_loss = grads
        else:
            x2, a, mean, rstd, logits, lse = ctx.saved_tensors
            g_logits, g_loss = grads[0], None
        V = logits.shape[-1]
        if ctx.fused:
            return HeadLossFn._fused_backward(ctx, x2, a, mean, rstd, logits, lse, t1 if ctx.has_targets else None,
                                              g_logits, g_loss)
        dl = torch.empty((M, V), dtype=torch.float32, device=x2.device)
        if g_loss is not None:
            ops.ce_bwd(logits, t1, lse, g_loss.reshape(1).float().contiguous(), 1.0 / M, dl, None)
            if g_logits is not None:
                dl.add_(g_logits.reshape(M, V))
        else:
            dl.copy_(g_logits.reshape(M, V))
        dl_op = dl if act == torch.float32 else to_act(dl, act)
        g, beta, f_lw = lm_w.grad_target()
        if g is not None:
            linear_wgrad(dl_op, a, g, beta, g is lm_w.slot)
        g, beta, f_lb = lm_b.grad_target()
        if g is not None:
            colsum_into(dl, g, beta)
        da = torch.empty((M, C), dtype=act, device=x2.device)
        linear_dgrad(dl_op, lm_w.operand(act), da)
        dx, _, f_ln = layernorm_bwd(da, x2, ln_w, ln_b, mean, rstd, link=ctx.in_link)
        return (dx.view(B, T, C), None, None, None, None, None, None, *f_ln, *f_lw(), *f_lb())

    # -- bf16 fast path: cg_head_fwd/bwd + K-padded MFMA GEMMs (csrc/head.hip) -------------
    @staticmethod
    def _fused_forward(ctx, x, x2, targets, act, a, mean, rstd, regs):
        ln_w, ln_b, lm_w, lm_b = regs
        B, T, C = x.shape
        M, V = B * T, lm_w.master.shape[0]
        wpad = lm_w.padded[0]
        logits = torch.empty((M, V), dtype=torch.float32, device=x.device)
        lse = torch.empty(M, dtype=torch.float32, device=x.device)
        ctx.regs, ctx.shape, ctx.act = regs, (B, T, C), act
        ctx.set_materialize_grads(False)
        if targets is None:
            ops.head_fwd(a, wpad, lm_b.master, None, logits, lse, None, None)
            ctx.save_for_backward(x2, a, mean, rstd, logits, lse)
            ctx.has_targets = False
            return logits.view(B, T, V)
        t1 = targets.reshape(M)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        ws = torch.empty(ops.head_workspace(M, V) // 4, dtype=torch.float32, device=x.device)
        ops.head_fwd(a, wpad, lm_b.master, t1, logits, lse, loss, ws)
        ctx.save_for_backward(x2, a, mean, rstd, logits, lse, t1)
        ctx.has_targets = True
        return logits, loss

    @staticmethod
    def _fused_backward(ctx, x2, a, mean, rstd, logits, lse, t1, g_logits, g_loss):
        ln_w, ln_b, lm_w, lm_b = ctx.regs
        B, T, C = ctx.shape
        M, V = logits.shape
        wpad, gpad = lm_w.padded
        KP = wpad.shape[0]
        dl = torch.empty((M, KP), dtype=torch.bfloat16, device=x2.device)
        gb, beta_b, f_lb = lm_b.grad_target()
        ws = torch.empty(ops.head_workspace(M, V) // 4, dtype=torch.float32, device=x2.device)
        gl = None if g_logits is None else g_logits.reshape(M, V).float().contiguous()
        if g_loss is None:
            t1 = None
        # the lm_head bias gradient's column-sum reduce joins DEFER's multi-job flush when it targets the slot
        with DEFER.partials(ws) if (gb is not None and gb is lm_b.slot) else contextlib.nullcontext(False) as queued:
            ops.head_bwd(logits, lse, t1, None if g_loss is None else g_loss.reshape(1).float().contiguous(), 1.0 / M,
                         gl, dl, gb, bool(beta_b), ws, queued)
        g, beta, f_lw = lm_w.grad_target()
        if g is not None:
            if g.data_ptr() == lm_w.slot.data_ptr():
                with SIDE.run(x2.device, dl, a):
                    linear_wgrad(dl, a, gpad, beta, True)   # rows >= V get exact zeros (dl pad columns are 0)
            else:
                tmp = torch.empty((KP, C), dtype=torch.float32, device=x2.device)
                linear_wgrad(dl, a, tmp, 0.0)
                if beta:
                    g.add_(tmp[:V])
                else:
                    g.copy_(tmp[:V])
        da = torch.empty((M, C), dtype=torch.bfloat16, device=x2.device)
        linear_dgrad(dl, wpad, da)
        dx, _, f_ln = layernorm_bwd(da, x2, ln_w, ln_b, mean, rstd, link=ctx.in_link)
        return (dx.view(B, T, C), None, None, None, None, None, None, *f_ln, *f_lw(), *f_lb())


def _head_fused_ok(act, lm_w, M, C, V):
    return (act == torch.bfloat16 and lm_w.padded is not None and lm_w.slot is not None and V <= 128
            and M % 16 == 0 and C % 32 == 0)


# ---------------------------------------------------------------------------------------
# standalone module paths (GPT1.py classes used on their own)
# ---------------------------------------------------------------------------------------
class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_reg, b_reg, eps, *params):
        shp = x.shape
        x2 = _flat2(x.float().contiguous())
        y, mean, rstd = layernorm(x2, w_reg.master, b_reg.master, torch.float32, eps)
        ctx.save_for_backward(x2, mean, rstd)
        ctx.regs = (w_reg, b_reg)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd = ctx.saved_tensors
        w_reg, b_reg = ctx.regs
        dx, _, f = layernorm_bwd(_flat2(dy.float().contiguous()), x2, w_reg, b_reg, mean, rstd)
        return (dx.view(dy.shape), None, None, None, *f)


class MHAFn(torch.autograd.Function):
    """MultiHeadAttention.forward / Head.forward on an arbitrary (already normalised) input:
    out = [proj](cat_h softmax(mask(q_h k_h^T * C^-0.5)) v_h)  (GPT1.py:109-123,134-136).
    proj_w None -> single Head (no projection)."""

    @staticmethod
    def forward(ctx, x, lc, qkv_w, proj_w, proj_b, *params):
        B, T, C = x.shape
        act = lc.act
        x2 = to_act(_flat2(x.float().contiguous()), act)
        d = lc.n_head * lc.head_size
        qkv = torch.empty((B * T, 3 * d), dtype=act, device=x.device)
        linear_fwd(x2, qkv_w.operand(act), qkv)
        o = torch.empty((B * T, d), dtype=act, device=x.device)
        lse, ctx.mask = attention_fwd(qkv, B, T, lc.n_head, lc.head_size, o, lc.scale, lc.p, lc.seed, lc.rng_call,
                                      lc.site, lc.premask)
        if proj_w is not None:
            out = torch.empty((B * T, proj_w.master.shape[0]), dtype=torch.float32, device=x.device)
            linear_fwd(o, proj_w.operand(act), out, "bias", bias=proj_b.master)
        else:
            out = o.float()
        ctx.save_for_backward(x2, qkv, o, lse)
        ctx.lc, ctx.regs, ctx.shape = lc, (qkv_w, proj_w, proj_b), (B, T, C)
        return out.view(B, T, -1)

    @staticmethod
    def backward(ctx, dout):
        x2, qkv, o, lse = ctx.saved_tensors
        lc = ctx.lc
        qkv_w, proj_w, proj_b = ctx.regs
        B, T, C = ctx.shape
        act = lc.act
        d32 = _flat2(dout.float().contiguous())
        rets = []
        if proj_w is not None:
            dy = to_act(d32, act)
            g, beta, f_pw = proj_w.grad_target()
            if g is not None:
                linear_wgrad(dy, o, g, beta, g is proj_w.slot)
            g, beta, f_pb = proj_b.grad_target()
            if g is not None:
                colsum_into(dy, g, beta)
            do = torch.empty(o.shape, dtype=act, device=o.device)
            linear_dgrad(dy, proj_w.operand(act), do)
            rets = [*f_pw(), *f_pb()]
        else:
            do = to_act(d32, act)
        dqkv = attention_bwd(qkv, B, T, lc.n_head, lc.head_size, o, do, lse, lc.scale, lc.p, lc.seed, lc.rng_call,
                             lc.site, ctx.mask)
        g, beta, f_qkv = qkv_w.grad_target()
        if g is not None:
            linear_wgrad(dqkv, x2, g, beta, g is qkv_w.slot)
        dx = torch.empty((B * T, C), dtype=torch.float32, device=o.device)
        linear_dgrad(dqkv, qkv_w.operand(act), dx)
        return (dx.view(B, T, C), None, None, None, None, *f_qkv(), *rets)


class FFNFn(torch.autograd.Function):
    """FeedForward.forward (GPT1.py:142-150) on an arbitrary input: Dropout(W2 relu(W1 x + b1) + b2)."""

    @staticmethod
    def forward(ctx, x, lc, w1, b1, w2, b2, *params):
        B, T, C = x.shape
        act = lc.act
        x2 = to_act(_flat2(x.float().contiguous()), act)
        h = torch.empty((B * T, w1.master.shape[0]), dtype=act, device=x.device)
        linear_fwd(x2, w1.operand(act), h, "bias_relu", bias=b1.master)
        out = torch.empty((B * T, C), dtype=torch.float32, device=x.device)
        linear_fwd(h, w2.operand(act), out, "bias_drop_resid", bias=b2.master, resid=None, dropout_p=lc.p,
                   seed=lc.seed, rng_call=lc.rng_call, site=lc.site)
        ctx.save_for_backward(x2, h)
        ctx.lc, ctx.regs, ctx.shape = lc, (w1, b1, w2, b2), (B, T, C)
        return out.view(B, T, C)

    @staticmethod
    def backward(ctx, dout):
        x2, h = ctx.saved_tensors
        lc = ctx.lc
        w1, b1, w2, b2 = ctx.regs
        B, T, C = ctx.shape
        act = lc.act
        d32 = _flat2(dout.float().contiguous())
        dz2 = torch.empty((B * T, C), dtype=act, device=h.device)
        ops.dropout_apply(d32, dz2, float(lc.p), int(lc.seed), lc.rng_call, int(lc.site))
        g, beta, f_w2 = w2.grad_target()
        if g is not None:
            linear_wgrad(dz2, h, g, beta, g is w2.slot)
        g, beta, f_b2 = b2.grad_target()
        if g is not None:
            colsum_into(dz2, g, beta)
        dz1 = torch.empty_like(h)
        linear_dgrad(dz2, w2.operand(act), dz1, "relu_bwd", aux=h)
        g, beta, f_w1 = w1.grad_target()
        if g is not None:
            linear_wgrad(dz1, x2, g, beta, g is w1.slot)
        g, beta, f_b1 = b1.grad_target()
        if g is not None:
            colsum_into(dz1, g, beta)
        dx = torch.empty((B * T, C), dtype=torch.float32, device=h.device)
        linear_dgrad(dz1, w1.operand(act), dx)
        return (dx.view(B, T, C), None, None, None, None, None, *f_w1(), *f_b1(), *f_w2(), *f_b2())


class LinearFn(torch.autograd.Function):
    """nn.Linear on its own (exact fp32 GEMMs): y = x W^T + b."""

    @staticmethod
    def forward(ctx, x, w_reg, b_reg, *params):
        shp = x.shape
        x2 = _flat2(x.float().contiguous())
        N = w_reg.master.shape[0]
        out = torch.empty((x2.shape[0], N), dtype=torch.float32, device=x.device)
        linear_fwd(x2, w_reg.master, out, "bias" if b_reg is not None else "store",
                   bias=b_reg.master if b_reg is not None else None)
        ctx.save_for_backward(x2)
        ctx.regs = (w_reg, b_reg)
        return out.view(*shp[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        (x2,) = ctx.saved_tensors
        w_reg, b_reg = ctx.regs
        d2 = _flat2(dy.float().contiguous())
        g, beta, fw = w_reg.grad_target()
        if g is not None:
            linear_wgrad(d2, x2, g, beta, g is w_reg.slot)
        rets = fw()
        if b_reg is not None:
            g, beta, fb = b_reg.grad_target()
            if g is not None:
                colsum_into(d2, g, beta)
            rets = rets + fb()
        dx = torch.empty(x2.shape, dtype=torch.float32, device=x2.device)
        linear_dgrad(d2, w_reg.master, dx)
        return (dx.view(*dy.shape[:-1], x2.shape[-1]), None, None, *rets)


def attention_scale(n_embd):
    """Q1: the reference scales by C ** -0.5 with C = n_embd (GPT1.py:110,114), not head_size."""
    return float(n_embd) ** -0.5
