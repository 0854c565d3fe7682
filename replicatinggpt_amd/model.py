"""The char-level GPT of GPT1.py (Head / MultiHeadAttention / FeedForward / Block /
BigramLanguageModel) with the reference's constructor signatures, module tree, parameter
init order and state-dict keys, executed by charpt HIP kernels.

* Construction draws the seeded init in the reference's order, so
  ``torch.manual_seed(1337); BigramLanguageModel()`` yields the reference's weights and leaves the
  CPU generator in the reference's state (batch indices stay bit-identical).
* ``BigramLanguageModel`` packs every parameter into one flat fp32 buffer (plus a flat fp32
  gradient buffer and a bf16 shadow of the weights for the GEMMs).  The per-head
  ``key/query/value`` weights stay separate nn.Parameters (state-dict compatible) but are views of
  one [3*n_embd, n_embd] QKV region, so a whole MultiHeadAttention is one GEMM + one fused
  attention launch.
* There is no CPU path: forward on a non-HIP device raises.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as Fn
from . import ops
from .config import GPTConfig, get_default

ALIGN = 64  # elements (256 B) between flat regions


def _require_hip(t):
    if t.device.type != "cuda":
        raise RuntimeError("charpt: the char-GPT hot path runs only on an AMD GPU (HIP) device; got "
                           f"{t.device}. The CPU restatement lives in oracle/ and is test infrastructure.")


def _act_dtype(cfg):
    return torch.bfloat16 if cfg.dtype == "bf16" else torch.float32


class _Ctx:
    """Forward-call state shared by the blocks of one model forward."""
    rng_call = None


# ---------------------------------------------------------------------------------------
# leaf modules
# ---------------------------------------------------------------------------------------
class Linear(nn.Linear):
    """nn.Linear (same init, same state dict) whose forward runs the charpt GEMM."""

    def forward(self, x):
        _require_hip(x)
        w = Fn.Region.of(self.weight)
        if self.bias is None:
            return Fn.LinearFn.apply(x, w, None, self.weight)
        b = Fn.Region.of(self.bias)
        return Fn.LinearFn.apply(x, w, b, self.weight, self.bias)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (GPT1.py:159-160,173) on the charpt LayerNorm kernels."""

    def forward(self, x):
        _require_hip(x)
        w, b = self._regions()
        return Fn.LayerNormFn.apply(x, w, b, self.eps, self.weight, self.bias)

    def _regions(self):
        st = getattr(self, "_charpt_regions", None)
        if st is not None:
            return st
        return Fn.Region.of(self.weight), Fn.Region.of(self.bias)


class Head(nn.Module):
    """One self-attention head (GPT1.py:100-123)."""

    def __init__(self, head_size, n_embd, config=None):
        super().__init__()
        cfg = config or get_default()
        self.config = cfg
        self.n_embd = n_embd
        self.key = Linear(n_embd, head_size, bias=False)      # GPT1.py:103
        self.query = Linear(n_embd, head_size, bias=False)    # GPT1.py:104
        self.value = Linear(n_embd, head_size, bias=False)    # GPT1.py:105
        self.register_buffer("tril", torch.tril(torch.ones(cfg.block_size, cfg.block_size)))  # GPT1.py:106
        self.dropout = nn.Dropout(cfg.dropout)                # GPT1.py:107

    def forward(self, x):
        _require_hip(x)
        B, T, C = x.shape
        hs = self.key.out_features
        p = self.dropout.p if self.training else 0.0
        rng = _snapshot_for(self, x) if p > 0 else None
        lc = Fn.LayerCtx(1, hs, Fn.attention_scale(C), p, self.config.dropout_seed, rng, 0,
                         _act_dtype(self.config))
        qkv = Fn.Region.of(self.query.weight, self.key.weight, self.value.weight)
        return Fn.MHAFn.apply(x, lc, qkv, None, None, *qkv.params)


class MultiHeadAttention(nn.Module):
    """n_heads Heads + output projection (GPT1.py:126-136); one QKV GEMM + one fused attention."""

    def __init__(self, n_heads, head_size, config=None):
        super().__init__()
        cfg = config or get_default()
        self.config = cfg
        self.heads = nn.ModuleList([Head(head_size, cfg.n_embd, cfg) for _ in range(n_heads)])  # GPT1.py:130
        self.proj = Linear(cfg.n_embd, cfg.n_embd)            # GPT1.py:131
        self.dropout = nn.Dropout(cfg.dropout)                # GPT1.py:132 (never applied)
        self.site = 0

    def qkv_region(self):
        r = getattr(self, "_charpt_qkv", None)
        if r is not None:
            return r
        ws = [h.query.weight for h in self.heads] + [h.key.weight for h in self.heads] + \
             [h.value.weight for h in self.heads]
        return Fn.Region.of(*ws)

    def proj_regions(self):
        r = getattr(self, "_charpt_proj", None)
        return r if r is not None else (Fn.Region.of(self.proj.weight), Fn.Region.of(self.proj.bias))

    def layer_ctx(self, x, C):
        p = self.heads[0].dropout.p if self.training else 0.0
        rng = _snapshot_for(self, x) if p > 0 else None
        root = getattr(self, "_charpt_root", None)
        pm = root._premasks.get(self.site) if (p > 0 and root is not None and root._premasks) else None
        return Fn.LayerCtx(len(self.heads), self.heads[0].key.out_features, Fn.attention_scale(C), p,
                           self.config.dropout_seed, rng, self.site, _act_dtype(self.config), pm)

    def forward(self, x):
        _require_hip(x)
        C = x.shape[-1]
        lc = self.layer_ctx(x, C)
        qkv = self.qkv_region()
        pw, pb = self.proj_regions()
        return Fn.MHAFn.apply(x, lc, qkv, pw, pb, *qkv.params, *pw.params, *pb.params)


class FeedForward(nn.Module):
    """Linear(d,4d) -> ReLU -> Linear(4d,d) -> Dropout (GPT1.py:138-150)."""

    def __init__(self, n_embd, config=None):
        super().__init__()
        cfg = config or get_default()
        self.config = cfg
        self.net = nn.Sequential(
            Linear(n_embd, n_embd * 4),       # GPT1.py:143
            nn.ReLU(),                        # GPT1.py:144
            Linear(4 * n_embd, n_embd),       # GPT1.py:145
            nn.Dropout(cfg.dropout),          # GPT1.py:146
        )
        self.site = 1

    def regions(self):
        r = getattr(self, "_charpt_regions", None)
        if r is not None:
            return r
        n = self.net
        return (Fn.Region.of(n[0].weight), Fn.Region.of(n[0].bias), Fn.Region.of(n[2].weight),
                Fn.Region.of(n[2].bias))

    def layer_ctx(self, x):
        p = self.net[3].p if self.training else 0.0
        rng = _snapshot_for(self, x) if p > 0 else None
        return Fn.LayerCtx(0, 0, 0.0, p, self.config.dropout_seed, rng, self.site, _act_dtype(self.config))

    def forward(self, x):
        _require_hip(x)
        lc = self.layer_ctx(x)
        w1, b1, w2, b2 = self.regions()
        return Fn.FFNFn.apply(x, lc, w1, b1, w2, b2, *w1.params, *b1.params, *w2.params, *b2.params)


class Block(nn.Module):
    """Pre-LN transformer block (GPT1.py:152-165) as two fused autograd nodes."""

    def __init__(self, n_embd, n_head, config=None):
        super().__init__()
        cfg = config or get_default()
        self.config = cfg
        head_size = n_embd // n_head                                  # GPT1.py:156
        self.sa_heads = MultiHeadAttention(n_head, head_size, cfg)    # GPT1.py:157
        self.ffwd = FeedForward(n_embd, cfg)                          # GPT1.py:158
        self.ln1 = LayerNorm(n_embd)                                  # GPT1.py:159
        self.ln2 = LayerNorm(n_embd)                                  # GPT1.py:160

    def set_layer_index(self, l):
        self.sa_heads.site = 2 * l
        self.ffwd.site = 2 * l + 1

    def forward(self, x):
        _require_hip(x)
        C = x.shape[-1]
        lc = self.sa_heads.layer_ctx(x, C)
        ln1w, ln1b = self.ln1._regions()
        qkv = self.sa_heads.qkv_region()
        pw, pb = self.sa_heads.proj_regions()
        ln2w, ln2b = self.ln2._regions()
        lc.next_ln = (ln2w, ln2b, self.ln2.eps)   # the projection GEMM also computes ln2 (functional.pre_ln)
        y = Fn.attn_sublayer_infer(x, lc, ln1w, ln1b, qkv, pw, pb) if not torch.is_grad_enabled() else None
        if y is not None:   # inference: the row-resident fp32 Linears where they apply
            x = y
        else:
            x = Fn.AttnSublayerFn.apply(x, lc, ln1w, ln1b, qkv, pw, pb, *ln1w.params, *ln1b.params, *qkv.params,
                                        *pw.params, *pb.params)
        lc2 = self.ffwd.layer_ctx(x)
        # the next block's ln1 or the model's ln_f, from the FFN GEMM's epilogue -- not ln1 when that
        # block's attention drops out: its LayerNorm launch also makes the keep bits (functional.
        # layernorm_attn_mask), cheaper than a keep-bit launch of their own (profiles/r5_gemm_ln_ab.txt)
        nxt, att = getattr(self, "_charpt_next_ln", (None, None))
        if nxt is not None and (att is None or not (self.training and att.heads[0].dropout.p > 0)):
            lc2.next_ln = (*nxt._regions(), nxt.eps)
        w1, b1, w2, b2 = self.ffwd.regions()
        if not torch.is_grad_enabled():   # inference: the fused fp32 FFN where it applies
            y = Fn.ffn_sublayer_infer(x, lc2, ln2w, ln2b, w1, b1, w2, b2)
            if y is not None:
                return y
        return Fn.FFNSublayerFn.apply(x, lc2, ln2w, ln2b, w1, b1, w2, b2, *ln2w.params, *ln2b.params, *w1.params,
                                      *b1.params, *w2.params, *b2.params)


# ---------------------------------------------------------------------------------------
# dropout stream bookkeeping
# ---------------------------------------------------------------------------------------
def _snapshot_for(module, x):
    """Device uint64 snapshot of the dropout call counter for this forward (one per model
    forward; standalone modules take their own)."""
    root = getattr(module, "_charpt_root", None)
    if root is not None and root._fwd_rng is not None:
        return root._fwd_rng
    ctr = getattr(module, "_charpt_counter", None)
    if ctr is None or ctr.device != x.device:
        ctr = torch.zeros(1, dtype=torch.int64, device=x.device)
        object.__setattr__(module, "_charpt_counter", ctr)
    snap = torch.empty(1, dtype=torch.int64, device=x.device)
    ops.rng_snapshot(ctr, snap)
    return snap


# ---------------------------------------------------------------------------------------
# flat parameter storage
# ---------------------------------------------------------------------------------------
class FlatStore:
    """One fp32 master buffer, one fp32 gradient buffer and one bf16 shadow for all parameters."""

    def __init__(self, plan, device, pad_rows=None):
        # plan: list of (key, [(module, attr)]) -- parameters of a region are concatenated.
        # pad_rows: {key: rows} -- allocate the (single-parameter, 2-D) region with that many rows,
        # the extra rows zero forever (zero gradient, zero AdamW update): the LM head's K-padded
        # GEMM operand (functional.HeadLossFn) lives in the shadow without a copy.
        self.plan = plan
        self.pad_rows = dict(pad_rows or {})
        self.offsets = {}
        off = 0
        for key, members in plan:
            n = sum(getattr(m, a).numel() for m, a in members)
            self.offsets[key] = (off, n)
            alloc = n
            if key in self.pad_rows:
                cols = getattr(*members[0]).shape[-1]
                alloc = max(n, self.pad_rows[key] * cols)
            off += -(-alloc // ALIGN) * ALIGN
        self.numel = off
        master = torch.zeros(self.numel, dtype=torch.float32, device=device)
        with torch.no_grad():
            for key, members in plan:
                o, _ = self.offsets[key]
                for m, a in members:
                    p = getattr(m, a)
                    master[o:o + p.numel()].copy_(p.detach().reshape(-1))
                    o += p.numel()
        self._bind(master)

    def _bind(self, master):
        self.master = master
        self.grad = torch.zeros_like(master)
        self.shadow = torch.zeros(self.numel, dtype=torch.bfloat16, device=master.device)
        self.regions = {}
        for key, members in self.plan:
            o, n = self.offsets[key]
            shape = self._region_shape(members)
            mview = master[o:o + n].view(shape)
            parts, po = [], 0
            for m, a in members:
                old = getattr(m, a)
                pv = master[o + po:o + po + old.numel()].view(old.shape)
                if isinstance(old, nn.Parameter) and old.data_ptr() != pv.data_ptr():
                    if getattr(old, "_charpt_bound", False):
                        old.data = pv
                        newp = old
                    else:
                        newp = nn.Parameter(pv, requires_grad=old.requires_grad)
                        newp._charpt_bound = True
                        m._parameters[a] = newp
                else:
                    newp = old
                if isinstance(newp, nn.Parameter):
                    newp._charpt_store = self   # lets optim.AdamW find the flat buffers
                parts.append((newp, po))
                po += old.numel()
            padded = None
            if key in self.pad_rows and self.pad_rows[key] >= shape[0]:
                pr = self.pad_rows[key]
                padded = (self.shadow[o:o + pr * shape[1]].view(pr, shape[1]),
                          self.grad[o:o + pr * shape[1]].view(pr, shape[1]))
            self.regions[key] = Fn.Region(mview, parts, self.grad[o:o + n].view(shape),
                                          self.shadow[o:o + n].view(shape), padded)
        self.refresh_shadow()

    @staticmethod
    def _region_shape(members):
        shapes = [m._parameters[a].shape for m, a in members]
        if len(shapes) == 1:
            return shapes[0]
        rows = sum(s[0] for s in shapes)
        return torch.Size([rows, shapes[0][1]])

    def block_starts(self):
        """Flat offset of each transformer block's first region (the plan keeps a block's
        parameters contiguous: [embeddings | block 0 | ... | block L-1 | ln_f + lm_head])."""
        out, l = [], 0
        while f"{l}.qkv" in self.offsets:
            out.append(self.offsets[f"{l}.qkv"][0])
            l += 1
        return out

    def params(self):
        out = []
        for r in self.regions.values():
            out += r.params
        return out

    def version(self):
        return sum(p._version for p in self.params())

    def refresh_shadow(self):
        if self.master.device.type == "cuda":
            ops.cast_bf16(self.master, self.shadow)
        else:
            self.shadow.copy_(self.master.to(torch.bfloat16))
        self._shadow_version = self.version()

    def to(self, fn):
        new = fn(self.master)
        if new.dtype != torch.float32:
            raise TypeError("charpt: parameters stay fp32 masters (compute dtype is GPTConfig.dtype)")
        for p in self.params():
            p._charpt_bound = True
        self._bind(new.contiguous())


# ---------------------------------------------------------------------------------------
class BigramLanguageModel(nn.Module):
    """The char-level GPT (GPT1.py:167-212)."""

    def __init__(self, config=None):
        super().__init__()
        cfg = config or get_default()
        self.config = cfg
        d = cfg.n_embd
        self.token_embedding_table = nn.Embedding(cfg.vocab_size, d)             # GPT1.py:170
        self.position_embedding_table = nn.Embedding(cfg.block_size, d)          # GPT1.py:171
        self.blocks = nn.Sequential(*[Block(d, cfg.n_head, cfg) for _ in range(cfg.n_layers)])  # GPT1.py:172
        self.ln_f = LayerNorm(d)                                                 # GPT1.py:173
        self.lm_head = Linear(d, cfg.vocab_size)                                 # GPT1.py:174
        for l, blk in enumerate(self.blocks):
            blk.set_layer_index(l)
            # the LayerNorm that reads this block's output (functional.linear_fwd_resid_ln)
            nxt = (self.blocks[l + 1].ln1, self.blocks[l + 1].sa_heads) if l + 1 < len(self.blocks) else (self.ln_f, None)
            object.__setattr__(blk, "_charpt_next_ln", nxt)
        self._fwd_rng = None
        self._premasks = None
        self.register_buffer("_rng_counter", torch.zeros(1, dtype=torch.int64), persistent=False)
        self._store = None
        self._pack()

    # -- flat storage ------------------------------------------------------------------
    def _plan(self):
        plan = [("wte", [(self.token_embedding_table, "weight")]),
                ("wpe", [(self.position_embedding_table, "weight")])]
        for l, blk in enumerate(self.blocks):
            heads = blk.sa_heads.heads
            plan.append((f"{l}.qkv", [(h.query, "weight") for h in heads] + [(h.key, "weight") for h in heads] +
                         [(h.value, "weight") for h in heads]))
            plan += [(f"{l}.proj_w", [(blk.sa_heads.proj, "weight")]), (f"{l}.proj_b", [(blk.sa_heads.proj, "bias")]),
                     (f"{l}.w1", [(blk.ffwd.net[0], "weight")]), (f"{l}.b1", [(blk.ffwd.net[0], "bias")]),
                     (f"{l}.w2", [(blk.ffwd.net[2], "weight")]), (f"{l}.b2", [(blk.ffwd.net[2], "bias")]),
                     (f"{l}.ln1_w", [(blk.ln1, "weight")]), (f"{l}.ln1_b", [(blk.ln1, "bias")]),
                     (f"{l}.ln2_w", [(blk.ln2, "weight")]), (f"{l}.ln2_b", [(blk.ln2, "bias")])]
        plan += [("lnf_w", [(self.ln_f, "weight")]), ("lnf_b", [(self.ln_f, "bias")]),
                 ("lm_w", [(self.lm_head, "weight")]), ("lm_b", [(self.lm_head, "bias")])]
        return plan

    def _pack(self):
        dev = self.token_embedding_table.weight.device
        V = self.config.vocab_size
        pad = {"lm_w": 128} if V <= 128 else None   # K-padded operand of the fused head (HeadLossFn)
        self._store = FlatStore(self._plan(), dev, pad)
        self._attach_regions()

    def _attach_regions(self):
        R = self._store.regions
        for l, blk in enumerate(self.blocks):
            object.__setattr__(blk.sa_heads, "_charpt_qkv", R[f"{l}.qkv"])
            object.__setattr__(blk.sa_heads, "_charpt_proj", (R[f"{l}.proj_w"], R[f"{l}.proj_b"]))
            object.__setattr__(blk.ffwd, "_charpt_regions", (R[f"{l}.w1"], R[f"{l}.b1"], R[f"{l}.w2"], R[f"{l}.b2"]))
            object.__setattr__(blk.ln1, "_charpt_regions", (R[f"{l}.ln1_w"], R[f"{l}.ln1_b"]))
            object.__setattr__(blk.ln2, "_charpt_regions", (R[f"{l}.ln2_w"], R[f"{l}.ln2_b"]))
        object.__setattr__(self.ln_f, "_charpt_regions", (R["lnf_w"], R["lnf_b"]))
        for m in self.modules():
            if m is not self:
                object.__setattr__(m, "_charpt_root", self)

    @property
    def flat(self):
        return self._store

    def set_dropout_rank(self, rank):
        """Data parallel: give rank ``rank`` its own Philox dropout key (base seed + 7919 * rank),
        so the W replicas draw independent masks (GPT1.py:117,146) -- rank 0 keeps the base seed,
        i.e. the single-GPU stream.  Idempotent; the engine (engine.TrainStep) calls it."""
        base = self.__dict__.setdefault("_dropout_seed_base", self.config.dropout_seed)
        old = self.config
        new = old.with_(dropout_seed=base + 7919 * int(rank))   # never mutate a (possibly shared) config
        for m in self.modules():
            if getattr(m, "config", None) is old:
                m.config = new
        return new.dropout_seed

    def _apply(self, fn, recurse=True):
        store = self._store
        if store is None:
            return super()._apply(fn, recurse)
        store.to(fn)
        self._attach_regions()
        for m in self.modules():
            for k, b in list(m._buffers.items()):
                if b is not None:
                    m._buffers[k] = fn(b)
        return self

    def state_dict(self, *args, **kwargs):
        """Reference layout (GPT1.py:239-241): independent fp32 tensors, incl. the tril buffers."""
        sd = super().state_dict(*args, **kwargs)
        for k, v in list(sd.items()):
            if isinstance(v, torch.Tensor):
                sd[k] = v.detach().clone()
        return sd

    def _sync_shadow(self):
        st = self._store
        if st.version() != st._shadow_version:
            st.refresh_shadow()

    # -- forward (GPT1.py:176-194) -----------------------------------------------------
    def forward(self, idx, targets=None):
        _require_hip(idx)
        cfg = self.config
        idx = idx.contiguous()          # generate() passes a column slice idx[:, -block_size:]
        if targets is not None:
            targets = targets.contiguous()
        B, T = idx.shape
        if T > cfg.block_size:
            raise ValueError(f"sequence length {T} exceeds block_size {cfg.block_size}")
        act = _act_dtype(cfg)
        if act == torch.bfloat16:
            self._sync_shadow()
        R = self._store.regions
        p = cfg.dropout if self.training else 0.0
        if p > 0:
            snap = torch.empty(1, dtype=torch.int64, device=idx.device)
            ops.rng_snapshot(self._rng_counter, snap)
            self._fwd_rng = snap
            hs = cfg.n_embd // cfg.n_head
            if Fn.SIDE.premask and Fn.premask_ok(act, T, hs) and self.blocks[0].sa_heads.heads[0].dropout.p > 0:
                self._launch_premasks(idx.device, B, T)
        try:
            wte, wpe = R["wte"], R["wpe"]
            x = Fn.EmbeddingFn.apply(idx, wte, wpe, *wte.params, *wpe.params)
            x = self.blocks(x)
            lw, lb, hw, hb = R["lnf_w"], R["lnf_b"], R["lm_w"], R["lm_b"]
            out = Fn.HeadLossFn.apply(x, targets, act, lw, lb, hw, hb, *lw.params, *lb.params, *hw.params,
                                      *hb.params)
        finally:
            self._fwd_rng = None
            self._premasks = None
        if targets is None:
            return out, None
        return out

    def _launch_premasks(self, dev, B, T):
        """Every layer's attention-dropout keep bits, generated on the side stream at the start of
        the forward (Philox is VALU work that overlaps the embedding / LN / QKV GEMM kernels); each
        attention forward waits on its layer's event."""
        cfg = self.config
        H = cfg.n_head
        n = ops.attn_mask_bytes(B, H, T) // 8
        cur = torch.cuda.current_stream(dev)
        side = Fn.SIDE.stream(dev)
        side.wait_stream(cur)
        pm = {}
        with torch.cuda.stream(side):
            for blk in self.blocks:
                site = blk.sa_heads.site
                p = blk.sa_heads.heads[0].dropout.p
                mask = torch.empty(n, dtype=torch.int64, device=dev)
                ops.attn_dropmask(B, H, T, float(p), int(cfg.dropout_seed), self._fwd_rng, int(site), mask)
                ev = torch.cuda.Event()
                ev.record(side)
                mask.record_stream(cur)   # read by the main stream (forward + backward)
                pm[site] = (mask, ev)
        self._premasks = pm

    # -- generate (GPT1.py:196-212) ----------------------------------------------------
    def generate(self, idx, max_new_tokens, greedy=False, generator=None, engine=True):
        """Autoregressive sampling as GPT1.py:196-212 (crop to block_size, forward, last row,
        softmax, multinomial, append).  On the GPU this runs the batched decode engine
        (decode.DecodeEngine: K/V-cached prefix phase, sliding-window phase, device sampling, one
        hipGraph per phase); ``greedy=True`` takes the argmax (the parity mode).  Sampled draws use
        a seed taken from ``generator`` (torch's CPU multinomial stream is not reproducible on a
        GPU).  ``engine=False`` runs the reference's loop literally (one full forward per token); so
        does a model in train mode with dropout on, as GPT1.py:235-236 calls it: the
        engine computes the eval-mode forward only."""
        dropout_on = self.training and self.config.dropout > 0
        if engine and not dropout_on and idx.device.type == "cuda" and max_new_tokens > 0:
            from .decode import DecodeEngine
            B, L0 = idx.shape
            key = (B, L0 + max_new_tokens, bool(greedy), idx.device)
            cache = self.__dict__.setdefault("_decode_engines", {})
            eng = cache.get(key)
            if eng is None or eng.m is not self:
                eng = cache[key] = DecodeEngine(self, B, L0 + max_new_tokens, greedy=greedy)
            seed = None if greedy else int(torch.randint(0, 2 ** 62, (1,), generator=generator))
            return eng.generate(idx, max_new_tokens, seed=seed)
        for _ in range(max_new_tokens):
            idx_cond = idx[:, -self.config.block_size:]                 # GPT1.py:200
            logits, _ = self(idx_cond)                                   # GPT1.py:202
            logits = logits[:, -1, :]                                    # GPT1.py:204
            if greedy:
                idx_next = torch.argmax(logits, dim=-1, keepdim=True)
            else:
                probs = F.softmax(logits, dim=-1)                        # GPT1.py:206
                idx_next = torch.multinomial(probs, num_samples=1, generator=generator)  # GPT1.py:208
            idx = torch.cat((idx, idx_next), dim=1)                     # GPT1.py:210
        return idx
