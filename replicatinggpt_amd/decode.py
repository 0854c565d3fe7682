"""Batched autoregressive decode engine for ``BigramLanguageModel.generate`` (GPT1.py:196-212).

The reference loop (per new token): crop ``idx[:, -block_size:]`` (GPT1.py:200), full forward
(:202), last row (:204), softmax (:206), multinomial (:208), append (:210).  Same token stream here,
computed as:

* phase 1 -- context length <= block_size: the window starts at position 0, so positions never
  change and each step pushes only the newest token through the blocks against a per-layer K/V
  cache (``cg_decode_embed``, ``cg_decode_kv_append``, ``cg_decode_attn``), plus ln_f / lm_head
  on those B rows;
* phase 2 -- context longer than block_size: the crop re-indexes positions from 0 every step
  (absolute learned position embeddings), so no K/V survives a step: the full window
  forward runs (``cg_decode_window`` gathers it on the device), except that the LAST block needs
  its queries / attention / projection / FFN only for the final row and ln_f / lm_head run on B
  rows instead of B x block_size;
* sampling on the device (``cg_decode_sample``): greedy = argmax (torch.argmax tie rule, the
  parity mode), else inverse-CDF draws from a Philox stream keyed by (seed, length, row) --
  torch.multinomial's CPU-generator stream is not reproducible on a GPU, so the sampled
  (non-greedy) stream is charpt's own, statistically the same distribution.

The current length lives in a device int64, so each phase's step is one static-shape hipGraph
captured once and replayed per token (prefill of a longer prompt replays the phase-1 graph without
sampling).  fp32 models give the reference's greedy stream (tests/test_gpu_model.py).
"""
import os

import torch

from . import functional as Fn
from . import ops

# CHARPT_DECODE_ROWS=0: the per-token LayerNorms in their own launches before ln1/ln2/lnf's Linears (A/B)
DECODE_ROWS = os.environ.get("CHARPT_DECODE_ROWS", "1") == "1"
# CHARPT_LAST_KV_SPLIT=0: the window step's last block computes Q for every row too (A/B)
LAST_KV_SPLIT = os.environ.get("CHARPT_LAST_KV_SPLIT", "1") == "1"


class DecodeEngine:
    def __init__(self, model, batch, max_len, greedy=True, seed=0, use_graph=True):
        cfg = model.config
        self.m, self.B, self.max_len = model, int(batch), int(max_len)
        self.T, self.C, self.H = cfg.block_size, cfg.n_embd, cfg.n_head
        self.D = self.C // self.H
        self.V = cfg.vocab_size
        self.L = len(model.blocks)
        self.greedy = bool(greedy)
        self.act = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
        self.dev = model.flat.master.device
        self.scale = Fn.attention_scale(self.C)
        dev, B, C = self.dev, self.B, self.C
        self.idx = torch.zeros((B, self.max_len), dtype=torch.int64, device=dev)
        self.len = torch.zeros(1, dtype=torch.int64, device=dev)
        self.seed = torch.full((1,), int(seed), dtype=torch.int64, device=dev)   # read by the sampler
        self.kc = torch.zeros((self.L, B, self.H, self.T, self.D), dtype=torch.float32, device=dev)
        self.vc = torch.zeros_like(self.kc)
        self.win = torch.empty((B, self.T), dtype=torch.int64, device=dev)
        self.x1 = torch.empty((B, C), dtype=torch.float32, device=dev)
        self.logits = torch.empty((B, self.V), dtype=torch.float32, device=dev)
        self.use_graph = use_graph and dev.type == "cuda"
        self.g1 = self.g1_prefill = self.g2 = None

    # -- regions -------------------------------------------------------------------------
    def _R(self, key):
        return self.m.flat.regions[key]

    def _w(self, key):
        return self._R(key).operand(self.act)

    def _b(self, key):
        return self._R(key).master

    def _ln(self, x2, key):
        y, _, _ = Fn.layernorm(x2, self._b(key + "_w"), self._b(key + "_b"), self.act)
        return y

    def _ln_linear(self, x2, key, w, out, bias=None, relu=False):
        """out = act(LayerNorm_key(x2) @ w^T [+ bias]): fp32 per-token rows in one launch
        (ops.linear_rows_f32, k_gemm_f32r with the LayerNorm in its prologue -- the bits of the two
        launches); else the LayerNorm launch and the GEMM."""
        lw, lb = self._b(key + "_w"), self._b(key + "_b")
        M, K = x2.shape
        if (DECODE_ROWS and self.act == torch.float32 and M <= 2048 and x2.stride(0) % 2 == 0
                and ops.linear_rows_f32_supported(M, w.shape[0], K) and w.stride(0) % 2 == 0
                and ((x2.data_ptr() | w.data_ptr()) & 7) == 0):
            ops.linear_rows_f32(x2, lw, lb, 1e-5, w, bias, None, out, relu)
            return
        a = self._ln(x2, key)
        if bias is None:
            Fn.linear_fwd(a, w, out)
        else:
            Fn.linear_fwd(a, w, out, "bias_relu" if relu else "bias", bias=bias)

    def _ffn_tail(self, l, x2):
        """x + W2 relu(W1 ln2(x) + b1) + b2 for rows x2 [R, C] (eval: no dropout)."""
        h = torch.empty((x2.shape[0], 4 * self.C), dtype=self.act, device=self.dev)
        self._ln_linear(x2, f"{l}.ln2", self._w(f"{l}.w1"), h, bias=self._b(f"{l}.b1"), relu=True)
        out = torch.empty_like(x2)
        Fn.linear_fwd(h, self._w(f"{l}.w2"), out, "bias_resid", bias=self._b(f"{l}.b2"), resid=x2)
        return out

    def _head(self, x2):
        self._ln_linear(x2, "lnf", self._R("lm_w").operand(self.act), self.logits, bias=self._b("lm_b"))

    # -- phase 1: one token against the K/V caches ---------------------------------------------
    def _step1(self, sample):
        C, B = self.C, self.B
        ops.decode_embed(self.idx, self._b("wte"), self._b("wpe"), self.len, self.x1)
        x = self.x1
        for l in range(self.L):
            qkv = torch.empty((B, 3 * C), dtype=self.act, device=self.dev)
            wq = self._w(f"{l}.qkv")
            if (DECODE_ROWS and self.act == torch.float32 and B <= 2048 and C <= 128 and C % 2 == 0
                    and x.stride(0) % 2 == 0 and wq.stride(0) % 2 == 0 and ((x.data_ptr() | wq.data_ptr()) & 7) == 0):
                # ln1 + QKV + the K / V append in one launch
                ops.decode_qkv_f32(x, self._b(f"{l}.ln1_w"), self._b(f"{l}.ln1_b"), 1e-5, wq, qkv, self.len,
                                   self.kc[l], self.vc[l])
                qkv32 = qkv
            else:
                self._ln_linear(x, f"{l}.ln1", wq, qkv)
                qkv32 = qkv if qkv.dtype == torch.float32 else qkv.float()
                ops.decode_kv_append(qkv32, C, 2 * C, self.len, self.kc[l], self.vc[l])
            o = torch.empty((B, C), dtype=torch.float32, device=self.dev)
            T, H, D = self.T, self.H, self.D
            ops.decode_attn(qkv32, qkv32.stride(0), self.kc[l], 0, self.vc[l], 0, H * T * D, T * D, D, B, H, D,
                            self.len, 0, self.scale, o)
            o = o if self.act == torch.float32 else o.to(self.act)
            x2 = torch.empty((B, C), dtype=torch.float32, device=self.dev)
            Fn.linear_fwd(o, self._w(f"{l}.proj_w"), x2, "bias_resid", bias=self._b(f"{l}.proj_b"), resid=x)
            x = self._ffn_tail(l, x2)
        if sample:
            self._head(x)
            ops.decode_sample(self.logits, self.greedy, self.seed, self.len, self.idx)
        ops.counter_add(self.len, 1)

    # -- phase 2: the sliding window -------------------------------------------------------
    def _step2(self):
        B, T, C, H, D = self.B, self.T, self.C, self.H, self.D
        ops.decode_window(self.idx, self.len, self.win)
        x = torch.empty((B, T, C), dtype=torch.float32, device=self.dev)
        ops.embed_fwd(self.win, self._b("wte"), self._b("wpe"), x)
        for blk in self.m.blocks[:-1]:
            x = blk(x)
        # last block: K/V for every row, everything else for the final row only
        l = self.L - 1
        x2 = x.reshape(B * T, C)
        lw, lb = self._b(f"{l}.ln1_w"), self._b(f"{l}.ln1_b")
        wq = self._w(f"{l}.qkv")   # [3C, C]: Q rows, then K, then V
        o = torch.empty((B, C), dtype=torch.float32, device=self.dev)
        xl = x[:, T - 1, :]        # the final rows in place (row stride T C)
        if (LAST_KV_SPLIT and self.act == torch.float32 and Fn.ATTN_ROWS and Fn.FFN_LN and B * T > 2048
                and ops.linear_rows_f32_supported(B * T, 2 * C, C) and C % 2 == 0
                and ((lw.data_ptr() | lb.data_ptr() | x2.data_ptr() | wq.data_ptr()) & 7) == 0):
            # ln1 + the K / V columns for every row, ln1 + Q for the final rows only: each value the
            # same k-ordered chain as in the full QKV product, a third of its MFMAs skipped
            kv = torch.empty((B * T, 2 * C), dtype=torch.float32, device=self.dev)
            ops.linear_rows_f32(x2, lw, lb, 1e-5, wq[C:], None, None, kv)
            q = torch.empty((B, C), dtype=torch.float32, device=self.dev)
            self._ln_linear(xl, f"{l}.ln1", wq[:C], q)
            ops.decode_attn(q, q.stride(0), kv, 0, kv, C, T * 2 * C, D, 2 * C, B, H, D, None, T, self.scale, o)
        else:
            qkv = torch.empty((B * T, 3 * C), dtype=self.act, device=self.dev)
            Fn.linear_fwd(self._ln(x2, f"{l}.ln1"), wq, qkv)
            qkv32 = qkv if qkv.dtype == torch.float32 else qkv.float()
            qlast = qkv32.view(B, T, 3 * C)[:, T - 1, :]
            ld = qkv32.stride(0)
            ops.decode_attn(qlast, qlast.stride(0), qkv32, C, qkv32, 2 * C, T * ld, D, ld, B, H, D, None, T,
                            self.scale, o)
        o = o if self.act == torch.float32 else o.to(self.act)
        x3 = torch.empty((B, C), dtype=torch.float32, device=self.dev)
        Fn.linear_fwd(o, self._w(f"{l}.proj_w"), x3, "bias_resid", bias=self._b(f"{l}.proj_b"), resid=xl)
        x4 = self._ffn_tail(l, x3)
        self._head(x4)
        ops.decode_sample(self.logits, self.greedy, self.seed, self.len, self.idx)
        ops.counter_add(self.len, 1)

    # -- driver ------------------------------------------------------------------------------
    def _graph(self, fn):
        if not self.use_graph:
            return None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = self.len.clone()
        with torch.cuda.stream(s):
            fn()                       # warm-up (allocator, kernels); state restored below
        torch.cuda.current_stream().wait_stream(s)
        self.len.copy_(saved)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        self.len.copy_(saved)          # capture does not execute, but keep the invariant explicit
        return g

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, seed=None):
        B, L0 = idx.shape
        if B != self.B or L0 < 1 or L0 + max_new_tokens > self.max_len:
            raise ValueError(f"DecodeEngine(batch={self.B}, max_len={self.max_len}) cannot run idx {tuple(idx.shape)} "
                             f"+ {max_new_tokens} tokens")
        was_training = self.m.training
        self.m.eval()
        try:
            if self.act == torch.bfloat16:
                self.m._sync_shadow()
            run1 = lambda: self._step1(True)      # noqa: E731
            run1p = lambda: self._step1(False)    # noqa: E731
            if self.use_graph and self.g1 is None:
                # capture before the prompt is written: the warm-up runs scribble on idx / caches
                self.len.fill_(1)
                self.g1 = self._graph(run1)
                self.g1_prefill = self._graph(run1p)
                if self.max_len > self.T:
                    self.g2 = self._graph(self._step2)
            if seed is not None:
                self.seed.fill_(int(seed))
            self.idx[:, :L0].copy_(idx)
            total = L0 + max_new_tokens
            if L0 > self.T:                        # prompt longer than the window: phase 2 only
                self.len.fill_(L0)
                n = L0
            else:
                self.len.fill_(1)
                n = 1                              # tokens present, mirrored on the host
            while n < L0:                          # prompt prefill: positions 0..L0-2
                self.g1_prefill.replay() if self.g1_prefill else run1p()
                n += 1
            while n < total:
                if n <= self.T:
                    self.g1.replay() if self.g1 else run1()
                else:
                    self.g2.replay() if self.g2 else self._step2()
                n += 1
            return self.idx[:, :total].clone()
        finally:
            self.m.train(was_training)
