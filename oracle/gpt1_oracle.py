"""TEST INFRASTRUCTURE ONLY -- CPU restatement of GPT1.py's char-level hot path.

A functional (parameter-dict) rewrite of the reference's algorithm on torch CPU tensors,
used by tests/ as the numerical oracle for the charpt HIP path and by bench.py as the
timed CPU baseline ("port").  The reference itself cannot travel to the GPU box, so this
restatement is what runs there; it is pinned against vectors produced by the reference
(tests/golden/, tests/test_oracle_golden.py).

Line citations are to /root/reference/GPT1.py.
"""
import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from . import philox


@dataclass
class OracleConfig:
    vocab_size: int = 65          # len(chars), GPT1.py:59
    block_size: int = 256         # GPT1.py:13
    n_embd: int = 126             # GPT1.py:14
    n_head: int = 6               # GPT1.py:21
    n_layers: int = 6             # GPT1.py:22
    dropout: float = 0.2          # GPT1.py:23
    # timing mode for the CPU baseline (bench.py): dropout through torch's own CPU op, as
    # nn.Dropout does it in the reference (bernoulli_ on the CPU generator, GPT1.py:117,146) --
    # the cost the reference pays; masks are then not the Philox ones, so never for parity
    torch_dropout: bool = False

    @property
    def head_size(self):          # n_embd // n_head, GPT1.py:156
        return self.n_embd // self.n_head


# ----------------------------------------------------------------------------------------
# data: tokenizer (GPT1.py:54-66), split (GPT1.py:68-70), batch sampling (GPT1.py:75-83)
# ----------------------------------------------------------------------------------------
def build_vocab(text):
    chars = sorted(set(text))                       # GPT1.py:58
    return chars, {c: i for i, c in enumerate(chars)}


def encode(stoi, s):
    return [stoi[c] for c in s]                     # GPT1.py:63


def decode(chars, ids):
    return "".join(chars[i] for i in ids)           # GPT1.py:64


def split(data):
    n = int(0.9 * len(data))                        # GPT1.py:68
    return data[:n], data[n:]


def draw_ix(n_tokens, block_size, batch, generator=None):
    """GPT1.py:78 -- one torch.randint draw on the (default) CPU generator."""
    return torch.randint(n_tokens - block_size, (batch,), generator=generator)


def windows(data, ix, block_size):
    """GPT1.py:79-80 -- x = data[i:i+T], y = data[i+1:i+T+1] stacked."""
    offs = torch.arange(block_size)
    pos = ix[:, None] + offs[None, :]
    return data[pos], data[pos + 1]


# ----------------------------------------------------------------------------------------
# parameters: names/shapes of the reference state dict (GPT1.py:100-174) and its init order
# ----------------------------------------------------------------------------------------
def param_specs(cfg):
    """(name, shape, init) in reference construction order; init in {'normal','uniform','one','zero'}."""
    d, hs, V, T = cfg.n_embd, cfg.head_size, cfg.vocab_size, cfg.block_size
    specs = [("token_embedding_table.weight", (V, d), "normal"),        # GPT1.py:170
             ("position_embedding_table.weight", (T, d), "normal")]     # GPT1.py:171
    for l in range(cfg.n_layers):                                       # GPT1.py:172
        b = f"blocks.{l}."
        for h in range(cfg.n_head):                                     # GPT1.py:130
            for w in ("key", "query", "value"):                         # GPT1.py:103-105
                specs.append((f"{b}sa_heads.heads.{h}.{w}.weight", (hs, d), ("uniform", d)))
        specs.append((f"{b}sa_heads.proj.weight", (d, d), ("uniform", d)))   # GPT1.py:131
        specs.append((f"{b}sa_heads.proj.bias", (d,), ("uniform", d)))
        specs.append((f"{b}ffwd.net.0.weight", (4 * d, d), ("uniform", d)))  # GPT1.py:143
        specs.append((f"{b}ffwd.net.0.bias", (4 * d,), ("uniform", d)))
        specs.append((f"{b}ffwd.net.2.weight", (d, 4 * d), ("uniform", 4 * d)))  # GPT1.py:145
        specs.append((f"{b}ffwd.net.2.bias", (d,), ("uniform", 4 * d)))
        for ln in ("ln1", "ln2"):                                       # GPT1.py:159-160
            specs.append((f"{b}{ln}.weight", (d,), "one"))
            specs.append((f"{b}{ln}.bias", (d,), "zero"))
    specs += [("ln_f.weight", (d,), "one"), ("ln_f.bias", (d,), "zero"),   # GPT1.py:173
              ("lm_head.weight", (V, d), ("uniform", d)), ("lm_head.bias", (V,), ("uniform", d))]  # :174
    return specs


def init_params(cfg):
    """Draw the seeded init in the reference's module-construction order:
    nn.Embedding -> normal_(0,1); nn.Linear -> kaiming_uniform(a=sqrt 5) == U(+-1/sqrt(fan_in))
    for weight and bias (torch/nn/modules/linear.py reset_parameters)."""
    P = {}
    with torch.no_grad():
        for name, shape, init in param_specs(cfg):
            t = torch.empty(shape)
            if init == "normal":
                t.normal_(0.0, 1.0)
            elif init == "one":
                t.fill_(1.0)
            elif init == "zero":
                t.zero_()
            else:
                fan_in = init[1]
                if name.endswith("weight"):
                    gain = math.sqrt(2.0 / (1 + 5.0))            # calculate_gain('leaky_relu', sqrt 5)
                    bound = math.sqrt(3.0) * gain / math.sqrt(fan_in)
                else:
                    bound = 1.0 / math.sqrt(fan_in)
                t.uniform_(-bound, bound)
            P[name] = t
    return P


# ----------------------------------------------------------------------------------------
# forward (GPT1.py:109-194) with the counter-based dropout substituted for nn.Dropout
# ----------------------------------------------------------------------------------------
def site_stream(call, site):
    """Dropout stream id: per training forward ``call`` and per call site (attention of layer
    l -> 2l, FFN of layer l -> 2l+1).  Shared with replicatinggpt_amd.functional."""
    return (int(call) << 8) | int(site)


def _dropout(x, p, seed, stream, idx_of_element):
    keep = philox.keep_mask(seed, stream, idx_of_element, p)
    scale = np.float32(1.0 / (1.0 - p))
    return x * torch.from_numpy(keep.reshape(x.shape)).to(device=x.device, dtype=x.dtype) * float(scale)


def layer_norm(x, w, b, eps=1e-5):                        # nn.LayerNorm, GPT1.py:159-160,173
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


def attention(xn, P, prefix, cfg, train, seed, stream, scale_dim=None):
    """All heads of MultiHeadAttention (GPT1.py:134-136), each as Head.forward (GPT1.py:109-123)."""
    B, T, C = xn.shape
    H, hs = cfg.n_head, cfg.head_size
    scale = (scale_dim or C) ** -0.5                      # Q1: C ** -0.5 with C = n_embd, GPT1.py:114
    causal = torch.tril(torch.ones(T, T, dtype=torch.bool, device=xn.device))
    outs = []
    for h in range(H):
        hp = f"{prefix}sa_heads.heads.{h}."
        k = xn @ P[hp + "key.weight"].t()                 # GPT1.py:111
        q = xn @ P[hp + "query.weight"].t()               # GPT1.py:112
        s = (q @ k.transpose(-2, -1)) * scale             # GPT1.py:114
        s = s.masked_fill(~causal, float("-inf"))         # GPT1.py:115
        p = torch.softmax(s, dim=-1)                      # GPT1.py:116
        if train and cfg.dropout > 0 and cfg.torch_dropout:
            p = F.dropout(p, cfg.dropout, training=True)  # GPT1.py:117 as the reference runs it
        elif train and cfg.dropout > 0:                   # GPT1.py:117
            bi = torch.arange(B)[:, None, None]
            qi = torch.arange(T)[None, :, None]
            ki = torch.arange(T)[None, None, :]
            idx = (((bi * H + h) * T + qi) * T + ki).numpy()
            p = _dropout(p, cfg.dropout, seed, stream, idx)
        v = xn @ P[hp + "value.weight"].t()               # GPT1.py:121
        outs.append(p @ v)                                # GPT1.py:122
    cat = torch.cat(outs, dim=-1)                         # GPT1.py:135
    return cat @ P[prefix + "sa_heads.proj.weight"].t() + P[prefix + "sa_heads.proj.bias"]  # :136


def feed_forward(xn, P, prefix, cfg, train, seed, stream):
    """FeedForward.net (GPT1.py:142-147): Linear -> ReLU -> Linear -> Dropout."""
    h = torch.relu(xn @ P[prefix + "ffwd.net.0.weight"].t() + P[prefix + "ffwd.net.0.bias"])
    y = h @ P[prefix + "ffwd.net.2.weight"].t() + P[prefix + "ffwd.net.2.bias"]
    if train and cfg.dropout > 0 and cfg.torch_dropout:
        y = F.dropout(y, cfg.dropout, training=True)      # GPT1.py:146 as the reference runs it
    elif train and cfg.dropout > 0:
        idx = np.arange(y.numel(), dtype=np.uint64).reshape(y.shape)
        y = _dropout(y, cfg.dropout, seed, stream, idx)
    return y


def forward(P, idx, cfg, targets=None, train=False, seed=0, call=0):
    """BigramLanguageModel.forward (GPT1.py:176-194). Returns (logits, loss) with the same
    shapes: logits (B*T, V) when targets are given, (B, T, V) otherwise."""
    B, T = idx.shape
    x = P["token_embedding_table.weight"][idx] + P["position_embedding_table.weight"][torch.arange(T, device=idx.device)]
    for l in range(cfg.n_layers):                         # Block.forward, GPT1.py:162-165
        pre = f"blocks.{l}."
        x = x + attention(layer_norm(x, P[pre + "ln1.weight"], P[pre + "ln1.bias"]), P, pre, cfg, train,
                          seed, site_stream(call, 2 * l))
        x = x + feed_forward(layer_norm(x, P[pre + "ln2.weight"], P[pre + "ln2.bias"]), P, pre, cfg, train,
                             seed, site_stream(call, 2 * l + 1))
    x = layer_norm(x, P["ln_f.weight"], P["ln_f.bias"])
    logits = x @ P["lm_head.weight"].t() + P["lm_head.bias"]
    if targets is None:
        return logits, None
    logits = logits.view(B * T, -1)
    return logits, F.cross_entropy(logits, targets.view(B * T))


def loss_and_grads(P, idx, targets, cfg, train=False, seed=0, call=0):
    leaf = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    logits, loss = forward(leaf, idx, cfg, targets, train, seed, call)
    loss.backward()
    return logits.detach(), loss.detach(), {k: v.grad for k, v in leaf.items()}


# ----------------------------------------------------------------------------------------
# AdamW (GPT1.py:218,233 -> torch/optim/adam.py _single_tensor_adam, decoupled decay)
# ----------------------------------------------------------------------------------------
class AdamWOracle:
    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        self.P = params
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, weight_decay
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}
        self.step_count = 0

    @torch.no_grad()
    def step(self, grads):
        self.step_count += 1
        t = self.step_count
        bc1 = 1 - self.b1 ** t
        bc2 = 1 - self.b2 ** t
        for k, p in self.P.items():
            g = grads[k]
            p.mul_(1 - self.lr * self.wd)                         # adam.py:419
            self.m[k].lerp_(g, 1 - self.b1)                       # adam.py:457
            self.v[k].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)  # adam.py:476
            denom = (self.v[k].sqrt() / (bc2 ** 0.5)).add_(self.eps)
            p.addcdiv_(self.m[k], denom, value=-(self.lr / bc1))  # adam.py:547


# ----------------------------------------------------------------------------------------
# generate (GPT1.py:196-212): window crop, full forward, last row; greedy variant for parity
# ----------------------------------------------------------------------------------------
@torch.no_grad()
def generate_greedy(P, idx, cfg, max_new_tokens):
    for _ in range(max_new_tokens):
        logits, _ = forward(P, idx[:, -cfg.block_size:], cfg)     # GPT1.py:200-202
        nxt = torch.argmax(logits[:, -1, :], dim=-1, keepdim=True)  # argmax in place of GPT1.py:208
        idx = torch.cat((idx, nxt), dim=1)                          # GPT1.py:210
    return idx
