"""Hyper-parameters of the char-level GPT (GPT1.py:8-23) as a dataclass.

The reference keeps them as module globals that its classes read at construction time; the
charpt modules take a ``GPTConfig`` (or fall back to the process-wide default, which is the
as-shipped GPT1.py configuration with ``encoder='base'``).
"""
from dataclasses import dataclass, replace


@dataclass
class GPTConfig:
    vocab_size: int = 65            # len(sorted(set(text))), GPT1.py:58-59
    block_size: int = 256           # GPT1.py:13
    n_embd: int = 126               # GPT1.py:14
    n_head: int = 6                 # GPT1.py:21
    n_layers: int = 6               # GPT1.py:22
    dropout: float = 0.2            # GPT1.py:23 ("Dropout")
    batch_size: int = 64            # GPT1.py:12
    max_iters: int = 3000           # GPT1.py:15
    eval_interval: int = 200        # GPT1.py:16
    eval_iters: int = 200           # GPT1.py:19
    learning_rate: float = 2e-4     # GPT1.py:17 (declared; the optimizer uses 5e-1, GPT1.py:218 -- SURVEY Q4)
    optimizer_lr: float = 5e-1      # GPT1.py:218, as shipped
    seed: int = 1337                # GPT1.py:10
    # charpt additions
    dtype: str = "bf16"             # activation / GEMM operand dtype: "bf16" (perf) or "fp32" (exact)
    dropout_seed: int = 0x1337      # key of the Philox dropout stream (never touches the CPU RNG)

    @property
    def head_size(self):
        return self.n_embd // self.n_head      # GPT1.py:156

    def with_(self, **kw):
        return replace(self, **kw)


# named configurations from BASELINE.json
PRESETS = {
    "c1": GPTConfig(),                                                       # GPT1.py as shipped
    "c2": GPTConfig(n_embd=384, n_head=6, n_layers=6, block_size=256, batch_size=64),
    "c4": GPTConfig(n_embd=768, n_head=12, n_layers=12, block_size=1024, batch_size=64),
}

_default = GPTConfig()


def get_default():
    return _default


def set_default(cfg):
    global _default
    _default = cfg
    return cfg
