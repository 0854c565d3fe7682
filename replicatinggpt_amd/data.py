"""Tokenizer, train/val split and get_batch (GPT1.py:25-83), MI355X-side.

* ``CharTokenizer`` -- the ``encoder == 'base'`` branch (GPT1.py:54-66): sorted character
  vocabulary, encode/decode.  (The tiktoken/nltk branches need the network and are out of scope,
  SURVEY §0.)
* ``TokenStream`` -- the int64 token tensor and its 90/10 split (GPT1.py:66-70), kept resident in
  HBM as uint8 (the vocabulary has 65 symbols).
* ``BatchSampler.get_batch`` -- GPT1.py:75-83: the offsets ``ix`` are drawn with ``torch.randint``
  on the CPU default generator exactly like the reference (so index streams are bit-identical for a
  fixed seed), then the (B,T) windows and shifted targets are gathered on the device by a HIP
  kernel instead of 2*B Python slices + stack + H2D copy.  With data parallelism every rank draws the
  same global ``B*W`` offsets and keeps its own slice (one draw of B*W == W consecutive reference
  draws).
"""
import os

import torch

from . import ops

DEFAULT_INPUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "input.txt")


class CharTokenizer:
    def __init__(self, text):
        self.chars = sorted(list(set(text)))               # GPT1.py:58
        self.vocab_size = len(self.chars)                   # GPT1.py:59
        self.stoi = {ch: i for i, ch in enumerate(self.chars)}   # GPT1.py:61
        self.itos = {i: ch for i, ch in enumerate(self.chars)}   # GPT1.py:62

    def encode(self, s):
        return [self.stoi[c] for c in s]                    # GPT1.py:63

    def decode(self, ids):
        return "".join([self.itos[i] for i in ids])          # GPT1.py:64


class TokenStream:
    def __init__(self, data, device=None):
        self.data = data                                    # int64 CPU, GPT1.py:66
        n = int(0.9 * len(data))                            # GPT1.py:68
        self.n = n
        self.train_cpu = data[:n]                           # GPT1.py:69
        self.val_cpu = data[n:]                             # GPT1.py:70
        self.device = None
        self.train_dev = self.val_dev = None
        if device is not None:
            self.to(device)

    def to(self, device):
        device = torch.device(device)
        self.device = device
        dt = torch.uint8 if int(self.data.max()) < 256 else torch.int64
        self.train_dev = self.train_cpu.to(dt).to(device)
        self.val_dev = self.val_cpu.to(dt).to(device)
        return self

    @classmethod
    def from_file(cls, path=DEFAULT_INPUT, device=None):
        with open(path, "r", encoding="utf-8") as f:        # GPT1.py:26-27,55-56
            text = f.read()
        tok = CharTokenizer(text)
        data = torch.tensor(tok.encode(text), dtype=torch.long)
        return tok, cls(data, device)

    @classmethod
    def synthetic(cls, n_tokens=1 << 20, vocab=65, seed=1337, device=None):
        """SURVEY §8d synthetic stream: randint(65, (2^20,)) on a seeded private generator."""
        g = torch.Generator().manual_seed(seed)
        return cls(torch.randint(vocab, (n_tokens,), generator=g, dtype=torch.long), device)


class BatchSampler:
    def __init__(self, stream, block_size, batch_size, world_size=1, rank=0, generator=None):
        self.s = stream
        self.T = block_size
        self.B = batch_size
        self.W = world_size
        self.rank = rank
        self.generator = generator
        self._ring = None
        self._ring_i = 0

    def _staging(self, dev):
        """Ring of pinned host buffers; an event per slot keeps a host write behind the H2D copy
        that last read the slot (no stream-wide synchronisation)."""
        if self._ring is None:
            pin = dev.type == "cuda"
            self._ring = [(torch.empty(self.B, dtype=torch.int64, pin_memory=pin), None) for _ in range(4)]
        i = self._ring_i
        self._ring_i = (i + 1) % len(self._ring)
        buf, ev = self._ring[i]
        if ev is not None:
            ev.synchronize()
        return i, buf

    def draw_ix(self, split):
        """GPT1.py:78 -- global draw of B*W offsets on the CPU generator (rank-sliced)."""
        n = len(self.s.train_cpu if split == "train" else self.s.val_cpu)
        ix = torch.randint(n - self.T, (self.B * self.W,), generator=self.generator)
        return ix[self.rank * self.B:(self.rank + 1) * self.B]

    def get_batch(self, split, out=None):
        ix = self.draw_ix(split)
        data = self.s.train_dev if split == "train" else self.s.val_dev
        dev = data.device
        i, buf = self._staging(dev)
        buf.copy_(ix)
        ix_dev = buf.to(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring[i] = (buf, ev)
        if out is None:
            x = torch.empty((self.B, self.T), dtype=torch.int64, device=dev)
            y = torch.empty((self.B, self.T), dtype=torch.int64, device=dev)
        else:
            x, y = out
        ops.gather_batch(data, ix_dev, x, y)
        return x, y
