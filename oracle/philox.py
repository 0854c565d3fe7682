"""TEST INFRASTRUCTURE ONLY.  numpy restatement of the counter-based dropout RNG that the
charpt HIP kernels use (replicatinggpt_amd/csrc/philox.h).

The reference draws dropout masks from torch's stateful CPU generator (nn.Dropout,
GPT1.py:107,117,146); those draws cannot be reproduced on a GPU.  charpt
replaces them with Philox4x32-10 (Salmon et al., SC'11; Random123) keyed by a per-model seed
and addressed by (stream, element index), so that forward and backward regenerate the same
mask and so that this oracle can apply the *identical* mask on the CPU.

Mask spec (shared with csrc/philox.h):
  group = idx >> 2, word = idx & 3
  ctr   = (group & 0xffffffff, group >> 32, stream & 0xffffffff, stream >> 32)
  key   = (seed & 0xffffffff, seed >> 32)
  keep  = philox4x32_10(ctr, key)[word] >= threshold(p),  threshold = min(round(p*2^32), 2^32-1)
  kept values are scaled by float32(1/(1-p)).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over uint64 arrays holding 32-bit values."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint64) & MASK32 for v in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint64) & MASK32
    k1 = np.asarray(k1, dtype=np.uint64) & MASK32
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK32
            k1 = (k1 + W1) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return c0, c1, c2, c3


def threshold(p):
    return min(int(round(p * 4294967296.0)), 0xFFFFFFFF)


def keep_mask(seed, stream, idx, p):
    """Boolean keep-mask for element indices ``idx`` (any int array)."""
    idx = np.asarray(idx, dtype=np.uint64)
    group = idx >> np.uint64(2)
    word = (idx & np.uint64(3)).astype(np.int64)
    seed = np.uint64(seed)
    stream = np.uint64(stream)
    out = philox4x32_10(group & MASK32, group >> np.uint64(32), stream & MASK32, stream >> np.uint64(32),
                        seed & MASK32, seed >> np.uint64(32))
    r = np.choose(word, out)
    return r >= np.uint64(threshold(p))
