"""TEST INFRASTRUCTURE ONLY.  numpy restatement of the counter-based dropout RNG that the
charpt HIP kernels use (replicatinggpt_amd/csrc/philox.h).

The reference draws dropout masks from torch's stateful CPU generator (nn.Dropout,
GPT1.py:107,117,146); those draws cannot be reproduced on a GPU.  charpt
replaces them with Philox4x32-10 (Salmon et al., SC'11; Random123) keyed by a per-model seed
and addressed by (stream, element index), so that forward and backward regenerate the same
mask and so that this oracle can apply the *identical* mask on the CPU.

Mask spec (shared with csrc/common.h): 16-bit decisions, 8 consecutive elements per Philox call
  group = idx >> 3, word = (idx >> 1) & 3, half = idx & 1
  ctr   = (group & 0xffffffff, group >> 32, stream & 0xffffffff, stream >> 32)
  key   = (seed & 0xffffffff, seed >> 32)
  u16   = (philox4x32_10(ctr, key)[word] >> (16 * half)) & 0xffff
  keep  = u16 >= threshold(p),  threshold = clamp(round(p * 2^16), 1, 2^16 - 1) for p > 0
  kept values are scaled by float32(1/(1-p)).  (p = 0.2: threshold 13107, keep probability
  52429/65536 = 0.7999878.)
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
    if not p > 0:
        return 0
    return min(max(int(round(p * 65536.0)), 1), 0xFFFF)


def keep_mask(seed, stream, idx, p):
    """Boolean keep-mask for element indices ``idx`` (any int array)."""
    idx = np.asarray(idx, dtype=np.uint64)
    group = idx >> np.uint64(3)
    word = ((idx >> np.uint64(1)) & np.uint64(3)).astype(np.int64)
    half = idx & np.uint64(1)
    seed = np.uint64(seed)
    stream = np.uint64(stream)
    out = philox4x32_10(group & MASK32, group >> np.uint64(32), stream & MASK32, stream >> np.uint64(32),
                        seed & MASK32, seed >> np.uint64(32))
    r = np.choose(word, out)
    u16 = (r >> (np.uint64(16) * half)) & np.uint64(0xFFFF)
    return u16 >= np.uint64(threshold(p))
