"""charpt -- MI355X-native char-level GPT training / generation hot path of
ChaitIITB/ReplicatingGPT GPT1.py (HIP kernels for gfx950 behind torch.library ops)."""
from .config import GPTConfig, PRESETS, get_default, set_default
from .model import BigramLanguageModel, Block, FeedForward, Head, LayerNorm, Linear, MultiHeadAttention
from .optim import AdamW

__all__ = ["GPTConfig", "PRESETS", "get_default", "set_default", "BigramLanguageModel", "Block", "FeedForward",
           "Head", "LayerNorm", "Linear", "MultiHeadAttention", "AdamW"]
