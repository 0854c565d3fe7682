"""GPT1.py's script on charpt (GPT1.py:1-241 with encoder='base').

Hyper-parameters (GPT1.py:8-23), tokenizer and split (:25-70), get_batch (:75-83), estimate_loss
(:85-98), the training loop (:221-233), the final sample (:235-236) and the model.pth save
(:239-241), printing the reference's lines::

    python -m replicatinggpt_amd.gpt1                          # as shipped: C1 shape, lr 5e-1
    python -m replicatinggpt_amd.gpt1 --lr 2e-4 --max-iters 500 --dtype bf16

Deliberate differences from GPT1.py:

* the training step replays a hipGraph (engine.TrainStep).  The warm-up steps of its capture are
  rolled back (weights, AdamW moments and step, dropout counter, CPU generator), so iteration 0
  starts from exactly the state the reference starts from;
* estimate_loss keeps its per-batch losses on the device and reads them once per split (GPT1.py:94
  synchronises on ``loss.item()`` once per batch); each evaluation forward replays a hipGraph
  (engine.Evaluator).  The mean is taken on the host over the same float32 values, as at :95;
* dropout masks come from charpt's Philox stream, so with Dropout > 0 the loss
  curve matches the reference's within tolerance, not bit for bit (tests/test_gpu_train.py).
"""
import argparse

import torch

from . import checkpoint
from .config import PRESETS
from .data import DEFAULT_INPUT, BatchSampler, TokenStream
from .engine import Evaluator, TrainStep
from .model import BigramLanguageModel
from .optim import AdamW


@torch.no_grad()
def estimate_loss(model, sampler, eval_iters, evaluator=None):
    """GPT1.py:85-98: mean loss over ``eval_iters`` batches of each split, in eval mode."""
    out = {}
    model.eval()                                                              # :88
    dev = model.flat.master.device
    for split in ("train", "val"):                                            # :89
        losses = torch.zeros(eval_iters, dtype=torch.float32, device=dev)     # :90
        for k in range(eval_iters):                                           # :91
            if evaluator is not None:
                losses[k] = evaluator.loss(split)                             # :92-93, graph replay
            else:
                X, Y = sampler.get_batch(split)                               # :92
                _, loss = model(X, Y)                                         # :93
                losses[k] = loss                                              # :94 (no host sync)
        out[split] = losses.cpu().mean()                                      # :95
    model.train()                                                             # :96
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="GPT1.py on charpt (MI355X)")
    ap.add_argument("--preset", default="c1", choices=sorted(PRESETS), help="model shape (c1: GPT1.py as shipped)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"], help="GEMM operand / activation dtype")
    ap.add_argument("--input", default=DEFAULT_INPUT)
    ap.add_argument("--batch-size", type=int)
    ap.add_argument("--max-iters", type=int)
    ap.add_argument("--eval-interval", type=int)
    ap.add_argument("--eval-iters", type=int)
    ap.add_argument("--dropout", type=float)
    ap.add_argument("--lr", type=float, help="optimizer lr (GPT1.py:218 uses 5e-1; its learning_rate = 2e-4 is unused)")
    ap.add_argument("--max-new-tokens", type=int, default=500)
    ap.add_argument("--out", default="model.pth", help="state dict file (GPT1.py:240); '' to skip")
    ap.add_argument("--save-checkpoint", default=None, help="also write a resumable training checkpoint")
    ap.add_argument("--resume", default=None, help="continue from a --save-checkpoint file")
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of hipGraph replay")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    print(torch.cuda.is_available())                                          # GPT1.py:7
    if not torch.cuda.is_available():
        raise SystemExit("charpt: the GPT1 driver needs an AMD GPU (HIP); the hot path has no CPU version")
    device = "cuda"
    over = {k: v for k, v in dict(batch_size=a.batch_size, max_iters=a.max_iters, eval_interval=a.eval_interval,
                                  eval_iters=a.eval_iters, dropout=a.dropout).items() if v is not None}
    cfg = PRESETS[a.preset].with_(dtype=a.dtype, **over)
    torch.manual_seed(cfg.seed)                                               # GPT1.py:10
    tok, stream = TokenStream.from_file(a.input, device=device)               # GPT1.py:25-70
    cfg = cfg.with_(vocab_size=tok.vocab_size)
    model = BigramLanguageModel(cfg)                                          # GPT1.py:215
    m = model.to(device)                                                      # GPT1.py:216
    optimizer = AdamW(m.parameters(), lr=a.lr if a.lr is not None else cfg.optimizer_lr)   # GPT1.py:218
    sampler = BatchSampler(stream, cfg.block_size, cfg.batch_size)           # GPT1.py:75-83
    start = checkpoint.load_checkpoint(a.resume, m, optimizer) if a.resume else 0
    step = TrainStep(m, optimizer, sampler, use_graph=not a.no_graph)
    step.capture(restore=True)
    evaluator = Evaluator(m, sampler, use_graph=not a.no_graph)
    for it in range(start, cfg.max_iters):                                    # GPT1.py:221
        if it % cfg.eval_interval == 0:                                       # GPT1.py:223
            losses = estimate_loss(m, sampler, cfg.eval_iters, evaluator)     # GPT1.py:224
            print(f"step {it} : train loss {losses['train']:.4f}, val loss = {losses['val']:.4f}",  # GPT1.py:225
                  flush=True)
        step.step()                                                           # GPT1.py:227-233
    if a.save_checkpoint:
        checkpoint.save_checkpoint(a.save_checkpoint, m, optimizer, cfg.max_iters)
    context = torch.zeros((1, 1), dtype=torch.long, device=device)            # GPT1.py:235
    print(tok.decode(m.generate(context, max_new_tokens=a.max_new_tokens)[0].tolist()))   # GPT1.py:236
    if a.out:
        checkpoint.save_model(m, a.out)                                       # GPT1.py:239-241
    return m


if __name__ == "__main__":
    main()
