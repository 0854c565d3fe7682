"""model.pth interop and resumable training checkpoints (GPT1.py:239-241).

* ``save_model`` / ``load_model`` -- the reference's own format, ``torch.save(m.state_dict(), f)``
  (GPT1.py:240-241): 210 fp32 tensors including the 36 ``tril`` buffers.  A file GPT1.py writes
  loads here and the reverse.  Loading never executes code from the file (``weights_only=True``).
* ``save_checkpoint`` / ``load_checkpoint`` -- what the reference lacks (it saves the final weights
  only, so a run cannot resume): the state dict above, the optimizer in torch.optim.AdamW's own
  format (optim.AdamW.state_dict), the iteration, the CPU generator that get_batch draws from
  (GPT1.py:78) and the device dropout-call counter.  A resumed run draws the same batch offsets and
  dropout masks as an uninterrupted one (tests/test_gpu_train.py).
"""
import dataclasses

import torch

FORMAT = "charpt-train-checkpoint/1"


def save_model(model, path):
    """GPT1.py:239-241."""
    with open(path, "wb") as f:
        torch.save(model.state_dict(), f)


def load_model(model, path, strict=True):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return model.load_state_dict(sd, strict=strict)


def save_checkpoint(path, model, optimizer, iteration, generator=None):
    """``generator``: the CPU generator get_batch draws from (None: torch's default generator, as
    GPT1.py:78 uses)."""
    payload = {
        "format": FORMAT,
        "iter": int(iteration),
        "model": model.state_dict(),
        "optimizer": optimizer.state_dict(),
        "cpu_rng": generator.get_state() if generator is not None else torch.get_rng_state(),
        "dropout_counter": model._rng_counter.detach().cpu().clone(),
        "config": dataclasses.asdict(model.config),
    }
    torch.save(payload, path)


def load_checkpoint(path, model, optimizer=None, generator=None):
    """Restore what save_checkpoint wrote; returns the iteration to continue from."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(ck, dict) or ck.get("format") != FORMAT:
        raise ValueError(f"{path}: not a charpt training checkpoint (a bare model.pth loads with load_model)")
    model.load_state_dict(ck["model"])
    if optimizer is not None:
        optimizer.load_state_dict(ck["optimizer"])
    with torch.no_grad():
        model._rng_counter.copy_(ck["dropout_counter"])
    if generator is not None:
        generator.set_state(ck["cpu_rng"])
    else:
        torch.set_rng_state(ck["cpu_rng"])
    return int(ck["iter"])
