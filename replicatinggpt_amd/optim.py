"""Fused AdamW over the model's flat fp32 buffers (torch.optim.AdamW, GPT1.py:218,231,233).

One kernel launch updates every parameter, its two moments and the bf16 weight shadow the
GEMMs read.  The step count lives on the device, so the whole optimizer step is capturable in a
hipGraph.  Numerics follow torch/optim/adam.py ``_single_tensor_adam`` (decoupled weight decay,
bias-corrected moments, same fp32 operation order).
"""
import torch

from . import functional as Fn
from . import ops


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self._store = None
        self._m = self._v = None
        self._step_t = None

    # the model whose flat store holds these parameters is discovered lazily (after .to())
    def _find_store(self):
        from .model import BigramLanguageModel  # noqa: F401  (type only)
        ps = [p for g in self.param_groups for p in g["params"]]
        root = None
        for p in ps:
            st = getattr(p, "_charpt_store", None)
            if st is not None:
                root = st
                break
        return root, ps

    def attach(self, model):
        """Bind to a BigramLanguageModel's flat storage (call once after model.to(device))."""
        st = model.flat
        ids = {id(p) for g in self.param_groups for p in g["params"]}
        if {id(p) for p in st.params()} != ids or len(self.param_groups) != 1:
            raise ValueError("charpt AdamW: the optimizer must own exactly the model's parameters in one group")
        self._store = st
        self._m = torch.zeros_like(st.master)
        self._v = torch.zeros_like(st.master)
        self._step_t = torch.zeros(1, dtype=torch.int64, device=st.master.device)
        return self

    def _ensure(self):
        if self._store is None:
            raise RuntimeError("charpt AdamW: call .attach(model) before step()")
        st = self._store
        if self._m.device != st.master.device:
            self._m = self._m.to(st.master.device)
            self._v = self._v.to(st.master.device)
            self._step_t = self._step_t.to(st.master.device)

    def zero_grad(self, set_to_none=True):
        for g in self.param_groups:
            for p in g["params"]:
                if set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._ensure()
        Fn.SIDE.join()   # weight gradients computed on the side stream must be final
        st = self._store
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        ops.counter_add(self._step_t, 1)
        # gradients must sit in the flat slots; copy strays in (rare: user-assigned grads)
        all_in_slots = True
        for r in st.regions.values():
            for p, off in r.parts:
                slot = r.slot.view(-1)[off:off + p.numel()].view(p.shape)
                if p.grad is None:
                    slot.zero_()
                    all_in_slots = False
                elif p.grad.data_ptr() != slot.data_ptr():
                    slot.copy_(p.grad)
        ops.adamw(st.master, st.grad, self._m, self._v, st.shadow, float(grp["lr"]), float(b1), float(b2),
                  float(grp["eps"]), float(grp["weight_decay"]), self._step_t)
        st._shadow_version = st.version()
        return loss

    def state_dict(self):
        sd = super().state_dict()
        sd["charpt"] = {"m": self._m, "v": self._v, "step": self._step_t}
        return sd

    def load_state_dict(self, sd):
        extra = sd.get("charpt") if isinstance(sd, dict) else None
        if extra is not None:
            sd = {k: v for k, v in sd.items() if k != "charpt"}
        super().load_state_dict(sd)
        if extra is not None:
            self._ensure()
            self._m.copy_(extra["m"])
            self._v.copy_(extra["v"])
            self._step_t.copy_(extra["step"])
