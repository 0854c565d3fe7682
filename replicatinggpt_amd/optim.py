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
        self._psteps = None   # per-parameter step counts, once a step skipped some parameter
        self._early = None    # flat (offset, n) ranges updated early this step (functional.EARLY)
        self._poisoned = None  # why the state is half a step ahead (a failed backward after early updates ran)

    # the model whose flat store holds these parameters is found from the parameters, so
    # ``AdamW(m.parameters(), lr=5e-1)`` works exactly as GPT1.py:218 writes it
    def _find_store(self):
        for g in self.param_groups:
            for p in g["params"]:
                st = getattr(p, "_charpt_store", None)
                if st is not None:
                    return st
        return None

    def attach(self, model=None):
        """Bind to a BigramLanguageModel's flat storage (found from the parameters when ``model``
        is None).  The optimizer must own exactly that model's parameters, in one group."""
        st = model.flat if model is not None else self._find_store()
        if st is None:
            raise RuntimeError("charpt AdamW: the parameters do not belong to a charpt BigramLanguageModel")
        ids = {id(p) for g in self.param_groups for p in g["params"]}
        if {id(p) for p in st.params()} != ids or len(self.param_groups) != 1:
            raise ValueError("charpt AdamW: the optimizer must own exactly the model's parameters in one group")
        self._store = st
        self._m = torch.zeros_like(st.master)
        self._v = torch.zeros_like(st.master)
        self._step_t = torch.zeros(1, dtype=torch.int64, device=st.master.device)
        self._psteps = None
        return self

    def _ensure(self):
        if self._store is None:
            self.attach()
        st = self._store
        if self._m.device != st.master.device:
            self._m = self._m.to(st.master.device)
            self._v = self._v.to(st.master.device)
            self._step_t = self._step_t.to(st.master.device)
            if self._psteps is not None:
                self._psteps = self._psteps.to(st.master.device)

    # -- early updates (functional.EarlyAdam, engine.TrainStep) -----------------------------------
    def _args(self):
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        return (float(grp["lr"]), float(b1), float(b2), float(grp["eps"]), float(grp["weight_decay"]))

    def early_ok(self):
        """One step count for every parameter, all of them trained, flat buffers on the GPU."""
        self._ensure()
        return (self._psteps is None and self._store.master.is_cuda and
                all(p.requires_grad for g in self.param_groups for p in g["params"]))

    def _check_poisoned(self):
        if self._poisoned is not None:
            raise RuntimeError(f"charpt AdamW: {self._poisoned}; load a checkpoint (load_state_dict) to continue")

    def early_begin(self):
        """The step count for this step, on the device, before any early update reads it."""
        self._check_poisoned()
        ops.counter_add(self._step_t, 1)
        self._early = []

    def early_abort(self, updates_taken):
        """The backward of a step with early updates failed and its deferred work was discarded
        (functional.DEFER).  No update ran (``updates_taken`` == 0): the step count goes back and the
        state is exactly as before the step.  Otherwise some weight matrices already took this step's
        update and the rest did not: the optimizer refuses further steps until its state is reloaded."""
        if self._early is None:
            return
        self._early = None
        if updates_taken == 0:
            ops.counter_add(self._step_t, -1)
        else:
            self._poisoned = (f"a failed backward left a half-applied step ({updates_taken} weight-matrix updates "
                              "ran beside it, the rest did not)")

    def early_region(self, region):
        """Queue the update of one packed region whose gradient is final (cg_adamw_defer)."""
        st = self._store
        off = (region.slot.data_ptr() - st.grad.data_ptr()) // st.grad.element_size()
        n = region.slot.numel()
        if off < 0 or off + n > st.numel or n % 4 or off % 4:
            return
        Fn.DEFER.note_stream()   # the job sits on this stream's deferral queue until a GEMM takes it / the flush
        ops.adamw_defer(st.master[off:off + n], st.grad[off:off + n], self._m[off:off + n], self._v[off:off + n],
                        st.shadow[off:off + n], *self._args(), self._step_t)
        self._early.append((off, n))

    def _rest_segments_of(self, early):
        segs, pos = [], 0
        for off, n in sorted(early):
            if off > pos:
                segs += [pos, off - pos]
            pos = max(pos, off + n)
        if pos < self._store.numel:
            segs += [pos, self._store.numel - pos]
        return segs

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
        self._check_poisoned()
        Fn.SIDE.join()   # weight gradients computed on the side stream must be final
        st = self._store
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        # gradients must sit in the flat slots; copy strays in (rare: user-assigned grads)
        missing = []
        for r in st.regions.values():
            for p, off in r.parts:
                if p.grad is None:
                    missing.append(p)
                    continue
                slot = r.slot.view(-1)[off:off + p.numel()].view(p.shape)
                if p.grad.data_ptr() != slot.data_ptr():
                    slot.copy_(p.grad)
        args = (float(grp["lr"]), float(b1), float(b2), float(grp["eps"]), float(grp["weight_decay"]))
        if self._early is not None:
            # the step count was advanced when the backward began and the weight matrices were
            # updated beside the backward's GEMMs (functional.EarlyAdam): the rest, same arithmetic
            early, self._early = self._early, None
            if missing:
                self._early_step_with_missing(early, missing, args)
                st._shadow_version = st.version()
                return loss
            segs = self._rest_segments_of(early)
            if len(segs) // 2 <= 64:
                ops.adamw_segments(st.master, st.grad, self._m, self._v, st.shadow, segs, *args, self._step_t)
            else:
                for i in range(0, len(segs), 2):
                    a, n = segs[i], segs[i + 1]
                    ops.adamw(st.master[a:a + n], st.grad[a:a + n], self._m[a:a + n], self._v[a:a + n],
                              st.shadow[a:a + n], *args, self._step_t)
        elif not missing and self._psteps is None:
            # the training path: every parameter has a gradient, one launch over the flat buffers
            ops.counter_add(self._step_t, 1)
            ops.adamw(st.master, st.grad, self._m, self._v, st.shadow, *args, self._step_t)
        else:
            # torch.optim.AdamW skips parameters whose .grad is None (no decay, no moment update,
            # no step count): per-parameter launches over the flat slices, per-parameter step counts
            self._split_steps()
            skip = {id(p) for p in missing}
            for i, p, off in self._param_slices():
                if id(p) in skip:
                    continue
                n = p.numel()
                step = self._psteps[i:i + 1]
                ops.counter_add(step, 1)
                ops.adamw(st.master[off:off + n], st.grad[off:off + n], self._m[off:off + n], self._v[off:off + n],
                          st.shadow[off:off + n], *args, step)
        st._shadow_version = st.version()
        return loss

    def _early_step_with_missing(self, early, missing, args):
        """A step with early updates in which some parameters had no gradient (torch.optim.AdamW
        skips those: no decay, no moment update, no step count).  The early updates ran with the
        shared count, already advanced; switch to per-parameter counts, take the advance back for
        the skipped parameters and update the remaining ones one by one with their own counts.  A
        parameter whose .grad was dropped AFTER its region's early update (weights and moments already
        advanced from the flat gradient) keeps the advance: taking the count back would leave it
        inconsistent with its moments; it stepped as if its gradient had stayed."""
        st = self._store
        self._split_steps()   # every count already includes this step's advance
        skip = {id(p) for p in missing}
        for i, p, off in self._param_slices():
            updated = any(a <= off < a + n for a, n in early)
            if id(p) in skip and not updated:
                ops.counter_add(self._psteps[i:i + 1], -1)
                continue
            if updated:
                continue   # updated beside the backward
            n = p.numel()
            ops.adamw(st.master[off:off + n], st.grad[off:off + n], self._m[off:off + n], self._v[off:off + n],
                      st.shadow[off:off + n], *args, self._psteps[i:i + 1])

    def _split_steps(self):
        """Switch to per-parameter step counts (first step on which some parameter had no grad)."""
        if self._psteps is None:
            n = len(self.param_groups[0]["params"])
            self._psteps = self._step_t.repeat(n).contiguous()

    # -- checkpoints: torch.optim.AdamW's own state-dict layout ------------------------------
    def _param_slices(self):
        """(index in the group, parameter, element offset in the flat buffers) per parameter."""
        st = self._store
        base = st.master.data_ptr()
        for i, p in enumerate(self.param_groups[0]["params"]):
            yield i, p, (p.data_ptr() - base) // st.master.element_size()

    def state_dict(self):
        """``{"state": {i: {step, exp_avg, exp_avg_sq}}, "param_groups": [...]}`` exactly as
        torch.optim.AdamW writes it, so optimizer state moves between the two in either direction.
        Like torch, no per-parameter entries exist before the first step."""
        self._ensure()
        grp = self.param_groups[0]
        groups = [{"lr": grp["lr"], "betas": tuple(grp["betas"]), "eps": grp["eps"],
                   "weight_decay": grp["weight_decay"], "amsgrad": False, "maximize": False, "foreach": None,
                   "capturable": False, "differentiable": False, "fused": None, "decoupled_weight_decay": True,
                   "params": list(range(len(grp["params"])))}]
        state = {}
        steps = self._psteps.tolist() if self._psteps is not None else None
        step_all = int(self._step_t.item())
        for i, p, off in self._param_slices():
            step = steps[i] if steps is not None else step_all
            if step > 0:
                n = p.numel()
                state[i] = {"step": torch.tensor(float(step)),
                            "exp_avg": self._m[off:off + n].view(p.shape).clone(),
                            "exp_avg_sq": self._v[off:off + n].view(p.shape).clone()}
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, state_dict):
        grp = self.param_groups[0]
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(grp["params"]):
            raise ValueError("charpt AdamW: the state dict does not match this optimizer's parameter group")
        for k in ("lr", "betas", "eps", "weight_decay"):
            grp[k] = groups[0][k]
        if groups[0].get("amsgrad") or groups[0].get("maximize"):
            raise ValueError("charpt AdamW: amsgrad / maximize state cannot be resumed by the fused kernel")
        self._ensure()
        ids = groups[0]["params"]
        steps = []
        with torch.no_grad():
            self._m.zero_()
            self._v.zero_()
            for i, p, off in self._param_slices():
                s = state_dict["state"].get(ids[i])
                if s is None:
                    steps.append(0)
                    continue
                n = p.numel()
                self._m[off:off + n].copy_(s["exp_avg"].reshape(-1))
                self._v[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
                steps.append(int(float(s["step"])))
        self._poisoned = None
        if len(set(steps)) <= 1:
            self._psteps = None
            self._step_t.fill_(steps[0] if steps else 0)
        else:   # parameters that skipped steps (grad None) resume with their own counts
            self._psteps = torch.tensor(steps, dtype=torch.int64, device=self._step_t.device)
