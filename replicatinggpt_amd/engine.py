"""Training-step executor: one iteration of GPT1.py's loop (GPT1.py:227-233) -- get_batch,
forward, zero_grad, backward, [data-parallel gradient all-reduce], AdamW -- replayed from
hipGraphs so the ~230 kernel launches of a step cost a few graph launches instead of ~230 Python
dispatches.

Single GPU: the whole step (forward + backward + optimizer) is one graph.

Data parallel (one process per GPU, RCCL over xGMI): the backward is captured as SEGMENTS cut at
block boundaries (``torch.autograd.backward(..., inputs=[block input])`` stops the backward at a
residual-stream tensor; the next segment resumes from its gradient).  Parameters live in one flat
buffer laid out [embeddings | block 0 | ... | block L-1 | ln_f + lm_head], so the gradients a
segment finishes form one contiguous range of the flat gradient buffer.  After segment i's graph
is replayed, that range's ``all_reduce(AVG)`` is enqueued (async, RCCL's own stream) and segment
i+1's graph replays on the compute stream meanwhile -- the gradient all-reduce overlaps the rest
of the backward with only eager collectives (no collective is captured in a graph, so nothing
here depends on RCCL graph capture).  The optimizer is a final graph replayed after the
collectives have been waited on.
"""
import torch
import torch.distributed as dist

from . import functional as Fn


class GradReducer:
    """Averages the model's flat gradient buffer across ranks in fixed-size buckets."""

    def __init__(self, flat_grad, bucket_bytes=32 << 20, group=None):
        self.flat = flat_grad
        self.group = group
        self.per = max(1, bucket_bytes // flat_grad.element_size())
        n = flat_grad.numel()
        # reverse order: the backward finishes the last layers' gradients first
        self.buckets = [(max(0, e - self.per), e) for e in range(n, 0, -self.per)]
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.avg_native = init and dist.get_backend(group) == "nccl"

    def launch(self, start, end):
        """Async all-reduce of flat[start:end] (bucket-sized pieces); returns the work handles.
        RCCL's stream waits for the work already queued on the current stream, so this runs
        behind the graph segment that produced the range and beside whatever is queued next."""
        works = []
        if self.world == 1 or end <= start:
            return works
        op = dist.ReduceOp.AVG if self.avg_native else dist.ReduceOp.SUM
        for s in range(start, end, self.per):
            e = min(end, s + self.per)
            works.append(dist.all_reduce(self.flat[s:e], op=op, group=self.group, async_op=True))
        return works

    def finish(self, works, ranges=None):
        for w in works:
            w.wait()
        if not self.avg_native and self.world > 1:
            for s, e in (ranges or [(0, self.flat.numel())]):
                self.flat[s:e].div_(self.world)

    def all_reduce(self):
        if self.world == 1:
            return
        works = []
        for s, e in self.buckets:
            works += self.launch(s, e)
        self.finish(works)


def segment_plan(model, seg_layers):
    """Block indices where the backward is cut (descending) and, per segment, the contiguous flat
    gradient range it finalizes: segment 0 = forward + loss .. block cuts[0] (ln_f/lm_head and
    blocks cuts[0]..L-1), ..., last = blocks 0..cuts[-1]-1 + embeddings."""
    L = len(model.blocks)
    cuts = list(range(L - seg_layers, 0, -seg_layers)) if seg_layers > 0 else []
    starts = model.flat.block_starts()            # flat offset of block l's first region
    numel = model.flat.numel
    bounds = [numel] + [starts[c] for c in cuts] + [0]
    ranges = [(bounds[i + 1], bounds[i]) for i in range(len(bounds) - 1)]
    return cuts, ranges


class TrainStep:
    def __init__(self, model, optimizer, sampler, reducer=None, use_graph=True, overlap=None, seg_layers=2):
        self.model, self.opt, self.sampler, self.reducer = model, optimizer, sampler, reducer
        dev = model.flat.master.device
        B, T = sampler.B, sampler.T
        self.x = torch.empty((B, T), dtype=torch.int64, device=dev)
        self.y = torch.empty((B, T), dtype=torch.int64, device=dev)
        self.use_graph = use_graph and dev.type == "cuda"
        self.g_fb = self.g_opt = None
        self.g_seg = []
        self.loss = None
        # d loss / d loss = 1, allocated once: loss.backward() would launch a fill kernel per step
        self._one = torch.ones((), dtype=torch.float32, device=dev)
        self.overlap = (reducer is not None and reducer.world > 1) if overlap is None else bool(overlap)
        # per-rank dropout key: the replicas must not draw identical masks
        if reducer is not None and reducer.world > 1:
            model.set_dropout_rank(dist.get_rank(reducer.group))
        self.cuts, self.ranges = segment_plan(model, seg_layers) if self.overlap else ([], [])

    # -- eager ----------------------------------------------------------------------------
    def _fwd_bwd(self):
        _, loss = self.model(self.x, self.y)           # GPT1.py:230
        self.opt.zero_grad(set_to_none=True)           # GPT1.py:231
        # one rank: the weight matrices' AdamW beside the backward's GEMMs
        early = self.reducer is None and Fn.EARLY.begin(self.opt)
        try:
            with Fn.DEFER:                             # split-K reduces in later GEMMs' tails
                loss.backward(self._one)               # GPT1.py:232
        except BaseException:
            # DEFER discarded the queued work; the optimizer takes its step count back, or -- when
            # some early updates had already run -- refuses further steps (optim.AdamW.early_abort)
            if early:
                self.opt.early_abort(Fn.DEFER.aborted_adam)
            raise
        finally:
            Fn.EARLY.end()
        return loss

    def _eager(self):
        loss = self._fwd_bwd()
        if self.reducer is not None:
            self.reducer.all_reduce()
        self.opt.step()                                # GPT1.py:233
        return loss

    # -- segmented backward (DP overlap) ------------------------------------------------------
    def _forward_with_cuts(self):
        """Forward with the residual stream cut at the segment boundaries: block j (j in cuts)
        receives a detached leaf copy-free alias of its input, so each backward segment ends at a
        leaf (autograd would still run the grad_fn of a non-leaf ``inputs=`` target).
        Returns (loss, {j: (block input, leaf alias)})."""
        xs = {}

        def grab(j):
            def hook(mod, args):
                leaf = args[0].detach().requires_grad_(True)
                link = getattr(args[0], "_charpt_link", None)
                if link is not None:   # the fused gradient hand-off (functional.GradLink) spans the cut
                    leaf._charpt_link = link
                xs[j] = (args[0], leaf)
                return (leaf,) + tuple(args[1:])
            return hook
        hooks = [self.model.blocks[j].register_forward_pre_hook(grab(j)) for j in self.cuts]
        try:
            _, loss = self.model(self.x, self.y)
        finally:
            for h in hooks:
                h.remove()
        return loss, xs

    def _segment(self, i, loss, xs):
        """Backward of segment i (0 = from the loss): stops at the next cut's leaf alias, whose
        .grad the following segment feeds into the real block-input tensor."""
        with Fn.DEFER:   # flushed at the segment's end, before its gradient range is all-reduced
            if i == 0:
                torch.autograd.backward(loss, grad_tensors=self._one)
            else:
                src, leaf = xs[self.cuts[i - 1]]
                torch.autograd.backward(src, grad_tensors=leaf.grad)
        Fn.SIDE.join()

    def _eager_segmented(self):
        loss, xs = self._forward_with_cuts()
        self.opt.zero_grad(set_to_none=True)
        works = []
        for i in range(len(self.cuts) + 1):
            self._segment(i, loss, xs)
            works += self.reducer.launch(*self.ranges[i])
        self.reducer.finish(works, self.ranges)
        self.opt.step()
        return loss

    # -- capture ------------------------------------------------------------------------------
    def capture(self, warmup=2, restore=False):
        """Run ``warmup`` eager steps (allocator, kernels) and capture the step graph(s).
        restore=True rolls the warm-up steps back afterwards -- weights, AdamW moments and step,
        the dropout-call counter and the CPU generator get_batch draws from -- so the first replayed
        step is the step an eager loop would take next (the GPT1 driver needs this: its loss curve
        starts from the reference's state)."""
        if not self.use_graph:
            return
        saved = self._save_state() if restore else None
        try:
            self._capture(warmup)
        finally:
            if saved is not None:
                self._restore_state(saved)

    def _save_state(self):
        st, opt = self.model.flat, self.opt
        opt._ensure()
        gen = self.sampler.generator
        return {"master": st.master.detach().clone(), "m": opt._m.clone(), "v": opt._v.clone(),
                "step": opt._step_t.clone(), "counter": self.model._rng_counter.clone(),
                "rng": gen.get_state() if gen is not None else torch.get_rng_state()}

    def _restore_state(self, s):
        torch.cuda.synchronize()
        st, opt = self.model.flat, self.opt
        with torch.no_grad():
            st.master.copy_(s["master"])
            opt._m.copy_(s["m"])
            opt._v.copy_(s["v"])
            opt._step_t.copy_(s["step"])
            self.model._rng_counter.copy_(s["counter"])
        st.refresh_shadow()
        gen = self.sampler.generator
        if gen is not None:
            gen.set_state(s["rng"])
        else:
            torch.set_rng_state(s["rng"])
        torch.cuda.synchronize()

    def _capture(self, warmup):
        self._capture_graphs(warmup)

    def _capture_graphs(self, warmup):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.sampler.get_batch("train", out=(self.x, self.y))
                if self.overlap:
                    self._eager_segmented()
                else:
                    self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.opt.zero_grad(set_to_none=True)
        if self.overlap:
            self._capture_segmented()
            return
        self.g_fb = torch.cuda.CUDAGraph()
        if self.reducer is None:
            with torch.cuda.graph(self.g_fb):
                self.loss = self._fwd_bwd()
                self.opt.step()
        else:
            with torch.cuda.graph(self.g_fb):
                self.loss = self._fwd_bwd()
            self.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_opt, pool=self.g_fb.pool()):
                self.opt.step()
        torch.cuda.synchronize()

    def _capture_segmented(self):
        g0 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g0):
            loss, xs = self._forward_with_cuts()
            self.opt.zero_grad(set_to_none=True)
            self._segment(0, loss, xs)
        self.g_seg = [g0]
        for i in range(1, len(self.cuts) + 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=g0.pool()):
                self._segment(i, loss, xs)
            self.g_seg.append(g)
        self.g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_opt, pool=g0.pool()):
            self.opt.step()
        self.loss = loss
        self._xs = xs   # keep the segment boundary tensors (and their .grad) alive
        torch.cuda.synchronize()

    # -- one training step ----------------------------------------------------------------
    def step(self):
        self.sampler.get_batch("train", out=(self.x, self.y))   # GPT1.py:227
        if self.g_seg:
            works = []
            for i, g in enumerate(self.g_seg):
                g.replay()
                works += self.reducer.launch(*self.ranges[i])
            self.reducer.finish(works, self.ranges)
            self.g_opt.replay()
            return self.loss
        if self.g_fb is None:
            self.loss = self._eager_segmented() if self.overlap else self._eager()
            return self.loss
        self.g_fb.replay()
        if self.reducer is not None:
            self.reducer.all_reduce()
            self.g_opt.replay()
        return self.loss


class Evaluator:
    """The forward of estimate_loss (GPT1.py:92-93) replayed from one hipGraph: get_batch writes
    the batch into static buffers, the replay computes the mean loss into a static scalar.  Built
    on first use, in whatever mode the model is in then -- estimate_loss calls it in eval mode with
    autograd off (GPT1.py:85,88)."""

    def __init__(self, model, sampler, use_graph=True):
        self.model, self.sampler = model, sampler
        dev = model.flat.master.device
        self.x = torch.empty((sampler.B, sampler.T), dtype=torch.int64, device=dev)
        self.y = torch.empty_like(self.x)
        self.use_graph = use_graph and dev.type == "cuda"
        self.graph = None
        self.out = None

    def _forward(self):
        _, loss = self.model(self.x, self.y)
        return loss

    @torch.no_grad()
    def loss(self, split):
        """Draw a batch of ``split`` (one get_batch, as GPT1.py:92) and return its mean loss as a
        device scalar (valid until the next call)."""
        self.sampler.get_batch(split, out=(self.x, self.y))
        if not self.use_graph:
            return self._forward()
        if self.graph is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._forward()                 # warm-up on this batch; the replay recomputes it
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self._forward()
        self.graph.replay()
        return self.out
