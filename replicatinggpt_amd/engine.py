"""Training-step executor: one iteration of GPT1.py's loop (GPT1.py:227-233) -- get_batch,
forward, zero_grad, backward, [data-parallel gradient all-reduce], AdamW -- replayed from
hipGraphs so the ~150 kernel launches of a step cost one graph launch instead of ~150 Python
dispatches.

Single GPU: the whole step (forward + backward + optimizer) is one graph.
Data parallel: forward + backward is one graph; the flat fp32 gradient buffer is averaged with
bucketed RCCL all-reduces (dist.ReduceOp.AVG over xGMI); the optimizer step is a second graph.
"""
import torch
import torch.distributed as dist


class GradReducer:
    """Averages the model's flat gradient buffer across ranks in fixed-size buckets."""

    def __init__(self, flat_grad, bucket_bytes=32 << 20, group=None):
        self.flat = flat_grad
        self.group = group
        n = flat_grad.numel()
        per = max(1, bucket_bytes // flat_grad.element_size())
        # reverse order: the backward finishes the last layers' gradients first
        self.buckets = [(max(0, e - per), e) for e in range(n, 0, -per)]
        self.world = dist.get_world_size(group)
        self.avg_native = dist.get_backend(group) == "nccl"

    def all_reduce(self):
        if self.world == 1:
            return
        works = []
        for s, e in self.buckets:
            op = dist.ReduceOp.AVG if self.avg_native else dist.ReduceOp.SUM
            works.append(dist.all_reduce(self.flat[s:e], op=op, group=self.group, async_op=True))
        for w in works:
            w.wait()
        if not self.avg_native:
            self.flat.div_(self.world)


class TrainStep:
    def __init__(self, model, optimizer, sampler, reducer=None, use_graph=True):
        self.model, self.opt, self.sampler, self.reducer = model, optimizer, sampler, reducer
        dev = model.flat.master.device
        B, T = sampler.B, sampler.T
        self.x = torch.empty((B, T), dtype=torch.int64, device=dev)
        self.y = torch.empty((B, T), dtype=torch.int64, device=dev)
        self.use_graph = use_graph and dev.type == "cuda"
        self.g_fb = self.g_opt = None
        self.loss = None

    def _fwd_bwd(self):
        _, loss = self.model(self.x, self.y)           # GPT1.py:230
        self.opt.zero_grad(set_to_none=True)           # GPT1.py:231
        loss.backward()                                # GPT1.py:232
        return loss

    def _eager(self):
        loss = self._fwd_bwd()
        if self.reducer is not None:
            self.reducer.all_reduce()
        self.opt.step()                                # GPT1.py:233
        return loss

    def capture(self, warmup=2):
        if not self.use_graph:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.sampler.get_batch("train", out=(self.x, self.y))
                self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.opt.zero_grad(set_to_none=True)
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

    def step(self):
        self.sampler.get_batch("train", out=(self.x, self.y))   # GPT1.py:227
        if self.g_fb is None:
            self.loss = self._eager()
            return self.loss
        self.g_fb.replay()
        if self.reducer is not None:
            self.reducer.all_reduce()
            self.g_opt.replay()
        return self.loss
