"""Data-parallel host logic on CPU with the gloo backend (world_size 2): rank-sliced batch
offsets equal the single-stream reference draws, and the bucketed flat-gradient all-reduce
averages exactly like a single-process mean."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import golden_path


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from replicatinggpt_amd.data import BatchSampler, TokenStream
        from replicatinggpt_amd.engine import GradReducer
        # sampler: every rank draws the same global B*W offsets and keeps its slice
        ts = TokenStream.synthetic(n_tokens=1 << 16)
        s = BatchSampler(ts, 32, 4, world_size=world, rank=rank, generator=torch.Generator().manual_seed(7))
        mine = [s.draw_ix("train") for _ in range(3)]
        # reducer: flat grads, small buckets to exercise bucketing
        g = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        red = GradReducer(g, bucket_bytes=1024)
        red.all_reduce()
        # overlapped form (engine.TrainStep DP path): per-segment ranges launched async, then finished
        g2 = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        red2 = GradReducer(g2, bucket_bytes=1024)
        ranges = [(700, 1000), (250, 700), (0, 250)]
        works = []
        for r0, r1 in ranges:
            works += red2.launch(r0, r1)
        red2.finish(works, ranges)
        q.put((rank, [m.tolist() for m in mine], g.tolist(), len(red.buckets), g2.tolist(), len(works)))
    finally:
        dist.destroy_process_group()


def test_dp_sampler_and_reducer_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(world):
        r, ix, g, nb, g2, nw = q.get(timeout=120)
        res[r] = (ix, g, nb, g2, nw)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-stream equivalent: one draw of B*W per step
    gen = torch.Generator().manual_seed(7)
    n = int(0.9 * (1 << 16))
    for step in range(3):
        full = torch.randint(n - 32, (8,), generator=gen)
        for r in range(world):
            assert res[r][0][step] == full[r * 4:(r + 1) * 4].tolist()
    want = (torch.arange(1000, dtype=torch.float32) * 1.5).tolist()
    for r in range(world):
        assert res[r][1] == want
        assert res[r][2] == 4
        assert res[r][3] == want          # segmented launch/finish == one-shot average
        assert res[r][4] == 2 + 2 + 1     # 256-element buckets inside each range


def test_segment_plan_partitions_flat_buffer():
    """The DP overlap cuts (engine.segment_plan) give contiguous flat-gradient ranges that tile the
    whole buffer, each ending on a block boundary, head range first (backward order)."""
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    from replicatinggpt_amd.engine import segment_plan
    cfg = GPTConfig(block_size=32, n_embd=64, n_head=2, n_layers=5, dropout=0.0, dtype="bf16")
    m = BigramLanguageModel(cfg)
    starts = m.flat.block_starts()
    assert len(starts) == 5 and starts == sorted(starts)
    for seg in (1, 2, 3):
        cuts, ranges = segment_plan(m, seg)
        assert cuts == list(range(5 - seg, 0, -seg))
        assert ranges[0][1] == m.flat.numel and ranges[-1][0] == 0
        for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
            assert b1 == a0 and a0 > b0
        assert [r[0] for r in ranges[:-1]] == [starts[c] for c in cuts]
        # every parameter falls in exactly one range, and a block's parameters in one range
        for l, blk in enumerate(m.blocks):
            offs = [p.data_ptr() for p in blk.parameters()]
            base = m.flat.master.data_ptr()
            idx = {next(i for i, (r0, r1) in enumerate(ranges) if r0 <= (o - base) // 4 < r1) for o in offs}
            assert len(idx) == 1


def _avg_worker(rank, world, port, q):
    """GradReducer's RCCL branch (avg_native: backend "nccl" -> one all_reduce(AVG), no division
    afterwards) run under gloo with the backend query and the collective replaced by a fake that
    implements AVG as SUM / world -- the op, bucket ranges and finish() arithmetic the RCCL path
    takes, on CPU."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from replicatinggpt_amd import engine
        seen = []
        real_all_reduce, real_backend = dist.all_reduce, dist.get_backend

        def fake_all_reduce(t, op=None, group=None, async_op=False):
            seen.append(op)
            assert op == dist.ReduceOp.AVG
            w = real_all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)
            w.wait()
            t.div_(world)

            class _Done:
                def wait(self):
                    return True
            return _Done()

        engine.dist.all_reduce = fake_all_reduce
        engine.dist.get_backend = lambda group=None: "nccl"
        try:
            g = torch.arange(1000, dtype=torch.float32) * (rank + 1)
            red = engine.GradReducer(g, bucket_bytes=1024)
            assert red.avg_native
            ranges = [(700, 1000), (0, 700)]
            works = []
            for r0, r1 in ranges:
                works += red.launch(r0, r1)
            red.finish(works, ranges)          # must not divide a second time
        finally:
            engine.dist.all_reduce, engine.dist.get_backend = real_all_reduce, real_backend
        q.put((rank, g.tolist(), len(seen)))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_avg_native_branch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, g, n = q.get(timeout=120)
        res[r] = (g, n)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = (torch.arange(1000, dtype=torch.float32) * 1.5).tolist()
    for r in range(world):
        assert res[r][0] == want
        assert res[r][1] == 2 + 3          # 256-element buckets: 300 -> 2, 700 -> 3
