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
        q.put((rank, [m.tolist() for m in mine], g.tolist(), len(red.buckets)))
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
        r, ix, g, nb = q.get(timeout=120)
        res[r] = (ix, g, nb)
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
