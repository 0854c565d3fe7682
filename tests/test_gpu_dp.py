"""Data-parallel equivalence on one MI355X (SURVEY §4 tier 4, §8e): W = 2 ranks emulated as two
processes sharing cuda:0, each running the real engine.TrainStep DP path -- rank-sliced sampler
from one global draw (GPT1.py:78), segmented backward captured as hipGraph segments, per-segment
bucketed gradient all-reduce (gloo here; RCCL over xGMI on a node), AdamW (GPT1.py:232-233) --
against the W = 1 step on the concatenated batch.  Dropout 0 and the exact fp32 path, so the
averaged gradients and the updated weights must agree to fp32 summation-order rounding."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
STEPS, B_RANK, WORLD = 3, 4, 2


def _cfg():
    from replicatinggpt_amd import GPTConfig
    return GPTConfig(block_size=64, n_embd=64, n_head=2, n_layers=3, dropout=0.0, dtype="fp32",
                     batch_size=B_RANK)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(world, rank, batch, group_init=None):
    from replicatinggpt_amd import AdamW, BigramLanguageModel
    from replicatinggpt_amd.data import BatchSampler, TokenStream
    from replicatinggpt_amd.engine import GradReducer, TrainStep
    cfg = _cfg()
    torch.manual_seed(1337)
    model = BigramLanguageModel(cfg).to("cuda")
    opt = AdamW(model.parameters(), lr=1e-3).attach(model)
    sampler = BatchSampler(TokenStream.synthetic(n_tokens=1 << 16, device="cuda"), cfg.block_size, batch,
                           world_size=world, rank=rank, generator=torch.Generator().manual_seed(5))
    reducer = GradReducer(model.flat.grad, bucket_bytes=64 << 10) if world > 1 else None
    step = TrainStep(model, opt, sampler, reducer, use_graph=True, seg_layers=1)
    step.capture(restore=True)
    losses = [float(step.step().detach()) for _ in range(STEPS)]
    torch.cuda.synchronize()
    return losses, model.flat.master.detach().cpu().clone(), len(step.g_seg), model.config.dropout_seed


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.cuda.set_device(0)
        q.put((rank,) + _train(WORLD, rank, B_RANK))
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_equal_one_rank_on_concatenated_batch():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(WORLD):
            r, losses, master, nseg, seed = q.get(timeout=300)
            res[r] = (losses, master, nseg, seed)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    want_losses, want_master, nseg1, seed1 = _train(1, 0, WORLD * B_RANK)
    assert nseg1 == 0 and res[0][2] == res[1][2] == 3          # W=1: one graph; W=2: 3 backward segments
    # the engine gives each rank its own dropout key (rank 0 keeps the base stream)
    assert res[0][3] == seed1 and res[1][3] == seed1 + 7919
    # replicas stay identical: every rank applied the same averaged gradient
    assert torch.equal(res[0][1], res[1][1])
    scale = float(want_master.abs().max())
    assert float((res[0][1] - want_master).abs().max()) / scale < 1e-5
    for i in range(STEPS):   # global loss = mean of the two ranks' means (equal token counts)
        got = 0.5 * (res[0][0][i] + res[1][0][i])
        assert abs(got - want_losses[i]) < 1e-5 * max(1.0, abs(want_losses[i])), (i, got, want_losses[i])
