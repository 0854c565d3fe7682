"""bench.py's N-rank launch on CPU (no GPU touched): `python bench.py --gpus N --dry-run` must start
N ranks itself (torch.distributed.run, gloo), each with its own RANK / LOCAL_RANK, slice the global
get_batch draw by rank (GPT1.py:75-83 drawn once for B*W), time between barriers, and
print exactly ONE JSON line with n_gpus = N."""
import json
import os
import re
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=timeout, env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "4"])
    assert r.returncode == 0, r.stderr[-3000:]
    # gloo's own C++ logging may share stdout; the contract is one JSON line
    lines = [ln for ln in r.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["config"]["world_size"] == n and out["config"]["backend"] == "gloo"
    assert out["config"]["global_batch"] == 4 * n and out["steps"] == 3
    seen = re.findall(r"\[rank (\d+) local (\d+) world (\d+)\] first offsets (\[[^\]]*\]) grad ([0-9.]+)", r.stderr)
    assert sorted((int(a), int(b), int(c)) for a, b, c, _, _ in seen) == [(i, i, n) for i in range(n)]
    # every rank's first offsets are its slice of ONE global draw of B*W (seed 1337, 2^16 stream)
    gen = torch.Generator().manual_seed(1337)
    full = torch.randint(int(0.9 * (1 << 16)) - 256, (4 * n,), generator=gen)
    for rank, _, _, offs, g in seen:
        assert json.loads(offs) == full[int(rank) * 4:int(rank) * 4 + 4].tolist()
        assert float(g) == pytest.approx(sum(range(1, n + 1)) / n)   # all-reduce AVG of (rank + 1)


def test_bench_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_single_rank_dry_run():
    r = _run(["--dry-run", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 1
