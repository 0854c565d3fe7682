"""bench.py's data-parallel path run end to end on one GPU, so that the first
8-GPU lease runs code that has already executed.  `python bench.py --gpus 2` becomes the launcher
(torch.distributed.run, two ranks on 127.0.0.1); with the test hooks CHARPT_DP_BACKEND=gloo and
CHARPT_DP_ONE_DEVICE=1 both ranks share cuda:0 and average their gradients over gloo (GradReducer's
SUM + divide branch) instead of RCCL.  Exercised: the rank-sliced sampler (GPT1.py:75-83), the
segmented backward graphs with the per-segment bucketed all-reduce (engine.TrainStep overlap), the
barriers and max-over-ranks timing around the timed region, the rank-0 census and in-step probe
between the barriers, and the one-line JSON contract."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_dp_two_ranks_on_one_gpu():
    env = dict(os.environ, CHARPT_DP_BACKEND="gloo", CHARPT_DP_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-generate"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 prints ONE line, rank 1 none
    res = json.loads(lines[0])
    print(json.dumps({k: res[k] for k in ("n_gpus", "ms_per_step", "value")}), res["config"])
    assert res["n_gpus"] == 2 and res["config"]["world_size"] == 2
    assert res["config"]["backend"] == "gloo" and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 128
    assert res["config"]["step_path"].startswith("segmented backward graphs")
    assert res["config"]["grad_allreduce"].startswith("gloo SUM + divide overlapped: 3 backward segments")
    assert res["value"] > 0 and res["ms_per_step"] > 0
    assert res["roofline"] is not None and res["roofline"]["frac"] > 0
    assert res["final_loss"] == res["final_loss"]   # not NaN
