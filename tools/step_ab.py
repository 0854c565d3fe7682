"""Same-process interleaved A/B of training-step PATHS (engine.TrainStep variants) on one GPU:
every variant is its own model + optimizer + captured graphs; rounds time each variant's
``--steps`` replays in turn (synchronize on both sides) and report median / min ms per step, so
box drift cancels out of the comparison.

variants: single          one graph: fwd + bwd (+ early AdamW) + AdamW (the 1-GPU bench path)
          seg<k>          the DP path at W = 1: backward graph segments of k blocks, reducer, AdamW graph
          red             reducer without overlap: fwd+bwd graph, (no-op) all-reduce, AdamW graph
          <v>:<knob>=<int>  variant v captured with cg_set_tuning(knob, int) (reset to 0 after its
                           capture; the kernel choice / arguments it sets are baked into the graphs);
                           <v>:Fn.<NAME>=<int>  the same with a functional.py module switch (e.g. GEMM_LN)
usage: python tools/step_ab.py [c2|c4] single,seg1,seg2 [rounds] [steps]"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import AdamW, BigramLanguageModel, PRESETS  # noqa: E402
from replicatinggpt_amd.data import BatchSampler, TokenStream  # noqa: E402
from replicatinggpt_amd.engine import GradReducer, TrainStep  # noqa: E402


def make(variant, cfgname, dev):
    knob = None
    if ":" in variant:
        variant, kv = variant.split(":", 1)
        k, v = kv.split("=")
        knob = (k.encode(), int(v))
        if k.startswith("Fn."):
            from replicatinggpt_amd import functional as Fn
            knob = (k, getattr(Fn, k[3:]))
            setattr(Fn, k[3:], type(knob[1])(int(v)))
        else:
            from replicatinggpt_amd import _lib as L
            L.check(L.load().cg_set_tuning(knob[0], knob[1]), "tuning")
    cfg = PRESETS[cfgname].with_(dtype="bf16")
    torch.manual_seed(cfg.seed)
    model = BigramLanguageModel(cfg).to(dev)
    opt = AdamW(model.parameters(), lr=cfg.learning_rate).attach(model)
    sampler = BatchSampler(TokenStream.synthetic(device=dev), cfg.block_size, cfg.batch_size,
                           generator=torch.Generator().manual_seed(cfg.seed))
    if variant == "single":
        step = TrainStep(model, opt, sampler, None)
    elif variant == "red":
        step = TrainStep(model, opt, sampler, GradReducer(model.flat.grad), overlap=False)
    elif variant.startswith("seg"):
        step = TrainStep(model, opt, sampler, GradReducer(model.flat.grad), overlap=True,
                         seg_layers=int(variant[3:]))
    else:
        raise ValueError(variant)
    step.capture()
    if knob is not None and isinstance(knob[0], str):
        from replicatinggpt_amd import functional as Fn
        setattr(Fn, knob[0][3:], knob[1])   # restore the module switch
    elif knob is not None:
        from replicatinggpt_amd import _lib as L
        L.check(L.load().cg_set_tuning(knob[0], 1 if knob[0] == b"attn_bwd_lpt" else 0), "tuning")
    return step


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "c2"
    variants = (sys.argv[2] if len(sys.argv) > 2 else "single,seg1").split(",")
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
    dev = torch.device("cuda")
    runs = {v: make(v, cfgname, dev) for v in variants}
    for st in runs.values():
        for _ in range(10):
            st.step()
    torch.cuda.synchronize()
    res = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            st = runs[v]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                st.step()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / steps * 1e3)
        print(f"round {r}: " + "  ".join(f"{v} {res[v][-1]:.4f}" for v in variants), flush=True)
    out = {v: {"median_ms": round(statistics.median(x), 4), "min_ms": round(min(x), 4),
               "all": [round(t, 4) for t in x]} for v, x in res.items()}
    print(json.dumps({"config": cfgname, "steps_per_round": steps, "rounds": rounds, "variants": out}))


if __name__ == "__main__":
    main()
