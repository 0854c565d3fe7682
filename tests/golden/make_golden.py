"""Golden-vector generator for the charpt parity suite.

Runs the REFERENCE ``GPT1.py`` (read as text from ``/root/reference`` and executed via
``ast`` with the edits SURVEY.md §8c lists) on the CPU of the build container and writes
small fixtures next to this file.  It is the only code in the repository that executes
the reference; the reference itself never travels (the GPU box has no /root/reference),
only the vectors below do.

Edits applied to GPT1.py before exec (and nothing else):
  * drop ``import tiktoken`` (GPT1.py:4) and the ``print`` (GPT1.py:7);
  * ``encoder = 'base'`` (GPT1.py:20), ``device = 'cpu'`` (GPT1.py:18);
  * optional overrides of the hyper-parameter globals (GPT1.py:12-23);
  * stop before the train loop (GPT1.py:221) -- the loop, final sample and save are
    re-driven from here so that lr / iteration counts can be chosen.

Usage:  python tests/golden/make_golden.py [--skip-train]
"""
import argparse
import ast
import hashlib
import json
import os
import sys
import time

import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
# the GPT1.py these fixtures were generated from; a different file is refused (it is untrusted
# public content and is executed below)
GPT1_SHA256 = "38818880dff1983cea405e926b8e5ac06fad4cad4dac850dbdc0d58011c13a92"
# top-level statement kinds allowed to run (GPT1.py:1-216): imports of torch, the seed call, the
# hyper-parameter globals, the input read, the encoder branch, function and class definitions
_ALLOWED = (ast.Import, ast.ImportFrom, ast.Assign, ast.With, ast.If, ast.FunctionDef, ast.ClassDef)


def load_reference(overrides=None, build_model=True):
    """Exec GPT1.py up to (and optionally including) model construction (GPT1.py:215-216)."""
    ov = {"encoder": "base", "device": "cpu"}
    ov.update(overrides or {})
    raw = open(os.path.join(REF, "GPT1.py"), "rb").read()
    if hashlib.sha256(raw).hexdigest() != GPT1_SHA256:
        raise SystemExit("make_golden: /root/reference/GPT1.py differs from the pinned file; refusing to execute it")
    tree = ast.parse(raw.decode())
    body = []
    for node in tree.body:
        if node.lineno >= 218:  # optimizer (lr literal), train loop, sample, save
            break
        if isinstance(node, ast.Import) and any(a.name == "tiktoken" for a in node.names):
            continue
        if isinstance(node, ast.Expr) and ast.unparse(node).startswith("print("):
            continue
        if isinstance(node, ast.Expr) and ast.unparse(node) == "torch.manual_seed(1337)":
            body.append(node)
            continue
        if not isinstance(node, _ALLOWED):
            raise SystemExit(f"make_golden: unexpected statement at GPT1.py:{node.lineno}: {type(node).__name__}")
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            mods = [node.module] if isinstance(node, ast.ImportFrom) else [a.name for a in node.names]
            if not all(m == "torch" or m.startswith("torch.") for m in mods):
                raise SystemExit(f"make_golden: unexpected import at GPT1.py:{node.lineno}: {mods}")
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name in ("model", "m") and not build_model:
                continue
            if name in ov:
                node = ast.Assign(targets=node.targets, value=ast.Constant(ov[name]))
                ast.copy_location(node, tree.body[0])
        body.append(node)
    mod = ast.Module(body=body, type_ignores=[])
    ast.fix_missing_locations(mod)
    ns = {"__name__": "gpt1_reference"}
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        exec(compile(mod, os.path.join(REF, "GPT1.py"), "exec"), ns)
    finally:
        os.chdir(cwd)
    return ns


class RandintRecorder:
    """Records every torch.randint result (get_batch's only RNG draw, GPT1.py:78)."""

    def __init__(self):
        self.calls = []
        self._orig = torch.randint

    def __enter__(self):
        orig = self._orig

        def rec(*a, **k):
            r = orig(*a, **k)
            self.calls.append(r.clone())
            return r

        torch.randint = rec
        return self

    def __exit__(self, *exc):
        torch.randint = self._orig


def tensor_stats(t):
    t = t.detach().double()
    return {"sum": float(t.sum()), "sumsq": float((t * t).sum()), "first": t.flatten()[:6].tolist()}


def fx_tokenizer():
    ns = load_reference(build_model=False)
    raw = open(os.path.join(REF, "input.txt"), "rb").read()
    data = ns["data"]
    text = ns["text"]
    out = {
        "input_sha256": hashlib.sha256(raw).hexdigest(),
        "n_chars": len(text),
        "chars": ns["chars"],
        "vocab_size": ns["vocab_size"],
        "encode_first_1000": ns["encode"](text[:1000]),
        "data_len": int(data.numel()),
        "n_train": int(ns["n"]),
        "data_sha256_int64le": hashlib.sha256(data.numpy().astype("<i8").tobytes()).hexdigest(),
        "decode_check": ns["decode"](list(range(65))),
    }
    json.dump(out, open(os.path.join(OUT, "tokenizer.json"), "w"), indent=0)
    print("tokenizer.json", out["vocab_size"], out["data_len"], out["n_train"])


def fx_batches():
    """Batch-index streams after the seeded C1 init (GPT1.py:10,215), Dropout=0 (no CPU RNG
    use by dropout: the reference's device='cuda' semantics)."""
    res = {}
    ns = load_reference({"Dropout": 0.0})  # builds model -> consumes init RNG
    res["init_param_stats"] = {k: tensor_stats(v) for k, v in ns["model"].state_dict().items() if "tril" not in k}
    with RandintRecorder() as rec:
        for split in ["train", "val"]:  # estimate_loss() draw pattern, GPT1.py:89-92
            for _ in range(ns["eval_iters"]):
                ns["get_batch"](split)
        xb, yb = ns["get_batch"]("train")
        for _ in range(63):
            ns["get_batch"]("train")
    ix = torch.stack(rec.calls)
    res["ix_eval_train"] = ix[:200]
    res["ix_eval_val"] = ix[200:400]
    res["ix_train_after_eval"] = ix[400:464]
    res["first_train_x0"] = xb[:4, 0].clone()
    res["first_train_row0_text"] = ns["decode"](xb[0, :40].tolist())
    res["first_train_y_row0"] = yb[0, :40].clone()

    ns = load_reference({"Dropout": 0.0})
    with RandintRecorder() as rec:
        for _ in range(64):
            ns["get_batch"]("train")
    res["ix_train_no_eval"] = torch.stack(rec.calls)
    # batch B*W draw == W consecutive get_batch draws -- pin it
    ns = load_reference({"Dropout": 0.0})
    res["ix_one_draw_512"] = torch.randint(len(ns["train_data"]) - ns["block_size"], (512,))
    meta = {"first_train_row0_text": res.pop("first_train_row0_text"), "init_param_stats": res.pop("init_param_stats")}
    torch.save(res, os.path.join(OUT, "batches_c1.pt"))
    json.dump(meta, open(os.path.join(OUT, "batches_c1_meta.json"), "w"), indent=0)
    print("batches_c1", res["first_train_x0"].tolist(), meta["first_train_row0_text"][:30])


def _perturb_ln(model, gen):
    with torch.no_grad():
        for name, p in model.named_parameters():
            if "ln" in name:
                p.add_(0.1 * torch.randn(p.shape, generator=gen))


def _module_case(mod, x, gen):
    x = x.clone().requires_grad_(True)
    mod.zero_grad(set_to_none=True)
    out = mod(x)
    g = torch.randn(out.shape, generator=gen)
    out.backward(g)
    case = {"x": x.detach().clone(), "out": out.detach().clone(), "grad_out": g, "grad_x": x.grad.clone()}
    for n, p in mod.named_parameters():
        case["grad." + n] = p.grad.clone()
    return case


def fx_ops_small():
    """Per-module forward/backward vectors from the reference classes, tiny shapes, p=0."""
    cfgs = {
        "S": dict(block_size=16, n_embd=24, n_head=4, n_layers=2, batch_size=2),
        "S_odd": dict(block_size=12, n_embd=18, n_head=3, n_layers=2, batch_size=3),
    }
    allres = {}
    for tag, cfg in cfgs.items():
        ns = load_reference(dict(cfg, Dropout=0.0))
        model = ns["model"]
        gen = torch.Generator().manual_seed(7)
        _perturb_ln(model, gen)
        res = {"state_dict": {k: v.clone() for k, v in model.state_dict().items() if "tril" not in k}}
        B, T, C = cfg["batch_size"], cfg["block_size"], cfg["n_embd"]
        blk = model.blocks[0]
        x = torch.randn(B, T, C, generator=gen)
        res["ln1"] = _module_case(blk.ln1, x, gen)
        res["head0"] = _module_case(blk.sa_heads.heads[0], x, gen)
        res["head0_short"] = _module_case(blk.sa_heads.heads[0], x[:, : T - 5].contiguous(), gen)
        res["mha"] = _module_case(blk.sa_heads, x, gen)
        res["ffwd"] = _module_case(blk.ffwd, x, gen)
        res["block0"] = _module_case(blk, x, gen)
        idx = torch.randint(0, ns["vocab_size"], (B, T), generator=gen)
        tgt = torch.randint(0, ns["vocab_size"], (B, T), generator=gen)
        model.zero_grad(set_to_none=True)
        logits, loss = model(idx, tgt)
        loss.backward()
        full = {"idx": idx, "targets": tgt, "logits": logits.detach().clone(), "loss": loss.detach().clone()}
        for n, p in model.named_parameters():
            full["grad." + n] = p.grad.clone()
        with torch.no_grad():
            lg, ls = model(idx[:, : T - 3])
        full["logits_notarget_short"] = lg.clone()
        full["loss_notarget_is_none"] = torch.tensor(ls is None)
        res["model"] = full
        res["config"] = torch.tensor([B, T, C, cfg["n_head"], cfg["n_layers"]])
        allres[tag] = res
    torch.save(allres, os.path.join(OUT, "ops_small.pt"))
    print("ops_small", {k: float(v["model"]["loss"]) for k, v in allres.items()})


def fx_model_c1_grads():
    """Full C1-shape model (d=126,h=6,hs=21,L=6,T=256) at seeded init: loss + grads, small batch."""
    ns = load_reference({"Dropout": 0.0})
    model = ns["model"]
    gen = torch.Generator().manual_seed(11)
    idx = torch.randint(0, 65, (2, 64), generator=gen)
    tgt = torch.randint(0, 65, (2, 64), generator=gen)
    logits, loss = model(idx, tgt)
    loss.backward()
    keep = ["lm_head.bias", "lm_head.weight", "ln_f.weight", "blocks.0.sa_heads.heads.0.key.weight",
            "blocks.5.sa_heads.heads.5.value.weight", "blocks.3.ffwd.net.0.bias", "position_embedding_table.weight"]
    res = {"idx": idx, "targets": tgt, "loss": loss.detach().clone(), "logits_head": logits[:8].detach().clone(),
           "grad_norms": {n: float(p.grad.double().norm()) for n, p in model.named_parameters()},
           "grads": {n: p.grad.clone() for n, p in model.named_parameters() if n in keep}}
    torch.save(res, os.path.join(OUT, "model_c1_grads.pt"))
    print("model_c1_grads loss", float(loss))


def fx_train_deterministic():
    """GPT1.py:221-233 driven for a few steps at Dropout=0 (so the CPU RNG only feeds
    get_batch): per-step training losses, lr=2e-4 (declared) and lr=0.5 (as shipped, Q4/Q5)."""
    res = {}
    for lr, steps in [(2e-4, 12), (0.5, 5)]:
        ns = load_reference({"Dropout": 0.0})
        m = ns["model"]
        opt = torch.optim.AdamW(m.parameters(), lr=lr)
        losses = []
        for _ in range(steps):
            xb, yb = ns["get_batch"]("train")
            logits, loss = m(xb, yb)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        res[f"lr{lr}"] = torch.tensor(losses, dtype=torch.float64)
        print("train lr", lr, losses)
    torch.save(res, os.path.join(OUT, "train_c1_p0.pt"))


def fx_trained_and_greedy(steps=200, eval_every=50, eval_iters=20):
    """Train the reference C1 model (Dropout 0.2, lr 2e-4) briefly, record the eval-loss
    curve (estimate_loss, GPT1.py:85-98), save the state dict exactly as GPT1.py:239-241
    does (minus tril buffers, see compact format), then a greedy (argmax instead of
    multinomial at GPT1.py:208) 500-token stream in eval mode from zeros(1,1)."""
    ns = load_reference({"eval_iters": eval_iters})
    m = ns["model"]
    opt = torch.optim.AdamW(m.parameters(), lr=2e-4)
    curve = []
    t0 = time.time()
    for it in range(steps + 1):
        if it % eval_every == 0:
            losses = ns["estimate_loss"]()
            curve.append((it, float(losses["train"]), float(losses["val"])))
            print(f"step {it} : train loss {losses['train']:.4f}, val loss = {losses['val']:.4f}  ({time.time()-t0:.0f}s)", flush=True)
        if it == steps:
            break
        xb, yb = ns["get_batch"]("train")
        logits, loss = m(xb, yb)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    sd = {k: v.clone() for k, v in m.state_dict().items() if "tril" not in k}
    from safetensors.torch import save_file
    save_file(sd, os.path.join(OUT, "model_c1_trained.safetensors"))
    m.eval()
    bs = ns["block_size"]
    with torch.no_grad():
        streams = {}
        for tag, start in [("zeros", torch.zeros((1, 1), dtype=torch.long)),
                           ("batch4", torch.tensor([[0], [13], [40], [52]]))]:
            idx = start
            margins = []
            for _ in range(500):
                logits, _ = m(idx[:, -bs:])
                last = logits[:, -1, :]
                top2 = torch.topk(last, 2, dim=-1).values
                margins.append((top2[:, 0] - top2[:, 1]).min().item())
                nxt = torch.argmax(last, dim=-1, keepdim=True)
                idx = torch.cat((idx, nxt), dim=1)
            streams[tag] = {"tokens": idx.clone(), "margins": torch.tensor(margins, dtype=torch.float64)}
            print("greedy", tag, "min margin", min(margins), repr(ns["decode"](idx[0].tolist())[:60]))
    torch.save({"curve": torch.tensor(curve, dtype=torch.float64), "streams": streams,
                "config": {"steps": steps, "eval_every": eval_every, "eval_iters": eval_iters, "lr": 2e-4, "Dropout": 0.2}},
               os.path.join(OUT, "trained_c1.pt"))


def fx_model_pth():
    """A model.pth in the reference's own format (GPT1.py:239-241: torch.save of the full state_dict,
    tril buffers included) at a small shape, plus the reference's logits/loss for a fixed batch:
    the GPU suite loads it with load_state_dict(strict=True)."""
    cfg = dict(block_size=32, n_embd=48, n_head=3, n_layers=2, batch_size=2)
    ns = load_reference(dict(cfg, Dropout=0.0))
    model = ns["model"]
    gen = torch.Generator().manual_seed(21)
    _perturb_ln(model, gen)
    torch.save(model.state_dict(), os.path.join(OUT, "model_small_ref.pth"))
    idx = torch.randint(0, 65, (2, 32), generator=gen)
    tgt = torch.randint(0, 65, (2, 32), generator=gen)
    with torch.no_grad():
        logits, loss = model(idx, tgt)
    torch.save({"config": cfg, "idx": idx, "targets": tgt, "logits": logits.clone(), "loss": loss.clone(),
                "n_keys": len(model.state_dict())}, os.path.join(OUT, "model_small_ref_io.pt"))
    print("model_small_ref.pth", len(model.state_dict()), "keys, loss", float(loss))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-train", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    torch.set_num_threads(8)
    jobs = {"tokenizer": fx_tokenizer, "batches": fx_batches, "ops": fx_ops_small, "c1grads": fx_model_c1_grads,
            "train": fx_train_deterministic, "trained": fx_trained_and_greedy, "modelpth": fx_model_pth}
    for name, fn in jobs.items():
        if a.only and name not in a.only.split(","):
            continue
        if a.skip_train and name in ("train", "trained"):
            continue
        fn()
