"""Error statistics that the bf16 parity bars are set from (GPU only; oracle as the checker):
(1) bf16 attention at the C2 / C4 head geometry (p = 0.2) against fp64 with the oracle's keep mask:
    max|err| / max|ref|, ||err|| / ||ref||, and the share of elements outside |err| <= rtol |ref| +
    atol rms(ref) for a few (rtol, atol);
(2) one C2 full-size bf16 training forward/backward (B=64, T=256, d=384, dropout 0.2) against the
    CPU oracle (fp32, same init, same Philox masks): loss and per-parameter gradient errors.
usage: python tools/parity_probe.py [attn|model|all]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gpt1_oracle as O  # noqa: E402
from oracle import philox  # noqa: E402

DEV = "cuda"


def stats(got, ref):
    g = got.detach().double().cpu().flatten()
    r = ref.detach().double().cpu().flatten()
    e = (g - r).abs()
    rms = float(r.pow(2).mean().sqrt())
    out = dict(maxrel=float(e.max() / r.abs().max()), normrel=float(e.norm() / r.norm()))
    for rt, at in ((2e-2, 0.0), (2e-2, 1e-2), (2e-2, 2e-2), (3e-2, 3e-2)):
        out[f"viol({rt},{at})"] = float((e > rt * r.abs() + at * rms).double().mean())
    return out


def attn_ref(q, k, v, scale, p, seed, stream):
    B, T, H, D = q.shape
    s = torch.einsum("bthd,bshd->bhts", q, k) * scale
    s = s.masked_fill(~torch.tril(torch.ones(T, T, dtype=torch.bool)), float("-inf"))
    P = torch.softmax(s, -1)
    if p > 0:
        idx = np.arange(B * H * T * T, dtype=np.uint64).reshape(B, H, T, T)
        keep = torch.from_numpy(philox.keep_mask(seed, stream, idx, p))
        P = P * keep.double() * float(np.float32(1 / (1 - p)))
    return torch.einsum("bhts,bshd->bthd", P, v)


def probe_attn():
    from replicatinggpt_amd import functional as Fn
    for (B, T, H, C) in ((2, 256, 6, 384), (1, 1024, 12, 768)):
        D, p, site = 64, 0.2, 4
        torch.manual_seed(41)
        d = H * D
        qkv = (torch.randn(B * T, 3 * d) * 0.8).to(torch.bfloat16)
        q = qkv[:, :d].double().view(B, T, H, D).requires_grad_(True)
        k = qkv[:, d:2 * d].double().view(B, T, H, D).requires_grad_(True)
        v = qkv[:, 2 * d:].double().view(B, T, H, D).requires_grad_(True)
        scale = C ** -0.5
        ref = attn_ref(q, k, v, scale, p, 77, (3 << 8) | site)
        dout = torch.randn(B, T, H, D).to(torch.bfloat16)
        ref.backward(dout.double())
        call = torch.tensor([3], dtype=torch.int64, device=DEV)
        qd = qkv.to(DEV)
        o = torch.empty(B * T, d, dtype=torch.bfloat16, device=DEV)
        lse, mask = Fn.attention_fwd(qd, B, T, H, D, o, scale, p, 77, call, site)
        dqkv = Fn.attention_bwd(qd, B, T, H, D, o, dout.reshape(B * T, d).to(DEV), lse, scale, p, 77, call, site, mask)
        torch.cuda.synchronize()
        print(f"attention B={B} T={T} H={H} p={p}", flush=True)
        print("   o ", stats(o, ref.reshape(B * T, d)))
        for i, t in enumerate((q, k, v)):
            print("  d" + "qkv"[i], stats(dqkv[:, i * d:(i + 1) * d], t.grad.reshape(B * T, d)), flush=True)


def probe_model():
    from replicatinggpt_amd import BigramLanguageModel, PRESETS
    cfg = PRESETS["c2"].with_(dtype="bf16")
    ocfg = O.OracleConfig(block_size=256, n_embd=384, n_head=6, n_layers=6, dropout=cfg.dropout)
    g = torch.Generator().manual_seed(17)
    idx = torch.randint(0, 65, (64, 256), generator=g)
    tgt = torch.randint(0, 65, (64, 256), generator=g)
    torch.manual_seed(1337)
    m = BigramLanguageModel(cfg).to(DEV)
    _, loss = m(idx.to(DEV), tgt.to(DEV))
    loss.backward()
    torch.manual_seed(1337)
    P = O.init_params(ocfg)
    t0 = time.time()
    _, rl, rg = O.loss_and_grads(P, idx, tgt, ocfg, train=True, seed=cfg.dropout_seed, call=0)
    print(f"model C2 bf16 vs oracle fp32 (p={cfg.dropout}): loss {float(loss):.6f} vs {float(rl):.6f} "
          f"rel {abs(float(loss) - float(rl)) / float(rl):.2e}  (oracle {time.time() - t0:.1f} s)", flush=True)
    worst = []
    for name, prm in m.named_parameters():
        s = stats(prm.grad, rg[name])
        a, b = prm.grad.double().cpu().flatten(), rg[name].double().flatten()
        s["cos"] = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
        worst.append((s["normrel"], name, s))
    worst.sort(reverse=True)
    for nr, name, s in worst[:12]:
        print(f"  {name:40s} {s}")
    print("  median normrel", sorted(w[0] for w in worst)[len(worst) // 2], flush=True)


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("attn", "all"):
        probe_attn()
    if what in ("model", "all"):
        probe_model()
