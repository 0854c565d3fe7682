"""Pins the CPU oracle (oracle/) to vectors produced by the reference GPT1.py itself."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import golden_path, ROOT
from oracle import gpt1_oracle as O
from oracle import philox

INPUT = os.path.join(ROOT, "data", "input.txt")


def _cfg_from(t, dropout=0.0):
    B, T, C, H, L = [int(v) for v in t]
    return O.OracleConfig(block_size=T, n_embd=C, n_head=H, n_layers=L, dropout=dropout), B


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 R=10
    cases = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
             ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
             ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
              (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for c, k, want in cases:
        got = tuple(int(x) for x in philox.philox4x32_10(*c, *k))
        assert got == want


def test_philox_keep_rate():
    keep = philox.keep_mask(1234, 7, np.arange(1 << 18), 0.2)
    assert abs(keep.mean() - 0.8) < 0.004
    assert philox.threshold(0.2) == 13107 and philox.threshold(1e-9) == 1 and philox.threshold(0.0) == 0


def test_philox_keep_spec_16bit():
    """keep(idx) = half (idx & 1) of word ((idx >> 1) & 3) of Philox(group idx >> 3) >= round(p 2^16),
    restated element by element from the KAT-pinned philox4x32_10, plus a regression pin of the packed
    bits (csrc/common.h keep_of / keep4_bits / keep8_bits follow the same spec)."""
    seed, stream, p = 0x1337, (5 << 8) | 3, 0.5
    idx = np.arange(64, dtype=np.uint64) + np.uint64(1 << 33)
    got = philox.keep_mask(seed, stream, idx, p)
    for i, e in enumerate(idx.tolist()):
        g = e >> 3
        out = philox.philox4x32_10(g & 0xFFFFFFFF, g >> 32, stream & 0xFFFFFFFF, stream >> 32, seed, 0)
        w = int(out[(e >> 1) & 3])
        u = (w >> 16) if (e & 1) else (w & 0xFFFF)
        assert bool(got[i]) == (u >= 32768), e
    pack = lambda k: sum(int(b) << i for i, b in enumerate(k))
    assert pack(got) == 0xb8ff66c6338a74a9
    assert pack(philox.keep_mask(1234, 7, np.arange(64), 0.2)) == 0x7fff7d76dbf72d66


def test_tokenizer_matches_reference():
    g = json.load(open(golden_path("tokenizer.json")))
    raw = open(INPUT, "rb").read()
    assert hashlib.sha256(raw).hexdigest() == g["input_sha256"]
    text = raw.decode("utf-8")
    chars, stoi = O.build_vocab(text)
    assert chars == g["chars"] and len(chars) == g["vocab_size"] == 65
    assert O.encode(stoi, text[:1000]) == g["encode_first_1000"]
    data = torch.tensor(O.encode(stoi, text), dtype=torch.long)
    assert data.numel() == g["data_len"]
    assert hashlib.sha256(data.numpy().astype("<i8").tobytes()).hexdigest() == g["data_sha256_int64le"]
    tr, va = O.split(data)
    assert len(tr) == g["n_train"]
    assert O.decode(chars, list(range(65))) == g["decode_check"]


def test_init_and_batch_stream_match_reference():
    b = torch.load(golden_path("batches_c1.pt"), weights_only=True)
    meta = json.load(open(golden_path("batches_c1_meta.json")))
    cfg = O.OracleConfig(dropout=0.0)
    torch.manual_seed(1337)
    P = O.init_params(cfg)
    for k, st in meta["init_param_stats"].items():
        t = P[k].double()
        assert abs(float(t.sum()) - st["sum"]) <= 1e-9 * max(1.0, abs(st["sum"])) + 1e-9, k
        assert t.flatten()[:6].tolist() == st["first"], k
    text = open(INPUT, encoding="utf-8").read()
    chars, stoi = O.build_vocab(text)
    data = torch.tensor(O.encode(stoi, text), dtype=torch.long)
    tr, va = O.split(data)
    draws = [O.draw_ix(len(tr if i < 200 else va), 256, 64) for i in range(400)]
    assert torch.equal(torch.stack(draws[:200]), b["ix_eval_train"])
    assert torch.equal(torch.stack(draws[200:]), b["ix_eval_val"])
    first = O.draw_ix(len(tr), 256, 64)
    assert torch.equal(first, b["ix_train_after_eval"][0])
    x, y = O.windows(tr, first, 256)
    assert torch.equal(x[:4, 0], b["first_train_x0"])
    assert torch.equal(y[0, :40], b["first_train_y_row0"])
    assert O.decode(chars, x[0, :40].tolist()) == meta["first_train_row0_text"]


def test_one_draw_equals_consecutive_draws():
    b = torch.load(golden_path("batches_c1.pt"), weights_only=True)
    assert torch.equal(b["ix_one_draw_512"], b["ix_train_no_eval"][:8].reshape(-1))


@pytest.mark.parametrize("tag", ["S", "S_odd"])
def test_model_forward_backward_matches_reference(tag):
    g = torch.load(golden_path("ops_small.pt"), weights_only=True)[tag]
    cfg, B = _cfg_from(g["config"])
    P = {k: v.clone() for k, v in g["state_dict"].items()}
    m = g["model"]
    logits, loss, grads = O.loss_and_grads(P, m["idx"], m["targets"], cfg)
    torch.testing.assert_close(loss, m["loss"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(logits, m["logits"], rtol=1e-5, atol=1e-6)
    for k, gr in grads.items():
        torch.testing.assert_close(gr, m["grad." + k], rtol=1e-4, atol=1e-6, msg=k)
    lg, ls = O.forward(P, m["idx"][:, : cfg.block_size - 3], cfg)
    assert ls is None and lg.shape == m["logits_notarget_short"].shape
    torch.testing.assert_close(lg, m["logits_notarget_short"], rtol=1e-5, atol=1e-6)


def test_c1_shape_grads_match_reference():
    g = torch.load(golden_path("model_c1_grads.pt"), weights_only=True)
    cfg = O.OracleConfig(dropout=0.0)
    torch.manual_seed(1337)
    P = O.init_params(cfg)
    logits, loss, grads = O.loss_and_grads(P, g["idx"], g["targets"], cfg)
    torch.testing.assert_close(loss, g["loss"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(logits[:8], g["logits_head"], rtol=1e-5, atol=1e-5)
    for k, n in g["grad_norms"].items():
        assert abs(float(grads[k].double().norm()) - n) <= 1e-4 * n + 1e-7, k
    for k, gr in g["grads"].items():
        torch.testing.assert_close(grads[k], gr, rtol=1e-4, atol=1e-6)


def test_train_steps_match_reference_p0():
    """A few GPT1.py:221-233 iterations with Dropout=0 (CPU RNG only feeds get_batch)."""
    g = torch.load(golden_path("train_c1_p0.pt"), weights_only=True)
    text = open(INPUT, encoding="utf-8").read()
    chars, stoi = O.build_vocab(text)
    data = torch.tensor(O.encode(stoi, text), dtype=torch.long)
    tr, _ = O.split(data)
    cfg = O.OracleConfig(dropout=0.0)
    for key, lr in [("lr0.0002", 2e-4), ("lr0.5", 0.5)]:
        want = g[key]
        n = min(len(want), 4)
        torch.manual_seed(1337)
        P = O.init_params(cfg)
        opt = O.AdamWOracle(P, lr=lr)
        for i in range(n):
            ix = O.draw_ix(len(tr), 256, 64)
            x, y = O.windows(tr, ix, 256)
            _, loss, grads = O.loss_and_grads(P, x[:, :], y, cfg)
            assert abs(float(loss) - float(want[i])) < 2e-4 * (i + 1), (key, i, float(loss), float(want[i]))
            opt.step(grads)
