"""Host-side checks that run without a GPU: the C-ABI library loads and exports every symbol
include/charpt.h declares, module construction reproduces the reference init, state-dict layout,
tokenizer and batch-index streams."""
import json

import pytest
import torch

from conftest import golden_path


def test_library_exports_header_symbols():
    from replicatinggpt_amd import _lib
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib._SIGS, f"{s} has no ctypes signature"
    assert lib.cg_version() >= 1
    assert lib.cg_gemm_workspace(128, 256, 4) == 4 * 128 * 256 * 4
    # two orientations x lower-triangle 32x32 blocks (8 * 9 / 2 at T = 256) x 128 B
    assert lib.cg_attn_mask_bytes(2, 6, 256) == 2 * (2 * 6 * 20 * 256)   # NB = 8: 8 + 49 // 4 tiles
    assert lib.cg_attn_bwd_workspace(2, 256, 6, 64) == 2 * 6 * 256 * 4 + lib.cg_attn_mask_bytes(2, 6, 256)


def test_torch_ops_registered():
    from replicatinggpt_amd import ops  # noqa: F401
    for name in ["gemm", "attn_fwd", "attn_bwd", "layernorm_fwd", "layernorm_bwd", "embed_fwd", "embed_bwd",
                 "ce_fwd", "ce_bwd", "adamw", "colsum", "dropout_apply", "gather_batch", "rng_snapshot"]:
        assert hasattr(torch.ops.charpt, name), name


def test_cpu_forward_fails_loudly():
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    m = BigramLanguageModel(GPTConfig(block_size=8, n_embd=16, n_head=2, n_layers=1))
    with pytest.raises(RuntimeError, match="HIP"):
        m(torch.zeros(1, 8, dtype=torch.long))


def test_init_matches_reference_and_state_dict_layout():
    from replicatinggpt_amd import BigramLanguageModel
    meta = json.load(open(golden_path("batches_c1_meta.json")))
    b = torch.load(golden_path("batches_c1.pt"), weights_only=True)
    torch.manual_seed(1337)
    m = BigramLanguageModel()
    sd = m.state_dict()
    assert len(sd) == 210
    assert sum(p.numel() for p in m.parameters()) == 1199585
    tril = [k for k in sd if k.endswith("tril")]
    assert len(tril) == 36 and sd[tril[0]].shape == (256, 256)
    for k, st in meta["init_param_stats"].items():
        t = sd[k].double()
        assert t.flatten()[:6].tolist() == st["first"], k
        assert abs(float(t.sum()) - st["sum"]) <= 1e-9 * max(1.0, abs(st["sum"])), k
    # the CPU generator is left exactly where the reference leaves it
    assert torch.equal(torch.randint(1003853 - 256, (64,)), b["ix_train_no_eval"][0])
    # params are views of one flat fp32 buffer; state_dict entries are independent tensors
    st = m.flat
    assert st.master.numel() >= 1199585
    q0 = m.blocks[0].sa_heads.heads[0].query.weight
    assert q0.data_ptr() == st.regions["0.qkv"].master.data_ptr()
    assert sd["blocks.0.sa_heads.heads.0.query.weight"].data_ptr() != q0.data_ptr()


def test_load_state_dict_roundtrip(tmp_path):
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    cfg = GPTConfig(block_size=16, n_embd=24, n_head=4, n_layers=2)
    torch.manual_seed(0)
    a = BigramLanguageModel(cfg)
    path = tmp_path / "model.pth"
    with open(path, "wb") as f:
        torch.save(a.state_dict(), f)            # GPT1.py:239-241
    torch.manual_seed(1)
    b = BigramLanguageModel(cfg)
    b.load_state_dict(torch.load(path, weights_only=True))
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)
    assert b.flat.version() != b.flat._shadow_version   # shadow refresh is pending after the load


def test_tokenizer_and_sampler_match_reference():
    from replicatinggpt_amd.data import BatchSampler, TokenStream
    g = json.load(open(golden_path("tokenizer.json")))
    b = torch.load(golden_path("batches_c1.pt"), weights_only=True)
    tok, ts = TokenStream.from_file()
    assert tok.chars == g["chars"] and tok.vocab_size == 65
    assert tok.encode(tok.decode(list(range(65)))) == list(range(65))
    assert len(ts.train_cpu) == g["n_train"]
    s = BatchSampler(ts, 256, 64)
    torch.manual_seed(1337)
    from replicatinggpt_amd import BigramLanguageModel
    BigramLanguageModel()  # consumes the init draws
    for i in range(3):
        assert torch.equal(s.draw_ix("train"), b["ix_train_no_eval"][i])
    # data-parallel slicing: rank r of W gets slice r of the global B*W draw
    torch.manual_seed(1337)
    BigramLanguageModel()
    s2 = BatchSampler(ts, 256, 64, world_size=8, rank=3)
    assert torch.equal(s2.draw_ix("train"), b["ix_one_draw_512"][3 * 64:4 * 64])


def _torch_adamw_stepped(model, lr=3e-3, steps=2, seed=5):
    """torch.optim.AdamW after ``steps`` steps on synthetic gradients (CPU)."""
    ref = torch.optim.AdamW(model.parameters(), lr=lr)
    g = torch.Generator().manual_seed(seed)
    for _ in range(steps):
        for p in model.parameters():
            p.grad = torch.randn(p.shape, generator=g)
        ref.step()
    return ref


def test_adamw_state_dict_is_torch_format():
    """optim.AdamW finds the flat buffers from the parameters (GPT1.py:218 as written), and its
    state dict is torch.optim.AdamW's: state moves from torch to charpt and back unchanged."""
    from replicatinggpt_amd import AdamW, BigramLanguageModel, GPTConfig
    cfg = GPTConfig(block_size=16, n_embd=24, n_head=4, n_layers=2)
    torch.manual_seed(0)
    m = BigramLanguageModel(cfg)
    ref = _torch_adamw_stepped(m)
    ours = AdamW(m.parameters(), lr=5e-1)
    assert ours.state_dict()["state"] == {}            # never stepped: no per-parameter state
    ours.load_state_dict(ref.state_dict())
    sd, rsd = ours.state_dict(), ref.state_dict()
    assert sd["param_groups"][0]["lr"] == 3e-3 and sd["param_groups"][0]["params"] == rsd["param_groups"][0]["params"]
    assert set(sd["state"]) == set(rsd["state"])
    for i, s in rsd["state"].items():
        assert float(sd["state"][i]["step"]) == float(s["step"]) == 2.0
        assert torch.equal(sd["state"][i]["exp_avg"], s["exp_avg"])
        assert torch.equal(sd["state"][i]["exp_avg_sq"], s["exp_avg_sq"])
    back = torch.optim.AdamW(m.parameters(), lr=1.0)
    back.load_state_dict(sd)
    for p in m.parameters():
        assert torch.equal(back.state[p]["exp_avg"], ref.state[p]["exp_avg"])
    assert back.param_groups[0]["lr"] == 3e-3 and back.param_groups[0]["decoupled_weight_decay"]


def test_checkpoint_roundtrip_cpu(tmp_path):
    """checkpoint.save_checkpoint / load_checkpoint restore weights, optimizer moments, the
    iteration, the CPU generator (get_batch's offsets) and the dropout counter; save_model writes
    the reference's 210-key model.pth."""
    from replicatinggpt_amd import AdamW, BigramLanguageModel, GPTConfig
    from replicatinggpt_amd import checkpoint as ck
    cfg = GPTConfig(block_size=16, n_embd=24, n_head=4, n_layers=2)
    torch.manual_seed(0)
    a = BigramLanguageModel(cfg)
    opt = AdamW(a.parameters(), lr=1e-3)
    opt.load_state_dict(_torch_adamw_stepped(a).state_dict())
    with torch.no_grad():
        a._rng_counter.fill_(7)
    torch.manual_seed(42)
    path = tmp_path / "ck.pt"
    ck.save_checkpoint(path, a, opt, 123)
    want_draw = torch.randint(1000, (5,))
    torch.manual_seed(1)
    b = BigramLanguageModel(cfg)
    opt_b = AdamW(b.parameters(), lr=9.0)
    assert ck.load_checkpoint(path, b, opt_b) == 123
    assert torch.equal(torch.randint(1000, (5,)), want_draw)
    assert int(b._rng_counter) == 7
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)
    sa, sb = opt.state_dict(), opt_b.state_dict()
    assert sb["param_groups"][0]["lr"] == 3e-3   # from the torch state loaded into opt
    for i in sa["state"]:
        assert torch.equal(sa["state"][i]["exp_avg_sq"], sb["state"][i]["exp_avg_sq"])
    mp = tmp_path / "model.pth"
    ck.save_model(b, mp)
    sd = torch.load(mp, weights_only=True)
    assert len(sd) == len(b.state_dict()) and sum(k.endswith("tril") for k in sd) == 2 * 4
    with pytest.raises(ValueError):
        ck.load_checkpoint(mp, b)


def test_gemm_operand_extent_guard():
    """ops.gemm checks on the host that every element cg_gemm will address lies in its operand's
    storage (the C ABI sees only pointers): a transposed-B layout given an [N, K] tensor is refused
    before any launch; a column-block view addressed through its parent's row stride passes."""
    from replicatinggpt_amd.ops import _gemm_extents
    parent = torch.empty(100, 30)
    _gemm_extents(parent[:, 10:20], torch.empty(5, 10), torch.empty(100, 5), False, False, 100, 5, 10, 30, 10, 5)
    with pytest.raises(ValueError, match="operand B"):
        _gemm_extents(torch.empty(256, 64), torch.empty(32, 64), torch.empty(256, 32), False, True, 256, 32, 64, 64,
                      64, 32)
    with pytest.raises(ValueError, match="operand C"):
        _gemm_extents(torch.empty(256, 64), torch.empty(32, 64), torch.empty(255, 32), False, False, 256, 32, 64, 64,
                      64, 32)
