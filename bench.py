"""charpt training-throughput benchmark (BASELINE.json metric: train tokens/sec at 1/2/4/8
MI355X + MFMA util, char-GPT block 256).

Workload (default, --config c2): BASELINE configs[1] -- the char-GPT shape 6L/6H/384d, block 256,
batch 64 per GPU, bf16 activations/GEMM operands with fp32 master weights, dropout 0.2 as the model
does, synthetic char tokens (randint(65) stream, seed 1337), AdamW.  One "step" = one iteration of
GPT1.py:227-233 (get_batch, forward, zero_grad, backward, [grad all-reduce], optimizer step),
replayed from a hipGraph.  N > 1 GPUs: data parallel, weak scaling (64 sequences per GPU),
bucketed RCCL all-reduce of the fp32 gradient buffer.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E


def flops_per_token(cfg, T):
    """F = 6 (L 12 d^2 + d V) + 6 L (T+1) d   (fwd+bwd, causal attention)."""
    L, d, V = cfg.n_layers, cfg.n_embd, cfg.vocab_size
    return 6 * (L * 12 * d * d + d * V) + 6 * L * (T + 1) * d


def _cpu_info():
    """Host CPU model (lscpu 'Model name') and the cores this process may run on."""
    model = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    # a container's CPU quota can be far below its affinity mask (the GPU box exports the share it
    # grants as OMP_NUM_THREADS): more threads than that only contend
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        cores = min(cores, int(omp))
    return model, cores


def cpu_baseline(cfg, seconds=12.0, batch=16):
    """The oracle (CPU fp32 restatement of GPT1.py, 'port') timed on this host on the benchmarked
    workload: the same model shape and block size, dropout ON through torch's own CPU dropout op
    (nn.Dropout's bernoulli_, the reference's dominant CPU cost -- SURVEY §6), fwd + bwd + AdamW,
    all cores this process may use.  Bounded sample: ``batch`` sequences per step (the bench's 64 at
    C2 take ~4 s per CPU step; per-token throughput is batch-independent at B >= 16) for ~``seconds``."""
    from oracle import gpt1_oracle as O
    model_name, cores = _cpu_info()
    torch.set_num_threads(cores)
    ocfg = O.OracleConfig(vocab_size=cfg.vocab_size, block_size=cfg.block_size, n_embd=cfg.n_embd,
                          n_head=cfg.n_head, n_layers=cfg.n_layers, dropout=cfg.dropout, torch_dropout=True)
    torch.manual_seed(1337)
    P = O.init_params(ocfg)
    opt = O.AdamWOracle(P, lr=2e-4)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 65, (batch, cfg.block_size), generator=g)
    y = torch.randint(0, 65, (batch, cfg.block_size), generator=g)
    _, _, gr = O.loss_and_grads(P, x, y, ocfg, train=True)   # warm-up
    opt.step(gr)
    n, t0 = 0, time.perf_counter()
    while True:
        _, _, gr = O.loss_and_grads(P, x, y, ocfg, train=True)
        opt.step(gr)
        n += 1
        if time.perf_counter() - t0 > seconds and n >= 2:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n * batch * cfg.block_size / dt, 1), "unit": "tokens/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu_model": model_name,
            "sample": f"oracle fp32 train step (fwd+bwd+AdamW, dropout {cfg.dropout} via torch CPU bernoulli_ as "
                      f"GPT1.py:117,146), {n} steps of batch {batch} x block {cfg.block_size}, "
                      f"{cfg.n_layers}L/{cfg.n_head}H/{cfg.n_embd}d (the bench workload's shape)"}


COLD_BYTES = 1 << 29   # census operand sets cycle through >= 512 MB: twice the 256 MB Infinity Cache


def census_op(name, M, N, K, at, bt, kind, dev, p=0.2, cold=False, capture=None):
    """Operands and a launch closure for one census GEMM with the epilogue the training step uses
    (functional.py AttnSublayerFn / FFNSublayerFn): "store" (bf16 output), "bias_resid" (fp32
    output = x + o W^T + b: the attention projection), "bias_relu_bits" (bf16 relu(a W1^T + b1) and
    its ReLU keep bits), "bias_drop_resid" (fp32 x + dropout(h W2^T + b2)), "relu_bwd_colpart"
    (bf16 relu'(h) (dz2 W2) from the keep bits, with the b1 column partials), "store_rowdot" (bf16
    dO = dy Wp and the attention backward's delta = rowsum(dO * O) per head, T = 256), "wgrad" (fp32,
    deterministic split-K through bf16 slabs as in the step: the GEMM and its slab reduce).  cold: successive calls cycle through as
    many operand sets as make >= COLD_BYTES, so no call finds its operands in the Infinity Cache
    (in the training step every activation operand was last touched a whole sublayer or more
    earlier).  Returns (run, kernels per call)."""
    from replicatinggpt_amd import functional as Fn, ops
    from replicatinggpt_amd import _lib as L
    lib = L.load()
    fp32_out = kind in ("wgrad", "bias_resid", "bias_drop_resid")
    split = Fn._wgrad_split(M, N, K, True) if kind == "wgrad" else 1
    lda, ldb = (M if at else K), (N if bt else K)
    relu_bits = kind == "bias_relu_bits" and lib.cg_gemm_relu_bits_supported(0, 0, M, N, K, lda, ldb, N)
    colpart = kind == "relu_bwd_colpart" and lib.cg_gemm_colpart_supported(0, 1, M, N, K, lda, ldb, N)
    rowdot_T = 256 if M % 256 == 0 else 128
    rowdot = kind == "store_rowdot" and lib.cg_gemm_rowdot_supported(0, 1, M, N, K, lda, ldb, N)

    def make_set():
        st = {"A": torch.randn((K, M) if at else (M, K), device=dev).to(torch.bfloat16),
              "B": torch.randn((K, N) if bt else (N, K), device=dev).to(torch.bfloat16),
              "out": torch.empty(M, N, dtype=torch.float32 if fp32_out else torch.bfloat16, device=dev)}
        if kind == "wgrad" and split > 1:
            st["ws"] = torch.empty(ops.gemm_workspace(M, N, split) // 4, dtype=torch.float32, device=dev)
        if kind in ("bias_resid", "bias_drop_resid"):
            st["resid"] = torch.randn(M, N, device=dev)
        if kind in ("bias_relu_bits", "relu_bwd_colpart"):
            st["bits"] = torch.randint(-2 ** 31, 2 ** 31 - 1, (M, N // 32), dtype=torch.int32, device=dev)
        if colpart:
            st["part"] = torch.empty((M // 64, N), dtype=torch.float32, device=dev)
        if rowdot:
            st["o"] = torch.randn(M, N, device=dev).to(torch.bfloat16)
            st["delta"] = torch.empty(M * N // 64, dtype=torch.float32, device=dev)
        return st

    first = make_set()
    if capture is not None:   # the caller reads the first operand set's outputs (A/B tools)
        capture.update(first)
    nbytes = sum(t.numel() * t.element_size() for t in first.values())
    sets = [first] + [make_set() for _ in range(max(1, -(-COLD_BYTES // max(1, nbytes))) - 1)] if cold else [first]
    bias = torch.randn(N, device=dev) * 0.1
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    ctr = [0]

    def run():
        st = sets[ctr[0] % len(sets)]
        ctr[0] += 1
        A, B, out = st["A"], st["B"], st["out"]
        if kind == "wgrad":   # the step's slot weight gradients: bf16 split-K slabs (functional.linear_wgrad)
            flags = L.GEMM_SLAB_BF16 if Fn.SLAB_BF16 and split > 1 else 0
            ops.gemm(A, B, out, True, bool(at), bool(bt), M, N, K, lda, ldb, N, 0, None, None, 0, None, 0,
                     0.0, 0, None, 0, 0.0, split, st.get("ws"), flags)
        elif kind == "store_rowdot" and rowdot:
            ops.gemm_store_rowdot(A, B, out, M, N, K, lda, ldb, N, st["o"], N, rowdot_T, st["delta"])
        elif kind in ("store", "store_rowdot"):   # store_rowdot unsupported: the step's plain dgrad
            ops.gemm(A, B, out, True, bool(at), bool(bt), M, N, K, lda, ldb, N, 0, None, None, 0, None, 0,
                     0.0, 0, None, 0, 0.0, 1, None)
        elif kind in ("bias_resid", "bias_drop_resid"):
            drop = kind == "bias_drop_resid"
            epi = Fn.EPI["bias_drop_resid" if drop else "bias_resid"]
            ops.gemm(A, B, out, True, bool(at), bool(bt), M, N, K, lda, ldb, N, epi, bias, st["resid"], N, None, 0,
                     p if drop else 0.0, 4919 if drop else 0, call if drop else None, 3 if drop else 0, 0.0, 1, None)
        elif kind == "bias_relu_bits":
            if relu_bits:
                ops.gemm_bias_relu_bits(A, B, out, M, N, K, lda, ldb, N, bias, st["bits"], st["bits"].stride(0))
            else:   # the step's fallback
                ops.gemm(A, B, out, True, False, False, M, N, K, lda, ldb, N, Fn.EPI["bias_relu"], bias, None, 0,
                         None, 0, 0.0, 0, None, 0, 0.0, 1, None)
        elif kind == "relu_bwd_colpart":
            if colpart:
                ops.gemm_relu_bwd_colpart(A, B, out, M, N, K, lda, ldb, N, st["bits"], st["bits"].stride(0),
                                          st["part"])
            else:   # the step's fallback (no partials)
                ops.gemm(A, B, out, True, False, True, M, N, K, lda, ldb, N, Fn.EPI["relu_bwd"], None, None, 0,
                         st["bits"], st["bits"].stride(0), 0.0, 0, None, 0, 0.0, 1, None)
        else:
            raise ValueError(kind)
    return run, (2 if split > 1 else 1)


def time_gemm(name, M, N, K, at, bt, kind, dev, reps=30, cold=False):
    """Average duration (ms) of one charpt bf16 GEMM launch of this shape with the step's epilogue
    (census_op; cold: operands cycled past the Infinity Cache): reps back-to-back launches replayed
    from one hipGraph, HIP events on the replay stream."""
    run, _ = census_op(name, M, N, K, at, bt, kind, dev, cold=cold)
    for _ in range(3):
        run()
    # the reps launches replayed from a hipGraph, as in the training step: eagerly, the smallest
    # products (C2 proj fwd / dgrad, 15 us kernels) are host-launch-bound at ~27 us per call
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for _ in range(reps):
            run()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()   # the replay runs on the current stream
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def census_shapes(cfg, Bsz, T):
    """Every bf16 GEMM of one training step with the epilogue the step gives it:
    (name, M, N, K, a_trans, b_trans, epilogue kind (census_op), launches/step)."""
    M, d, L = Bsz * T, cfg.n_embd, cfg.n_layers
    F4 = 4 * d
    return [
        ("qkv_fwd", M, 3 * d, d, 0, 0, "store", L), ("proj_fwd", M, d, d, 0, 0, "bias_resid", L),
        ("ffn1_fwd", M, F4, d, 0, 0, "bias_relu_bits", L), ("ffn2_fwd", M, d, F4, 0, 0, "bias_drop_resid", L),
        ("proj_dgrad", M, d, d, 0, 1, "store_rowdot" if T <= 256 and d % 64 == 0 else "store", L),
        ("qkv_dgrad", M, d, 3 * d, 0, 1, "store", L),
        ("ffn2_dgrad", M, F4, d, 0, 1, "relu_bwd_colpart", L), ("ffn1_dgrad", M, d, F4, 0, 1, "store", L),
        ("proj_wgrad", d, d, M, 1, 1, "wgrad", L), ("qkv_wgrad", 3 * d, d, M, 1, 1, "wgrad", L),
        ("ffn2_wgrad", d, F4, M, 1, 1, "wgrad", L), ("ffn1_wgrad", F4, d, M, 1, 1, "wgrad", L),
    ]


def gemm_census(cfg, Bsz, T, dev, cold=False):
    """Average launch time of every GEMM of one training step, each with its step epilogue (HIP
    events, time_gemm; cold: operands cycled past the Infinity Cache)."""
    from replicatinggpt_amd import functional as Fn
    out = []
    for name, m, n, k, at, bt, kind, cnt in census_shapes(cfg, Bsz, T):
        ms = time_gemm(name, m, n, k, at, bt, kind, dev, cold=cold)
        split = Fn._wgrad_split(m, n, k, True) if kind == "wgrad" else 1
        out.append({"name": name, "M": m, "N": n, "K": k, "epilogue": kind, "ms": ms, "launches": cnt,
                    "flops": 2.0 * m * n * k, "split": split, "layout": (bool(at), bool(bt)),
                    "kernel": gemm_kernel_name(m, n, at, bt, split, dev, kind)})
        torch.cuda.empty_cache()
    return out


def gemm_kernel_name(M, N, at, bt, split, dev, kind="store"):
    """The kernel cg_gemm's default dispatch picks (gemm_bf16.hip pick_variant, gemm_pk.hip
    launch_n96): the 8-wave 256x256 tile at >= 2 such tiles per CU (no split, A not transposed);
    128x96 tiles for the fp32 residual forwards where they shorten the busiest slot's work (rounds
    of items x tile width; cg_set_tuning gemm_n96); else 128x128."""
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    if split == 1 and not at and M % 256 == 0 and N % 256 == 0 and (M // 256) * (N // 256) >= 2 * cus:
        return "k_gemm_p8<256x256>"
    n96 = 1
    for kv in filter(None, os.environ.get("CHARPT_TUNING", "").split(",")):
        k, _, v = kv.partition("=")
        if k.strip() == "gemm_n96":
            n96 = int(v)
    if (n96 and split == 1 and not at and not bt and kind in ("bias_resid", "bias_drop_resid") and M % 128 == 0
            and N % 96 == 0):
        slots = 2 * cus
        crit96 = -(-(M // 128) * (N // 96) // slots) * 96
        crit128 = -(-(M // 128) * (N // 128) // slots) * 128 if N % 128 == 0 else float("inf")
        if crit96 < crit128:
            return "k_gemm_pk<128x96>"
    if split > 1:
        from replicatinggpt_amd import functional as Fn
        return "k_gemm_pk<128x128>" + (" + k_slab16_reduce8 (bf16 slabs)" if Fn.SLAB_BF16 else " + k_splitk_reduce4")
    return "k_gemm_pk<128x128>"


def _time_ms(fn, reps=20, warm=3):
    """Average duration (ms) of fn() over reps back-to-back calls replayed from one hipGraph (as in
    the training step; eagerly the small LayerNorm launches are host-bound), HIP events on the
    replay stream (the stream every charpt op launches on), after ``warm`` eager calls."""
    for _ in range(warm):
        fn()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for _ in range(reps):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def kernel_census(cfg, Bsz, T, dev):
    """The non-GEMM kernels of the step at the step's shapes, each against its roofline (north_star:
    MFMA utilisation for attention, achieved HBM GB/s for the norm / optimizer kernels):
      attention fwd (on premade keep bits: the Philox keep-bit kernel runs on the side stream at the
        start of the forward, overlapped with the embedding / LN / QKV kernels, and is reported on its
        own as attention_dropmask, VALU-bound decisions/s) / bwd: causal algorithmic FLOPs
        fwd 4*B*H*(T(T+1)/2)*D, bwd 2x fwd (S recompute not counted) vs the bf16 MFMA peak, and their
        algorithmic HBM bytes (fwd: q,k,v read + o written + lse + FWD keep words; bwd: q,k,v,dO
        (+ o unless delta comes precomputed, as in the C2 step) read + dq,dk,dv written + lse, delta +
        both keep-word halves) vs the HBM peak -- at T = 256
        the attention kernels are memory/latency-bound;
      LayerNorm fwd: M*C*(4 read + 2 write) B; LayerNorm bwd (dy bf16, x, residual grad, dx, the
        consumer's dropout-applied bf16 copy): M*C*(2+4+4+4+2) B; AdamW: 30 B/param (p, g, m, v
        fp32 + bf16 shadow) -- vs HBM peak."""
    from replicatinggpt_amd import functional as Fn, ops
    M, C, H = Bsz * T, cfg.n_embd, cfg.n_head
    D = C // H
    p = float(cfg.dropout)
    out = {}
    qkv = (torch.randn(M, 3 * C, device=dev) * 0.5).to(torch.bfloat16)
    o = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    do = torch.randn(M, C, device=dev).to(torch.bfloat16)
    call = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = C ** -0.5
    mbytes = ops.attn_mask_bytes(Bsz, H, T) if p > 0 else 0
    mask = torch.empty(max(mbytes, 8) // 8, dtype=torch.int64, device=dev)
    lse = torch.empty((Bsz, H, T), dtype=torch.float32, device=dev)
    if p > 0:
        t_m = _time_ms(lambda: ops.attn_dropmask(Bsz, H, T, p, 1, call, 0, mask))
        dec = Bsz * H * T * (T + 1) / 2
        out["attention_dropmask"] = {"ms": round(t_m, 4), "decisions": dec, "achieved": round(dec / t_m / 1e6, 1),
                                     "unit": "G keep decisions/s (VALU-bound Philox, side stream)"}
        ops.attn_dropmask(Bsz, H, T, p, 1, call, 0, mask)
    t_f = _time_ms(lambda: ops.attn_fwd(qkv, Bsz, T, H, D, 0, C, 2 * C, qkv.stride(0), o, C, lse, scale, p, 1, call,
                                        0, mask if p > 0 else None, p > 0))
    # the step's form: delta = rowsum(dO * O) from the projection dgrad's epilogue where it applies
    # (functional.rowdot_ok: T <= 256, head 64), so the backward reads delta instead of O
    din = Fn.ROWDOT and D == 64 and T <= 256 and T % 64 == 0
    delta = ((do.float() * o.float()).view(Bsz, T, H, D).sum(-1).permute(0, 2, 1).contiguous() if din else None)
    t_b = _time_ms(lambda: Fn.attention_bwd(qkv, Bsz, T, H, D, o, do, lse, scale, p, 1, call, 0,
                                            mask if p > 0 else None, delta))
    fl = 4.0 * Bsz * H * (T * (T + 1) / 2) * D
    stat = Bsz * H * T * 4
    fbytes = 4 * M * C * 2 + stat + mbytes // 2
    bbytes = (7 if din else 8) * M * C * 2 + 2 * stat + mbytes
    for name, t, f, byts in (("attention_fwd", t_f, fl, fbytes), ("attention_bwd", t_b, 2 * fl, bbytes)):
        tf = f / (t * 1e-3) / 1e12
        gbs = byts / (t * 1e-3) / 1e9
        out[name] = {"ms": round(t, 4), "achieved": round(tf, 1), "unit": "TFLOP/s", "peak": PEAK_BF16_TFLOPS,
                     "frac": round(tf / PEAK_BF16_TFLOPS, 4), "bytes": byts, "GB/s": round(gbs, 1),
                     "hbm_frac": round(gbs / PEAK_HBM_GBS, 4)}
    del qkv, o, do, mask
    x = torch.randn(M, C, device=dev)
    w, b = torch.randn(C, device=dev), torch.randn(C, device=dev)
    y = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    t = _time_ms(lambda: ops.layernorm_fwd(x, w, b, y, mean, rstd, 1e-5))
    dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dres, dx = torch.randn(M, C, device=dev), torch.empty(M, C, device=dev)
    lp = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    dw, db, cs = (torch.empty(C, device=dev) for _ in range(3))
    ws = torch.empty(ops.layernorm_bwd_workspace(M, C) // 4 + 1, device=dev)
    t2 = _time_ms(lambda: ops.layernorm_bwd(dy, x, w, mean, rstd, dres, dx, lp, dw, db, False, ws, cs, False, p, 1,
                                            call, 3))
    # the row kernel alone: in the training step its column-sum reduce runs on the side stream
    # (functional.GradLink -> layernorm_bwd_rows on the main stream, layernorm_bwd_reduce beside it)
    t3 = _time_ms(lambda: ops.layernorm_bwd_rows(dy, x, w, mean, rstd, dres, dx, lp, ws, True, p, 1, call, 3))
    for name, tt, byts in (("layernorm_fwd", t, M * C * 6), ("layernorm_bwd", t2, M * C * 16),
                           ("layernorm_bwd_rows", t3, M * C * 16)):
        gbs = byts / (tt * 1e-3) / 1e9
        out[name] = {"ms": round(tt, 4), "bytes": byts, "achieved": round(gbs, 1), "unit": "GB/s",
                     "peak": PEAK_HBM_GBS, "frac": round(gbs / PEAK_HBM_GBS, 4)}
    del x, y, dy, dres, dx, lp
    n = sum(t.numel() for t in _param_shapes(cfg))
    n = (n + 63) // 64 * 64
    pp, g, m, v = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
    v.abs_()
    p16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    step_t = torch.ones(1, dtype=torch.int64, device=dev)
    # steady state: the step's optimizer buffers are long-lived; on freshly allocated ones the first
    # launches ran up to 20 % slower (profiles/r4_adamw_ab.txt)
    t = _time_ms(lambda: ops.adamw(pp, g, m, v, p16, 1e-3, 0.9, 0.999, 1e-8, 0.01, step_t), warm=20)
    gbs = 30 * n / (t * 1e-3) / 1e9
    # the box's ceiling for AdamW's near-1:1 read/write mix: a copy reading 16 B and writing 14 B per
    # parameter (profiles/r6_adamw_ceiling_c4.txt: LayerNorm's 2:1 read-heavy stream runs faster)
    src = torch.empty(4 * n, dtype=torch.float32, device=dev)
    dst = torch.empty(7 * n // 2, dtype=torch.float32, device=dev)
    tc = _time_ms(lambda: dst.copy_(src[:dst.numel()]), warm=5)
    cgbs = 28 * n / (tc * 1e-3) / 1e9
    del src, dst
    out["adamw"] = {"ms": round(t, 4), "params": n, "bytes": 30 * n, "achieved": round(gbs, 1), "unit": "GB/s",
                    "peak": PEAK_HBM_GBS, "frac": round(gbs / PEAK_HBM_GBS, 4),
                    "copy_same_mix_GB/s": round(cgbs, 1), "frac_of_copy": round(gbs / cgbs, 4)}
    return out


def _param_shapes(cfg):
    """Parameter tensors of the model (for AdamW sizing) without building it."""
    d, L, V, T = cfg.n_embd, cfg.n_layers, 65, cfg.block_size
    shapes = [(V, d), (T, d), (d,), (d,), (V, d), (V,)]
    for _ in range(L):
        shapes += [(3 * d, d), (d, d), (d,), (4 * d, d), (4 * d,), (d, 4 * d), (d,), (d,), (d,), (d,), (d,)]
    return [torch.empty(s, device="meta") for s in shapes]


def gemm_family(census):
    """All GEMM launches of one step together: algorithmic FLOPs / summed launch time."""
    fl = sum(c["flops"] * c["launches"] for c in census)
    ms = sum(c["ms"] * c["launches"] for c in census)
    return {"launches_per_step": sum(c["launches"] for c in census), "ms_per_step": round(ms, 4),
            "achieved": round(fl / (ms * 1e-3) / 1e12, 1), "frac": round(fl / (ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4)}


def pmc_traffic(config, dom):
    """HBM (L2-miss) bytes per launch of the dominant op from the committed rocprofv3 PMC passes
    (tools/pmc_gemm_traffic.sh + tools/pmc_gemm.py -> profiles/r<N>_pmc_gemm_traffic_<config>.json,
    the latest round's file first); None when no file covers this exact shape, split and epilogue
    (files before round 4 timed every forward / dgrad with a plain store: they match only the
    plain-store and weight-gradient ops)."""
    for rnd in ("r6", "r5", "r4", "r3", "r2", "r1"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_gemm_traffic_{config}.json")
        try:
            op = json.load(open(path))["ops"][dom["name"]]
        except (OSError, KeyError, ValueError):
            continue
        epi = op.get("epilogue", "wgrad" if op["split"] > 1 or dom["name"].endswith("wgrad") else "store")
        if (op["M"], op["N"], op["K"], op["split"], epi) == (dom["M"], dom["N"], dom["K"], dom["split"],
                                                             dom["epilogue"]):
            return {"bytes": op["hbm_bytes"], "algorithmic_bytes": op.get("algorithmic_bytes"),
                    "source": os.path.relpath(path, ROOT)}
    return None


GEMM_FNS = {"relu_bwd_colpart": "gemm_relu_bwd_colpart", "bias_relu_bits": "gemm_bias_relu_bits",
            "store_rowdot": "gemm_store_rowdot"}


class _TimingEvent:
    """A HIP event recorded through the library (cg_timing_event_record): inside a graph capture an
    external event-record node, which torch's own Event may not create on ROCm."""

    def __init__(self, lib):
        import ctypes
        from replicatinggpt_amd import _lib as L
        self.lib, self.L, self.h = lib, L, ctypes.c_void_p()
        L.check(lib.cg_timing_event_create(ctypes.byref(self.h)), "timing_event_create")

    def record(self):
        self.L.check(self.lib.cg_timing_event_record(self.h, self.L.stream_ptr()), "timing_event_record")

    def elapsed_ms(self, end):
        import ctypes
        ms = ctypes.c_float()
        self.L.check(self.lib.cg_timing_event_elapsed(self.h, end.h, ctypes.byref(ms)), "timing_event_elapsed")
        return ms.value

    def __del__(self):
        try:
            self.lib.cg_timing_event_destroy(self.h)
        except Exception:   # noqa: BLE001 -- interpreter shutdown
            pass


def in_step_launch_ms(model, opt, sampler, dom, replays=7):
    """The dominant op's average launch duration INSIDE the training step, measured live: one more
    hipGraph of the whole step (forward, backward, AdamW -- the timed region's graph, same model) is
    captured with an external timing event recorded before and after every launch of that op (the
    ops-module entry it goes through, matched on M, N, K and layout; cg_timing_event_record),
    replayed ``replays`` times after the timed region, and the event pairs of each replay averaged
    (median over replays).  In the step a launch also runs whatever deferred split-K reduce / AdamW
    work it hosts on free slots, and finds its operands as the step leaves them (colder than the
    census's back-to-back replays).  HIP events on the step's stream: the record nodes sit between
    the op's kernel and its neighbours: an extra record node right before each start event times one
    node-to-node hand-off, which is subtracted (the raw figure is reported beside it).  Returns (ms,
    launches per step, the probe graph's ms per step, raw ms) or None when the events cannot be
    captured."""
    from replicatinggpt_amd import _lib as L, ops
    from replicatinggpt_amd.engine import TrainStep
    lib = L.load()
    fname = GEMM_FNS.get(dom["epilogue"], "gemm")
    orig = getattr(ops, fname)
    pairs = []

    def probe(*a, **k):
        if fname == "gemm":
            key, lay = (a[6], a[7], a[8]), (bool(a[4]), bool(a[5]))
        else:
            key, lay = (a[3], a[4], a[5]), dom["layout"]
        want = (dom["M"], dom["N"], dom["K"]) == key and lay == dom["layout"]
        if not (want and torch.cuda.is_current_stream_capturing()):
            return orig(*a, **k)
        z, s, e = _TimingEvent(lib), _TimingEvent(lib), _TimingEvent(lib)
        z.record()   # z -> s: two adjacent record nodes, the cost of one node hand-off
        s.record()
        r = orig(*a, **k)
        e.record()
        pairs.append((z, s, e))
        return r
    setattr(ops, fname, probe)
    st = None
    try:
        st = TrainStep(model, opt, sampler, None, use_graph=True)
        st.capture(warmup=1)
        if not pairs:
            return None
        per, raw, steps = [], [], []
        for _ in range(replays):
            t0 = time.perf_counter()
            st.step()
            torch.cuda.synchronize()
            steps.append((time.perf_counter() - t0) * 1e3)
            r = sum(s.elapsed_ms(e) for _, s, e in pairs) / len(pairs)
            d = sum(z.elapsed_ms(s) for z, s, _ in pairs) / len(pairs)
            raw.append(r)
            per.append(r - d)
    except Exception as ex:   # noqa: BLE001 -- a runtime without timed external events: no live figure
        _log(f"in-step probe unavailable: {type(ex).__name__}: {ex}")
        return None
    finally:
        setattr(ops, fname, orig)
        del st
        torch.cuda.empty_cache()
    med = lambda x: sorted(x)[len(x) // 2]   # noqa: E731
    return med(per), len(pairs), med(steps), med(raw)


def step_kernel(config, dom):
    """The dominant op's in-step launch time from the committed rocprofv3 kernel trace of a bench run
    (tools/gpu_prof_bench.sh -> tools/step_kernels.py -> profiles/r<N>_step_kernels_<config>.json, the
    latest round first): in the step a launch may host deferred reduces / AdamW jobs on free slots
    and finds its operands colder than the census's back-to-back replays.  None when no file has it.
    Not a measurement of this run: the bench line carries it under roofline.committed_trace."""
    for rnd in ("r6", "r5"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_step_kernels_{config}.json")
        try:
            op = json.load(open(path))["ops"][dom["name"]]
        except (OSError, KeyError, ValueError):
            continue
        if op.get("in_step_avg_us") is None:
            return None
        return {"in_step_avg_launch_ms": round(op["in_step_avg_us"] / 1e3, 5), "in_step_kernel": op["kernel"],
                "in_step_census_ms_same_trace": round(op["census_us"] / 1e3, 5), "in_step_shared_with": op["shared_with"],
                "in_step_source": os.path.relpath(path, ROOT)}
    return None


PEAK_FP32_TFLOPS = 157.3     # MI355X f32 MFMA / vector peak (MI355X_MICROARCH.md)


def generate_flops(cfg, B, L0, new):
    """Algorithmic forward FLOPs of GPT1.py's generate(): while the context fits the
    block, one new token per sequence per step against the cached prefix,
    2 (L 12 d^2 + d V) + 4 L t d (t = current length); once it slides (Q7: positions re-indexed, no
    K/V reuse), the full block_size-token window forward per step -- GEMMs 2 T (L 12 d^2), causal
    attention 4 L d T (T+1)/2, lm_head on the last row 2 d V."""
    L, d, V, T = cfg.n_layers, cfg.n_embd, cfg.vocab_size, cfg.block_size
    total = 0.0
    for i in range(new):
        t = L0 + i + 1
        if t <= T:
            total += 2 * (L * 12 * d * d + d * V) + 4 * L * t * d
        else:
            total += 2 * T * (L * 12 * d * d) + 4 * L * d * T * (T + 1) / 2 + 2 * d * V
    return B * total


def bench_generate(dev, B=256, new=500):
    """BASELINE configs[4] (C5): generate() batched decode, 256 sequences x 500 new tokens from
    the reference-trained C1-shape weights (tests/golden/model_c1_trained.safetensors -- the
    model.pth of GPT1.py:239-241 as produced by the reference), fp32, through the decode engine
    (K/V-cached prefix phase + sliding-window phase, one hipGraph per phase): greedy (the parity
    mode) and sampled (GPT1.py:206-208's multinomial, device inverse-CDF draw).  ``frac`` =
    algorithmic forward FLOPs (generate_flops) / time against the fp32 peak (the model runs fp32)."""
    from safetensors.torch import load_file
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    sd = load_file(os.path.join(ROOT, "tests", "golden", "model_c1_trained.safetensors"))
    m = BigramLanguageModel(GPTConfig(dtype="fp32"))
    m.load_state_dict(sd, strict=False)
    m = m.to(dev).eval()
    idx = torch.zeros((B, 1), dtype=torch.long, device=dev)
    res = {}
    with torch.no_grad():
        for mode, greedy in (("greedy", True), ("sampled", False)):
            gen = torch.Generator().manual_seed(1337)
            m.generate(idx, new, greedy=greedy, generator=gen)       # capture + warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = m.generate(idx, new, greedy=greedy, generator=gen)
            torch.cuda.synchronize()
            res[mode] = (time.perf_counter() - t0, int(out.sum()))
    T = m.config.block_size
    fl = generate_flops(m.config, B, 1, new)
    dt, ck = res["greedy"]
    ach = fl / dt / 1e12
    return {"metric": "generate tokens/sec (C5: 256 seqs x 500 new tokens, model.pth C1 shape, fp32 greedy)",
            "value": round(B * new / dt, 1), "unit": "tokens/s", "seconds": round(dt, 4),
            "phases": {"kv_cached_steps": T, "sliding_window_steps": new - T},
            "roofline": {"bound": "mfma_f32", "achieved": round(ach, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / PEAK_FP32_TFLOPS, 4), "flops": fl},
            "sampled": {"value": round(B * new / res["sampled"][0], 1), "unit": "tokens/s",
                        "seconds": round(res["sampled"][0], 4)},
            "checksum": ck}


_T_START = time.perf_counter()


def _log(msg):
    """Progress on stderr (stdout carries only the one JSON line)."""
    print(f"[bench {time.perf_counter() - _T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """``bench.py --gpus N`` started without a launcher: run N ranks of this same command under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a CHILD process -- this
    process has touched no GPU and execs nothing -- and return the worst rank's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    _log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def dry_run(args, world, rank, local):
    """The N-rank launch path without a GPU (gloo on CPU): every rank builds the data-parallel
    sampler and the bucketed gradient reducer exactly as the GPU run does, times ``--steps`` steps of
    (get_batch offsets draw, fake gradient, all-reduce AVG) between barriers, takes the max over ranks
    and rank 0 prints the one JSON line -- so the launcher, the rank/rendezvous plumbing, the sampler
    slicing and the single-line output contract are testable on the build container."""
    from replicatinggpt_amd import PRESETS
    from replicatinggpt_amd.data import BatchSampler, TokenStream
    from replicatinggpt_amd.engine import GradReducer
    if world > 1:
        dist.init_process_group("gloo")
    cfg = PRESETS[args.config]
    Bsz, T = args.batch or cfg.batch_size, cfg.block_size
    sampler = BatchSampler(TokenStream.synthetic(n_tokens=1 << 16), T, Bsz, world_size=world, rank=rank,
                           generator=torch.Generator().manual_seed(cfg.seed))
    grad = torch.zeros(1 << 12)
    red = GradReducer(grad, bucket_bytes=4096)
    first = []
    for i in range(args.warmup + args.steps):
        if i == args.warmup:
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
        ix = sampler.draw_ix("train")
        if not first:
            first = ix[:4].tolist()
        grad.fill_(float(rank + 1))
        red.all_reduce()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    print(f"[rank {rank} local {local} world {world}] first offsets {first} grad {float(grad[0])}",
          file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps({"metric": "dry run (no GPU): launcher + sampler + gradient all-reduce", "value": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 4), "dry_run": True,
                          "config": {"workload": args.config, "global_batch": Bsz * world, "seq_len": T,
                                     "parallelism": f"dp{world}", "world_size": world,
                                     "backend": "gloo" if world > 1 else None}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c1"])
    ap.add_argument("--batch", type=int, default=None, help="sequences per GPU (default: config)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-census", action="store_true")
    ap.add_argument("--no-generate", action="store_true", help="skip the C5 batched-decode measurement")
    ap.add_argument("--overlap", type=int, default=None, choices=[0, 1],
                    help="force the segmented (DP-overlap) backward on/off (default: on when N > 1)")
    ap.add_argument("--seg-layers", type=int, default=2,
                    help="DP: blocks per backward graph segment (gradient all-reduce overlaps the next segment; "
                         "the last segment, blocks 0..seg-1 + embeddings, is exposed: DESIGN.md section 6. "
                         "2: +0.7 %% at W = 1 against +1.8 %% for 1, profiles/r5_dp_path_w1_step_ab.txt)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the N-rank launch, sampler slicing and reducer on gloo")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # started as `python bench.py --gpus N`: become the launcher of N ranks (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    if args.dry_run:
        return dry_run(args, world, rank, local)
    # test hooks (tests/test_gpu_bench_dp.py): CHARPT_DP_BACKEND=gloo and CHARPT_DP_ONE_DEVICE=1 run the
    # N-rank path on one GPU -- every rank on cuda:0, gradients averaged over gloo (SUM + divide)
    backend = os.environ.get("CHARPT_DP_BACKEND", "nccl")
    local_dev = 0 if os.environ.get("CHARPT_DP_ONE_DEVICE") == "1" else local
    if world > 1:
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_dev)

    from replicatinggpt_amd import AdamW, BigramLanguageModel, PRESETS
    from replicatinggpt_amd.data import BatchSampler, TokenStream
    from replicatinggpt_amd.engine import GradReducer, TrainStep

    cfg = PRESETS[args.config].with_(dtype="bf16" if args.config != "c1" else "fp32")
    Bsz = args.batch or cfg.batch_size
    T = cfg.block_size
    torch.manual_seed(cfg.seed)
    model = BigramLanguageModel(cfg).to(dev)
    opt = AdamW(model.parameters(), lr=cfg.learning_rate).attach(model)
    stream = TokenStream.synthetic(device=dev)
    sampler = BatchSampler(stream, T, Bsz, world_size=world, rank=rank,
                           generator=torch.Generator().manual_seed(cfg.seed))
    reducer = GradReducer(model.flat.grad) if (world > 1 or args.overlap) else None
    step = TrainStep(model, opt, sampler, reducer, use_graph=not args.no_graph, seg_layers=args.seg_layers,
                     overlap=None if args.overlap is None else bool(args.overlap))
    step.capture()
    _log("captured; warmup")
    for _ in range(args.warmup):
        step.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    final_loss = float(loss.detach())
    tokens = world * Bsz * T * args.steps
    value = tokens / elapsed
    ms_step = elapsed / args.steps * 1e3
    F = flops_per_token(cfg, T)
    mfu = value * F / (world * PEAK_BF16_TFLOPS * 1e12)

    result = None
    _log(f"timed {args.steps} steps: {elapsed / args.steps * 1e3:.3f} ms/step")
    step_path = ("segmented backward graphs + bucketed all-reduce (DP)" if step.overlap
                 else "single graph (fwd + bwd + AdamW)")
    graphed, nseg = step.g_fb is not None or bool(step.g_seg), len(step.ranges)
    overlap = step.overlap
    red_kind = "RCCL AVG" if backend == "nccl" else f"{backend} SUM + divide"
    del step   # the probe below captures its own graph of the step
    torch.cuda.empty_cache()
    if rank == 0:
        roofline, census = None, None
        if not args.no_census:
            census = gemm_census(cfg, Bsz, T, dev)
            dom = max(census, key=lambda c: c["ms"] * c["launches"])
            c_ach = dom["flops"] / (dom["ms"] * 1e-3) / 1e12
            kname = (f"cg_gemm bf16 {dom['name']} M={dom['M']} N={dom['N']} K={dom['K']}"
                     f" ({dom['kernel']}, split {dom['split']}, epilogue {dom['epilogue']})")
            # the line's figure: the op's launches inside the training step, timed live (HIP events
            # in a graph of the step); the census (same op, 30 back-to-back launches) beside it
            _log("in-step probe of the dominant op")
            live = in_step_launch_ms(model, opt, sampler, dom)
            ms_op = live[0] if live else dom["ms"]
            achieved = dom["flops"] / (ms_op * 1e-3) / 1e12
            roofline = {"bound": "mfma", "kernel": kname,
                        "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "flops_per_launch": dom["flops"],
                        "avg_launch_ms": round(ms_op, 5),
                        "timing": ("in-step: HIP events around each of the op's launches in a hipGraph of the "
                                   f"training step, {live[1]} launches per step, median of 7 replays after the "
                                   f"timed region, less one event-node hand-off (raw {live[3] * 1e3:.2f} us; that "
                                   f"graph's step {live[2]:.3f} ms incl. host sync)"
                                   if live else "census (in-step probe unavailable)"),
                        "census_avg_launch_ms": round(dom["ms"], 5), "census_achieved": round(c_ach, 1),
                        "census_frac": round(c_ach / PEAK_BF16_TFLOPS, 4),
                        "traffic": None, "gemm_family": gemm_family(census)}
            pt = pmc_traffic(args.config, dom)
            if pt is not None:
                roofline["traffic"], roofline["traffic_source"] = pt["bytes"], pt["source"]
            sk = step_kernel(args.config, dom)
            if sk is not None:   # a committed rocprofv3 trace of an earlier run: not this run's measurement
                roofline["committed_trace"] = sk
        result = {
            "metric": "train tokens/sec at 1/2/4/8 MI355X + MFMA util, char-GPT block 256",
            "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"{args.config}: char-GPT {cfg.n_layers}L/{cfg.n_head}H/{cfg.n_embd}d, "
                                   f"block {T}, batch {Bsz}/GPU, dropout {cfg.dropout}, AdamW, full train step",
                       "global_batch": Bsz * world, "seq_len": T, "parallelism": f"dp{world}",
                       "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                       "backend": ((f"{dist.get_backend()} (RCCL)" if dist.get_backend() == "nccl" else dist.get_backend())
                                   if dist.is_initialized() else None),
                       "step_path": step_path, "graph": graphed,
                       "grad_allreduce": (f"{red_kind} overlapped: {nseg} backward segments"
                                          if overlap else (f"{red_kind} after backward" if world > 1 else None))},
            "mfu_step": round(mfu, 4), "flops_per_token": F, "final_loss": round(final_loss, 4),
            "roofline": roofline,
        }
        if census is not None:
            _log("gemm census done; kernel census")
            result["gemm_census_ms"] = {c["name"]: round(c["ms"], 4) for c in census}
            result["kernel_census"] = kernel_census(cfg, Bsz, T, dev)
        if world == 1 and not args.no_generate:
            _log("generate (C5)")
            result["generate_c5"] = bench_generate(dev)
        if world == 1 and not args.no_cpu_baseline:
            _log("cpu baseline")
            result["cpu_baseline"] = cpu_baseline(cfg)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
