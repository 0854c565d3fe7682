"""fp32 forward GEMM A/B: k_gemm_f32 (gemm_variant 98) against the default dispatch (round 6: the
persistent k_gemm_f32p for M > 2048; outputs compared bitwise) at the C5 generate() window shapes (256 x 256 rows, C1 width 126), per-launch time from a
hipGraph replay of 20 launches (HIP events), rounds interleaved; then, with `gen`, one C5 generate
(256 x 500 greedy, fp32, C1 golden weights) timed under the variant named second.
usage: python tools/f32_fwd_ab.py [rounds]            (kernel A/B, 98 vs 0)
       python tools/f32_fwd_ab.py now [rounds]        (the current library's fp32 products at those shapes)
       python tools/f32_fwd_ab.py small [variant]     (the 256-row products of generate()'s steps)
       python tools/f32_fwd_ab.py gen <98|0> [knob]   (generate with cg_set_tuning(knob, value), knob
                                                      gemm_variant by default; fresh process)"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replicatinggpt_amd import _lib as L, ops  # noqa: E402

SHAPES = [("qkv", 65536, 378, 126, 0), ("proj", 65536, 126, 126, 3), ("ffn1", 65536, 504, 126, 2),
          ("ffn2", 65536, 126, 504, 3)]
SMALL = [("qkv", 256, 378, 126, 0), ("proj", 256, 126, 126, 3), ("ffn1", 256, 504, 126, 2),
         ("ffn2", 256, 126, 504, 3), ("head", 256, 65, 126, 1)]


def launch_fn(M, N, K, kind, dev, outs=None):
    torch.manual_seed(5)
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    out = torch.empty(M, N, device=dev)
    bias = torch.randn(N, device=dev)
    resid = torch.randn(M, N, device=dev)

    def run():
        ops.gemm(A, B, out, False, False, False, M, N, K, K, K, N, kind, bias if kind else None,
                 resid if kind == 3 else None, N if kind == 3 else 0, None, 0, 0.0, 0, None, 0, 0.0, 1, None)
    if outs is not None:
        run()
        torch.cuda.synchronize()
        outs.append(out.clone())
    return run


def graph_us(run, reps=20):
    run()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            run()
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def kernels(rounds):
    lib = L.load()
    dev = torch.device("cuda")
    t = {(n, v): [] for n, *_ in SHAPES for v in (98, 0)}
    for name, M, N, K, kind in SHAPES:
        outs = []
        for v in (98, 0):
            L.check(lib.cg_set_tuning(b"gemm_variant", v))
            launch_fn(M, N, K, kind, dev, outs)
        same = torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
        print(f"{name:5s} bitwise 98 vs 0: {'equal' if same else 'DIFFERENT'}", flush=True)
        del outs
    for _ in range(rounds):
        for name, M, N, K, kind in SHAPES:
            for v in (98, 0):
                L.check(lib.cg_set_tuning(b"gemm_variant", v))
                t[(name, v)].append(graph_us(launch_fn(M, N, K, kind, dev)))
                torch.cuda.empty_cache()
    L.check(lib.cg_set_tuning(b"gemm_variant", 0))
    for name, M, N, K, kind in SHAPES:
        a, b = statistics.median(t[(name, 98)]), statistics.median(t[(name, 0)])
        tf = 2 * M * N * K / 1e12
        print(f"{name:5s} M={M} N={N} K={K} epi {kind}: k_gemm_f32 {a:7.1f} us ({tf / a * 1e6:6.1f} TF/s)  "
              f"default {b:7.1f} us ({tf / b * 1e6:6.1f} TF/s)  {b / a - 1:+.1%}", flush=True)


def gen(variant, knob="gemm_variant"):
    from safetensors.torch import load_file
    from replicatinggpt_amd import BigramLanguageModel, GPTConfig
    L.check(L.load().cg_set_tuning(knob.encode(), variant))
    sd = load_file(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                                "model_c1_trained.safetensors"))
    m = BigramLanguageModel(GPTConfig(dtype="fp32"))
    m.load_state_dict(sd, strict=False)
    m = m.to("cuda").eval()
    idx = torch.zeros((256, 1), dtype=torch.long, device="cuda")
    with torch.no_grad():
        m.generate(idx, 500, greedy=True, generator=torch.Generator().manual_seed(1337))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = m.generate(idx, 500, greedy=True, generator=torch.Generator().manual_seed(1337))
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{knob} {variant}: generate 256x500 {dt * 1e3:.1f} ms = {256 * 500 / dt:.0f} tok/s, "
          f"checksum {int(out.sum())}", flush=True)


def now(rounds, shapes=None):
    SHAPES = shapes or globals()["SHAPES"]
    L.load()
    dev = torch.device("cuda")
    t = {n: [] for n, *_ in SHAPES}
    for _ in range(rounds):
        for name, M, N, K, kind in SHAPES:
            t[name].append(graph_us(launch_fn(M, N, K, kind, dev)))
            torch.cuda.empty_cache()
    for name, M, N, K, kind in SHAPES:
        a = statistics.median(t[name])
        print(f"{name:5s} M={M} N={N} K={K} epi {kind}: {a:7.1f} us ({2 * M * N * K / a / 1e6:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "now":
        now(int(sys.argv[2]) if len(sys.argv) > 2 else 5)
    elif len(sys.argv) > 1 and sys.argv[1] == "small":   # generate()'s 256-row products, knob gemm_variant
        L.check(L.load().cg_set_tuning(b"gemm_variant", int(sys.argv[2]) if len(sys.argv) > 2 else 0))
        now(3, SMALL)
    elif len(sys.argv) > 1 and sys.argv[1] == "gen":
        gen(int(sys.argv[2]), *(sys.argv[3:4]))
    else:
        kernels(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
