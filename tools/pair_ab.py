"""cg_gemm_pair (one persistent launch for a Linear's dgrad + weight gradient) against the two
launches it replaces, at the C2 backward shapes (GPT1.py:111-112,136,143,145): each form replayed
as 20 back-to-back calls from a hipGraph (bench._time_ms), the step's epilogues (projection dgrad with
the attention delta, FFN2 ReLU-backward dgrad from keep bits with the b1 partials, plain dgrads;
weight gradients through bf16 split-K slabs with their reduce), over weight-gradient splits; the pair
form bitwise against the two calls.  GPU only.  usage: python tools/pair_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import _time_ms  # noqa: E402
from replicatinggpt_amd import _lib as L, functional as Fn, ops  # noqa: E402


def case(name, M, N, K, epi, dev, splits):
    """dy [M, N], w [N, K] (dgrad out [M, K]); weight gradient [N, K] = dy^T x, x [M, K]"""
    g = torch.Generator(device=dev).manual_seed(1)
    dy = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=g) * N ** -0.5).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    dout = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
    gout = torch.empty(N, K, dtype=torch.float32, device=dev)
    aux, ld_aux, colpart, T = None, 0, None, 0
    if epi == L.EPI_RELU_BWD:
        aux = torch.randint(-2 ** 31, 2 ** 31 - 1, (M, K // 32), dtype=torch.int32, device=dev)
        ld_aux, colpart = aux.stride(0), torch.empty(M // 64, K, device=dev)
    elif epi == L.EPI_STORE_ROWDOT:
        aux = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        ld_aux, T, colpart = K, 256, torch.empty(M * K // 64, device=dev)
    wflags = L.GEMM_SLAB_BF16
    for split in splits:
        ws = torch.empty(ops.gemm_workspace(N, K, split) // 4, dtype=torch.float32, device=dev)
        outs = {}

        def two():
            e = L.Epilogue(epi, None, None, T, L.ptr(aux), L.dtype_code(aux.dtype) if aux is not None else 0, ld_aux,
                           0.0, 0, None, 0, 0.0, L.ptr(colpart), 0)
            L.check(L.load().cg_gemm(L.CG_BF16, 0, 1, M, K, N, L.ptr(dy), N, L.ptr(w), K, L.ptr(dout), L.CG_BF16, K,
                                     e, 1, None, L.stream_ptr()), "dgrad")
            ops.gemm(dy, x, gout, True, True, True, N, K, M, N, K, K, 0, None, None, 0, None, 0, 0.0, 0, None, 0,
                     0.0, split, ws, wflags)

        def pair():
            ops.gemm_pair(dy, w, dout, epi, aux, ld_aux, colpart, T, x, gout, 0.0, split, ws, wflags)
        sup = ops.gemm_pair_supported(dy, w, dout, epi, aux, ld_aux, colpart, T, x, gout, 0.0, split, ws, wflags)
        for nm, fn in (("two", two), ("pair", pair)):
            dout.fill_(float("nan"))
            gout.fill_(float("nan"))
            if colpart is not None:
                colpart.fill_(float("nan"))
            fn()
            torch.cuda.synchronize()
            outs[nm] = (dout.clone(), gout.clone(), None if colpart is None else colpart.clone())
        same = all(torch.equal(a, b) for a, b in zip(outs["two"], outs["pair"]) if a is not None)
        t2, tp = _time_ms(two), _time_ms(pair)
        print(f"{name:6s} split {split:2d} supported {int(sup)} bitwise {'equal' if same else 'DIFFERENT'} | "
              f"two launches {t2 * 1e3:6.1f} us  pair {tp * 1e3:6.1f} us  ({(tp / t2 - 1) * 100:+.1f} %)", flush=True)


def main():
    dev = torch.device("cuda:0")
    M = 16384
    case("proj", M, 384, 384, L.EPI_STORE_ROWDOT, dev, (8, 12, 16, 24, 32))
    case("qkv", M, 1152, 384, L.EPI_STORE, dev, (8, 12, 16, 18, 23, 28))
    case("ffn2", M, 384, 1536, L.EPI_RELU_BWD, dev, (8, 12, 14, 16, 20))
    case("ffn1", M, 1536, 384, L.EPI_STORE, dev, (8, 12, 14, 16, 20))


if __name__ == "__main__":
    main()
