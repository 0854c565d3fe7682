"""HBM traffic of every bf16 GEMM of the bench census (bench.census_shapes), for the roofline
`traffic` field.  Run under rocprofv3 in two passes (FETCH_SIZE and WRITE_SIZE do not fit one
pass, MI355X_MICROARCH.md 'rocprofv3 PMC slots'):

    rocprofv3 --pmc FETCH_SIZE -d <dir> -o fetch -- python3 tools/pmc_gemm.py run [c2]
    rocprofv3 --pmc WRITE_SIZE -d <dir> -o write -- python3 tools/pmc_gemm.py run [c2]
    python tools/pmc_gemm.py parse <fetch counter csv> <write counter csv> <out.json> [c2]

`run` launches each census op (bench.census_op: the step's fused epilogue) REPS times back to back,
in census order, after all operands exist
(so the charpt dispatches in the trace are exactly that sequence); an op is one cg_gemm call: the
GEMM kernel plus, for split-K weight gradients, its reduce kernel.  `parse` walks the charpt
dispatches in order, assigns them to ops, and reports per-launch bytes averaged over launches 2..REPS
(launch 1 runs cache-cold; the training step feeds each GEMM operands written just before).
FETCH_SIZE is doubled (gfx950 reports half the bytes of wide coalesced reads); WRITE_SIZE is exact
for 16-B stores.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REPS = 6


def plan(config):
    import bench
    from replicatinggpt_amd import PRESETS
    from replicatinggpt_amd import functional as Fn
    cfg = PRESETS[config]
    ops = []
    for name, m, n, k, at, bt, kind, _cnt in bench.census_shapes(cfg, cfg.batch_size, cfg.block_size):
        split = Fn._wgrad_split(m, n, k, True) if kind == "wgrad" else 1
        ops.append({"name": name, "M": m, "N": n, "K": k, "at": at, "bt": bt, "split": split, "epilogue": kind,
                    "kernels": 2 if split > 1 else 1})
    return ops


def algorithmic_bytes(op):
    """Operands read once + output written once + the epilogue's own operands (bench.census_op)."""
    M, N, K, kind = op["M"], op["N"], op["K"], op["epilogue"]
    b = 2 * (M * K + N * K)
    if kind == "wgrad":
        return b + 4 * M * N
    if kind == "store":
        return b + 2 * M * N
    if kind == "store_rowdot":
        return b + 2 * M * N + 2 * M * N + 4 * (M * N // 64)   # bf16 dO, O read, delta
    if kind in ("bias_resid", "bias_drop_resid"):
        return b + 4 * N + 4 * M * N + 4 * M * N          # bias, fp32 residual read, fp32 output
    if kind == "bias_relu_bits":
        return b + 4 * N + 2 * M * N + M * N // 8        # bias, bf16 output, keep bits
    if kind == "relu_bwd_colpart":
        return b + M * N // 8 + 2 * M * N + 4 * (M // 64) * N   # keep bits, bf16 output, column partials
    raise ValueError(kind)


def run(config):
    import torch
    import bench
    dev = torch.device("cuda")
    todo = []
    for op in plan(config):
        fn, nk = bench.census_op(op["name"], op["M"], op["N"], op["K"], op["at"], op["bt"], op["epilogue"], dev)
        assert nk == op["kernels"]
        todo.append(fn)
    torch.cuda.synchronize()
    for fn in todo:
        for _ in range(REPS):
            fn()
    torch.cuda.synchronize()


def _dispatches(path, counter):
    rows = collections.OrderedDict()
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if r["Counter_Name"] != counter or not ("k_gemm" in name or "k_splitk_reduce" in name or "k_slab16_reduce" in name):
                continue
            key = int(r.get("Dispatch_Id") or r["Correlation_Id"])
            rows[key] = rows.get(key, 0.0) + float(r["Counter_Value"]) * 1024.0   # KiB -> bytes
    return [rows[k] for k in sorted(rows)]


def parse(fetch_csv, write_csv, out_json, config):
    fetch = _dispatches(fetch_csv, "FETCH_SIZE")
    write = _dispatches(write_csv, "WRITE_SIZE")
    ops = plan(config)
    need = sum(op["kernels"] * REPS for op in ops)
    if len(fetch) != need or len(write) != need:
        raise SystemExit(f"expected {need} charpt dispatches, got fetch {len(fetch)} / write {len(write)}")
    res, i = {}, 0
    for op in ops:
        nk = op["kernels"]
        f = [2.0 * sum(fetch[i + r * nk:i + (r + 1) * nk]) for r in range(REPS)]
        w = [sum(write[i + r * nk:i + (r + 1) * nk]) for r in range(REPS)]
        i += nk * REPS
        fb, wb = sum(f[1:]) / (REPS - 1), sum(w[1:]) / (REPS - 1)
        alg = algorithmic_bytes(op)
        res[op["name"]] = {"M": op["M"], "N": op["N"], "K": op["K"], "split": op["split"], "epilogue": op["epilogue"],
                           "fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb),
                           "algorithmic_bytes": alg, "cold_first_launch_bytes": round(f[0] + w[0])}
        print(f"{op['name']:11s} {op['epilogue']:16s} split {op['split']:2d}  hbm {(fb + wb) / 1e6:8.2f} MB/launch  "
              f"(algorithmic {alg / 1e6:7.2f} MB, cold {(f[0] + w[0]) / 1e6:8.2f} MB)")
    json.dump({"config": config, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of "
               "tools/pmc_gemm.py run; FETCH_SIZE x2 (gfx950); mean of launches 2..%d per op" % REPS,
               "ops": res}, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2] if len(sys.argv) > 2 else "c2")
    else:
        parse(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else "c2")
