"""In-step kernel times of the census GEMM ops, from the rocprofv3 kernel trace of one bench.py run.

bench.py first replays the training step (the last `steps` replays = the window between the last
steps + 1 k_embed_fwd launches, one per step), then times every census GEMM op as a burst of >= 30
identical launches (time_gemm; a weight gradient's burst alternates GEMM and split-K reduce).  The
bursts give each census op its kernel (name + grid); the window gives that kernel's average
duration and launches per step inside the training step.  A kernel that two census ops share
(same instantiation and grid) gets the mixed in-step average and lists the other ops.
skip: training-step replays at the end of the trace that are not the timed region's (bench.py's
in-step probe replays 1 eager + 7 graph steps after it: pass 8).
usage: python tools/step_kernels.py <run_kernel_trace.csv> <c2|c4> <out.json> [steps] [skip]"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def clean(name):
    return re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", "")).replace("void ", "").replace("cg::", "")


def main():
    path, config, out = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    skip = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), clean(r["Kernel_Name"]), grid))
    rows.sort()
    marks = [s for s, e, n, g in rows if "k_embed_fwd" in n]
    if skip:
        marks = marks[:-skip]
    if len(marks) < steps + 1:
        raise SystemExit(f"only {len(marks)} steps in the trace")
    t0, t1 = marks[-steps - 1], marks[-1]
    inwin = {}
    for s, e, n, g in rows:
        if t0 <= s < t1:
            c = inwin.setdefault((n, g), [0, 0])
            c[0] += 1
            c[1] += e - s
    # census bursts after the window, in census order
    rest = [(s, e, n, g) for s, e, n, g in rows if s >= t1]
    bursts, i = [], 0
    while i < len(rest):
        n0 = rest[i][2]
        if "gemm" not in n0:
            i += 1
            continue
        found = False
        for period in (1, 2):
            j = i
            while j + period < len(rest) and rest[j + period][2] == rest[j][2] and rest[j + period][3] == rest[j][3] and \
                    ("gemm" in rest[j][2] or "splitk" in rest[j][2] or "slab" in rest[j][2]):
                j += 1
            k = (j + period - i) // period
            if k >= 30:
                seg = rest[i:i + k * period]
                bursts.append((rest[i][2], rest[i][3], sum(e - s for s, e, _, _ in seg) / k / 1e3))
                i += k * period
                found = True
                break
        if not found:
            i += 1
    from bench import census_shapes
    from replicatinggpt_amd.config import PRESETS
    cfg = PRESETS[config]
    shapes = census_shapes(cfg, cfg.batch_size, cfg.block_size)
    if len(bursts) < len(shapes):
        raise SystemExit(f"{len(bursts)} census bursts for {len(shapes)} ops")
    bursts = bursts[:len(shapes)]
    ops = {}
    for sh, (name, grid, busy) in zip(shapes, bursts):
        cnt, tot = inwin.get((name, grid), (0, 0))
        grids = [grid]
        if not cnt:   # in the step the launch got extra blocks (pending reduces on its free slots): same kernel
            grids = sorted(g for (n, g) in inwin if n == name)
            cnt = sum(inwin[(name, g)][0] for g in grids)
            tot = sum(inwin[(name, g)][1] for g in grids)
        ops[sh[0]] = {"kernel": name, "grid": grid, "in_step_grids": grids, "census_us": round(busy, 2),
                      "in_step_launches_per_step": round(cnt / steps, 2),
                      "in_step_avg_us": round(tot / cnt / 1e3, 2) if cnt else None,
                      "launches_per_step": sh[7]}
    for k, v in ops.items():
        v["shared_with"] = [k2 for k2, v2 in ops.items()
                            if k2 != k and v2["kernel"] == v["kernel"] and set(v2["in_step_grids"]) & set(v["in_step_grids"])]
    res = {"source": os.path.basename(path), "config": config, "steps": steps,
           "note": "tools/step_kernels.py: census op -> kernel from the census bursts, its in-step duration from the "
                   "last `steps` training-step replays of the same rocprofv3 kernel trace",
           "ops": ops}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in ops.items():
        print(f"{k:11s} census {v['census_us']:7.2f} us  in step {v['in_step_avg_us']} us x {v['in_step_launches_per_step']}"
              f" (census {v['launches_per_step']}/step) {'shared ' + ','.join(v['shared_with']) if v['shared_with'] else ''}")


if __name__ == "__main__":
    main()
