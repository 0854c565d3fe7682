#!/bin/bash
# Same-box A/B of two library builds on the full bench (C2 step + GEMM census), interleaved:
# usage: tools/lib_ab.sh <tag> <libB.so> [rounds] [config]   (A = the product library)
set -o pipefail
tag=$1; libb=$2; rounds=${3:-3}; cfg=${4:-c2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out/ab_$tag
for r in $(seq 1 $rounds); do
  for v in A B; do
    if [ $v = A ]; then lib=$R/replicatinggpt_amd/libcharpt_hip.so; else lib=$R/replicatinggpt_amd/$libb; fi
    CHARPT_LIB=$lib timeout -k 10 300 python3 $R/bench.py --config $cfg --steps 30 --warmup 10 --no-cpu-baseline \
      --no-generate > $R/gpurun_out/ab_$tag/${v}_$r.json 2> $R/gpurun_out/ab_$tag/${v}_$r.err || exit $?
  done
done
python3 - "$R/gpurun_out/ab_$tag" $rounds <<'PY'
import json, sys, statistics as st
d, n = sys.argv[1], int(sys.argv[2])
res = {v: [json.load(open(f"{d}/{v}_{r}.json")) for r in range(1, n + 1)] for v in "AB"}
for v in "AB":
    print(v, "ms/step", [x["ms_per_step"] for x in res[v]], "median", st.median(x["ms_per_step"] for x in res[v]))
names = list(res["A"][0]["gemm_census_ms"])
for k in names:
    a = st.median(x["gemm_census_ms"][k] for x in res["A"]) * 1e3
    b = st.median(x["gemm_census_ms"][k] for x in res["B"]) * 1e3
    print(f"  {k:12s} A {a:7.2f} us  B {b:7.2f} us  ({(b / a - 1) * 100:+.1f} %)")
for v in "AB":
    print(v, "family", [x["roofline"]["gemm_family"]["ms_per_step"] for x in res[v]], "in-step dom",
          [round(x["roofline"]["avg_launch_ms"] * 1e3, 2) for x in res[v]])
PY
