#!/bin/bash
# embedding backward 4-wave partials: tests (stop on failure), model tests, then the C2 step A/B needs the
# previous library (the step's embedding kernels timed from the rocprof trace instead)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "embedding" tests/test_gpu_model.py -m gpu > gpurun_out/r3s3_emb_tests.log 2>&1 || { tail -30 gpurun_out/r3s3_emb_tests.log; exit 5; }
tail -1 gpurun_out/r3s3_emb_tests.log
for r in a b; do timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/$r /" || exit 7; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3s3_prof_emb -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-generate --no-census > $GRAFT_REPO_ROOT/gpurun_out/r3s3_prof_emb.log 2>&1 || exit 8
