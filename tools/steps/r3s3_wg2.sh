#!/bin/bash
# grouped weight gradients: products per grouped launch (wgrad_group) vs off, C2 and C4, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in a b; do
  CHARPT_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/c2 off $r /" || exit 7
  for gsz in 2 4 8; do
    CHARPT_TUNING=wgrad_group=$gsz timeout -k 10 200 python bench.py --no-cpu-baseline --no-generate --no-census --steps 60 2>&1 | grep timed | sed "s/^/c2 g$gsz $r /" || exit 8
  done
done
CHARPT_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-generate --no-census --steps 8 --warmup 3 2>&1 | grep timed | sed "s/^/c4 off /" || exit 9
for gsz in 2 4; do
  CHARPT_TUNING=wgrad_group=$gsz timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-generate --no-census --steps 8 --warmup 3 2>&1 | grep timed | sed "s/^/c4 g$gsz /" || exit 10
done
