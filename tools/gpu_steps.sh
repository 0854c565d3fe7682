#!/bin/bash
# Run GPU steps in order; each line of the argument file is "<timeout_s> <logname> <command...>".
# A pytest failure (exit 1) does not stop the sequence; a crash, abort or timeout does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
while IFS= read -r line; do
  [ -z "$line" ] && continue
  t=$(echo "$line" | awk '{print $1}'); log=$(echo "$line" | awk '{print $2}'); cmd=$(echo "$line" | cut -d' ' -f3-)
  echo "=== [$log] $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== [$log] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done < "$1"
