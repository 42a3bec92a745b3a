#!/bin/bash
# Run named GPU stages in order; stop at the first fault / timeout / abort (exit codes other than
# 0 = ok and 1 = test failures).  Usage: bash tools/gpu_stage.sh "<name>|<timeout s>|<command>" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (timeout ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "--- $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
exit 0
