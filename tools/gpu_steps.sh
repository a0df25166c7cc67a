#!/bin/bash
# Run GPU steps in order, each under its own time limit, and stop at the first step that
# crashed, aborted, faulted or timed out (exit status >= 124, or a signal); a plain test /
# assertion failure (status 1..123) is reported and the next step still runs.
#   STEPS: newline-separated "name|seconds|command" (command runs under bash -c)
# Logs: gpurun_out/step_<name>.log; summary lines on stdout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
worst=0
while IFS='|' read -r name secs cmd; do
  [ -z "$name" ] && continue
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > gpurun_out/step_$name.log 2>&1
  rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -n ${TAIL:-4} gpurun_out/step_$name.log | cut -c1-400
  [ $rc -gt $worst ] && worst=$rc
  if [ $rc -ge 124 ]; then
    echo "[$name] crashed / timed out: no further GPU steps"
    exit $rc
  fi
done <<< "$STEPS"
exit $worst
