#!/bin/bash
# Round-4 check: -m gpu suite, then the default bench line (with the same-run parity leg).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_parity.log 2>&1 || { tail -30 gpurun_out/bench_parity.log; exit 1; }
tail -1 gpurun_out/bench_parity.log
