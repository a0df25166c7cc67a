#!/bin/bash
# GPU pass: all -m gpu tests, then the fp32 and bf16 bench lines (no CPU baseline).
# Each GPU step has its own time limit; the first failure ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "${PYTEST_K:-}" > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dtype $dt > gpurun_out/bench_$dt.log 2>&1 || { tail -30 gpurun_out/bench_$dt.log; exit 1; }
  grep '^{"metric' gpurun_out/bench_$dt.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dtype'], d['value'], d['ms_per_step'], [(r['kernel'], r['avg_us'], r['frac']) for r in d['rooflines']])"
done
