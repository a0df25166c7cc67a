#!/bin/bash
# GPU check of the tree: -m gpu suite, fp32 + bf16 bench lines, kbench.
# Each GPU step has its own time limit; the first failure ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -k "${PYTEST_K:-}" > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
  tail -3 gpurun_out/gputests.log
fi
for dt in fp32 bf16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dtype $dt > gpurun_out/bench_$dt.log 2>&1 || { tail -30 gpurun_out/bench_$dt.log; exit 1; }
  grep '^{"metric' gpurun_out/bench_$dt.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dtype'], d['value'], d['ms_per_step'], [(r['kernel'][:30], r['avg_us'], r.get('median_us'), r['frac']) for r in d['rooflines']])"
done
timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench.txt 2>&1
cat gpurun_out/kbench.txt
