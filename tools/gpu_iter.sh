#!/bin/bash
# Quick GPU iteration: parity tests, GEMM census, bench line (no CPU baseline).
# Every GPU step has its own time limit; the first failure ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 300 python tools/gemm_census.py --top 80 > gpurun_out/census.txt 2>&1
head -2 gpurun_out/census.txt | tail -1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_iter.log 2>&1
grep '^{"metric' gpurun_out/bench_iter.log | cut -c1-260
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_iter -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/prof_iter.log 2>&1
echo "trace done"
