#!/bin/bash
# One GPU-box pass: parity tests, the bench line, a rocprofv3 kernel trace of the
# bench, two PMC passes (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of K1, and the
# kernel microbenchmark. Every GPU step has its own time limit; the first failure
# ends the pass.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1
grep '^{"metric' gpurun_out/bench_full.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "kernel trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
echo "pmc done"
timeout -k 10 120 tools/kbench 20 > gpurun_out/kbench.txt 2>&1
echo "kbench done"
