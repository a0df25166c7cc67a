#!/bin/bash
# rocprofv3 kernel trace of a short bench run (HIP-graph mode), for tools/step_profile.py.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
grep '^{"metric' gpurun_out/prof_bench.log | cut -c1-200
