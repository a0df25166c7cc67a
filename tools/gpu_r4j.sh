#!/bin/bash
# halo forward schedule change: conv3x3 tests (bitwise vs the engine), gbench A/B, bench
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 240 --timeout-method thread -k "conv3x3" > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -n 2 gpurun_out/c3_tests.log
: > gpurun_out/c3_ab.txt
for rep in 1 2; do
  for v in 1 0; do
    echo "== ACCUNET_CONV3_HALO=$v" >> gpurun_out/c3_ab.txt
    ACCUNET_CONV3_HALO=$v GB_ONLY=rspth timeout -k 10 120 tools/gbench 20 >> gpurun_out/c3_ab.txt 2>&1
  done
done
cat gpurun_out/c3_ab.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1
grep '^{"metric' gpurun_out/bench_c3.log | cut -c1-200
