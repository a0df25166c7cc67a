#!/bin/bash
# SE middle step in one launch (last-arriver channel step): SE / model tests, then the
# step A/B against the previous library (_ab/se2 = git HEAD~0 before the change)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_bf16_gpu.py -x -q --timeout 240 --timeout-method thread -k "se_ or eager or graph or bit_identical or matches_oracle" > gpurun_out/se_tests.log 2>&1 || { tail -30 gpurun_out/se_tests.log; exit 1; }
tail -n 2 gpurun_out/se_tests.log
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export ACCUNET_LIB_OVERRIDE=$PWD/_ab/se2/libaccunet_hip.so; else unset ACCUNET_LIB_OVERRIDE; fi
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-probe > gpurun_out/bench_se_$v.log 2>&1
    echo "$v rep $rep"; grep '^{"metric' gpurun_out/bench_se_$v.log | cut -c1-190
  done
done
unset ACCUNET_LIB_OVERRIDE
for v in new; do
  timeout -k 10 400 python bench.py --dtype bf16 --no-cpu-baseline --no-probe > gpurun_out/bench_se_bf16.log 2>&1
  echo "bf16 $v"; grep '^{"metric' gpurun_out/bench_se_bf16.log | cut -c1-190
done
