#!/bin/bash
# bf16 GEMM register prefetch depth A/B: the in-tree library (depth 2 for the fp32-output
# split-K / weight-gradient instances) against abx/pf1 (tools/build_alt.sh of the tree
# with depth 1 everywhere): the bf16 / GEMM GPU tests in-tree, then bench.py bf16
# alternating, then the bf16 GEMM census of each
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bf16_gpu.py tests/test_gemm_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pf2_tests.log 2>&1 || { tail -30 gpurun_out/pf2_tests.log; exit 1; }
tail -n 1 gpurun_out/pf2_tests.log
DT=bf16 REPS="1 2 3" BENCH_ARGS="--no-parity" VARIANTS="pf1:abx/pf1: cur:-:" bash tools/gpu_ab.sh
for v in pf1 cur; do
  if [ $v = cur ]; then unset ACCUNET_LIB_OVERRIDE; else export ACCUNET_LIB_OVERRIDE=$PWD/abx/$v/libaccunet_hip.so; fi
  timeout -k 10 300 python tools/gemm_census.py --dtype bf16 --top 80 > gpurun_out/census_$v.txt 2>&1
  head -n 2 gpurun_out/census_$v.txt | tail -n 1
done
