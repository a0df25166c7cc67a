#!/bin/bash
# few-tiles threshold A/B over every GEMM of one step (tools/gemm_census.py) and the step
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 128 256 512; do
  ACCUNET_FEW_TILES=$v timeout -k 10 300 python tools/gemm_census.py --top 200 > gpurun_out/census_few$v.txt 2>&1
  echo "few=$v: $(grep 'total GEMM time' gpurun_out/census_few$v.txt)"
done
for rep in 1 2; do
  for v in 128 256; do
    ACCUNET_FEW_TILES=$v timeout -k 10 400 python bench.py --no-cpu-baseline --no-probe > gpurun_out/bench_few$v.log 2>&1
    echo "fp32 few=$v rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/bench_few$v.log)"
  done
done
