#!/bin/bash
# measure only: few-tiles threshold 256 (default) vs 512 on the whole step, fp32 and bf16
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for dt in fp32 bf16; do
    for v in 256 512; do
      ACCUNET_FEW_TILES=$v timeout -k 10 400 python bench.py --dtype $dt --no-cpu-baseline --no-probe > gpurun_out/bench_few_${dt}_$v.log 2>&1
      echo "$dt few=$v rep $rep: $(grep -o '"value": [0-9.]*' gpurun_out/bench_few_${dt}_$v.log)"
    done
  done
done
