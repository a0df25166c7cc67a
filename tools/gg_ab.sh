#!/bin/bash
# A/B of the LDS-DMA fp32 GEMM engine (ACCUNET_GEMM_G=1 default vs 0) in one box session
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$PYTEST_K" > gpurun_out/gg_tests.txt 2>&1 || { tail -30 gpurun_out/gg_tests.txt; exit 1; }
  tail -2 gpurun_out/gg_tests.txt
fi
for v in 1 0; do
  ACCUNET_GEMM_G=$v timeout -k 10 300 python tools/gemm_census.py --top 200 > gpurun_out/census_g$v.txt 2>&1
  ACCUNET_GEMM_G=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_g$v.txt 2>&1
  echo "== G=$v"; head -2 gpurun_out/census_g$v.txt | tail -1; grep -o '"value": [0-9.]*' gpurun_out/bench_g$v.txt
done
